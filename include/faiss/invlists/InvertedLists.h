// faiss/invlists/InvertedLists.h — ArrayInvertedLists, SubsetType
#pragma once
#include "../impl/faiss_amd_names.h"
