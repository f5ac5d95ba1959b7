// faiss/impl/AuxIndexStructures.h — RangeSearchResult
#pragma once
#include "faiss_amd_names.h"
