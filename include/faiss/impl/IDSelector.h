// faiss/impl/IDSelector.h — the IDSelector family of the search path
#pragma once
#include "faiss_amd_names.h"
