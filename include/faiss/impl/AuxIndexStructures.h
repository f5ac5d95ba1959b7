// faiss/impl/AuxIndexStructures.h — RangeSearchResult, InterruptCallback,
// TimeoutCallback
#pragma once
#include "faiss_amd_names.h"
