// faiss/IndexIVF.h — IndexIVF, SearchParametersIVF, IndexIVFStats, QueryLatencyStats
#pragma once
#include "impl/faiss_amd_names.h"
