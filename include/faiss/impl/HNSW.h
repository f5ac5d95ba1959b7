// faiss/impl/HNSW.h — HNSW, SearchParametersHNSW, HNSWStats / hnsw_stats
#pragma once
#include "faiss_amd_names.h"
