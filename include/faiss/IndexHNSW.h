// faiss/IndexHNSW.h — IndexHNSW / IndexHNSWFlat (and faiss/impl/HNSW.h)
#pragma once
#include "impl/faiss_amd_names.h"
