// faiss/IndexIVFPQ.h — IndexIVFPQ (and faiss/impl/ProductQuantizer.h)
#pragma once
#include "impl/faiss_amd_names.h"
