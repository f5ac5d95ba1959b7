// faiss/impl/ProductQuantizer.h — ProductQuantizer (PQ8 codebooks)
#pragma once
#include "faiss_amd_names.h"
