// faiss/utils/random.h — float_rand (faiss/utils/random.cpp:95-112, bit-exact)
#pragma once
#include "../impl/faiss_amd_names.h"
