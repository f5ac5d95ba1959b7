// faiss/Index.h — faiss::Index, SearchParameters (faiss/Index.h:63-181)
#pragma once
#include "impl/faiss_amd_names.h"
