// faiss/index_factory.h — index_factory (Flat, IVFn[_HNSWm],Flat|PQm, HNSWm)
#pragma once
#include "impl/faiss_amd_names.h"
