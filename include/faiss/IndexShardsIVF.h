// faiss/IndexShardsIVF.h — IndexShardsIVF
#pragma once
#include "impl/faiss_amd_names.h"
