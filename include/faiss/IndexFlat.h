// faiss/IndexFlat.h — IndexFlat / IndexFlatL2 / IndexFlatIP
#pragma once
#include "impl/faiss_amd_names.h"
