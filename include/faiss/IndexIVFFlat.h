// faiss/IndexIVFFlat.h — IndexIVFFlat
#pragma once
#include "impl/faiss_amd_names.h"
