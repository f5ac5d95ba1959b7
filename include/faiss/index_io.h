// faiss/index_io.h — read_index / write_index and the IO_FLAG_* values
#pragma once
#include "impl/faiss_amd_names.h"
