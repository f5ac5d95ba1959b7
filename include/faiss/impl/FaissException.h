// faiss/impl/FaissException.h — faiss::FaissException
#pragma once
#include "faiss_amd_names.h"
