// faiss/MetricType.h — idx_t, MetricType (faiss/MetricType.h:22-44)
#pragma once
#include "impl/faiss_amd_names.h"
