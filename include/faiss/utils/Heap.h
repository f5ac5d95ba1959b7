// faiss/utils/Heap.h — merge_knn_results (faiss/utils/Heap.cpp:159-230, host
// form: ties to the lower shard, missing results padded (+-FLT_MAX, -1)).
// The heap templates themselves (heap_push / heap_pop / CMax ...) are the
// reference's CPU scanner internals and are not part of this library's API:
// the GPU path keeps its top-k in wave queues.
#pragma once
#include "../impl/faiss_amd_names.h"
