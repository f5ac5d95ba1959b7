/*
 * clone_index_c.h — drop-in for the reference C API header `c_api/clone_index_c.h`
 * (Quaternijkon/hnsw-ivf = Faiss 1.10.0).  A C caller of the reference keeps
 * its `#include "clone_index_c.h"` (or <faiss/c_api/clone_index_c.h>) and links
 * libfaiss_amd.so: the declarations — faiss_clone_index —
 * are this library's, with the reference's names, signatures and return codes
 * (include/faiss_amd_c.h, which cites each reference declaration).
 */
#ifndef FAISS_CLONE_INDEX_C_H
#define FAISS_CLONE_INDEX_C_H

#include "faiss_c.h"

#endif /* FAISS_CLONE_INDEX_C_H */
