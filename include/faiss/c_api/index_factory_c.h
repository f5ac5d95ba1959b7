/*
 * index_factory_c.h — drop-in for the reference C API header `c_api/index_factory_c.h`
 * (Quaternijkon/hnsw-ivf = Faiss 1.10.0).  A C caller of the reference keeps
 * its `#include "index_factory_c.h"` (or <faiss/c_api/index_factory_c.h>) and links
 * libfaiss_amd.so: the declarations — index_factory ("Flat", "IVF<n>[_HNSW<m>],Flat|PQ<M>", "HNSW<m>") —
 * are this library's, with the reference's names, signatures and return codes
 * (include/faiss_amd_c.h, which cites each reference declaration).
 */
#ifndef FAISS_INDEX_FACTORY_C_H
#define FAISS_INDEX_FACTORY_C_H

#include "faiss_c.h"

#endif /* FAISS_INDEX_FACTORY_C_H */
