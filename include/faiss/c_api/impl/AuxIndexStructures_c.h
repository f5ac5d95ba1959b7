/*
 * impl/AuxIndexStructures_c.h — drop-in for the reference C API header `c_api/impl/AuxIndexStructures_c.h`
 * (Quaternijkon/hnsw-ivf = Faiss 1.10.0).  A C caller of the reference keeps
 * its `#include "AuxIndexStructures_c.h"` (or <faiss/c_api/impl/AuxIndexStructures_c.h>) and links
 * libfaiss_amd.so: the declarations — RangeSearchResult and the IDSelector family (Range, Batch,
 * Bitmap, Not, And, Or, XOr) —
 * are this library's, with the reference's names, signatures and return codes
 * (include/faiss_amd_c.h, which cites each reference declaration).
 */
#ifndef FAISS_AUX_INDEX_STRUCTURES_C_H
#define FAISS_AUX_INDEX_STRUCTURES_C_H

/* ../faiss_c.h; under `gcc -I- -I<this c_api dir>` (a caller compiled in
 * place next to the reference's own headers) the same file on the -I path */
#if defined(__has_include)
#if __has_include("../faiss_c.h")
#include "../faiss_c.h"
#else
#include "faiss_c.h"
#endif
#else
#include "../faiss_c.h"
#endif

#endif /* FAISS_AUX_INDEX_STRUCTURES_C_H */
