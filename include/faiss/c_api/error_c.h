/*
 * error_c.h — drop-in for the reference C API header `c_api/error_c.h`
 * (Quaternijkon/hnsw-ivf = Faiss 1.10.0).  A C caller of the reference keeps
 * its `#include "error_c.h"` (or <faiss/c_api/error_c.h>) and links
 * libfaiss_amd.so: the declarations — FaissErrorCode and faiss_get_last_error —
 * are this library's, with the reference's names, signatures and return codes
 * (include/faiss_amd_c.h, which cites each reference declaration).
 */
#ifndef FAISS_ERROR_C_H
#define FAISS_ERROR_C_H

#include "faiss_c.h"

#endif /* FAISS_ERROR_C_H */
