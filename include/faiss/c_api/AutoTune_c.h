/*
 * AutoTune_c.h — drop-in for the reference C API header `c_api/AutoTune_c.h`
 * (Quaternijkon/hnsw-ivf = Faiss 1.10.0).  A C caller of the reference keeps
 * its `#include "AutoTune_c.h"` (or <faiss/c_api/AutoTune_c.h>) and links
 * libfaiss_amd.so: the declarations — ParameterSpace new / free / set_index_parameter ("nprobe",
 * "efSearch", "quantizer_efSearch", "max_codes") —
 * are this library's, with the reference's names, signatures and return codes
 * (include/faiss_amd_c.h, which cites each reference declaration).
 */
#ifndef FAISS_AUTO_TUNE_C_H
#define FAISS_AUTO_TUNE_C_H

#include "faiss_c.h"

#endif /* FAISS_AUTO_TUNE_C_H */
