/*
 * index_io_c.h — drop-in for the reference C API header `c_api/index_io_c.h`
 * (Quaternijkon/hnsw-ivf = Faiss 1.10.0).  A C caller of the reference keeps
 * its `#include "index_io_c.h"` (or <faiss/c_api/index_io_c.h>) and links
 * libfaiss_amd.so: the declarations — write_index / read_index on FILE* and file names —
 * are this library's, with the reference's names, signatures and return codes
 * (include/faiss_amd_c.h, which cites each reference declaration).
 */
#ifndef FAISS_INDEX_IO_C_H
#define FAISS_INDEX_IO_C_H

#include "faiss_c.h"

/* the reference C header's flag values (passed to faiss_read_index*) */
#ifndef FAISS_IO_FLAG_MMAP
#define FAISS_IO_FLAG_MMAP 1
#define FAISS_IO_FLAG_READ_ONLY 2
#endif

#endif /* FAISS_INDEX_IO_C_H */
