// faiss/impl/io.h — the reference's IOReader / IOWriter layer.  On this path
// the readers and writers are the FILE* / file-name forms of faiss/index_io.h
// (read_index(FILE*), write_index(const Index*, FILE*)), which this header
// brings in; the format is the reference's (index_write.cpp / index_read.cpp).
#pragma once
#include <cstdio>
#include "faiss_amd_names.h"
