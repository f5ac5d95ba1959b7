/*
 * The reference benchmark harness's search sequence, written against the
 * C ABI (include/faiss_amd_c.h) and compiled with a plain C compiler:
 *   read_index(fname, IO_FLAG_MMAP) -> nprobe / quantizer efSearch /
 *   parallel_mode 0 -> IndexIVF::search_stats -> QPS, latency percentiles
 * (reference tutorial/cpp/benchmark-hnsw-ivf/benchmark_hnsw_ivf.cpp:361-404).
 * Queries are faiss float_rand(nq * d, seed).  Writes D then I (raw) to
 * out_file and one summary line to stdout.
 *
 * usage: harness index_file nq k nprobe efSearch seed out_file
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "faiss_amd_c.h"

#define CHECK(call)                                                          \
    do {                                                                     \
        if ((call) != 0) {                                                   \
            fprintf(stderr, "%s failed: %s\n", #call, faiss_get_last_error()); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

static int cmp_double(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc != 8) {
        fprintf(stderr, "usage: %s index nq k nprobe efSearch seed out\n", argv[0]);
        return 2;
    }
    const idx_t nq = atoll(argv[2]), k = atoll(argv[3]);
    const size_t nprobe = (size_t)atoll(argv[4]);
    const int ef = atoi(argv[5]);
    const int64_t seed = atoll(argv[6]);
    FaissIndex* index = NULL;
    /* faiss::IO_FLAG_MMAP (faiss/index_io.h:52): IO_FLAG_SKIP_IVF_DATA | 0x646f0000 */
    CHECK(faiss_read_index_fname(argv[1], 8 | 0x646f0000, &index));
    const int d = faiss_Index_d(index);
    faiss_IndexIVF_set_nprobe(index, nprobe);
    FaissIndex* q = faiss_IndexIVF_quantizer(index);
    if (ef > 0) faiss_amd_IndexHNSW_set_efSearch(q, ef);
    faiss_amd_IndexIVF_set_parallel_mode(index, 0);
    float* xq = (float*)malloc(sizeof(float) * (size_t)nq * d);
    float* D = (float*)malloc(sizeof(float) * (size_t)nq * k);
    idx_t* I = (idx_t*)malloc(sizeof(idx_t) * (size_t)nq * k);
    FaissQueryLatencyStats* lat =
            (FaissQueryLatencyStats*)malloc(sizeof(FaissQueryLatencyStats) * (size_t)nq);
    double* ms = (double*)malloc(sizeof(double) * (size_t)nq);
    CHECK(faiss_amd_float_rand(xq, (size_t)nq * d, seed));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    CHECK(faiss_amd_IndexIVF_search_stats(index, nq, xq, k, NULL, D, I, lat));
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double s = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    double mean = 0;
    for (idx_t i = 0; i < nq; i++) {
        ms[i] = lat[i].total_us / 1000.0;
        mean += ms[i];
    }
    mean /= (double)nq;
    qsort(ms, (size_t)nq, sizeof(double), cmp_double);
    printf("{\"nq\": %lld, \"qps\": %.1f, \"mean_ms\": %.6f, \"p50_ms\": %.6f, "
           "\"p95_ms\": %.6f, \"p99_ms\": %.6f}\n",
           (long long)nq, nq / s, mean, ms[(size_t)(nq * 0.50)], ms[(size_t)(nq * 0.95)],
           ms[(size_t)(nq * 0.99)]);
    FILE* f = fopen(argv[7], "wb");
    if (!f) return 1;
    fwrite(D, sizeof(float), (size_t)nq * k, f);
    fwrite(I, sizeof(idx_t), (size_t)nq * k, f);
    fclose(f);
    faiss_Index_free(index);
    free(xq);
    free(D);
    free(I);
    free(lat);
    free(ms);
    return 0;
}
