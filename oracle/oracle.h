/*
 * oracle.h — CPU restatement of the reference IVF search path (TEST
 * INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the MI355X implementation and the
 * timed CPU baseline ("port") in bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  It is never linked into or
 * called by the product library (hnsw-ivf_amd/lib/libfaiss_amd.so).
 *
 * It restates, function by function, Quaternijkon/hnsw-ivf (Faiss 1.10.0):
 *   float_rand            faiss/utils/random.cpp:35-53,95-112
 *   heaps (CMax / CMin)   faiss/utils/Heap.h:47-150,316-450,
 *                         faiss/utils/ordered_key_value.h:42-80
 *   knn (flat quantizer)  faiss/utils/distances.cpp:170-199 (seq),
 *                         :259-342 (BLAS form), :807-823 (dispatch at nx>=20),
 *                         faiss/impl/ResultHandler.h:187-287 (heap handler)
 *   IndexIVF::search      faiss/IndexIVF.cpp:303-397 (query slices)
 *   search_preassigned    faiss/IndexIVF.cpp:399-723 (parallel_mode 0)
 *   IVFFlat scanner       faiss/IndexIVFFlat.cpp:129-179
 *   IVFPQ tables / scan   faiss/IndexIVFPQ.cpp:364-459 (precomputed table),
 *                         :560-566,:634-700 (tables 0/1), :861-933 (scan),
 *                         faiss/impl/code_distance/code_distance-generic.h
 *   HNSW search           faiss/impl/HNSW.cpp:605-741,852-924,943-996,
 *                         1096-1342 (generic pop_min)
 *   merge_knn_results     faiss/utils/Heap.cpp:159-230
 *
 * fp32 evaluation order.  The reference leaves it to BLAS (sgemm) and to GCC
 * auto-vectorisation (faiss/impl/platform_macros.h:168-181).  The oracle
 * fixes ONE order, the same as the GPU kernels: every dot / squared distance
 * is a sequential fmaf chain over j = 0..d-1, and the BLAS-form coarse
 * distance is fmaf(-2, ip, |x|^2 + |y|^2) clamped at 0.  The oracle's
 * primitives are pinned against the reference's own compiled sources
 * (oracle/ref, tests/golden) to <= 1e-6 relative; everything integer
 * (heaps, ties, slicing, probe order, padding) is reproduced exactly.
 * `fast` variants (8 partial sums, vectorisable) exist only for the timed
 * CPU baseline.
 */
#ifndef ORACLE_H
#define ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void oracle_float_rand(float* x, size_t n, int64_t seed);

float oracle_fvec_L2sqr(const float* x, const float* y, size_t d);
float oracle_fvec_inner_product(const float* x, const float* y, size_t d);
float oracle_fvec_norm_L2sqr(const float* x, size_t d);

/* heap primitives on (float, int64) — C = 1 for CMax (L2), 0 for CMin (IP) */
void oracle_heap_heapify(int cmax, size_t k, float* val, int64_t* ids);
void oracle_heap_replace_top(int cmax, size_t k, float* val, int64_t* ids, float v, int64_t id);
/* heap_addn: strict admission of x[i] (ids[i]) in order */
void oracle_heap_addn(int cmax, size_t k, float* val, int64_t* ids, const float* x,
                      const int64_t* xids, size_t n);
size_t oracle_heap_reorder(int cmax, size_t k, float* val, int64_t* ids);

/* exact kNN of x[nx] among y[ny]; metric 1 = L2, 0 = IP.  blas_form: 1 =
 * norm expansion (nx >= 20 in the reference), 0 = direct distances. */
void oracle_knn(const float* x, const float* y, size_t d, size_t nx, size_t ny, size_t k,
                int metric, int blas_form, float* D, int64_t* I, int nthreads);

typedef struct {
    int32_t entry_point;
    int32_t max_level;
    int64_t ntotal;
    const int32_t* levels;      /* [ntotal], level + 1 */
    const uint64_t* offsets;    /* [ntotal + 1] */
    const int32_t* neighbors;
    const int32_t* cum_nneighbor_per_level;
    const float* storage;       /* [ntotal][d] */
    int d;
} oracle_hnsw_t;

/* IndexHNSW::search for n queries (k results, L2) */
void oracle_hnsw_search(const oracle_hnsw_t* g, const float* x, size_t n, size_t k,
                        int efSearch, float* D, int64_t* I, int nthreads);

typedef struct {
    int d;
    int64_t nlist;
    int metric;                 /* 1 = L2, 0 = IP */
    const float* centroids;     /* [nlist][d] (flat quantizer) */
    const oracle_hnsw_t* hnsw;  /* non-NULL: HNSW coarse quantizer */
    const int64_t* list_off;    /* [nlist + 1] */
    const uint8_t* codes;       /* concatenated lists, code_size bytes per entry */
    size_t code_size;
    const int64_t* ids;
    /* PQ (pq_M = 0 for IVF-Flat) */
    int pq_M;
    int pq_nbits;
    const float* pq_centroids;  /* [M][ksub][dsub] */
    int by_residual;
    int use_precomputed_table;  /* 0 or 1, decided as faiss does */
    float* precomputed_table;   /* [nlist][M][ksub] when table 1 (filled by prepare) */
} oracle_ivf_t;

/* PQ table entry of one sub-vector in the reference's fvec_*_ny order
 * (faiss/utils/distances_simd.cpp:1362-1410, AVX2 specialisations) */
float oracle_pq_ny_ip(const float* x, const float* y, int dsub);
float oracle_pq_ny_l2(const float* x, const float* y, int dsub);
/* distance_single_code / distance_four_codes, PQDecoder8, AVX2 order
 * (faiss/impl/code_distance/code_distance-avx2.h) */
float oracle_pq_code_sum(int M, const float* sim, int ksub, const uint8_t* code);
/* IndexIVFPQ::encode_vectors + ProductQuantizer::compute_codes (dsub < 16) */
void oracle_ivfpq_encode(const oracle_ivf_t* ivf, size_t n, const float* x,
                         const int64_t* list_nos, uint8_t* codes);
/* faiss/IndexIVFPQ.cpp:364-459: fills precomputed_table when table 1 */
void oracle_ivfpq_prepare(oracle_ivf_t* ivf);

void oracle_ivf_search_preassigned(const oracle_ivf_t* ivf, size_t n, const float* x, size_t k,
                                   size_t nprobe, const int64_t* keys, const float* coarse_dis,
                                   float* D, int64_t* I, int nthreads);
/* the same with max_codes (0 = unlimited, IndexIVF.cpp:452-454, :609-622)
 * and the ndis total (indexIVF_stats.ndis) */
void oracle_ivf_search_preassigned_mc(const oracle_ivf_t* ivf, size_t n, const float* x,
                                      size_t k, size_t nprobe, const int64_t* keys,
                                      const float* coarse_dis, int64_t max_codes, float* D,
                                      int64_t* I, int64_t* ndis, int nthreads);

/* IndexIVF::search: nslices query slices (the reference uses
 * min(omp_max_threads, n)), coarse per slice, then search_preassigned. */
void oracle_ivf_search(const oracle_ivf_t* ivf, size_t n, const float* x, size_t k,
                       size_t nprobe, int efSearch, int nslices, float* D, int64_t* I,
                       int64_t* coarse_I, float* coarse_D, int nthreads);

/* fast (vectorisable, 8 partial sums) IVF-Flat scan — cpu_baseline only */
void oracle_ivf_search_fast(const oracle_ivf_t* ivf, size_t n, const float* x, size_t k,
                            size_t nprobe, float* D, int64_t* I, int nthreads);

void oracle_merge_knn_results(size_t n, size_t k, int nshard, const float* all_distances,
                              const int64_t* all_labels, float* distances, int64_t* labels,
                              int metric);

int oracle_max_threads(void);

/* IVF range search restated (faiss/IndexIVF.cpp:1243-1400,
 * faiss/IndexIVFFlat.cpp:181-201, faiss/IndexIVFPQ.cpp:1254-1279); returns
 * the number of results; coarse_dis used by PQ table 1 only */
int64_t oracle_ivf_range_preassigned(const oracle_ivf_t* ivf, size_t n, const float* x,
                                     size_t nprobe, const int64_t* keys,
                                     const float* coarse_dis, float radius,
                                     const uint8_t* selmask, size_t* lims, float* D, int64_t* I,
                                     int64_t cap);

#ifdef __cplusplus
}
#endif
#endif

