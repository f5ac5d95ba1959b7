/*
 * oracle.c — CPU restatement of the reference IVF search path.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker and the timed CPU baseline.
 * Never linked into the product library.  See oracle.h for the reference
 * file:line each function follows and for the fixed fp32 evaluation order.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------ mt19937 */
/* std::mt19937 (the generator behind faiss::RandomGenerator) */
typedef struct {
    uint32_t mt[624];
    int idx;
} mt19937_t;

static void mt_seed(mt19937_t* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->idx = 624;
}
static uint32_t mt_next(mt19937_t* s) {
    if (s->idx >= 624) {
        for (int i = 0; i < 624; i++) {
            uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
            s->mt[i] = s->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        s->idx = 0;
    }
    uint32_t y = s->mt[s->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* faiss/utils/random.cpp:95-112: 1024 independent streams (n >= 1024) */
void oracle_float_rand(float* x, size_t n, int64_t seed) {
    const size_t nblock = n < 1024 ? 1 : 1024;
    mt19937_t r0;
    mt_seed(&r0, (uint32_t)seed);
    int a0 = (int)(mt_next(&r0) & 0x7fffffff);
    int b0 = (int)(mt_next(&r0) & 0x7fffffff);
    const float mx = (float)4294967295u;
#pragma omp parallel for if (n > 1000000)
    for (int64_t j = 0; j < (int64_t)nblock; j++) {
        mt19937_t r;
        mt_seed(&r, (uint32_t)(int64_t)(a0 + j * (int64_t)b0));
        size_t i0 = j * n / nblock, i1 = (j + 1) * n / nblock;
        for (size_t i = i0; i < i1; i++) x[i] = (float)mt_next(&r) / mx;
    }
}

/* ------------------------------------------------------------ distances */
/* faiss/utils/distances_simd.cpp:220-230 (fvec_L2sqr) and its inner-product
 * and norm siblings, as GCC compiles them under the reference's
 * FAISS_PRAGMA_IMPRECISE_FUNCTION_BEGIN (associative-math) + AVX2/FMA flags:
 * 8 fma accumulators over i < d & ~7, reduced (j,j+4),(j,j+2),(0,1); a
 * 4-term epilogue rounded alone and reduced (0,2),(1,3),(0,1), then added;
 * the last d % 4 terms fma'd in order.  Pinned bit-for-bit against the
 * reference sources compiled by oracle/ref (tests/test_oracle_golden.py). */
static inline float ref_dist_(const float* x, const float* y, size_t d, int l2) {
    float c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const size_t n8 = d & ~(size_t)7;
    for (size_t i = 0; i < n8; i += 8)
        for (int j = 0; j < 8; j++) {
            if (l2) {
                const float t = x[i + j] - y[i + j];
                c[j] = fmaf(t, t, c[j]);
            } else {
                c[j] = fmaf(x[i + j], y[i + j], c[j]);
            }
        }
    const float x0 = c[0] + c[4], x1 = c[1] + c[5], x2 = c[2] + c[6], x3 = c[3] + c[7];
    float r = (x0 + x2) + (x1 + x3);
    size_t i = n8;
    if (d - n8 >= 4) {
        float e[4];
        for (int j = 0; j < 4; j++) {
            if (l2) {
                const float t = x[n8 + j] - y[n8 + j];
                e[j] = t * t;
            } else {
                e[j] = x[n8 + j] * y[n8 + j];
            }
        }
        r = r + ((e[0] + e[2]) + (e[1] + e[3]));
        i += 4;
    }
    for (; i < d; i++) {
        if (l2) {
            const float t = x[i] - y[i];
            r = fmaf(t, t, r);
        } else {
            r = fmaf(x[i], y[i], r);
        }
    }
    return r;
}
float oracle_fvec_L2sqr(const float* x, const float* y, size_t d) { return ref_dist_(x, y, d, 1); }
float oracle_fvec_inner_product(const float* x, const float* y, size_t d) {
    return ref_dist_(x, y, d, 0);
}
float oracle_fvec_norm_L2sqr(const float* x, size_t d) { return ref_dist_(x, x, d, 0); }
/* The BLAS-form inner product <x, c> of the coarse quantizer comes from
 * sgemm (MKL / OpenBLAS order, not reproducible); the restatement fixes it
 * to the sequential fma chain, which is what the fp32 MFMA tile computes. */
float oracle_ip_seq(const float* x, const float* y, size_t d) {
    float acc = 0.f;
    for (size_t j = 0; j < d; j++) acc = fmaf(x[j], y[j], acc);
    return acc;
}

/* ------------------------------------------------------------ heaps */
/* faiss/utils/ordered_key_value.h: CMax (cmax=1) / CMin (cmax=0) */
static inline int cmp_(int cmax, float a, float b) { return cmax ? a > b : a < b; }
static inline int cmp2_(int cmax, float a1, float b1, int64_t a2, int64_t b2) {
    return cmax ? (a1 > b1 || (a1 == b1 && a2 > b2)) : (a1 < b1 || (a1 == b1 && a2 < b2));
}
static inline float neutral_(int cmax) { return cmax ? FLT_MAX : -FLT_MAX; }

/* faiss/utils/Heap.h:47-79 */
static void heap_pop_(int cmax, size_t k, float* bv, int64_t* bi) {
    bv--;
    bi--;
    float val = bv[k];
    int64_t id = bi[k];
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k) break;
        if ((i2 == k + 1) || cmp2_(cmax, bv[i1], bv[i2], bi[i1], bi[i2])) {
            if (cmp2_(cmax, val, bv[i1], id, bi[i1])) break;
            bv[i] = bv[i1];
            bi[i] = bi[i1];
            i = i1;
        } else {
            if (cmp2_(cmax, val, bv[i2], id, bi[i2])) break;
            bv[i] = bv[i2];
            bi[i] = bi[i2];
            i = i2;
        }
    }
    bv[i] = bv[k];
    bi[i] = bi[k];
}
/* Heap.h:84-105 */
static void heap_push_(int cmax, size_t k, float* bv, int64_t* bi, float val, int64_t id) {
    bv--;
    bi--;
    size_t i = k, f;
    while (i > 1) {
        f = i >> 1;
        if (!cmp2_(cmax, val, bv[f], id, bi[f])) break;
        bv[i] = bv[f];
        bi[i] = bi[f];
        i = f;
    }
    bv[i] = val;
    bi[i] = id;
}
/* Heap.h:112-149 */
void oracle_heap_replace_top(int cmax, size_t k, float* bv, int64_t* bi, float val, int64_t id) {
    bv--;
    bi--;
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k) break;
        if ((i2 == k + 1) || cmp2_(cmax, bv[i1], bv[i2], bi[i1], bi[i2])) {
            if (cmp2_(cmax, val, bv[i1], id, bi[i1])) break;
            bv[i] = bv[i1];
            bi[i] = bi[i1];
            i = i1;
        } else {
            if (cmp2_(cmax, val, bv[i2], id, bi[i2])) break;
            bv[i] = bv[i2];
            bi[i] = bi[i2];
            i = i2;
        }
    }
    bv[i] = val;
    bi[i] = id;
}
/* Heap.h:316-339 (k0 = 0) */
void oracle_heap_heapify(int cmax, size_t k, float* bv, int64_t* bi) {
    for (size_t i = 0; i < k; i++) {
        bv[i] = neutral_(cmax);
        bi[i] = -1;
    }
}
/* Heap.h:366-390 */
void oracle_heap_addn(int cmax, size_t k, float* bv, int64_t* bi, const float* x,
                      const int64_t* xids, size_t n) {
    for (size_t i = 0; i < n; i++)
        if (cmp_(cmax, bv[0], x[i]))
            oracle_heap_replace_top(cmax, k, bv, bi, x[i], xids ? xids[i] : (int64_t)i);
}
/* Heap.h:421-450 */
size_t oracle_heap_reorder(int cmax, size_t k, float* bv, int64_t* bi) {
    size_t i, ii;
    for (i = 0, ii = 0; i < k; i++) {
        float val = bv[0];
        int64_t id = bi[0];
        heap_pop_(cmax, k - i, bv, bi);
        bv[k - ii - 1] = val;
        bi[k - ii - 1] = id;
        if (id != -1) ii++;
    }
    size_t nel = ii;
    memmove(bv, bv + k - ii, ii * sizeof(*bv));
    memmove(bi, bi + k - ii, ii * sizeof(*bi));
    for (; ii < k; ii++) {
        bv[ii] = neutral_(cmax);
        bi[ii] = -1;
    }
    return nel;
}

/* ------------------------------------------------------------ kNN */
/* faiss/utils/distances.cpp:170-199 / 259-342 with HeapBlockResultHandler */
void oracle_knn(const float* x, const float* y, size_t d, size_t nx, size_t ny, size_t k,
                int metric, int blas_form, float* D, int64_t* I, int nthreads) {
    const int cmax = metric == 1;
    float* yn = NULL;
    if (metric == 1 && blas_form) {
        yn = (float*)malloc(sizeof(float) * (ny ? ny : 1));
        for (size_t j = 0; j < ny; j++) yn[j] = oracle_fvec_norm_L2sqr(y + j * d, d);
    }
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 16)
    for (int64_t i = 0; i < (int64_t)nx; i++) {
        const float* xi = x + i * d;
        float* hv = D + i * k;
        int64_t* hi = I + i * k;
        oracle_heap_heapify(cmax, k, hv, hi);
        float xn = (metric == 1 && blas_form) ? oracle_fvec_norm_L2sqr(xi, d) : 0.f;
        float thr = hv[0];
        for (size_t j = 0; j < ny; j++) {
            const float* yj = y + j * d;
            float dis;
            if (metric == 1) {
                if (blas_form) {
                    float ip = oracle_ip_seq(xi, yj, d);
                    dis = fmaf(-2.f, ip, xn + yn[j]);
                    if (dis < 0) dis = 0;
                } else {
                    dis = oracle_fvec_L2sqr(xi, yj, d);
                }
            } else {
                dis = blas_form ? oracle_ip_seq(xi, yj, d) : oracle_fvec_inner_product(xi, yj, d);
            }
            if (cmp_(cmax, thr, dis)) {
                oracle_heap_replace_top(cmax, k, hv, hi, dis, (int64_t)j);
                thr = hv[0];
            }
        }
        oracle_heap_reorder(cmax, k, hv, hi);
    }
    free(yn);
}

/* ------------------------------------------------------------ HNSW */
/* MinimaxHeap on CMax<float, int32> (faiss/impl/HNSW.cpp:1096-1342) */
typedef struct {
    int n, k, nvalid;
    int32_t* ids;
    float* dis;
} mmheap_t;

static inline int cmp2i_(float a1, float b1, int32_t a2, int32_t b2) {
    return a1 > b1 || (a1 == b1 && a2 > b2);
}
static void hpop_i(size_t k, float* bv, int32_t* bi) {
    bv--;
    bi--;
    float val = bv[k];
    int32_t id = bi[k];
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k) break;
        if ((i2 == k + 1) || cmp2i_(bv[i1], bv[i2], bi[i1], bi[i2])) {
            if (cmp2i_(val, bv[i1], id, bi[i1])) break;
            bv[i] = bv[i1];
            bi[i] = bi[i1];
            i = i1;
        } else {
            if (cmp2i_(val, bv[i2], id, bi[i2])) break;
            bv[i] = bv[i2];
            bi[i] = bi[i2];
            i = i2;
        }
    }
    bv[i] = bv[k];
    bi[i] = bi[k];
}
static void hpush_i(size_t k, float* bv, int32_t* bi, float val, int32_t id) {
    bv--;
    bi--;
    size_t i = k, f;
    while (i > 1) {
        f = i >> 1;
        if (!cmp2i_(val, bv[f], id, bi[f])) break;
        bv[i] = bv[f];
        bi[i] = bi[f];
        i = f;
    }
    bv[i] = val;
    bi[i] = id;
}
static void mm_push(mmheap_t* h, int32_t i, float v) {
    if (h->k == h->n) {
        if (v >= h->dis[0]) return;
        if (h->ids[0] != -1) --h->nvalid;
        hpop_i(h->k--, h->dis, h->ids);
    }
    hpush_i(++h->k, h->dis, h->ids, v, i);
    ++h->nvalid;
}
static int32_t mm_pop_min(mmheap_t* h, float* vmin_out) {
    int i = h->k - 1;
    while (i >= 0) {
        if (h->ids[i] != -1) break;
        i--;
    }
    if (i == -1) return -1;
    int imin = i;
    float vmin = h->dis[i];
    i--;
    while (i >= 0) {
        if (h->ids[i] != -1 && h->dis[i] < vmin) {
            vmin = h->dis[i];
            imin = i;
        }
        i--;
    }
    if (vmin_out) *vmin_out = vmin;
    int32_t ret = h->ids[imin];
    h->ids[imin] = -1;
    --h->nvalid;
    return ret;
}
static int mm_count_below(const mmheap_t* h, float thresh) {
    int n = 0;
    for (int i = 0; i < h->k; i++)
        if (h->dis[i] < thresh) n++;
    return n;
}

static void hnsw_range(const oracle_hnsw_t* g, int64_t no, int level, size_t* b, size_t* e) {
    size_t o = g->offsets[no];
    *b = o + g->cum_nneighbor_per_level[level];
    *e = o + g->cum_nneighbor_per_level[level + 1];
}

/* one query: HNSW::search with a HeapBlockResultHandler<CMax> of size k */
static void hnsw_search_one(const oracle_hnsw_t* g, const float* q, size_t k, int efSearch,
                            float* hv, int64_t* hi, uint8_t* visited) {
    oracle_heap_heapify(1, k, hv, hi);
    if (g->entry_point != -1) {
        const int d = g->d;
        int32_t nearest = g->entry_point;
        float d_nearest = oracle_fvec_L2sqr(q, g->storage + (size_t)nearest * d, d);
        /* greedy_update_nearest (HNSW.cpp:852-924) */
        for (int level = g->max_level; level >= 1; level--) {
            for (;;) {
                int32_t prev = nearest;
                size_t b, e;
                hnsw_range(g, nearest, level, &b, &e);
                for (size_t j = b; j < e; j++) {
                    int32_t v = g->neighbors[j];
                    if (v < 0) break;
                    float dv = oracle_fvec_L2sqr(q, g->storage + (size_t)v * d, d);
                    if (dv < d_nearest) {
                        nearest = v;
                        d_nearest = dv;
                    }
                }
                if (nearest == prev) break;
            }
        }
        int ef = efSearch > (int)k ? efSearch : (int)k;
        mmheap_t h;
        h.n = ef;
        h.k = 0;
        h.nvalid = 0;
        h.ids = (int32_t*)malloc(sizeof(int32_t) * ef);
        h.dis = (float*)malloc(sizeof(float) * ef);
        mm_push(&h, nearest, d_nearest);
        /* search_from_candidates (HNSW.cpp:605-741) */
        float threshold = hv[0];
        for (int i = 0; i < h.nvalid; i++) {
            int32_t v1 = h.ids[i];
            float dd = h.dis[i];
            if (dd < threshold) {
                if (cmp_(1, hv[0], dd)) {
                    oracle_heap_replace_top(1, k, hv, hi, dd, v1);
                    threshold = hv[0];
                }
            }
            visited[v1] = 1;
        }
        int32_t* buf = (int32_t*)malloc(sizeof(int32_t) * 1024);
        while (h.nvalid > 0) {
            float d0 = 0;
            int32_t v0 = mm_pop_min(&h, &d0);
            if (mm_count_below(&h, d0) >= efSearch) break;
            size_t b, e;
            hnsw_range(g, v0, 0, &b, &e);
            size_t jmax = b;
            for (size_t j = b; j < e; j++) {
                if (g->neighbors[j] < 0) break;
                jmax++;
            }
            threshold = hv[0];
            int nb = 0;
            for (size_t j = b; j < jmax; j++) {
                int32_t v1 = g->neighbors[j];
                int vget = visited[v1];
                visited[v1] = 1;
                if (!vget) buf[nb++] = v1;
            }
            for (int t = 0; t < nb; t++) {
                int32_t v1 = buf[t];
                float dis = oracle_fvec_L2sqr(q, g->storage + (size_t)v1 * d, d);
                if (dis < threshold) {
                    if (cmp_(1, hv[0], dis)) {
                        oracle_heap_replace_top(1, k, hv, hi, dis, v1);
                        threshold = hv[0];
                    }
                }
                mm_push(&h, v1, dis);
            }
        }
        free(buf);
        free(h.ids);
        free(h.dis);
    }
    oracle_heap_reorder(1, k, hv, hi);
}

void oracle_hnsw_search(const oracle_hnsw_t* g, const float* x, size_t n, size_t k,
                        int efSearch, float* D, int64_t* I, int nthreads) {
#pragma omp parallel num_threads(nthreads)
    {
        uint8_t* visited = (uint8_t*)calloc(g->ntotal > 0 ? g->ntotal : 1, 1);
#pragma omp for schedule(dynamic, 4)
        for (int64_t i = 0; i < (int64_t)n; i++) {
            memset(visited, 0, g->ntotal > 0 ? g->ntotal : 1);
            hnsw_search_one(g, x + i * g->d, k, efSearch, D + i * k, I + i * k, visited);
        }
        free(visited);
    }
}

/* ------------------------------------------------------------ IVF-PQ */
/* PQ table entries: fvec_inner_products_ny / fvec_L2sqr_ny
 * (faiss/utils/distances_simd.cpp:1362-1410) as the AVX2 build compiles them:
 * dsub 1: one rounded product; dsub 2/4/8: fvec_op_ny_D{2,4,8} AVX2
 * specialisations (:579-702, :845-975, :1167-1341; ksub = 256 is a multiple of
 * 8, so the 8-row transposed loop covers every row): acc = t0 (rounded), then
 * acc = fma(., ., acc) over dims 1..dsub-1; dsub 12: fvec_op_ny_D12 (:1344-1360,
 * three rounded 4-lane terms added per lane, then horizontal_sum); any other
 * dsub: the _ref loops (:160-190), i.e. fvec_L2sqr / fvec_inner_product. */
static float ny_term_(const float* x, const float* y, int dsub, int l2) {
    switch (dsub) {
        case 1: {
            if (l2) {
                const float t = x[0] - y[0];
                return t * t;
            }
            return x[0] * y[0];
        }
        case 2:
        case 4:
        case 8: {
            float acc;
            if (l2) {
                const float t = x[0] - y[0];
                acc = t * t;
            } else {
                acc = x[0] * y[0];
            }
            for (int j = 1; j < dsub; j++) {
                if (l2) {
                    const float t = x[j] - y[j];
                    acc = fmaf(t, t, acc);
                } else {
                    acc = fmaf(x[j], y[j], acc);
                }
            }
            return acc;
        }
        case 12: {
            float a[4];
            for (int j = 0; j < 4; j++) {
                float t0, t1, t2;
                if (l2) {
                    const float u0 = x[j] - y[j], u1 = x[4 + j] - y[4 + j], u2 = x[8 + j] - y[8 + j];
                    t0 = u0 * u0, t1 = u1 * u1, t2 = u2 * u2;
                } else {
                    t0 = x[j] * y[j], t1 = x[4 + j] * y[4 + j], t2 = x[8 + j] * y[8 + j];
                }
                a[j] = (t0 + t1) + t2;
            }
            return (a[0] + a[2]) + (a[1] + a[3]);
        }
        default:
            return ref_dist_(x, y, (size_t)dsub, l2);
    }
}
float oracle_pq_ny_ip(const float* x, const float* y, int dsub) { return ny_term_(x, y, dsub, 0); }
float oracle_pq_ny_l2(const float* x, const float* y, int dsub) { return ny_term_(x, y, dsub, 1); }

/* distance_single_code / distance_four_codes with PQDecoder8 as the AVX2 build
 * compiles them (faiss/impl/code_distance/code_distance-avx2.h:253-347,
 * :383-530; both give the same value per code):
 *   M = 4: horizontal_sum of the 4 gathered entries, (t0+t2)+(t1+t3) (:42-79);
 *   M = 8: horizontal_sum of 8, ((t0+t4)+(t2+t6))+((t1+t5)+(t3+t7)) (:82-119);
 *   M >= 16: 8 lanes, lane l accumulates t[16i+l] then t[16i+8+l] for each
 *   16-block i in order, reduced as the M = 8 case; then the M % 16 leftover
 *   entries are added one by one (:270-346);
 *   other M < 16: 0 + t0 + t1 + ... in order. */
float oracle_pq_code_sum(int M, const float* sim, int ksub, const uint8_t* code) {
    if (M == 4) {
        const float t0 = sim[code[0]], t1 = sim[ksub + code[1]];
        const float t2 = sim[2 * ksub + code[2]], t3 = sim[3 * ksub + code[3]];
        return (t0 + t2) + (t1 + t3);
    }
    float r = 0.f;
    int m = 0;
    if (M == 8 || M >= 16) {
        float p[8];
        for (int l = 0; l < 8; l++) p[l] = sim[(size_t)l * ksub + code[l]];
        m = 8;
        if (M != 8) {
            const int m16 = M / 16 * 16;
            for (; m < m16; m += 8)
                for (int l = 0; l < 8; l++) p[l] += sim[(size_t)(m + l) * ksub + code[m + l]];
        }
        r = ((p[0] + p[4]) + (p[2] + p[6])) + ((p[1] + p[5]) + (p[3] + p[7]));
    }
    for (; m < M; m++) r += sim[(size_t)m * ksub + code[m]];
    return r;
}

/* ProductQuantizer::compute_code for dsub < 16 (faiss/impl/ProductQuantizer.cpp:
 * 195-271): fvec_L2sqr_ny_nearest per sub-quantizer.  dsub 2/4/8: the AVX2
 * _D{2,4,8} kernels (faiss/utils/distances_simd.cpp:1908-2271): 8 lanes keep
 * `old < new ? old : new` (an equal later distance takes the lane), lanes
 * scanned 0..7 with a strict `>`; other dsub: fvec_L2sqr_ny + first strict
 * minimum (:2298-2317, :125-140). */
static int pq_nearest_(const float* x, const float* cent, int dsub, int ksub) {
    if (dsub == 2 || dsub == 4 || dsub == 8) {
        float lmin[8];
        int lidx[8];
        for (int l = 0; l < 8; l++) lmin[l] = HUGE_VALF, lidx[l] = 0;
        for (int j = 0; j < ksub; j++) {
            const float s = ny_term_(x, cent + (size_t)j * dsub, dsub, 1);
            const int l = j & 7;
            if (!(lmin[l] < s)) lmin[l] = s, lidx[l] = j;
        }
        float cur = HUGE_VALF;
        int idx = 0;
        for (int l = 0; l < 8; l++)
            if (cur > lmin[l]) cur = lmin[l], idx = lidx[l];
        return idx;
    }
    float best = HUGE_VALF;
    int idx = 0;
    for (int j = 0; j < ksub; j++) {
        const float s = ny_term_(x, cent + (size_t)j * dsub, dsub, 1);
        if (s < best) best = s, idx = j;
    }
    return idx;
}

/* IndexIVFPQ::encode_vectors (faiss/IndexIVFPQ.cpp:142-190): residual x - y_C
 * (Index::compute_residual; zeros for list_no < 0) when by_residual, then
 * compute_codes.  codes: [n][M] bytes. */
void oracle_ivfpq_encode(const oracle_ivf_t* ivf, size_t n, const float* x,
                         const int64_t* list_nos, uint8_t* codes) {
    const int M = ivf->pq_M, ksub = 1 << ivf->pq_nbits, d = ivf->d, dsub = d / M;
#pragma omp parallel
    {
        float* r = (float*)malloc(sizeof(float) * d);
#pragma omp for
        for (int64_t i = 0; i < (int64_t)n; i++) {
            const float* xi = x + i * d;
            if (ivf->by_residual) {
                const int64_t key = list_nos[i];
                if (key < 0) {
                    memset(r, 0, sizeof(float) * d);
                } else {
                    const float* c = ivf->hnsw ? ivf->hnsw->storage + key * d
                                               : ivf->centroids + key * d;
                    for (int j = 0; j < d; j++) r[j] = xi[j] - c[j];
                }
            } else {
                memcpy(r, xi, sizeof(float) * d);
            }
            for (int m = 0; m < M; m++)
                codes[i * M + m] = (uint8_t)pq_nearest_(
                        r + m * dsub, ivf->pq_centroids + (size_t)m * ksub * dsub, dsub, ksub);
        }
        free(r);
    }
}

void oracle_ivfpq_prepare(oracle_ivf_t* ivf) {
    /* faiss/IndexIVFPQ.cpp:380-406 decision, :408-432 table 1:
     * P[key][m][j] = fvec_madd(r_norms, 2.0, <y_C,m, c_mj>) = fma(2, ip, |c_mj|^2)
     * (fvec_madd AVX2, distances_simd.cpp:3292-3345, is one fma per entry) */
    const int M = ivf->pq_M, ksub = 1 << ivf->pq_nbits, d = ivf->d, dsub = d / M;
    ivf->use_precomputed_table = 0;
    if (!(ivf->metric == 1 && ivf->by_residual)) return;
    size_t table_size = (size_t)M * ksub * ivf->nlist * sizeof(float);
    if (table_size > ((size_t)1 << 31)) return;
    ivf->use_precomputed_table = 1;
    float* rn = (float*)malloc(sizeof(float) * M * ksub);
    for (int m = 0; m < M; m++)
        for (int j = 0; j < ksub; j++)
            rn[m * ksub + j] = oracle_fvec_norm_L2sqr(ivf->pq_centroids + ((size_t)m * ksub + j) * dsub,
                                                      dsub);
    ivf->precomputed_table = (float*)malloc(table_size);
#pragma omp parallel for
    for (int64_t i = 0; i < ivf->nlist; i++) {
        const float* c = ivf->hnsw ? ivf->hnsw->storage + i * d : ivf->centroids + i * d;
        float* tab = ivf->precomputed_table + (size_t)i * M * ksub;
        for (int m = 0; m < M; m++)
            for (int j = 0; j < ksub; j++) {
                const float ip =
                        ny_term_(c + m * dsub, ivf->pq_centroids + ((size_t)m * ksub + j) * dsub, dsub, 0);
                tab[m * ksub + j] = fmaf(2.f, ip, rn[m * ksub + j]);
            }
    }
    free(rn);
}

/* QueryTables (faiss/IndexIVFPQ.cpp:483-751) for one query: init_query
 * (:545-566) fills sim2 (table 1: <x_m, c>) or sim (not by residual: the
 * distance / inner-product table of x, also the IP table by residual). */
static void pq_init_query_(const oracle_ivf_t* ivf, const float* xi, float* sim, float* sim2) {
    const int M = ivf->pq_M, ksub = 1 << ivf->pq_nbits, dsub = ivf->d / M;
    const int l2 = ivf->metric == 1;
    for (int m = 0; m < M; m++)
        for (int j = 0; j < ksub; j++) {
            const float* c = ivf->pq_centroids + ((size_t)m * ksub + j) * dsub;
            if (!l2)
                sim[m * ksub + j] = ny_term_(xi + m * dsub, c, dsub, 0);
            else if (!ivf->by_residual)
                sim[m * ksub + j] = ny_term_(xi + m * dsub, c, dsub, 1);
            else if (ivf->use_precomputed_table == 1)
                sim2[m * ksub + j] = ny_term_(xi + m * dsub, c, dsub, 0);
        }
}
/* precompute_list_tables (:604-700): returns dis0 and fills sim for list key */
static float pq_set_list_(const oracle_ivf_t* ivf, const float* xi, int64_t key, float cdis,
                          float* sim, const float* sim2, float* resid) {
    const int M = ivf->pq_M, ksub = 1 << ivf->pq_nbits, d = ivf->d, dsub = d / M;
    if (!ivf->by_residual) return 0.f;
    const float* c = ivf->hnsw ? ivf->hnsw->storage + key * d : ivf->centroids + key * d;
    if (ivf->metric != 1) /* precompute_list_tables_IP (:612-628) */
        return oracle_fvec_inner_product(xi, c, d);
    if (ivf->use_precomputed_table == 1) {
        const float* P = ivf->precomputed_table + (size_t)key * M * ksub;
        for (int e = 0; e < M * ksub; e++) sim[e] = fmaf(-2.f, sim2[e], P[e]);
        return cdis;
    }
    for (int j = 0; j < d; j++) resid[j] = xi[j] - c[j]; /* Index::compute_residual */
    for (int m = 0; m < M; m++)
        for (int j = 0; j < ksub; j++)
            sim[m * ksub + j] = ny_term_(resid + m * dsub,
                                         ivf->pq_centroids + ((size_t)m * ksub + j) * dsub, dsub, 1);
    return 0.f;
}

/* ------------------------------------------------------------ preassigned */
/* faiss/IndexIVF.cpp:595-631 (parallel_mode 0): probes in coarse order; with
 * max_codes > 0 a list is cut to max_codes - nscan rows (scan_one_list's
 * list_size_max, :546-550) and the scan stops once nscan >= max_codes. */
void oracle_ivf_search_preassigned(const oracle_ivf_t* ivf, size_t n, const float* x, size_t k,
                                   size_t nprobe, const int64_t* keys, const float* coarse_dis,
                                   float* D, int64_t* I, int nthreads) {
    oracle_ivf_search_preassigned_mc(ivf, n, x, k, nprobe, keys, coarse_dis, 0, D, I, NULL,
                                     nthreads);
}

void oracle_ivf_search_preassigned_mc(const oracle_ivf_t* ivf, size_t n, const float* x,
                                      size_t k, size_t nprobe, const int64_t* keys,
                                      const float* coarse_dis, int64_t max_codes, float* D,
                                      int64_t* I, int64_t* ndis, int nthreads) {
    int64_t ndis_tot = 0;
    const int cmax = ivf->metric == 1;
    const int d = ivf->d;
    const int M = ivf->pq_M;
    const int ksub = M ? 1 << ivf->pq_nbits : 0;
#pragma omp parallel num_threads(nthreads)
    {
        float* sim2 = M ? (float*)malloc(sizeof(float) * M * ksub) : NULL;
        float* sim = M ? (float*)malloc(sizeof(float) * M * ksub) : NULL;
        float* resid = (float*)malloc(sizeof(float) * d);
#pragma omp for schedule(dynamic, 8) reduction(+ : ndis_tot)
        for (int64_t i = 0; i < (int64_t)n; i++) {
            const float* xi = x + i * d;
            int64_t nscan = 0;
            float* hv = D + i * k;
            int64_t* hi = I + i * k;
            oracle_heap_heapify(cmax, k, hv, hi);
            if (M) pq_init_query_(ivf, xi, sim, sim2);
            for (size_t ik = 0; ik < nprobe; ik++) {
                int64_t key = keys[i * nprobe + ik];
                if (key < 0 || key >= ivf->nlist) continue;
                int64_t l0 = ivf->list_off[key], l1 = ivf->list_off[key + 1];
                if (l1 == l0) continue;
                if (max_codes > 0 && l1 - l0 > max_codes - nscan) l1 = l0 + (max_codes - nscan);
                nscan += l1 - l0;
                if (!M) {
                    /* IVFFlatScanner::scan_codes */
                    for (int64_t j = l0; j < l1; j++) {
                        const float* yj = (const float*)(ivf->codes + j * ivf->code_size);
                        float dis = cmax ? oracle_fvec_L2sqr(xi, yj, d)
                                         : oracle_fvec_inner_product(xi, yj, d);
                        if (cmp_(cmax, hv[0], dis))
                            oracle_heap_replace_top(cmax, k, hv, hi, dis, ivf->ids[j]);
                    }
                } else {
                    const float dis0 = pq_set_list_(ivf, xi, key, coarse_dis[i * nprobe + ik],
                                                    sim, sim2, resid);
                    for (int64_t j = l0; j < l1; j++) {
                        const uint8_t* code = ivf->codes + j * ivf->code_size;
                        const float dis = dis0 + oracle_pq_code_sum(M, sim, ksub, code);
                        if (cmp_(cmax, hv[0], dis))
                            oracle_heap_replace_top(cmax, k, hv, hi, dis, ivf->ids[j]);
                    }
                }
                if (max_codes > 0 && nscan >= max_codes) break;
            }
            ndis_tot += nscan;
            oracle_heap_reorder(cmax, k, hv, hi);
        }
        free(sim2);
        free(sim);
        free(resid);
    }
    if (ndis) *ndis = ndis_tot;
}

void oracle_ivf_search(const oracle_ivf_t* ivf, size_t n, const float* x, size_t k,
                       size_t nprobe, int efSearch, int nslices, float* D, int64_t* I,
                       int64_t* coarse_I, float* coarse_D, int nthreads) {
    if (nprobe > (size_t)ivf->nlist) nprobe = ivf->nlist;
    int nt = nslices < (int)n ? nslices : (int)n;
    if (nt < 1) nt = 1;
    for (int s = 0; s < nt; s++) {
        size_t i0 = n * s / nt, i1 = n * (s + 1) / nt;
        size_t ns = i1 - i0;
        if (!ns) continue;
        const float* xs = x + i0 * ivf->d;
        int64_t* ci = coarse_I + i0 * nprobe;
        float* cd = coarse_D + i0 * nprobe;
        if (ivf->hnsw)
            oracle_hnsw_search(ivf->hnsw, xs, ns, nprobe, efSearch, cd, ci, nthreads);
        else
            oracle_knn(xs, ivf->centroids, ivf->d, ns, ivf->nlist, nprobe, ivf->metric,
                       ns >= 20, cd, ci, nthreads);
        oracle_ivf_search_preassigned(ivf, ns, xs, k, nprobe, ci, cd, D + i0 * k, I + i0 * k,
                                      nthreads);
    }
}

/* ------------------------------------------------------------ fast path */
/* the reference order (ref_dist_: 8 independent fma lanes) vectorises as
 * the reference's own compiled loop does */
static inline float l2_fast(const float* x, const float* y, int d) {
    return ref_dist_(x, y, (size_t)d, 1);
}

void oracle_ivf_search_fast(const oracle_ivf_t* ivf, size_t n, const float* x, size_t k,
                            size_t nprobe, float* D, int64_t* I, int nthreads) {
    int64_t* ci = (int64_t*)malloc(sizeof(int64_t) * n * nprobe);
    float* cd = (float*)malloc(sizeof(float) * n * nprobe);
    oracle_knn(x, ivf->centroids, ivf->d, n, ivf->nlist, nprobe, 1, 1, cd, ci, nthreads);
    const int d = ivf->d;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 8)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        const float* xi = x + i * d;
        float* hv = D + i * k;
        int64_t* hi = I + i * k;
        oracle_heap_heapify(1, k, hv, hi);
        for (size_t ik = 0; ik < nprobe; ik++) {
            int64_t key = ci[i * nprobe + ik];
            if (key < 0) continue;
            for (int64_t j = ivf->list_off[key]; j < ivf->list_off[key + 1]; j++) {
                float dis = l2_fast(xi, (const float*)(ivf->codes + j * ivf->code_size), d);
                if (hv[0] > dis) oracle_heap_replace_top(1, k, hv, hi, dis, ivf->ids[j]);
            }
        }
        oracle_heap_reorder(1, k, hv, hi);
    }
    free(ci);
    free(cd);
}

/* ------------------------------------------------------------ merge */
/* faiss/utils/Heap.cpp:159-230 with heap_push/heap_pop on (dist, shard):
 * CMin<float,int> for L2, CMax<float,int> for IP. */
void oracle_merge_knn_results(size_t n, size_t k, int nshard, const float* all_d,
                              const int64_t* all_l, float* D, int64_t* L, int metric) {
    const int cmax = metric != 1; /* L2 -> CMin heap */
    const size_t stride = n * k;
    int* pointer = (int*)malloc(sizeof(int) * nshard);
    int64_t* shard_ids = (int64_t*)malloc(sizeof(int64_t) * nshard);
    float* heap_vals = (float*)malloc(sizeof(float) * nshard);
    for (size_t i = 0; i < n; i++) {
        const float* Din = all_d + i * k;
        const int64_t* Iin = all_l + i * k;
        int heap_size = 0;
        for (int s = 0; s < nshard; s++) {
            pointer[s] = 0;
            if (Iin[stride * s] >= 0)
                heap_push_(cmax, ++heap_size, heap_vals, shard_ids, Din[stride * s], s);
        }
        float* Do = D + i * k;
        int64_t* Io = L + i * k;
        size_t j;
        for (j = 0; j < k && heap_size > 0; j++) {
            int s = (int)shard_ids[0];
            int* p = &pointer[s];
            Do[j] = heap_vals[0];
            Io[j] = Iin[stride * s + *p];
            heap_pop_(cmax, heap_size--, heap_vals, shard_ids);
            (*p)++;
            if ((size_t)*p < k && Iin[stride * s + *p] >= 0)
                heap_push_(cmax, ++heap_size, heap_vals, shard_ids, Din[stride * s + *p], s);
        }
        for (; j < k; j++) {
            Io[j] = -1;
            Do[j] = metric == 1 ? FLT_MAX : -FLT_MAX;
        }
    }
    free(pointer);
    free(shard_ids);
    free(heap_vals);
}

/* IVF range search, parallel_mode 0 (faiss/IndexIVF.cpp:1243-1400 with
 * IVFFlatScanner::scan_codes_range, faiss/IndexIVFFlat.cpp:181-201, and
 * IVFPQScanner::scan_codes_range, faiss/IndexIVFPQ.cpp:1254-1279 with
 * RangeSearchResults :780-799 — the same tables as the k-NN scan above): per
 * query, probes in order, rows in list order; a row is kept when
 * C::cmp(radius, dis) (L2: dis < radius, IP: dis > radius) and, with a
 * selector mask (per concatenated row, may be NULL), when it is a member.
 * Writes lims[n+1]; D/I are written up to `cap` entries; returns the total.
 * PQ: L2 and inner product. */
int64_t oracle_ivf_range_preassigned(const oracle_ivf_t* ivf, size_t n, const float* x,
                                     size_t nprobe, const int64_t* keys,
                                     const float* coarse_dis, float radius,
                                     const uint8_t* selmask, size_t* lims, float* D, int64_t* I,
                                     int64_t cap) {
    const int l2 = ivf->metric == 1;
    const int d = ivf->d;
    const int M = ivf->pq_M;
    const int ksub = M ? 1 << ivf->pq_nbits : 0;
    float* sim = M ? (float*)malloc(sizeof(float) * M * ksub) : NULL;
    float* sim2 = M ? (float*)malloc(sizeof(float) * M * ksub) : NULL;
    float* resid = (float*)malloc(sizeof(float) * d);
    int64_t tot = 0;
    for (size_t i = 0; i < n; i++) {
        lims[i] = (size_t)tot;
        const float* xi = x + i * d;
        if (M) pq_init_query_(ivf, xi, sim, sim2);
        for (size_t ik = 0; ik < nprobe; ik++) {
            const int64_t key = keys[i * nprobe + ik];
            if (key < 0 || key >= ivf->nlist) continue;
            const float dis0 =
                    M ? pq_set_list_(ivf, xi, key, coarse_dis[i * nprobe + ik], sim, sim2, resid)
                      : 0.f;
            for (int64_t r = ivf->list_off[key]; r < ivf->list_off[key + 1]; r++) {
                if (selmask && !selmask[r]) continue;
                float dis;
                if (M) {
                    const uint8_t* code = ivf->codes + (size_t)r * ivf->code_size;
                    dis = dis0 + oracle_pq_code_sum(M, sim, ksub, code);
                } else {
                    const float* y = (const float*)(ivf->codes + (size_t)r * ivf->code_size);
                    dis = ref_dist_(xi, y, d, l2);
                }
                if (l2 ? (dis < radius) : (radius < dis)) {
                    if (tot < cap) {
                        D[tot] = dis;
                        I[tot] = ivf->ids[r];
                    }
                    tot++;
                }
            }
        }
    }
    lims[n] = (size_t)tot;
    free(sim);
    free(sim2);
    free(resid);
    return tot;
}
