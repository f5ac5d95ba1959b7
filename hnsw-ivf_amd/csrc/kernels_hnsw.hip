// kernels_hnsw.hip — HNSW coarse-quantizer search, one wavefront per query.
//
// Reference semantics (faiss/impl/HNSW.cpp):
//   * HNSW::search (:943-996): greedy descent max_level..1 from the entry
//     point, then search_from_candidates at level 0 with a MinimaxHeap of
//     capacity ef = max(efSearch, k) and a k-result heap.
//   * greedy_update_nearest (:852-924): move to the closest neighbour while
//     it is strictly closer.
//   * search_from_candidates (:605-741): pop_min, stop when
//     count_below(d0) >= efSearch (the raw efSearch, not ef), visit
//     unvisited neighbours in stored order, add each to the result heap when
//     dis < threshold and push it to the candidate heap.
//   * MinimaxHeap (:1096-1342): push into a full heap drops v >= max and
//     otherwise evicts the max (popped "dead" slots included); pop_min marks
//     the slot dead; count_below counts every slot, dead ones included.
//
// GPU form: a hop's new neighbours are handled as one batch.  For distinct
// distances the sequential bounded-heap updates are equivalent to keeping the
// ef (resp. k) smallest of the union, so both heaps are wave64 bitonic queues:
// the candidate set is a sorted 128-slot queue (2 slots per lane, positions >=
// ef are the evicted ones), the result set a sorted 64-slot queue.  Distances
// are one sequential fma chain per lane, the same order as the CPU oracle.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "common.h"
#include "kernels.h"
#include "ref_arith.h"
#include "wave_select.h"

namespace faiss_amd {
namespace kern {

// faiss FlatL2Dis (faiss/IndexFlat.cpp:111-170): fvec_L2sqr and
// fvec_L2sqr_batch_4 evaluate in the same reference order (ref_arith.h)
__device__ __forceinline__ float l2_row(const float* __restrict__ qs, const float* __restrict__ y,
                                        int d) {
    return ref_l2(qs, y, d);
}

// merge a sorted 64-batch into a sorted 128-queue (c0: positions 0..63,
// c1: 64..127), keeping the 128 smallest.
__device__ __forceinline__ void merge128(float& d0, long long& i0, float& d1, long long& i1,
                                         float bd, long long bi, int lane) {
    float rd = __shfl(bd, 63 - lane);
    long long ri = shfl_ll(bi, 63 - lane);
    if (key_less(rd, ri, d1, i1)) {
        d1 = rd;
        i1 = ri;
    }
    // stride 64: in-lane
    if (key_less(d1, i1, d0, i0)) {
        float td = d0; long long ti = i0;
        d0 = d1; i0 = i1;
        d1 = td; i1 = ti;
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
        cas_lane(d0, i0, j, (lane & j) == 0);
        cas_lane(d1, i1, j, (lane & j) == 0);
    }
}

template <bool LDS_VISITED>
__global__ __launch_bounds__(64) void k_hnsw_search(HNSWDevice g, const float* __restrict__ x,
                                                    int ldx, int64_t n, int k, int efSearch,
                                                    int ef, float* __restrict__ D,
                                                    int64_t* __restrict__ I,
                                                    int32_t* __restrict__ I32,
                                                    uint32_t* __restrict__ vis_global,
                                                    int64_t vwords,
                                                    unsigned long long* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* qs = sm;  // [ld]
    uint32_t* vis = LDS_VISITED ? (uint32_t*)(sm + g.ld) : vis_global + blockIdx.x * vwords;
    const int lane = threadIdx.x;
    const int64_t q = blockIdx.x;
    for (int j = lane; j < g.ld; j += 64) qs[j] = j < g.d ? x[q * ldx + j] : 0.f;
    if (LDS_VISITED)
        for (int64_t w = lane; w < vwords; w += 64) vis[w] = 0u;
    __syncthreads();

    float res_d = WS_INF;
    long long res_i = WS_NOID;
    // HNSWStats (faiss/impl/HNSW.h:234-246): n1, n2, ndis, nhops of this query
    uint32_t st_n2 = 0, st_ndis = 0, st_nhops = 0;
    if (g.entry_point >= 0) {
        // ---- greedy descent on the upper levels
        int nearest = g.entry_point;
        float d_nearest = l2_row(qs, g.storage + (int64_t)nearest * g.ld, g.d);
        for (int level = g.max_level; level >= 1; level--) {
            for (;;) {
                const uint64_t o = g.offsets[nearest];
                const int b = g.cum_nb[level], e = g.cum_nb[level + 1];
                const int cnt = e - b;
                int v = lane < cnt ? g.neighbors[o + b + lane] : -1;
                unsigned long long neg = __ballot(lane < cnt && v < 0) | (cnt < 64 ? (~0ull << cnt) : 0ull);
                const int first_neg = neg ? __ffsll((long long)neg) - 1 : 64;
                float dis = WS_INF;
                if (lane < first_neg) dis = l2_row(qs, g.storage + (int64_t)v * g.ld, g.d);
                // greedy_update_nearest (HNSW.cpp:883-918): every valid
                // neighbour is a distance, every pass a hop
                st_ndis += (uint32_t)min(first_neg, 64);
                st_nhops += 1;
                // min (dis, lane) over the wave
                float md = dis;
                int ml = lane;
#pragma unroll
                for (int m = 32; m > 0; m >>= 1) {
                    float od = __shfl_xor(md, m);
                    int ol = __shfl_xor(ml, m);
                    if (od < md || (od == md && ol < ml)) {
                        md = od;
                        ml = ol;
                    }
                }
                if (md < d_nearest) {
                    d_nearest = md;
                    nearest = __shfl(v, ml);
                } else {
                    break;
                }
            }
        }
        // ---- level 0: bounded best-first search
        // candidate queue (128 sorted slots), key2 = (id << 1) | alive
        float c0d = WS_INF, c1d = WS_INF;
        long long c0i = WS_NOID, c1i = WS_NOID;
        if (lane == 0) {
            c0d = d_nearest;
            c0i = ((long long)nearest << 1) | 1;
        }
        // result heap: strict admission of the entry point (threshold FLT_MAX)
        {
            float cd = (lane == 0 && d_nearest < FLT_MAX) ? d_nearest : WS_INF;
            long long ci = (lane == 0 && d_nearest < FLT_MAX) ? (long long)nearest : WS_NOID;
            float td = WS_INF;
            long long ti = WS_NOID;
            wave_offer(res_d, res_i, cd, ci, td, ti, k, lane);
        }
        if (lane == 0) atomicOr(&vis[nearest >> 5], 1u << (nearest & 31));
        __syncthreads();
        for (;;) {
            // alive slots among the ef kept positions
            const bool in0 = lane < ef, in1 = 64 + lane < ef;
            const bool a0 = in0 && c0i != WS_NOID && (c0i & 1);
            const bool a1 = in1 && c1i != WS_NOID && (c1i & 1);
            unsigned long long m0 = __ballot(a0), m1 = __ballot(a1);
            if (!m0 && !m1) {  // candidates.size() == 0
                st_n2 = 1;
                break;
            }
            // pop_min: smallest alive slot
            int pos;
            if (m0) pos = __ffsll((long long)m0) - 1;
            else pos = 64 + __ffsll((long long)m1) - 1;
            float d0v = pos < 64 ? __shfl(c0d, pos) : __shfl(c1d, pos - 64);
            long long k0v = pos < 64 ? shfl_ll(c0i, pos) : shfl_ll(c1i, pos - 64);
            const int v0 = (int)(k0v >> 1);
            if (pos < 64) {
                if (lane == pos) c0i &= ~1ll;
            } else {
                if (lane == pos - 64) c1i &= ~1ll;
            }
            // count_below(d0) over every filled slot (dead included)
            const bool f0 = in0 && c0i != WS_NOID && c0d < d0v;
            const bool f1 = in1 && c1i != WS_NOID && c1d < d0v;
            const int n_below = __popcll(__ballot(f0)) + __popcll(__ballot(f1));
            if (n_below >= efSearch) {
                // HNSW.cpp:732-735: n2 counts an exhausted candidate heap
                const bool b0 = in0 && c0i != WS_NOID && (c0i & 1);
                const bool b1 = in1 && c1i != WS_NOID && (c1i & 1);
                st_n2 = (__ballot(b0) | __ballot(b1)) == 0ull ? 1u : 0u;
                break;
            }
            // neighbours of v0 at level 0
            const uint64_t o = g.offsets[v0];
            const int b = g.cum_nb[0], e = g.cum_nb[1];
            const int cnt = e - b;
            int v = lane < cnt ? g.neighbors[o + b + lane] : -1;
            unsigned long long neg = __ballot(lane < cnt && v < 0) | (cnt < 64 ? (~0ull << cnt) : 0ull);
            const int jmax = neg ? __ffsll((long long)neg) - 1 : 64;
            bool fresh = false;
            if (lane < jmax) {
                uint32_t bit = 1u << (v & 31);
                uint32_t old = atomicOr(&vis[v >> 5], bit);
                fresh = (old & bit) == 0;
            }
            float dis = WS_INF;
            if (fresh) dis = l2_row(qs, g.storage + (int64_t)v * g.ld, g.d);
            const unsigned long long fm = __ballot(fresh);
            st_ndis += (uint32_t)__popcll(fm);
            st_nhops += 1;  // nstep
            if (fm == 0ull) continue;
            // result heap: k smallest (dis, id) of the union, strict admission
            {
                float cd = (fresh && dis < FLT_MAX) ? dis : WS_INF;
                long long ci = (fresh && dis < FLT_MAX) ? (long long)v : WS_NOID;
                wave_offer_q(res_d, res_i, cd, ci, k, lane);
            }
            // candidate heap: ef smallest of the union (dead slots included)
            {
                float cd = fresh ? dis : WS_INF;
                long long ci = fresh ? (((long long)v << 1) | 1) : WS_NOID;
                wave_sort64(cd, ci, lane);
                merge128(c0d, c0i, c1d, c1i, cd, ci, lane);
            }
        }
    }
    if (stats && lane == 0 && g.entry_point >= 0) {
        atomicAdd(&stats[0], 1ull);
        atomicAdd(&stats[1], (unsigned long long)st_n2);
        atomicAdd(&stats[2], (unsigned long long)st_ndis);
        atomicAdd(&stats[3], (unsigned long long)st_nhops);
    }
    if (lane < k) {
        float dis;
        long long id;
        from_key(1, res_d, res_i, dis, id);
        if (D) D[q * k + lane] = dis;
        if (I) I[q * k + lane] = id;
        if (I32) I32[q * k + lane] = (int32_t)id;
    }
}

void hnsw_search(const HNSWDevice& g, const float* x, int ldx, int64_t n, int k, int efSearch,
                 float* D, int64_t* I, int32_t* I32, uint32_t* visited_scratch,
                 int64_t visited_words_per_query, unsigned long long* stats, hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT_MSG(k >= 1 && k <= kMaxK, "k must be in [1, 64] on this path");
    const int ef = efSearch > k ? efSearch : k;
    FAISS_THROW_IF_NOT_MSG(ef <= 128, "max(efSearch, k) must be <= 128 on this path");
    FAISS_THROW_IF_NOT(g.ld % 4 == 0);
    const int64_t vwords = visited_words_per_query;
    const size_t lds_q = sizeof(float) * g.ld;
    const bool lds_vis = vwords * 4 <= 64 * 1024;
    if (lds_vis) {
        size_t lds = lds_q + sizeof(uint32_t) * vwords;
        k_hnsw_search<true><<<dim3((unsigned)n), dim3(64), lds, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats);
    } else {
        FAISS_THROW_IF_NOT(visited_scratch != nullptr);
        HIP_CHECK(hipMemsetAsync(visited_scratch, 0, sizeof(uint32_t) * vwords * n, s));
        k_hnsw_search<false><<<dim3((unsigned)n), dim3(64), lds_q, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats);
    }
    HIP_LAUNCH_CHECK();
}

}  // namespace kern
}  // namespace faiss_amd
