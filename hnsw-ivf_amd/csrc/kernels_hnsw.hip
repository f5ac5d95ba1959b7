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
                                                    unsigned long long* __restrict__ stats,
                                                    uint32_t* __restrict__ tie_flags) {
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
    bool tie = false;  // an exact distance tie where the batched form may differ
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
            // Ties: the sequential heaps (strict admission, MinimaxHeap's
            // push / pop_min rules) and the batched union agree only for
            // distinct distances.  A fresh distance equal to the current k-th
            // result or ef-th candidate, or two equal distances among the ef
            // kept candidates (checked after the merge below), flags the query
            // for the sequential kernel (k_hnsw_exact).
            {
                const float kth = __shfl(res_d, k - 1);
                const float eth = ef <= 64 ? __shfl(c0d, ef - 1) : __shfl(c1d, ef - 65);
                tie |= __ballot(fresh && (dis == kth || dis == eth)) != 0ull;
            }
            // result heap: k smallest (dis, id) of the union, strict admission
            {
                float cd = (fresh && dis < FLT_MAX) ? dis : WS_INF;
                long long ci = (fresh && dis < FLT_MAX) ? (long long)v : WS_NOID;
                wave_offer_q(res_d, res_i, cd, ci, k, lane);
                const float rn = __shfl(res_d, (lane + 1) & 63);
                tie |= __ballot(lane + 1 < k && res_d < WS_INF && res_d == rn) != 0ull;
            }
            // candidate heap: ef smallest of the union (dead slots included)
            {
                float cd = fresh ? dis : WS_INF;
                long long ci = fresh ? (((long long)v << 1) | 1) : WS_NOID;
                wave_sort64(cd, ci, lane);
                merge128(c0d, c0i, c1d, c1i, cd, ci, lane);
                // equal neighbours among the kept positions (sorted queue)
                const float n0 = __shfl(c0d, (lane + 1) & 63), n1 = __shfl(c1d, (lane + 1) & 63);
                const float nx = lane < 63 ? n0 : __shfl(c1d, 0);
                const bool e0 = lane + 1 < ef && c0d < WS_INF && c0d == nx;
                const bool e1 = 65 + lane < ef && lane < 63 && c1d < WS_INF && c1d == n1;
                tie |= __ballot(e0 || e1) != 0ull;
            }
        }
    }
    if (tie_flags && lane == 0) tie_flags[q] = tie ? 1u : 0u;
    if (tie && tie_flags) return;  // the sequential kernel redoes this query
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

// ---------------------------------------------------------------- sequential
// HNSW::search with the reference's own data structures, operation for
// operation (faiss/impl/HNSW.cpp:605-741, :943-996; MinimaxHeap :1096-1342;
// heap_push / heap_pop / heap_replace_top / heap_reorder, faiss/utils/Heap.h):
// one wave per query, heaps in LDS, lane 0 applies every heap update in the
// reference's arrival order; the lanes compute the distances of a hop's
// neighbours (fvec_L2sqr order) and run pop_min / count_below as wave
// reductions with the reference's tie rules (pop_min: the highest slot among
// equal minima; count_below: every slot, dead ones included).  Used for
// max(efSearch, k) > 128, k > 64, and the queries the batched kernel flags.
namespace {
// binary heaps on (float, int32) with CMax cmp2 (faiss/utils/Heap.h:47-149)
__device__ __forceinline__ bool cmp2_gt(float a1, float b1, int32_t a2, int32_t b2) {
    return a1 > b1 || (a1 == b1 && a2 > b2);
}
__device__ void hx_pop(int k, float* bv, int32_t* bi) {
    bv--;
    bi--;
    const float val = bv[k];
    const int32_t id = bi[k];
    int i = 1;
    for (;;) {
        const int i1 = i << 1, i2 = i1 + 1;
        if (i1 > k) break;
        if (i2 == k + 1 || cmp2_gt(bv[i1], bv[i2], bi[i1], bi[i2])) {
            if (cmp2_gt(val, bv[i1], id, bi[i1])) break;
            bv[i] = bv[i1];
            bi[i] = bi[i1];
            i = i1;
        } else {
            if (cmp2_gt(val, bv[i2], id, bi[i2])) break;
            bv[i] = bv[i2];
            bi[i] = bi[i2];
            i = i2;
        }
    }
    bv[i] = bv[k];
    bi[i] = bi[k];
}
__device__ void hx_push(int k, float* bv, int32_t* bi, float val, int32_t id) {
    bv--;
    bi--;
    int i = k;
    while (i > 1) {
        const int f = i >> 1;
        if (!cmp2_gt(val, bv[f], id, bi[f])) break;
        bv[i] = bv[f];
        bi[i] = bi[f];
        i = f;
    }
    bv[i] = val;
    bi[i] = id;
}
__device__ void hx_replace_top(int k, float* bv, int32_t* bi, float val, int32_t id) {
    bv--;
    bi--;
    int i = 1;
    for (;;) {
        const int i1 = i << 1, i2 = i1 + 1;
        if (i1 > k) break;
        if (i2 == k + 1 || cmp2_gt(bv[i1], bv[i2], bi[i1], bi[i2])) {
            if (cmp2_gt(val, bv[i1], id, bi[i1])) break;
            bv[i] = bv[i1];
            bi[i] = bi[i1];
            i = i1;
        } else {
            if (cmp2_gt(val, bv[i2], id, bi[i2])) break;
            bv[i] = bv[i2];
            bi[i] = bi[i2];
            i = i2;
        }
    }
    bv[i] = val;
    bi[i] = id;
}
}  // namespace

template <bool LDS_VISITED>
__global__ __launch_bounds__(64) void k_hnsw_exact(HNSWDevice g, const float* __restrict__ x,
                                                   int ldx, int64_t n, int k, int efSearch,
                                                   int ef, float* __restrict__ D,
                                                   int64_t* __restrict__ I,
                                                   int32_t* __restrict__ I32,
                                                   uint32_t* __restrict__ vis_global,
                                                   int64_t vwords,
                                                   unsigned long long* __restrict__ stats,
                                                   const uint32_t* __restrict__ only) {
    const int64_t q = blockIdx.x;
    if (only && only[q] == 0u) return;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* qs = sm;                              // [ld]
    float* cdis = qs + g.ld;                     // [ef] MinimaxHeap dis
    int32_t* cid = (int32_t*)(cdis + ef);        // [ef] MinimaxHeap ids
    float* rdis = (float*)(cid + ef);            // [k] result heap
    int32_t* rid = (int32_t*)(rdis + k);         // [k]
    float* fd = (float*)(rid + k);               // [64] fresh neighbours of a hop
    int32_t* fi = (int32_t*)(fd + 64);           // [64]
    int32_t* sh = fi + 64;                       // [8] scalars: hk, nvalid, nfresh, ...
    uint32_t* vis = LDS_VISITED ? (uint32_t*)(sh + 8) : vis_global + blockIdx.x * vwords;
    const int lane = threadIdx.x;
    for (int j = lane; j < g.ld; j += 64) qs[j] = j < g.d ? x[q * ldx + j] : 0.f;
    for (int j = lane; j < k; j += 64) {
        rdis[j] = FLT_MAX;  // heap_heapify<CMax> (Heap.h:316-339)
        rid[j] = -1;
    }
    for (int64_t w = lane; w < vwords; w += 64) vis[w] = 0u;
    __syncthreads();
    uint32_t st_n2 = 0, st_ndis = 0, st_nhops = 0;
    if (g.entry_point >= 0) {
        // ---- greedy descent (HNSW.cpp:852-924), as in k_hnsw_search
        int nearest = g.entry_point;
        float d_nearest = l2_row(qs, g.storage + (int64_t)nearest * g.ld, g.d);
        for (int level = g.max_level; level >= 1; level--) {
            for (;;) {
                const uint64_t o = g.offsets[nearest];
                const int b = g.cum_nb[level], e = g.cum_nb[level + 1];
                const int cnt = e - b;
                int v = lane < cnt ? g.neighbors[o + b + lane] : -1;
                unsigned long long neg =
                        __ballot(lane < cnt && v < 0) | (cnt < 64 ? (~0ull << cnt) : 0ull);
                const int first_neg = neg ? __ffsll((long long)neg) - 1 : 64;
                float dis = WS_INF;
                if (lane < first_neg) dis = l2_row(qs, g.storage + (int64_t)v * g.ld, g.d);
                st_ndis += (uint32_t)min(first_neg, 64);
                st_nhops += 1;
                float md = dis;
                int ml = lane;
#pragma unroll
                for (int m = 32; m > 0; m >>= 1) {
                    const float od = __shfl_xor(md, m);
                    const int ol = __shfl_xor(ml, m);
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
        // ---- level 0: MinimaxHeap candidates(ef) seeded with the entry
        if (lane == 0) {
            int hk = 0;
            hx_push(++hk, cdis, cid, d_nearest, nearest);  // MinimaxHeap::push on empty
            sh[0] = hk;
            sh[1] = 1;  // nvalid
            // search_from_candidates (:624-637): the seeds enter the results
            float threshold = rdis[0];
            for (int i = 0; i < hk; i++) {
                const int32_t v1 = cid[i];
                const float dd = cdis[i];
                if (dd < threshold && rdis[0] > dd) {
                    hx_replace_top(k, rdis, rid, dd, v1);
                    threshold = rdis[0];
                }
                vis[v1 >> 5] |= 1u << (v1 & 31);
            }
        }
        __syncthreads();
        for (;;) {
            const int hk = sh[0];
            if (sh[1] <= 0) {  // candidates.size() == 0
                st_n2 = 1;
                break;
            }
            // pop_min (:1299-1330): the smallest dis among alive slots, the
            // highest slot index among equal minima
            float bd = FLT_MAX;
            int bp = -1;
            for (int i = lane; i < hk; i += 64)
                if (cid[i] != -1 && (bp < 0 || cdis[i] < bd || (cdis[i] == bd && i > bp))) {
                    bd = cdis[i];
                    bp = i;
                }
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) {
                const float od = __shfl_xor(bd, m);
                const int op = __shfl_xor(bp, m);
                if (op >= 0 && (bp < 0 || od < bd || (od == bd && op > bp))) {
                    bd = od;
                    bp = op;
                }
            }
            const int32_t v0 = cid[bp];
            const float d0 = bd;
            // count_below(d0): every slot, dead ones included
            int nb = 0;
            for (int i = lane; i < hk; i += 64) nb += cdis[i] < d0;
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) nb += __shfl_xor(nb, m);
            __syncthreads();
            if (lane == 0) {
                cid[bp] = -1;
                sh[1] -= 1;
            }
            __syncthreads();
            if (nb >= efSearch) {
                st_n2 = sh[1] == 0 ? 1u : 0u;
                break;
            }
            // neighbours of v0 in stored order; visited test-and-set in order
            const uint64_t o = g.offsets[v0];
            const int b = g.cum_nb[0], e = g.cum_nb[1];
            const int cnt = e - b;
            if (lane == 0) {
                int nf = 0;
                for (int j = 0; j < cnt; j++) {
                    const int32_t v1 = g.neighbors[o + b + j];
                    if (v1 < 0) break;
                    const uint32_t bit = 1u << (v1 & 31);
                    const uint32_t old = vis[v1 >> 5];
                    vis[v1 >> 5] = old | bit;
                    if (!(old & bit)) fi[nf++] = v1;
                }
                sh[2] = nf;
            }
            __syncthreads();
            const int nf = sh[2];
            if (lane < nf) fd[lane] = l2_row(qs, g.storage + (int64_t)fi[lane] * g.ld, g.d);
            st_ndis += (uint32_t)nf;
            st_nhops += 1;
            __syncthreads();
            if (lane == 0) {
                int hk2 = sh[0], nvalid = sh[1];
                float threshold = rdis[0];
                for (int t = 0; t < nf; t++) {
                    const int32_t v1 = fi[t];
                    const float dis = fd[t];
                    // add_to_heap (:678-689)
                    if (dis < threshold && rdis[0] > dis) {
                        hx_replace_top(k, rdis, rid, dis, v1);
                        threshold = rdis[0];
                    }
                    // MinimaxHeap::push (:1096-1107)
                    if (hk2 == ef) {
                        if (dis >= cdis[0]) continue;
                        if (cid[0] != -1) --nvalid;
                        hx_pop(hk2--, cdis, cid);
                    }
                    hx_push(++hk2, cdis, cid, dis, v1);
                    ++nvalid;
                }
                sh[0] = hk2;
                sh[1] = nvalid;
            }
            __syncthreads();
        }
    }
    if (stats && lane == 0 && g.entry_point >= 0) {
        atomicAdd(&stats[0], 1ull);
        atomicAdd(&stats[1], (unsigned long long)st_n2);
        atomicAdd(&stats[2], (unsigned long long)st_ndis);
        atomicAdd(&stats[3], (unsigned long long)st_nhops);
    }
    // heap_reorder<CMax> (Heap.h:421-450) by lane 0, then the lanes write out
    if (lane == 0) {
        int ii = 0;
        for (int i = 0; i < k; i++) {
            const float val = rdis[0];
            const int32_t id = rid[0];
            hx_pop(k - i, rdis, rid);
            rdis[k - ii - 1] = val;
            rid[k - ii - 1] = id;
            if (id != -1) ii++;
        }
        // memmove to the front, pad (FLT_MAX, -1)
        for (int i = 0; i < ii; i++) {
            rdis[i] = rdis[k - ii + i];
            rid[i] = rid[k - ii + i];
        }
        for (int i = ii; i < k; i++) {
            rdis[i] = FLT_MAX;
            rid[i] = -1;
        }
    }
    __syncthreads();
    for (int j = lane; j < k; j += 64) {
        if (D) D[q * k + j] = rdis[j];
        if (I) I[q * k + j] = rid[j];
        if (I32) I32[q * k + j] = rid[j];
    }
}

void hnsw_search(const HNSWDevice& g, const float* x, int ldx, int64_t n, int k, int efSearch,
                 float* D, int64_t* I, int32_t* I32, uint32_t* visited_scratch,
                 int64_t visited_words_per_query, unsigned long long* stats, uint32_t* flags,
                 hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT_FMT(k >= 1 && k <= kMaxKExact, "k = %d must be in [1, %d]", k,
                           kMaxKExact);
    const int ef = efSearch > k ? efSearch : k;
    FAISS_THROW_IF_NOT(g.ld % 4 == 0);
    const int64_t vwords = visited_words_per_query;
    const size_t lds_q = sizeof(float) * g.ld;
    const bool batched = ef <= 128 && k <= kMaxK;
    // sequential kernel: query | ef heap | k heap | 64 fresh | 8 scalars | visited
    const size_t lds_x = lds_q + 8 * (size_t)ef + 8 * (size_t)k + 8 * 64 + 4 * 8;
    const bool x_lds_vis = lds_x + vwords * 4 <= 64 * 1024;
    FAISS_THROW_IF_NOT_FMT(lds_x <= 64 * 1024, "max(efSearch, k) = %d too large for LDS", ef);
    const bool lds_vis = vwords * 4 <= 64 * 1024;
    if ((batched && !lds_vis) || (!x_lds_vis)) {
        FAISS_THROW_IF_NOT(visited_scratch != nullptr);
        HIP_CHECK(hipMemsetAsync(visited_scratch, 0, sizeof(uint32_t) * vwords * n, s));
    }
    auto exact = [&](const uint32_t* only) {
        if (x_lds_vis)
            k_hnsw_exact<true><<<dim3((unsigned)n), dim3(64), lds_x + vwords * 4, s>>>(
                    g, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, only);
        else
            k_hnsw_exact<false><<<dim3((unsigned)n), dim3(64), lds_x, s>>>(
                    g, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats,
                    only);
        HIP_LAUNCH_CHECK();
    };
    if (!batched) {
        exact(nullptr);
        return;
    }
    if (lds_vis) {
        size_t lds = lds_q + sizeof(uint32_t) * vwords;
        k_hnsw_search<true><<<dim3((unsigned)n), dim3(64), lds, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, flags);
    } else {
        k_hnsw_search<false><<<dim3((unsigned)n), dim3(64), lds_q, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats, flags);
    }
    HIP_LAUNCH_CHECK();
    if (flags) {
        // the flagged queries again, sequentially; the visited scratch of a
        // flagged query is reset by the kernel itself
        exact(flags);
    }
}

}  // namespace kern
}  // namespace faiss_amd
