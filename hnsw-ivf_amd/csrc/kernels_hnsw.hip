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

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

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
// Returns the smallest distance it discarded (+inf when none).
__device__ __forceinline__ float merge128(float& d0, long long& i0, float& d1, long long& i1,
                                          float bd, long long bi, int lane) {
    float rd = __shfl(bd, 63 - lane);
    long long ri = shfl_ll(bi, 63 - lane);
    float disc = rd;
    if (key_less(rd, ri, d1, i1)) {
        disc = d1;
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
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) disc = fminf(disc, __shfl_xor(disc, j));
    return disc;
}
// wave_merge64 (wave_select.h) that also returns the smallest distance it
// discarded (+inf when none)
__device__ __forceinline__ float merge64_disc(float& qd, long long& qi, float cd, long long ci,
                                              int lane) {
    const float rd = __shfl(cd, 63 - lane);
    const long long ri = shfl_ll(ci, 63 - lane);
    float disc = rd;
    if (key_less(rd, ri, qd, qi)) {
        disc = qd;
        qd = rd;
        qi = ri;
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) cas_lane(qd, qi, j, (lane & j) == 0);
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) disc = fminf(disc, __shfl_xor(disc, j));
    return disc;
}

// Move the lanes with `sel` to lanes 0..m-1 (order kept) and give the others
// (+inf, NOID); returns m.  One ds_permute per 32-bit word: every lane pushes
// its key to its destination (a permutation of the 64 lanes).
__device__ __forceinline__ int wave_compact(float& d, long long& i, bool sel, int lane) {
    const unsigned long long bm = __ballot(sel);
    const int m = __popcll(bm);
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int dst = sel ? __popcll(bm & lt) : m + __popcll(~bm & lt);
    const int a = dst << 2;
    d = __int_as_float(__builtin_amdgcn_ds_permute(a, __float_as_int(d)));
    const int lo = __builtin_amdgcn_ds_permute(a, (int)(i & 0xffffffffLL));
    const int hi = __builtin_amdgcn_ds_permute(a, (int)(i >> 32));
    i = ((long long)hi << 32) | (unsigned int)lo;
    if (lane >= m) {
        d = WS_INF;
        i = WS_NOID;
    }
    return m;
}

// ascending bitonic sort of lanes [0, W) (W a power of two); lanes >= W hold
// (+inf, NOID), so the whole wave ends sorted
template <int W>
__device__ __forceinline__ void wave_sort_w(float& d, long long& i, int lane) {
#pragma unroll
    for (int k = 2; k <= W; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) cas_lane(d, i, j, ((lane & j) == 0) == ((lane & k) == 0));
    }
}
// sort a batch whose real keys are compacted to lanes 0..m-1: the narrowest
// network that covers them (a hop rarely brings more than a few keys that can
// enter a queue, so most batches need 1-3 stages instead of 21)
__device__ __forceinline__ void wave_sort_m(float& d, long long& i, int lane, int m) {
    if (m <= 1) return;
    if (m <= 2) wave_sort_w<2>(d, i, lane);
    else if (m <= 4) wave_sort_w<4>(d, i, lane);
    else if (m <= 8) wave_sort_w<8>(d, i, lane);
    else if (m <= 16) wave_sort_w<16>(d, i, lane);
    else if (m <= 32) wave_sort_w<32>(d, i, lane);
    else wave_sort_w<64>(d, i, lane);
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
    uint32_t tie = 0u;  // exact distance ties where the batched form may differ (reason bits)
    float rdisc = WS_INF;  // smallest distance the result heap ever turned away
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
            // pop_min among equal alive minima picks by heap slot in the
            // reference (MinimaxHeap::pop_min): an order the batched queue
            // does not keep
            if (__popcll(__ballot(a0 && c0d == d0v)) + __popcll(__ballot(a1 && c1d == d0v)) > 1)
                tie |= 1u;  // pop order
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
            // neighbours of v0 at level 0 (the regular table: no offsets load)
            const int cnt = g.cum_nb[1] - g.cum_nb[0];
            int v = -1;
            if (lane < cnt)
                v = g.nb0 ? g.nb0[(int64_t)v0 * g.nb0_stride + lane]
                          : g.neighbors[g.offsets[v0] + g.cum_nb[0] + lane];
            unsigned long long neg = __ballot(lane < cnt && v < 0) | (cnt < 64 ? (~0ull << cnt) : 0ull);
            const int jmax = neg ? __ffsll((long long)neg) - 1 : 64;
            bool fresh = false;
            if (lane < jmax) {
                uint32_t bit = 1u << (v & 31);
                uint32_t old = atomicOr(&vis[v >> 5], bit);
                fresh = (old & bit) == 0;
            }
            float dis = WS_INF;
            const unsigned long long fm = __ballot(fresh);
            st_ndis += (uint32_t)__popcll(fm);
            st_nhops += 1;  // nstep
            if (fm == 0ull) continue;
            if (g.d <= 128) {
                // the fresh neighbours compacted to lanes 0..nf-1 (a hop's
                // neighbours are one batch: their lane order is immaterial)
                // and evaluated 4 lanes per row, 16 rows per pass, in the
                // reference order: a wave-instruction stream of ~16 rows'
                // cost per pass instead of one full row per lane
                const int nf = __popcll(fm);
                const unsigned long long lt = (1ull << lane) - 1ull;
                const int dst = fresh ? __popcll(fm & lt) : nf + __popcll(~fm & lt);
                v = __builtin_amdgcn_ds_permute(dst << 2, v);
                fresh = lane < nf;
                dis = ref_rows64_4lane<true, 16>(qs, qs, g.storage, g.ld, g.d,
                                                 fresh ? (uint32_t)v : 0u, fresh, lane);
                if (!fresh) dis = WS_INF;
            } else if (fresh) {
                dis = l2_row(qs, g.storage + (int64_t)v * g.ld, g.d);
            }
            // Ties: the sequential heaps (strict admission, MinimaxHeap's
            // push / pop_min rules) and the batched union agree only for
            // distinct distances.  A fresh distance equal to the current k-th
            // result or ef-th candidate, or two equal distances among the ef
            // kept candidates (checked after the merge below), flags the query
            // for the sequential kernel (k_hnsw_exact).
            {
                const float eth = ef <= 64 ? __shfl(c0d, ef - 1) : __shfl(c1d, ef - 65);
                if (__ballot(fresh && dis == eth) != 0ull) tie |= 2u;  // push at the max
            }
            // result heap: k smallest (dis, id) of the union, strict admission;
            // only keys below the current k-th can enter: they are compacted
            // and sorted by the narrowest network that holds them
            {
                const float thr_d = __shfl(res_d, k - 1);
                const long long thr_i = shfl_ll(res_i, k - 1);
                const bool pass = fresh && dis < FLT_MAX && key_less(dis, (long long)v, thr_d, thr_i);
                float cd = pass ? dis : WS_INF;
                long long ci = pass ? (long long)v : WS_NOID;
                // the result heap never steers the traversal (only the
                // candidate heap does), so the strict-admission / (dis, id)
                // difference can only show in the final set: it is checked
                // once, after the search, against the smallest distance the
                // heap ever turned away (rejected entrants, evicted keys)
                float rej = (fresh && !pass && dis < FLT_MAX) ? dis : WS_INF;
#pragma unroll
                for (int j = 32; j > 0; j >>= 1) rej = fminf(rej, __shfl_xor(rej, j));
                rdisc = fminf(rdisc, rej);
                const int m = wave_compact(cd, ci, pass, lane);
                if (m > 0) {
                    wave_sort_m(cd, ci, lane, m);
                    rdisc = fminf(rdisc, merge64_disc(res_d, res_i, cd, ci, lane));
                }
            }
            // candidate heap: ef smallest of the union (dead slots included);
            // a key above the ef-th kept slot would land past ef (positions
            // never read), so only the ones below it are merged
            {
                const float ed = ef <= 64 ? __shfl(c0d, ef - 1) : __shfl(c1d, ef - 65);
                const long long ei = ef <= 64 ? shfl_ll(c0i, ef - 1) : shfl_ll(c1i, ef - 65);
                const long long key2 = ((long long)v << 1) | 1;
                const bool enter = fresh && key_less(dis, key2, ed, ei);
                float cd = enter ? dis : WS_INF;
                long long ci = enter ? key2 : WS_NOID;
                const int m = wave_compact(cd, ci, enter, lane);
                if (m > 0) {
                    wave_sort_m(cd, ci, lane, m);
                    const float disc = merge128(c0d, c0i, c1d, c1i, cd, ci, lane);
                    // MinimaxHeap::push drops v >= max and evicts the max
                    // with popped slots at id -1: only an equal distance at
                    // the ef boundary can make the kept sets differ
                    const float ld = ef <= 64 ? __shfl(c0d, ef - 1) : __shfl(c1d, ef - 65);
                    const float nd = ef < 64 ? __shfl(c0d, ef)
                                     : ef < 128 ? __shfl(c1d, ef - 64) : disc;
                    if (nd < WS_INF && ld == nd) tie |= 4u;  // candidate boundary
                }
            }
        }
    }
    {
        // the final k-set equals the sequential heap's unless its k-th
        // distance is shared by a key it turned away (or kept past k)
        const float kd = __shfl(res_d, k - 1);
        const float nd = fminf(rdisc, k < 64 ? __shfl(res_d, k) : WS_INF);
        if (nd < WS_INF && kd == nd) tie |= 8u;  // result boundary
    }
    if (tie_flags && lane == 0) tie_flags[q] = tie;
    if (tie && tie_flags) return;  // the sequential kernel redoes this query
    if (stats && lane == 0 && g.entry_point >= 0) {
        atomicAdd(&stats[0], 1ull);
        atomicAdd(&stats[1], (unsigned long long)st_n2);
        atomicAdd(&stats[2], (unsigned long long)st_ndis);
        atomicAdd(&stats[3], (unsigned long long)st_nhops);
        atomicAdd(&stats[4], (unsigned long long)st_ndis);
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
// The heaps as faiss lays them out (1-based binary heaps, faiss/utils/Heap.h),
// one 64-bit key per slot: the distance's bits (>= 0: they order as unsigned)
// over the id biased by 2^31, so CMax's cmp2 (dis, then id) is one unsigned
// compare; a MinimaxHeap slot killed by pop_min keeps its distance with id -1,
// as faiss's does.  The code runs wave-uniform (every lane computes the same
// serial steps; lane 0 stores), so the lanes can load a push's ancestors and a
// sift's next three levels at once.
// the sequential kernel's arrival log (k_hnsw_exact without the result
// heap): per running work group a slot of `cap` keys from a pool of `slots`
// (ctr: the slots handed out, zeroed before the launch)
struct ArrivalLog {
    uint64_t* base = nullptr;
    uint32_t* ctr = nullptr;
    int64_t slots = 0;
    int64_t cap = 0;
};
__device__ __forceinline__ uint64_t sx_key(float d, int32_t id) {
    return ((uint64_t)(uint32_t)__float_as_int(d) << 32) | (uint32_t)(id ^ (int32_t)0x80000000);
}
__device__ __forceinline__ float sx_dis(uint64_t k) { return __int_as_float((int)(k >> 32)); }
__device__ __forceinline__ int32_t sx_id(uint64_t k) { return (int32_t)((uint32_t)k ^ 0x80000000u); }
__host__ __device__ inline int seq_qpad(int ld) { return ld < 128 ? 128 : ld; }
// slots of a heap of capacity c (1-based, index 0 unused, sibling pairs
// (2i, 2i + 1) 16-byte aligned and always inside the array)
__host__ __device__ inline size_t seq_slots(int c) { return (size_t)((c + 2) & ~1); }
__host__ __device__ inline size_t seq_heap_bytes(int ef, int k) {
    return 8 * (seq_slots(ef) + seq_slots(k));
}
// LDS of the sequential kernel: query | candidate heap | result heap | 64
// fresh neighbours (id) | visited (when it fits)
__host__ __device__ inline size_t seq_lds_bytes(int ld, int ef, int k) {
    return 4 * (size_t)seq_qpad(ld) + seq_heap_bytes(ef, k) + 4 * 64;
}
__host__ __device__ inline size_t seq_lds_bytes_gheap(int ld) { return 4 * (size_t)seq_qpad(ld) + 4 * 64; }

// heap_pop (val = b[n], n the size before the pop) / heap_replace_top (val
// the new key, n the size) of faiss/utils/Heap.h:112-149, CMax: the sift from
// the root, the serial loop's decisions exactly (i2 == n + 1 takes i1; an
// equal child is followed); one 16-byte LDS read of the children pair per
// level.  (A three-level lookahead per LDS round trip measured slower: the
// kernel is bound by instruction issue across its waves, not by latency.)
__device__ __forceinline__ void sx_sift(uint64_t* b, int n, uint64_t val, int lane) {
    int i = 1;
    for (;;) {
        const int i1 = 2 * i;
        if (i1 > n) break;
        const uint4 pv = *(const uint4*)(b + i1);
        const uint64_t k1 = ((uint64_t)pv.y << 32) | pv.x, k2 = ((uint64_t)pv.w << 32) | pv.z;
        const bool first = i1 + 1 == n + 1 || k1 > k2;
        const uint64_t kj = first ? k1 : k2;
        if (val > kj) break;
        if (lane == 0) b[i] = kj;
        i = first ? i1 : i1 + 1;
    }
    if (lane == 0) b[i] = val;
}

// heap_push of faiss/utils/Heap.h:150-170, CMax, after the size became n:
// the ancestors n >> j (j = 1 .. log2 n) are loaded at once, one per lane;
// the serial loop moves them down while val > ancestor (the run of such
// ancestors from the parent up) and stores val where it stopped
__device__ __forceinline__ void sx_push(uint64_t* b, int n, uint64_t val, int lane) {
    const int L = 31 - __clz(n);
    const int j = lane + 1;
    const bool in = j <= L;
    const uint64_t a = in ? b[n >> (j & 31)] : 0ull;
    const unsigned long long gt = __ballot(in && val > a);
    const int m = __builtin_ctzll(~gt);
    if (j <= m) b[n >> (j - 1)] = a;
    if (lane == 0) b[n >> m] = val;
}
}  // namespace

// HNSW::search with the reference's own data structures, operation for
// operation (faiss/impl/HNSW.cpp:605-741, :943-996; MinimaxHeap :1096-1342;
// heap_push / heap_pop / heap_replace_top / heap_reorder, faiss/utils/Heap.h):
// one wave per query, both heaps in LDS in faiss's layout (sx_* above), the
// hop's fresh neighbours evaluated by the lanes (4 lanes per row in the
// reference order) and applied in arrival order; pop_min / count_below are
// wave scans with the reference's tie rules (pop_min: the highest slot among
// equal minima; count_below: every slot, dead ones included).  Serves
// max(efSearch, k) > 64 (beyond 128 always), k > 64, and the queries the
// batched kernel flags.
// GH: the two heaps in global scratch (gheap: seq_heap_bytes per block) —
// max(efSearch, k) beyond what the work group's LDS holds (the reference's
// harness sweeps efSearch up to 3 nprobe, nprobe into the thousands)
// The search of query q (input row q, output row qo) by one wave: the body
// of k_hnsw_exact, also run in place by k_hnsw_wide<.., INPLACE> for the
// queries it flags.  blk: the work group's slot of the global heaps and
// visited words; sm: the work group's dynamic LDS (seq_lds_bytes + visited).
template <bool LDS_VISITED, bool GH>
__device__ __forceinline__ void hnsw_exact_query(
        HNSWDevice g, const float* __restrict__ x, int ldx, int k, int efSearch, int ef,
        float* __restrict__ D, int64_t* __restrict__ I, int32_t* __restrict__ I32,
        uint32_t* __restrict__ vis_global, int64_t vwords, unsigned long long* __restrict__ stats,
        float* __restrict__ gheap, ArrivalLog alog, int64_t q, int64_t qo, int64_t blk,
        float* sm) {
    const int qpad = seq_qpad(g.ld);
    float* qs = sm;  // [qpad]
    uint64_t* cb = GH ? (uint64_t*)((char*)gheap + blk * seq_heap_bytes(ef, k))
                      : (uint64_t*)(sm + qpad);         // MinimaxHeap [1 .. ef]
    uint64_t* rb = cb + seq_slots(ef);                  // result heap [1 .. k]
    int32_t* fi = GH ? (int32_t*)(sm + qpad) : (int32_t*)((char*)(sm + qpad) + seq_heap_bytes(ef, k));
    uint32_t* vis = LDS_VISITED ? (uint32_t*)(fi + 64) : vis_global + blk * vwords;
    const int lane = threadIdx.x;
    for (int j = lane; j < qpad; j += 64) qs[j] = j < g.d ? x[q * ldx + j] : 0.f;
    const uint64_t rinit = sx_key(FLT_MAX, -1);  // heap_heapify<CMax> (Heap.h:316-339)
    for (int j = lane; j < k; j += 64) rb[1 + j] = rinit;
    for (int64_t w = lane; w < vwords; w += 64) vis[w] = 0u;
    // without the result heap (ArrivalLog): the query's arrivals logged in
    // order, the results selected from them at the end (a log slot per
    // work group from the pool; none left: the result heap as before)
    uint64_t* lg = nullptr;
    if (!GH && alog.base) {
        uint32_t slot = 0u;
        if (lane == 0) slot = atomicAdd(alog.ctr, 1u);
        slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)slot);
        if ((int64_t)slot < alog.slots) lg = alog.base + (int64_t)slot * alog.cap;
    }
    int64_t lpos = 0;
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
        // ---- level 0: MinimaxHeap candidates(ef) seeded with the entry;
        // search_from_candidates (:624-637): the seed enters the results
        int hk = 1, nvalid = 1;
        if (lane == 0) {
            cb[1] = sx_key(d_nearest, nearest);
            vis[nearest >> 5] |= 1u << (nearest & 31);
        }
        __syncthreads();
        float rthr = sx_dis(rb[1]);
        if (lg) {
            if (lane == 0) lg[0] = sx_key(d_nearest, nearest);
            lpos = 1;
        } else if (d_nearest < rthr) {
            sx_sift(rb, k, sx_key(d_nearest, nearest), lane);
            rthr = sx_dis(rb[1]);
        }
        const int cnt = g.cum_nb[1] - g.cum_nb[0];
        for (;;) {
            if (nvalid <= 0) {  // candidates.size() == 0
                st_n2 = 1;
                break;
            }
            // pop_min (:1299-1330): the smallest dis among alive slots, the
            // highest slot among equal minima
            float bd = FLT_MAX;
            int bp = -1;
            // (the slots' distances stay in registers for count_below when
            // the heap has at most 64 SX_CACHE slots)
            constexpr int SX_CACHE = 16;
            float dc[SX_CACHE];
            const bool cached = hk <= 64 * SX_CACHE;
            if (cached) {
#pragma unroll
                for (int u = 0; u < SX_CACHE; u++) {
                    const int i = 1 + lane + 64 * u;
                    dc[u] = FLT_MAX;
                    if (i <= hk) {
                        const uint64_t kv = cb[i];
                        const float dv = sx_dis(kv);
                        dc[u] = dv;
                        if (sx_id(kv) != -1 && (bp < 0 || dv < bd || (dv == bd && i > bp))) {
                            bd = dv;
                            bp = i;
                        }
                    }
                }
            } else {
                for (int i = 1 + lane; i <= hk; i += 64) {
                    const uint64_t kv = cb[i];
                    const float dv = sx_dis(kv);
                    if (sx_id(kv) != -1 && (bp < 0 || dv < bd || (dv == bd && i > bp))) {
                        bd = dv;
                        bp = i;
                    }
                }
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
            const int32_t v0 = sx_id(cb[bp]);
            const float d0 = bd;
            // count_below(d0): every slot, dead ones included
            int nb = 0;
            if (cached) {
#pragma unroll
                for (int u = 0; u < SX_CACHE; u++) nb += dc[u] < d0;  // (padding: FLT_MAX)
            } else {
                for (int i = 1 + lane; i <= hk; i += 64) nb += sx_dis(cb[i]) < d0;
            }
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) nb += __shfl_xor(nb, m);
#ifdef HNSW_SEQ_DEBUG
            if (q == 0 && lane == 0 && st_nhops < 12)
                printf("hop %u: bp %d v0 %d d0 %g nb %d hk %d nvalid %d rthr %g rb1 %llx cb1 %llx\n",
                       st_nhops, bp, v0, d0, nb, hk, nvalid, rthr, (unsigned long long)rb[1],
                       (unsigned long long)cb[1]);
#endif
            if (lane == 0) cb[bp] = sx_key(d0, -1);
            nvalid--;
            if (nb >= efSearch) {
                st_n2 = nvalid == 0 ? 1u : 0u;
                break;
            }
            // neighbours of v0 in stored order; visited test-and-set in order
            // (neighbour j is fresh when its bit was clear before this hop and
            // no earlier neighbour of the list is the same node; the fresh
            // ones keep their stored order)
            int32_t v1 = -1;
            if (lane < cnt)
                v1 = g.nb0 ? g.nb0[(int64_t)v0 * g.nb0_stride + lane]
                           : g.neighbors[g.offsets[v0] + g.cum_nb[0] + lane];
            const unsigned long long neg =
                    __ballot(lane < cnt && v1 < 0) | (cnt < 64 ? (~0ull << cnt) : 0ull);
            const int jmax = neg ? __ffsll((long long)neg) - 1 : 64;
            // (the bits as they were before this hop decide; a node listed
            // twice — the atomic then finds the bit another lane of this hop
            // set — is visited at its first position, so only then the lanes
            // are compared pairwise)
            const uint32_t vbit = 1u << (v1 & 31);
            bool fresh = lane < jmax && !(vis[v1 >> 5] & vbit);
            uint32_t old = 0u;
            if (fresh) old = atomicOr(&vis[v1 >> 5], vbit);
            if (__ballot(fresh && (old & vbit)) != 0ull)
                for (int i = 0; i < jmax; i++)
                    fresh &= !(i < lane && __builtin_amdgcn_readlane(v1, i) == v1);
            const unsigned long long fm = __ballot(fresh);
            const int nf = __popcll(fm);
            const unsigned long long lt = (1ull << lane) - 1ull;
            const int dst = fresh ? __popcll(fm & lt) : nf + __popcll(~fm & lt);
            const int32_t fv = __builtin_amdgcn_ds_permute(dst << 2, v1);
            // the fresh rows, 4 lanes per row (reference order)
            float fdis = 0.f;
            if (g.d <= 128)
                fdis = ref_rows64_4lane_pb<true, 16, 1>(qs, qs, g.storage, g.ld, g.d,
                                                        lane < nf ? (uint32_t)fv : 0u, nf, lane);
            else if (lane < nf)
                fdis = l2_row(qs, g.storage + (int64_t)fv * g.ld, g.d);
            st_ndis += (uint32_t)nf;
            st_nhops += 1;
            // add_to_heap (:678-689) in arrival order; an arrival that can
            // enter neither heap (dis >= the result threshold, and >= the
            // full candidate heap's top) changes nothing
            uint64_t top = hk == ef ? cb[1] : 0ull;  // the full heap's top
            if (lg) {  // the hop's arrivals, in order
                if (lane < nf) lg[lpos + lane] = sx_key(fdis, fv);
                lpos += nf;
            }
            for (int t = 0; t < nf; t++) {
                const float dis = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fdis), t));
                const bool cin = hk < ef || dis < sx_dis(top);
                const bool rin = !lg && dis < rthr;
                if (!rin && !cin) continue;
                const int32_t id = __builtin_amdgcn_readlane(fv, t);
                const uint64_t key = sx_key(dis, id);
                if (rin) {
                    sx_sift(rb, k, key, lane);  // res.add_result: heap_replace_top
                    rthr = sx_dis(rb[1]);
                }
                // MinimaxHeap::push (:1096-1107)
                if (!cin) continue;
                if (hk == ef) {
                    if (sx_id(top) != -1) --nvalid;
                    sx_sift(cb, hk, cb[hk], lane);  // heap_pop(k--)
                    hk--;
                }
                sx_push(cb, ++hk, key, lane);
                ++nvalid;
                if (hk == ef) top = cb[1];
            }
            __syncthreads();
        }
    }
    if (stats && lane == 0 && g.entry_point >= 0) {
        atomicAdd(&stats[0], 1ull);
        atomicAdd(&stats[1], (unsigned long long)st_n2);
        atomicAdd(&stats[2], (unsigned long long)st_ndis);
        atomicAdd(&stats[3], (unsigned long long)st_nhops);
        atomicAdd(&stats[4], (unsigned long long)st_ndis);
    }
    if (lg) {
        __syncthreads();
        // the result heap's final content from the arrival log (lg[0, L)):
        // it holds the k smallest arrivals by distance when the k-th
        // distance is not shared (strict admission keeps any k smallest, and
        // an arrival it turned away was at least its k-th); a shared k-th
        // distance leaves the kept ids to the arrival order, and the heap is
        // then rebuilt by replaying the log
        uint64_t* sb = (uint64_t*)(sm + qpad);  // the heaps' LDS (dead now)
        const int64_t L = lpos;
        bool replay = false;
        int nsel = (int)min<int64_t>(L, (int64_t)k);
        uint32_t T = 0xffffffffu;  // select dis bits <= T
        if (L > k) {
            // radix select of the k-th smallest distance (bits as unsigned)
            uint32_t* hist = (uint32_t*)sb;
            uint32_t prefix = 0u, pmask = 0u;
            int64_t kk = k;
            for (int sh = 24; sh >= 0; sh -= 8) {
                for (int j = lane; j < 256; j += 64) hist[j] = 0u;
                __syncthreads();
                for (int64_t i = lane; i < L; i += 64) {
                    const uint32_t bits = (uint32_t)(lg[i] >> 32);
                    if ((bits & pmask) == prefix) atomicAdd(&hist[(bits >> sh) & 255u], 1u);
                }
                __syncthreads();
                // the bin holding the kk-th: 4 bins per lane, a lane scan
                uint32_t c4[4], cs = 0u;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    c4[u] = hist[4 * lane + u];
                    cs += c4[u];
                }
                uint32_t inc = cs;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t v = __shfl_up(inc, off);
                    if (lane >= off) inc += v;
                }
                const uint32_t exc = inc - cs;
                const unsigned long long hit = __ballot((int64_t)exc < kk && kk <= (int64_t)inc);
                const int hl = __ffsll((long long)hit) - 1;
                uint32_t below = (uint32_t)__builtin_amdgcn_readlane((int)exc, hl);
                int bin = 4 * hl;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t cu = (uint32_t)__builtin_amdgcn_readlane((int)c4[u], hl);
                    if (bin == 4 * hl + u && (int64_t)(below + cu) < kk) {
                        below += cu;
                        bin++;
                    }
                }
                kk -= below;
                prefix |= (uint32_t)bin << sh;
                pmask |= 255u << sh;
                __syncthreads();
            }
            T = prefix;
            int64_t nle = 0;
            for (int64_t i0 = 0; i0 < L; i0 += 64) {
                const int64_t i = i0 + lane;
                const uint32_t bits = i < L ? (uint32_t)(lg[i] >> 32) : 0xffffffffu;
                nle += __popcll(__ballot(i < L && bits <= T));
            }
            replay = nle > k;
            nsel = k;
        }
        if (replay) {
            // heap_heapify + every arrival through res.add_result, in order
            for (int j = lane; j < k; j += 64) rb[1 + j] = rinit;
            __syncthreads();
            float rt = FLT_MAX;
            for (int64_t i0 = 0; i0 < L; i0 += 64) {
                const int64_t i = i0 + lane;
                const uint64_t e = i < L ? lg[i] : ~0ull;
                const int nl = (int)min<int64_t>(64, L - i0);
                for (int t = 0; t < nl; t++) {
                    const uint64_t kt =
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(e >> 32), t) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, t);
                    if (sx_dis(kt) < rt) {
                        sx_sift(rb, k, kt, lane);
                        rt = sx_dis(rb[1]);
                    }
                }
            }
            __syncthreads();
        } else {
            // the selected arrivals ascending by (dis, id): a bitonic sort
            int P = 1;
            while (P < nsel) P <<= 1;
            int m = 0;
            for (int64_t i0 = 0; i0 < L; i0 += 64) {
                const int64_t i = i0 + lane;
                const uint64_t e = i < L ? lg[i] : ~0ull;
                const bool in = i < L && (uint32_t)(e >> 32) <= T;
                const unsigned long long bm = __ballot(in);
                if (in) sb[m + __popcll(bm & ((1ull << lane) - 1ull))] = e;
                m += __popcll(bm);
            }
            for (int j = m + lane; j < P; j += 64) sb[j] = ~0ull;
            __syncthreads();
            for (int sz = 2; sz <= P; sz <<= 1) {
                for (int st = sz >> 1; st > 0; st >>= 1) {
                    for (int t = lane; t < P / 2; t += 64) {
                        const int i = 2 * t - (t & (st - 1));
                        const int jx = i + st;
                        const bool up = (i & sz) == 0;
                        const uint64_t ai = sb[i], aj = sb[jx];
                        if ((ai > aj) == up) {
                            sb[i] = aj;
                            sb[jx] = ai;
                        }
                    }
                    __syncthreads();
                }
            }
            for (int j = lane; j < k; j += 64) {
                float dv = FLT_MAX;
                int32_t id = -1;
                if (j < nsel) {
                    dv = sx_dis(sb[j]);
                    id = sx_id(sb[j]);
                }
                if (D) D[qo * k + j] = dv;
                if (I) I[qo * k + j] = id;
                if (I32) I32[qo * k + j] = id;
            }
            return;
        }
    }
    // heap_reorder<CMax> (Heap.h:421-450): pops into the vacated tail, then
    // the kept ones to the front and (FLT_MAX, -1) padding
    int ii = 0;
    for (int i = 0; i < k; i++) {
        const uint64_t top = rb[1];
        sx_sift(rb, k - i, rb[k - i], lane);
        if (lane == 0) rb[k - ii] = top;  // 0-based slot k - ii - 1
        if (sx_id(top) != -1) ii++;
    }
    __syncthreads();
    for (int j = lane; j < k; j += 64) {
        float dv = FLT_MAX;
        int32_t id = -1;
        if (j < ii) {
            const uint64_t kv = rb[1 + k - ii + j];
            dv = sx_dis(kv);
            id = sx_id(kv);
        }
        if (D) D[qo * k + j] = dv;
        if (I) I[qo * k + j] = id;
        if (I32) I32[qo * k + j] = id;
    }
}

template <bool LDS_VISITED, bool GH = false>
__global__ __launch_bounds__(64) void k_hnsw_exact(HNSWDevice g, const float* __restrict__ x,
                                                   int ldx, int64_t n, int k, int efSearch,
                                                   int ef, float* __restrict__ D,
                                                   int64_t* __restrict__ I,
                                                   int32_t* __restrict__ I32,
                                                   uint32_t* __restrict__ vis_global,
                                                   int64_t vwords,
                                                   unsigned long long* __restrict__ stats,
                                                   const uint32_t* __restrict__ only,
        const uint32_t* __restrict__ qidx, float* __restrict__ gheap = nullptr,
        ArrivalLog alog = ArrivalLog{}) {
    // qidx: compact launch over listed queries (input row qidx[b], output
    // row b); else query b, output row b
    const int64_t q = qidx ? (int64_t)qidx[blockIdx.x] : (int64_t)blockIdx.x;
    const int64_t qo = blockIdx.x;
    if (only && only[q] == 0u) return;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    hnsw_exact_query<LDS_VISITED, GH>(g, x, ldx, k, efSearch, ef, D, I, I32, vis_global, vwords,
                                      stats, gheap, alog, q, qo, (int64_t)blockIdx.x, sm);
}

// The same sequential search for ef, k <= 64 with both heaps in registers.
// A heap entry is one 64-bit key: the distance's bits (>= 0: they order as
// unsigned) over the id biased by 2^31, so faiss's cmp2 (dis, then id) is a
// single unsigned compare.  The candidate MinimaxHeap keeps faiss's binary-
// heap layout exactly (pop_min's tie rule and heap_pop's choice among equal
// tops depend on it): heap position p (1-based, faiss/utils/Heap.h) lives in
// lane p & 63 (position 64 in lane 0), so siblings 2f, 2f + 1 are a DPP lane
// pair, and ballots rotated right by one put position p at bit p - 1.  Each
// of heap_push / heap_pop is a few wave-wide steps with the serial loop's
// exact outcome (tests/test_hnsw_wave_heap.py restates them lane by lane
// against the serial loops, dead MinimaxHeap slots and ties included).
namespace {
__device__ __forceinline__ uint64_t hkey(float d, int32_t id) {
    return ((uint64_t)(uint32_t)__float_as_int(d) << 32) | (uint32_t)(id ^ 0x80000000);
}
__device__ __forceinline__ float hkey_dis(uint64_t k) { return __int_as_float((int)(k >> 32)); }
__device__ __forceinline__ int32_t hkey_id(uint64_t k) { return (int32_t)((uint32_t)k ^ 0x80000000u); }
constexpr uint32_t HKEY_DEAD_LO = 0x7fffffffu;  // id -1
__device__ __forceinline__ uint64_t rotr1(uint64_t m) { return (m >> 1) | (m << 63); }
__device__ __forceinline__ uint64_t rotl1(uint64_t m) { return (m << 1) | (m >> 63); }
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t bperm64(uint64_t v, int src_lane) {
    const uint32_t lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)v, CTRL, 0xf, 0xf, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}

struct KHeap {
    uint64_t key;  // lane L: heap position L ? L : 64
    __device__ __forceinline__ uint64_t at(int p) const { return rdlane64(key, p & 63); }
    // heap_push(k, ...) (Heap.h): position k takes the new key and climbs
    // while it beats its parent: the climb stops below the deepest ancestor
    // it does not beat (one ballot), the path below moves down one level
    __device__ __forceinline__ void push(int k, uint64_t nk, int lane) {
        const int s = lane ? lane : 64;
        const int dk = 31 - __builtin_clz((unsigned)k);
        const int ds = 31 - __builtin_clz((unsigned)s);
        const bool anc = s < k && (k >> (dk - ds)) == s;
        const uint64_t nbt = rotr1(__ballot(anc && !(nk > key)));
        int p = 1;
        if (nbt) {
            const int f = 64 - __builtin_clzll(nbt);  // deepest ancestor not beaten
            p = k >> (dk - (31 - __builtin_clz((unsigned)f)) - 1);
        }
        const uint64_t pk = bperm64(key, (s >> 1) & 63);
        key = ((s == k || anc) && s > p) ? pk : (s == p ? nk : key);
    }
    // the sift of heap_pop / heap_replace_top over positions 1..k: the
    // serial descent follows the larger child (siblings by DPP, the path by a
    // scalar walk of one ballot), stops at the first path node nk beats; the
    // nodes above it move up one level and nk takes the freed position
    __device__ __forceinline__ void sift(int k, uint64_t nk, int lane) {
        const int s = lane ? lane : 64;
        const uint64_t sk = dpp64<0xB1>(key);  // quad_perm [1,0,3,2]: lane ^ 1
        bool larger = (s & 1) ? !(sk > key) : (s == k || key > sk);
        larger = larger && s >= 2 && s <= k;
        const uint64_t lm = rotr1(__ballot(larger));
        uint64_t path = 0;
        for (int c = 1; 2 * c <= k;) {
            c = ((lm >> ((2 * c - 1) & 63)) & 1ull) ? 2 * c : 2 * c + 1;
            path |= 1ull << ((c - 1) & 63);
        }
        const uint64_t stop = rotr1(__ballot(((rotl1(path) >> lane) & 1ull) && nk > key));
        const uint64_t moved = stop ? (path & ((stop & (~stop + 1ull)) - 1ull)) : path;
        const int p = moved ? 64 - __builtin_clzll(moved) : 1;
        const int c2 = 2 * s;
        const bool m0 = c2 <= 64 && ((moved >> ((c2 - 1) & 63)) & 1ull);
        const bool m1 = c2 < 64 && ((moved >> (c2 & 63)) & 1ull);
        const uint64_t ck = bperm64(key, (m1 ? c2 + 1 : c2) & 63);
        key = (m0 || m1) ? ck : (s == p ? nk : key);
    }
    __device__ __forceinline__ void pop(int k, int lane) { sift(k, at(k), lane); }  // heap_pop
};

// minimum of a 32-bit unsigned key over the wave (every lane active): DPP
// within quads, half-rows and rows, then the four row minima as scalars
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xf, 0xf, false));   // quad [1,0,3,2]
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xf, 0xf, false));   // quad [2,3,0,1]
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x141, 0xf, 0xf, false));  // half-row mirror
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x140, 0xf, 0xf, false));  // row mirror
    const uint32_t a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 16);
    const uint32_t c = __builtin_amdgcn_readlane(x, 32), e = __builtin_amdgcn_readlane(x, 48);
    return min(min(a, b), min(c, e));
}
// The result heap of search_from_candidates (HeapBlockResultHandler<CMax>,
// faiss/impl/ResultHandler.h + heap_replace_top, faiss/utils/Heap.h:112-149)
// as a sorted queue: lane j holds the j-th smallest key of the k kept.  Its
// observable behaviour depends on the kept set only — admission is
// `dis < top.dis`, replace_top evicts the top, the unique cmp2-largest key
// (a valid heap: no slot is ever killed), heap_reorder emits the set in
// ascending order — so the sorted set gives the reference's result exactly,
// with an insert of one ballot and one DPP shift.
struct SortedQ {
    uint64_t key;
    // nk whose dis is below the k-th kept dis: the largest leaves
    __device__ __forceinline__ void insert(int k, uint64_t nk, int lane) {
        const int pos = __popcll(__ballot(lane < k && key < nk));
        const uint64_t up = dpp64<0x138>(key);  // wave_shr:1
        key = lane > pos ? up : (lane == pos ? nk : key);
    }
};
// The candidate MinimaxHeap (faiss/impl/HNSW.cpp:1096-1342) of the register
// kernel, in two forms with one interface.
//  * CandLayout keeps faiss's heap array (KHeap): exact in every case.
//  * CandSet keeps the entries sorted by distance in lanes 0..hk-1 (one
//    ballot + one DPP shift per update).  The MinimaxHeap's observable
//    decisions depend on its entry set alone, except two that read the heap
//    layout: pop_min among several alive entries of the smallest distance
//    (the highest slot wins) and heap_pop of a full heap whose largest
//    distance is shared (which of them is the top).  CandSet reports either
//    case (returns false) and the query is searched again with CandLayout;
//    otherwise it evolves exactly as the heap's set does.
struct CandLayout {
    static constexpr bool kMerge = false;
    KHeap h;
    int hk;
    __device__ __forceinline__ void init(int) {
        h.key = hkey(FLT_MAX, -1);
        hk = 0;
    }
    __device__ __forceinline__ void seed(uint64_t nk, int lane) { h.push(++hk, nk, lane); }
    __device__ __forceinline__ float top_dis() const { return hkey_dis(h.at(1)); }
    // pop_min + count_below(d0) (:1299-1342): the smallest alive distance,
    // the highest position among equal ones (distances >= 0: their bits
    // order as unsigned)
    __device__ __forceinline__ bool pop_min(int lane, int32_t& v0, int& nb) {
        const int spos = lane ? lane : 64;
        const uint32_t chi = (uint32_t)(h.key >> 32);
        const bool alive = spos <= hk && (uint32_t)h.key != HKEY_DEAD_LO;
        const uint32_t kmin = wave_min_u32(alive ? chi : 0xffffffffu);
        const uint64_t at = rotr1(__ballot(alive && chi == kmin));
        const int bpos = 64 - __builtin_clzll(at);
        v0 = hkey_id(h.at(bpos));
        nb = __popcll(__ballot(spos <= hk && chi < kmin));
        if (spos == bpos) h.key = (h.key & 0xffffffff00000000ull) | HKEY_DEAD_LO;
        return true;
    }
    // the alive entry pop_min would take now (prefetch hint; ~0 when none)
    __device__ __forceinline__ uint64_t peek_min(int lane) const {
        const int spos = lane ? lane : 64;
        const uint32_t chi = (uint32_t)(h.key >> 32);
        const bool alive = spos <= hk && (uint32_t)h.key != HKEY_DEAD_LO;
        const unsigned long long am = __ballot(alive);
        if (!am) return ~0ull;
        const uint32_t kmin = wave_min_u32(alive ? chi : 0xffffffffu);
        const uint64_t at = rotr1(__ballot(alive && chi == kmin));
        return h.at(64 - __builtin_clzll(at));
    }
    // MinimaxHeap::push (:1096-1107)
    __device__ __forceinline__ bool push(int ef, uint64_t nk, float dis, int& nvalid, int lane) {
        if (hk == ef) {
            const uint64_t top = h.at(1);
            if (dis >= hkey_dis(top)) return true;
            if ((uint32_t)top != HKEY_DEAD_LO) --nvalid;
            h.pop(hk--, lane);
        }
        h.push(++hk, nk, lane);
        ++nvalid;
        return true;
    }
};
struct CandSet {
    static constexpr bool kMerge = true;
    uint64_t key;    // lane j < hk: the j-th entry by (distance, id)
    uint64_t amask;  // the alive entries (popped ones stay, as in the heap)
    int hk;
    int kres;        // k of the results: they are derived from this set (below)
    __device__ __forceinline__ void init(int k) {
        key = hkey(FLT_MAX, -1);
        amask = 0ull;
        hk = 0;
        kres = k;
    }
    // the alive mask with a slot opened at pos (entries pos.. move up one lane)
    __device__ __forceinline__ static uint64_t open_bit(uint64_t m, int pos) {
        const uint64_t low = (1ull << pos) - 1ull;  // pos <= 63
        return (m & low) | (1ull << pos) | ((m & ~low) << 1);
    }
    __device__ __forceinline__ void insert(int n, uint64_t nk, int lane) {
        // into lanes 0..n (n entries kept sorted; lane n is free)
        const int pos = __popcll(__ballot(lane < n && key < nk));
        const uint64_t up = dpp64<0x138>(key);  // wave_shr:1
        key = lane > pos ? up : (lane == pos ? nk : key);
        amask = open_bit(amask, pos);
    }
    __device__ __forceinline__ void seed(uint64_t nk, int lane) { insert(hk++, nk, lane); }
    __device__ __forceinline__ float top_dis() const { return hkey_dis(rdlane64(key, hk - 1)); }
    __device__ __forceinline__ uint64_t peek_min(int lane) const {
        return amask ? rdlane64(key, __builtin_ctzll(amask)) : ~0ull;
    }
    __device__ __forceinline__ bool pop_min(int lane, int32_t& v0, int& nb) {
        const uint32_t chi = (uint32_t)(key >> 32);
        const int first = __builtin_ctzll(amask);  // the sorted order: the smallest alive
        const uint32_t kmin = __builtin_amdgcn_readlane(chi, first);
        if (__popcll(__ballot(chi == kmin) & amask) > 1) return false;  // layout decides
        v0 = hkey_id(rdlane64(key, first));
        nb = __popcll(__ballot(lane < hk && chi < kmin));
        amask &= ~(1ull << first);
        return true;
    }
    __device__ __forceinline__ bool push(int ef, uint64_t nk, float dis, int& nvalid, int lane) {
        if (hk == ef) {
            const uint64_t top = rdlane64(key, hk - 1);
            if (dis >= hkey_dis(top)) return true;
        }
        // results smaller than the set (k < ef) keep, among equal distances,
        // the earliest arrivals, not the smallest ids: an arrival equal to a
        // kept entry ends this form
        if (kres < ef &&
            __ballot(lane < hk && (uint32_t)(key >> 32) == (uint32_t)__float_as_int(dis)))
            return false;
        if (hk == ef) {
            // the heap's top among several entries of the largest distance
            // depends on its layout
            if (hk >= 2 && (uint32_t)(rdlane64(key, hk - 2) >> 32) ==
                                   (uint32_t)(rdlane64(key, hk - 1) >> 32))
                return false;
            if ((amask >> (hk - 1)) & 1ull) --nvalid;
            amask &= ~(1ull << (hk - 1));
            insert(hk - 1, nk, lane);  // the top leaves, nk enters
        } else {
            insert(hk++, nk, lane);
        }
        ++nvalid;
        return true;
    }
    // search_from_candidates' result heap (HeapBlockResultHandler, strict
    // admission): every entry of this set below FLT_MAX that ranks < k — the
    // set holds the ef >= k smallest arrivals, the results the k smallest
    __device__ __forceinline__ void results(SortedQ& R, int k, int lane) const {
        const bool v = lane < hk && lane < k && (uint32_t)(key >> 32) < 0x7f7fffffu;
        R.key = v ? key : hkey(FLT_MAX, -1);
    }
};
// One hop's add_to_heap calls for the arrivals `todo` (lanes, arrival order)
// as one merge into CandSet: when no two of the distances involved are equal
// (the arrivals' among themselves and with the kept entries), the sequential
// pushes leave the set holding the ef smallest of its old entries and the
// arrivals — an arrival the set rejects has ef entries below it, and an
// eviction takes the largest — so each arrival's place is its rank among the
// set plus its rank among the arrivals, and the kept entries fill the other
// places in order.  False (nothing changed) on any equality, or on a tie
// inside the set when the merge evicts: then the hop runs the sequential
// pushes.
__device__ __forceinline__ bool hop_merge(CandSet& C, int ef, unsigned long long todo, float fdis,
                                          int32_t fv, int lane, int& nvalid) {
    const uint32_t cd = (uint32_t)(C.key >> 32);
    const uint32_t fd = (uint32_t)__float_as_int(fdis);
    const int hk = C.hk, m = __popcll(todo);
    const uint64_t cm = hk >= 64 ? ~0ull : ((1ull << hk) - 1ull);
    if (hk + m > ef) {
        const uint32_t cprev = __builtin_amdgcn_update_dpp(0u, cd, 0x138, 0xf, 0xf, false);
        if (__ballot(lane >= 1 && lane < hk && cprev == cd)) return false;
    }
    int arr = 0;  // lane r: the lane of the arrival of rank r
    uint64_t da = 0, tie = 0;
    for (unsigned long long t = todo; t; t &= t - 1ull) {
        const int j = __builtin_ctzll(t);
        const uint32_t a = __builtin_amdgcn_readlane(fd, j);
        const int ra = __popcll(__ballot(fd < a) & todo);
        const int pc = __popcll(__ballot(cd < a) & cm) + ra;
        tie |= (__ballot(cd == a) & cm) | (__ballot(fd == a) & todo & ~(1ull << j));
        if (pc < 64) da |= 1ull << pc;
        arr = lane == ra ? j : arr;
    }
    if (tie) return false;
    const uint64_t lt = (1ull << lane) - 1ull;
    const int nh = min(ef, hk + m);
    const int na = __popcll(da & lt);
    const bool isa = (da >> lane) & 1ull;
    const int al = __builtin_amdgcn_ds_bpermute(na << 2, arr);
    const uint64_t fa = bperm64(hkey(fdis, fv), al);
    const int src = (lane - na) & 63;
    const uint64_t fc = bperm64(C.key, src);
    C.key = isa ? fa : fc;
    C.amask = __ballot(lane < nh && (isa || ((C.amask >> src) & 1ull)));
    C.hk = nh;
    nvalid = __popcll(C.amask);
    return true;
}
}  // namespace

// the register kernel's query copy: ld floats, at least 128 for ref_rows64_4lane
__host__ __device__ inline int exact_reg_qpad(const HNSWDevice& g) {
    return g.ld < 128 ? 128 : g.ld;
}
// LDS before the visited bitmap: the query copy, its int8 image (128 B) and
// the image's scalars (6 doubles)
__host__ __device__ inline int exact_reg_head(const HNSWDevice& g) {
    return 4 * exact_reg_qpad(g) + 128 + 48;
}

namespace {
// The int8 prefilter of a hop's fresh neighbours (the rows' image:
// IndexHNSW::sync_device).  The query gets the same kind of image:
// xq = round((x - ox) / sx) with ox = min x, sx = (max x - min x) / 255, and
// with xh = sx xq + ox (exact real), ex >= |x - xh|.  For a row image
// yq = s q + o (ey >= |y - yq|):
//   |xh - yq|^2 = A2 + B2 - 2 (s (sx P + ox Q1) + o SA),
// A2 = |xh|^2, SA = sum xh, B2 = |yq|^2, Q1 = sum q, P = sum xq q (exact
// integers, v_dot4_u32_u8), and |x - y| >= |xh - yq| - ex - ey.  Evaluated in
// double with margins for B2's fp32 rounding and the double rounding, and the
// bound scaled by 1 - (2d + 16) 2^-24 so that it stays below the reference's
// own fp32 evaluation of the distance (ref_arith.h order).
__device__ __forceinline__ void q8_query_prep(const float* qs, int d, uint8_t* q8x, double* qd,
                                              int lane) {
    const float x0 = qs[lane], x1 = qs[lane + 64];
    const bool v0 = lane < d, v1 = lane + 64 < d;
    float mn = fminf(v0 ? x0 : INFINITY, v1 ? x1 : INFINITY);
    float mx = fmaxf(v0 ? x0 : -INFINITY, v1 ? x1 : -INFINITY);
#pragma unroll
    for (int m = 32; m; m >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, m));
        mx = fmaxf(mx, __shfl_xor(mx, m));
    }
    const double ox = (double)mn;
    double sx = ((double)mx - (double)mn) / 255.0;
    if (!(sx > 0.0)) sx = 1.0;
    double e2 = 0.0, a2 = 0.0, sa = 0.0;
    uint32_t q[2] = {0u, 0u};
    const float xv[2] = {x0, x1};
    const bool vv[2] = {v0, v1};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        if (!vv[h]) continue;
        const double t = rint(((double)xv[h] - ox) / sx);
        q[h] = (uint32_t)fmin(255.0, fmax(0.0, t));
        const double xh = sx * (double)q[h] + ox;
        const double e = (double)xv[h] - xh;
        e2 += e * e;
        a2 += xh * xh;
        sa += xh;
    }
    q8x[lane] = (uint8_t)q[0];
    q8x[lane + 64] = (uint8_t)q[1];
#pragma unroll
    for (int m = 32; m; m >>= 1) {
        e2 += __shfl_xor(e2, m);
        a2 += __shfl_xor(a2, m);
        sa += __shfl_xor(sa, m);
    }
    if (lane == 0) {
        qd[0] = sx;
        qd[1] = ox;
        qd[2] = a2;
        qd[3] = sa;
        qd[4] = sqrt(e2) * (1.0 + 1e-12) + 1e-12 * sqrt(a2) + 1e-300;
        qd[5] = 1.0 - (2.0 * d + 16.0) * 0x1p-24;
    }
}

// Lanes < nf hold the hop's fresh ids (arrival order).  Rows whose lower
// bound reaches thr (neither heap can take them) are dropped; the others
// are compacted to the low lanes in arrival order (sv); returns their count.
#ifndef HNSW_Q8PB
#define HNSW_Q8PB 2
#endif
__device__ __forceinline__ int q8_filter(const HNSWDevice& g, const uint8_t* q8x, const double* qd,
                                         int32_t fv, int nf, float thr, int lane, int32_t& sv) {
    const int gq = lane >> 2, jp = lane & 3;
    const int npass = (nf + 15) >> 4;
    const uint4 x0 = *(const uint4*)(q8x + 32 * jp), x1 = *(const uint4*)(q8x + 32 * jp + 16);
    const double sx = qd[0], ox = qd[1], a2 = qd[2], sa = qd[3], ex = qd[4], mref = qd[5];
    const double thr_d = (double)thr;
    bool keep = false;
    // HNSW_Q8PB passes of 16 rows with their loads in flight together
#pragma unroll 1
    for (int p0 = 0; p0 < npass; p0 += HNSW_Q8PB) {
        uint4 c0[HNSW_Q8PB], c1[HNSW_Q8PB];
        float pp[HNSW_Q8PB], q1[HNSW_Q8PB];
#pragma unroll
        for (int b = 0; b < HNSW_Q8PB; b++) {
            const int r = 16 * (p0 + b) + gq;
            const int32_t rg = __shfl(fv, r & 63);
            const uint32_t row = r < nf ? (uint32_t)rg : 0u;
            const uint4* cp = (const uint4*)(g.q8 + (size_t)row * 128 + 32 * jp);
            c0[b] = cp[0];
            c1[b] = cp[1];
            pp[b] = g.q8p[(size_t)row * 4 + jp];
            q1[b] = g.q8q1[row];
        }
#pragma unroll
        for (int b = 0; b < HNSW_Q8PB; b++) {
            const int p = p0 + b;
            if (p >= npass) break;  // wave-uniform
            uint32_t P = __builtin_amdgcn_udot4(x0.x, c0[b].x, 0u, false);
            P = __builtin_amdgcn_udot4(x0.y, c0[b].y, P, false);
            P = __builtin_amdgcn_udot4(x0.z, c0[b].z, P, false);
            P = __builtin_amdgcn_udot4(x0.w, c0[b].w, P, false);
            P = __builtin_amdgcn_udot4(x1.x, c1[b].x, P, false);
            P = __builtin_amdgcn_udot4(x1.y, c1[b].y, P, false);
            P = __builtin_amdgcn_udot4(x1.z, c1[b].z, P, false);
            P = __builtin_amdgcn_udot4(x1.w, c1[b].w, P, false);
            P += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)P, 0xB1, 0xf, 0xf, false);  // quad ^1
            P += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)P, 0x4E, 0xf, 0xf, false);  // quad ^2
            const int pb = __float_as_int(pp[b]);
            const float o = __int_as_float(__builtin_amdgcn_update_dpp(0, pb, 0x00, 0xf, 0xf, false));
            const float sc = __int_as_float(__builtin_amdgcn_update_dpp(0, pb, 0x55, 0xf, 0xf, false));
            const float ey = __int_as_float(__builtin_amdgcn_update_dpp(0, pb, 0xAA, 0xf, 0xf, false));
            const float b2 = __int_as_float(__builtin_amdgcn_update_dpp(0, pb, 0xFF, 0xf, 0xf, false));
            const double sab = (double)sc * (sx * (double)P + ox * (double)q1[b]) + (double)o * sa;
            const double d2 = a2 + (double)b2 - 2.0 * sab;
            const double mag = a2 + (double)b2 + 2.0 * fabs(sab);
            const double d2lo = d2 - 1e-7 * mag;
            bool rej = false;
            if (d2lo > 0.0) {
                const double t = sqrt(d2lo) * (1.0 - 1e-12) - ex - (double)ey;
                rej = t > 0.0 && t * t * mref >= thr_d;
            }
            // row 16 p + gq -> lane 16 p + gq
            const int got = __shfl((int)!rej, 4 * (lane & 15));
            if ((lane >> 4) == p) keep = got != 0;
        }
    }
    keep = keep && lane < nf;
    const unsigned long long sm = __ballot(keep);
    const int ns = __popcll(sm);
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int dst = keep ? __popcll(sm & lt) : ns + __popcll(~sm & lt);
    sv = __builtin_amdgcn_ds_permute(dst << 2, fv);
    return ns;
}
}  // namespace

// passes of 16 rows whose loads the register kernel issues together
#ifndef HNSW_PB
#define HNSW_PB 1
#endif
// fp32 rows 8 lanes per row, 8 per pass (half the registers of the 4-lane
// form; measured slower, also at 6 waves per SIMD: off)
#ifndef HNSW_FP32_8LANE
#define HNSW_FP32_8LANE 0
#endif
// the register kernel's waves per SIMD (its VGPR budget: 512 / HNSW_WPE)
#ifndef HNSW_WPE
#define HNSW_WPE 5
#endif
// Trace of the register kernel (FAISS_AMD_HNSW_TRACE=<file>, profiling): per
// query the core-clock cycles of each level-0 hop phase summed over its hops:
// [0] pop_min + count_below, [1] neighbour ids, [2] visited test-and-set,
// [3] distances, [4] heap updates, [5] hops, [6] fresh neighbours, [7] whole
// query, [8] 1 if the query was searched again with the heap layout, [9]
// replayed log entries, [10] arrivals that can enter a heap, [11] hops before
// the candidates fill, [12] fp32 rows after the int8 bound, [13] the
// next-pop prediction, [14] the replay log (of [4])
struct HopTrace {
    unsigned long long t[16];
    unsigned long long tc;
    __device__ __forceinline__ void tick(int ph) {
        const unsigned long long n = clock64();
        t[ph] += n - tc;
        tc = n;
    }
};

// The level-0 loop's state between a CandSet run that stopped at a
// layout-dependent decision and its continuation with CandLayout.  The CandSet
// run logs, per hop, a pop marker and the hop's arrivals in arrival order
// (the heap updates the layout depends on); replaying that log into a
// CandLayout rebuilds the reference's heap array at the stopping point, and
// the search goes on from there: the results, the visited table and every
// distance computed so far depend on the entry set alone and are kept.
constexpr uint64_t RLOG_POP = ~0ull;  // the marker (dis bits 0xffffffff: no distance)
constexpr int RLOG_CAP = (int)kHnswReplayCap;  // entries per query (global memory)
constexpr int RLOG_LDS = 640;  // entries per query when the log lives in the LDS
struct L0Run {
    int nvalid;
    float rmax;
    unsigned long long todo;  // the stopped hop's arrivals not yet applied (0: at pop_min)
    float fdis;               // that hop's arrivals (lanes)
    int32_t fv;
    int logpos;               // log entries written (> the log's capacity: overflowed)
    int stop;                 // log entries the replay applies
};

// the seed (:624-637): the entry point enters the candidates and the results
template <class CQ>
__device__ __forceinline__ void level0_seed(CQ& C, SortedQ& R, L0Run& S, uint32_t* vis, int k,
                                            int lane, int nearest, float d_nearest) {
    C.init(k);
    C.seed(hkey(d_nearest, nearest), lane);
    if (d_nearest < FLT_MAX) R.insert(k, hkey(d_nearest, nearest), lane);
    S.nvalid = 1;
    S.rmax = hkey_dis(rdlane64(R.key, k - 1));
    S.todo = 0ull;
    S.logpos = 0;
    if (lane == 0) vis[nearest >> 5] |= 1u << (nearest & 31);
    __syncthreads();
}

// search_from_candidates at level 0 (faiss/impl/HNSW.cpp:605-741) from state
// S with the candidate structure CQ (S.todo != 0: first the stopped hop's
// remaining arrivals); false when CQ (CandSet) met a decision that depends on
// the heap layout, with S describing where (rlog: CandSet's update log, or
// nullptr)
template <class CQ, bool TRACE, bool NB0>
__device__ __forceinline__ bool hnsw_level0(const HNSWDevice& g, const float* qs, uint32_t* vis,
                                            int k, int efSearch, int ef, int lane, CQ& C,
                                            L0Run& S, SortedQ& R, uint32_t& st_n2,
                                            uint32_t& st_ndis, uint32_t& st_nhops, HopTrace& tr,
                                            uint64_t* __restrict__ rlog, const uint8_t* q8x,
                                            const double* q8d, uint32_t& st_q8,
                                            uint32_t& st_x32, int logcap) {
    int nvalid = S.nvalid;
    float rmax = S.rmax;
    // the sequential add_to_heap calls (:678-689) for the arrivals `todo`
    // (lanes fdis, fv) of the hop whose log entries start at hp; false when C
    // stops (S then says where)
    auto apply = [&](unsigned long long todo, unsigned long long hop_todo, float fdis, int32_t fv,
                     int hp) -> bool {
        while (todo) {
            const int t = __builtin_ctzll(todo);
            const int32_t vt = __builtin_amdgcn_readlane(fv, t);
            const float dis = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fdis), t));
            const uint64_t nk = hkey(dis, vt);
            if (!C.push(ef, nk, dis, nvalid, lane)) {
                if constexpr (CQ::kMerge) {
                    C.results(R, k, lane);
                    rmax = hkey_dis(rdlane64(R.key, k - 1));
                }
                S.nvalid = nvalid;
                S.rmax = rmax;
                S.todo = todo;
                S.fdis = fdis;
                S.fv = fv;
                S.stop = hp + 1 + __popcll(hop_todo & ((1ull << t) - 1ull));
                return false;
            }
            todo &= todo - 1ull;
            if constexpr (!CQ::kMerge) {  // (CandSet: the results are derived from it)
                if (dis < rmax) {
                    R.insert(k, nk, lane);
                    rmax = hkey_dis(rdlane64(R.key, k - 1));
                }
            }
        }
        return true;
    };
    if (S.todo && !apply(S.todo, S.todo, S.fdis, S.fv, 0)) return false;
    if (TRACE) tr.tick(7);
    const int cnt = g.cum_nb[1] - g.cum_nb[0];
    // the next hop's neighbour ids, loaded during this hop's heap updates for
    // the node pop_min is predicted to take (pf_v; a hint: a wrong guess only
    // costs the load)
    int32_t pf_v = -1, pf_nb = -1;
    for (;;) {
        {
            if (nvalid <= 0) {  // candidates.size() == 0
                st_n2 = 1;
                break;
            }
            int32_t v0;
            int nb;
            if (!C.pop_min(lane, v0, nb)) {
                if constexpr (CQ::kMerge) {
                    C.results(R, k, lane);
                    rmax = hkey_dis(rdlane64(R.key, k - 1));
                }
                S.nvalid = nvalid;
                S.rmax = rmax;
                S.todo = 0ull;
                S.stop = S.logpos;
                return false;
            }
            nvalid--;
            if (nb >= efSearch) {
                st_n2 = nvalid == 0 ? 1u : 0u;
                break;
            }
            if (TRACE) tr.tick(0);
            // neighbours of v0 in stored order, fresh ones compacted to lanes
            // 0..nf-1 (their arrival order)
            int32_t v1 = -1;
            if (v0 == pf_v)
                v1 = pf_nb;
            else if (lane < cnt)
                v1 = NB0 ? g.nb0[(int64_t)v0 * g.nb0_stride + lane]
                         : g.neighbors[g.offsets[v0] + g.cum_nb[0] + lane];
            const unsigned long long neg =
                    __ballot(lane < cnt && v1 < 0) | (cnt < 64 ? (~0ull << cnt) : 0ull);
            const int jmax = neg ? __ffsll((long long)neg) - 1 : 64;
            if (TRACE) tr.tick(1);
            // visited test-and-set: the bits as they were before this hop
            // decide; a node listed twice in this neighbour list (the atomic
            // then finds the bit another lane of this hop set) is visited at
            // its first position, so only then the lanes are compared pairwise
            const uint32_t vbit = 1u << (v1 & 31);
            bool fresh = lane < jmax && !(vis[v1 >> 5] & vbit);
            uint32_t old = 0u;
            if (fresh) old = atomicOr(&vis[v1 >> 5], vbit);
            if (__ballot(fresh && (old & vbit)) != 0ull)
                for (int i = 0; i < jmax; i++)
                    fresh &= !(i < lane && __builtin_amdgcn_readlane(v1, i) == v1);
            const unsigned long long fm = __ballot(fresh);
            int nf = __popcll(fm);
            const unsigned long long lt = (1ull << lane) - 1ull;
            const int dst = fresh ? __popcll(fm & lt) : nf + __popcll(~fm & lt);
            int32_t fv = __builtin_amdgcn_ds_permute(dst << 2, v1);
            if (TRACE) tr.tick(2);
            st_ndis += (uint32_t)nf;  // (every fresh neighbour is a distance computation)
            // the bounds every arrival of this hop must beat to enter a heap:
            // the result's rmax and, once full, the candidates' top (both only
            // fall during the hop)
            const bool full0 = C.hk == ef;
            const float ctop0 = full0 ? C.top_dis() : FLT_MAX;
            if (NB0 && g.q8 && full0 && nf > 0) {
                // int8 lower bounds first: only the rows that may enter a
                // heap have their fp32 row read (c4: ~5 of ~42 per hop)
                int32_t sv;
                st_q8 += (uint32_t)nf;
                // (CandSet: the results' bound is one of its entries, <= ctop0)
                nf = q8_filter(g, q8x, q8d, fv, nf, CQ::kMerge ? ctop0 : fmaxf(rmax, ctop0),
                               lane, sv);
                st_x32 += (uint32_t)nf;
                fv = sv;
                if (TRACE) tr.t[12] += (unsigned long long)nf;
            }
            // 4 lanes per row, 16 rows per pass, HNSW_PB passes' loads in flight
            // (reference order)
            float fdis = 0.f;
            if (g.d <= 128)
#if HNSW_FP32_8LANE
                fdis = ref_rows64_8lane<true, 16>(qs, qs, g.storage, g.ld, g.d,
                                                  lane < nf ? (uint32_t)fv : 0u, nf, lane);
#else
                fdis = ref_rows64_4lane_pb<true, 16, HNSW_PB>(qs, qs, g.storage, g.ld, g.d,
                                                        lane < nf ? (uint32_t)fv : 0u, nf, lane);
#endif
            else if (lane < nf)
                fdis = l2_row(qs, g.storage + (int64_t)fv * g.ld, g.d);
            st_nhops += 1;
            if (TRACE) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                tr.tick(3);
                tr.t[5] += 1;
                tr.t[6] += (unsigned long long)nf;
            }
            // add_to_heap (:678-689) for each fresh neighbour in arrival
            // order.  Only arrivals that can change a heap are visited: the
            // result admits dis < rmax (rmax only falls during the hop); a full
            // candidate heap admits dis < its top (which only falls while
            // full); a heap not yet full takes every arrival.
            if (NB0) {
                // next pop: the closest arrival if it enters and beats the
                // closest alive candidate, else that candidate
                const uint32_t fb = lane < nf ? (uint32_t)__float_as_int(fdis) : 0xffffffffu;
                const uint32_t amin = wave_min_u32(fb);
                const uint64_t cmin = C.peek_min(lane);
                int32_t pred = cmin != ~0ull ? hkey_id(cmin) : -1;
                if (nf > 0 && (!full0 || __int_as_float((int)amin) < ctop0) &&
                    amin < (uint32_t)(cmin >> 32))
                    pred = __builtin_amdgcn_readlane(
                            fv, __builtin_ctzll(__ballot(lane < nf && fb == amin)));
                pf_v = pred;
                if (pred >= 0 && lane < cnt) pf_nb = g.nb0[(int64_t)pred * g.nb0_stride + lane];
            }
            if (TRACE) tr.tick(13);
            unsigned long long todo = __ballot(
                    lane < nf && (!full0 || fdis < ctop0 || (!CQ::kMerge && fdis < rmax)));
            const unsigned long long hop_todo = todo;
            if (TRACE) {
                tr.t[10] += (unsigned long long)__popcll(todo);
                tr.t[11] += full0 ? 0ull : 1ull;
            }
            int hp = 0;  // this hop's log position
            if constexpr (CQ::kMerge) {
                // the replay log: this hop's pop, then its arrivals in order
                if (rlog) {
                    hp = S.logpos;
                    const int m = __popcll(todo);
                    if (hp + 1 + m <= logcap) {
                        // streaming stores: the log is read back only
                        // after a tie (~1.5 % of c4's queries)
                        if (lane == 0) __builtin_nontemporal_store(RLOG_POP, rlog + hp);
                        if ((todo >> lane) & 1ull)
                            __builtin_nontemporal_store(hkey(fdis, fv),
                                                        rlog + hp + 1 + __popcll(todo & lt));
                    }
                    S.logpos = hp + 1 + m;
                }
                if (TRACE) tr.tick(14);
                if (todo && hop_merge(C, ef, todo, fdis, fv, lane, nvalid)) todo = 0ull;
            }
            if (todo && !apply(todo, hop_todo, fdis, fv, hp)) return false;
        }
        if (TRACE) tr.tick(4);
    }
    if constexpr (CQ::kMerge) C.results(R, k, lane);
    return true;
}

// CandSet's log up to S.stop into a fresh CandLayout seeded like it: the
// heap array the reference holds at that point (the pops before the stop
// took a unique minimum, the evictions a unique top)
// (took the heap).  Every entry below S.stop was written by this query's
// CandSet run (a hop is logged only when all of it fits the capacity, and the
// replay runs only when nothing overflowed), so an entry that names no node
// means the log is corrupt: the replay stops there and returns the number of
// such entries read (the caller then searches level 0 again and counts it in
// the `replay_bad` statistic, which the tests assert to be 0).
__device__ __forceinline__ int level0_replay(CandLayout& C, const uint64_t* __restrict__ rlog,
                                             int stop, int ef, int ntotal, int lane,
                                             int nearest, float d_nearest) {
    C.init(0);
    C.seed(hkey(d_nearest, nearest), lane);
    int dummy = 0;
    for (int base = 0; base < stop; base += 64) {
        const uint64_t e = base + lane < stop ? rlog[base + lane] : RLOG_POP;
        const int cnt = stop - base < 64 ? (int)(stop - base) : 64;
        // an entry is a pop marker or a key naming a node of the graph
        const bool bad = base + lane < stop && e != RLOG_POP &&
                         (uint32_t)hkey_id(e) >= (uint32_t)ntotal;
        const unsigned long long badm = __ballot(bad);
        if (badm) return __popcll(badm);
        for (int i = 0; i < cnt; i++) {
            const uint64_t v = rdlane64(e, i);
            if (v == RLOG_POP) {
                int32_t v0;
                int nb;
                C.pop_min(lane, v0, nb);
            } else {
                C.push(ef, v, hkey_dis(v), dummy, lane);
            }
        }
    }
    return 0;
}

// The reference's HNSW::search for ef, k <= 64, one wave per query: the
// greedy descent, then level 0 with the CandSet form (int8 prefilter, one
// merge per hop, results derived from the set); a query whose search meets a
// layout-dependent decision continues with CandLayout from its replayed log
// (rlog, or the LDS when LOGLDS), or searches level 0 again when the log
// overflowed (layout = 1: every query with CandLayout — tests).  Results are
// the reference's, bit for bit, either way.
template <bool LDS_VISITED, bool TRACE, bool NB0, bool LOGLDS>
__global__ __launch_bounds__(64, HNSW_WPE) void k_hnsw_exact_reg(HNSWDevice g, const float* __restrict__ x,
                                                       int ldx, int64_t n, int k, int efSearch,
                                                       int ef, float* __restrict__ D,
                                                       int64_t* __restrict__ I,
                                                       int32_t* __restrict__ I32,
                                                       uint32_t* __restrict__ vis_global,
                                                       int64_t vwords,
                                                       unsigned long long* __restrict__ stats,
                                                       const uint32_t* __restrict__ only,
                                                       const uint32_t* __restrict__ qidx, int layout,
                                                       unsigned long long* __restrict__ trace,
                                                       uint64_t* __restrict__ rlog, int rcap) {
    // qidx: compact launch over listed queries (input row qidx[b], output
    // row b); else query b, output row b.  rcap: entries of the replay log a
    // query may use (<= RLOG_CAP for rlog, <= RLOG_LDS in the LDS; smaller in
    // tests, to force the overflow path)
    const int64_t q = qidx ? (int64_t)qidx[blockIdx.x] : (int64_t)blockIdx.x;
    const int64_t qo = blockIdx.x;
    if (only && only[q] == 0u) return;
    HopTrace tr;
    if (TRACE) {
#pragma unroll
        for (int j = 0; j < 16; j++) tr.t[j] = 0;
        tr.tc = clock64();
    }
    const unsigned long long tq = TRACE ? tr.tc : 0ull;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int qpad = exact_reg_qpad(g);
    float* qs = sm;  // [qpad]
    uint8_t* q8x = (uint8_t*)(sm + qpad);      // [128] the query's int8 image
    double* q8d = (double*)(q8x + 128);        // [6] its scalars
    uint32_t* vis = LDS_VISITED ? (uint32_t*)((char*)sm + exact_reg_head(g))
                                : vis_global + blockIdx.x * vwords;
    const int lane = threadIdx.x;
    for (int j = lane; j < qpad; j += 64) qs[j] = j < g.d ? x[q * ldx + j] : 0.f;
    for (int64_t w = lane; w < vwords; w += 64) vis[w] = 0u;
    SortedQ R;  // results: heap_heapify<CMax> (Heap.h:316-339) = k x (FLT_MAX, -1)
    R.key = hkey(FLT_MAX, -1);
    __syncthreads();
    if (NB0 && g.q8) {
        q8_query_prep(qs, g.d, q8x, q8d, lane);
        __syncthreads();
    }
    uint32_t st_n2 = 0, st_ndis = 0, st_nhops = 0;
    uint32_t st_q8 = 0, st_x32 = 0;  // rows the int8 bound read / of them read in fp32
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
        // ---- level 0
        const uint32_t up_ndis = st_ndis, up_nhops = st_nhops;
        // the replay log: in the LDS after the visited bitmap (LOGLDS), else
        // this query's slice of rlog
        const int logcap = LOGLDS ? min(rcap, RLOG_LDS) : min(rcap, RLOG_CAP);
        uint64_t* qlog = LOGLDS ? (uint64_t*)((char*)sm + exact_reg_head(g) +
                                              ((4 * vwords + 7) & ~(int64_t)7))
                                : (rlog ? rlog + (int64_t)blockIdx.x * RLOG_CAP : nullptr);
        L0Run S;
        bool done = false;
        if (!layout) {
            CandSet C;
            level0_seed(C, R, S, vis, k, lane, nearest, d_nearest);
            done = hnsw_level0<CandSet, TRACE, NB0>(g, qs, vis, k, efSearch, ef, lane, C, S, R, st_n2,
                                               st_ndis, st_nhops, tr, qlog, q8x, q8d, st_q8,
                                               st_x32, logcap);
        }
        if (!done) {
            CandLayout C;
            if (TRACE) tr.t[8] = 1;
            int how = 1;  // 0: replayed, 1: log overflowed or absent, 2: log corrupt
            if (!layout && qlog && S.logpos <= logcap) {
                // continue from the stopping point with the replayed heap
                how = level0_replay(C, qlog, S.stop, ef, g.ntotal, lane, nearest, d_nearest)
                              ? 2
                              : 0;
                if (TRACE) tr.t[9] = (unsigned long long)S.stop;
            }
            if (stats && lane == 0 && !layout)
                atomicAdd(&stats[6 + how], 1ull);
            if (how != 0) {
                // again from the start: fresh visited table, results, counters
                __syncthreads();
                for (int64_t w = lane; w < vwords; w += 64) vis[w] = 0u;
                R.key = hkey(FLT_MAX, -1);
                st_n2 = 0;
                st_ndis = up_ndis;
                st_nhops = up_nhops;
                st_q8 = st_x32 = 0;
                __syncthreads();
                level0_seed(C, R, S, vis, k, lane, nearest, d_nearest);
            }
            hnsw_level0<CandLayout, TRACE, NB0>(g, qs, vis, k, efSearch, ef, lane, C, S, R, st_n2,
                                                st_ndis, st_nhops, tr, nullptr, q8x, q8d, st_q8,
                                                st_x32, 0);
        }
    }
    if (TRACE && lane == 0) {
        tr.t[7] = clock64() - tq;
        for (int j = 0; j < 16; j++) trace[qo * 16 + j] = tr.t[j];
    }
    if (stats && lane == 0 && g.entry_point >= 0) {
        atomicAdd(&stats[0], 1ull);
        atomicAdd(&stats[1], (unsigned long long)st_n2);
        atomicAdd(&stats[2], (unsigned long long)st_ndis);
        atomicAdd(&stats[3], (unsigned long long)st_nhops);
        atomicAdd(&stats[4], (unsigned long long)(st_ndis - st_q8 + st_x32));
        atomicAdd(&stats[5], (unsigned long long)st_q8);
    }
    // heap_reorder<CMax> (Heap.h:421-450): the kept (dis, id) ascending, the
    // placeholders (id -1) after them as (FLT_MAX, -1)
    if (lane < k) {
        const int32_t id = hkey_id(R.key);
        const float dv = id != -1 ? hkey_dis(R.key) : FLT_MAX;
        if (D) D[qo * k + lane] = dv;
        if (I) I[qo * k + lane] = id;
        if (I32) I32[qo * k + lane] = id;
    }
}

// ---------------------------------------------------------------- wide
// max(efSearch, k) > 128 (the reference harness's grid: efSearch up to 3
// nprobe, nprobe into the thousands — 60 % of its rows past ef 64).  The
// batched form of k_hnsw_search with the candidate set in the LDS instead
// of registers: one wave per query, the MinimaxHeap's entries as one sorted
// array of 64-bit keys (distance bits | id << 1 | alive) of at most ef
// entries, so that
//   * pop_min is the first alive entry (a position kept across hops; the
//     next alive one is found by one 64-entry ballot), count_below(d0) its
//     position (minus the dead entries of equal distance just before it);
//   * a hop's arrivals that can enter (the set not full, or below its
//     largest key) are compacted, sorted by the narrowest network and merged:
//     arrival j lands at j + lower_bound(j) (one binary search per lane),
//     every entry from the first arrival's place on moves up by the number of
//     arrivals below it (a backward pass, 64 entries per step, read before
//     written), entries pushed past ef are evicted (MinimaxHeap::push evicts
//     the max, faiss/impl/HNSW.cpp:1096-1107);
//   * the results are not kept: the result heap holds the k smallest
//     arrivals with strict admission, the set the ef >= k smallest, so they
//     are the set's first k entries below FLT_MAX.
// For distinct distances every step equals the reference's sequential heap
// updates (faiss/impl/HNSW.cpp:605-741); an equal distance where the
// reference's heap layout or arrival order decides — pop_min among equal
// alive minima, an arrival at the full set's largest distance, equal
// distances at the kept-ef or the k-th boundary — flags the query for the
// sequential kernel, as k_hnsw_search does.  Fresh neighbours whose certified
// int8 lower bound exceeds the full set's largest distance (q8_filter) cannot
// enter: their fp32 rows are not read.
constexpr uint64_t kWAlive = 1ull << 31;
__device__ __forceinline__ uint64_t wkey(float d, int32_t id) {
    return ((uint64_t)__float_as_uint(d) << 32) | kWAlive | (uint64_t)(uint32_t)id;
}
__device__ __forceinline__ float wdis(uint64_t e) { return __uint_as_float((uint32_t)(e >> 32)); }
__device__ __forceinline__ int32_t wid(uint64_t e) { return (int32_t)((uint32_t)e & 0x7fffffffu); }
// entries of cs[0, S) below an alive key (dead entries of its distance
// included, whatever their ids): a branchless binary search
__device__ __forceinline__ int wide_lower_bound(const uint64_t* cs, int S, uint64_t key) {
    int lb = 0;
    int st = 1;
    while (2 * st <= S) st *= 2;
    for (; st > 0; st >>= 1)
        if (lb + st <= S && cs[lb + st - 1] < key) lb += st;
    return lb;
}

// the LDS head of the wide kernel: the query (>= 128 floats), its int8 image
// and scalars (exact_reg_head), then the candidate set and the visited bitmap
__host__ __device__ inline size_t wide_lds_bytes(const HNSWDevice& g, int ef) {
    return (size_t)exact_reg_head(g) + 8 * (size_t)ef;
}

// INPLACE (FAISS_AMD_HNSW_INPLACE=1): a flagged query is searched again by
// the sequential body right here, as soon as the wave knows (no re-run
// launch after the whole batch); its flag is written 0.  The launch's LDS
// then holds the larger of the two layouts.
template <bool LDS_VISITED, bool TRACE = false, bool INPLACE = false>
__global__ __launch_bounds__(64) void k_hnsw_wide(HNSWDevice g, const float* __restrict__ x,
                                                  int ldx, int64_t n, int k, int efSearch, int ef,
                                                  float* __restrict__ D, int64_t* __restrict__ I,
                                                  int32_t* __restrict__ I32,
                                                  uint32_t* __restrict__ vis_global,
                                                  int64_t vwords,
                                                  unsigned long long* __restrict__ stats,
                                                  uint32_t* __restrict__ tie_flags,
                                                  unsigned long long* __restrict__ tb = nullptr,
                                                  ArrivalLog alog = ArrivalLog{}) {
    // TRACE (FAISS_AMD_HNSW_TRACE, profiling): per query the cycles of the
    // level-0 phases summed over its hops — [0] pop_min + count_below, [1]
    // neighbour ids, [2] visited, [3] int8 bound, [4] fp32 rows, [5] compact +
    // sort + lower_bound, [6] merge, [7] whole query; [8] flagged, [9] hops,
    // [10] fresh, [11] arrivals that enter, [12] fp32 rows, [13] merge steps,
    // [14] hops pushed one at a time, [15] hops whose neighbour ids were
    // prefetched
    HopTrace tr;
    if (TRACE) {
#pragma unroll
        for (int j = 0; j < 16; j++) tr.t[j] = 0;
        tr.tc = clock64();
    }
    const unsigned long long tq = TRACE ? tr.tc : 0ull;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int qpad = exact_reg_qpad(g);
    float* qs = sm;                                   // [qpad]
    uint8_t* q8x = (uint8_t*)(sm + qpad);             // [128]
    double* q8d = (double*)(q8x + 128);               // [6]
    uint64_t* cs = (uint64_t*)(q8x + 176);            // sorted candidate set [ef]
    uint32_t* vis = LDS_VISITED ? (uint32_t*)(cs + ef) : vis_global + blockIdx.x * vwords;
    const int lane = threadIdx.x;
    const int64_t q = blockIdx.x;
    for (int j = lane; j < qpad; j += 64) qs[j] = j < g.d ? x[q * ldx + j] : 0.f;
    for (int64_t w = lane; w < vwords; w += 64) vis[w] = 0u;
    __syncthreads();
    const bool use_q8 = g.q8 != nullptr && g.d <= 128;
    if (use_q8) q8_query_prep(qs, g.d, q8x, q8d, lane);
    __syncthreads();
    uint32_t tie = 0u;     // 1 pop-tie window, 4 (k == ef) eviction at a tied max, 8 k-th boundary
    float dvmin = WS_INF;  // (k == ef) smallest distance of an eviction at a tied max
    uint32_t st_n2 = 0, st_ndis = 0, st_nhops = 0, st_q8 = 0, st_x32 = 0;
    int S = 0;             // entries of the set
    if (g.entry_point >= 0) {
        // ---- greedy descent on the upper levels (HNSW.cpp:852-924)
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
        // ---- level 0: the set seeded with the entry (HNSW.cpp:967-972)
        if (lane == 0) {
            cs[0] = wkey(d_nearest, nearest);
            vis[nearest >> 5] |= 1u << (nearest & 31);
        }
        S = 1;
        int nalive = 1, fa = 0;  // alive entries (MinimaxHeap::nvalid), first alive
        float win = WS_INF;      // the distance of an open pop-tie window
        // the next hop's neighbour ids, loaded during this hop for the entry
        // expected to be popped next (the next alive one; a hint: a wrong
        // guess only costs the load)
        int32_t pf_v = -1, pf_nb = -1;
        __syncthreads();
        const int cnt = g.cum_nb[1] - g.cum_nb[0];
        const unsigned long long lt = (1ull << lane) - 1ull;
        for (;;) {
            if (TRACE) tr.tick(7);
            // the window closes once its distance's members are all popped
            if (win < WS_INF && (nalive <= 0 || wdis(cs[fa]) > win)) win = WS_INF;
            if (nalive <= 0) {  // candidates.size() == 0
                st_n2 = 1;
                break;
            }
            // ---- pop_min: the first alive entry.  Another alive entry of its
            // distance (right after it: dead entries of a distance sort
            // first) — the reference pops the highest heap slot among them,
            // so the members' expansion order is its layout's: a window opens
            // in which an arrival at or below that distance flags the query
            // (one LDS read: lane l holds entry fa - 1 + l)
            const int ip = fa - 1 + lane;
            const uint64_t ew = ip >= 0 && ip < S ? cs[ip] : ~0ull;
            const uint64_t e0 = rdlane64(ew, 1);
            const float d0 = wdis(e0);
            const int32_t v0 = wid(e0);
            if (fa + 1 < S && wdis(rdlane64(ew, 2)) == d0) win = d0;
            const unsigned long long am = __ballot(lane >= 2 && ip < S && (ew & kWAlive)) >> 2;
            __syncthreads();
            if (lane == 0) cs[fa] = e0 & ~kWAlive;
            nalive--;
            int nfa = S;
            if (am) {
                nfa = fa + __ffsll((long long)am);
            } else if (nalive > 0) {
                for (int b0 = fa + 63; b0 < S; b0 += 64) {
                    const int ii = b0 + lane;
                    const unsigned long long m2 = __ballot(ii < S && (cs[ii] & kWAlive));
                    if (m2) {
                        nfa = b0 + __ffsll((long long)m2) - 1;
                        break;
                    }
                }
            }
            // ---- count_below(d0): every entry below d0, dead ones included
            int nb = fa;
            if (fa > 0 && wdis(rdlane64(ew, 0)) == d0) {
                for (int b1 = fa; b1 > 0; b1 -= 64) {
                    const int ii = b1 - 64 + lane;
                    const unsigned long long m3 = __ballot(ii >= 0 && wdis(cs[ii >= 0 ? ii : 0]) == d0);
                    nb -= __popcll(m3);
                    if (m3 != ~0ull) break;
                }
            }
            if (nb >= efSearch) {
                st_n2 = nalive == 0 ? 1u : 0u;
                break;
            }
            fa = nfa;
            // ---- neighbours of v0 in stored order, visited test-and-set (a
            // node listed twice is fresh at its first position only)
            if (TRACE) tr.tick(0);
            int32_t v1 = -1;
            if (v0 == pf_v) {
                v1 = pf_nb;
                if (TRACE) tr.t[15]++;
            } else if (lane < cnt) {
                v1 = g.nb0 ? g.nb0[(int64_t)v0 * g.nb0_stride + lane]
                           : g.neighbors[g.offsets[v0] + g.cum_nb[0] + lane];
            }
            pf_v = -1;
            if (g.nb0 && nfa < S) {
                pf_v = wid(cs[nfa]);
                pf_nb = lane < cnt ? g.nb0[(int64_t)pf_v * g.nb0_stride + lane] : -1;
            }
            const unsigned long long neg =
                    __ballot(lane < cnt && v1 < 0) | (cnt < 64 ? (~0ull << cnt) : 0ull);
            const int jmax = neg ? __ffsll((long long)neg) - 1 : 64;
            const uint32_t vbit = 1u << (v1 & 31);
            if (TRACE) tr.tick(1);
            bool fresh = lane < jmax && !(vis[v1 >> 5] & vbit);
            uint32_t old = 0u;
            if (fresh) old = atomicOr(&vis[v1 >> 5], vbit);
            if (__ballot(fresh && (old & vbit)) != 0ull)
                for (int i = 0; i < jmax; i++)
                    fresh &= !(i < lane && __builtin_amdgcn_readlane(v1, i) == v1);
            const unsigned long long fm = __ballot(fresh);
            const int nf = __popcll(fm);
            st_ndis += (uint32_t)nf;
            st_nhops += 1;
            if (nf == 0) {
                if (TRACE) {
                    tr.tick(2);
                    tr.t[9]++;
                }
                __syncthreads();
                continue;
            }
            const int dst = fresh ? __popcll(fm & lt) : nf + __popcll(~fm & lt);
            const int32_t fv = __builtin_amdgcn_ds_permute(dst << 2, v1);
            if (TRACE) {
                tr.tick(2);
                tr.t[9]++;
                tr.t[10] += (unsigned)nf;
            }
            // ---- the full set admits only keys below its largest distance:
            // the int8 bound drops rows that cannot reach it (strictly above
            // it, so no arrival at that distance is skipped)
            const bool full = S == ef;
            const float maxd = full ? wdis(cs[ef - 1]) : WS_INF;
            int32_t sv = fv;
            int ns = nf;
            if (use_q8 && full && maxd < FLT_MAX) {
                st_q8 += (uint32_t)nf;
                ns = q8_filter(g, q8x, q8d, fv, nf, __uint_as_float(__float_as_uint(maxd) + 1u),
                               lane, sv);
            }
            st_x32 += (uint32_t)ns;
            if (TRACE) {
                tr.tick(3);
                tr.t[12] += (unsigned)ns;
            }
            float fdis = WS_INF;
            if (ns > 0) {
                if (g.d <= 128)
                    fdis = ref_rows64_4lane_pb<true, 16, 1>(qs, qs, g.storage, g.ld, g.d,
                                                            lane < ns ? (uint32_t)sv : 0u, ns,
                                                            lane);
                else if (lane < ns)
                    fdis = l2_row(qs, g.storage + (int64_t)sv * g.ld, g.d);
            }
            if (TRACE) tr.tick(4);
            if (win < WS_INF) {
                // inside a window: an arrival reaching its distance, or one
                // at the full set's largest distance (dropped here, perhaps
                // entered in the reference's member order)
                if (__ballot(lane < ns && (fdis <= win || (full && fdis == maxd))) != 0ull) {
                    tie |= 1u;
                    break;
                }
            }
            // MinimaxHeap::push into the full set drops v >= max by distance
            // alone (HNSW.cpp:1096-1101)
            const bool enter = lane < ns && (!full || fdis < maxd);
            float cd = enter ? fdis : WS_INF;
            long long ci = enter ? (long long)(kWAlive | (uint32_t)sv) : WS_NOID;
            const int m = wave_compact(cd, ci, enter, lane);
            if (m > 0) {
                wave_sort_m(cd, ci, lane, m);
                const uint64_t akey =
                        lane < m ? (((uint64_t)__float_as_uint(cd) << 32) | (uint32_t)ci) : ~0ull;
                if (TRACE) {
                    tr.tick(5);
                    tr.t[11] += (unsigned)m;
                }
                // ---- the merge, from the top of the set down, 64 entries a
                // step: each step's entries move up by the arrivals below
                // them; an arrival is placed (its lower_bound lbr) in the step
                // whose entries it exceeds, the largest first.  The top step
                // decides, before anything is written, whether the largest
                // kept distance is shared by an arrival (then the hop's
                // pushes go one at a time, in arrival order)
                int lbr = S;      // lane j: arrival j's lower_bound once placed
                int jhi = m;      // arrivals [0, jhi) not yet placed
                int evl = 0;      // alive entries evicted
                float disc = WS_INF;  // smallest distance pushed past ef
                bool btie = false;
                for (int top = S;; top -= 64) {
                    const int base = top - 64;
                    const int i = base + lane;
                    const bool vv = i >= 0;
                    const uint64_t e = vv ? cs[i] : 0ull;
                    int jlo = jhi;
                    int le = 0;  // arrivals placed here at or below this lane's entry
                    while (jlo > 0) {
                        const uint64_t kj = rdlane64(akey, jlo - 1);
                        const int cj = __popcll(__ballot(vv && e < kj));
                        if (cj == 0 && base > 0) break;  // below this step
                        const int lbj = (base > 0 ? base : 0) + cj;
                        jlo--;
                        if (lane == jlo) lbr = lbj;
                        le += lbj <= i ? 1 : 0;
                    }
                    const int np = i + jlo + le;
                    if (top == S && S + m > ef) {
                        // arrivals kept: those below this step, and the ones
                        // placed here that land below ef
                        const int a = jlo + __popcll(__ballot(lane >= jlo && lane < m &&
                                                              lbr + lane < ef));
                        float Bd = a > 0 ? __int_as_float(__builtin_amdgcn_readlane(
                                                   __float_as_int(cd), a - 1))
                                         : -WS_INF;
                        const int sl = ef - a - 1;  // the last set entry kept
                        float ds0 = -WS_INF, ds1 = -WS_INF;
                        if (sl >= 0) ds0 = wdis(sl >= base ? rdlane64(e, sl - base) : cs[sl]);
                        if (sl + 1 < S) ds1 = wdis(sl + 1 >= base ? rdlane64(e, sl + 1 - base) : cs[sl + 1]);
                        Bd = fmaxf(Bd, ds0);
                        const int na = __popcll(__ballot(lane < ns && fdis == Bd));
                        btie = na >= 1 && (na >= 2 || ds0 == Bd || ds1 == Bd);
                        if (btie) break;  // (nothing written yet)
                    }
                    __syncthreads();
                    if (vv && np < ef) cs[np] = e;
                    const unsigned long long evm = __ballot(vv && np >= ef);
                    if (evm) {
                        evl += __popcll(__ballot(vv && np >= ef && (e & kWAlive)));
                        disc = fminf(disc, wdis(rdlane64(e, __ffsll((long long)evm) - 1)));
                    }
                    if (TRACE) tr.t[13]++;
                    jhi = jlo;
                    if (jhi == 0) break;
                }
                if (btie && win < WS_INF) {
                    tie |= 1u;
                    break;
                }
                if (btie) {
                    if (TRACE) tr.t[14]++;
                    // the hop's pushes one at a time in arrival order
                    for (int j = 0; j < ns; j++) {
                        const float dv =
                                __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fdis), j));
                        const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane(sv, j);
                        if (S == ef && dv >= wdis(cs[ef - 1])) continue;
                        const uint64_t key = ((uint64_t)__float_as_uint(dv) << 32) | kWAlive | vj;
                        const int p = wide_lower_bound(cs, S, key);
                        const int S1 = S < ef ? S + 1 : ef;
                        const uint64_t ev = S == ef ? cs[ef - 1] : 0ull;
                        for (int hi = S1 - 1; hi > p; hi -= 64) {
                            const int i = hi - lane;
                            const uint64_t e = i > p ? cs[i - 1] : 0ull;
                            __syncthreads();
                            if (i > p) cs[i] = e;
                            __syncthreads();
                        }
                        if (lane == 0) cs[p] = key;
                        __syncthreads();
                        nalive += 1;
                        if (S == ef) {
                            nalive -= (int)((ev & kWAlive) != 0ull);
                            if (wdis(ev) == wdis(cs[ef - 1])) dvmin = fminf(dvmin, wdis(ev));
                        }
                        if (p <= fa) fa = p;
                        S = S1;
                    }
                } else {
                    const int pa = lane + lbr;
                    const bool kept = lane < m && pa < ef;
                    if (kept) cs[pa] = akey;
                    // (arrival j lands at j + lbr_j, increasing: the kept ones
                    // are a prefix)
                    const int nk = __popcll(__ballot(kept));
                    if (nk < m)
                        disc = fminf(disc, __int_as_float(__builtin_amdgcn_readlane(
                                                   __float_as_int(cd), nk)));
                    // new first alive: the old one's new place, or the first arrival
                    const int cfa = __popcll(__ballot(lane < m && lbr <= fa));
                    nalive += nk - evl;
                    int nfa2 = fa < S && fa + cfa < ef ? fa + cfa : ef;
                    const int lb0 = __builtin_amdgcn_readfirstlane(lbr);
                    if (lb0 < ef) nfa2 = min(nfa2, lb0);
                    S = min(S + m, ef);
                    fa = min(nfa2, S);
                    __syncthreads();
                    // (k == ef) an eviction at a largest distance shared by a
                    // kept entry: the result heap evicts by (dis, id), the set
                    // dead entries first — they may keep different ids there
                    if (S == ef && disc < WS_INF && wdis(cs[ef - 1]) == disc)
                        dvmin = fminf(dvmin, disc);
                }
                if (TRACE) tr.tick(6);
            }
            __syncthreads();
        }
    }
    if (tie == 0u) {
        // the k-th boundary (k < ef): the reference's result heap admits
        // strictly, so its k-th distance shared by the next entry leaves the
        // kept ids to the arrival order
        if (k < ef && S > k) {
            const float kd = wdis(cs[k - 1]);
            if (kd < FLT_MAX && wdis(cs[k]) == kd) tie |= 8u;
        }
        // (k == ef) the divergent eviction's distance still the largest kept
        if (k == ef && S == ef && dvmin == wdis(cs[ef - 1])) tie |= 4u;
    }
    if (tie_flags && lane == 0) tie_flags[q] = INPLACE ? 0u : tie;
    if (TRACE && lane == 0) {
        tr.t[7] = clock64() - tq;
        tr.t[8] = tie != 0u;
#pragma unroll
        for (int j = 0; j < 16; j++) tb[q * 16 + j] = tr.t[j];
    }
    if (tie && tie_flags) {  // the sequential kernel redoes this query
        if constexpr (INPLACE) {
            __syncthreads();  // the set's LDS becomes the heaps'
            hnsw_exact_query<LDS_VISITED, false>(g, x, ldx, k, efSearch, ef, D, I, I32,
                                                 vis_global, vwords, stats, nullptr, alog, q, q,
                                                 (int64_t)blockIdx.x, sm);
        }
        return;
    }
    if (stats && lane == 0 && g.entry_point >= 0) {
        atomicAdd(&stats[0], 1ull);
        atomicAdd(&stats[1], (unsigned long long)st_n2);
        atomicAdd(&stats[2], (unsigned long long)st_ndis);
        atomicAdd(&stats[3], (unsigned long long)st_nhops);
        atomicAdd(&stats[4], (unsigned long long)(st_ndis - st_q8 + st_x32));
        atomicAdd(&stats[5], (unsigned long long)st_q8);
    }
    // heap_reorder (Heap.h:421-450): ascending by (dis, id) — the set orders
    // equal distances dead entries first, so a run of equal distances is
    // ranked by id
    const int kk = min(S, k);
    for (int j = lane; j < k; j += 64) {
        float dv = FLT_MAX;
        int32_t id = -1;
        int pos = j;
        if (j < kk) {
            const uint64_t e = cs[j];
            dv = wdis(e);
            id = wid(e);
            if (!(dv < FLT_MAX)) {
                dv = FLT_MAX;
                id = -1;
            } else if ((j > 0 && wdis(cs[j - 1]) == dv) || (j + 1 < kk && wdis(cs[j + 1]) == dv)) {
                int s0 = j, s1 = j;
                while (s0 > 0 && wdis(cs[s0 - 1]) == dv) s0--;
                while (s1 + 1 < kk && wdis(cs[s1 + 1]) == dv) s1++;
                pos = s0;
                for (int i = s0; i <= s1; i++) pos += wid(cs[i]) < id ? 1 : 0;
            }
        }
        if (D) D[q * k + pos] = dv;
        if (I) I[q * k + pos] = id;
        if (I32) I32[q * k + pos] = id;
    }
}

// the sequential kernel's arrival log (see hnsw_exact_launch); empty when off
static ArrivalLog make_arrival_log(const HNSWDevice& g, int k, int ef, void* alog,
                                   size_t alog_bytes, hipStream_t s) {
    ArrivalLog al;
    const char* nenv = getenv("FAISS_AMD_HNSW_NORB");
    const bool norb_on = nenv ? strcmp(nenv, "0") != 0 : k <= 512;
    if (alog && norb_on && g.ntotal > 0) {
        size_t P = 1;
        while (P < (size_t)k) P <<= 1;
        const size_t region = 8 * (seq_slots(ef) + seq_slots(k));
        al.cap = (int64_t)g.ntotal + 2;
        al.slots = alog_bytes > 256 ? (int64_t)((alog_bytes - 256) / (8 * (size_t)al.cap)) : 0;
        if (8 * P <= region && region >= 1024 && al.slots > 0) {
            al.ctr = (uint32_t*)alog;
            al.base = (uint64_t*)((char*)alog + 256);
            HIP_CHECK(hipMemsetAsync(al.ctr, 0, sizeof(uint32_t), s));
        } else {
            al = ArrivalLog{};
        }
    }
    return al;
}
// the sequential kernel over n queries (qidx: the listed ones, compact
// outputs), register heaps for ef, k <= 64
static void hnsw_exact_launch(const HNSWDevice& g, const float* x, int ldx, int64_t n, int k,
                              int efSearch, float* D, int64_t* I, int32_t* I32,
                              uint32_t* visited_scratch, int64_t vwords,
                              unsigned long long* stats, const uint32_t* only,
                              const uint32_t* qidx, hipStream_t s, float* gheap = nullptr,
                              uint64_t* rlog = nullptr, int rcap = 0, void* alog = nullptr,
                              size_t alog_bytes = 0) {
    const int ef = efSearch > k ? efSearch : k;
    const size_t lds_x = seq_lds_bytes(g.ld, ef, k);
    const bool x_lds_vis = lds_x + vwords * 4 <= 64 * 1024;
    if (lds_x > 64 * 1024) {
        // heaps in global scratch; the LDS keeps the query, the hop's fresh
        // neighbours and (when it fits) the visited bitmap
        FAISS_THROW_IF_NOT(gheap != nullptr);
        const size_t lds_g = seq_lds_bytes_gheap(g.ld);
        if (lds_g + vwords * 4 <= 64 * 1024)
            k_hnsw_exact<true, true><<<kgrid(n, 64), dim3(64), lds_g + vwords * 4, s>>>(
                    g, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, only, qidx,
                    gheap);
        else
            k_hnsw_exact<false, true><<<kgrid(n, 64), dim3(64), lds_g, s>>>(
                    g, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats, only,
                    qidx, gheap);
        HIP_LAUNCH_CHECK();
        return;
    }
    if (ef <= 64 && k <= 64) {  // register heaps
        const size_t lds_r = (size_t)exact_reg_head(g);
        const bool rvis = lds_r + vwords * 4 <= 64 * 1024;
        // FAISS_AMD_HNSW_LAYOUT=1: every query with the heap-layout form (tests)
        const char* lenv = getenv("FAISS_AMD_HNSW_LAYOUT");
        const int layout = lenv && !strcmp(lenv, "1") ? 1 : 0;
        // FAISS_AMD_HNSW_LOG=lds: the replay log in the LDS when it fits
        // beside the query and the visited bitmap within the 8 KB per work
        // group that keeps 20 of them on a CU (c4: 2 KB of bitmap); measured
        // no faster than the nontemporal stores to rlog (1.715 vs 1.692 ms,
        // same box), so rlog is the default
        const char* genv = getenv("FAISS_AMD_HNSW_LOG");
        const size_t lds_logb = (size_t)RLOG_LDS * 8 + ((vwords * 4) & 7);
        const bool lds_log = rlog && rvis && g.nb0 && genv && !strcmp(genv, "lds") &&
                             lds_r + (size_t)vwords * 4 + lds_logb <= 8192;
        const size_t lds_logx = lds_log ? lds_logb : 0;
        // FAISS_AMD_HNSW_TRACE=<file>: per-query hop-phase cycles (profiling)
        const char* tenv = getenv("FAISS_AMD_HNSW_TRACE");
        if (tenv && rvis) {
            unsigned long long* tb = nullptr;
            HIP_CHECK(hipMalloc(&tb, 128 * std::max<int64_t>(n, 1)));
            HIP_CHECK(hipMemsetAsync(tb, 0, 128 * std::max<int64_t>(n, 1), s));
            auto kt = lds_log ? k_hnsw_exact_reg<true, true, true, true>
                              : (g.nb0 ? k_hnsw_exact_reg<true, true, true, false>
                                       : k_hnsw_exact_reg<true, true, false, false>);
            kt<<<kgrid(n, 64), dim3(64), lds_r + vwords * 4 + lds_logx, s>>>(
                    g, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, only, qidx,
                    layout, tb, rlog, rcap);
            HIP_LAUNCH_CHECK();
            std::vector<unsigned long long> h((size_t)n * 16);
            HIP_CHECK(hipMemcpyAsync(h.data(), tb, 128 * n, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            HIP_CHECK(hipFree(tb));
            if (FILE* f = fopen(tenv, "ab")) {
                fwrite(h.data(), 128, n, f);
                fclose(f);
            }
            return;
        }
        auto kr = lds_log ? k_hnsw_exact_reg<true, false, true, true>
                  : rvis  ? (g.nb0 ? k_hnsw_exact_reg<true, false, true, false>
                                   : k_hnsw_exact_reg<true, false, false, false>)
                          : (g.nb0 ? k_hnsw_exact_reg<false, false, true, false>
                                   : k_hnsw_exact_reg<false, false, false, false>);
        kr<<<kgrid(n, 64), dim3(64), rvis ? lds_r + vwords * 4 + lds_logx : lds_r, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, rvis ? nullptr : visited_scratch, vwords,
                stats, only, qidx, layout, nullptr, rlog, rcap);
        HIP_LAUNCH_CHECK();
        return;
    }
    // the arrival log instead of the result heap (FAISS_AMD_HNSW_NORB=0: off,
    // =1: at any k): a pool of per-query slots after a 256-byte counter, when
    // the final selection's sort fits the heaps' LDS; by default for k <= 512
    // (c4 quantizer, 2000 queries all sequential: k 256 / ef 768 7.74 ->
    // 6.97 ms; k = ef = 1024 13.41 -> 13.55 ms, the selection's cost growing
    // with k while a replace_top near the heap's top stays shallow)
    const ArrivalLog al = make_arrival_log(g, k, ef, alog, alog_bytes, s);
    if (x_lds_vis)
        k_hnsw_exact<true><<<kgrid(n, 64), dim3(64), lds_x + vwords * 4, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, only, qidx,
                nullptr, al);
    else
        k_hnsw_exact<false><<<kgrid(n, 64), dim3(64), lds_x, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats, only,
                qidx, nullptr, al);
    HIP_LAUNCH_CHECK();
}
size_t hnsw_arrival_log_bytes(int64_t n, int64_t ntotal) {
    // (at most 256 MiB; slots past the pool fall back to the result heap)
    const size_t per = 8 * (size_t)(std::max<int64_t>(ntotal, 0) + 2);
    return std::min<size_t>((size_t)256 << 20, 256 + per * (size_t)std::max<int64_t>(n, 1));
}

// flagged queries -> compact list (any order: the queries are independent)
__global__ void k_flag_compact(const uint32_t* __restrict__ flags, int64_t n,
                               uint32_t* __restrict__ idx, uint32_t* __restrict__ count) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool f = q < n && flags[q] != 0u;
    const unsigned long long m = __ballot(f);
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (m && lane == __ffsll((long long)m) - 1) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1);
    if (f) idx[base + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)q;
}

void hnsw_flag_compact(const uint32_t* flags, int64_t n, uint32_t* idx, uint32_t* count,
                       hipStream_t s) {
    HIP_CHECK(hipMemsetAsync(count, 0, sizeof(uint32_t), s));
    if (n <= 0) return;
    k_flag_compact<<<kgrid(cdiv(n, 256), 256), dim3(256), 0, s>>>(flags, n, idx, count);
    HIP_LAUNCH_CHECK();
}

void hnsw_exact_listed(const HNSWDevice& g, const float* x, int ldx, const uint32_t* qidx,
                       int64_t nf, int k, int efSearch, float* D, int32_t* I32,
                       uint32_t* visited_scratch, int64_t vwords, unsigned long long* stats,
                       hipStream_t s, void* arrival_log, size_t arrival_log_bytes) {
    if (nf <= 0) return;
    hnsw_exact_launch(g, x, ldx, nf, k, efSearch, D, nullptr, I32, visited_scratch, vwords,
                      stats, nullptr, qidx, s, nullptr, nullptr, 0, arrival_log,
                      arrival_log_bytes);
}

size_t hnsw_heap_scratch_words(int k, int efSearch, int ld) {
    const int ef = efSearch > k ? efSearch : k;
    return seq_lds_bytes(ld, ef, k) > 64 * 1024 ? seq_heap_bytes(ef, k) / 4 : 0;
}
// FAISS_AMD_HNSW_WIDE_GVIS=1: the wide kernel's visited bitmap in global
// scratch even where it fits the LDS (fewer LDS bytes per wave: occupancy)
static bool wide_global_visited() {
    const char* e = getenv("FAISS_AMD_HNSW_WIDE_GVIS");
    return e && !strcmp(e, "1");
}
bool hnsw_visited_scratch_needed(int ld, int k, int efSearch, int64_t vwords) {
    // mirrors the LDS choices of the three kernels: any query may reach the
    // sequential kernel (ties of the batched one), the register kernel keeps
    // its own head (exact_reg_head) before the bitmap
    constexpr size_t kL = 64 * 1024;
    const int ef = efSearch > k ? efSearch : k;
    const size_t vb = 4 * (size_t)std::max<int64_t>(vwords, 0);
    const size_t lds_q = sizeof(float) * (size_t)ld;
    const size_t lds_x = seq_lds_bytes(ld, ef, k);
    const size_t lds_xg = lds_x > kL ? seq_lds_bytes_gheap(ld) : lds_x;
    bool need = lds_xg + vb > kL;
    if (ef <= 64 && k <= 64 && lds_x <= kL) {
        HNSWDevice g{};
        g.ld = ld;
        need = need || (size_t)exact_reg_head(g) + vb > kL;
    }
    if (hnsw_uses_wide(k, efSearch)) {
        HNSWDevice g{};
        g.ld = ld;
        need = need || wide_lds_bytes(g, ef) + vb > kL || wide_global_visited();
    } else if (hnsw_uses_batched(k, efSearch)) {
        need = need || lds_q + vb > kL;
    }
    return need;
}
bool hnsw_register_eligible(int k, int efSearch) {
    const int ef = efSearch > k ? efSearch : k;
    return ef <= 64 && k <= 64;
}
// the wide kernel (k_hnsw_wide): 128 < ef <= kHnswWideMaxEf (its sorted set
// in the LDS, 8 B per entry); FAISS_AMD_HNSW_WIDE=0: the sequential kernel
bool hnsw_uses_wide(int k, int efSearch) {
    const int ef = efSearch > k ? efSearch : k;
    const char* wenv = getenv("FAISS_AMD_HNSW_WIDE");
    if (wenv && !strcmp(wenv, "0")) return false;
    return ef > 128 && ef <= kHnswWideMaxEf;
}
bool hnsw_uses_batched(int k, int efSearch) {
    const int ef = efSearch > k ? efSearch : k;
    const char* menv = getenv("FAISS_AMD_HNSW");
    const bool prefer_batched = menv && !strcmp(menv, "batched");
    return (ef <= 128 && k <= kMaxK && (prefer_batched || !hnsw_register_eligible(k, efSearch))) ||
           hnsw_uses_wide(k, efSearch);
}
void hnsw_search(const HNSWDevice& g, const float* x, int ldx, int64_t n, int k, int efSearch,
                 float* D, int64_t* I, int32_t* I32, uint32_t* visited_scratch,
                 int64_t visited_words_per_query, unsigned long long* stats, uint32_t* flags,
                 hipStream_t s, KernelTimes* kt, bool defer, float* heap_scratch,
                 uint64_t* replay_log, int64_t replay_cap, void* arrival_log,
                 size_t arrival_log_bytes) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT_FMT(k >= 1, "k = %d must be >= 1", k);
    const int ef = efSearch > k ? efSearch : k;
    FAISS_THROW_IF_NOT(g.ld % 4 == 0);
    const int64_t vwords = visited_words_per_query;
    const size_t lds_q = sizeof(float) * g.ld;
    // FAISS_AMD_HNSW=batched: the batched kernel (+ sequential re-runs of
    // tied queries) also where the register kernel serves every query
    const bool batched = hnsw_uses_batched(k, efSearch);
    // sequential kernel: query | ef heap | k heap | 64 fresh | 8 scalars | visited
    // (heaps in global scratch when they do not fit)
    // the batched kernel: query | visited in the LDS when both fit
    const bool lds_vis = lds_q + (size_t)vwords * 4 <= 64 * 1024;
    if (hnsw_visited_scratch_needed(g.ld, k, efSearch, vwords)) {
        FAISS_THROW_IF_NOT(visited_scratch != nullptr);
        HIP_CHECK(hipMemsetAsync(visited_scratch, 0, sizeof(uint32_t) * vwords * n, s));
    }
    auto exact = [&](const uint32_t* only) {
        ScopedKernelTimer tm(kt, "hnsw_exact", 0.0, s);
        hnsw_exact_launch(g, x, ldx, n, k, efSearch, D, I, I32, visited_scratch, vwords, stats,
                          only, nullptr, s, heap_scratch, replay_cap > 0 ? replay_log : nullptr,
                          (int)std::min<int64_t>(replay_cap, kHnswReplayCap), arrival_log,
                          arrival_log_bytes);
    };
    // FAISS_AMD_HNSW_EXACT=1: every query through the sequential kernel (tests)
    const char* xenv = getenv("FAISS_AMD_HNSW_EXACT");
    if (!batched || (xenv && !strcmp(xenv, "1"))) {
        exact(nullptr);
        return;
    }
    if (hnsw_uses_wide(k, efSearch)) {
        ScopedKernelTimer tm(kt, "hnsw_wide", 0.0, s);
        const size_t lds_w = wide_lds_bytes(g, ef);
        // FAISS_AMD_HNSW_WIDE_Q8=0: every fresh row's fp32 distance (no int8 bound)
        const char* wq = getenv("FAISS_AMD_HNSW_WIDE_Q8");
        HNSWDevice gw = g;
        if (wq && !strcmp(wq, "0")) gw.q8 = nullptr;
        // FAISS_AMD_HNSW_TRACE=<file>: per-query level-0 phase cycles (profiling)
        const char* tenv = getenv("FAISS_AMD_HNSW_TRACE");
        // FAISS_AMD_HNSW_INPLACE=1: a flagged query is searched again by the
        // sequential body inside the wide kernel (its heaps in the LDS: the
        // launch holds the larger layout), not by a re-run after the batch
        const char* ienv = getenv("FAISS_AMD_HNSW_INPLACE");
        const size_t lds_x = seq_lds_bytes(g.ld, ef, k);
        const size_t lds_wi = std::max(lds_w, lds_x);
        const bool inplace = ienv && !strcmp(ienv, "1") && flags != nullptr &&
                             lds_wi <= 64 * 1024;
        if (tenv && lds_w + (size_t)vwords * 4 <= 64 * 1024) {
            unsigned long long* tb = nullptr;
            HIP_CHECK(hipMalloc(&tb, 128 * n));
            HIP_CHECK(hipMemsetAsync(tb, 0, 128 * n, s));
            k_hnsw_wide<true, true><<<kgrid(n, 64), dim3(64), lds_w + vwords * 4, s>>>(
                    gw, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, flags, tb);
            HIP_LAUNCH_CHECK();
            std::vector<unsigned long long> h((size_t)n * 16);
            HIP_CHECK(hipMemcpyAsync(h.data(), tb, 128 * n, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            HIP_CHECK(hipFree(tb));
            if (FILE* f = fopen(tenv, "ab")) {
                fwrite(h.data(), 128, n, f);
                fclose(f);
            }
        } else if (inplace) {
            const ArrivalLog al = make_arrival_log(g, k, ef, arrival_log, arrival_log_bytes, s);
            if (lds_wi + (size_t)vwords * 4 <= 64 * 1024 && !wide_global_visited())
                k_hnsw_wide<true, false, true><<<kgrid(n, 64), dim3(64), lds_wi + vwords * 4, s>>>(
                        gw, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, flags,
                        nullptr, al);
            else
                k_hnsw_wide<false, false, true><<<kgrid(n, 64), dim3(64), lds_wi, s>>>(
                        gw, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats,
                        flags, nullptr, al);
        } else if (lds_w + (size_t)vwords * 4 <= 64 * 1024 && !wide_global_visited())
            k_hnsw_wide<true><<<kgrid(n, 64), dim3(64), lds_w + vwords * 4, s>>>(
                    gw, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, flags);
        else
            k_hnsw_wide<false><<<kgrid(n, 64), dim3(64), lds_w, s>>>(
                    gw, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats,
                    flags);
        HIP_LAUNCH_CHECK();
    } else {
    ScopedKernelTimer tm(kt, "hnsw_search", 0.0, s);
    if (lds_vis) {
        size_t lds = lds_q + sizeof(uint32_t) * vwords;
        k_hnsw_search<true><<<kgrid(n, 64), dim3(64), lds, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, nullptr, vwords, stats, flags);
    } else {
        k_hnsw_search<false><<<kgrid(n, 64), dim3(64), lds_q, s>>>(
                g, x, ldx, n, k, efSearch, ef, D, I, I32, visited_scratch, vwords, stats, flags);
    }
    HIP_LAUNCH_CHECK();
    }
    if (flags) {
        if (getenv("FAISS_AMD_HNSW_STATS")) {  // debug: how many queries tie (synchronises)
            std::vector<uint32_t> h((size_t)n);
            HIP_CHECK(hipMemcpyAsync(h.data(), flags, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            size_t c = 0, r[4] = {0, 0, 0, 0};
            for (uint32_t f : h) {
                c += f != 0u;
                for (int b = 0; b < 4; b++) r[b] += (f >> b) & 1u;
            }
            fprintf(stderr,
                    "[faiss_amd] hnsw: %zu of %lld queries flagged for the sequential kernel "
                    "(pop order %zu, push at the max %zu, candidate boundary %zu, result "
                    "boundary %zu)\n",
                    c, (long long)n, r[0], r[1], r[2], r[3]);
        }
        // the flagged queries again, sequentially; the visited scratch of a
        // flagged query is reset by the kernel itself.  defer: the caller
        // re-runs them (hnsw_flag_compact + hnsw_exact_listed), overlapped
        // with its own work
        if (!defer) exact(flags);
    }
}

__global__ void k_gather_rows(const float* __restrict__ in, int ldi,
                              const uint32_t* __restrict__ idx, int64_t n, int d,
                              float* __restrict__ out, int ldo) {
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const float* src = in + (int64_t)idx[i] * ldi;
    for (int j = threadIdx.x; j < d; j += blockDim.x) out[i * ldo + j] = src[j];
}
void gather_rows(const float* in, int ldi, const uint32_t* idx, int64_t n, int d, float* out,
                 int ldo, hipStream_t s) {
    if (n <= 0) return;
    k_gather_rows<<<kgrid(n, 64), dim3(64), 0, s>>>(in, ldi, idx, n, d, out, ldo);
    HIP_LAUNCH_CHECK();
}
__global__ void k_scatter_rows(const uint32_t* __restrict__ src, int words,
                               const uint32_t* __restrict__ idx, int64_t n,
                               uint32_t* __restrict__ dst) {
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const int64_t q = idx[i];
    for (int j = threadIdx.x; j < words; j += blockDim.x) dst[q * words + j] = src[i * words + j];
}
void scatter_rows(const void* src, int row_words, const uint32_t* idx, int64_t n, void* dst,
                  hipStream_t s) {
    if (n <= 0 || row_words <= 0) return;
    k_scatter_rows<<<kgrid(n, 64), dim3(64), 0, s>>>((const uint32_t*)src, row_words, idx,
                                                         n, (uint32_t*)dst);
    HIP_LAUNCH_CHECK();
}

}  // namespace kern
}  // namespace faiss_amd
