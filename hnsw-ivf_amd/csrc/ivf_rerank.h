// ivf_rerank.h — the certified exact re-rank of the list-centric
// MFMA filters (IVF-Flat and IVF-PQ), split from kernels_ivf_mfma.hip so the
// two halves compile in parallel.
//
// (the filters: kernels_ivf_mfma.hip, kernels_pq_mfma.hip)
//
// Below: the original notes of the IVF-Flat scan.
//
// Reference hot loop: faiss/IndexIVFFlat.cpp:155-179 (exact sum (x-y)^2 per
// code, strict heap admission) driven by faiss/IndexIVF.cpp:595-631.
//
// Results are EXACT: bit-identical to the reference's fvec_L2sqr /
// fvec_inner_product evaluation order (ref_arith.h), which the CPU oracle
// restates:
//  A  k_ivf_mfma_filter: list-centric (list x 64 queries per workgroup).
//     <x,y> for a 64x64 tile on v_mfma_f32_32x32x2_f32 (one 32x32 block per
//     wave), approx = |x|^2 + |y|^2 - 2<x,y>; per (query, list) the KQ best
//     approx keys survive (4 threads per query, register queues).
//  B  k_ivf_rerank: one wave per query.  With B(c) a rigorous bound on
//     |approx - exact| (fp32 error analysis below), U = k-th smallest
//     approx+B over the kept candidates bounds the exact k-th distance;
//     every kept candidate with approx-B <= U gets its exact distance
//     (sequential fma chain, fp32 rows from HBM) and the exact top-k by
//     (dist, id) is emitted.  A list whose KQ-th kept candidate still has
//     approx - Bmax(list) <= U may have dropped a member: the query is
//     flagged.
//
// Error bound (d terms, u = 2^-24, g = d u / (1 - d u)):
//   |ip_mfma - ip| <= g sum|x_i y_i| <= g (|x|^2 + |y|^2) / 2
//   |approx - true| <= (2g + 3u)(|x|^2 + |y|^2)
//   |exact  - true| <= (g + 2u) * 2 (|x|^2 + |y|^2)
//   => |approx - exact| <= (4g + 7u)(|x|^2 + |y|^2); we use twice that.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "wave_select.h"
#include "exact_select.h"
#include "pq_ref.h"
#include "ref_arith.h"
#include "bf3.h"

namespace faiss_amd {
namespace kern {

// ---------------------------------------------------------------- B
// One wave per query.  U = k-th smallest upper bound over the kept entries
// bounds the exact k-th key.  A probe whose dropped bound is <= U "fails":
// all of its rows are re-ranked.  Every other probe contributes its kept
// entries with lb <= U.  The exact top-k over that candidate stream (with the
// reference tie rule, exact_select.h) is the reference result.
//
// Latency layout (two dependent global round trips on the common path):
//   1. the kept entries' raw 32-bit keys (V per lane), the probes' records
//      (dropped bound, largest margin M, arena offset / length) and the
//      query, all independent;  ub' = approx_hi + M and lb' = approx_lo - M
//      bracket each entry's exact key (M >= the entry's own margin);
//   2. the survivors' rows and ids.
// Invalid / empty probes carry empty entries (k_bucket_fill), so neither the
// assignment nor the list geometry arrays are read.
// Exact distances: 4 lanes per row (ref_arith.h order, see eval_rows64_direct).
constexpr int RR_CAP = 512;
constexpr int RR_XM = BDM / 8;
constexpr int RR_W = 1;  // waves (queries) per block: one, for fine-grained packing
// (the re-rank's barriers sit in wave-uniform branches: one wave per block)
static_assert(RR_W == 1, "k_ivf_rerank assumes one wave per block");

// Exact reference-order distance of the row `grow` each lane names: ref_arith.h
// ref_rows64_4lane (4 lanes per row, 16 rows per pass, no LDS staging).
// passes of 16 rows whose loads the Flat re-rank issues together when its
// candidates fill a prefix of the lanes (one round trip per RR_PB passes).
// 2 measured no faster: c4 re-rank 0.283 ms (1), 0.310 (2, spilling at 4
// waves per SIMD), 0.282 (2 at 3 waves per SIMD)
#ifndef RR_PB
#define RR_PB 1
#endif
template <bool L2>
__device__ __forceinline__ float eval_rows64_direct(const float* xr, const float* __restrict__ xq,
                                                    const float* __restrict__ codes, int ldc,
                                                    int d, uint32_t grow, bool valid, int lane) {
    return ref_rows64_4lane<L2, RR_XM>(xr, xq, codes, ldc, d, grow, valid, lane);
}

// IVF-PQ exact distance of the code at arena row `grow`, probe list l, in the
// reference's own arithmetic (pq_ref.h; faiss/IndexIVFPQ.cpp:604-700 tables,
// :861-933 scan, code_distance-avx2.h sum order):
//   table 1: dis0 = coarse_dis, sim = fma(-2, <x_m, c>, fma(2, <y_C,m, c>, |c|^2))
//   table 0: dis0 = 0, sim = |(x - y_C)_m - c|^2
// with the table entries in the fvec_*_ny order and the code sum in the
// distance_four_codes order.  xs: the query (LDS or global).
template <int PQD>
__device__ __forceinline__ float pq_sim(const PQArgs& pa, const float* xm, const float* ym,
                                        const float* c) {
    if (pa.table1) {
        const float s2 = ny_entry_c<false, PQD>(xm, c);
        const float P = fmaf(2.f, ny_entry_c<false, PQD>(ym, c), ref_norm(c, PQD));
        return fmaf(-2.f, s2, P);
    }
    float rr[PQD];
#pragma unroll
    for (int i = 0; i < PQD; i++) rr[i] = xm[i] - ym[i];
    return ny_entry_c<true, PQD>(rr, c);
}

template <int PQD>
__device__ __forceinline__ float pq_exact(const PQArgs& pa, const float* xs, uint32_t grow,
                                          uint32_t l, float d0) {
    const uint8_t* cp = pa.codes + (size_t)grow * pa.cs;
    const float* yc = pa.cent + (size_t)l * pa.ldcent;
    const int M = pa.M;
    const int m16 = pq_lane_span(M);
    float p[8], r = 0.f;
    int m0 = 0;
    // blocks of 8 sub-quantizers: their code bytes, centroid rows and coarse
    // rows are loaded together (code rows are 4-B aligned, m0 % 8 == 0)
    for (; m0 + 8 <= M; m0 += 8) {
        const uint32_t w0 = *(const uint32_t*)(cp + m0), w1 = *(const uint32_t*)(cp + m0 + 4);
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t j = ((u < 4 ? w0 : w1) >> (8 * (u & 3))) & 0xffu;
            const int m = m0 + u;
            t[u] = pq_sim<PQD>(pa, xs + m * PQD, yc + m * PQD,
                               pa.pq_cent + ((size_t)m * 256 + j) * PQD);
        }
        if (m0 < m16) {
#pragma unroll
            for (int u = 0; u < 8; u++) p[u] = m0 == 0 ? t[u] : p[u] + t[u];
            if (m0 + 8 == m16) r = reduce8(p);
        } else {
#pragma unroll
            for (int u = 0; u < 8; u++) r += t[u];
        }
    }
    for (int m = m0; m < M; m++) {
        const int j = cp[m];
        r += pq_sim<PQD>(pa, xs + m * PQD, yc + m * PQD, pa.pq_cent + ((size_t)m * 256 + j) * PQD);
    }
    return (pa.table1 ? d0 : 0.f) + r;
}

template <bool L2, int PQD = 0>
struct RerankStream {
    const uint32_t* surv;    // arena rows of the candidates (LDS)
    const uint16_t* sprobe;  // their probe rank
    const int64_t* ids;
    const float* xq;
    const float* codes;
    const float* xs;  // LDS copy of the query (first d & ~7 dims)
    int ldc, d, lane, nsv, KE, KT, E;
    uint32_t lowmask;
    bool overflow;  // candidate list did not fit: re-derive it from global
    const uint32_t* keys;
    float U;
    uint32_t my_fail;         // lane r: failing streams of probe r (4 bits)
    float my_m;               // lane r: probe r's margin
    uint32_t my_off, my_len;  // lane r: probe r's arena geometry
    uint32_t my_l;            // PQ: lane r: probe r's list
    float my_d0;              // PQ: lane r: probe r's coarse distance
    PQArgs pa;
    const uint8_t* sel;       // IDSelector mask of the arena rows (nullptr: all)
    bool fold;                // folded filter keys (ivf_decode_lo)

    // nv >= 0: the valid lanes are exactly 0..nv-1 (their rows' loads then
    // go out RR_PB passes at a time); nv < 0: any lanes
    __device__ __forceinline__ void emit(bool ok, uint32_t grow, int r, float& k1,
                                         long long& k2, int nv = -1) const {
        // the id load is issued before the rows', so both share one round trip
        const long long idv = ok ? (long long)ids[grow] : 0ll;
        float dis;
        if constexpr (PQD > 0) {
            const uint32_t l = __shfl(my_l, r);
            const float d0 = __shfl(my_d0, r);
            dis = ok ? pq_exact<PQD>(pa, xs, grow, l, d0) : 0.f;
        } else {
            if (nv >= 0)
                dis = ref_rows64_4lane_pb<L2, RR_XM, RR_PB>(xs, xq, codes, ldc, d, grow, nv, lane);
            else
                dis = eval_rows64_direct<L2>(xs, xq, codes, ldc, d, grow, ok, lane);
        }
        k1 = WS_INF;
        k2 = WS_NOID;
        if (ok) to_key(L2 ? 1 : 0, dis, idv, k1, k2);
    }
    template <class F>
    __device__ __forceinline__ void for_each(F f) const {
        if (!overflow) {
            for (int s0 = 0; s0 < nsv; s0 += 64) {
                bool ok = s0 + lane < nsv;
                const uint32_t grow = ok ? surv[s0 + lane] : 0u;
                const int rp = ok ? (int)sprobe[s0 + lane] : 0;
                const long long rank = ok ? (((long long)rp << 32) | grow) : 0;
                float k1;
                long long k2;
                emit(ok, grow, rp, k1, k2, min(64, nsv - s0));
                f(ok && key_admissible(k1), k1, k2, rank);
            }
            return;
        }
        // kept entries under U of the streams that did not fail
        for (int c0 = 0; c0 < E; c0 += 64) {
            const int c = c0 + lane;
            const int r = c < E ? c / KE : 0;
            const int sl = (c - r * KE) / KT;
            const float mr = __shfl(my_m, r);
            const uint32_t orr = __shfl(my_off, r);
            const uint32_t fl = __shfl(my_fail, r);
            bool ok = false;
            uint32_t grow = 0;
            if (c < E && !((fl >> sl) & 1u)) {
                const uint32_t key = keys[c];
                ok = key != 0xffffffffu && ivf_decode_lo<L2>(key, lowmask, fold) - mr <= U;
                grow = orr + ivf_key_row(key, lowmask, sl);
            }
            if (__ballot(ok) == 0ull) continue;
            const long long rank = ((long long)r << 32) | grow;
            float k1;
            long long k2;
            emit(ok, grow, r, k1, k2);
            f(ok && key_admissible(k1), k1, k2, rank);
        }
        // every row of the failing streams
        unsigned long long m = __ballot(my_fail != 0u);
        while (m) {
            const int r = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const uint32_t o = __shfl(my_off, r), len = __shfl(my_len, r);
            const uint32_t fl = __shfl(my_fail, r);
            const int ne = (int)cdiv_dev(len, BV) * 16;
            for (int sl = 0; sl < 4; sl++) {
                if (!((fl >> sl) & 1u)) continue;
                for (int e0 = 0; e0 < ne; e0 += 64) {
                    const int row = ivf_stream_row(e0 + lane, sl);
                    const bool ok = e0 + lane < ne && row < (int)len && (!sel || sel[o + row]);
                    const uint32_t grow = o + (uint32_t)(ok ? row : 0);
                    const long long rank = ((long long)r << 32) | grow;
                    float k1;
                    long long k2;
                    emit(ok, grow, r, k1, k2);
                    f(ok && key_admissible(k1), k1, k2, rank);
                }
            }
        }
    }
};

#ifndef RR_WAVES
#define RR_WAVES 4  // waves per SIMD the re-rank is compiled for (tuning)
#endif
template <bool L2, int V, int PQD = 0>
__global__ __launch_bounds__(64 * RR_W, RR_WAVES) void k_ivf_rerank(
        const uint32_t* __restrict__ keys, const ProbeRec* __restrict__ recs,
        const float* __restrict__ x, int ldx, const float* __restrict__ codes, int ldc,
        const int64_t* __restrict__ ids, int d, int64_t n, int nprobe, int KT, int obits, int k,
        float* __restrict__ D, int64_t* __restrict__ I, uint32_t* __restrict__ stats,
        unsigned long long* __restrict__ trace, PQArgs pa, const uint8_t* __restrict__ sel,
        unsigned long long* __restrict__ qdone, int fold_keys) {
    const unsigned long long t_start = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const bool fold = fold_keys != 0;
    __shared__ uint32_t surv[RR_W][RR_CAP];
    __shared__ uint16_t sprobe[RR_W][RR_CAP];
    __shared__ __attribute__((aligned(16))) float xsh[RR_W][BDM];
    // scratch of the small-batch compaction (64 NB keys + labels, NB <= 4)
    __shared__ __attribute__((aligned(16))) float stg[RR_W][64 * 4 * 3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q0 = (int64_t)blockIdx.x * RR_W + w;
    const bool valid = q0 < n;
    const int64_t q = valid ? q0 : 0;
    const int KE = 4 * KT;
    const int E = valid ? nprobe * KE : 0;
    const uint32_t lowmask = (1u << obits) - 1u;
    // ---- round trip 1: keys, probe records, query.  Lane l holds the V
    // consecutive entries l V .. l V + V - 1, all of probe lp = l V / KE
    // (V <= KE, both powers of two).
    const uint32_t* kq = keys + q * (int64_t)nprobe * KE;
    uint32_t kv[V];
    const bool has = lane * V < E;
    if constexpr (V >= 4) {
#pragma unroll
        for (int i = 0; i < V; i += 4) {
            const uint4 v4 = has ? *(const uint4*)(kq + lane * V + i)
                                 : make_uint4(~0u, ~0u, ~0u, ~0u);
            kv[i] = v4.x;
            kv[i + 1] = v4.y;
            kv[i + 2] = v4.z;
            kv[i + 3] = v4.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < V; i++) kv[i] = has ? kq[lane * V + i] : 0xffffffffu;
    }
    ProbeRec pr;
#pragma unroll
    for (int sl = 0; sl < 4; sl++) pr.pb[sl] = WS_INF;
    pr.mmax = 0.f;
    pr.off = 0u;
    pr.len = 0u;
    pr.pad = 0u;
    float my_d0 = 0.f;
    if (valid && lane < nprobe) {
        pr = recs[q * nprobe + lane];
        if constexpr (PQD > 0) my_d0 = pa.table1 ? pa.cdis[q * nprobe + lane] : 0.f;
    }
    const float* xq = x + q * ldx;
    if (lane < BDM / 4 && 4 * lane < (d & ~3))
        *(float4*)(&xsh[w][4 * lane]) = *(const float4*)(xq + 4 * lane);
    const int lp = has ? lane * V / KE : 0;  // this lane's probe
    const float lm = __shfl(pr.mmax, lp);
    const uint32_t loff = __shfl(pr.off, lp);
    // ---- U = k-th smallest ub' over the kept entries, in two stages: T =
    // the k-th smallest lane minimum (>= U: the k lanes below it hold k
    // values <= T), then the exact k-th among the values <= T when they fit
    // one per lane
    float ub[V];
    float lmin = WS_INF;
#pragma unroll
    for (int i = 0; i < V; i++) {
        ub[i] = kv[i] != 0xffffffffu ? ivf_decode_hi<L2>(kv[i], lowmask, fold) + lm : WS_INF;
        lmin = fminf(lmin, ub[i]);
    }
    float U;
    {
        const float lmv[1] = {lmin};
        const float T = wave_kth_smallest<1, 12>(lmv, k);  // (upper bounds: wave_select.h)
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < V; i++) cnt += __popcll(__ballot(ub[i] <= T));
        if (T < WS_INF && cnt <= 64) {
            // compact the values <= T to lanes 0..cnt-1 through LDS
            float* cb = reinterpret_cast<float*>(surv[w]);
            int pos = 0;
#pragma unroll
            for (int i = 0; i < V; i++) {
                const bool in = ub[i] <= T;
                const unsigned long long m = __ballot(in);
                if (in) cb[pos + __popcll(m & ((1ull << lane) - 1ull))] = ub[i];
                pos += __popcll(m);
            }
            __syncthreads();
            const float cv[1] = {lane < cnt ? cb[lane] : WS_INF};
            __syncthreads();
            U = wave_kth_smallest<1, 12>(cv, k);
        } else {
            U = wave_kth_smallest<V, 12>(ub, k);
        }
    }
    if (!(U <= WS_INF)) U = WS_INF;  // NaN guard
    const unsigned long long t_u = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // failing streams: one that dropped a candidate that may be <= U
    uint32_t my_fail = 0u;
#pragma unroll
    for (int sl = 0; sl < 4; sl++)
        my_fail |= (pr.pb[sl] < WS_INF && pr.pb[sl] <= U) ? (1u << sl) : 0u;
    const unsigned long long fmask = __ballot(my_fail != 0u);
    const uint32_t lfail = __shfl(my_fail, lp);
    // ---- candidates -> LDS as arena rows: kept entries with lb' <= U of the
    // streams that did not fail, then every row of the failing streams
    int ns = 0;
#pragma unroll
    for (int i = 0; i < V; i++) {
        const int sl = ((lane * V + i) % KE) / KT;
        bool sv = false;
        uint32_t grow = 0;
        if (kv[i] != 0xffffffffu && !((lfail >> sl) & 1u)) {
            sv = ivf_decode_lo<L2>(kv[i], lowmask, fold) - lm <= U;
            grow = loff + ivf_key_row(kv[i], lowmask, sl);
        }
        const unsigned long long m = __ballot(sv);
        const int pos = ns + __popcll(m & ((1ull << lane) - 1ull));
        if (sv && pos < RR_CAP) {
            surv[w][pos] = grow;
            sprobe[w][pos] = (uint16_t)lp;
        }
        ns += __popcll(m);
    }
    const int nkept = ns;
    {
        unsigned long long m = fmask;
        while (m) {
            const int r = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const uint32_t o = __shfl(pr.off, r), len = __shfl(pr.len, r);
            const uint32_t fl = __shfl(my_fail, r);
            const int ne = (int)cdiv_dev(len, BV) * 16;
            for (int sl = 0; sl < 4; sl++) {
                if (!((fl >> sl) & 1u)) continue;
                for (int e0 = 0; e0 < ne; e0 += 64) {
                    const int row = ivf_stream_row(e0 + lane, sl);
                    const bool in = e0 + lane < ne && row < (int)len && (!sel || sel[o + row]);
                    const unsigned long long bm = __ballot(in);
                    const int pos = ns + __popcll(bm & ((1ull << lane) - 1ull));
                    if (in && pos < RR_CAP) {
                        surv[w][pos] = o + (uint32_t)row;
                        sprobe[w][pos] = (uint16_t)r;
                    }
                    ns += __popcll(bm);
                }
            }
        }
    }
    __syncthreads();  // the LDS query copy and candidate list (every wave gets here)
    const unsigned long long t_c = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    RerankStream<L2, PQD> st;
    st.surv = surv[w];
    st.sprobe = sprobe[w];
    st.ids = ids;
    st.xq = xq;
    st.codes = codes;
    st.xs = xsh[w];
    st.ldc = ldc;
    st.d = d;
    st.lane = lane;
    st.nsv = ns;
    st.KE = KE;
    st.KT = KT;
    st.E = E;
    st.lowmask = lowmask;
    st.overflow = ns > RR_CAP;
    st.keys = kq;
    st.U = U;
    st.my_fail = my_fail;
    st.my_m = pr.mmax;
    st.my_off = pr.off;
    st.my_len = pr.len;
    st.my_l = pr.pad;
    st.my_d0 = my_d0;
    st.pa = pa;
    st.sel = sel;
    st.fold = fold;
    // ---- round trip 2: candidate rows and ids; up to 4 batches are ranked
    // directly, anything else goes through the general resolve
    bool done = false;
    unsigned long long t_e = 0ull;
    auto small = [&](auto nbc) {
        constexpr int NB = decltype(nbc)::value;
        float k1[NB];
        long long k2[NB];
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const bool ok = 64 * b + lane < ns;
            st.emit(ok, ok ? surv[w][64 * b + lane] : 0u, ok ? (int)sprobe[w][64 * b + lane] : 0,
                    k1[b], k2[b], max(0, min(64, ns - 64 * b)));
            if (!(ok && key_admissible(k1[b]))) {
                k1[b] = WS_INF;
                k2[b] = WS_NOID;
            }
        }
        t_e = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
        if constexpr (NB > 1) {
            // only keys <= U can be in the top k (at least k kept entries have
            // exact keys <= their ub' <= U; boundary ties are <= U too): the
            // order-preserving compaction of those (failing streams add whole
            // slots of rows, most of them far above U) ranks in one batch
            float* ck1 = stg[w];
            long long* ck2 = reinterpret_cast<long long*>(stg[w] + 64 * NB);
            int m = 0;
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const bool in = 64 * b + lane < ns && k1[b] < WS_INF && k1[b] <= U;
                const unsigned long long bm = __ballot(in);
                const int pos = m + __popcll(bm & ((1ull << lane) - 1ull));
                if (in) {
                    ck1[pos] = k1[b];
                    ck2[pos] = k2[b];
                }
                m += __popcll(bm);
            }
            if (m <= 64) {
                __syncthreads();  // one wave per block
                float c1[1] = {lane < m ? ck1[lane] : WS_INF};
                long long c2[1] = {lane < m ? ck2[lane] : WS_NOID};
                __syncthreads();
                return exact_topk_small<1>(c1, c2, m, k, L2 ? 1 : 0, lane, valid, D + q * k,
                                           I + q * k);
            }
        }
        return exact_topk_small<NB>(k1, k2, ns, k, L2 ? 1 : 0, lane, valid, D + q * k,
                                    I + q * k);
    };
    if (ns <= 64) done = small(std::integral_constant<int, 1>());
    else if (ns <= 128) done = small(std::integral_constant<int, 2>());
    else if (ns <= 256) done = small(std::integral_constant<int, 4>());
    if (!done) exact_topk_resolve(st, k, L2 ? 1 : 0, lane, valid, D + q * k, I + q * k);
    if (stats && valid && lane == 0) {
        atomicAdd(&stats[0], (uint32_t)min(nkept, RR_CAP));
        atomicAdd(&stats[1], (uint32_t)__popcll(fmask));
        atomicAdd(&stats[2], st.overflow ? 1u : 0u);
        atomicAdd(&stats[3], done ? 0u : 1u);
    }
    // search_stats: the query's completion on the device clock
    if (qdone && valid && lane == 0) qdone[q] = __builtin_amdgcn_s_memrealtime();
    if (trace && valid && lane == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        trace[8 * q + 0] = t_start;
        trace[8 * q + 1] = t_end;
        trace[8 * q + 2] = (unsigned long long)ns | ((unsigned long long)__popcll(fmask) << 32);
        trace[8 * q + 3] = t_u;
        trace[8 * q + 4] = t_c;
        trace[8 * q + 5] = t_e;
    }
}

// ---------------------------------------------------------------- B, wide
// The re-rank for nprobe > 64 (the reference harness's grid reaches nprobe
// 2048: tutorial/cpp/benchmark-hnsw-ivf/benchmark.config nprobe_ratio up to
// 0.128 of nlist).  One wave per query walks its probes in chunks of 64, lane
// r holding probe 64 c + r with its KE keys, and certifies exactly as
// k_ivf_rerank does:
//   T = the k-th smallest probe minimum of ub' (a running k-smallest set
//       merged chunk by chunk) — k probes hold a value <= T, so T >= U;
//   U = the k-th smallest ub' among the values <= T (at most (k + ties) KE of
//       them: only probes whose minimum is <= T hold any), or T when they do
//       not fit the LDS;
//   candidates = kept entries with lb' <= U of the streams whose dropped bound
//       is > U, and every row of the streams whose dropped bound is <= U.
// The exact top-k over the candidates (arrival order = probe rank, then
// arena row) is the reference result.  Each stage re-reads the query's keys
// and records (L2-resident: 16 + 32 B per probe at KE = 4).
constexpr int RRW_CB = 1024;  // values <= T ranked exactly (LDS)

template <bool L2, int KE, int PQD>
struct WideStream {
    const uint32_t* surv;    // candidates' arena rows (LDS)
    const uint16_t* sprobe;  // their probe rank
    int nsv;
    bool overflow;           // the candidate list did not fit: re-walk the probes
    const uint32_t* kq;      // this query's keys [nprobe][KE]
    const ProbeRec* rq;      // its probe records [nprobe]
    const float* cdq;        // PQ table 1: its coarse distances [nprobe]
    const int64_t* ids;
    const float* xq;
    const float* codes;
    const float* xs;
    int ldc, d, lane, nprobe;
    uint32_t lowmask;
    float U;
    PQArgs pa;
    const uint8_t* sel;
    bool fold;
    static constexpr int KT = KE / 4;

    __device__ __forceinline__ void emit(bool ok, uint32_t grow, int r, float& k1, long long& k2,
                                         int nv = -1) const {
        const long long idv = ok ? (long long)ids[grow] : 0ll;
        float dis;
        if constexpr (PQD > 0) {
            const uint32_t l = ok ? rq[r].pad : 0u;
            const float d0 = ok && pa.table1 ? cdq[r] : 0.f;
            dis = ok ? pq_exact<PQD>(pa, xs, grow, l, d0) : 0.f;
        } else {
            if (nv >= 0)
                dis = ref_rows64_4lane_pb<L2, RR_XM, RR_PB>(xs, xq, codes, ldc, d, grow, nv, lane);
            else
                dis = eval_rows64_direct<L2>(xs, xq, codes, ldc, d, grow, ok, lane);
        }
        k1 = WS_INF;
        k2 = WS_NOID;
        if (ok) to_key(L2 ? 1 : 0, dis, idv, k1, k2);
    }
    __device__ __forceinline__ void load_keys(int p, bool has, uint32_t (&kv)[KE]) const {
#pragma unroll
        for (int i = 0; i < KE; i += 4) {
            const uint4 v4 = has ? *(const uint4*)(kq + (int64_t)p * KE + i)
                                 : make_uint4(~0u, ~0u, ~0u, ~0u);
            kv[i] = v4.x;
            kv[i + 1] = v4.y;
            kv[i + 2] = v4.z;
            kv[i + 3] = v4.w;
        }
    }
    __device__ __forceinline__ uint32_t fail_bits(const ProbeRec& pr) const {
        uint32_t f = 0u;
#pragma unroll
        for (int sl = 0; sl < 4; sl++) f |= (pr.pb[sl] < WS_INF && pr.pb[sl] <= U) ? (1u << sl) : 0u;
        return f;
    }
    template <class F>
    __device__ __forceinline__ void for_each(F f) const {
        if (!overflow) {
            for (int s0 = 0; s0 < nsv; s0 += 64) {
                const bool ok = s0 + lane < nsv;
                const uint32_t grow = ok ? surv[s0 + lane] : 0u;
                const int rp = ok ? (int)sprobe[s0 + lane] : 0;
                const long long rank = ok ? (((long long)rp << 32) | grow) : 0;
                float k1;
                long long k2;
                emit(ok, grow, rp, k1, k2, min(64, nsv - s0));
                f(ok && key_admissible(k1), k1, k2, rank);
            }
            return;
        }
        for (int c0 = 0; c0 < nprobe; c0 += 64) {
            const int p = c0 + lane;
            const bool has = p < nprobe;
            ProbeRec pr;
            if (has) pr = rq[p];
            uint32_t kv[KE];
            load_keys(p, has, kv);
            const uint32_t fl = has ? fail_bits(pr) : 0u;
#pragma unroll
            for (int i = 0; i < KE; i++) {
                const int sl = i / KT;
                bool ok = false;
                uint32_t grow = 0u;
                if (has && kv[i] != 0xffffffffu && !((fl >> sl) & 1u)) {
                    ok = ivf_decode_lo<L2>(kv[i], lowmask, fold) - pr.mmax <= U;
                    grow = pr.off + ivf_key_row(kv[i], lowmask, sl);
                }
                if (__ballot(ok) == 0ull) continue;
                float k1;
                long long k2;
                emit(ok, grow, p, k1, k2);
                f(ok && key_admissible(k1), k1, k2, ((long long)p << 32) | grow);
            }
            unsigned long long m = __ballot(fl != 0u);
            while (m) {
                const int r = __ffsll((long long)m) - 1;
                m &= m - 1ull;
                const uint32_t o = __shfl(has ? pr.off : 0u, r), len = __shfl(has ? pr.len : 0u, r);
                const uint32_t flr = __shfl(fl, r);
                const int ne = (int)cdiv_dev(len, BV) * 16;
                for (int sl = 0; sl < 4; sl++) {
                    if (!((flr >> sl) & 1u)) continue;
                    for (int e0 = 0; e0 < ne; e0 += 64) {
                        const int row = ivf_stream_row(e0 + lane, sl);
                        const bool ok = e0 + lane < ne && row < (int)len && (!sel || sel[o + row]);
                        const uint32_t grow = o + (uint32_t)(ok ? row : 0);
                        float k1;
                        long long k2;
                        emit(ok, grow, c0 + r, k1, k2);
                        f(ok && key_admissible(k1), k1, k2, ((long long)(c0 + r) << 32) | grow);
                    }
                }
            }
        }
    }
};

template <bool L2, int KE, int PQD = 0>
__global__ __launch_bounds__(64, RR_WAVES) void k_ivf_rerank_wide(
        const uint32_t* __restrict__ keys, const ProbeRec* __restrict__ recs,
        const float* __restrict__ x, int ldx, const float* __restrict__ codes, int ldc,
        const int64_t* __restrict__ ids, int d, int64_t n, int nprobe, int obits, int k,
        float* __restrict__ D, int64_t* __restrict__ I, uint32_t* __restrict__ stats, PQArgs pa,
        const uint8_t* __restrict__ sel, unsigned long long* __restrict__ qdone, int fold_keys) {
    constexpr int KT = KE / 4;
    const bool fold = fold_keys != 0;
    __shared__ uint32_t surv[RR_CAP];
    __shared__ uint16_t sprobe[RR_CAP];
    __shared__ __attribute__((aligned(16))) float xsh[BDM];
    __shared__ __attribute__((aligned(16))) float stg[64 * 4 * 3];
    __shared__ float cb[RRW_CB];
    const int lane = threadIdx.x;
    const int64_t q = blockIdx.x;
    if (q >= n) return;  // (one wave per block: the whole block leaves)
    const uint32_t lowmask = (1u << obits) - 1u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    WideStream<L2, KE, PQD> st;
    st.kq = keys + q * (int64_t)nprobe * KE;
    st.rq = recs + q * (int64_t)nprobe;
    st.cdq = pa.cdis ? pa.cdis + q * (int64_t)nprobe : nullptr;
    st.ids = ids;
    st.xq = x + q * ldx;
    st.codes = codes;
    st.xs = xsh;
    st.ldc = ldc;
    st.d = d;
    st.lane = lane;
    st.nprobe = nprobe;
    st.lowmask = lowmask;
    st.pa = pa;
    st.sel = sel;
    st.fold = fold;
    st.U = WS_INF;
    if (lane < BDM / 4 && 4 * lane < (d & ~3))
        *(float4*)(&xsh[4 * lane]) = *(const float4*)(st.xq + 4 * lane);
    // ---- T: running set of the k smallest probe minima (lanes < k)
    float rv = WS_INF, T = WS_INF;
    for (int c0 = 0; c0 < nprobe; c0 += 64) {
        const int p = c0 + lane;
        const bool has = p < nprobe;
        const float mm = has ? st.rq[p].mmax : 0.f;
        uint32_t kv[KE];
        st.load_keys(p, has, kv);
        float pm = WS_INF;
#pragma unroll
        for (int i = 0; i < KE; i++)
            if (kv[i] != 0xffffffffu) pm = fminf(pm, ivf_decode_hi<L2>(kv[i], lowmask, fold) + mm);
        const float mv[2] = {rv, pm};
        const float t = wave_kth_smallest<2>(mv, k);
        // the new set: the values < t (fewer than k), then t up to k
        const bool a = rv < t, b = pm < t;
        const unsigned long long ma = __ballot(a), mb = __ballot(b);
        if (a) cb[__popcll(ma & lt)] = rv;
        if (b) cb[__popcll(ma) + __popcll(mb & lt)] = pm;
        __syncthreads();
        const int cnt = __popcll(ma) + __popcll(mb);
        rv = lane < cnt ? cb[lane] : (lane < k ? t : WS_INF);
        __syncthreads();
        T = t;
    }
    if (!(T <= WS_INF)) T = WS_INF;  // NaN guard
    // ---- U: the k-th smallest ub' among the values <= T
    float U = T;
    if (T < WS_INF) {
        int cnt = 0;
        for (int c0 = 0; c0 < nprobe; c0 += 64) {
            const int p = c0 + lane;
            const bool has = p < nprobe;
            const float mm = has ? st.rq[p].mmax : 0.f;
            uint32_t kv[KE];
            st.load_keys(p, has, kv);
#pragma unroll
            for (int i = 0; i < KE; i++) {
                const float ub = kv[i] != 0xffffffffu ? ivf_decode_hi<L2>(kv[i], lowmask, fold) + mm
                                                      : WS_INF;
                const bool in = ub <= T;
                const unsigned long long m = __ballot(in);
                const int pos = cnt + __popcll(m & lt);
                if (in && pos < RRW_CB) cb[pos] = ub;
                cnt += __popcll(m);
            }
        }
        __syncthreads();
        if (cnt <= RRW_CB) {
            float v[RRW_CB / 64];
#pragma unroll
            for (int i = 0; i < RRW_CB / 64; i++)
                v[i] = 64 * i + lane < cnt ? cb[64 * i + lane] : WS_INF;
            U = wave_kth_smallest<RRW_CB / 64, 12>(v, k);
        }
        __syncthreads();
    }
    st.U = U;
    // ---- candidates -> LDS: kept entries under U of the streams that did not
    // fail, then every row of the failing streams
    int ns = 0, nfail = 0, nkept = 0;
    for (int c0 = 0; c0 < nprobe; c0 += 64) {
        const int p = c0 + lane;
        const bool has = p < nprobe;
        ProbeRec pr;
        if (has) pr = st.rq[p];
        uint32_t kv[KE];
        st.load_keys(p, has, kv);
        const uint32_t fl = has ? st.fail_bits(pr) : 0u;
#pragma unroll
        for (int i = 0; i < KE; i++) {
            const int sl = i / KT;
            bool sv = false;
            uint32_t grow = 0u;
            if (has && kv[i] != 0xffffffffu && !((fl >> sl) & 1u)) {
                sv = ivf_decode_lo<L2>(kv[i], lowmask, fold) - pr.mmax <= U;
                grow = pr.off + ivf_key_row(kv[i], lowmask, sl);
            }
            const unsigned long long m = __ballot(sv);
            const int pos = ns + __popcll(m & lt);
            if (sv && pos < RR_CAP) {
                surv[pos] = grow;
                sprobe[pos] = (uint16_t)p;
            }
            ns += __popcll(m);
        }
        nkept = ns;
        unsigned long long m = __ballot(fl != 0u);
        nfail += __popcll(m);
        while (m) {
            const int r = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const uint32_t o = __shfl(has ? pr.off : 0u, r), len = __shfl(has ? pr.len : 0u, r);
            const uint32_t flr = __shfl(fl, r);
            const int ne = (int)cdiv_dev(len, BV) * 16;
            for (int sl = 0; sl < 4; sl++) {
                if (!((flr >> sl) & 1u)) continue;
                for (int e0 = 0; e0 < ne; e0 += 64) {
                    const int row = ivf_stream_row(e0 + lane, sl);
                    const bool in = e0 + lane < ne && row < (int)len && (!sel || sel[o + row]);
                    const unsigned long long bm = __ballot(in);
                    const int pos = ns + __popcll(bm & lt);
                    if (in && pos < RR_CAP) {
                        surv[pos] = o + (uint32_t)row;
                        sprobe[pos] = (uint16_t)(c0 + r);
                    }
                    ns += __popcll(bm);
                }
            }
        }
    }
    __syncthreads();  // the LDS query copy and candidate list
    st.surv = surv;
    st.sprobe = sprobe;
    st.nsv = ns;
    st.overflow = ns > RR_CAP;
    // ---- exact top-k: up to 4 batches ranked directly, else the general resolve
    bool done = false;
    auto small = [&](auto nbc) {
        constexpr int NB = decltype(nbc)::value;
        float k1[NB];
        long long k2[NB];
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const bool ok = 64 * b + lane < ns;
            st.emit(ok, ok ? surv[64 * b + lane] : 0u, ok ? (int)sprobe[64 * b + lane] : 0, k1[b],
                    k2[b], max(0, min(64, ns - 64 * b)));
            if (!(ok && key_admissible(k1[b]))) {
                k1[b] = WS_INF;
                k2[b] = WS_NOID;
            }
        }
        if constexpr (NB > 1) {
            float* ck1 = stg;
            long long* ck2 = reinterpret_cast<long long*>(stg + 64 * NB);
            int m = 0;
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const bool in = 64 * b + lane < ns && k1[b] < WS_INF && k1[b] <= U;
                const unsigned long long bm = __ballot(in);
                const int pos = m + __popcll(bm & lt);
                if (in) {
                    ck1[pos] = k1[b];
                    ck2[pos] = k2[b];
                }
                m += __popcll(bm);
            }
            if (m <= 64) {
                __syncthreads();
                float c1[1] = {lane < m ? ck1[lane] : WS_INF};
                long long c2[1] = {lane < m ? ck2[lane] : WS_NOID};
                __syncthreads();
                return exact_topk_small<1>(c1, c2, m, k, L2 ? 1 : 0, lane, true, D + q * k,
                                           I + q * k);
            }
        }
        return exact_topk_small<NB>(k1, k2, ns, k, L2 ? 1 : 0, lane, true, D + q * k, I + q * k);
    };
    if (ns <= 64) done = small(std::integral_constant<int, 1>());
    else if (ns <= 128) done = small(std::integral_constant<int, 2>());
    else if (ns <= 256) done = small(std::integral_constant<int, 4>());
    if (!done) exact_topk_resolve(st, k, L2 ? 1 : 0, lane, true, D + q * k, I + q * k);
    if (stats && lane == 0) {
        atomicAdd(&stats[0], (uint32_t)min(nkept, RR_CAP));
        atomicAdd(&stats[1], (uint32_t)nfail);
        atomicAdd(&stats[2], st.overflow ? 1u : 0u);
        atomicAdd(&stats[3], done ? 0u : 1u);
    }
    if (qdone && lane == 0) qdone[q] = __builtin_amdgcn_s_memrealtime();
}

// IVF-PQ re-rank launch for one sub-quantizer width (explicitly instantiated
// per DS in kernels_ivfpq_rerank_d<DS>.hip: the 24 PQ kernel instantiations
// compile as three translation units in parallel)

template <int DS>
void ivfpq_rerank_ds(const uint32_t* keys, const ProbeRec* recs, const float* x, int ldx, int d,
                     const int64_t* ids, const PQArgs& pa, int64_t n, int nprobe, int KT,
                     int obits, int k, const uint8_t* sel, float* D, int64_t* I,
                     uint32_t* stats, hipStream_t s, unsigned long long* qdone, int fold) {
    const int KE = 4 * KT;
    const int E = nprobe * KE;
    const int V = E <= 128 ? 2 : E <= 256 ? 4 : E <= 512 ? 8 : E <= 1024 ? 16 : 32;
#define LAUNCH_P(VV)                                                                            \
    k_ivf_rerank<true, VV, DS><<<kgrid(cdiv(n, RR_W), 64 * RR_W), dim3(64 * RR_W), 0, s>>>(       \
            keys, recs, x, ldx, nullptr, 0, ids, d, n, nprobe, KT, obits, k, D, I, stats,         \
            nullptr, pa, sel, qdone, fold)
#define LAUNCH_PW(KEV)                                                                         \
    k_ivf_rerank_wide<true, KEV, DS><<<kgrid(n, 64), dim3(64), 0, s>>>(                     \
            keys, recs, x, ldx, nullptr, 0, ids, d, n, nprobe, obits, k, D, I, stats, pa, sel,  \
            qdone, fold)
    if (nprobe > 64) {  // probes walked in chunks of 64 (k_ivf_rerank_wide)
        if (KE == 8) LAUNCH_PW(8);
        else if (KE == 16) LAUNCH_PW(16);
        else LAUNCH_PW(32);
    } else if (V == 2) LAUNCH_P(2);
    else if (V == 4) LAUNCH_P(4);
    else if (V == 8) LAUNCH_P(8);
    else if (V == 16) LAUNCH_P(16);
    else LAUNCH_P(32);
    HIP_LAUNCH_CHECK();
#undef LAUNCH_PW
#undef LAUNCH_P
}

}  // namespace kern
}  // namespace faiss_amd
