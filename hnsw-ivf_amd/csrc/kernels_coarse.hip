// kernels_coarse.hip — coarse quantizer top-nprobe on bf16x3 MFMA with a
// certified exact re-rank.
//
// Reference: IndexFlat::search for query blocks >= 20
// (faiss/utils/distances.cpp:259-342 exhaustive_L2sqr_blas, :807-823):
//   dis(i, j) = max(0, ||x_i||^2 + ||c_j||^2 - 2 <x_i, c_j>)     (L2)
//   dis(i, j) = <x_i, c_j>                                         (IP)
// with the norms from fvec_norms_L2sqr (reference order, ref_arith.h) and the
// inner product from sgemm.  The sgemm order is not reproducible; this path
// fixes it to the sequential fma chain (what the fp32-MFMA tile of
// pairwise_distances and the oracle compute), and the top-k follows the
// HeapBlockResultHandler (centroids arrive in id order, strict admission).
//
// A  k_coarse_bf3_filter: work item = 64 queries x one split of the
//    centroids; approx distances from bf16x3 MFMA; every thread keeps the KT
//    best 32-bit keys of its 16-per-tile share (bf3.h, same layout as the
//    IVF-Flat filter).  Output per (query, split, thread): lb keys, ub, and
//    per (query, split) a lower bound of every dropped centroid.
// B  k_coarse_rerank: one wave per query.  U = k-th smallest ub; every kept
//    entry with lb <= U and every centroid of a split whose dropped bound is
//    <= U is evaluated exactly; exact top-k with the reference tie rule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstdlib>

#include "bf3.h"
#include "common.h"
#include "exact_select.h"
#include "kernels.h"
#include "ref_arith.h"
#include "wave_select.h"

namespace faiss_amd {
namespace kern {

// sequential fma chain (the fixed order of the BLAS-form inner product);
// operands are fetched 32 floats at a time so a lane has 16 loads in flight
__device__ __forceinline__ float ip_seq(const float* __restrict__ a, const float* __restrict__ b,
                                        int d) {
    float acc = 0.f;
    int j = 0;
    for (; j + 32 <= d; j += 32) {
        float4 av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            av[u] = *(const float4*)(a + j + 4 * u);
            bv[u] = *(const float4*)(b + j + 4 * u);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            acc = fmaf(av[u].x, bv[u].x, acc);
            acc = fmaf(av[u].y, bv[u].y, acc);
            acc = fmaf(av[u].z, bv[u].z, acc);
            acc = fmaf(av[u].w, bv[u].w, acc);
        }
    }
    for (; j + 4 <= d; j += 4) {
        const float4 av = *(const float4*)(a + j), bv = *(const float4*)(b + j);
        acc = fmaf(av.x, bv.x, acc);
        acc = fmaf(av.y, bv.y, acc);
        acc = fmaf(av.z, bv.z, acc);
        acc = fmaf(av.w, bv.w, acc);
    }
    for (; j < d; j++) acc = fmaf(a[j], b[j], acc);
    return acc;
}

template <bool L2, int KT, int NS>
__global__ __launch_bounds__(256, 2) void k_coarse_bf3_filter(
        const float* __restrict__ x, int ldx, int64_t n, int d, const __bf16* __restrict__ cbf,
        const float* __restrict__ cnorm, const float* __restrict__ xnorm, int nlist,
        int nsplit, int split_len, float coef, const float* __restrict__ cnmax_p, int obits,
        unsigned long long* __restrict__ part, float* __restrict__ pub,
        float* __restrict__ pbound) {
    __shared__ __attribute__((aligned(16))) uint8_t tiles[2 * BV * (4 * 16 * NS + 16)];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // blocks b and b+8 share an XCD: consecutive splits of one query block
    // stay together
    const int64_t qb = blockIdx.x / nsplit;
    const int sp = (int)(blockIdx.x % nsplit);
    const int c0 = sp * split_len;
    const int len = min(split_len, nlist - c0);
    constexpr int DB = 16 * NS, CSB = 4 * DB + 16, RU = DB / 4;
    const int bi = w >> 1, bj = w & 1, li = lane & 31, lh = lane >> 5;
    const int slot = 2 * bi + lh, qloc = 32 * bj + li;
    const int64_t q = qb * BQ + qloc;
    bf16x8 bh[NS], bl[NS];
    float xn_approx;
    load_query_frags<NS>(x, ldx, d, q < n ? (int)q : -1, lh, bh, bl, xn_approx);
    const float xn = q < n ? xnorm[q] : 0.f;  // the reference-order norm (exact side)
    const float cnmax = *cnmax_p;

    uint4 pf[8];
    auto fetch = [&](int v0n) {
        const int nvn = min(BV, len - v0n);
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const int e = t + 256 * s;
            const int r = e / RU, c = e - r * RU;
            pf[s] = make_uint4(0u, 0u, 0u, 0u);
            if (e < BV * RU && r < nvn)
                pf[s] = *(const uint4*)(cbf + (int64_t)(c0 + v0n + r) * (2 * DB) + 8 * c);
        }
    };
    auto stash = [&](int buf) {
        uint8_t* T = tiles + buf * BV * CSB;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const int e = t + 256 * s;
            const int r = e / RU, c = e - r * RU;
            if (e < BV * RU) *(uint4*)(T + r * CSB + 16 * c) = pf[s];
        }
    };
    fetch(0);
    stash(0);
    if (BV < len) fetch(BV);
    __syncthreads();

    ThreadQueue32<KT> tq;
    tq.init();
    const uint32_t lowmask = (1u << obits) - 1u;
    const float* cn = cnorm + c0;
    for (int v0 = 0, tile = 0; v0 < len; v0 += BV, tile++) {
        const int buf = tile & 1;
        if (v0 + BV < len) {
            stash(buf ^ 1);
            if (v0 + 2 * BV < len) fetch(v0 + 2 * BV);
        }
        float yv[16];
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int cr = v0 + 32 * bi + 4 * lh + 8 * g + c;
                yv[4 * g + c] = cr < len ? cn[cr] : 0.f;
            }
        const floatx16 acc =
                bf3_block<NS>(tiles + buf * BV * CSB + (32 * bi + li) * CSB + 16 * lh, bh, bl);
        const uint32_t ordbase = (uint32_t)tile << 4;
        const bool full = v0 + BV <= len;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            // L2: clamped at 0 inside key_encode, as the reference clamps
            const float a = L2 ? fmaf(-2.f, acc[r], xn + yv[r]) : -acc[r];
            uint32_t key = key_encode<L2>(a, lowmask, ordbase | (uint32_t)r);
            if (!full) {
                const int cr = v0 + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
                key = cr < len ? key : 0xffffffffu;
            }
            tq.push(key);
        }
        __syncthreads();
    }
    const float bnd = tq.q[KT - 1] != 0xffffffffu ? key_decode_lo<L2>(tq.q[KT - 1], lowmask)
                                                 : WS_INF;
    if (q < n) {
        const int64_t e = q * nsplit + sp;
        unsigned long long* po = part + e * (4 * KT) + slot * KT;
        float* pu = pub + e * (4 * KT) + slot * KT;
#pragma unroll
        for (int i = 0; i < KT; i++) {
            const uint32_t key = tq.q[i];
            if (key != 0xffffffffu) {
                const uint32_t ord = key & lowmask;
                const int r = (int)(ord & 15u);
                const uint32_t row =
                        (ord >> 4) * BV + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
                const float m = coef * (xn + cn[row]) + 1e-30f;
                const float alo = key_decode_lo<L2>(key, lowmask);
                const float ahi = key_decode_hi<L2>(key, lowmask);
                po[i] = ((unsigned long long)ordered_f32(alo - m) << 32) | (uint32_t)(c0 + row);
                pu[i] = ahi + m;
            } else {
                po[i] = ~0ull;
                pu[i] = WS_INF;
            }
        }
        // per-thread stream bound: a failing stream is re-scanned alone
        pbound[e * 4 + slot] = bnd < WS_INF ? bnd - (coef * (xn + cnmax) + 1e-30f) : WS_INF;
    }
}

constexpr int CR_CAP = 512;

template <bool L2>
struct CoarseStream {
    const unsigned long long* part;  // this query's [nsplit][E1]
    const float* xq;
    const float* cent;
    const float* cnorm;
    float xn;
    int ldc, d, nlist, nsplit, split_len, E, KT, lane, nsv;
    bool overflow;
    unsigned long long fmask;  // failing streams: bit 4 * split + slot
    float U;
    const uint32_t* surv;

    __device__ __forceinline__ bool survivor(int c) const {
        if ((fmask >> (c / KT)) & 1ull) return false;  // entries of stream c / KT
        const unsigned long long key = part[c];
        return key != ~0ull && unordered_f32((uint32_t)(key >> 32)) <= U;
    }
    __device__ __forceinline__ void eval(int j, float& k1, long long& k2, long long& rank) const {
        const float ip = ip_seq(xq, cent + (int64_t)j * ldc, d);
        float dis;
        if (L2) {
            dis = fmaf(-2.f, ip, xn + cnorm[j]);
            dis = dis < 0.f ? 0.f : dis;
        } else {
            dis = ip;
        }
        to_key(L2 ? 1 : 0, dis, (long long)j, k1, k2);
        rank = j;
    }
    template <class F>
    __device__ __forceinline__ void for_each(F f) const {
        if (!overflow) {
            for (int s0 = 0; s0 < nsv; s0 += 64) {
                float k1 = WS_INF;
                long long k2 = WS_NOID, rank = 0;
                bool ok = s0 + lane < nsv;
                if (ok) {
                    eval((int)surv[s0 + lane], k1, k2, rank);
                    ok = key_admissible(k1);
                }
                f(ok, k1, k2, rank);
            }
        } else {
            for (int c0 = 0; c0 < E; c0 += 64) {
                const int c = c0 + lane;
                float k1 = WS_INF;
                long long k2 = WS_NOID, rank = 0;
                bool ok = c < E && survivor(c);
                if (__ballot(ok) == 0ull) continue;
                if (ok) {
                    eval((int)(uint32_t)part[c], k1, k2, rank);
                    ok = key_admissible(k1);
                }
                f(ok, k1, k2, rank);
            }
        }
        // failing streams: thread slot (bi, lh) of split s saw, per 64-row
        // tile, rows 32 bi + 4 lh + 8 g + c (g, c < 4)
        unsigned long long m = fmask;
        while (m) {
            const int sidx = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const int s = sidx >> 2, slot = sidx & 3, bi = slot >> 1, lh = slot & 1;
            const int j0 = s * split_len, j1 = min(nlist, j0 + split_len);
            const int ntile = (j1 - j0 + BV - 1) / BV;
            for (int t0 = 0; t0 < ntile * 16; t0 += 64) {
                const int e = t0 + lane;  // tile e >> 4, register e & 15
                const int r = e & 15;
                const int j = j0 + (e >> 4) * BV + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
                float k1 = WS_INF;
                long long k2 = WS_NOID, rank = 0;
                bool ok = e < ntile * 16 && j < j1;
                if (ok) {
                    eval(j, k1, k2, rank);
                    ok = key_admissible(k1);
                }
                f(ok, k1, k2, rank);
            }
        }
    }
};

template <bool L2, class OutIdx, int V>
__global__ __launch_bounds__(256) void k_coarse_rerank(
        const unsigned long long* __restrict__ part, const float* __restrict__ pub,
        const float* __restrict__ pbound, const float* __restrict__ x, int ldx,
        const float* __restrict__ xnorm, const float* __restrict__ cent, int ldc,
        const float* __restrict__ cnorm, int64_t n, int d, int nlist, int nsplit, int split_len,
        int E1, int k, float* __restrict__ D, OutIdx* __restrict__ I,
        uint32_t* __restrict__ stats) {
    __shared__ uint32_t surv[4][CR_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q0 = (int64_t)blockIdx.x * 4 + w;
    const bool valid = q0 < n;
    const int64_t q = valid ? q0 : 0;
    CoarseStream<L2> st;
    st.E = nsplit * E1;
    st.part = part + q * st.E;
    st.xq = x + q * ldx;
    st.cent = cent;
    st.cnorm = cnorm;
    st.xn = xnorm ? xnorm[q] : 0.f;
    st.ldc = ldc;
    st.d = d;
    st.nlist = nlist;
    st.nsplit = nsplit;
    st.split_len = split_len;
    st.KT = E1 / 4;
    st.lane = lane;
    st.fmask = 0u;
    st.U = WS_INF;
    const int total = valid ? st.E : 0;
    const float* pu = pub + q * st.E;
    float ub[V];
#pragma unroll
    for (int i = 0; i < V; i++) {
        const int c = i * 64 + lane;
        ub[i] = c < total ? pu[c] : WS_INF;
    }
    float U = wave_kth_smallest<V>(ub, k);
    if (!(U <= WS_INF)) U = WS_INF;
    st.U = U;
    {
        bool fl = false;
        if (valid && lane < 4 * nsplit) {
            const float pb = pbound[q * 4 * nsplit + lane];
            fl = pb < WS_INF && pb <= U;
        }
        st.fmask = __ballot(fl);
    }
    int ns = 0;
    for (int c0 = 0; c0 < total; c0 += 64) {
        const int c = c0 + lane;
        const bool sv = c < total && st.survivor(c);
        const unsigned long long m = __ballot(sv);
        const int pos = ns + __popcll(m & ((1ull << lane) - 1ull));
        if (sv && pos < CR_CAP) surv[w][pos] = (uint32_t)st.part[c];  // centroid id
        ns += __popcll(m);
    }
    st.overflow = ns > CR_CAP;
    st.nsv = ns;
    st.surv = surv[w];
    exact_topk_resolve(st, k, L2 ? 1 : 0, lane, valid, D + q * k, I + q * k);
    if (stats && valid && lane == 0) {
        atomicAdd(&stats[0], (uint32_t)min(ns, CR_CAP));
        atomicAdd(&stats[1], (uint32_t)__popcll(st.fmask));
        atomicAdd(&stats[2], st.overflow ? 1u : 0u);
    }
}

__global__ void k_array_max(const float* __restrict__ a, int64_t n, float* __restrict__ out) {
    __shared__ float red[16];
    float m = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, a[i]);
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = 0.f;
        for (int i = 0; i < (int)(blockDim.x >> 6); i++) r = fmaxf(r, red[i]);
        *out = r;
    }
}

// ---------------------------------------------------------------- host
CoarsePlan coarse_bf3_plan(int64_t n, int nlist, int d, int k) {
    CoarsePlan p{};
    if (n < 20 || nlist <= 0 || k < 1 || k > kMaxK || bf3_db(d) > BDM)
        return p;
    int nsplit = nlist >= 2048 ? 4 : nlist >= 1024 ? 2 : 1;
    const int per = (int)cdiv((size_t)k, (size_t)(4 * nsplit));
    if (per > 4) return p;
    int kt = 4;
    while (kt < 4 * per) kt <<= 1;
    const int split_len = (int)roundup(cdiv((size_t)nlist, (size_t)nsplit), BV);
    nsplit = (int)cdiv((size_t)nlist, (size_t)split_len);
    const int tiles = (int)cdiv((size_t)split_len, BV);
    int b = 0;
    while ((1 << b) < tiles) b++;
    if (4 + b > 14) return p;
    p.ok = true;
    p.nsplit = nsplit;
    p.split_len = split_len;
    p.kt = kt;
    p.obits = 4 + b;
    p.entries = nsplit * 4 * kt;
    return p;
}

void coarse_bf3_knn(const CoarsePlan& p, const float* x, int64_t n, int ldx, const float* xnorm,
                    const float* cent, int ldc, const void* cbf, const float* cnorm,
                    const float* cnmax, int nlist, int d, int k, int metric_l2,
                    unsigned long long* part, float* pub, float* pbound, float* D, int32_t* I32,
                    int64_t* I64, hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT(p.ok);
    static uint32_t* stats = nullptr;  // FAISS_AMD_IVF_STATS debug counters
    const bool dbg = getenv("FAISS_AMD_IVF_STATS") != nullptr;
    if (dbg && !stats) HIP_CHECK(hipMalloc(&stats, 16));
    if (dbg) HIP_CHECK(hipMemsetAsync(stats, 0, 16, s));
    FAISS_THROW_IF_NOT(ldx % 4 == 0 && ldc % 4 == 0);
    const int NS = bf3_db(d) / 16;
    const float coef = (float)ivf_bf3_coef(d);
    const int64_t nqb = (int64_t)cdiv((size_t)n, BQ);
    const int64_t grid = nqb * p.nsplit;
    FAISS_THROW_IF_NOT(grid < (1ll << 31));
#define LAUNCH_NS(L2V, KTV, NSV)                                                              \
    k_coarse_bf3_filter<L2V, KTV, NSV><<<dim3((unsigned)grid), dim3(256), 0, s>>>(            \
            x, ldx, n, d, (const __bf16*)cbf, cnorm, xnorm, nlist, p.nsplit, p.split_len,     \
            coef, cnmax, p.obits, part, pub, pbound)
#define LAUNCH_A(L2V, KTV)                     \
    do {                                       \
        if (NS == 2) LAUNCH_NS(L2V, KTV, 2);   \
        else if (NS == 4) LAUNCH_NS(L2V, KTV, 4); \
        else if (NS == 6) LAUNCH_NS(L2V, KTV, 6); \
        else LAUNCH_NS(L2V, KTV, 8);           \
    } while (0)
#define DISPATCH(L2V)                      \
    do {                                   \
        if (p.kt == 4) LAUNCH_A(L2V, 4);   \
        else if (p.kt == 8) LAUNCH_A(L2V, 8); \
        else LAUNCH_A(L2V, 16);            \
    } while (0)
    if (metric_l2) DISPATCH(true);
    else DISPATCH(false);
#undef DISPATCH
#undef LAUNCH_A
#undef LAUNCH_NS
    HIP_LAUNCH_CHECK();
    const dim3 g2((unsigned)cdiv((size_t)n, 4)), b2(256);
    const int E1 = 4 * p.kt;
    const int E = p.nsplit * E1;
    const int V = E <= 128 ? 2 : E <= 256 ? 4 : E <= 512 ? 8 : 16;
    FAISS_THROW_IF_NOT(E <= 1024);
#define LAUNCH_R(L2V, OT, OUT, VV)                                                              \
    k_coarse_rerank<L2V, OT, VV><<<g2, b2, 0, s>>>(part, pub, pbound, x, ldx, xnorm, cent, ldc, \
                                                   cnorm, n, d, nlist, p.nsplit, p.split_len,   \
                                                   E1, k, D, OUT, st_ptr)
#define LAUNCH_RV(L2V, OT, OUT)                  \
    do {                                         \
        if (V == 2) LAUNCH_R(L2V, OT, OUT, 2);   \
        else if (V == 4) LAUNCH_R(L2V, OT, OUT, 4); \
        else if (V == 8) LAUNCH_R(L2V, OT, OUT, 8); \
        else LAUNCH_R(L2V, OT, OUT, 16);         \
    } while (0)
    uint32_t* const st_ptr = dbg ? stats : nullptr;
    if (metric_l2) {
        if (I32) LAUNCH_RV(true, int32_t, I32);
        else LAUNCH_RV(true, int64_t, I64);
    } else {
        if (I32) LAUNCH_RV(false, int32_t, I32);
        else LAUNCH_RV(false, int64_t, I64);
    }
#undef LAUNCH_RV
#undef LAUNCH_R
    if (dbg) {
        uint32_t h[4];
        HIP_CHECK(hipMemcpyAsync(h, stats, 16, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        fprintf(stderr, "[faiss_amd] coarse bf3: nq=%lld k=%d survivors/q=%.2f failing streams/q=%.4f "
                "overflow=%u\n", (long long)n, k, h[0] / (double)n, h[1] / (double)n, h[2]);
    }
    HIP_LAUNCH_CHECK();
}

void array_max(const float* a, int64_t n, float* out, hipStream_t s) {
    k_array_max<<<dim3(1), dim3(1024), 0, s>>>(a, n, out);
    HIP_LAUNCH_CHECK();
}

}  // namespace kern
}  // namespace faiss_amd
