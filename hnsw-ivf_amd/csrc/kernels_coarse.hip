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
#include <cstring>
#include <type_traits>
#include <vector>

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

// the query's margin: bf16x3, coef (|x|^2 + max|c|^2); bf16x2 (centroids
// rounded to bf16, queries split), Cauchy-Schwarz on the centroid rounding
// residual: 2 (2 |x| max|c - bf16(c)| + coef (|x|^2 + max|c|^2)).
// cm = {max |c|^2, max |c - bf16(c)|}
__device__ __forceinline__ float coarse_margin(float xn, const float* __restrict__ cm, float coef,
                                               bool y3) {
    return y3 ? coef * (xn + cm[0]) + 1e-30f
              : 2.f * (2.f * sqrtf(xn) * cm[1] + coef * (xn + cm[0])) + 1e-30f;
}

// Pipeline as in the IVF-Flat filter (kernels_ivf_mfma.hip): one barrier per
// 64-centroid tile, tile t+1 stashed from registers while t is computed, the
// centroid norms (L2) / a +inf bias for rows past the split (IP) travel with
// the tile, so the compute never waits on a same-iteration global load and
// padding rows need no per-candidate test (their keys sort last and are
// dropped by index in the epilogue).
//
// Output per (query, split, thread stream): the KT raw 32-bit keys (~0 =
// empty) and a lower bound of every candidate the stream dropped (+inf when
// none), after subtracting the query's largest margin M = coef (|x|^2 +
// max|c|^2) (the re-rank uses the same M for every entry of the query).
template <bool L2, int KT, int NS, bool Y3>
__global__ __launch_bounds__(256, 2) void k_coarse_bf3_filter(
        const float* __restrict__ x, int ldx, int64_t n, int d, const __bf16* __restrict__ cbf,
        const float* __restrict__ cnorm, const float* __restrict__ xnorm, int nlist,
        int nsplit, int split_len, float coef, const float* __restrict__ cnmax_p, int obits,
        uint32_t* __restrict__ keys, float* __restrict__ pbs) {
    // Y3: centroid rows hi | lo (bf16x3); else hi only (bf16x2, half the bytes)
    __shared__ __attribute__((aligned(16))) uint8_t tiles[2 * BV * ((Y3 ? 4 : 2) * 16 * NS + 16)];
    __shared__ __attribute__((aligned(16))) float ynt[2][BV];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // blocks b and b+8 share an XCD: consecutive splits of one query block
    // stay together
    const int64_t qb = blockIdx.x / nsplit;
    const int sp = (int)(blockIdx.x % nsplit);
    const int c0 = sp * split_len;
    const int len = min(split_len, nlist - c0);
    constexpr int DB = 16 * NS, CSB = (Y3 ? 4 : 2) * DB + 16, RU = Y3 ? DB / 4 : DB / 8;
    constexpr int PF = (BV * RU + 255) / 256;  // uint4 per thread per tile
    const int bi = w >> 1, bj = w & 1, li = lane & 31, lh = lane >> 5;
    const int slot = 2 * bi + lh, qloc = 32 * bj + li;
    const int64_t q = qb * BQ + qloc;
    bf16x8 bh[NS], bl[NS];
    float xn_approx;
    load_query_frags<NS>(x, ldx, d, q < n ? (int)q : -1, lh, bh, bl, xn_approx);
    const float xn = q < n ? xnorm[q] : 0.f;  // the reference-order norm (exact side)
    const float* cn = cnorm + c0;

    uint4 pf[PF];
    float4 pn = make_float4(0.f, 0.f, 0.f, 0.f);
    auto fetch = [&](int v0n) {
        const int nvn = min(BV, len - v0n);
#pragma unroll
        for (int s = 0; s < PF; s++) {
            const int e = t + 256 * s;
            const int r = e / RU, c = e - r * RU;
            pf[s] = make_uint4(0u, 0u, 0u, 0u);
            if (e < BV * RU && r < nvn)
                pf[s] = *(const uint4*)(cbf + (int64_t)(c0 + v0n + r) * (2 * DB) + 8 * c);
        }
        if (t < BV / 4) {
            const int r = 4 * t;
            float v[4];
#pragma unroll
            for (int c = 0; c < 4; c++)
                v[c] = r + c < nvn ? (L2 ? cn[v0n + r + c] : 0.f) : WS_INF;
            pn = make_float4(v[0], v[1], v[2], v[3]);
        }
    };
    auto stash = [&](int buf) {
        uint8_t* T = tiles + buf * BV * CSB;
#pragma unroll
        for (int s = 0; s < PF; s++) {
            const int e = t + 256 * s;
            const int r = e / RU, c = e - r * RU;
            if (e < BV * RU) *(uint4*)(T + r * CSB + 16 * c) = pf[s];
        }
        if (t < BV / 4) *(float4*)(&ynt[buf][4 * t]) = pn;
    };
    fetch(0);
    stash(0);
    if (BV < len) fetch(BV);
    __syncthreads();

    ThreadQueue32<KT> tq;
    tq.init();
    const uint32_t lowmask = (1u << obits) - 1u;
    for (int v0 = 0, tile = 0; v0 < len; v0 += BV, tile++) {
        const int buf = tile & 1;
        if (v0 + BV < len) {
            stash(buf ^ 1);
            if (v0 + 2 * BV < len) fetch(v0 + 2 * BV);
        }
        float4 yq[4];
#pragma unroll
        for (int g = 0; g < 4; g++) yq[g] = *(const float4*)(&ynt[buf][32 * bi + 4 * lh + 8 * g]);
        const uint8_t* arow = tiles + buf * BV * CSB + (32 * bi + li) * CSB + 16 * lh;
        const floatx16 acc = Y3 ? bf3_block<NS>(arow, bh, bl) : bf2_block<NS>(arow, bh, bl);
        const uint32_t ordbase = (uint32_t)tile << 4;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int g = r >> 2, c = r & 3;
            const float yv = c == 0 ? yq[g].x : c == 1 ? yq[g].y : c == 2 ? yq[g].z : yq[g].w;
            // L2: clamped at 0 inside key_encode, as the reference clamps
            const float a = L2 ? fmaf(-2.f, acc[r], xn + yv) : yv - acc[r];
            tq.push(key_encode<L2>(a, lowmask, ordbase | (uint32_t)r));
        }
        __syncthreads();
    }
    if (q < n) {
        const float M = coarse_margin(xn, cnmax_p, coef, Y3);
        const int E1 = 4 * KT;
        uint32_t* ko = keys + (q * nsplit + sp) * E1 + slot * KT;
#pragma unroll
        for (int i = 0; i < KT; i++) {
            const uint32_t key = tq.q[i];
            const uint32_t row = ivf_key_row(key, lowmask, slot);
            ko[i] = (key != 0xffffffffu && row < (uint32_t)len) ? key : 0xffffffffu;
        }
        const uint32_t last = tq.q[KT - 1];
        float bnd = WS_INF;
        if (last != 0xffffffffu && ivf_key_row(last, lowmask, slot) < (uint32_t)len)
            bnd = key_decode_lo<L2>(last, lowmask);
        pbs[(q * nsplit + sp) * 4 + slot] = bnd < WS_INF ? bnd - M : WS_INF;
    }
}

// Streamed form (the default): 128 queries x one split per work group, the
// split's 64-centroid tiles copied global -> LDS by global_load_lds from the
// coarse stream image (per centroid: bf16 hi | bf16 lo | fp32 norm | 12 B; the
// image is padded to 64 rows with +inf-norm rows), two tile buffers, one raw
// barrier per tile (the IVF-Flat filter's k_ivf_bf2_stream pattern, here with
// bf16x3 blocks).  Work groups are ordered split-major per XCD (split s on
// XCD s mod 8, every query block of a split on the same XCD): a split's tiles
// are read from HBM once per XCD and then served from its L2.  Same keys and
// dropped bounds as k_coarse_bf3_filter; the 4 thread streams of a (query,
// split) are slot = 2 bi + lh.
template <int N>
__device__ __forceinline__ void cwait_vmcnt() {  // s_waitcnt vmcnt(N) alone
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Work groups per CU: the two tile buffers (2 x 64 x (4 DB + 16) bytes) fit
// three times in the LDS up to DB = 96 (d <= 96), twice at DB = 128; the
// register budget follows (three waves per SIMD need <= 168 VGPRs, which
// KT = 16 queues do not leave).
// FOLD (L2, fold image): the centroid and query norms enter the MFMA as one
// more k-step (A = the row's tail {-|c|^2/2 in three bf16 parts, 1, 1, 1, 0,
// 0}, B = {1, 1, 1, -|x|^2/2 in three parts, 0, 0}), the accumulator is
// -approx/2 and a candidate's key is one v_bfi_b32 of its bits (bf3.h
// fold_key_bits) instead of add + fma + max + bfi; no norm reads from LDS.
template <bool L2, int KT, int NS, bool FOLD = false>
__global__ __launch_bounds__(256, NS <= 6 && KT <= 8 ? 3 : 2) void k_coarse_stream(
        const float* __restrict__ x, int ldx, int64_t n, int d, const uint8_t* __restrict__ cst,
        const float* __restrict__ xnorm, int nlist, int nsplit, int split_len, int nqb,
        float coef, const float* __restrict__ cnmax_p, int obits, uint32_t* __restrict__ keys,
        float* __restrict__ pbs, unsigned long long* __restrict__ trace,
        const uint8_t* __restrict__ qimg) {
    // FAISS_AMD_COARSE_TRACE: per work group (wave 0) s_memtime stamps —
    // [0] start, [1] query fragments loaded, then per tile j: [2 + 2j] before
    // the tile wait, [3 + 2j] after its barrier
    unsigned long long* tr = (trace && threadIdx.x == 0) ? trace + 160ull * blockIdx.x : nullptr;
    if (tr) tr[0] = __builtin_amdgcn_s_memtime();
    constexpr int DB = 16 * NS;       // bf16 per part
    constexpr int SR = 4 * DB + 16;   // bytes per image row: hi | lo | norm | pad
    constexpr int TB = BV * SR;       // bytes per tile (whole KB)
    static_assert(TB % 1024 == 0, "tile = whole 1 KB glds blocks");
    constexpr int NG = TB / 1024;
    constexpr int G0 = (NG + 3) / 4;
    constexpr int G3 = NG / 4;
    __shared__ __attribute__((aligned(16))) uint8_t tiles[2 * TB];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int li = lane & 31, lh = lane >> 5;
    // split-major per XCD: blocks b = 8 m + xcd, m = j * nqb + qb, split
    // 8 j + xcd (nsplit a multiple of 8) — or block = sp * nqb + qb otherwise
    int sp, qb;
    if ((nsplit & 7) == 0) {
        const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
        sp = 8 * (m / nqb) + xcd;
        qb = m % nqb;
    } else {
        sp = blockIdx.x / nqb;
        qb = blockIdx.x % nqb;
    }
    const int c0 = sp * split_len;
    const int len = min(split_len, nlist - c0);
    const int ntile = (len + BV - 1) / BV;
    const int qloc = 32 * w + li;
    const int64_t q = (int64_t)qb * 128 + qloc;
    const bool active = (int64_t)qb * 128 + 32 * w < n;  // wave-uniform

    auto issue = [&](int j, int b) {
        const uint8_t* src = cst + ((int64_t)c0 + (int64_t)j * BV) * SR + 16 * lane;
        uint8_t* dst = tiles + b * TB;
#pragma unroll
        for (int g = 0; g < G0; g++) {
            const int blk = w + 4 * g;
            if (g < G3 || blk < NG)
                __builtin_amdgcn_global_load_lds(
                        (const void*)(src + blk * 1024),
                        (__attribute__((address_space(3))) void*)(dst + blk * 1024), 16, 0, 0);
        }
    };
    issue(0, 0);
    bf16x8 bh[NS], bl[NS];
    float xn_approx;
    if (active) {
        if (qimg)  // fragments prepared once per query (k_query_prep)
            load_query_image<NS>(qimg, nullptr, q < n ? (int)q : -1, lh, bh, bl, xn_approx);
        else
            load_query_frags<NS>(x, ldx, d, q < n ? (int)q : -1, lh, bh, bl, xn_approx);
    }
    const float xn = (active && q < n) ? xnorm[q] : 0.f;  // the reference-order norm
    if (tr) tr[1] = __builtin_amdgcn_s_memtime();
    static_assert(!FOLD || L2, "fold: L2 only");
    // FOLD: the bias B fragment {1, 1, 1, -|x|^2/2 in three parts, 0, 0} (lh = 0)
    bf16x8 bq;
    if constexpr (FOLD) {
        __bf16 h, m, lo;
        split3_bf16(-0.5f * xn, h, m, lo);
        const __bf16 one = (__bf16)1.f, zero = (__bf16)0.f;
        bq[0] = lh ? zero : one;
        bq[1] = lh ? zero : one;
        bq[2] = lh ? zero : one;
        bq[3] = lh ? zero : h;
        bq[4] = lh ? zero : m;
        bq[5] = lh ? zero : lo;
        bq[6] = zero;
        bq[7] = zero;
    }

    ThreadQueue32<KT> tq[2];
    tq[0].init();
    tq[1].init();
    const uint32_t lowmask = (1u << obits) - 1u;
    // the 16 norms of block bi of tile T: rows 32 bi + 4 lh + 8 g + c
    auto norms = [&](const uint8_t* T, int bi, float (&nv)[16]) {
        const uint8_t* nrow = T + (32 * bi + 4 * lh) * SR + 4 * DB;
#pragma unroll
        for (int r = 0; r < 16; r++) nv[r] = *(const float*)(nrow + (8 * (r >> 2) + (r & 3)) * SR);
    };
    auto push1 = [&](ThreadQueue32<KT>& pq, float accr, float yv0, uint32_t ord) {
        if constexpr (FOLD) {  // accr = -approx/2 already (read guarded by the caller)
            pq.push(key_insert(fold_key_bits(accr), lowmask, ord));
            return;
        }
        const float yv = L2 ? yv0 : (yv0 < WS_INF ? 0.f : WS_INF);  // IP: padding +inf
        // L2: clamped at 0 inside key_bits, as the reference clamps
        const float a = L2 ? fmaf(-2.f, accr, xn + yv) : yv - accr;
        pq.push(key_insert(key_bits<L2>(a), lowmask, ord));
    };
    // bf16x3 MFMAs of block bi of tile T with the 16 pushes of the previous
    // block interleaved between its k-steps (their VALU issues in the MFMA
    // gaps of this wave instead of after the chain)
    auto mfma_push = [&](const uint8_t* T, int bi, const floatx16& pacc, const float (&pn)[16],
                         const uint8_t* pnT, uint32_t pord, ThreadQueue32<KT>& pq) {
        const uint8_t* arow = T + (32 * bi + li) * SR + 16 * lh;
        bf16x8 ah[NS], al[NS];
#pragma unroll
        for (int s2 = 0; s2 < NS; s2++) {
            ah[s2] = *(const bf16x8*)(arow + 32 * s2);
            al[s2] = *(const bf16x8*)(arow + 2 * DB + 32 * s2);
        }
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < NS; s2++) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[s2], bh[s2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s2], bl[s2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s2], bh[s2], acc, 0, 0, 0);
            // FOLD: the inline-asm key insert reads pacc (an MFMA result)
            if (FOLD && s2 == 0) mfma_read_guard();
#pragma unroll
            for (int r = 16 * s2 / NS; r < 16 * (s2 + 1) / NS; r++)
                push1(pq, pacc[r],
                      FOLD ? 0.f
                           : pnT ? *(const float*)(pnT + (8 * (r >> 2) + (r & 3)) * SR) : pn[r],
                      pord | (uint32_t)r);
        }
        if constexpr (FOLD) {
            // the row's bias fragment (lh = 1: its hi bytes, times 0)
            const bf16x8 ab = *(const bf16x8*)(T + (32 * bi + li) * SR + (lh ? 0 : 4 * DB));
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bq, acc, 0, 0, 0);
        }
        return acc;
    };
    // software pipeline over blocks: phase A = MFMAs of (tile j, block 1) +
    // pushes of (j, 0); phase B = MFMAs of (j + 1, 0) + pushes of (j, 1).
    // The norms of a block are read with its MFMAs (its buffer is refilled
    // before its pushes may run).
    floatx16 acc0, acc1;
    float n1[16];
    cwait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // tile 0 (every wave's part)
    if (ntile > 1) issue(1, 1);
    if (active) {
        acc0 = bf3_block<NS>(tiles + (0 * SR) + li * SR + 16 * lh, bh, bl);
        if constexpr (FOLD) {
            const bf16x8 ab = *(const bf16x8*)(tiles + li * SR + (lh ? 0 : 4 * DB));
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bq, acc0, 0, 0, 0);
        }
    }
    int b = 0;
    for (int j = 0; j < ntile; j++) {
        const uint8_t* T = tiles + b * TB;
        const uint32_t ordbase = (uint32_t)j << 4;
        if (active) {
            // (block 0's norms straight from LDS: tile j stays until the barrier)
            acc1 = mfma_push(T, 1, acc0, n1, T + 4 * lh * SR + 4 * DB, ordbase, tq[0]);
            if constexpr (!FOLD) norms(T, 1, n1);
        }
        if (j + 1 < ntile) {
            if (tr && j < 78) tr[2 + 2 * j] = __builtin_amdgcn_s_memtime();
            cwait_vmcnt<0>();  // tile j + 1 (this wave's part)
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0): tile j read
            __builtin_amdgcn_s_barrier();  // every wave: tile j + 1 landed, tile j consumed
            if (tr && j < 78) tr[3 + 2 * j] = __builtin_amdgcn_s_memtime();
            if (j + 2 < ntile) issue(j + 2, b);
            const uint8_t* T1 = tiles + (b ^ 1) * TB;
            if (active) {
                acc0 = mfma_push(T1, 0, acc1, n1, nullptr, ordbase, tq[1]);
            }
        } else if (active) {
            if constexpr (FOLD) mfma_read_guard();
#pragma unroll
            for (int r = 0; r < 16; r++)
                push1(tq[1], acc1[r], FOLD ? 0.f : n1[r], ordbase | (uint32_t)r);
        }
        b ^= 1;
    }
    if (active && q < n) {
        const float M = coarse_margin(xn, cnmax_p, coef, true);
        const int E1 = 4 * KT;
#pragma unroll
        for (int bi = 0; bi < 2; bi++) {
            const int slot = 2 * bi + lh;
            uint32_t* ko = keys + (q * nsplit + sp) * E1 + slot * KT;
#pragma unroll
            for (int i = 0; i < KT; i++) {
                const uint32_t key = tq[bi].q[i];
                const uint32_t row = ivf_key_row(key, lowmask, slot);
                ko[i] = (key != 0xffffffffu && row < (uint32_t)len) ? key : 0xffffffffu;
            }
            const uint32_t last = tq[bi].q[KT - 1];
            float bnd = WS_INF;
            if (last != 0xffffffffu && ivf_key_row(last, lowmask, slot) < (uint32_t)len)
                bnd = FOLD ? fold_decode_lo(last, lowmask) : key_decode_lo<L2>(last, lowmask);
            pbs[(q * nsplit + sp) * 4 + slot] = bnd < WS_INF ? bnd - M : WS_INF;
        }
    }
}

// coarse stream image: row r < rows = bf16 hi | bf16 lo of the centroid (DB
// dims each, zero past d) | its norm | 12 zero bytes; rows past `rows` (up to
// the 64-row padding) are zero with a +inf norm
__global__ void k_coarse_image(const float* __restrict__ codes, int64_t rows, int64_t rows_pad,
                               int d, int ldc, int DB, const float* __restrict__ norms,
                               uint8_t* __restrict__ out, int fold) {
    const int per = DB + 4;  // slots per row: DB (hi, lo) pairs, norm, 3 pad words
    GRID_STRIDE(i, rows_pad * per) {
        const int64_t r = i / per;
        const int j = (int)(i - r * per);
        uint8_t* row = out + r * (int64_t)(4 * DB + 16);
        if (j < DB) {
            const float v = (r < rows && j < d) ? codes[r * ldc + j] : 0.f;
            const __bf16 h = (__bf16)v;
            ((__bf16*)row)[j] = h;
            ((__bf16*)row)[DB + j] = (__bf16)(v - (float)h);
        } else if (fold) {
            // bias A-fragment {-|c|^2/2 in three bf16 parts, 1, 1, 1, 0, 0}
            // (padding rows: -inf, 0, 0, 1, 1, 1, 0, 0): two bf16 per slot
            __bf16 h = (__bf16)(-WS_INF), m = (__bf16)0.f, lo = (__bf16)0.f;
            if (r < rows) split3_bf16(-0.5f * norms[r], h, m, lo);
            const __bf16 one = (__bf16)1.f, zero = (__bf16)0.f;
            const int t = j - DB;  // bf16 pair t of the 16-byte tail
            __bf16* tail = (__bf16*)(row + 4 * DB);
            const __bf16 v[8] = {h, m, lo, one, one, one, zero, zero};
            tail[2 * t] = v[2 * t];
            tail[2 * t + 1] = v[2 * t + 1];
        } else {
            float* tail = (float*)(row + 4 * DB);
            tail[j - DB] = j == DB ? (r < rows ? norms[r] : WS_INF) : 0.f;
        }
    }
}
void coarse_stream_image(const float* codes, int64_t rows, int d, int ldc, const float* norms,
                         void* out, hipStream_t s, int fold) {
    const int DB = bf3_db(d);
    const int64_t rows_pad = (int64_t)roundup((size_t)std::max<int64_t>(rows, 1), BV);
    k_coarse_image<<<stride_grid(rows_pad * (DB + 4), 256), dim3(256), 0, s>>>(
            codes, rows, rows_pad, d, ldc, DB, norms, (uint8_t*)out, fold);
    HIP_LAUNCH_CHECK();
}
size_t coarse_stream_image_bytes(int64_t rows, int d) {
    return (size_t)roundup((size_t)std::max<int64_t>(rows, 1), BV) * (4 * bf3_db(d) + 16);
}

// Query preparation: 32 queries per 64-lane block, lane (li, lh) builds the
// fragments load_query_frags would build for query li (lh = which 8-dim half
// of each 16-dim step) and stores them in the query image; lanes lh == 0
// also write |x|^2 (the fragments' order) and the reference-order norm.
template <int NS>
__global__ __launch_bounds__(64) void k_query_prep(const float* __restrict__ x, int64_t n,
                                                   int ldx, int d, float* __restrict__ ref_norms,
                                                   uint8_t* __restrict__ qimg,
                                                   float* __restrict__ qxn) {
    const int lane = threadIdx.x, li = lane & 31, lh = lane >> 5;
    const int64_t q = (int64_t)blockIdx.x * 32 + li;
    const int qr = q < n ? (int)q : -1;
    bf16x8 bh[NS], bl[NS];
    float xn;
    load_query_frags<NS>(x, ldx, d, qr, lh, bh, bl, xn);  // every lane: the shfl pairs halves
    if (qr < 0) return;
    uint8_t* row = qimg + q * (64 * NS) + 16 * lh;
#pragma unroll
    for (int s = 0; s < NS; s++) {
        *(bf16x8*)(row + 32 * s) = bh[s];
        *(bf16x8*)(row + 32 * NS + 32 * s) = bl[s];
    }
    if (lh == 0) {
        if (qxn) qxn[q] = xn;
        if (ref_norms) ref_norms[q] = ref_norm(x + q * ldx, d);
    }
}

void query_prep(const float* x, int64_t n, int ldx, int d, float* ref_norms, void* qimg,
                float* qxn, hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT(ldx % 4 == 0 && bf3_db(d) <= BDM && qimg != nullptr);
    const int NS = bf3_db(d) / 16;
    const dim3 grid((unsigned)cdiv(n, 32)), blk(64);
    uint8_t* qi = (uint8_t*)qimg;
    if (NS == 2) k_query_prep<2><<<grid, blk, 0, s>>>(x, n, ldx, d, ref_norms, qi, qxn);
    else if (NS == 4) k_query_prep<4><<<grid, blk, 0, s>>>(x, n, ldx, d, ref_norms, qi, qxn);
    else if (NS == 6) k_query_prep<6><<<grid, blk, 0, s>>>(x, n, ldx, d, ref_norms, qi, qxn);
    else k_query_prep<8><<<grid, blk, 0, s>>>(x, n, ldx, d, ref_norms, qi, qxn);
    HIP_LAUNCH_CHECK();
}

constexpr int CR_CAP = 512;

// exact coarse distance of centroid j (the fixed BLAS-form order: sequential
// fma chain for <x, c>, then fma(-2, ip, |x|^2 + |c|^2) clamped at 0 for L2),
// query from LDS, centroid rows L2-resident (one lane per centroid)
template <bool L2>
__device__ __forceinline__ float coarse_exact(const float* xs, const float* __restrict__ cent,
                                              int ldc, const float* __restrict__ cnorm, float xn,
                                              int d, int j) {
    const float ip = ip_seq(xs, cent + (int64_t)j * ldc, d);
    if (!L2) return ip;
    const float dis = fmaf(-2.f, ip, xn + cnorm[j]);
    return dis < 0.f ? 0.f : dis;
}

template <bool L2>
struct CoarseStream {
    const uint32_t* surv;  // candidate centroids (LDS)
    const uint32_t* keys;  // this query's [nsplit * 4 * KT] raw keys
    const float* xs;       // LDS copy of the query
    const float* cent;
    const float* cnorm;
    float xn, M, U;
    int ldc, d, nlist, nsplit, split_len, E, KT, lane, nsv;
    uint32_t lowmask;
    bool overflow;
    bool fold;                 // folded filter keys (ivf_decode_lo)
    unsigned long long fmask;  // failing streams: bit 4 * split + slot

    __device__ __forceinline__ void emit(bool ok, int j, float& k1, long long& k2) const {
        k1 = WS_INF;
        k2 = WS_NOID;
        if (ok) to_key(L2 ? 1 : 0, coarse_exact<L2>(xs, cent, ldc, cnorm, xn, d, j), j, k1, k2);
    }
    template <class F>
    __device__ __forceinline__ void for_each(F f) const {
        if (!overflow) {
            for (int s0 = 0; s0 < nsv; s0 += 64) {
                const bool ok = s0 + lane < nsv;
                const int j = ok ? (int)surv[s0 + lane] : 0;
                float k1;
                long long k2;
                emit(ok, j, k1, k2);
                f(ok && key_admissible(k1), k1, k2, (long long)j);
            }
            return;
        }
        for (int c0 = 0; c0 < E; c0 += 64) {
            const int c = c0 + lane;
            const int st = c < E ? c / KT : 0;  // stream 4 * split + slot
            bool ok = false;
            int j = 0;
            if (c < E && !((fmask >> st) & 1ull)) {
                const uint32_t key = keys[c];
                ok = key != 0xffffffffu && ivf_decode_lo<L2>(key, lowmask, fold) - M <= U;
                j = (st >> 2) * split_len + (int)ivf_key_row(key, lowmask, st & 3);
            }
            if (__ballot(ok) == 0ull) continue;
            float k1;
            long long k2;
            emit(ok, j, k1, k2);
            f(ok && key_admissible(k1), k1, k2, (long long)j);
        }
        unsigned long long m = fmask;
        while (m) {
            const int sidx = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const int sp = sidx >> 2, slot = sidx & 3;
            const int j0 = sp * split_len, j1 = min(nlist, j0 + split_len);
            const int ne = (int)cdiv_dev((uint32_t)(j1 - j0), BV) * 16;
            for (int e0 = 0; e0 < ne; e0 += 64) {
                const int j = j0 + ivf_stream_row(e0 + lane, slot);
                const bool ok = e0 + lane < ne && j < j1;
                float k1;
                long long k2;
                emit(ok, j, k1, k2);
                f(ok && key_admissible(k1), k1, k2, (long long)j);
            }
        }
    }
};

// One wave per query (block = one wave).  Same structure as k_ivf_rerank:
// round trip 1 = the raw keys (V consecutive per lane, one stream per lane),
// the streams' dropped bounds and the query; U = k-th smallest ub' = approx_hi
// + M; candidates = entries with approx_lo - M <= U of the streams that did
// not fail, plus every centroid of the failing streams; exact evaluation and a
// rank-based top-k (exact_topk_resolve when a tie crosses the boundary).
template <bool L2, class OutIdx, int V>
#ifndef CR_WAVES
#define CR_WAVES 4  // waves per SIMD the re-rank is compiled for (tuning)
#endif
__global__ __launch_bounds__(64, CR_WAVES) void k_coarse_rerank(
        const uint32_t* __restrict__ keys, const float* __restrict__ pbs,
        const float* __restrict__ x, int ldx, const float* __restrict__ xnorm,
        const float* __restrict__ cent, int ldc, const float* __restrict__ cnorm,
        const float* __restrict__ cnmax_p, float coef, int y3, int64_t n, int d, int nlist,
        int nsplit, int split_len, int KT, int obits, int k, float* __restrict__ D,
        OutIdx* __restrict__ I, uint32_t* __restrict__ stats,
        unsigned long long* __restrict__ trace, int fold_keys) {
    const bool fold = L2 && fold_keys != 0;
    const unsigned long long t_start = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    __shared__ uint32_t surv[CR_CAP];
    __shared__ float ck1[256];      // compaction scratch of the small-batch select
    __shared__ long long ck2[256];
    __shared__ __attribute__((aligned(16))) float xsh[BDM];
    const int lane = threadIdx.x;
    const int64_t q0 = blockIdx.x;
    const bool valid = q0 < n;
    const int64_t q = valid ? q0 : 0;
    const int E1 = 4 * KT, E = valid ? nsplit * E1 : 0, NST = 4 * nsplit;
    const uint32_t lowmask = (1u << obits) - 1u;
    // ---- round trip 1
    const uint32_t* kq = keys + q * (int64_t)nsplit * E1;
    uint32_t kv[V];
    const bool has = lane * V < E;
#pragma unroll
    for (int i = 0; i < V; i++) kv[i] = has ? kq[lane * V + i] : 0xffffffffu;
    const float my_pb = (valid && lane < NST) ? pbs[q * NST + lane] : WS_INF;
    const float xn = xnorm ? xnorm[q] : 0.f;
    const float* xq = x + q * ldx;
    if (lane < BDM / 4 && 4 * lane < ((d + 3) & ~3))
        *(float4*)(&xsh[4 * lane]) = *(const float4*)(xq + 4 * lane);
    const float M = coarse_margin(xn, cnmax_p, coef, y3 != 0);
    // ---- U
    float ub[V];
#pragma unroll
    for (int i = 0; i < V; i++)
        ub[i] = kv[i] != 0xffffffffu ? ivf_decode_hi<L2>(kv[i], lowmask, fold) + M : WS_INF;
    float U = wave_kth_smallest<V, 12>(ub, k);  // an upper bound (wave_select.h)
    const unsigned long long t_u = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (!(U <= WS_INF)) U = WS_INF;
    const unsigned long long fmask = __ballot(my_pb < WS_INF && my_pb <= U);
    const int lst = has ? lane * V / KT : 0;  // this lane's stream (V <= KT)
    const bool lfail = (fmask >> lst) & 1ull;
    // ---- candidates -> LDS
    int ns = 0;
#pragma unroll
    for (int i = 0; i < V; i++) {
        bool sv = false;
        uint32_t j = 0;
        if (kv[i] != 0xffffffffu && !lfail) {
            sv = ivf_decode_lo<L2>(kv[i], lowmask, fold) - M <= U;
            j = (uint32_t)((lst >> 2) * split_len) + ivf_key_row(kv[i], lowmask, lst & 3);
        }
        const unsigned long long m = __ballot(sv);
        const int pos = ns + __popcll(m & ((1ull << lane) - 1ull));
        if (sv && pos < CR_CAP) surv[pos] = j;
        ns += __popcll(m);
    }
    {
        unsigned long long m = fmask;
        while (m) {
            const int sidx = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const int sp = sidx >> 2, slot = sidx & 3;
            const int j0 = sp * split_len, j1 = min(nlist, j0 + split_len);
            const int ne = (int)cdiv_dev((uint32_t)(j1 - j0), BV) * 16;
            for (int e0 = 0; e0 < ne; e0 += 64) {
                const int j = j0 + ivf_stream_row(e0 + lane, slot);
                const bool in = e0 + lane < ne && j < j1;
                const unsigned long long bm = __ballot(in);
                const int pos = ns + __popcll(bm & ((1ull << lane) - 1ull));
                if (in && pos < CR_CAP) surv[pos] = (uint32_t)j;
                ns += __popcll(bm);
            }
        }
    }
    __syncthreads();  // one wave per block: the LDS query and candidate list
    const unsigned long long t_c = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    CoarseStream<L2> st;
    st.surv = surv;
    st.keys = kq;
    st.xs = xsh;
    st.cent = cent;
    st.cnorm = cnorm;
    st.xn = xn;
    st.M = M;
    st.U = U;
    st.ldc = ldc;
    st.d = d;
    st.nlist = nlist;
    st.nsplit = nsplit;
    st.split_len = split_len;
    st.E = E;
    st.KT = KT;
    st.lane = lane;
    st.nsv = ns;
    st.lowmask = lowmask;
    st.overflow = ns > CR_CAP;
    st.fold = fold;
    st.fmask = fmask;
    bool done = false;
    unsigned long long t_e = 0ull;
    auto small = [&](auto nbc) {
        constexpr int NB = decltype(nbc)::value;
        float k1[NB];
        long long k2[NB];
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const bool ok = 64 * b + lane < ns;
            st.emit(ok, ok ? (int)surv[64 * b + lane] : 0, k1[b], k2[b]);
            if (!(ok && key_admissible(k1[b]))) {
                k1[b] = WS_INF;
                k2[b] = WS_NOID;
            }
        }
        if (trace) t_e = __builtin_amdgcn_s_memrealtime();
        if constexpr (NB > 1) {
            // only keys <= U can be in the top k (at least k candidates have
            // exact keys <= their ub <= U): a failing split adds a whole
            // split of candidates, most far above U; the order-preserving
            // compaction of the others ranks in one batch (as k_ivf_rerank)
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
                return exact_topk_small<1, OutIdx>(c1, c2, m, k, L2 ? 1 : 0, lane, valid,
                                                   D + q * k, I + q * k);
            }
        }
        return exact_topk_small<NB, OutIdx>(k1, k2, ns, k, L2 ? 1 : 0, lane, valid, D + q * k,
                                            I + q * k);
    };
    if (ns <= 64) done = small(std::integral_constant<int, 1>());
    else if (ns <= 128) done = small(std::integral_constant<int, 2>());
    else if (ns <= 256) done = small(std::integral_constant<int, 4>());
    if (!done) exact_topk_resolve(st, k, L2 ? 1 : 0, lane, valid, D + q * k, I + q * k);
    if (trace && valid && lane == 0) {  // FAISS_AMD_CRERANK_TRACE (scripts/rtrace_summary.py)
        trace[8 * q + 0] = t_start;
        trace[8 * q + 1] = __builtin_amdgcn_s_memrealtime();
        trace[8 * q + 2] = (unsigned long long)ns | ((unsigned long long)__popcll(fmask) << 32);
        trace[8 * q + 3] = t_u;
        trace[8 * q + 4] = t_c;
        trace[8 * q + 5] = t_e;
    }
    if (stats && valid && lane == 0) {
        atomicAdd(&stats[0], (uint32_t)min(ns, CR_CAP));
        atomicAdd(&stats[1], (uint32_t)__popcll(fmask));
        atomicAdd(&stats[2], st.overflow ? 1u : 0u);
        atomicAdd(&stats[3], done ? 0u : 1u);
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
    // At most 16 splits (the re-rank keeps one thread stream per lane).
    // Each of the 4 * nsplit thread streams keeps KT keys; it "fails" (is
    // re-scanned exactly) when more than KT of the top-k + margin fall in it.
    // With lam = k / (4 nsplit) expected members per stream, KT = 4 / 8 / 16
    // for lam <= 1/4 / 2 / 4 keeps the Poisson tail below ~1e-3 per query.
    //
    // The split count sets the grid: cdiv(n, 128) query blocks x nsplit work
    // groups, two resident per CU (k_coarse_stream's two 64-centroid tile
    // buffers).  The kernel's time is (rounds of resident groups) x (tiles
    // per group) x (per-tile cost, growing with KT), so the split count is
    // the one minimising that product — e.g. c2 (10k queries, 4096
    // centroids): 6 splits of 11 tiles in one round instead of 8 splits of 8
    // tiles in two.  When the centroid image exceeds one XCD's L2, split
    // counts that are not a multiple of 8 lose the split-major XCD order
    // (each split read from HBM once per XCD) and are charged for it.
    int ncu = 256, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
        ncu = 256;
    (void)hipGetLastError();
    const int64_t nqb = (int64_t)cdiv((size_t)n, 128);

    const bool big_image = coarse_stream_image_bytes(nlist, d) > ((size_t)4 << 20);
    int nsplit = 0, kt = 0, split_len = 0;
    double best = 0.0;
    const char* nsenv = getenv("FAISS_AMD_COARSE_NSPLIT");  // forces the split count (tuning)
    const int ns_force = nsenv ? atoi(nsenv) : 0;
    for (int ns = 1; ns <= std::min(16, std::max(1, nlist / BV)); ns++) {
        if (ns_force > 0 && ns != ns_force) continue;
        if (k > 16 * ns) continue;
        const double lam = (double)k / (4.0 * ns);
        if (lam > 4.0) continue;
        const int kt1 = lam <= 0.25 ? 4 : lam <= 2.0 ? 8 : 16;
        const int sl = (int)roundup(cdiv((size_t)nlist, (size_t)ns), BV);
        const int nsp = (int)cdiv((size_t)nlist, (size_t)sl);
        if ((size_t)sl > ((size_t)BV << 10)) continue;  // ordinals: 4 + log2(tiles) <= 14 bits
        // resident work groups (k_coarse_stream: 3 per CU for DB <= 96 and
        // KT <= 8, else 2)
        const int64_t slots = (bf3_db(d) <= 96 && kt1 <= 8 ? 3 : 2) * (int64_t)ncu;
        const int64_t rounds = (int64_t)cdiv((size_t)(nqb * nsp), (size_t)slots);
        double cost = (double)rounds * (double)cdiv((size_t)sl, BV) * (kt1 + 12);
        if (big_image && nsp % 8 != 0) cost *= 1.15;
        if (nsplit == 0 || cost < best) {
            best = cost;
            nsplit = nsp;
            kt = kt1;
            split_len = sl;
        }
    }
    if (nsplit == 0) return p;
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
                    const float* cnmax, int nlist, int d, int k, int metric_l2, uint32_t* keys,
                    float* pbs, float* D, int32_t* I32, int64_t* I64, hipStream_t s,
                    const void* cst, const void* qimg, KernelTimes* kt, int fold) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT(p.ok);
    static uint32_t* stats = nullptr;  // FAISS_AMD_IVF_STATS debug counters
    const bool dbg = getenv("FAISS_AMD_IVF_STATS") != nullptr;
    if (dbg && !stats) HIP_CHECK(hipMalloc(&stats, 16));
    if (dbg) HIP_CHECK(hipMemsetAsync(stats, 0, 16, s));
    FAISS_THROW_IF_NOT(ldx % 4 == 0 && ldc % 4 == 0);
    const int NS = bf3_db(d) / 16;
    // bf16x3 by default.  FAISS_AMD_COARSE_PREC=bf16x2 (two MFMA passes, half
    // the centroid bytes) is exact too, but its Cauchy-Schwarz margin on the
    // centroids' bf16 rounding (cnmax[1]) is ~20x wider than the bf16x3 one:
    // centroids near a query are dense, so on uniform data (c2: 0.4 -> 1.9 ms
    // per step) the streams overflow and fail; kept for clustered data
    const char* prec = getenv("FAISS_AMD_COARSE_PREC");
    const bool y3 = !(prec && !strcmp(prec, "bf16x2"));
    // streamed bf16x3 kernel (default when the image exists;
    // FAISS_AMD_COARSE=staged: the register-staged one)
    const char* cenv = getenv("FAISS_AMD_COARSE");
    const bool stream = cst && y3 && !(cenv && !strcmp(cenv, "staged"));
    // fold: the image's tails are bias fragments (only the streamed L2 kernel
    // reads the image)
    const bool fk = stream && fold != 0 && metric_l2;
    const float coef = (float)(fk ? ivf_bf3f_coef(d) : y3 ? ivf_bf3_coef(d) : ivf_bf2_coef(d));
    static unsigned long long* ctrace_buf = nullptr;
    static int64_t ctrace_n = 0;
    const char* ctr = getenv("FAISS_AMD_COARSE_TRACE");
    unsigned long long* ctrace = nullptr;
    const int64_t nqb = (int64_t)cdiv((size_t)n, stream ? 128 : BQ);
    const int64_t grid = nqb * p.nsplit;
    FAISS_THROW_IF_NOT(grid < (1ll << 31));
    if (ctr && stream) {
        if (ctrace_n < grid) {
            if (ctrace_buf) HIP_CHECK(hipFree(ctrace_buf));
            HIP_CHECK(hipMalloc(&ctrace_buf, 160 * 8 * grid));
            ctrace_n = grid;
        }
        HIP_CHECK(hipMemsetAsync(ctrace_buf, 0, 160 * 8 * grid, s));
        ctrace = ctrace_buf;
    }
#define LAUNCH_NS(L2V, KTV, NSV)                                                              \
    do {                                                                                      \
        if (stream)                                                                           \
            (fk ? k_coarse_stream<L2V, KTV, NSV, L2V> : k_coarse_stream<L2V, KTV, NSV, false>) \
                    <<<kgrid(grid, 256), dim3(256), 0, s>>>(                              \
                    x, ldx, n, d, (const uint8_t*)cst, xnorm, nlist, p.nsplit, p.split_len,   \
                    (int)nqb, coef, cnmax, p.obits, keys, pbs, ctrace,                        \
                    (const uint8_t*)qimg);                                                    \
        else if (y3)                                                                          \
            k_coarse_bf3_filter<L2V, KTV, NSV, true><<<kgrid(grid, 256), dim3(256), 0, s>>>( \
                    x, ldx, n, d, (const __bf16*)cbf, cnorm, xnorm, nlist, p.nsplit,          \
                    p.split_len, coef, cnmax, p.obits, keys, pbs);                            \
        else                                                                                  \
            k_coarse_bf3_filter<L2V, KTV, NSV, false><<<kgrid(grid, 256), dim3(256), 0, s>>>( \
                    x, ldx, n, d, (const __bf16*)cbf, cnorm, xnorm, nlist, p.nsplit,          \
                    p.split_len, coef, cnmax, p.obits, keys, pbs);                            \
    } while (0)
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
    {
        ScopedKernelTimer tm(kt, "coarse_filter", 0.0, s);
        if (metric_l2) DISPATCH(true);
        else DISPATCH(false);
    }
#undef DISPATCH
#undef LAUNCH_A
#undef LAUNCH_NS
    HIP_LAUNCH_CHECK();
    if (ctrace) {
        std::vector<unsigned long long> h(160 * grid);
        HIP_CHECK(hipMemcpyAsync(h.data(), ctrace, 160 * 8 * grid, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if (FILE* f = fopen(ctr, "wb")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
    const int E = p.entries;
    const int V = E <= 64 ? 1 : E <= 128 ? 2 : E <= 256 ? 4 : E <= 512 ? 8 : 16;
    FAISS_THROW_IF_NOT(E <= 1024 && V <= p.kt);
#define LAUNCH_R(L2V, OT, OUT, VV)                                                              \
    k_coarse_rerank<L2V, OT, VV><<<kgrid(n, 64), dim3(64), 0, s>>>(                       \
            keys, pbs, x, ldx, xnorm, cent, ldc, cnorm, cnmax, coef, y3 ? 1 : 0, n, d, nlist,  \
            p.nsplit,                                                                           \
            p.split_len, p.kt, p.obits, k, D, OUT, st_ptr, crtrace, fk ? 1 : 0)
#define LAUNCH_RV(L2V, OT, OUT)                  \
    do {                                         \
        if (V == 1) LAUNCH_R(L2V, OT, OUT, 1);   \
        else if (V == 2) LAUNCH_R(L2V, OT, OUT, 2); \
        else if (V == 4) LAUNCH_R(L2V, OT, OUT, 4); \
        else if (V == 8) LAUNCH_R(L2V, OT, OUT, 8); \
        else LAUNCH_R(L2V, OT, OUT, 16);         \
    } while (0)
    uint32_t* const st_ptr = dbg ? stats : nullptr;
    // FAISS_AMD_CRERANK_TRACE=<file>: per-query wave stamps (profiling only)
    static unsigned long long* crtrace_buf = nullptr;
    static int64_t crtrace_n = 0;
    const char* crt = getenv("FAISS_AMD_CRERANK_TRACE");
    unsigned long long* crtrace = nullptr;
    if (crt) {
        if (crtrace_n < n) {
            if (crtrace_buf) HIP_CHECK(hipFree(crtrace_buf));
            HIP_CHECK(hipMalloc(&crtrace_buf, 64 * n));
            crtrace_n = n;
        }
        HIP_CHECK(hipMemsetAsync(crtrace_buf, 0, 64 * n, s));
        crtrace = crtrace_buf;
    }
    {
        ScopedKernelTimer tm(kt, "coarse_rerank", 0.0, s);
        if (metric_l2) {
            if (I32) LAUNCH_RV(true, int32_t, I32);
            else LAUNCH_RV(true, int64_t, I64);
        } else {
            if (I32) LAUNCH_RV(false, int32_t, I32);
            else LAUNCH_RV(false, int64_t, I64);
        }
    }
#undef LAUNCH_RV
#undef LAUNCH_R
    if (crtrace) {
        std::vector<unsigned long long> h(8 * n);
        HIP_CHECK(hipMemcpyAsync(h.data(), crtrace, 64 * n, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if (FILE* f = fopen(crt, "wb")) {
            fwrite(h.data(), 64, n, f);
            fclose(f);
        }
    }
    if (dbg) {
        uint32_t h[4];
        HIP_CHECK(hipMemcpyAsync(h, stats, 16, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        fprintf(stderr, "[faiss_amd] coarse bf3: nq=%lld k=%d survivors/q=%.2f failing streams/q=%.4f "
                "overflow=%u general-resolve=%u\n", (long long)n, k, h[0] / (double)n,
                h[1] / (double)n, h[2], h[3]);
    }
    HIP_LAUNCH_CHECK();
}

void array_max(const float* a, int64_t n, float* out, hipStream_t s) {
    k_array_max<<<dim3(1), dim3(1024), 0, s>>>(a, n, out);
    HIP_LAUNCH_CHECK();
}

}  // namespace kern
}  // namespace faiss_amd
