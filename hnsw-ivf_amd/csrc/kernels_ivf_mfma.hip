// kernels_ivf_mfma.hip — IVF-Flat scan on fp32 MFMA with an exact re-rank.
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

static_assert(FQ == IVF_FLAT_QT, "host and filter must agree on the work-item width");


// ---------------------------------------------------------------- A
// Filter on bf16x3 MFMA (v_mfma_f32_32x32x16_bf16).  Every f32 value is
// split x = xh + xl (+ xr), xh = bf16(x), xl = bf16(x - xh), |xr| <= 2^-16|x|;
// <x,y> ~ xh.yh + xh.yl + xl.yh (products exact in f32, accumulated in f32).
//   |ip_approx - ip| <= (3.1 * 2^-16 + 3 d u) sum|x_i y_i|
// so with the f32 rounding of the norms, of the approx formula and of the
// exact sequential evaluation (same analysis as above):
//   |approx - exact| <= (3.1 * 2^-16 + (6d + 8) u) (|x|^2 + |y|^2)
// The kernel uses twice that (host: ivf_bf3_coef) plus 1e-30 absolute.
//
// Roles: A = codes (rows = 32 codes per wave), B = queries (columns = 32
// queries per wave, held in registers for the whole work item).  A lane's 16
// accumulators are ONE query against 16 codes, so the per-thread queues are
// fed straight from the MFMA result: 4 threads (2 waves x 2 lane halves) per
// query, no LDS transpose.
//
// Keys are 32 bit: ordered_f32(approx) with the low `obits` bits replaced by
// the thread-local candidate ordinal (tile << 4 | r).  The truncation only
// widens the [lb, ub] interval (decoded with the low bits cleared / set).
//
// Per (query, list) output, 4*KT entries (4 threads x KT keys each):
//   part[e][i] = ordered_f32(lb) << 32 | arena row   (~0 = empty)
//   pub[e][i]  = ub                             (upper bound of the exact key)
//   pbound[e]  = lower bound of the exact key of every dropped candidate of
//                the list (min over the 4 threads of their KT-th key, minus
//                the list's largest margin); +inf if none was dropped.
// f32 arena -> bf16 hi/lo arena: row r = hi[DB] | lo[DB], zero beyond d
__global__ void k_split_bf16(const float* __restrict__ codes, int64_t rows, int d, int ldc, int DB,
                             __bf16* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * DB) return;
    const int64_t r = i / DB;
    const int j = (int)(i - r * DB);
    const float v = j < d ? codes[r * ldc + j] : 0.f;
    const __bf16 h = (__bf16)v;
    out[r * 2 * DB + j] = h;
    out[r * 2 * DB + DB + j] = (__bf16)(v - (float)h);
}

// Y3: bf16x3 (codes split hi + lo, three MFMAs per k-step);  !Y3: bf16x2
// (codes rounded to bf16, queries split: two MFMAs per k-step, half the code
// bytes streamed; wider margin, ivf_bf2_coef).  Both read the same hi|lo
// image; !Y3 touches only the hi half of every row.
//
// Pipeline (one barrier per 64-row tile): tile t+1 is stashed from registers
// into the other LDS buffer while tile t is computed, and tile t+2 is fetched
// into registers; the row norms travel with the tile (LDS), so the compute of
// a tile never waits on a global load issued in the same iteration.  Rows
// past the list end get norm +inf (L2) / bias +inf (IP): their keys sort
// after every real candidate and the epilogue drops them by row index.
// Waves whose 32 query columns are all unused skip the MFMA and selection.
// HS: an IDSelector mask is present (a separate instantiation, so the
// unfiltered hot path carries no mask loads or registers).
template <bool L2, int KT, int NS, bool Y3, bool HS>
__global__ __launch_bounds__(256, Y3 ? 2 : 3) void k_ivf_bf3_filter(
        const float* __restrict__ x, int ldx, int d, const __bf16* __restrict__ cbf,
        const float* __restrict__ ynorm, const float* __restrict__ ynmax,
        const float* __restrict__ rres, const float* __restrict__ rmax,
        const uint32_t* __restrict__ list_off, const uint32_t* __restrict__ list_len, int nlist,
        int nprobe, float coef, int obits, const uint32_t* __restrict__ bucket_off,
        const uint32_t* __restrict__ item_off, const ItemDesc* __restrict__ item_desc,
        const uint32_t* __restrict__ item_entries, uint32_t max_items,
        const uint32_t* __restrict__ lim, const uint8_t* __restrict__ sel,
        uint32_t* __restrict__ keys, ProbeRec* __restrict__ recs,
        unsigned long long* __restrict__ ftrace) {
    const unsigned long long ft0 = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // two code tiles (double buffer), row stride CSB bytes = (Y3 ? 4 : 2) * DB + 16
    __shared__ __attribute__((aligned(16))) uint8_t tiles[2 * BV * ((Y3 ? 4 : 2) * 16 * NS + 16)];
    __shared__ __attribute__((aligned(16))) float ynt[2][BV];  // row norm (L2) / bias (IP)
    __shared__ uint32_t ent_s[FQ];
    __shared__ int32_t qrow_s[FQ];
    __shared__ float bnd_s[FQ][4];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t xcd = blockIdx.x & 7u, rest = blockIdx.x >> 3;
    const uint32_t item = 4u * ((rest >> 2) * 8u + xcd) + (rest & 3u);
    // one round trip: the item count, the item's descriptor and its entries
    // (fixed stride FQ) are independent loads
    const uint32_t nitems = item_off[nlist];
    const uint32_t it = item < max_items ? item : 0u;
    const ItemDesc dsc = item_desc[it];
    const uint32_t e_raw = t < FQ ? item_entries[(size_t)it * FQ + t] : 0u;
    if (item >= nitems) return;
    const int l = (int)dsc.l;
    const int nQ = (int)dsc.nq;
    if (t < FQ) {
        const uint32_t e = t < nQ ? e_raw : 0u;
        ent_s[t] = e;
        qrow_s[t] = t < nQ ? (int32_t)(e / (uint32_t)nprobe) : -1;
    }
    const int len = (int)dsc.len;
    const int64_t row0 = dsc.off;
    constexpr int DB = 16 * NS;
    constexpr int CSB = (Y3 ? 4 : 2) * DB + 16;  // LDS row stride (bytes)
    constexpr int RU = (Y3 ? DB / 4 : DB / 8);   // uint4 staged per code row
    constexpr int PF = (BV * RU + 255) / 256;    // uint4 per thread per tile
    // wave w owns query columns 32w .. 32w + 31 and both 32-row halves bi of
    // every tile: thread (li, lh) keeps streams slot = 2 bi + lh of query qloc
    const int li = lane & 31, lh = lane >> 5;
    const int qloc = 32 * w + li;     // this thread's query (0..127)
    const bool active = 32 * w < nQ;  // wave-uniform
    const float* ynl = ynorm + row0;

    // ---- code tiles: global -> registers -> LDS (+ the tile's row norms)
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
                pf[s] = *(const uint4*)(cbf + (row0 + v0n + r) * (int64_t)(2 * DB) + 8 * c);
        }
        if (t < BV / 4) {
            const int r = 4 * t;
            // rows < roundup(len, 16) are inside the list's arena slot
            float4 v = r < nvn ? *(const float4*)(ynl + v0n + r) : make_float4(0.f, 0.f, 0.f, 0.f);
            if (!L2) v = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (HS) {
                // non-members of an IDSelector are treated as padding rows
                uchar4 ms = make_uchar4(1, 1, 1, 1);
                if (r < nvn) ms = *(const uchar4*)(sel + row0 + v0n + r);
                pn.x = r + 0 < nvn && ms.x ? v.x : WS_INF;
                pn.y = r + 1 < nvn && ms.y ? v.y : WS_INF;
                pn.z = r + 2 < nvn && ms.z ? v.z : WS_INF;
                pn.w = r + 3 < nvn && ms.w ? v.w : WS_INF;
            } else {
                pn.x = r + 0 < nvn ? v.x : WS_INF;
                pn.y = r + 1 < nvn ? v.y : WS_INF;
                pn.z = r + 2 < nvn ? v.z : WS_INF;
                pn.w = r + 3 < nvn ? v.w : WS_INF;
            }
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
    // the first tile's loads go out before the query fragments' (which wait
    // on the entries -> query rows chain)
    fetch(0);
    __syncthreads();

    const unsigned long long fta = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // ---- query fragments (B operand): registers for the whole work item
    bf16x8 bh[NS], bl[NS];
    float xn = 0.f;
    if (active) load_query_frags<NS>(x, ldx, d, qrow_s[qloc], lh, bh, bl, xn);
    const unsigned long long ftb = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    stash(0);
    if (BV < len) fetch(BV);
    __syncthreads();
    const unsigned long long ft1 = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;

    ThreadQueue32<KT> tq[2];
    tq[0].init();
    tq[1].init();
    const uint32_t lowmask = (1u << obits) - 1u;

    for (int v0 = 0, tile = 0; v0 < len; v0 += BV, tile++) {
        const int buf = tile & 1;
        // next tile into the other buffer (its readers finished before the
        // barrier that ended the previous iteration), then prefetch the one after
        if (v0 + BV < len) {
            stash(buf ^ 1);
            if (v0 + 2 * BV < len) fetch(v0 + 2 * BV);
        }
        if (active) {
            const uint32_t ordbase = (uint32_t)tile << 4;
#pragma unroll
            for (int bi = 0; bi < 2; bi++) {
                // norms / biases of this lane's 16 rows: 32bi + 4lh + 8g + (0..3)
                float4 yq[4];
#pragma unroll
                for (int g = 0; g < 4; g++)
                    yq[g] = *(const float4*)(&ynt[buf][32 * bi + 4 * lh + 8 * g]);
                const uint8_t* arow = tiles + buf * BV * CSB + (32 * bi + li) * CSB + 16 * lh;
                const floatx16 acc =
                        Y3 ? bf3_block<NS>(arow, bh, bl) : bf2_block<NS>(arow, bh, bl);
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int g = r >> 2, c = r & 3;
                    const float yv =
                            c == 0 ? yq[g].x : c == 1 ? yq[g].y : c == 2 ? yq[g].z : yq[g].w;
                    const float a = L2 ? fmaf(-2.f, acc[r], xn + yv) : yv - acc[r];
                    tq[bi].push(key_encode<L2>(a, lowmask, ordbase | (uint32_t)r));
                }
            }
        }
        __syncthreads();
    }

    // ---- outputs
    const unsigned long long ft2 = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const bool qvalid = qloc < nQ;
#pragma unroll
    for (int bi = 0; bi < 2; bi++) {
        const uint32_t last = tq[bi].q[KT - 1];
        float bnd = WS_INF;  // lower bound of every dropped candidate (none: +inf)
        if (last != 0xffffffffu) {
            const uint32_t ord = last & lowmask;
            const int r = (int)(ord & 15u);
            const int row =
                    (int)((ord >> 4) * BV) + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
            // a padding row in the last slot: every real row of this stream is kept
            if (row < len) bnd = key_decode_lo<L2>(last, lowmask);
        }
        bnd_s[qloc][2 * bi + lh] = bnd;
    }
    __syncthreads();
    if (qvalid) {
        // raw 32-bit keys (the re-rank decodes the approx bracket and the row)
        const int64_t e = ent_s[qloc];
        // max_codes: only a prefix of the list is scanned for this query
        const uint32_t elen = lim ? min((uint32_t)len, lim[e]) : (uint32_t)len;
#pragma unroll
        for (int bi = 0; bi < 2; bi++) {
            const int slot = 2 * bi + lh;
            uint32_t* ko = keys + e * (4 * KT) + slot * KT;
#pragma unroll
            for (int i = 0; i < KT; i++) {
                const uint32_t key = tq[bi].q[i];
                const uint32_t ord = key & lowmask;
                const int r = (int)(ord & 15u);
                const uint32_t row = (ord >> 4) * BV + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
                if constexpr (HS)
                    ko[i] = (key != 0xffffffffu && row < elen && sel[row0 + row]) ? key
                                                                                   : 0xffffffffu;
                else
                    ko[i] = (key != 0xffffffffu && row < elen) ? key : 0xffffffffu;
            }
        }
        if (lh == 0) {
            // the list's largest margin bounds every kept row's margin:
            // Y3: coef (x^2 + y^2); bf16x2: Cauchy-Schwarz on the code
            // rounding residual, 2 (2 |x| |y - yh| + coef (x^2 + y^2))
            const float mmax = Y3 ? coef * (xn + ynmax[l]) + 1e-30f
                                  : 2.f * (2.f * sqrtf(xn) * rmax[l] + coef * (xn + ynmax[l])) +
                                            1e-30f;
            ProbeRec pr;
#pragma unroll
            for (int sl = 0; sl < 4; sl++) {
                const float b = bnd_s[qloc][sl];
                pr.pb[sl] = b < WS_INF ? b - mmax : WS_INF;
            }
            pr.mmax = mmax;
            pr.off = (uint32_t)row0;
            pr.len = elen;
            pr.pad = 0u;
            recs[e] = pr;
        }
    }
    if (ftrace && t == 0) {
        ftrace[8 * item + 0] = ft0;
        ftrace[8 * item + 1] = ft1;
        ftrace[8 * item + 2] = ft2;
        ftrace[8 * item + 3] = __builtin_amdgcn_s_memrealtime();
        ftrace[8 * item + 4] = fta;
        ftrace[8 * item + 5] = ftb;
        ftrace[8 * item + 6] = (unsigned long long)len | ((unsigned long long)nQ << 32);
    }
}

// ---------------------------------------------------------------- A'
// The bf16x2 filter with its code tiles streamed global -> LDS by
// global_load_lds (no register staging) and one raw s_barrier per tile.  NB
// LDS tile buffers: NB = 2 (used: 35 KB, 4 work groups per CU) keeps tile
// j + 1 in flight while tile j is computed; NB = 3 (3 groups per CU, counted
// vmcnt waits) tile j + 2 — measured equal or slower on c2 (the loaded
// latency of the work item's first loads, not the tile stream, bounds it).
// Same work item, math, keys and records as k_ivf_bf3_filter (the re-rank
// reads them unchanged).
// Source: the "stream image" of the arena, one SR = 2 DB + 16 byte row per
// code: bf16(code) hi part, then the row's fp32 norm (+inf for padding rows)
// and 12 zero bytes (split_bf16_stream).  Lists are aligned to BV rows, so a
// tile never leaves its list: padding rows' keys sort after every real
// candidate and the epilogue drops them by row index.  The LDS image is the
// rows back to back (glds writes 1 KB blocks linearly); the 16-B tail makes
// the row stride 4 banks mod 64, so the 16 rows of a ds_read_b128 quarter
// hit distinct banks without a swizzle.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {  // s_waitcnt vmcnt(N) alone
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void wait_lgkmcnt0() {  // s_waitcnt lgkmcnt(0) alone
    __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
}

// FOLD (L2, fold image): the row and query norms enter the MFMA as a ninth
// k-step (A = the row's tail {-|y|^2/2 in three bf16 parts, 1, 1, 1, 0, 0},
// B = {1, 1, 1, -|x|^2/2 in three parts, 0, 0}; lanes lh = 1 multiply code
// bytes by zero), so the accumulator is -approx/2 and a candidate's key is
// min + bfi instead of add + fma + max + bfi, with no norm reads from LDS
// (fold_key_bits; margin coefficient ivf_bf2f_coef).
//
// PQ (IVF-PQ by residual, L2, with FOLD): the image is the PQ stream image
// (pq_stream_image: bf16 of each row's decoded residual y_R and the bias
// fragment of -term/2, term = |y_R|^2 + 2 <y_C, y_R>), the query's bias part
// is -coarse_dis(query, probe) / 2, so the accumulator is -approx / 2 of
// coarse_dis + term - 2 <x, y_R> (the IVF-PQ filter's key); ynmax / rmax are
// the lists' max |y_R| / |y_R - bf16(y_R)|, margins as k_ivfpq_filter_w.
template <bool L2, int KT, int NS, bool PIPE, bool FOLD = false, bool PQ = false>
__global__ __launch_bounds__(256, PIPE ? 3 : 4) void k_ivf_bf2_stream(
        const float* __restrict__ x, int ldx, int d, const uint8_t* __restrict__ cbs,
        const float* __restrict__ ynmax, const float* __restrict__ rmax, int nprobe, float coef,
        int obits, const uint32_t* __restrict__ item_off, const ItemDesc* __restrict__ item_desc,
        const uint32_t* __restrict__ item_entries, uint32_t max_items, int nlist,
        const uint32_t* __restrict__ lim, uint32_t* __restrict__ keys,
        ProbeRec* __restrict__ recs, unsigned long long* __restrict__ ftrace,
        const uint8_t* __restrict__ qimg, const float* __restrict__ qxn,
        const float* __restrict__ pcdis = nullptr, const float* __restrict__ pcnorm = nullptr) {
    static_assert(!PQ || (FOLD && L2 && !PIPE), "PQ: the folded L2 sequential form");
    const unsigned long long ft0 = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    constexpr int DB = 16 * NS;          // bf16 per code row
    constexpr int SR = 2 * DB + 16;      // bytes per stream-image row
    constexpr int TB = BV * SR;          // bytes per tile (a multiple of 1 KB)
    static_assert(TB % 1024 == 0, "tile = whole 1 KB glds blocks");
    constexpr int NG = TB / 1024;        // glds blocks per tile
    constexpr int G0 = (NG + 3) / 4;     // blocks of wave 0 (waves w: blocks w, w+4, ...)
    constexpr int G1 = (NG + 2) / 4;
    constexpr int G2 = (NG + 1) / 4;
    constexpr int G3 = NG / 4;
    constexpr int NB = 2;
    static_assert(FQ * 4 * 4 <= TB, "bounds fit in a tile buffer");
    static_assert(!(FOLD && (PIPE || !L2)), "fold: L2, sequential form");
    // all LDS in one array (a second __shared__ object can make hipcc wait
    // vmcnt(0) before the tile reads): 2 tiles; after the loop tile buffer 0
    // holds the bounds [FQ][4].
    __shared__ __attribute__((aligned(16))) uint8_t smem[NB * TB];
    uint8_t* tiles = smem;
    float* bnd_s = (float*)smem;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t xcd = blockIdx.x & 7u, rest = blockIdx.x >> 3;
    const uint32_t item = 4u * ((rest >> 2) * 8u + xcd) + (rest & 3u);
    const uint32_t nitems = item_off[nlist];
    const uint32_t it = item < max_items ? item : 0u;
    const ItemDesc dsc = item_desc[it];
    const int li = lane & 31, lh = lane >> 5;
    const int qloc = 32 * w + li;  // this thread's query (0..127)
    const uint32_t my_e = item_entries[(size_t)it * FQ + qloc];
    if (item >= nitems) return;
    const int l = (int)dsc.l;
    const int nQ = (int)dsc.nq;
    const int len = (int)dsc.len;
    const int64_t row0 = dsc.off;
    const int ntile = (len + BV - 1) / BV;
    const bool active = 32 * w < nQ;  // wave-uniform
    const bool qvalid = qloc < nQ;

    // glds of tile j into buffer b: the tile's rows are contiguous in the
    // stream image and in LDS; wave w copies 1 KB blocks w, w + 4, ...
    auto issue = [&](int j, int b) {
        const uint8_t* src = cbs + (row0 + (int64_t)j * BV) * SR + 16 * lane;
        uint8_t* dst = tiles + b * TB;
#pragma unroll
        for (int g = 0; g < G0; g++) {
            const int blk = w + 4 * g;
            if (g < G3 || blk < NG)  // wave-uniform
                __builtin_amdgcn_global_load_lds(
                        (const void*)(src + blk * 1024),
                        (__attribute__((address_space(3))) void*)(dst + blk * 1024), 16, 0, 0);
        }
    };
    // wait until at most `tiles_ahead` tiles of this wave's glds are pending
    auto wait_tiles = [&](int tiles_ahead) {
        if (NB == 2 || tiles_ahead == 0) {
            wait_vmcnt<0>();
        } else if (w == 0) {
            wait_vmcnt<G0>();
        } else if (w == 1) {
            wait_vmcnt<G1>();
        } else if (w == 2) {
            wait_vmcnt<G2>();
        } else {
            wait_vmcnt<G3>();
        }
    };
    issue(0, 0);
    if (NB == 3 && ntile > 1) issue(1, 1);
    // epilogue operands, loaded now (their latency hides under the loop)
    const float rmax_l = rmax[l], ynmax_l = ynmax[l];
    const float cnorm_l = PQ ? pcnorm[l] : 0.f;
    const float cd_e = PQ ? pcdis[qvalid ? my_e : 0u] : 0.f;
    const uint32_t lim_e = (lim && qvalid) ? lim[my_e] : 0xffffffffu;

    // query fragments (B operand): registers for the whole work item
    bf16x8 bh[NS], bl[NS];
    float xn = 0.f;
    if (active) {
        const int32_t qr = qvalid ? (int32_t)(my_e / (uint32_t)nprobe) : -1;
        if (qimg)  // fragments prepared once per query (k_query_prep)
            load_query_image<NS>(qimg, qxn, qr, lh, bh, bl, xn);
        else
            load_query_frags<NS>(x, ldx, d, qr, lh, bh, bl, xn);
    }
    // FOLD: the bias B fragment {1, 1, 1, -|x|^2/2 in three parts, 0, 0} (lh = 0)
    bf16x8 bq;
    if constexpr (FOLD) {
        __bf16 h, m, lo;
        split3_bf16(-0.5f * (PQ ? cd_e : xn), h, m, lo);
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
    const unsigned long long ft1 = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // the 16 norms of block bi of tile T: rows 32 bi + 4 lh + 8 g + c
    auto norms = [&](const uint8_t* T, int bi, float (&nv)[16]) {
        const uint8_t* nrow = T + (32 * bi + 4 * lh) * SR + 2 * DB;
#pragma unroll
        for (int r = 0; r < 16; r++) nv[r] = *(const float*)(nrow + (8 * (r >> 2) + (r & 3)) * SR);
    };
    auto push1 = [&](ThreadQueue32<KT>& pq, float accr, float yv0, uint32_t ord) {
        const float yv = L2 ? yv0 : (yv0 < WS_INF ? 0.f : WS_INF);  // IP: padding +inf
        const float a = L2 ? fmaf(-2.f, accr, xn + yv) : yv - accr;
        pq.push(key_insert(key_bits<L2>(a), lowmask, ord));
    };
    // MFMAs of block bi of tile T with the previous block's 16 pushes
    // interleaved between its k-steps (their VALU issues in this wave's MFMA
    // gaps instead of after the chain)
    auto mfma_push = [&](const uint8_t* T, int bi, const floatx16& pacc, const float (&pn)[16],
                         const uint8_t* pnT, uint32_t pord, ThreadQueue32<KT>& pq) {
        const uint8_t* arow = T + (32 * bi + li) * SR + 16 * lh;
        bf16x8 ah[NS];
#pragma unroll
        for (int s2 = 0; s2 < NS; s2++) ah[s2] = *(const bf16x8*)(arow + 32 * s2);
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < NS; s2++) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s2], bl[s2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s2], bh[s2], acc, 0, 0, 0);
#pragma unroll
            for (int r = 16 * s2 / NS; r < 16 * (s2 + 1) / NS; r++)
                push1(pq, pacc[r],
                      pnT ? *(const float*)(pnT + (8 * (r >> 2) + (r & 3)) * SR) : pn[r],
                      pord | (uint32_t)r);
        }
        return acc;
    };
    if constexpr (PIPE) {
        // software pipeline over blocks: phase A = MFMAs of (tile j, block 1)
        // + pushes of (j, 0); phase B = MFMAs of (j + 1, 0) + pushes of (j, 1).
        // A block's norms are read with its MFMAs (its buffer is refilled
        // before its pushes run).
        floatx16 acc0, acc1;
        float n1[16];
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // tile 0 (every wave's part)
        if (ntile > 1) issue(1, 1);
        if (active) {
            acc0 = bf2_block<NS>(tiles + li * SR + 16 * lh, bh, bl);
        }
        int b = 0;
        for (int j = 0; j < ntile; j++) {
            const uint8_t* T = tiles + b * TB;
            const uint32_t ordbase = (uint32_t)j << 4;
            if (active) {
                // (block 0's norms straight from LDS: tile j stays until the barrier)
                acc1 = mfma_push(T, 1, acc0, n1, T + 4 * lh * SR + 2 * DB, ordbase, tq[0]);
                norms(T, 1, n1);
            }
            if (j + 1 < ntile) {
                wait_vmcnt<0>();  // tile j + 1 (this wave's part)
                wait_lgkmcnt0();  // this wave's reads of tile j
                __builtin_amdgcn_s_barrier();  // tile j + 1 landed, tile j consumed
                if (j + 2 < ntile) issue(j + 2, b);
                const uint8_t* T1 = tiles + (b ^ 1) * TB;
                if (active) {
                    acc0 = mfma_push(T1, 0, acc1, n1, nullptr, ordbase, tq[1]);
                }
            } else if (active) {
#pragma unroll
                for (int r = 0; r < 16; r++) push1(tq[1], acc1[r], n1[r], ordbase | (uint32_t)r);
            }
            b ^= 1;
        }
    } else {
        int b = 0;  // buffer of tile j
        for (int j = 0; j < ntile; j++) {
            // tile j landed (this wave's part); with NB = 3 tile j + 1 may still
            // be in flight
            wait_tiles(j + 1 < ntile ? 1 : 0);
            __builtin_amdgcn_s_barrier();  // every wave's part; tile j - 1 consumed
            if (j + NB - 1 < ntile) issue(j + NB - 1, b == 0 ? NB - 1 : b - 1);  // tile j - 1's buffer


            if (active) {
                const uint32_t ordbase = (uint32_t)j << 4;
                const uint8_t* T = tiles + b * TB;
#pragma unroll
                for (int bi = 0; bi < 2; bi++) {
                    const uint8_t* arow = T + (32 * bi + li) * SR + 16 * lh;
                    bf16x8 ah[NS];
#pragma unroll
                    for (int s = 0; s < NS; s++) ah[s] = *(const bf16x8*)(arow + 32 * s);
                    floatx16 acc;
#pragma unroll
                    for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
                    for (int s = 0; s < NS; s++) {
                        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bl[s], acc, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bh[s], acc, 0, 0, 0);
                    }
                    if constexpr (FOLD) {
                        // the row's bias fragment (lh = 1: its code bytes, times 0)
                        const bf16x8 ab = *(const bf16x8*)(T + (32 * bi + li) * SR + (lh ? 0 : 2 * DB));
                        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bq, acc, 0, 0, 0);
                        mfma_read_guard();  // key_insert reads acc (inline asm)
#pragma unroll
                        for (int r = 0; r < 16; r++)
                            tq[bi].push(key_insert(fold_key_bits(acc[r]), lowmask, ordbase | (uint32_t)r));
                        __builtin_amdgcn_sched_barrier(0);
                        continue;
                    }
                    // this lane's 16 rows: 32 bi + 4 lh + 8 g + c (norm at byte 2 DB)
                    const uint8_t* nrow = T + (32 * bi + 4 * lh) * SR + 2 * DB;
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const int g = r >> 2, c = r & 3;
                        const float yv0 = *(const float*)(nrow + (8 * g + c) * SR);
                        // IP: bias 0 for real rows, +inf for padding
                        const float yv = L2 ? yv0 : (yv0 < WS_INF ? 0.f : WS_INF);
                        const float a = L2 ? fmaf(-2.f, acc[r], xn + yv) : yv - acc[r];
                        tq[bi].push(key_insert(key_bits<L2>(a), lowmask, ordbase | (uint32_t)r));
                    }
                    // keep the two blocks' live ranges apart (register pressure)
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            b = b == NB - 1 ? 0 : b + 1;
        }
    }

    const unsigned long long ft2 = ftrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // ---- outputs (no glds in flight: plain barriers from here)
    __syncthreads();  // every wave is done with the tiles: bounds reuse buffer 0
#pragma unroll
    for (int bi = 0; bi < 2; bi++) {
        const uint32_t last = tq[bi].q[KT - 1];
        float bnd = WS_INF;  // lower bound of every dropped candidate (none: +inf)
        if (last != 0xffffffffu) {
            const uint32_t ord = last & lowmask;
            const int r = (int)(ord & 15u);
            const int row = (int)((ord >> 4) * BV) + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
            if (row < len) bnd = FOLD ? fold_decode_lo(last, lowmask) : key_decode_lo<L2>(last, lowmask);
        }
        bnd_s[qloc * 4 + 2 * bi + lh] = bnd;
    }
    __syncthreads();
    if (qvalid) {
        const int64_t e = my_e;
        const uint32_t elen = min((uint32_t)len, lim_e);
#pragma unroll
        for (int bi = 0; bi < 2; bi++) {
            uint32_t* ko = keys + e * (4 * KT) + (2 * bi + lh) * KT;
#pragma unroll
            for (int i = 0; i < KT; i++) {
                const uint32_t key = tq[bi].q[i];
                const uint32_t ord = key & lowmask;
                const int r = (int)(ord & 15u);
                const uint32_t row = (ord >> 4) * BV + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
                ko[i] = (key != 0xffffffffu && row < elen) ? key : 0xffffffffu;
            }
        }
        if (lh == 0) {
            float mmax;
            if constexpr (PQ) {
                // 2 |x| r + coef (|x| + |y_C| + R)^2 (k_ivfpq_filter_w), doubled
                const float xl = sqrtf(xn);
                const float sr = xl + cnorm_l + ynmax_l;
                mmax = 2.f * (2.f * xl * rmax_l + coef * sr * sr) + 1e-30f;
            } else {
                mmax = 2.f * (2.f * sqrtf(xn) * rmax_l + coef * (xn + ynmax_l)) + 1e-30f;
            }
            ProbeRec pr;
#pragma unroll
            for (int sl = 0; sl < 4; sl++) {
                const float bb = bnd_s[qloc * 4 + sl];
                pr.pb[sl] = bb < WS_INF ? bb - mmax : WS_INF;
            }
            pr.mmax = mmax;
            pr.off = (uint32_t)row0;
            pr.len = elen;
            pr.pad = PQ ? (uint32_t)l : 0u;  // the PQ re-rank's list
            recs[e] = pr;
        }
    }
    if (ftrace && t == 0) {  // per-item timestamps (FAISS_AMD_FILTER_TRACE)
        ftrace[8 * item + 0] = ft0;
        ftrace[8 * item + 1] = ft1;
        ftrace[8 * item + 2] = ft2;
        ftrace[8 * item + 3] = __builtin_amdgcn_s_memrealtime();
        // HW_ID (wave, simd, cu, sh, se) and XCC_ID registers
        ftrace[8 * item + 4] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                               ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
        ftrace[8 * item + 5] = (unsigned long long)l;
        ftrace[8 * item + 6] = (unsigned long long)len | ((unsigned long long)nQ << 32);
    }
}

// stream image row r: bf16(code) for dims < d (zero beyond, DB dims), then
// the fp32 norm (+inf for padding rows, row_list == ~0) and 12 zero bytes
__global__ void k_split_stream(const float* __restrict__ codes, int64_t rows, int d, int ldc,
                               int DB, const float* __restrict__ ynorm,
                               const uint32_t* __restrict__ row_list, uint8_t* __restrict__ out,
                               int fold) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int per = DB + 8;  // bf16 slots per row (the last 8 = the 16-B tail)
    if (i >= rows * per) return;
    const int64_t r = i / per;
    const int j = (int)(i - r * per);
    uint8_t* row = out + r * (int64_t)(2 * DB + 16);
    if (j < DB) {
        const float v = j < d ? codes[r * ldc + j] : 0.f;
        ((__bf16*)row)[j] = (__bf16)v;
    } else if (fold) {
        // bias A-fragment {-|y|^2/2 in three bf16 parts, 1, 1, 1, 0, 0}
        const int t = j - DB;
        __bf16 v = (__bf16)0.f;
        if (t < 3) {
            __bf16 h = (__bf16)(-WS_INF), m = (__bf16)0.f, lo = (__bf16)0.f;
            if (row_list[r] != 0xffffffffu) split3_bf16(-0.5f * ynorm[r], h, m, lo);
            v = t == 0 ? h : t == 1 ? m : lo;
        } else if (t < 6) {
            v = (__bf16)1.f;
        }
        ((__bf16*)row)[j] = v;
    } else if (j == DB) {
        *(float*)(row + 2 * DB) = row_list[r] == 0xffffffffu ? WS_INF : ynorm[r];
    } else if (j > DB + 1) {
        ((uint16_t*)row)[DB + (j - DB)] = 0;  // bytes 2 DB + 4 .. 2 DB + 15
    }
}
void split_bf16_stream(const float* codes, int64_t rows, int d, int ldc, int DB,
                       const float* ynorm, const uint32_t* row_list, void* out, hipStream_t s,
                       int fold) {
    if (rows <= 0) return;
    const int64_t tot = rows * (DB + 8);
    k_split_stream<<<dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, s>>>(
            codes, rows, d, ldc, DB, ynorm, row_list, (uint8_t*)out, fold);
    HIP_LAUNCH_CHECK();
}

// PQ stream image row r (k_ivf_bf2_stream<..., PQ>): bf16 of the row's
// decoded residual y_R (dims < d; zero up to DB), then the bias A-fragment
// {-term/2 in three bf16 parts, 1, 1, 1, 0, 0} (padding rows: -inf, 0, 0, 1,
// 1, 1, 0, 0).  The decode is the reference's: y_R dims [m dsub, (m+1) dsub)
// = pq centroid codes[m] of sub-quantizer m (faiss/impl/ProductQuantizer.cpp
// decode).
__global__ void k_pq_stream_image(const uint8_t* __restrict__ codes, int cs, int64_t rows, int d,
                                  int dsub, const float* __restrict__ pq_cent,
                                  const float* __restrict__ terms,
                                  const uint32_t* __restrict__ row_list, int DB,
                                  uint8_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int per = DB + 8;
    if (i >= rows * per) return;
    const int64_t r = i / per;
    const int j = (int)(i - r * per);
    __bf16* row = (__bf16*)(out + r * (int64_t)(2 * DB + 16));
    const bool pad = row_list[r] == 0xffffffffu;
    if (j < DB) {
        float v = 0.f;
        if (j < d && !pad) {
            const int m = j / dsub;
            const int c = codes[r * cs + m];
            v = pq_cent[((int64_t)m * 256 + c) * dsub + (j - m * dsub)];
        }
        row[j] = (__bf16)v;
    } else {
        const int t = j - DB;
        __bf16 v = (__bf16)0.f;
        if (t < 3) {
            __bf16 h = (__bf16)(-WS_INF), m = (__bf16)0.f, lo = (__bf16)0.f;
            if (!pad) split3_bf16(-0.5f * terms[r], h, m, lo);
            v = t == 0 ? h : t == 1 ? m : lo;
        } else if (t < 6) {
            v = (__bf16)1.f;
        }
        row[j] = v;
    }
}
void pq_stream_image(const uint8_t* codes, int cs, int64_t rows, int d, int dsub,
                     const float* pq_cent, const float* terms, const uint32_t* row_list, int DB,
                     void* out, hipStream_t s) {
    if (rows <= 0) return;
    const int64_t tot = rows * (DB + 8);
    k_pq_stream_image<<<dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, s>>>(
            codes, cs, rows, d, dsub, pq_cent, terms, row_list, DB, (uint8_t*)out);
    HIP_LAUNCH_CHECK();
}

// IVF-PQ filter + bound records over the PQ stream image (the IVF-Flat
// streamed kernel in its PQ form): coarse_dis, |y_C| per list, list maxima of
// |y_R| and |y_R - bf16(y_R)|
bool ivfpq_stream_eligible(int d, int M, int k, int nprobe) {
    if (d % M != 0 || d > BDM || k > 32 || nprobe > kMaxNprobeFilter) return false;
    const int NS = bf3_db_host(d) / 2 * 2 / 16;
    return ivf_mfma_kq(k, d, nprobe) > 0 && (NS == 2 || NS == 4 || NS == 6 || NS == 8);
}
double ivfpq_fold_coef(int d, int M) {
    // k_ivfpq_filter_w's coefficient, plus the folded bias: the accumulator
    // sums 2 d exact products and 6 exact bias products whose magnitudes add
    // to <= (1 + 2^-8) |x| R + |term| / 2 + coarse_dis / 2 <= 0.51 S^2
    // (S = |x| + |y_C| + R; term = R^2 + 2 <y_C, y_R>, coarse_dis = |x -
    // y_C|^2), so its rounding is <= 0.51 (2 d + 6) u S^2, doubled by
    // approx = -2 acc
    const double u = 1.0 / 16777216.0;
    return ivfpq_mfma_coef(d, M) + 1.02 * (2.0 * d + 6.0) * u;
}
void ivfpq_stream_filter(const float* x, int ldx, int d, int M, const void* pcbs,
                         const float* cdis, const float* cnorm, const float* lrmax,
                         const float* lRmax, int nlist, int64_t n, int nprobe, int k, int obits,
                         const IVFBuckets& b, int64_t max_items, uint32_t* keys, ProbeRec* recs,
                         int* kt_out, hipStream_t s, const void* qimg, const float* qxn) {
    FAISS_THROW_IF_NOT(ivfpq_stream_eligible(d, M, k, nprobe));
    FAISS_THROW_IF_NOT_MSG(qimg && qxn, "ivfpq_stream_filter needs the prepared query image");
    FAISS_THROW_IF_NOT(!b.sel && obits >= 4 && obits <= 14);
    const int KE = ivf_mfma_kq(k, d, nprobe);
    *kt_out = KE / 4;
    const int NS = bf3_db_host(d) / 2 * 2 / 16;
    const int64_t grid = (int64_t)roundup((size_t)max_items, 32);
    FAISS_THROW_IF_NOT(grid < (1ll << 31));
    const float coef = (float)ivfpq_fold_coef(d, M);
#define PQS(KTV, NSV)                                                                         \
    k_ivf_bf2_stream<true, KTV, NSV, false, true, true><<<dim3((unsigned)grid), dim3(256), 0, s>>>( \
            x, ldx, d, (const uint8_t*)pcbs, lRmax, lrmax, nprobe, coef, obits, b.item_off,  \
            b.item_desc, b.item_entries, (uint32_t)max_items, nlist, b.lim, keys, recs,      \
            nullptr, (const uint8_t*)qimg, qxn, cdis, cnorm)
#define PQS_NS(KTV)                 \
    do {                            \
        if (NS == 2) PQS(KTV, 2);   \
        else if (NS == 4) PQS(KTV, 4); \
        else if (NS == 6) PQS(KTV, 6); \
        else PQS(KTV, 8);           \
    } while (0)
    if (KE == 8) PQS_NS(2);
    else if (KE == 16) PQS_NS(4);
    else PQS_NS(8);
#undef PQS_NS
#undef PQS
    HIP_LAUNCH_CHECK();
}

__global__ void k_pad_rows_inf(float* __restrict__ v, const uint32_t* __restrict__ row_list,
                               int64_t rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < rows && row_list[i] == 0xffffffffu) v[i] = WS_INF;
}
void pad_rows_inf(float* v, const uint32_t* row_list, int64_t rows, hipStream_t s) {
    if (rows <= 0) return;
    k_pad_rows_inf<<<dim3((unsigned)cdiv(rows, 256)), dim3(256), 0, s>>>(v, row_list, rows);
    HIP_LAUNCH_CHECK();
}

// per-list max row norm (margin of dropped candidates)
__global__ void k_list_max(const float* __restrict__ yn, const uint32_t* __restrict__ off,
                           const uint32_t* __restrict__ len, int nlist, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (l >= nlist) return;
    float m = 0.f;
    for (uint32_t i = lane; i < len[l]; i += 64) m = fmaxf(m, yn[off[l] + i]);
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s));
    if (lane == 0) out[l] = m;
}

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
        const float T = wave_kth_smallest<1>(lmv, k);
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
            U = wave_kth_smallest<1>(cv, k);
        } else {
            U = wave_kth_smallest<V>(ub, k);
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
            U = wave_kth_smallest<RRW_CB / 64>(v, k);
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

// ---------------------------------------------------------------- host
void ivf_list_ynmax(const float* yn, const uint32_t* list_off, const uint32_t* list_len,
                    int nlist, float* out, hipStream_t s) {
    if (nlist <= 0) return;
    k_list_max<<<dim3((unsigned)cdiv(nlist, 4)), dim3(256), 0, s>>>(yn, list_off, list_len,
                                                                    nlist, out);
    HIP_LAUNCH_CHECK();
}

int ivf_mfma_kq(int k, int dp, int nprobe) {
    // entries kept per (query, list) = 4 threads x KT.  A thread stream that
    // drops a key which may reach the top-k "fails" and is re-scanned whole by
    // the re-rank; with few probes the top-k crowds into the query's nearest
    // lists (c1: k = 10 over 8 probes), so nprobe < k keeps 8 per stream.
    // (c2 with 2 per stream: filter 105 -> 96 us, but 3.3 failing probes per
    // query take the re-rank from 55 to 347 us.)
    if (bf3_db(dp) > BDM || k > 32) return 0;
    const int kt = k <= 2 ? 2 : k <= 12 ? 4 : 8;
    return 4 * (nprobe > 0 && nprobe < k ? 8 : kt);
}

int ivf_bf3_obits(uint32_t max_list_len) {
    const uint32_t tiles = std::max<uint32_t>(1u, (max_list_len + BV - 1) / BV);
    int b = 0;
    while ((1u << b) < tiles) b++;
    return 4 + b;
}

double ivf_bf3_coef(int d) {
    const double u = 1.0 / 16777216.0;
    return 2.0 * (3.1 / 65536.0 + (6.0 * d + 8.0) * u);
}

// bf16x2: <x, y> - <xh + xl, yh> = <x, y - yh> + <xr, yh>: the first term is
// bounded by |x| |y - yh| (Cauchy-Schwarz, |y - yh| stored per row), the
// second by 2^-16 (1 + 2^-8) |x||y|; plus the f32 accumulation, norm and
// exact-side roundings.  This is the (x^2 + y^2) coefficient of that bound.
// bf16x3 with the norms folded into the MFMA accumulation (coarse fold image):
// 3 dp exact products and 6 exact bias products, |sum| <= 1.51 (|x|^2 +
// |y|^2); as ivf_bf2f_coef, twice the bound
double ivf_bf3f_coef(int d) {
    const double u = 1.0 / 16777216.0;
    return 2.0 * (3.1 / 65536.0 + (9.1 * d + 24.0) * u);
}

double ivf_bf2_coef(int d) {
    const double u = 1.0 / 16777216.0;
    return 1.02 / 65536.0 + (6.1 * d + 8.0) * u;
}
// bf16x2 with the norms folded into the MFMA accumulation (fold image): the
// accumulator sums 2 dp exact products and 6 exact bias products, |sum| <=
// 2 (1 + 2^-8) sum|x_i y_i| + (|x|^2 + |y|^2) / 2 <= 1.51 (|x|^2 + |y|^2), so
// its rounding is <= 1.51 (2 d + 6) u (|x|^2 + |y|^2), doubled by approx =
// -2 acc; plus the norms' own roundings and the exact side, as above.
double ivf_bf2f_coef(int d) {
    const double u = 1.0 / 16777216.0;
    return 1.02 / 65536.0 + (9.1 * d + 24.0) * u;
}

// |y - bf16(y)| per row (rounded up), the bf16x2 residual norms
__global__ void k_row_resnorm(const float* __restrict__ codes, int64_t rows, int d, int ldc,
                              float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    double s = 0.0;
    for (int j = 0; j < d; j++) {
        const float v = codes[r * ldc + j];
        const double e = (double)v - (double)(float)(__bf16)v;
        s += e * e;
    }
    out[r] = (float)(sqrt(s) * (1.0 + 1e-6)) + 1e-38f;
}

void row_resnorm_bf16(const float* codes, int64_t rows, int d, int ldc, float* out,
                      hipStream_t s) {
    if (rows <= 0) return;
    k_row_resnorm<<<dim3((unsigned)cdiv(rows, 256)), dim3(256), 0, s>>>(codes, rows, d, ldc, out);
    HIP_LAUNCH_CHECK();
}

void split_bf16(const float* codes, int64_t rows, int d, int ldc, int DB, void* out,
                hipStream_t s) {
    if (rows <= 0) return;
    const int64_t n = rows * DB;
    k_split_bf16<<<dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s>>>(codes, rows, d, ldc, DB,
                                                                    (__bf16*)out);
    HIP_LAUNCH_CHECK();
}

void ivf_flat_scan_mfma(const float* x, int ldx, const float* codes, int ldc, const void* cbf,
                        const int64_t* ids, const float* ynorm, const float* ynmax,
                        const float* rres, const float* rmax,
                        const uint32_t* list_off, const uint32_t* list_len, int nlist, int d,
                        int obits, int64_t n, int nprobe, int k, int metric_l2, IVFBuckets b,
                        int64_t max_items, uint32_t* keys, ProbeRec* recs, uint32_t* stats,
                        float* D, int64_t* I, KernelTimes* kt, hipStream_t s, int list_align,
                        const void* cbs, void* qscratch, bool qready,
                        unsigned long long* qdone, int fold) {
    if (n <= 0) return;
    const bool aligned_lists = list_align % BV == 0 && cbs != nullptr;
    const int KE = ivf_mfma_kq(k, d, nprobe);
    FAISS_THROW_IF_NOT(KE > 0);
    FAISS_THROW_IF_NOT(ldc % 4 == 0);
    FAISS_THROW_IF_NOT(nprobe <= kMaxNprobeFilter);
    FAISS_THROW_IF_NOT(obits >= 4 && obits <= 14);
    const int NS = bf3_db(d) / 16;
    const int64_t grid = (int64_t)roundup((size_t)max_items, 32);
    FAISS_THROW_IF_NOT(grid < (1ll << 31));
    const bool l2 = metric_l2 != 0;
    // precision of the filter: bf16x2 (default: half the code bytes, Cauchy-
    // Schwarz margins) or bf16x3 (FAISS_AMD_IVF_PREC=bf16x3: tighter margins,
    // fewer re-ranked candidates on data where bf16x2 keeps too many).  The
    // 32-bit keys' truncation (2^(obits-23) relative) is bracketed by the
    // decode (low bits cleared / set).
    const char* prec = getenv("FAISS_AMD_IVF_PREC");
    // bf16x3 only without a selector (the selector variant is built for the
    // bf16x2 filter; both give the certified exact result)
    const bool y3 = prec && !strcmp(prec, "bf16x3") && !b.sel;
    // FAISS_AMD_FILTER_TRACE=<file>: per-work-item timestamps (profiling)
    static unsigned long long* ftrace_buf = nullptr;
    static int64_t ftrace_n = 0;
    const char* ftr = getenv("FAISS_AMD_FILTER_TRACE");
    unsigned long long* ftrace = nullptr;
    if (ftr) {
        if (ftrace_n < grid) {
            if (ftrace_buf) HIP_CHECK(hipFree(ftrace_buf));
            HIP_CHECK(hipMalloc(&ftrace_buf, 64 * grid));
            ftrace_n = grid;
        }
        HIP_CHECK(hipMemsetAsync(ftrace_buf, 0, 64 * grid, s));
        ftrace = ftrace_buf;
    }
    // streamed (glds) bf16x2 filter: the default; the register-staged kernel
    // serves bf16x3, IDSelectors and the per-item trace
    // (FAISS_AMD_IVF_FILTER=staged forces it)
    const char* fenv = getenv("FAISS_AMD_IVF_FILTER");
    const bool stream_ok = aligned_lists && !y3 && !b.sel && d <= BDM &&
                           !(fenv && !strcmp(fenv, "staged"));
    // fold: the stream image carries bias fragments (L2 only); only the
    // streamed kernel reads the image, so folded keys exist only when it runs
    // (the staged kernel writes plain distance keys)
    const bool fk = fold != 0 && l2 && stream_ok;
    const float coef = (float)(y3 ? ivf_bf3_coef(d) : fk ? ivf_bf2f_coef(d) : ivf_bf2_coef(d));
    // the sequential form (4 groups per CU) by default: measured faster on c2
    // (112 vs 117 us) than the block-pipelined one (FAISS_AMD_IVF_PIPE=1, 3
    // groups per CU, MFMAs of one block interleaved with the previous block's
    // selection)
    const char* penv = getenv("FAISS_AMD_IVF_PIPE");
    const bool spipe = penv && !strcmp(penv, "1") && !fk;
    // the streamed filter reads prepared query fragments: one k_query_prep
    // launch instead of every work item splitting its queries' fp32 rows
    const uint8_t* qimg = nullptr;
    const float* qxn = nullptr;
    if (stream_ok && qscratch && ldx % 4 == 0) {
        qimg = (const uint8_t*)qscratch;
        qxn = (const float*)((uint8_t*)qscratch + query_image_bytes(n, d));
        if (!qready) query_prep(x, n, ldx, d, nullptr, qscratch, (float*)qxn, s);
    }
    {
        ScopedKernelTimer tm(kt, "ivf_flat_scan", 0.0, s);
#define LAUNCH_NS(L2V, KTV, NSV)                                                              \
    do {                                                                                      \
        if (stream_ok)                                                                        \
            (spipe ? k_ivf_bf2_stream<L2V, KTV, NSV, true>                                   \
             : fk  ? k_ivf_bf2_stream<L2V, KTV, NSV, false, L2V>                              \
                   : k_ivf_bf2_stream<L2V, KTV, NSV, false>)<<<dim3((unsigned)grid), dim3(256), 0, s>>>( \
                    x, ldx, d, (const uint8_t*)cbs, ynmax, rmax, nprobe, coef, obits,         \
                    b.item_off, b.item_desc, b.item_entries, (uint32_t)max_items, nlist,      \
                    b.lim, keys, recs, ftrace, qimg, qxn, nullptr, nullptr);                  \
        else if (b.sel)                                                                       \
            k_ivf_bf3_filter<L2V, KTV, NSV, false, true><<<dim3((unsigned)grid), dim3(256), 0, s>>>( \
                    x, ldx, d, (const __bf16*)cbf, ynorm, ynmax, rres, rmax, list_off,       \
                    list_len, nlist, nprobe, coef, obits, b.bucket_off, b.item_off,           \
                    b.item_desc, b.item_entries, (uint32_t)max_items, b.lim, b.sel, keys, recs, ftrace);    \
        else if (y3)                                                                          \
            k_ivf_bf3_filter<L2V, KTV, NSV, true, false><<<dim3((unsigned)grid), dim3(256), 0, s>>>( \
                    x, ldx, d, (const __bf16*)cbf, ynorm, ynmax, rres, rmax, list_off,       \
                    list_len, nlist, nprobe, coef, obits, b.bucket_off, b.item_off,           \
                    b.item_desc, b.item_entries, (uint32_t)max_items, b.lim, b.sel, keys, recs, ftrace);    \
        else                                                                                  \
            k_ivf_bf3_filter<L2V, KTV, NSV, false, false><<<dim3((unsigned)grid), dim3(256), 0, s>>>(\
                    x, ldx, d, (const __bf16*)cbf, ynorm, ynmax, rres, rmax, list_off,       \
                    list_len, nlist, nprobe, coef, obits, b.bucket_off, b.item_off,           \
                    b.item_desc, b.item_entries, (uint32_t)max_items, b.lim, b.sel, keys, recs, ftrace);    \
    } while (0)
#define LAUNCH_A(L2V, KTV)                     \
    do {                                       \
        if (NS == 2) LAUNCH_NS(L2V, KTV, 2);   \
        else if (NS == 4) LAUNCH_NS(L2V, KTV, 4); \
        else if (NS == 6) LAUNCH_NS(L2V, KTV, 6); \
        else LAUNCH_NS(L2V, KTV, 8);           \
    } while (0)
#define DISPATCH(M, L2V)                  \
    do {                                  \
        if (KE == 8) M(L2V, 2);           \
        else if (KE == 16) M(L2V, 4);     \
        else M(L2V, 8);                   \
    } while (0)
        if (l2) DISPATCH(LAUNCH_A, true);
        else DISPATCH(LAUNCH_A, false);
        HIP_LAUNCH_CHECK();
        // FAISS_AMD_IVF_DUMP=<file>: the raw filter keys [n][nprobe][KE] and
        // probe records [n][nprobe] of this call (debugging)
        if (const char* dmp = getenv("FAISS_AMD_IVF_DUMP")) {
            std::vector<uint32_t> hk((size_t)n * nprobe * KE);
            std::vector<ProbeRec> hr((size_t)n * nprobe);
            HIP_CHECK(hipMemcpyAsync(hk.data(), keys, 4 * hk.size(), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipMemcpyAsync(hr.data(), recs, sizeof(ProbeRec) * hr.size(),
                                     hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            const int SRB = 2 * bf3_db(d) + 16;  // stream-image row bytes
            std::vector<uint8_t> hi(cbs ? 4 * (size_t)SRB : 0);
            if (cbs) HIP_CHECK(hipMemcpy(hi.data(), cbs, hi.size(), hipMemcpyDeviceToHost));
            if (FILE* f = fopen(dmp, "wb")) {
                fwrite(hk.data(), 4, hk.size(), f);
                fwrite(hr.data(), sizeof(ProbeRec), hr.size(), f);
                fwrite(hi.data(), 1, hi.size(), f);
                fclose(f);
            }
        }
        if (ftrace) {
            std::vector<unsigned long long> h(8 * grid);
            HIP_CHECK(hipMemcpyAsync(h.data(), ftrace, 64 * grid, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            if (FILE* f = fopen(ftr, "wb")) {
                fwrite(h.data(), 64, grid, f);
                fclose(f);
            }
        }
    }
    {
        ScopedKernelTimer tm(kt, "ivf_rerank", 0.0, s);
        const int E = nprobe * KE;
        const int V = E <= 128 ? 2 : E <= 256 ? 4 : E <= 512 ? 8 : E <= 1024 ? 16 : 32;
        // FAISS_AMD_RERANK_TRACE=<file>: per-query wave timestamps (profiling)
        static unsigned long long* trace_buf = nullptr;
        static int64_t trace_n = 0;
        const char* tr = getenv("FAISS_AMD_RERANK_TRACE");
        unsigned long long* trace = nullptr;
        if (tr) {
            if (trace_n < n) {
                if (trace_buf) HIP_CHECK(hipFree(trace_buf));
                HIP_CHECK(hipMalloc(&trace_buf, 64 * n));
                trace_n = n;
            }
            trace = trace_buf;
        }
#define LAUNCH_B(L2V, VV)                                                                      \
    k_ivf_rerank<L2V, VV><<<dim3((unsigned)cdiv(n, RR_W)), dim3(64 * RR_W), 0, s>>>(           \
            keys, recs, x, ldx, codes, ldc, ids, d, n, nprobe, KE / 4, obits, k, D, I, stats,   \
            trace, PQArgs{}, b.sel, qdone, fk ? 1 : 0)
#define DISPATCH_V(L2V)                      \
    do {                                     \
        if (V == 2) LAUNCH_B(L2V, 2);        \
        else if (V == 4) LAUNCH_B(L2V, 4);   \
        else if (V == 8) LAUNCH_B(L2V, 8);   \
        else if (V == 16) LAUNCH_B(L2V, 16); \
        else LAUNCH_B(L2V, 32);              \
    } while (0)
#define LAUNCH_W(L2V, KEV)                                                                     \
    k_ivf_rerank_wide<L2V, KEV><<<dim3((unsigned)n), dim3(64), 0, s>>>(                          \
            keys, recs, x, ldx, codes, ldc, ids, d, n, nprobe, obits, k, D, I, stats, PQArgs{},  \
            b.sel, qdone, fk ? 1 : 0)
#define DISPATCH_W(L2V)                      \
    do {                                     \
        if (KE == 8) LAUNCH_W(L2V, 8);       \
        else if (KE == 16) LAUNCH_W(L2V, 16); \
        else LAUNCH_W(L2V, 32);              \
    } while (0)
        if (nprobe > 64) {  // probes walked in chunks of 64 (k_ivf_rerank_wide)
            if (l2) DISPATCH_W(true);
            else DISPATCH_W(false);
        } else if (l2) DISPATCH_V(true);
        else DISPATCH_V(false);
        HIP_LAUNCH_CHECK();
#undef DISPATCH_W
#undef LAUNCH_W
        if (trace) {
            std::vector<unsigned long long> h(8 * n);
            HIP_CHECK(hipMemcpyAsync(h.data(), trace, 64 * n, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            if (FILE* f = fopen(tr, "wb")) {
                fwrite(h.data(), 64, n, f);
                fclose(f);
            }
        }
#undef DISPATCH_V
#undef LAUNCH_A
#undef LAUNCH_NS
#undef LAUNCH_B
#undef DISPATCH
    }
}

// IVF-PQ re-rank: the Flat re-rank's certified candidate selection with the
// reference LUT arithmetic as the exact evaluator (pq_exact)
void ivfpq_rerank(const uint32_t* keys, const ProbeRec* recs, const float* x, int ldx, int d,
                  const int64_t* ids, const PQArgs& pa, int dsub, int64_t n, int nprobe, int KT,
                  int obits, int k, const uint8_t* sel, float* D, int64_t* I, uint32_t* stats,
                  hipStream_t s, unsigned long long* qdone, int fold) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT(d <= BDM && d % 4 == 0);
    const int KE = 4 * KT;
    const int E = nprobe * KE;
    const int V = E <= 128 ? 2 : E <= 256 ? 4 : E <= 512 ? 8 : E <= 1024 ? 16 : 32;
#define LAUNCH_P(VV, DS)                                                                        \
    k_ivf_rerank<true, VV, DS><<<dim3((unsigned)cdiv(n, RR_W)), dim3(64 * RR_W), 0, s>>>(       \
            keys, recs, x, ldx, nullptr, 0, ids, d, n, nprobe, KT, obits, k, D, I, stats,         \
            nullptr, pa, sel, qdone, fold)
#define DISPATCH_P(DS)                       \
    do {                                     \
        if (V == 2) LAUNCH_P(2, DS);         \
        else if (V == 4) LAUNCH_P(4, DS);    \
        else if (V == 8) LAUNCH_P(8, DS);    \
        else if (V == 16) LAUNCH_P(16, DS);  \
        else LAUNCH_P(32, DS);               \
    } while (0)
#define LAUNCH_PW(KEV, DS)                                                                     \
    k_ivf_rerank_wide<true, KEV, DS><<<dim3((unsigned)n), dim3(64), 0, s>>>(                     \
            keys, recs, x, ldx, nullptr, 0, ids, d, n, nprobe, obits, k, D, I, stats, pa, sel,  \
            qdone, fold)
#define DISPATCH_PW(DS)                       \
    do {                                      \
        if (KE == 8) LAUNCH_PW(8, DS);        \
        else if (KE == 16) LAUNCH_PW(16, DS); \
        else LAUNCH_PW(32, DS);               \
    } while (0)
    FAISS_THROW_IF_NOT(nprobe <= kMaxNprobeFilter);
    FAISS_THROW_IF_NOT_MSG(dsub == 2 || dsub == 4 || dsub == 8,
                           "ivfpq_rerank: dsub must be 2, 4 or 8");
    if (nprobe > 64) {  // probes walked in chunks of 64 (k_ivf_rerank_wide)
        if (dsub == 2) DISPATCH_PW(2);
        else if (dsub == 4) DISPATCH_PW(4);
        else DISPATCH_PW(8);
    } else if (dsub == 2) DISPATCH_P(2);
    else if (dsub == 4) DISPATCH_P(4);
    else DISPATCH_P(8);
    HIP_LAUNCH_CHECK();
#undef DISPATCH_PW
#undef LAUNCH_PW
#undef DISPATCH_P
#undef LAUNCH_P
}

}  // namespace kern
}  // namespace faiss_amd
