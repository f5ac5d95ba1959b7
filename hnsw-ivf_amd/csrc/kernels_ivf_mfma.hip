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
    GRID_STRIDE(i, rows * DB) {
        const int64_t r = i / DB;
        const int j = (int)(i - r * DB);
        const float v = j < d ? codes[r * ldc + j] : 0.f;
        const __bf16 h = (__bf16)v;
        out[r * 2 * DB + j] = h;
        out[r * 2 * DB + DB + j] = (__bf16)(v - (float)h);
    }
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
// cache policy of the tile stream's global_load_lds: 2 = nt (streamed list
// tiles are read once per item; marked non-temporal they leave the L2 to
// what is re-read: the query fragments and the re-rank's rows).  r05 A/B on
// c2: step 0.2867 -> 0.2786 ms (filter 100.9 -> 100.2 us, Flat re-rank 58.0
// -> 54.5 us); 0 = the default policy
#ifndef IVF_TILE_AUX
#define IVF_TILE_AUX 2
#endif
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
    static_assert(!(FOLD && (PIPE || !L2)), "fold: L2, sequential form");
    // all LDS in one array (a second __shared__ object can make hipcc wait
    // vmcnt(0) before the tile reads): the 2 tile buffers
    __shared__ __attribute__((aligned(16))) uint8_t smem[NB * TB];
    uint8_t* tiles = smem;
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
                        (__attribute__((address_space(3))) void*)(dst + blk * 1024), 16, 0,
                        IVF_TILE_AUX);
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
    // ---- outputs.  A query's 4 thread streams (slot 2 bi + lh) live in
    // lanes li and li + 32 of one wave, so their dropped bounds meet by one
    // lane swap (r05: no LDS round trip, no work-group barriers)
    float bnd2[2];
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
        bnd2[bi] = bnd;
    }
    const float bnd_p0 = __shfl_xor(bnd2[0], 32), bnd_p1 = __shfl_xor(bnd2[1], 32);
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
            const float bb4[4] = {bnd2[0], bnd_p0, bnd2[1], bnd_p1};  // slots 0..3
#pragma unroll
            for (int sl = 0; sl < 4; sl++)
                pr.pb[sl] = bb4[sl] < WS_INF ? bb4[sl] - mmax : WS_INF;
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
    const int per = DB + 8;  // bf16 slots per row (the last 8 = the 16-B tail)
    GRID_STRIDE(i, rows * per) {
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
}
void split_bf16_stream(const float* codes, int64_t rows, int d, int ldc, int DB,
                       const float* ynorm, const uint32_t* row_list, void* out, hipStream_t s,
                       int fold) {
    if (rows <= 0) return;
    k_split_stream<<<stride_grid(rows * (DB + 8), 256), dim3(256), 0, s>>>(
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
    const int per = DB + 8;
    GRID_STRIDE(i, rows * per) {
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
}
void pq_stream_image(const uint8_t* codes, int cs, int64_t rows, int d, int dsub,
                     const float* pq_cent, const float* terms, const uint32_t* row_list, int DB,
                     void* out, hipStream_t s) {
    if (rows <= 0) return;
    k_pq_stream_image<<<stride_grid(rows * (DB + 8), 256), dim3(256), 0, s>>>(
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
    k_ivf_bf2_stream<true, KTV, NSV, false, true, true><<<kgrid(grid, 256), dim3(256), 0, s>>>( \
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
    k_pad_rows_inf<<<kgrid(cdiv(rows, 256), 256), dim3(256), 0, s>>>(v, row_list, rows);
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

// ---------------------------------------------------------------- host
void ivf_list_ynmax(const float* yn, const uint32_t* list_off, const uint32_t* list_len,
                    int nlist, float* out, hipStream_t s) {
    if (nlist <= 0) return;
    k_list_max<<<kgrid(cdiv(nlist, 4), 256), dim3(256), 0, s>>>(yn, list_off, list_len,
                                                                    nlist, out);
    HIP_LAUNCH_CHECK();
}

int ivf_mfma_kq(int k, int dp, int nprobe, int kt_min) {
    // entries kept per (query, list) = 4 threads x KT.  A thread stream that
    // drops a key which may reach the top-k "fails" and is re-scanned whole by
    // the re-rank; with few probes the top-k crowds into the query's nearest
    // lists (c1: k = 10 over 8 probes), so nprobe < k keeps 8 per stream.
    // (c2 with 2 per stream: filter 105 -> 96 us, but 3.3 failing probes per
    // query take the re-rank from 55 to 347 us.)
    if (bf3_db(dp) > BDM || k > 32) return 0;
    int kt = k <= 2 ? 2 : k <= 12 ? 4 : 8;
    if (kt_min == 2 || kt_min == 4 || kt_min == 8) kt = std::max(kt, kt_min);
    // FAISS_AMD_IVF_KT=2|4|8: at least that many (tuning; same results)
    if (const char* e = getenv("FAISS_AMD_IVF_KT")) {
        const int v = atoi(e);
        if (v == 2 || v == 4 || v == 8) kt = std::max(kt, v);
    }
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
    k_row_resnorm<<<kgrid(cdiv(rows, 256), 256), dim3(256), 0, s>>>(codes, rows, d, ldc, out);
    HIP_LAUNCH_CHECK();
}

void split_bf16(const float* codes, int64_t rows, int d, int ldc, int DB, void* out,
                hipStream_t s) {
    if (rows <= 0) return;
    k_split_bf16<<<stride_grid(rows * DB, 256), dim3(256), 0, s>>>(codes, rows, d, ldc, DB,
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
                        unsigned long long* qdone, int fold, int kt_min) {
    if (n <= 0) return;
    const bool aligned_lists = list_align % BV == 0 && cbs != nullptr;
    const int KE = ivf_mfma_kq(k, d, nprobe, kt_min);
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
                   : k_ivf_bf2_stream<L2V, KTV, NSV, false>)<<<kgrid(grid, 256), dim3(256), 0, s>>>( \
                    x, ldx, d, (const uint8_t*)cbs, ynmax, rmax, nprobe, coef, obits,         \
                    b.item_off, b.item_desc, b.item_entries, (uint32_t)max_items, nlist,      \
                    b.lim, keys, recs, ftrace, qimg, qxn, nullptr, nullptr);                  \
        else if (b.sel)                                                                       \
            k_ivf_bf3_filter<L2V, KTV, NSV, false, true><<<kgrid(grid, 256), dim3(256), 0, s>>>( \
                    x, ldx, d, (const __bf16*)cbf, ynorm, ynmax, rres, rmax, list_off,       \
                    list_len, nlist, nprobe, coef, obits, b.bucket_off, b.item_off,           \
                    b.item_desc, b.item_entries, (uint32_t)max_items, b.lim, b.sel, keys, recs, ftrace);    \
        else if (y3)                                                                          \
            k_ivf_bf3_filter<L2V, KTV, NSV, true, false><<<kgrid(grid, 256), dim3(256), 0, s>>>( \
                    x, ldx, d, (const __bf16*)cbf, ynorm, ynmax, rres, rmax, list_off,       \
                    list_len, nlist, nprobe, coef, obits, b.bucket_off, b.item_off,           \
                    b.item_desc, b.item_entries, (uint32_t)max_items, b.lim, b.sel, keys, recs, ftrace);    \
        else                                                                                  \
            k_ivf_bf3_filter<L2V, KTV, NSV, false, false><<<kgrid(grid, 256), dim3(256), 0, s>>>(\
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
    ivf_flat_rerank(keys, recs, x, ldx, codes, ldc, ids, d, n, nprobe, KE, obits, k, metric_l2,
                    b.sel, stats, D, I, kt, s, qdone, fk ? 1 : 0);
#undef LAUNCH_A
#undef LAUNCH_NS
#undef DISPATCH
}

}  // namespace kern
}  // namespace faiss_amd
