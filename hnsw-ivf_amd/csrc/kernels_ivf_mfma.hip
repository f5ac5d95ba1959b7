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
//  C  k_ivf_exact_fallback: exact scan of the flagged queries only.
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

#include "common.h"
#include "kernels.h"
#include "wave_select.h"
#include "exact_select.h"
#include "ref_arith.h"
#include "bf3.h"

namespace faiss_amd {
namespace kern {


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
//   part[e][i] = ordered_f32(lb) << 32 | row   (~0 = empty)
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
template <bool L2, int KT, int NS, bool Y3>
__global__ __launch_bounds__(256, Y3 ? 2 : 3) void k_ivf_bf3_filter(
        const float* __restrict__ x, int ldx, int d, const __bf16* __restrict__ cbf,
        const float* __restrict__ ynorm, const float* __restrict__ ynmax,
        const float* __restrict__ rres, const float* __restrict__ rmax,
        const uint32_t* __restrict__ list_off, const uint32_t* __restrict__ list_len, int nlist,
        int nprobe, float coef, int obits, const uint32_t* __restrict__ bucket_off,
        const uint32_t* __restrict__ item_off, const uint32_t* __restrict__ entries,
        unsigned long long* __restrict__ part, float* __restrict__ pub,
        float* __restrict__ pbound) {
    // two code tiles (double buffer), row stride CSB bytes = (Y3 ? 4 : 2) * DB + 16
    __shared__ __attribute__((aligned(16))) uint8_t tiles[2 * BV * ((Y3 ? 4 : 2) * 16 * NS + 16)];
    __shared__ __attribute__((aligned(16))) float ynt[2][BV];  // row norm (L2) / bias (IP)
    __shared__ uint32_t ent_s[BQ];
    __shared__ int32_t qrow_s[BQ];
    __shared__ float bnd_s[BQ][4];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t xcd = blockIdx.x & 7u, rest = blockIdx.x >> 3;
    const uint32_t item = 4u * ((rest >> 2) * 8u + xcd) + (rest & 3u);
    if (item >= item_off[nlist]) return;
    int lo = 0, hi = nlist;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (item_off[mid] <= item) lo = mid; else hi = mid;
    }
    const int l = lo;
    const uint32_t qb = bucket_off[l] + (item - item_off[l]) * BQ;
    const int nQ = (int)min((uint32_t)BQ, bucket_off[l + 1] - qb);
    if (t < BQ) {
        const uint32_t e = t < nQ ? entries[qb + t] : 0u;
        ent_s[t] = e;
        qrow_s[t] = t < nQ ? (int32_t)(e / (uint32_t)nprobe) : -1;
    }
    const int len = (int)list_len[l];
    const int64_t row0 = list_off[l];
    constexpr int DB = 16 * NS;
    constexpr int CSB = (Y3 ? 4 : 2) * DB + 16;  // LDS row stride (bytes)
    constexpr int RU = (Y3 ? DB / 4 : DB / 8);   // uint4 staged per code row
    constexpr int PF = (BV * RU + 255) / 256;    // uint4 per thread per tile
    const int bi = w >> 1, bj = w & 1;
    const int li = lane & 31, lh = lane >> 5;
    const int slot = 2 * bi + lh;    // this thread's share of its query's codes
    const int qloc = 32 * bj + li;   // this thread's query (0..63)
    const bool active = 32 * bj < nQ;  // wave-uniform
    const float* ynl = ynorm + row0;
    __syncthreads();

    // ---- query fragments (B operand): registers for the whole work item
    bf16x8 bh[NS], bl[NS];
    float xn = 0.f;
    if (active) load_query_frags<NS>(x, ldx, d, qrow_s[qloc], lh, bh, bl, xn);

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
            pn.x = r + 0 < nvn ? v.x : WS_INF;
            pn.y = r + 1 < nvn ? v.y : WS_INF;
            pn.z = r + 2 < nvn ? v.z : WS_INF;
            pn.w = r + 3 < nvn ? v.w : WS_INF;
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
        // next tile into the other buffer (its readers finished before the
        // barrier that ended the previous iteration), then prefetch the one after
        if (v0 + BV < len) {
            stash(buf ^ 1);
            if (v0 + 2 * BV < len) fetch(v0 + 2 * BV);
        }
        if (active) {
            // norms / biases of this lane's 16 rows: 32bi + 4lh + 8g + (0..3)
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
                const float a = L2 ? fmaf(-2.f, acc[r], xn + yv) : yv - acc[r];
                tq.push(key_encode<L2>(a, lowmask, ordbase | (uint32_t)r));
            }
        }
        __syncthreads();
    }

    // ---- outputs
    const bool qvalid = qloc < nQ;
    const uint32_t last = tq.q[KT - 1];
    float bnd = WS_INF;  // lower bound of every dropped candidate (none: +inf)
    if (last != 0xffffffffu) {
        const uint32_t ord = last & lowmask;
        const int r = (int)(ord & 15u);
        const int row = (int)((ord >> 4) * BV) + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
        // a padding row in the last slot: every real row of this stream is kept
        if (row < len) bnd = key_decode_lo<L2>(last, lowmask);
    }
    bnd_s[qloc][slot] = bnd;
    __syncthreads();
    if (qvalid) {
        const int64_t e = ent_s[qloc];
        unsigned long long* po = part + e * (4 * KT) + slot * KT;
        float* pu = pub + e * (4 * KT) + slot * KT;
#pragma unroll
        for (int i = 0; i < KT; i++) {
            const uint32_t key = tq.q[i];
            const uint32_t ord = key & lowmask;
            const int r = (int)(ord & 15u);
            const uint32_t row = (ord >> 4) * BV + 32 * bi + 4 * lh + 8 * (r >> 2) + (r & 3);
            if (key != 0xffffffffu && row < (uint32_t)len) {
                // Y3: coef (x^2 + y^2); bf16x2: Cauchy-Schwarz on the code
                // rounding residual, 2 (2 |x| |y - yh| + coef (x^2 + y^2))
                const float m = Y3 ? coef * (xn + ynl[row]) + 1e-30f
                                   : 2.f * (2.f * sqrtf(xn) * rres[row0 + row] +
                                            coef * (xn + ynl[row])) + 1e-30f;
                const float alo = key_decode_lo<L2>(key, lowmask);
                const float ahi = key_decode_hi<L2>(key, lowmask);
                po[i] = ((unsigned long long)ordered_f32(alo - m) << 32) | row;
                pu[i] = ahi + m;
            } else {
                po[i] = ~0ull;
                pu[i] = WS_INF;
            }
        }
        if (slot == 0) {
            const float b4 = fminf(fminf(bnd_s[qloc][0], bnd_s[qloc][1]),
                                   fminf(bnd_s[qloc][2], bnd_s[qloc][3]));
            const float mmax = Y3 ? coef * (xn + ynmax[l]) + 1e-30f
                                  : 2.f * (2.f * sqrtf(xn) * rmax[l] + coef * (xn + ynmax[l])) +
                                            1e-30f;
            pbound[e] = b4 < WS_INF ? b4 - mmax : WS_INF;
        }
    }
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
// Latency layout: lane r < nprobe holds probe r's list (offset, length,
// dropped bound); the kept entries' upper bounds are loaded V per lane in one
// round trip; U comes from a ballot radix select (no shuffles); survivors are
// compacted to LDS as global arena rows.
constexpr int RR_CAP = 512;

template <bool L2>
struct RerankStream {
    const uint32_t* surv;  // global arena rows of the survivors
    const uint16_t* sprobe;  // their probe rank
    const int64_t* ids;
    const float* xq;
    const float* codes;
    int ldc, d, lane, nsv;
    // overflow mode: re-scan the survivor predicate from global memory
    bool overflow;
    const unsigned long long* part;
    int E, KE;
    float U;
    unsigned long long okmask, fmask;
    uint32_t my_off, my_len;  // lane r: probe r

    __device__ __forceinline__ uint32_t off_of(int r) const { return __shfl(my_off, r); }
    __device__ __forceinline__ void eval_row(int r, uint32_t grow, uint32_t rank_row, float& k1,
                                             long long& k2, long long& rank) const {
        const float* yr = codes + (int64_t)grow * ldc;
        const float dis = L2 ? ref_l2(xq, yr, d) : ref_ip(xq, yr, d);
        to_key(L2 ? 1 : 0, dis, (long long)ids[grow], k1, k2);
        rank = ((long long)r << 32) | rank_row;
    }
    template <class F>
    __device__ __forceinline__ void for_each(F f) const {
        if (!overflow) {
            for (int s0 = 0; s0 < nsv; s0 += 64) {
                float k1 = WS_INF;
                long long k2 = WS_NOID, rank = 0;
                bool ok = s0 + lane < nsv;
                if (ok) {
                    const uint32_t grow = surv[s0 + lane];
                    const int r = sprobe[s0 + lane];
                    eval_row(r, grow, grow, k1, k2, rank);
                    ok = key_admissible(k1);
                }
                f(ok, k1, k2, rank);
            }
        } else {
            for (int c0 = 0; c0 < E; c0 += 64) {
                const int c = c0 + lane;
                const int r = c / KE;
                const uint32_t roff = off_of(r < 64 ? r : 0);
                float k1 = WS_INF;
                long long k2 = WS_NOID, rank = 0;
                bool ok = false;
                if (c < E && ((okmask >> r) & 1ull) && !((fmask >> r) & 1ull)) {
                    const unsigned long long key = part[c];
                    ok = key != ~0ull && unordered_f32((uint32_t)(key >> 32)) <= U;
                    if (ok) {
                        eval_row(r, roff + (uint32_t)key, roff + (uint32_t)key, k1, k2, rank);
                        ok = key_admissible(k1);
                    }
                }
                if (__ballot(ok) == 0ull) continue;
                f(ok, k1, k2, rank);
            }
        }
        // every row of the failing probes (rank = list row; the arena row
        // order within a list is the list order)
        unsigned long long m = fmask;
        while (m) {
            const int r = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const uint32_t o = off_of(r), len = __shfl(my_len, r);
            for (uint32_t v0 = 0; v0 < len; v0 += 64) {
                float k1 = WS_INF;
                long long k2 = WS_NOID, rank = 0;
                bool ok = v0 + lane < len;
                if (ok) {
                    eval_row(r, o + v0 + lane, o + v0 + lane, k1, k2, rank);
                    ok = key_admissible(k1);
                }
                f(ok, k1, k2, rank);
            }
        }
    }
};

template <bool L2, int V>
__global__ __launch_bounds__(256) void k_ivf_rerank(
        const unsigned long long* __restrict__ part, const float* __restrict__ pub,
        const float* __restrict__ pbound, const int32_t* __restrict__ assign,
        const uint32_t* __restrict__ list_off, const uint32_t* __restrict__ list_len, int nlist,
        const float* __restrict__ x, int ldx, const float* __restrict__ codes, int ldc,
        const int64_t* __restrict__ ids, int d, int64_t n, int nprobe, int KE, int k,
        float* __restrict__ D, int64_t* __restrict__ I, uint32_t* __restrict__ stats) {
    __shared__ uint32_t surv[4][RR_CAP];
    __shared__ uint16_t sprobe[4][RR_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q0 = (int64_t)blockIdx.x * 4 + w;
    const bool valid = q0 < n;
    const int64_t q = valid ? q0 : 0;
    const int E = valid ? nprobe * KE : 0;
    // per-probe state, lane r = probe r
    uint32_t my_off = 0, my_len = 0;
    float my_pb = WS_INF;
    bool my_ok = false;
    if (valid && lane < nprobe) {
        const int lst = assign[q * nprobe + lane];
        if (lst >= 0 && lst < nlist) {
            my_len = list_len[lst];
            my_off = list_off[lst];
            my_ok = my_len > 0;
            if (my_ok) my_pb = pbound[q * nprobe + lane];
        }
    }
    const unsigned long long okmask = __ballot(my_ok);
    // upper bounds, V per lane, one round trip
    const float* pu = pub + q * (int64_t)nprobe * KE;
    float ub[V];
#pragma unroll
    for (int i = 0; i < V; i++) {
        const int c = i * 64 + lane;
        ub[i] = (c < E && ((okmask >> (c / KE)) & 1ull)) ? pu[c] : WS_INF;
    }
    float U = wave_kth_smallest<V>(ub, k);
    if (!(U <= WS_INF)) U = WS_INF;  // NaN guard
    const unsigned long long fmask = __ballot(my_ok && my_pb < WS_INF && my_pb <= U);
    // survivors -> LDS (global arena row + probe rank)
    const unsigned long long* pp = part + q * (int64_t)nprobe * KE;
    int ns = 0;
#pragma unroll
    for (int i = 0; i < V; i++) {
        const int c = i * 64 + lane;
        const int r = c / KE;
        const uint32_t roff = __shfl(my_off, r < 64 ? r : 0);
        bool sv = false;
        uint32_t grow = 0;
        if (ub[i] < WS_INF && !((fmask >> r) & 1ull)) {
            const unsigned long long key = pp[c];
            sv = key != ~0ull && unordered_f32((uint32_t)(key >> 32)) <= U;
            grow = roff + (uint32_t)key;
        }
        const unsigned long long m = __ballot(sv);
        const int pos = ns + __popcll(m & ((1ull << lane) - 1ull));
        if (sv && pos < RR_CAP) {
            surv[w][pos] = grow;
            sprobe[w][pos] = (uint16_t)r;
        }
        ns += __popcll(m);
    }
    RerankStream<L2> st;
    st.surv = surv[w];
    st.sprobe = sprobe[w];
    st.ids = ids;
    st.xq = x + q * ldx;
    st.codes = codes;
    st.ldc = ldc;
    st.d = d;
    st.lane = lane;
    st.nsv = ns;
    st.overflow = ns > RR_CAP;
    st.part = pp;
    st.E = E;
    st.KE = KE;
    st.U = U;
    st.okmask = okmask;
    st.fmask = fmask;
    st.my_off = my_off;
    st.my_len = my_len;
    exact_topk_resolve(st, k, L2 ? 1 : 0, lane, valid, D + q * k, I + q * k);
    if (stats && valid && lane == 0) {
        atomicAdd(&stats[0], (uint32_t)min(ns, RR_CAP));
        atomicAdd(&stats[1], (uint32_t)__popcll(fmask));
        atomicAdd(&stats[2], st.overflow ? 1u : 0u);
    }
}

// ---------------------------------------------------------------- C
// Exact re-scan of flagged queries: every row of every probed list.
template <bool L2>
struct FullStream {
    const int32_t* asg;
    const uint32_t* list_off;
    const uint32_t* list_len;
    int nlist, nprobe, d, ldc, lane;
    const float* xq;
    const float* codes;
    const int64_t* ids;
    template <class F>
    __device__ __forceinline__ void for_each(F f) const {
        for (int r = 0; r < nprobe; r++) {
            const int lst = asg[r];
            if (lst < 0 || lst >= nlist) continue;
            const int len = (int)list_len[lst];
            for (int v0 = 0; v0 < len; v0 += 64) {
                float k1 = WS_INF;
                long long k2 = WS_NOID, rank = 0;
                bool ok = v0 + lane < len;
                if (ok) {
                    const int64_t grow = (int64_t)list_off[lst] + v0 + lane;
                    const float* yr = codes + grow * ldc;
                    const float dis = L2 ? ref_l2(xq, yr, d) : ref_ip(xq, yr, d);
                    to_key(L2 ? 1 : 0, dis, (long long)ids[grow], k1, k2);
                    ok = key_admissible(k1);
                    rank = ((long long)r << 32) | (uint32_t)(v0 + lane);
                }
                f(ok, k1, k2, rank);
            }
        }
    }
};

template <bool L2>
__global__ __launch_bounds__(64) void k_ivf_exact_fallback(
        const uint32_t* __restrict__ flags, const int32_t* __restrict__ assign,
        const uint32_t* __restrict__ list_off, const uint32_t* __restrict__ list_len, int nlist,
        const float* __restrict__ x, int ldx, const float* __restrict__ codes, int ldc,
        const int64_t* __restrict__ ids, int d, int nprobe, int k, float* __restrict__ D,
        int64_t* __restrict__ I) {
    const int64_t q = blockIdx.x;
    if (flags[q] == 0u) return;
    FullStream<L2> st{assign + q * nprobe, list_off, list_len, nlist, nprobe, d, ldc,
                      (int)threadIdx.x, x + q * ldx, codes, ids};
    exact_topk_resolve(st, k, L2 ? 1 : 0, (int)threadIdx.x, true, D + q * k, I + q * k);
}

void ivf_exact_fallback(const uint32_t* flags, const int32_t* assign, const uint32_t* list_off,
                        const uint32_t* list_len, int nlist, const float* x, int ldx,
                        const float* codes, int ldc, const int64_t* ids, int d, int64_t n,
                        int nprobe, int k, int metric_l2, float* D, int64_t* I, hipStream_t s) {
    if (n <= 0) return;
    if (metric_l2)
        k_ivf_exact_fallback<true><<<dim3((unsigned)n), dim3(64), 0, s>>>(
                flags, assign, list_off, list_len, nlist, x, ldx, codes, ldc, ids, d, nprobe, k,
                D, I);
    else
        k_ivf_exact_fallback<false><<<dim3((unsigned)n), dim3(64), 0, s>>>(
                flags, assign, list_off, list_len, nlist, x, ldx, codes, ldc, ids, d, nprobe, k,
                D, I);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- host
void ivf_list_ynmax(const float* yn, const uint32_t* list_off, const uint32_t* list_len,
                    int nlist, float* out, hipStream_t s) {
    if (nlist <= 0) return;
    k_list_max<<<dim3((unsigned)cdiv(nlist, 4)), dim3(256), 0, s>>>(yn, list_off, list_len,
                                                                    nlist, out);
    HIP_LAUNCH_CHECK();
}

int ivf_mfma_kq(int k, int dp) {
    // entries kept per (query, list) = 4 threads x KT
    if (bf3_db(dp) > BDM || k > 32) return 0;
    return 4 * (k <= 2 ? 2 : k <= 12 ? 4 : 8);
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
double ivf_bf2_coef(int d) {
    const double u = 1.0 / 16777216.0;
    return 1.02 / 65536.0 + (6.1 * d + 8.0) * u;
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
                        int64_t max_items, const int32_t* assign, unsigned long long* part,
                        float* pub, float* pbound, uint32_t* stats, float* D, int64_t* I,
                        KernelTimes* kt, hipStream_t s) {
    if (n <= 0) return;
    const int KE = ivf_mfma_kq(k, d);
    FAISS_THROW_IF_NOT(KE > 0);
    FAISS_THROW_IF_NOT(ldc % 4 == 0);
    FAISS_THROW_IF_NOT(nprobe <= 64);
    FAISS_THROW_IF_NOT(obits >= 4 && obits <= 14);
    const int NS = bf3_db(d) / 16;
    const int64_t grid = (int64_t)roundup((size_t)max_items, 32);
    FAISS_THROW_IF_NOT(grid < (1ll << 31));
    const bool l2 = metric_l2 != 0;
    // margin of the approximate keys: the bf16 split plus the relative
    // truncation of the 32-bit keys (2^(obits-23)) on |approx|, which the
    // decode (low bits cleared / set) already brackets
    // precision of the filter: bf16x2 (default: half the code bytes, Cauchy-
    // Schwarz margins) or bf16x3 (FAISS_AMD_IVF_PREC=bf16x3: tighter margins,
    // fewer re-ranked candidates on data where bf16x2 keeps too many)
    const char* prec = getenv("FAISS_AMD_IVF_PREC");
    const bool y3 = prec && !strcmp(prec, "bf16x3");
    const float coef = (float)(y3 ? ivf_bf3_coef(d) : ivf_bf2_coef(d));
    {
        ScopedKernelTimer tm(kt, "ivf_flat_scan", 0.0, s);
#define LAUNCH_NS(L2V, KTV, NSV)                                                              \
    do {                                                                                      \
        if (y3)                                                                               \
            k_ivf_bf3_filter<L2V, KTV, NSV, true><<<dim3((unsigned)grid), dim3(256), 0, s>>>( \
                    x, ldx, d, (const __bf16*)cbf, ynorm, ynmax, rres, rmax, list_off,       \
                    list_len, nlist,                                                          \
                    nprobe, coef, obits, b.bucket_off, b.item_off, b.entries, part, pub,      \
                    pbound);                                                                  \
        else                                                                                  \
            k_ivf_bf3_filter<L2V, KTV, NSV, false><<<dim3((unsigned)grid), dim3(256), 0, s>>>(\
                    x, ldx, d, (const __bf16*)cbf, ynorm, ynmax, rres, rmax, list_off,       \
                    list_len, nlist,                                                          \
                    nprobe, coef, obits, b.bucket_off, b.item_off, b.entries, part, pub,      \
                    pbound);                                                                  \
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
    }
    {
        ScopedKernelTimer tm(kt, "ivf_rerank", 0.0, s);
        const int E = nprobe * KE;
        const int V = E <= 128 ? 2 : E <= 256 ? 4 : E <= 512 ? 8 : E <= 1024 ? 16 : 32;
#define LAUNCH_B(L2V, VV)                                                                     \
    k_ivf_rerank<L2V, VV><<<dim3((unsigned)cdiv(n, 4)), dim3(256), 0, s>>>(                  \
            part, pub, pbound, assign, list_off, list_len, nlist, x, ldx, codes, ldc, ids, d, \
            n, nprobe, KE, k, D, I, stats)
#define DISPATCH_V(L2V)                      \
    do {                                     \
        if (V == 2) LAUNCH_B(L2V, 2);        \
        else if (V == 4) LAUNCH_B(L2V, 4);   \
        else if (V == 8) LAUNCH_B(L2V, 8);   \
        else if (V == 16) LAUNCH_B(L2V, 16); \
        else LAUNCH_B(L2V, 32);              \
    } while (0)
        if (l2) DISPATCH_V(true);
        else DISPATCH_V(false);
        HIP_LAUNCH_CHECK();
#undef DISPATCH_V
#undef LAUNCH_A
#undef LAUNCH_NS
#undef LAUNCH_B
#undef DISPATCH
    }
}

}  // namespace kern
}  // namespace faiss_amd
