// kernels_pq_mfma.hip — IVF-PQ list scan as a certified bf16 MFMA filter over
// decoded codes (reference: IVFPQScanner, faiss/IndexIVFPQ.cpp:483-933, and
// the scan loop faiss/IndexIVF.cpp:595-631).
//
// The query-centric LUT scan (kernels_pq.hip) pays one LDS gather per code
// byte per query and is bound by LDS bank conflicts.  Here the work is
// list-centric like the IVF-Flat filter: a work item is (list, <= 64 queries
// probing it), each 64-row tile of the list is decoded ONCE into bf16 MFMA
// A-fragments (one gather of dsub centroid values per code byte, from a bf16
// copy of the PQ centroids held in LDS for the whole kernel) and multiplied
// against the 64 queries' bf16 hi+lo fragments.  For the by-residual L2
// distance
//     ||x - y_C - y_R||^2 = coarse_dis + term(row) - 2 <x, y_R>,
//     term(row) = ||y_R||^2 + 2 <y_C, y_R>             (per arena row)
// so the filter key is  coarse_dis(q, probe) + term - 2 acc.
//
// Certification (the same scheme as the Flat filter, kernels_ivf_mfma.hip):
// with R = ||y_R||, r = ||y_R - bf16(y_R)|| (per row, list maxima rmax/Rmax),
// |approx - reference| <= 2 ||x|| r + coef (||x|| + ||y_C|| + R)^2, where coef
// covers the bf16 split of the query (2^-16), the f32 accumulation of the
// MFMA, the rounding of term, of the reference's LUT construction and
// summation (tables 0 and 1) and of coarse_dis (ivfpq_mfma_coef).  The kernel
// keeps, per (query, list), 4 thread streams x KT best 32-bit keys plus a
// lower bound of every dropped key; the re-rank (k_ivf_rerank with PQD > 0)
// evaluates every candidate that can reach the top-k with the reference's
// own table arithmetic (oracle_ivf_search_preassigned, IndexIVFPQ.cpp:
// 634-700 + code_distance-generic.h:16-79), so results equal the reference's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "bf3.h"
#include "common.h"
#include "kernels.h"
#include "wave_select.h"

namespace faiss_amd {
namespace kern {

// bf16 copy of the PQ centroids, [M][256][dsub] (the decode table)
__global__ void k_pq_dec_table(const float* __restrict__ pq_cent, int n, __bf16* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (__bf16)pq_cent[i];
}

// per arena row: R = ||y_R|| and r = ||y_R - bf16(y_R)|| (rounded up)
__global__ void k_pq_row_res(const uint8_t* __restrict__ codes, int cs, int64_t rows, int M,
                             int dsub, const float* __restrict__ pq_cent,
                             float* __restrict__ rnorm, float* __restrict__ rres) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= rows) return;
    double s = 0.0, e = 0.0;
    for (int m = 0; m < M; m++) {
        const int j = codes[v * cs + m];
        const float* c = pq_cent + ((int64_t)m * 256 + j) * dsub;
        for (int i = 0; i < dsub; i++) {
            const double y = c[i];
            const double yh = (double)(float)(__bf16)c[i];
            s += y * y;
            e += (y - yh) * (y - yh);
        }
    }
    rnorm[v] = (float)(sqrt(s) * (1.0 + 1e-6));
    rres[v] = (float)(sqrt(e) * (1.0 + 1e-6));
}

void pq_decode_prep(const float* pq_cent, int M, int dsub, const uint8_t* codes, int cs,
                    int64_t rows, void* dec, float* rnorm, float* rres, hipStream_t s) {
    const int n = M * 256 * dsub;
    k_pq_dec_table<<<kgrid(cdiv(n, 256), 256), dim3(256), 0, s>>>(pq_cent, n, (__bf16*)dec);
    HIP_LAUNCH_CHECK();
    if (rows > 0) {
        k_pq_row_res<<<kgrid(cdiv(rows, 256), 256), dim3(256), 0, s>>>(
                codes, cs, rows, M, dsub, pq_cent, rnorm, rres);
        HIP_LAUNCH_CHECK();
    }
}

double ivfpq_mfma_coef(int d, int M) {
    const double u = 1.0 / 16777216.0;
    // query split + MFMA accumulation + term + reference LUT build / sum +
    // coarse distance, each bounded by a multiple of (|x| + |y_C| + R)^2
    return 1.02 / 65536.0 + (4.0 * d + 2.0 * M + 64.0) * u;
}

// A fragment of one lane for k-step s: row `cw` (its code words), dims
// [16 s + 8 lh, +8) decoded from the LDS table (8 / DSUB entries of DSUB
// bf16 each).  Decoded one k-step at a time, just before its MFMAs, so only
// one fragment's gathers are live.
template <int DSUB, int NWC>
__device__ __forceinline__ bf16x8 pq_decode_frag(const uint32_t (&cw)[NWC], int lh,
                                                 const uint8_t* __restrict__ dec, int s) {
    constexpr int E = 8 / DSUB;  // subquantizers per fragment
    uint32_t w32[4];
#pragma unroll
    for (int u = 0; u < E; u++) {
        // byte m of the code, m = (16 s) / DSUB + lh * E + u
        const int mb = (16 * s) / DSUB + u;  // compile-time part
        const int m_lo = mb, m_hi = mb + E;  // lh = 0 / 1
        const uint32_t wl = cw[m_lo >> 2], wh = cw[m_hi >> 2];
        const uint32_t blo = (wl >> (8 * (m_lo & 3))) & 0xffu;
        const uint32_t bhi = (wh >> (8 * (m_hi & 3))) & 0xffu;
        const uint32_t j = lh ? bhi : blo;
        const int m = lh ? m_hi : m_lo;
        const uint8_t* src = dec + ((size_t)m * 256 + j) * (2 * DSUB);
        if constexpr (DSUB == 2) {
            w32[u] = *(const uint32_t*)src;
        } else if constexpr (DSUB == 4) {
            const uint2 v = *(const uint2*)src;
            w32[2 * u] = v.x;
            w32[2 * u + 1] = v.y;
        } else {
            const uint4 v = *(const uint4*)src;
            w32[0] = v.x;
            w32[1] = v.y;
            w32[2] = v.z;
            w32[3] = v.w;
        }
    }
    union {
        uint32_t w[4];
        bf16x8 v;
    } cv;
#pragma unroll
    for (int i = 0; i < 4; i++) cv.w[i] = w32[i];
    return cv.v;
}

// The same fragment with the lane half folded into a per-lane table base
// (dec_lh = dec + 4096 lh: sub-quantizer m + E lh starts E * 256 * 2 DSUB =
// 4096 bytes further) and into the byte's word / shift, so each gather is one
// bit-field extract + one address add, its sub-quantizer's table offset an
// immediate of the LDS read (pq_decode_frag selects between the two halves'
// bytes and sub-quantizers per gather).  Byte m = 16 s / DSUB + E lh + u:
//   DSUB 2: 8 s + 4 lh + u -> word 2 s + lh, byte u
//   DSUB 4: 4 s + 2 lh + u -> word s, byte 2 lh + u
//   DSUB 8: 2 s + lh       -> word s / 2, byte (2 s) % 4 + lh
template <int DSUB, int NWC>
__device__ __forceinline__ bf16x8 pq_decode_frag_l(const uint32_t (&cw)[NWC], int lh,
                                                   const uint8_t* __restrict__ dec_lh, int s) {
    static_assert(DSUB == 2 || DSUB == 4 || DSUB == 8, "dsub");
    // (v_bfe_u32 with the per-lane shift, 32-bit LDS offsets: one extract
    // and one v_lshl_add_u32 per gather; a shift-and-mask and 64-bit offset
    // arithmetic compiled to four)
    uint32_t w32[4];
    if constexpr (DSUB == 2) {
        const uint32_t w = lh ? cw[2 * s + 1] : cw[2 * s];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t j = __builtin_amdgcn_ubfe(w, 8u * u, 8u);
            w32[u] = *(const uint32_t*)(dec_lh + (int)((8 * s + u) * 1024) + (int)(j << 2));
        }
    } else if constexpr (DSUB == 4) {
        const uint32_t w = cw[s];
        const uint32_t sh = 16u * (uint32_t)lh;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t j = __builtin_amdgcn_ubfe(w, sh + 8u * u, 8u);
            const uint2 v = *(const uint2*)(dec_lh + (int)((4 * s + u) * 2048) + (int)(j << 3));
            w32[2 * u] = v.x;
            w32[2 * u + 1] = v.y;
        }
    } else {
        const uint32_t w = cw[s >> 1];
        const uint32_t j =
                __builtin_amdgcn_ubfe(w, 8u * (uint32_t)((2 * s) & 3) + 8u * (uint32_t)lh, 8u);
        const uint4 v = *(const uint4*)(dec_lh + (int)((2 * s) * 4096) + (int)(j << 4));
        w32[0] = v.x;
        w32[1] = v.y;
        w32[2] = v.z;
        w32[3] = v.w;
    }
    union {
        uint32_t w[4];
        bf16x8 v;
    } cv;
#pragma unroll
    for (int i = 0; i < 4; i++) cv.w[i] = w32[i];
    return cv.v;
}

// One work item = (list, <= 64 queries); persistent work-groups walk the
// items with stride gridDim.x, so the LDS decode table is loaded once per
// work-group.  Wave layout, keys, streams and outputs as k_ivf_bf3_filter.
// HS: an IDSelector mask is present (own instantiation; none on the hot path)
template <int DSUB, int NS, int KT, bool HS>
__global__ __launch_bounds__(256, 3) void k_ivfpq_filter(
        const float* __restrict__ x, int ldx, const __bf16* __restrict__ dec_g,
        const uint8_t* __restrict__ codes, const float* __restrict__ terms,
        const float* __restrict__ cdis, const float* __restrict__ cnorm,
        const float* __restrict__ lrmax, const float* __restrict__ lRmax, int nlist, int nprobe,
        float coef, int obits, const uint32_t* __restrict__ item_off,
        const ItemDesc* __restrict__ item_desc, const uint32_t* __restrict__ item_entries,
        const uint32_t* __restrict__ lim, const uint8_t* __restrict__ sel,
        uint32_t* __restrict__ keys, ProbeRec* __restrict__ recs,
        const uint8_t* __restrict__ qimg, const float* __restrict__ qxn) {
    constexpr int D = 16 * NS;
    constexpr int M = D / DSUB;
    constexpr int CS = (M + 3) & ~3;  // code stride (bytes)
    constexpr int NWC = CS / 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t dec[];  // [M][256][DSUB] bf16
    __shared__ __attribute__((aligned(16))) float ynt[2][BV];      // term per row (+inf pad)
    __shared__ float bnd_s[BQ][4];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    {
        constexpr int NW16 = M * 256 * DSUB * 2 / 16;
        const uint4* src = (const uint4*)dec_g;
        for (int i = t; i < NW16; i += 256) ((uint4*)dec)[i] = src[i];
    }
    __syncthreads();  // the decode table
    const int bi = w >> 1, bj = w & 1;
    const int li = lane & 31, lh = lane >> 5;
    const int slot = 2 * bi + lh;
    const int qloc = 32 * bj + li;
    const uint32_t lowmask = (1u << obits) - 1u;
    const uint32_t nitems = item_off[nlist];

    // Every global load is consumed one step after it is issued, so its
    // latency hides under other work: the next item's descriptor and this
    // lane's entry of it load while the current item runs, a tile's codes
    // and terms load while the previous tile is multiplied (the terms are
    // masked when they are stored, not when they arrive).
    uint32_t it = blockIdx.x;
    ItemDesc dsc{};
    uint32_t my_e = 0u;
    if (it < nitems) {
        dsc = item_desc[it];
        my_e = item_entries[(size_t)it * BQ + qloc];
    }
    for (; it < nitems; it += gridDim.x) {
        const uint32_t itn = it + gridDim.x;
        ItemDesc dscn{};
        uint32_t my_en = 0u;
        if (itn < nitems) {
            dscn = item_desc[itn];
            my_en = item_entries[(size_t)itn * BQ + qloc];
        }
        const int l = (int)dsc.l;
        const int nQ = (int)dsc.nq;
        const int len = (int)dsc.len;
        const int64_t row0 = dsc.off;
        const bool qvalid = qloc < nQ;
        const bool active = 32 * bj < nQ;  // wave-uniform
        // query fragments and coarse distance of this lane's column
        bf16x8 bh[NS], bl[NS];
        float xn = 0.f, base = 0.f;
        if (active) {
            const int32_t qr = qvalid ? (int32_t)(my_e / (uint32_t)nprobe) : -1;
            // fragments prepared once per query (k_query_prep; the host always
            // passes the image)
            load_query_image<NS>(qimg, qxn, qr, lh, bh, bl, xn);
            base = cdis[qvalid ? my_e : 0u];
        }
        // this lane's code row of a tile and the tile's terms (raw)
        uint32_t cw[NWC];
        auto load_codes = [&](int v0n) {
            const int r = v0n + 32 * bi + li;
            const uint8_t* cp = codes + (row0 + (r < len ? r : 0)) * CS;
            if constexpr (CS % 16 == 0) {
#pragma unroll
                for (int i = 0; i < NWC; i += 4) {
                    const uint4 v = *(const uint4*)(cp + 4 * i);
                    cw[i] = v.x;
                    cw[i + 1] = v.y;
                    cw[i + 2] = v.z;
                    cw[i + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < NWC; i++) cw[i] = *(const uint32_t*)(cp + 4 * i);
            }
        };
        float4 traw = make_float4(0.f, 0.f, 0.f, 0.f);
        uchar4 mraw = make_uchar4(1, 1, 1, 1);
        auto load_terms = [&](int v0n) {
            if (t < BV / 4) {
                const int r = 4 * t;
                const int nvn = min(BV, len - v0n);
                // rows < roundup(len, 16) are inside the list's arena slot
                if (r < nvn) {
                    traw = *(const float4*)(terms + row0 + v0n + r);
                    if constexpr (HS) mraw = *(const uchar4*)(sel + row0 + v0n + r);
                }
            }
        };
        auto store_terms = [&](int buf, int v0n) {
            if (t < BV / 4) {
                const int r = 4 * t;
                const int nvn = min(BV, len - v0n);
                float4 tn;
                if constexpr (HS) {
                    // non-members of an IDSelector are treated as padding rows
                    tn.x = r + 0 < nvn && mraw.x ? traw.x : WS_INF;
                    tn.y = r + 1 < nvn && mraw.y ? traw.y : WS_INF;
                    tn.z = r + 2 < nvn && mraw.z ? traw.z : WS_INF;
                    tn.w = r + 3 < nvn && mraw.w ? traw.w : WS_INF;
                } else {
                    tn.x = r + 0 < nvn ? traw.x : WS_INF;
                    tn.y = r + 1 < nvn ? traw.y : WS_INF;
                    tn.z = r + 2 < nvn ? traw.z : WS_INF;
                    tn.w = r + 3 < nvn ? traw.w : WS_INF;
                }
                *(float4*)(&ynt[buf][4 * t]) = tn;
            }
        };
        load_codes(0);
        load_terms(0);
        ThreadQueue32<KT> tq;
        tq.init();
        for (int v0 = 0, tile = 0; v0 < len; v0 += BV, tile++) {
            const int buf = tile & 1;
            const bool more = v0 + BV < len;
            store_terms(buf, v0);
            if (more) load_terms(v0 + BV);
            __syncthreads();  // ynt[buf]
            if (active) {
                floatx16 acc;
#pragma unroll
                for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
                for (int s = 0; s < NS; s++) {
                    const bf16x8 ah = pq_decode_frag<DSUB, NWC>(cw, lh, dec, s);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[s], acc, 0, 0, 0);
                }
                // the next tile's code words load under this tile's MFMAs and
                // pushes (cw is decoded)
                if (more) load_codes(v0 + BV);
                const uint32_t ordbase = (uint32_t)tile << 4;
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const float4 yq = *(const float4*)(&ynt[buf][32 * bi + 4 * lh + 8 * g]);
#pragma unroll
                    for (int c = 0; c < 4; c++) {
                        const int r = 4 * g + c;
                        const float yv = c == 0 ? yq.x : c == 1 ? yq.y : c == 2 ? yq.z : yq.w;
                        const float a = fmaf(-2.f, acc[r], base + yv);
                        tq.push(key_encode<true>(a, lowmask, ordbase | (uint32_t)r));
                    }
                }
            }
        }

        // ---- outputs (as k_ivf_bf3_filter)
        const uint32_t last = tq.q[KT - 1];
        float bnd = WS_INF;
        if (last != 0xffffffffu) {
            const int row = (int)ivf_key_row(last, lowmask, slot);
            if (row < len) bnd = key_decode_lo<true>(last, lowmask);
        }
        bnd_s[qloc][slot] = bnd;
        __syncthreads();
        if (qvalid) {
            const int64_t e = my_e;
            const uint32_t elen = lim ? min((uint32_t)len, lim[e]) : (uint32_t)len;
            uint32_t* ko = keys + e * (4 * KT) + slot * KT;
#pragma unroll
            for (int i = 0; i < KT; i++) {
                const uint32_t key = tq.q[i];
                const uint32_t row = ivf_key_row(key, lowmask, slot);
                if constexpr (HS)
                    ko[i] = (key != 0xffffffffu && row < elen && sel[row0 + row]) ? key
                                                                                  : 0xffffffffu;
                else
                    ko[i] = (key != 0xffffffffu && row < elen) ? key : 0xffffffffu;
            }
            if (slot == 0) {
                const float xl = sqrtf(xn);
                const float sr = xl + cnorm[l] + lRmax[l];
                const float mmax = 2.f * (2.f * xl * lrmax[l] + coef * sr * sr) + 1e-30f;
                ProbeRec pr;
#pragma unroll
                for (int sl = 0; sl < 4; sl++) {
                    const float b = bnd_s[qloc][sl];
                    pr.pb[sl] = b < WS_INF ? b - mmax : WS_INF;
                }
                pr.mmax = mmax;
                pr.off = (uint32_t)row0;
                pr.len = elen;
                pr.pad = (uint32_t)l;
                recs[e] = pr;
            }
        }
        __syncthreads();  // bnd_s / ynt are reused by the next item
        dsc = dscn;
        my_e = my_en;
    }
}

// Wave-independent form (the default): the same work items, keys and probe
// records, but every wave is its own worker with no barrier after the decode
// table is loaded.  A task is (item, query half bj): one wave, 32 query
// columns, both 32-row blocks of every tile (thread streams slot = 2 bi + lh
// of its queries, as above).  Each wave loads its own rows' code words and
// the tile's terms (through a wave-private LDS slot), keeps the next tile's
// loads in flight under the current tile's MFMAs, and assembles each query's
// probe record itself (the two lane halves of a column hold its 4 streams).
// Work groups of WPB waves share one decode table, so a CU holds as many
// workers as its registers allow instead of as many 4-wave groups as its LDS
// holds tables; waves desynchronise and hide each other's load latency.
template <int DSUB, int NS, int KT, bool HS>
__global__ __launch_bounds__(768, 3) void k_ivfpq_filter_w(
        const __bf16* __restrict__ dec_g, const uint8_t* __restrict__ codes,
        const float* __restrict__ terms, const float* __restrict__ cdis,
        const float* __restrict__ cnorm, const float* __restrict__ lrmax,
        const float* __restrict__ lRmax, int nlist, int nprobe, float coef, int obits,
        const uint32_t* __restrict__ item_off, const ItemDesc* __restrict__ item_desc,
        const uint32_t* __restrict__ item_entries, const uint32_t* __restrict__ lim,
        const uint8_t* __restrict__ sel, uint32_t* __restrict__ keys,
        ProbeRec* __restrict__ recs, const uint8_t* __restrict__ qimg,
        const float* __restrict__ qxn, uint32_t* __restrict__ task_ctr,
        unsigned long long* __restrict__ trace, int sched) {
    // FAISS_AMD_PQ_TRACE=<file>: per task [start, prologue done, end, info]
    // (s_memrealtime; info = len | nQ << 16 | bj << 24 | worker << 32)
    constexpr int D = 16 * NS;
    constexpr int M = D / DSUB;
    constexpr int CS = (M + 3) & ~3;  // code stride (bytes)
    constexpr int NWC = CS / 4;
    constexpr int TBL = M * 256 * DSUB * 2;  // decode table bytes
    extern __shared__ __attribute__((aligned(16))) uint8_t dec[];  // table | per-wave terms
    __shared__ uint32_t grp_next;  // the group's next task position (sched & 2)
    const int nthr = blockDim.x, wpb = nthr >> 6;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    {
        const uint4* src = (const uint4*)dec_g;
        for (int i = t; i < TBL / 16; i += nthr) ((uint4*)dec)[i] = src[i];
    }
    if (t == 0) grp_next = (uint32_t)wpb;
    __syncthreads();  // the decode table (the only barrier)
    const int li = lane & 31, lh = lane >> 5;
    const uint8_t* dec_lh = dec + (lh ? 4096 : 0);  // (pq_decode_frag_l)
    const uint32_t lowmask = (1u << obits) - 1u;
    const uint32_t nitems = item_off[nlist];
    const uint32_t ntask = 2u * nitems;
    const uint32_t nstatic = gridDim.x * (uint32_t)wpb;
    // Work assignment.  Static rounds of nstatic tasks over the items in
    // longest-list-first order (IVFBuckets::perm): position p of round r
    // (worker p of the grid) is task r nstatic + p, walked boustrophedon
    // (sched & 1: nstatic - 1 - p in odd rounds), so a position given a long
    // task in one round gets a short one in the next.  sched & 2: the group's
    // waves share its positions (blockIdx wpb + 0 .. wpb - 1 of every round)
    // and take the next one from an LDS counter when they finish a task, so a
    // CU's waves end together instead of a third of the span in the CU's own
    // tail (r05 per-task traces: with fixed positions the first wave of a CU
    // finished at 56 % (c3) / 77 % (c5) of the last one's end).  A global work
    // counter measured slower (c3 0.20 vs 0.13 ms): the same-address atomics
    // of 3072 waves serialise and each wave's later loads return behind its
    // claim.
    const uint32_t g0 = blockIdx.x * (uint32_t)wpb;
    const bool share = (sched & 2) != 0;
    const uint32_t cycle = share ? (uint32_t)wpb : 1u;  // positions per round per claimer
    uint32_t j = share ? (uint32_t)w : 0u;               // position index (this group / wave)
    auto task_of = [&](uint32_t jj) -> uint32_t {
        const uint32_t r = jj / cycle;
        const uint32_t p = share ? g0 + jj % cycle : g0 + (uint32_t)w;
        return r * nstatic + (((sched & 1) && (r & 1u)) ? nstatic - 1u - p : p);
    };
    auto next_pos = [&]() -> uint32_t {
        if (!share) return j + 1u;
        uint32_t v = 0u;
        if (lane == 0) v = atomicAdd(&grp_next, 1u);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    };
    // (a round whose first task is past the end ends the walk; within the
    // last round a position past the end is skipped)
    for (; (j / cycle) * nstatic < ntask;) {
        const uint32_t task = task_of(j);
        if (task >= ntask) {
            j = next_pos();
            continue;
        }
        const uint32_t it = task >> 1;
        const int bj = (int)(task & 1u);
        const unsigned long long t_s = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
        const ItemDesc dsc = item_desc[it];
        const int nQ = (int)dsc.nq;
        if (32 * bj >= nQ) {  // wave-uniform: an item of <= 32 queries
            j = next_pos();
            continue;
        }
        const int l = (int)dsc.l;
        const int len = (int)dsc.len;
        const int64_t row0 = dsc.off;
        const int qloc = 32 * bj + li;
        const bool qvalid = qloc < nQ;
        const uint32_t my_e = item_entries[(size_t)it * BQ + qloc];
        // list-level margin operands (uniform)
        const float cn_l = cnorm[l], rmax_l = lrmax[l], Rmax_l = lRmax[l];
        bf16x8 bh[NS], bl[NS];
        float xn = 0.f;
        load_query_image<NS>(qimg, qxn, qvalid ? (int32_t)(my_e / (uint32_t)nprobe) : -1, lh,
                             bh, bl, xn);
        const float base = cdis[qvalid ? my_e : 0u];
        const uint32_t elen = (lim && qvalid) ? min((uint32_t)len, lim[my_e]) : (uint32_t)len;
        // code words and term of this lane's two rows (li, 32 + li) of a tile
        // (rows past the list, and IDSelector non-members, get term +inf: the
        // padding key, sorted after every real one)
        uint32_t cw[2][NWC];
        float tv[2];
        auto load_codes = [&](int bi, int v0n) {
            const int r = v0n + 32 * bi + li;
            const uint8_t* cp = codes + (row0 + (r < len ? r : 0)) * CS;
            if constexpr (CS % 16 == 0) {
#pragma unroll
                for (int i = 0; i < NWC; i += 4) {
                    // (non-temporal code loads measured slower: r05 c3 filter
                    // 105 -> 114 us, c5 1.37 -> 1.55 ms)
                    const uint4 v = *(const uint4*)(cp + 4 * i);
                    cw[bi][i] = v.x;
                    cw[bi][i + 1] = v.y;
                    cw[bi][i + 2] = v.z;
                    cw[bi][i + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < NWC; i++) cw[bi][i] = *(const uint32_t*)(cp + 4 * i);
            }
            tv[bi] = r < len ? terms[row0 + r] : WS_INF;
            if constexpr (HS) {
                if (r < len && !sel[row0 + r]) tv[bi] = WS_INF;
            }
        };
        load_codes(0, 0);
        load_codes(1, 0);
        // folded bias (as the Flat filter's fold images): one more k-step with
        // A = {-term/2 in three bf16 parts, 1, 1, 1, 0, 0} (the row, lh = 0
        // lanes; zeros for lh = 1) and B = {1, 1, 1, -coarse_dis/2 in three
        // parts, 0, 0}, so the accumulator is -approx/2 of coarse_dis + term -
        // 2 <x, y_R> and a key is one v_bfi_b32 of its bits (ivfpq_fold_coef
        // covers the six bias products; r05: 7 VALU per candidate before)
        bf16x8 bq;
        {
            __bf16 h, m, lo;
            split3_bf16(-0.5f * base, h, m, lo);
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
        auto bias_frag = [&](float term) {
            __bf16 h, m, lo;
            split3_bf16(-0.5f * term, h, m, lo);
            const __bf16 one = (__bf16)1.f, zero = (__bf16)0.f;
            // padding rows and IDSelector non-members (term +inf): -inf, 0, 0
            // as the image builders write them, so the accumulator is -inf
            // (key 0xff80xxxx, after every real key) — split3 of -inf would
            // leave NaN in the residual parts and a NaN key, which sorts ahead
            // of the real keys and gives its stream a dropped bound of 0
            if (!(term < WS_INF)) {
                m = zero;
                lo = zero;
            }
            bf16x8 ab;
            ab[0] = lh ? zero : h;
            ab[1] = lh ? zero : m;
            ab[2] = lh ? zero : lo;
            ab[3] = lh ? zero : one;
            ab[4] = lh ? zero : one;
            ab[5] = lh ? zero : one;
            ab[6] = zero;
            ab[7] = zero;
            return ab;
        };
        ThreadQueue32<KT> tq[2];
        tq[0].init();
        tq[1].init();
        unsigned long long t_p = 0ull;
        if (trace) {  // (waits for the prologue's loads: profiling only)
            float acc0 = base + xn + tv[0];
#pragma unroll
            for (int i = 0; i < NWC; i++) acc0 += (float)(cw[0][i] & 1u);
            if (__builtin_amdgcn_readfirstlane(__float_as_uint(acc0)) == 0xffffffffu) t_p = 1ull;
            t_p += __builtin_amdgcn_s_memrealtime();
        }
        for (int v0 = 0, tile = 0; v0 < len; v0 += BV, tile++) {
            const bool more = v0 + BV < len;
            const uint32_t ordbase = (uint32_t)tile << 4;
#pragma unroll
            for (int bi = 0; bi < 2; bi++) {
                floatx16 acc;
#pragma unroll
                for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
                for (int s = 0; s < NS; s++) {
                    const bf16x8 ah = pq_decode_frag_l<DSUB, NWC>(cw[bi], lh, dec_lh, s);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[s], acc, 0, 0, 0);
                }
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bias_frag(tv[bi]), bq, acc, 0, 0, 0);
                // block bi decoded: its next code words load under the pushes
                if (more) load_codes(bi, v0 + BV);
                mfma_read_guard();  // key_insert reads acc (inline asm)
#pragma unroll
                for (int r = 0; r < 16; r++)
                    tq[bi].push(key_insert(fold_key_bits(acc[r]), lowmask, ordbase | (uint32_t)r));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- outputs: this lane's two streams (slot 2 bi + lh) of query qloc
        const float xl = sqrtf(xn);
        const float sr = xl + cn_l + Rmax_l;
        const float mmax = 2.f * (2.f * xl * rmax_l + coef * sr * sr) + 1e-30f;
        float pb[2];
#pragma unroll
        for (int bi = 0; bi < 2; bi++) {
            const int slot = 2 * bi + lh;
            const uint32_t last = tq[bi].q[KT - 1];
            float bnd = WS_INF;
            if (last != 0xffffffffu && (int)ivf_key_row(last, lowmask, slot) < len)
                bnd = fold_decode_lo(last, lowmask);
            pb[bi] = bnd < WS_INF ? bnd - mmax : WS_INF;
            if (qvalid) {
                uint32_t* ko = keys + (int64_t)my_e * (4 * KT) + slot * KT;
#pragma unroll
                for (int i = 0; i < KT; i++) {
                    const uint32_t key = tq[bi].q[i];
                    const uint32_t row = ivf_key_row(key, lowmask, slot);
                    if constexpr (HS)
                        ko[i] = (key != 0xffffffffu && row < elen && sel[row0 + row]) ? key
                                                                                      : 0xffffffffu;
                    else
                        ko[i] = (key != 0xffffffffu && row < elen) ? key : 0xffffffffu;
                }
            }
        }
        // slots 1 and 3 live in the other lane half of the column
        const float pb1 = __shfl_xor(pb[0], 32), pb3 = __shfl_xor(pb[1], 32);
        if (qvalid && lh == 0) {
            ProbeRec pr;
            pr.pb[0] = pb[0];
            pr.pb[1] = pb1;
            pr.pb[2] = pb[1];
            pr.pb[3] = pb3;
            pr.mmax = mmax;
            pr.off = (uint32_t)row0;
            pr.len = elen;
            pr.pad = (uint32_t)l;
            recs[my_e] = pr;
        }
        if (trace && lane == 0) {
            unsigned long long* tr = trace + 4ull * task;
            tr[0] = t_s;
            tr[1] = t_p;
            tr[2] = __builtin_amdgcn_s_memrealtime();
            tr[3] = (unsigned long long)(uint32_t)len | ((unsigned long long)(uint32_t)nQ << 16) |
                    ((unsigned long long)bj << 24) |
                    ((unsigned long long)(blockIdx.x * (uint32_t)wpb + (uint32_t)w) << 32);
        }
        j = next_pos();
    }
}

bool ivfpq_mfma_eligible(int d, int M, int k, int nprobe) {
    if (d % 16 != 0 || M <= 0 || d % M != 0 || k > 32 || nprobe > kMaxNprobeFilter) return false;
    const int dsub = d / M, NS = d / 16;
    if (dsub != 2 && dsub != 4 && dsub != 8) return false;
    return NS == 4 || NS == 6 || NS == 8;
}

void ivfpq_filter(const float* x, int ldx, int d, int M, const void* dec, const uint8_t* codes,
                  const float* terms, const float* cdis, const float* cnorm, const float* lrmax,
                  const float* lRmax, int nlist, int64_t n, int nprobe, int k, int obits,
                  const IVFBuckets& b, int64_t max_items, uint32_t* keys, ProbeRec* recs,
                  int* kt_out, hipStream_t s, const void* qimg, const float* qxn) {
    FAISS_THROW_IF_NOT(ivfpq_mfma_eligible(d, M, k, nprobe));
    FAISS_THROW_IF_NOT(b.item_desc && b.item_entries);
    FAISS_THROW_IF_NOT_MSG(qimg && qxn, "ivfpq_filter needs the prepared query image");
    FAISS_THROW_IF_NOT(obits >= 4 && obits <= 14);
    const int KE = ivf_mfma_kq(k, d, nprobe);
    FAISS_THROW_IF_NOT(KE > 0);
    *kt_out = KE / 4;
    const int dsub = d / M, NS = d / 16;
    const size_t lds = (size_t)M * 256 * dsub * 2;
    // persistent grid: enough work-groups to fill every CU at the occupancy
    // the LDS table allows, never more than the items
    int dev = 0, ncu = 256;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / (lds + 4096))));
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(max_items, (int64_t)ncu * per_cu));
    const float coef = (float)ivfpq_mfma_coef(d, M);
    // wave-independent kernel (default; FAISS_AMD_PQ_FILTER=wg: the 4-wave
    // work-group form): one group of 12 waves per CU sharing one table — the
    // 3 waves per SIMD its registers allow (<= 168 VGPRs), 3 on every SIMD.
    // (r05: two 6-wave groups per CU did not co-reside: each group's waves
    // land 2, 2, 1, 1 on the SIMDs and a second one would need 4 on two of
    // them, so half the groups waited for the first half to finish — c3's
    // per-task trace showed 256 groups starting at 0 us and 256 at ~60 us.)
    const char* fenv = getenv("FAISS_AMD_PQ_FILTER");
    if (!(fenv && !strcmp(fenv, "wg")) && b.item_ctr) {
        const size_t tbl = lds;
        const char* wenv = getenv("FAISS_AMD_PQ_WPB");  // (A/B: waves per group)
        const int wpb = std::max(1, std::min(12, wenv ? atoi(wenv) : 12));
        const int groups = std::max(1, 12 / wpb);
        const size_t ldsw = tbl;
        FAISS_THROW_IF_NOT(ldsw <= 160 * 1024);
        const float coefw = (float)ivfpq_fold_coef(d, M);  // (folded bias keys)
        // FAISS_AMD_PQ_SCHED (A/B): "stride" (fixed positions, plain stride),
        // "snake" (fixed positions, boustrophedon); default: shared, snake
        const char* denv = getenv("FAISS_AMD_PQ_SCHED");
        const int sched = !denv ? 3 : !strcmp(denv, "stride") ? 0 : !strcmp(denv, "snake") ? 1 : 3;
        const int64_t ntask = 2 * max_items;
        const int64_t gridw = std::max<int64_t>(
                1, std::min<int64_t>(cdiv(ntask, wpb), (int64_t)ncu * groups));
        // FAISS_AMD_PQ_TRACE=<file>: per-task stamps (profiling; synchronises)
        static unsigned long long* trace_buf = nullptr;
        static int64_t trace_n = 0;
        const char* trf = getenv("FAISS_AMD_PQ_TRACE");
        unsigned long long* trace = nullptr;
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (trf && hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone) {
            if (trace_n < ntask) {
                if (trace_buf) HIP_CHECK(hipFree(trace_buf));
                HIP_CHECK(hipMalloc(&trace_buf, 32 * ntask));
                trace_n = ntask;
            }
            HIP_CHECK(hipMemsetAsync(trace_buf, 0, 32 * ntask, s));
            trace = trace_buf;
        }
        auto dump = [&] {
            if (!trace) return;
            std::vector<unsigned long long> h(4 * ntask);
            HIP_CHECK(hipMemcpyAsync(h.data(), trace, 32 * ntask, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            if (FILE* f = fopen(trf, "wb")) {
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        };
#define PQW(DS, NSV, KTV)                                                                      \
    if (dsub == DS && NS == NSV && KE / 4 == KTV) {                                            \
        auto kfn = b.sel ? k_ivfpq_filter_w<DS, NSV, KTV, true>                                \
                         : k_ivfpq_filter_w<DS, NSV, KTV, false>;                               \
        HIP_CHECK(hipFuncSetAttribute((const void*)kfn,                                        \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsw)); \
        kfn<<<kgrid(gridw, 64 * wpb), dim3(64 * wpb), ldsw, s>>>(                               \
                (const __bf16*)dec, codes, terms, cdis, cnorm, lrmax, lRmax, nlist, nprobe,    \
                coefw, obits, b.item_off, b.item_desc, b.item_entries, b.lim, b.sel, keys,      \
                recs, (const uint8_t*)qimg, qxn, b.item_ctr, trace, sched);                    \
        HIP_LAUNCH_CHECK();                                                                    \
        dump();                                                                                \
        return;                                                                                \
    }
#define PQW_KT(DS, NSV) PQW(DS, NSV, 2) PQW(DS, NSV, 4) PQW(DS, NSV, 8)
#define PQW_NS(DS) PQW_KT(DS, 4) PQW_KT(DS, 6) PQW_KT(DS, 8)
        PQW_NS(2) PQW_NS(4) PQW_NS(8)
#undef PQW_NS
#undef PQW_KT
#undef PQW
    }
#define PQF(DS, NSV, KTV)                                                                      \
    if (dsub == DS && NS == NSV && KE / 4 == KTV) {                                            \
        auto kfn = b.sel ? k_ivfpq_filter<DS, NSV, KTV, true>                                  \
                         : k_ivfpq_filter<DS, NSV, KTV, false>;                                 \
        static bool attr[2] = {false, false};                                                  \
        if (!attr[b.sel ? 1 : 0]) {                                                            \
            HIP_CHECK(hipFuncSetAttribute((const void*)kfn,                                    \
                                          hipFuncAttributeMaxDynamicSharedMemorySize,          \
                                          (int)lds));                                          \
            attr[b.sel ? 1 : 0] = true;                                                        \
        }                                                                                      \
        kfn<<<kgrid(grid, 256), dim3(256), lds, s>>>(                                      \
                x, ldx, (const __bf16*)dec, codes, terms, cdis, cnorm, lrmax, lRmax, nlist,    \
                nprobe, coef, obits, b.item_off, b.item_desc, b.item_entries, b.lim, b.sel,    \
                keys, recs, (const uint8_t*)qimg, qxn);                                        \
        HIP_LAUNCH_CHECK();                                                                    \
        return;                                                                                \
    }
#define PQF_KT(DS, NSV) PQF(DS, NSV, 2) PQF(DS, NSV, 4) PQF(DS, NSV, 8)
#define PQF_NS(DS) PQF_KT(DS, 4) PQF_KT(DS, 6) PQF_KT(DS, 8)
    PQF_NS(2) PQF_NS(4) PQF_NS(8)
#undef PQF_NS
#undef PQF_KT
#undef PQF
    FAISS_THROW_MSG("ivfpq_filter: no kernel instance for this geometry");
}

}  // namespace kern
}  // namespace faiss_amd
