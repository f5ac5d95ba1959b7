// kernels_pq.hip — IVF-PQ search, encoding and per-code terms for gfx950.
//
// Reference: faiss/IndexIVFPQ.cpp
//   * precomputed "table 1": dis = coarse_dis + sum_m (P[key][m][c_m]
//     - 2 <x_m, c_{m,c_m}>) with P[key][m][j] = ||c_mj||^2 + 2 <yC_m, c_mj>
//     (:332-459, :634-653) — here the list-dependent part sum_m P[key][m][c_m]
//     is folded into one f32 "term" per stored code (computed once when the
//     lists are uploaded), so the 128 MB (nlist 4096) / 3.2 GB (nlist 65536)
//     table never has to be streamed and the query-only LUT T[m][j] =
//     -2 <x_m, c_mj> (M x 256 f32 = 32-48 KB) lives in LDS.
//   * table 0 (:637-643) computes ||r_m - c_mj||^2 with r = x - yC; it is the
//     same quantity, so one kernel serves both.
//   * scan: sum of M LUT gathers per code (:861-933, code_distance-generic.h).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "pq_ref.h"
#include "wave_select.h"

namespace faiss_amd {
namespace kern {

// ---------------------------------------------------------------- scan
// One workgroup (4 waves) per query.  LUT built in LDS; wave w scans probes
// w, w+4, ...; 64 codes per step (one per lane); the four per-wave queues are
// merged through LDS at the end.
__global__ __launch_bounds__(256) void k_ivfpq_scan(
        const float* __restrict__ x, int ldx, const float* __restrict__ pq_cent, int M, int ksub,
        int dsub, const uint8_t* __restrict__ codes, int code_stride,
        const float* __restrict__ terms, const int64_t* __restrict__ ids,
        const uint32_t* __restrict__ list_off, const uint32_t* __restrict__ list_len, int nlist,
        const int32_t* __restrict__ assign, const float* __restrict__ coarse_dis,
        const uint32_t* __restrict__ lim, const uint8_t* __restrict__ sel, int nprobe, int k,
        int by_residual, float* __restrict__ D, int64_t* __restrict__ I) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* T = smem;                    // [M * ksub]
    float* xq = T + M * ksub;           // [M * dsub]
    float* md = xq + ((M * dsub + 3) & ~3);
    long long* mi = (long long*)(md + 256);

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t q = blockIdx.x;
    const int d = M * dsub;
    for (int j = t; j < d; j += 256) xq[j] = x[q * ldx + j];
    __syncthreads();
    for (int e = t; e < M * ksub; e += 256) {
        const int m = e / ksub;
        const float* c = pq_cent + (int64_t)e * dsub;
        const float* xm = xq + m * dsub;
        float s = 0.f;
        if (by_residual) {
            for (int i = 0; i < dsub; i++) s = fmaf(xm[i], c[i], s);
            T[e] = -2.f * s;
        } else {
            for (int i = 0; i < dsub; i++) {
                float df = xm[i] - c[i];
                s = fmaf(df, df, s);
            }
            T[e] = s;
        }
    }
    __syncthreads();

    float qd = WS_INF;
    long long qi = WS_NOID;
    float thr_d = WS_INF;
    long long thr_i = WS_NOID;
    for (int r = w; r < nprobe; r += 4) {
        const int lst = assign[q * nprobe + r];
        if (lst < 0 || lst >= nlist) continue;
        const int len = (int)(lim ? min(lim[q * nprobe + r], list_len[lst]) : list_len[lst]);
        if (len == 0) continue;
        const float dis0 = by_residual ? coarse_dis[q * nprobe + r] : 0.f;
        const int64_t row0 = list_off[lst];
        for (int v0 = 0; v0 < len; v0 += 64) {
            const int v = v0 + lane;
            float k1 = WS_INF;
            long long k2 = WS_NOID;
            if (v < len && (!sel || sel[row0 + v])) {
                const int64_t row = row0 + v;
                const uint32_t* cw = (const uint32_t*)(codes + row * code_stride);
                float s = 0.f;
                int m = 0;
                for (int wd = 0; m < M; wd++) {
                    uint32_t word = cw[wd];
#pragma unroll
                    for (int b = 0; b < 4; b++, m++) {
                        if (m < M) s += T[m * ksub + ((word >> (8 * b)) & 0xff)];
                    }
                }
                float dis = by_residual ? dis0 + terms[row] + s : s;
                k1 = dis;
                k2 = ids[row];
                if (!key_admissible(k1)) {
                    k1 = WS_INF;
                    k2 = WS_NOID;
                }
            }
            wave_offer(qd, qi, k1, k2, thr_d, thr_i, k, lane);
        }
    }
    // merge the 4 wave queues
    md[w * 64 + lane] = qd;
    mi[w * 64 + lane] = qi;
    __syncthreads();
    if (w == 0) {
        float fd = WS_INF;
        long long fi = WS_NOID;
        float td = WS_INF;
        long long ti = WS_NOID;
        for (int ww = 0; ww < 4; ww++) {
            float cd = lane < k ? md[ww * 64 + lane] : WS_INF;
            long long ci = lane < k ? mi[ww * 64 + lane] : WS_NOID;
            wave_offer(fd, fi, cd, ci, td, ti, k, lane);
        }
        if (lane < k) {
            float dis;
            long long id;
            from_key(1, fd, fi, dis, id);
            D[q * k + lane] = dis;
            I[q * k + lane] = id;
        }
    }
}

// ---------------------------------------------------------------- scan v2
constexpr int PQ_PF = 3;  // code batches in flight per wave
// One workgroup (4 waves) per query, LUT T[m][j] (M x 256 f32) in LDS; the
// per-code work is M LDS gathers + adds (LDS-gather bound).  M is a template
// parameter (fully unrolled, codes read as 16-B words).  Selection: each wave
// keeps a 64-slot sorted queue; a code whose distance is <= the queue's k-th
// is appended to a per-wave LDS buffer (ballot compaction) and the buffer is
// folded into the queue 64 at a time, so the sorting network runs only for
// the few codes that can still enter the top-k.  Ties: (dis, id) order.
template <int M>
__global__ __launch_bounds__(256) void k_ivfpq_scan_m(
        const float* __restrict__ x, int ldx, const float* __restrict__ pq_cent, int dsub,
        const uint8_t* __restrict__ codes, const float* __restrict__ terms,
        const int64_t* __restrict__ ids, const uint32_t* __restrict__ list_off,
        const uint32_t* __restrict__ list_len, int nlist, const int32_t* __restrict__ assign,
        const float* __restrict__ coarse_dis, const uint32_t* __restrict__ lim,
        const uint8_t* __restrict__ sel, int nprobe, int k, int by_residual,
        float* __restrict__ D, int64_t* __restrict__ I) {
    constexpr int CS = (M + 3) & ~3;  // code stride (bytes)
    constexpr int NW = CS / 4;        // 32-bit words per code
    __shared__ float T[M * 256];
    // phase-shared scratch (4 KB): the query during the LUT build, then the
    // per-wave candidate buffers, then the final cross-wave merge
    __shared__ __attribute__((aligned(16))) uint8_t scratch[4 * 128 * 8];
    float* xs = reinterpret_cast<float*>(scratch);                          // [512] (d <= 512)
    float (*bd)[128] = reinterpret_cast<float (*)[128]>(scratch);           // [4][128]
    uint32_t (*br)[128] = reinterpret_cast<uint32_t (*)[128]>(scratch + 2048);  // [4][128]
    float (*md)[64] = reinterpret_cast<float (*)[64]>(scratch);             // [4][64]
    long long (*mi)[64] = reinterpret_cast<long long (*)[64]>(scratch + 1024);  // [4][64]
    __shared__ uint32_t p_len[64], p_off[64];
    __shared__ float p_d0[64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t q = blockIdx.x;
    const int d = M * dsub;
    for (int j = t; j < d; j += 256) xs[j] = x[q * ldx + j];
    __syncthreads();
    // LUT: table 1 (by_residual): -2 <x_m, c_mj>; otherwise ||x_m - c_mj||^2
    for (int e = t; e < M * 256; e += 256) {
        const int m = e >> 8;
        const float* c = pq_cent + (int64_t)e * dsub;
        const float* xm = xs + m * dsub;
        float acc = 0.f;
        if (by_residual) {
            for (int i = 0; i < dsub; i++) acc = fmaf(xm[i], c[i], acc);
            T[e] = -2.f * acc;
        } else {
            for (int i = 0; i < dsub; i++) {
                const float df = xm[i] - c[i];
                acc = fmaf(df, df, acc);
            }
            T[e] = acc;
        }
    }
    __syncthreads();

    // per-probe geometry in LDS (one round trip for all probes)
    if (t < nprobe) {
        const int lst = assign[q * nprobe + t];
        const bool ok = lst >= 0 && lst < nlist;
        // max_codes: a prefix of the list (lim), faiss/IndexIVF.cpp:546-550
        p_len[t] = ok ? (lim ? min(lim[q * nprobe + t], list_len[lst]) : list_len[lst]) : 0u;
        p_off[t] = ok ? list_off[lst] : 0u;
        p_d0[t] = by_residual ? coarse_dis[q * nprobe + t] : 0.f;
    }
    __syncthreads();

    float qd = WS_INF;
    long long qi = WS_NOID;
    float thr = WS_INF;  // the queue's k-th distance
    int bc = 0;          // buffered candidates (wave-uniform)
    auto fold = [&](int cnt) {
        // lanes < cnt take buffered entries 0..cnt-1
        float cd = WS_INF;
        long long ci = WS_NOID;
        if (lane < cnt) {
            cd = bd[w][lane];
            ci = (long long)ids[br[w][lane]];
        }
        wave_sort64(cd, ci, lane);
        wave_merge64(qd, qi, cd, ci, lane);
        thr = __shfl(qd, k - 1);
    };
    // flattened (probe, 64-code batch) sequence of this wave: probes w, w+4, ...
    // A ring of PQ_PF batches is in flight: a slot is refilled with the batch
    // PQ_PF ahead as soon as it has been gathered (HBM latency hidden across
    // batches and lists).
    auto advance = [&](int& rr, int& vv) {
        vv += 64;
        while (rr < nprobe && vv >= (int)p_len[rr]) {
            rr += 4;
            vv = 0;
        }
    };
    auto load = [&](int rr, int vv, uint32_t (&wo)[NW], float& to, uint32_t& ro, bool& vo) {
        vo = rr < nprobe && vv + lane < (int)p_len[rr < nprobe ? rr : 0];
        ro = (rr < nprobe ? p_off[rr] : 0u) + (uint32_t)(vo ? vv + lane : 0);
        vo = vo && (!sel || sel[ro]);  // IDSelector (use_sel)
        const uint8_t* cp = codes + (size_t)ro * CS;
        if constexpr (NW % 4 == 0) {
#pragma unroll
            for (int i = 0; i < NW; i += 4) {
                const uint4 u = *(const uint4*)(cp + 4 * i);
                wo[i] = u.x;
                wo[i + 1] = u.y;
                wo[i + 2] = u.z;
                wo[i + 3] = u.w;
            }
        } else if constexpr (NW % 2 == 0) {
#pragma unroll
            for (int i = 0; i < NW; i += 2) {
                const uint2 u = *(const uint2*)(cp + 4 * i);
                wo[i] = u.x;
                wo[i + 1] = u.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < NW; i++) wo[i] = *(const uint32_t*)(cp + 4 * i);
        }
        to = by_residual ? terms[ro] : 0.f;
    };
    constexpr int PF = PQ_PF;
    uint32_t wd[PF][NW];
    float term[PF];
    uint32_t row[PF];
    bool valid[PF];
    int rs[PF];  // probe of each slot (nprobe: empty)
    int pr = w, pv = 0;  // next batch to load
    while (pr < nprobe && p_len[pr] == 0u) pr += 4;
#pragma unroll
    for (int sl = 0; sl < PF; sl++) {
        rs[sl] = pr;
        if (pr < nprobe) {
            load(pr, pv, wd[sl], term[sl], row[sl], valid[sl]);
            advance(pr, pv);
        } else {
            valid[sl] = false;
        }
    }
    while (rs[0] < nprobe) {
#pragma unroll
        for (int sl = 0; sl < PF; sl++) {
            if (rs[sl] >= nprobe) break;  // wave-uniform: the sequence has ended
            float sum = 0.f;
#pragma unroll
            for (int m = 0; m < M; m++)
                sum += T[m * 256 + ((wd[sl][m >> 2] >> (8 * (m & 3))) & 0xffu)];
            const float dis = by_residual ? p_d0[rs[sl]] + term[sl] + sum : sum;
            const bool pass = valid[sl] && key_admissible(dis) && dis <= thr;
            const uint32_t prow = row[sl];
            // refill this slot with the batch PF ahead
            rs[sl] = pr;
            if (pr < nprobe) {
                load(pr, pv, wd[sl], term[sl], row[sl], valid[sl]);
                advance(pr, pv);
            } else {
                valid[sl] = false;
            }
            const unsigned long long pm = __ballot(pass);
            if (pm) {
                const int pos = bc + __popcll(pm & ((1ull << lane) - 1ull));
                if (pass) {
                    bd[w][pos] = dis;
                    br[w][pos] = prow;
                }
                bc += __popcll(pm);
                if (bc >= 64) {
                    fold(64);
                    // keep the overflow (< 64 entries) at the front
                    const bool mv = lane < bc - 64;
                    const float od = mv ? bd[w][64 + lane] : 0.f;
                    const uint32_t orw = mv ? br[w][64 + lane] : 0u;
                    if (mv) {
                        bd[w][lane] = od;
                        br[w][lane] = orw;
                    }
                    bc -= 64;
                }
            }
        }
    }
    if (bc > 0) fold(bc);
    __syncthreads();  // the candidate buffers are reused for the merge
    // merge the 4 wave queues
    md[w][lane] = qd;
    mi[w][lane] = qi;
    __syncthreads();
    if (w == 0) {
        float fd = WS_INF, td = WS_INF;
        long long fi = WS_NOID, ti = WS_NOID;
        for (int ww = 0; ww < 4; ww++) {
            const float cd = lane < k ? md[ww][lane] : WS_INF;
            const long long ci = lane < k ? mi[ww][lane] : WS_NOID;
            wave_offer(fd, fi, cd, ci, td, ti, k, lane);
        }
        if (lane < k) {
            float dis;
            long long id;
            from_key(1, fd, fi, dis, id);
            D[q * k + lane] = dis;
            I[q * k + lane] = id;
        }
    }
}

void ivfpq_scan(const float* x, int ldx, const float* pq_centroids, int M, int ksub, int dsub,
                const uint8_t* codes, const float* terms, const int64_t* ids,
                const uint32_t* list_off, const uint32_t* list_len, int nlist,
                const int32_t* assign, const float* coarse_dis, const uint32_t* lim,
                const uint8_t* sel, int64_t n, int nprobe, int k, int by_residual, float* D,
                int64_t* I, hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT_MSG(k >= 1 && k <= kMaxK, "k must be in [1, 64] on this path");
    FAISS_THROW_IF_NOT_MSG(nprobe >= 1 && nprobe <= 64, "nprobe must be in [1, 64] on this path");
    FAISS_THROW_IF_NOT_MSG(ksub == 256, "only 8-bit PQ codes are supported on this path");
    const int code_stride = (int)roundup((size_t)M, 4);
    if (M * dsub <= 512 && getenv("FAISS_AMD_PQ_SCAN_V1") == nullptr) {
#define PQ_M(MV)                                                                               \
    if (M == MV) {                                                                             \
        k_ivfpq_scan_m<MV><<<dim3((unsigned)n), dim3(256), 0, s>>>(                            \
                x, ldx, pq_centroids, dsub, codes, terms, ids, list_off, list_len, nlist, assign, \
                coarse_dis, lim, sel, nprobe, k, by_residual, D, I);                           \
        HIP_LAUNCH_CHECK();                                                                    \
        return;                                                                                \
    }
        PQ_M(8) PQ_M(16) PQ_M(32) PQ_M(48) PQ_M(64)
#undef PQ_M
    }
    size_t lds = sizeof(float) * ((size_t)M * ksub + roundup((size_t)M * dsub, 4) + 256) +
                 sizeof(long long) * 256;
    FAISS_THROW_IF_NOT_MSG(lds <= 160 * 1024, "PQ LUT does not fit in LDS");
    k_ivfpq_scan<<<dim3((unsigned)n), dim3(256), lds, s>>>(
            x, ldx, pq_centroids, M, ksub, dsub, codes, code_stride, terms, ids, list_off,
            list_len, nlist, assign, coarse_dis, lim, sel, nprobe, k, by_residual, D, I);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- terms
__global__ void k_ivfpq_terms(const uint8_t* __restrict__ codes, int code_stride,
                              const uint32_t* __restrict__ row_list, int64_t nrows,
                              const float* __restrict__ cent, int ldcent,
                              const float* __restrict__ pq_cent, int M, int ksub, int dsub,
                              float* __restrict__ terms) {
    int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    uint32_t l = row_list[row];
    if (l == 0xffffffffu) {
        terms[row] = 0.f;
        return;
    }
    const float* yc = cent + (int64_t)l * ldcent;
    const uint8_t* c = codes + row * code_stride;
    float s = 0.f;
    for (int m = 0; m < M; m++) {
        const float* cm = pq_cent + ((int64_t)m * ksub + c[m]) * dsub;
        const float* ym = yc + m * dsub;
        float nrm = 0.f, ip = 0.f;
        for (int i = 0; i < dsub; i++) {
            nrm = fmaf(cm[i], cm[i], nrm);
            ip = fmaf(ym[i], cm[i], ip);
        }
        s += fmaf(2.f, ip, nrm);
    }
    terms[row] = s;
}

void ivfpq_terms(const uint8_t* codes, const uint32_t* row_list, int64_t nrows,
                 const float* centroids, int ldcent, const float* pq_centroids, int M, int ksub,
                 int dsub, float* terms, hipStream_t s) {
    if (nrows <= 0) return;
    const int code_stride = (int)roundup((size_t)M, 4);
    k_ivfpq_terms<<<dim3((unsigned)cdiv(nrows, 256)), dim3(256), 0, s>>>(
            codes, code_stride, row_list, nrows, centroids, ldcent, pq_centroids, M, ksub, dsub,
            terms);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- encode
// ProductQuantizer::compute_codes for dsub < 16 (faiss/impl/ProductQuantizer.cpp:
// 398-427 -> compute_code :195-271): per sub-quantizer the nearest of the ksub
// centroids by fvec_L2sqr_ny_nearest (faiss/utils/distances_simd.cpp:2298-2317).
//   dsub 2 / 4 / 8: the AVX2 fvec_L2sqr_ny_nearest_D{2,4,8} (:1908-2271):
//     distances in the ny fma-chain order; 8 lanes (j mod 8) keep their
//     minimum with `old < new ? old : new` (an equal later distance takes the
//     lane), then lanes 0..7 are scanned with a strict `>`.
//   other dsub: fvec_L2sqr_ny (D1 / D12 kernels, else fvec_L2sqr order) and
//     the first strict minimum.
// dsub >= 16 takes the reference's BLAS branch (compute_distance_tables via
// sgemm), whose order is MKL's; the fvec_L2sqr order is used there.
// Thread per (vector, sub-quantizer); the sub-centroids of m live in LDS.
template <int DS>
__global__ __launch_bounds__(256) void k_pq_encode(const float* __restrict__ x, int ldx,
                                                   int64_t n, const int32_t* __restrict__ assign,
                                                   const float* __restrict__ cent, int ldcent,
                                                   const float* __restrict__ pq_cent, int M,
                                                   int ksub, uint8_t* __restrict__ codes,
                                                   int code_stride) {
    extern __shared__ float cs[];  // [ksub * DS]
    const int m = blockIdx.y;
    for (int e = threadIdx.x; e < ksub * DS; e += 256)
        cs[e] = pq_cent[(int64_t)m * ksub * DS + e];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float r[DS];
#pragma unroll
    for (int j = 0; j < DS; j++) {
        float v = x[i * ldx + m * DS + j];
        if (cent) v -= cent[(int64_t)assign[i] * ldcent + m * DS + j];
        r[j] = v;
    }
    constexpr bool lanes = DS == 2 || DS == 4 || DS == 8;
    int bj = 0;
    if constexpr (lanes) {
        float lmin[8];
        int lidx[8];
#pragma unroll
        for (int l = 0; l < 8; l++) {
            lmin[l] = HUGE_VALF;
            lidx[l] = 0;
        }
        for (int j0 = 0; j0 < ksub; j0 += 8)
#pragma unroll
            for (int l = 0; l < 8; l++) {
                const float s = ny_entry_c<true, DS>(r, cs + (j0 + l) * DS);
                const bool keep = lmin[l] < s;
                lidx[l] = keep ? lidx[l] : j0 + l;
                lmin[l] = keep ? lmin[l] : s;
            }
        float cur = HUGE_VALF;
#pragma unroll
        for (int l = 0; l < 8; l++)
            if (cur > lmin[l]) {
                cur = lmin[l];
                bj = lidx[l];
            }
    } else {
        float best = HUGE_VALF;
        for (int j = 0; j < ksub; j++) {
            const float s = ny_entry<true>(r, cs + j * DS, DS);
            if (s < best) {
                best = s;
                bj = j;
            }
        }
    }
    codes[i * code_stride + m] = (uint8_t)bj;
}

void pq_encode(const float* x, int ldx, int64_t n, const int32_t* assign, const float* centroids,
               int ldcent, const float* pq_centroids, int M, int ksub, int dsub, uint8_t* codes,
               hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT(ksub <= 256);
    // the 8-lane argmin assumes whole 8-row groups (ksub = 256 for nbits = 8)
    FAISS_THROW_IF_NOT(ksub % 8 == 0);
    const int code_stride = (int)roundup((size_t)M, 4);
    const dim3 grid((unsigned)cdiv(n, 256), (unsigned)M);
    const size_t lds = sizeof(float) * ksub * dsub;
#define ENC(DS)                                                                             \
    case DS:                                                                                \
        k_pq_encode<DS><<<grid, dim3(256), lds, s>>>(x, ldx, n, assign, centroids, ldcent,  \
                                                     pq_centroids, M, ksub, codes,          \
                                                     code_stride);                          \
        break;
    switch (dsub) {
        ENC(1) ENC(2) ENC(3) ENC(4) ENC(5) ENC(6) ENC(8) ENC(10) ENC(12) ENC(16) ENC(24)
        ENC(32)
        default:
            FAISS_THROW_FMT("PQ encode: dsub = %d not supported on this path", dsub);
    }
#undef ENC
    HIP_LAUNCH_CHECK();
}

}  // namespace kern
}  // namespace faiss_amd
