// kernels_pq.hip — IVF-PQ per-code terms (read by the MFMA filter) and PQ
// encoding for gfx950.
//
// Reference: faiss/IndexIVFPQ.cpp
//   * precomputed "table 1" term 2 (:332-459): ||y_R||^2 + 2 <y_C, y_R>, folded
//     into one f32 per stored code when the lists are uploaded; the MFMA
//     filter (kernels_pq_mfma.hip) adds it to its approximate -2 <x, y_R>.
//   * encoding: IndexIVFPQ::encode_vectors -> ProductQuantizer::compute_codes.
// Search-time distances in the reference's exact arithmetic live in
// kernels_exact.hip (general scan) and kernels_ivf_mfma.hip (re-rank).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "ref_arith.h"
#include "pq_ref.h"
#include "wave_select.h"

namespace faiss_amd {
namespace kern {

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
    k_ivfpq_terms<<<kgrid(cdiv(nrows, 256), 256), dim3(256), 0, s>>>(
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

// |x_q - c_l|^2 (fvec_L2sqr order) of every (query, probe) pair with l >= 0
__global__ void k_pair_l2(const float* __restrict__ x, int ldx, const float* __restrict__ cent,
                          int ldc, int d, const int32_t* __restrict__ assign, int64_t n, int np,
                          float* __restrict__ out) {
    GRID_STRIDE(e, n * np) {
        const int32_t l = assign[e];
        out[e] = l >= 0 ? ref_l2(x + (e / np) * ldx, cent + (int64_t)l * ldc, d) : 0.f;
    }
}
void pair_l2(const float* x, int ldx, const float* cent, int ldc, int d, const int32_t* assign,
             int64_t n, int np, float* out, hipStream_t s) {
    if (n <= 0 || np <= 0) return;
    k_pair_l2<<<stride_grid(n * np, 256), dim3(256), 0, s>>>(x, ldx, cent, ldc, d, assign, n,
                                                            np, out);
    HIP_LAUNCH_CHECK();
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
