// pq_ref.h — the reference's fp32 evaluation order for IVF-PQ distances
// (AVX2 build of faiss, pinned bit-for-bit by tests/test_ref_fixtures.py
// against arrays produced by the reference library compiled from source).
//
// * Table entries, fvec_inner_products_ny / fvec_L2sqr_ny
//   (faiss/utils/distances_simd.cpp:1362-1410): dsub 1 -> one rounded term;
//   dsub 2/4/8 -> the AVX2 fvec_op_ny_D{2,4,8} specialisations (:579-702,
//   :845-975, :1167-1341): acc = t0 (rounded), then fma over dims 1..dsub-1;
//   dsub 12 -> fvec_op_ny_D12 (:1344-1360); other dsub -> fvec_L2sqr /
//   fvec_inner_product (ref_arith.h order).
// * Table 1 (faiss/IndexIVFPQ.cpp:408-432, :645-653, fvec_madd = one fma):
//   P = fma(2, <y_C,m, c>, |c|^2), sim = fma(-2, <x_m, c>, P).
// * Code sum, distance_single_code / distance_four_codes with PQDecoder8
//   (faiss/impl/code_distance/code_distance-avx2.h:42-119, :253-347):
//   M = 4 -> (t0+t2)+(t1+t3); M = 8 or M >= 16 -> 8 lanes, lane l sums
//   t[m] for m = l (mod 8), m < m16 (m16 = 8 for M = 8, else 16*floor(M/16)),
//   reduced ((p0+p4)+(p2+p6))+((p1+p5)+(p3+p7)), then t[m16..M) added in
//   order; other M < 16 -> 0 + t0 + t1 + ... in order.
#pragma once

#include <hip/hip_runtime.h>

#include "ref_arith.h"

namespace faiss_amd {
namespace kern {

// fvec_L2sqr / fvec_inner_product / fvec_norm_L2sqr order (ref_arith.h) with
// scalar loads, for rows without 16-B alignment (PQ sub-vectors)
template <bool L2>
__device__ __forceinline__ float ref_dist_s(const float* __restrict__ x,
                                            const float* __restrict__ y, int d) {
    float c[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int n8 = d & ~7;
    for (int i = 0; i < n8; i += 8)
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = ref_term_fma<L2>(x[i + j], y[i + j], c[j]);
    float r = ((c[0] + c[4]) + (c[2] + c[6])) + ((c[1] + c[5]) + (c[3] + c[7]));
    int i = n8;
    if (d - n8 >= 4) {
        r = r + ((ref_term<L2>(x[i], y[i]) + ref_term<L2>(x[i + 2], y[i + 2])) +
                 (ref_term<L2>(x[i + 1], y[i + 1]) + ref_term<L2>(x[i + 3], y[i + 3])));
        i += 4;
    }
    for (; i < d; i++) r = ref_term_fma<L2>(x[i], y[i], r);
    return r;
}

template <bool L2>
__device__ __forceinline__ float ny_entry(const float* __restrict__ x, const float* __restrict__ y,
                                          int dsub) {
    switch (dsub) {
        case 1:
            return ref_term<L2>(x[0], y[0]);
        case 2:
        case 4:
        case 8: {
            float acc = ref_term<L2>(x[0], y[0]);
            for (int j = 1; j < dsub; j++) acc = ref_term_fma<L2>(x[j], y[j], acc);
            return acc;
        }
        case 12: {
            float a[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                a[j] = (ref_term<L2>(x[j], y[j]) + ref_term<L2>(x[4 + j], y[4 + j])) +
                       ref_term<L2>(x[8 + j], y[8 + j]);
            return (a[0] + a[2]) + (a[1] + a[3]);
        }
        default:
            return ref_dist_s<L2>(x, y, dsub);
    }
}

// compile-time dsub (2 / 4 / 8): the fma chain of the AVX2 ny kernels
template <bool L2, int DS>
__device__ __forceinline__ float ny_entry_c(const float* __restrict__ x,
                                            const float* __restrict__ y) {
    static_assert(DS == 1 || DS == 2 || DS == 4 || DS == 8, "chain form only");
    float acc = ref_term<L2>(x[0], y[0]);
#pragma unroll
    for (int j = 1; j < DS; j++) acc = ref_term_fma<L2>(x[j], y[j], acc);
    return acc;
}

__device__ __forceinline__ float reduce8(const float* p) {
    return ((p[0] + p[4]) + (p[2] + p[6])) + ((p[1] + p[5]) + (p[3] + p[7]));
}

// 16 * floor(M / 16), or 8 for M == 8 (the lanes' part of the code sum)
__device__ __forceinline__ int pq_lane_span(int M) { return M == 8 ? 8 : (M / 16) * 16; }

// Code sum in the reference order; T(m) returns the table entry of
// sub-quantizer m for this code.
template <class TF>
__device__ __forceinline__ float pq_code_sum(int M, TF&& T) {
    if (M == 4) return (T(0) + T(2)) + (T(1) + T(3));
    const int m16 = pq_lane_span(M);
    float r = 0.f;
    int m = 0;
    if (m16 > 0) {
        float p[8];
#pragma unroll
        for (int l = 0; l < 8; l++) p[l] = T(l);
        for (m = 8; m < m16; m += 8)
#pragma unroll
            for (int l = 0; l < 8; l++) p[l] += T(m + l);
        r = reduce8(p);
    }
    for (; m < M; m++) r += T(m);
    return r;
}

}  // namespace kern
}  // namespace faiss_amd
