// ref_arith.h — the reference's fp32 evaluation order for fine distances.
//
// faiss/utils/distances_simd.cpp:220-230 (fvec_L2sqr), the matching
// fvec_inner_product / fvec_norm_L2sqr and fvec_L2sqr_batch_4 (:268-300) are
// plain loops compiled with FAISS_PRAGMA_IMPRECISE_FUNCTION_BEGIN
// (faiss/impl/platform_macros.h:176-181: GCC associative-math) under the
// AVX2 flags (faiss/CMakeLists.txt:251).  GCC turns every one of them into
// the same order, pinned bit-for-bit against the reference sources compiled
// by oracle/ref (tests/test_oracle_golden.py):
//   * 8 accumulators, lane j takes terms i = 8m + j, i < n8 = d & ~7 (fma);
//   * reduce (j, j+4), then (j, j+2), then (0, 1);
//   * if d - n8 >= 4: the next 4 terms rounded alone, reduced (0,2)(1,3),(0,1)
//     and added to the result;
//   * the last d % 4 terms fma'd onto the result in order.
// Term = (x-y)^2 for L2 (difference rounded, then fma), x*y for IP.
#pragma once

#include <hip/hip_runtime.h>

namespace faiss_amd {
namespace kern {

template <bool L2>
__device__ __forceinline__ float ref_term_fma(float a, float b, float acc) {
    if (L2) {
        const float t = a - b;
        return fmaf(t, t, acc);
    }
    return fmaf(a, b, acc);
}
template <bool L2>
__device__ __forceinline__ float ref_term(float a, float b) {
    if (L2) {
        const float t = a - b;
        return t * t;
    }
    return a * b;
}

// a, b: 16-byte aligned rows of d floats
template <bool L2>
__device__ __forceinline__ float ref_dist(const float* __restrict__ a,
                                          const float* __restrict__ b, int d) {
    float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, c4 = 0.f, c5 = 0.f, c6 = 0.f, c7 = 0.f;
    const int n8 = d & ~7;
#pragma unroll 4
    for (int i = 0; i < n8; i += 8) {
        const float4 a0 = *(const float4*)(a + i), a1 = *(const float4*)(a + i + 4);
        const float4 b0 = *(const float4*)(b + i), b1 = *(const float4*)(b + i + 4);
        c0 = ref_term_fma<L2>(a0.x, b0.x, c0);
        c1 = ref_term_fma<L2>(a0.y, b0.y, c1);
        c2 = ref_term_fma<L2>(a0.z, b0.z, c2);
        c3 = ref_term_fma<L2>(a0.w, b0.w, c3);
        c4 = ref_term_fma<L2>(a1.x, b1.x, c4);
        c5 = ref_term_fma<L2>(a1.y, b1.y, c5);
        c6 = ref_term_fma<L2>(a1.z, b1.z, c6);
        c7 = ref_term_fma<L2>(a1.w, b1.w, c7);
    }
    const float x0 = c0 + c4, x1 = c1 + c5, x2 = c2 + c6, x3 = c3 + c7;
    float r = (x0 + x2) + (x1 + x3);
    int i = n8;
    if (d - n8 >= 4) {
        const float4 av = *(const float4*)(a + n8), bv = *(const float4*)(b + n8);
        const float e0 = ref_term<L2>(av.x, bv.x), e1 = ref_term<L2>(av.y, bv.y);
        const float e2 = ref_term<L2>(av.z, bv.z), e3 = ref_term<L2>(av.w, bv.w);
        r = r + ((e0 + e2) + (e1 + e3));
        i += 4;
    }
    for (; i < d; i++) r = ref_term_fma<L2>(a[i], b[i], r);
    return r;
}

__device__ __forceinline__ float ref_l2(const float* a, const float* b, int d) {
    return ref_dist<true>(a, b, d);
}
__device__ __forceinline__ float ref_ip(const float* a, const float* b, int d) {
    return ref_dist<false>(a, b, d);
}
__device__ __forceinline__ float ref_norm(const float* a, int d) { return ref_dist<false>(a, a, d); }

// Incremental form for tiles that stream dims in chunks of 8: feed the 8
// terms of dims [i, i+8) for i < n8, then finish with the epilogue/tail dims.
struct RefAcc8 {
    float c[8];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = 0.f;
    }
    __device__ __forceinline__ float reduce() const {
        const float x0 = c[0] + c[4], x1 = c[1] + c[5], x2 = c[2] + c[6], x3 = c[3] + c[7];
        return (x0 + x2) + (x1 + x3);
    }
};

}  // namespace kern
}  // namespace faiss_amd
