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

// Exact reference-order distance of the row `grow` each lane names (valid
// lanes only), 16 rows per pass, 4 lanes per row: lane j' of row g owns the
// reference's partial sums c[2j'] and c[2j'+1] (dims 8m + 2j' + {0,1}) and
// loads those float2 pairs straight from the arena — one load instruction
// covers 16 rows x 32 contiguous bytes, the 4 lanes of a row complete its
// cache lines.  x_j = c_j + c_{j+4}, then (x0 + x2) + (x1 + x3) (ref_arith.h
// order), then the epilogue dims.  No LDS staging and no barriers.  XM = max dims / 8
// (the query copy xr holds at least 8 XM floats).  Used by the IVF re-rank
// (kernels_ivf_mfma.hip) and the HNSW hop (kernels_hnsw.hip).
template <bool L2, int XM>
__device__ __forceinline__ float ref_rows64_4lane(const float* xr /* LDS copy of the query */,
                                                    const float* __restrict__ xq,
                                                    const float* __restrict__ codes, int ldc,
                                                    int d, uint32_t grow, bool valid, int lane) {
    const int g = lane >> 2, jp = lane & 3;
    const int n8 = d & ~7, nm = n8 >> 3;
    const unsigned long long vm = __ballot(valid);
    float out = 0.f;
#pragma unroll 1
    for (int p = 0; p < 4; p++) {
        if (((vm >> (16 * p)) & 0xffffull) == 0ull) continue;  // wave-uniform
        const uint32_t rg = __shfl(grow, 16 * p + g);
        const bool rv = (vm >> (16 * p + g)) & 1ull;
        const float* yr = codes + (int64_t)(rv ? rg : 0u) * ldc;
        float2 yv[XM];
#pragma unroll
        for (int m = 0; m < XM; m++)
            yv[m] = m < nm ? *(const float2*)(yr + 8 * m + 2 * jp) : make_float2(0.f, 0.f);
        const float* xj = xr + 2 * jp;
        float ca = 0.f, cb = 0.f;
#pragma unroll
        for (int m = 0; m < XM; m++) {
            const float2 xv = *(const float2*)(xj + 8 * m);
            const float ta = ref_term_fma<L2>(xv.x, yv[m].x, ca);
            const float tb = ref_term_fma<L2>(xv.y, yv[m].y, cb);
            ca = m < nm ? ta : ca;
            cb = m < nm ? tb : cb;
        }
        ca += __shfl_xor(ca, 2);
        cb += __shfl_xor(cb, 2);
        ca += __shfl_xor(ca, 1);  // x0 + x2
        cb += __shfl_xor(cb, 1);  // x1 + x3
        float r = ca + cb;
        if (n8 < d) {
            int i = n8;
            if (d - n8 >= 4) {
                const float e0 = ref_term<L2>(xq[n8], yr[n8]), e1 = ref_term<L2>(xq[n8 + 1], yr[n8 + 1]);
                const float e2 = ref_term<L2>(xq[n8 + 2], yr[n8 + 2]);
                const float e3 = ref_term<L2>(xq[n8 + 3], yr[n8 + 3]);
                r = r + ((e0 + e2) + (e1 + e3));
                i += 4;
            }
            for (; i < d; i++) r = ref_term_fma<L2>(xq[i], yr[i], r);
        }
        const float got = __shfl(r, 4 * (lane & 15));
        if ((lane >> 4) == p) out = got;
    }
    return out;
}

// ref_rows64_4lane for rows compacted to the low lanes (valid lanes 0..nv-1)
// with the loads of PB passes issued together: one memory round trip per PB
// passes instead of per pass (a hop of ~40 rows: 2 round trips at PB = 2
// instead of 3), at PB x 2 XM VGPRs of row data.
template <bool L2, int XM, int PB>
__device__ __forceinline__ float ref_rows64_4lane_pb(const float* xr, const float* __restrict__ xq,
                                                     const float* __restrict__ codes, int ldc,
                                                     int d, uint32_t grow, int nv, int lane) {
    const int g = lane >> 2, jp = lane & 3;
    const int n8 = d & ~7, nm = n8 >> 3;
    const int npass = (nv + 15) >> 4;
    float out = 0.f;
#pragma unroll 1
    for (int p0 = 0; p0 < npass; p0 += PB) {
        float2 yv[PB][XM];
        const float* yr[PB];
        // rows of a pass beyond the last one read row 0 (their results are
        // never used): every load is unconditional, one base per row
        const bool full = nm == XM;  // wave-uniform: no per-m selects
#pragma unroll
        for (int b = 0; b < PB; b++) {
            const int p = p0 + b;
            const uint32_t rg = __shfl(grow, (16 * p + g) & 63);
            const bool rv = p < npass && 16 * p + g < nv;
            yr[b] = codes + (int64_t)(rv ? rg : 0u) * ldc;
            if (full) {
#pragma unroll
                for (int m = 0; m < XM; m++) yv[b][m] = *(const float2*)(yr[b] + 8 * m + 2 * jp);
            } else {
#pragma unroll
                for (int m = 0; m < XM; m++)
                    yv[b][m] = m < nm ? *(const float2*)(yr[b] + 8 * m + 2 * jp)
                                      : make_float2(0.f, 0.f);
            }
        }
        const float* xj = xr + 2 * jp;
#pragma unroll
        for (int b = 0; b < PB; b++) {
            const int p = p0 + b;
            if (p >= npass) break;  // wave-uniform
            float ca = 0.f, cb = 0.f;
            if (full) {
#pragma unroll
                for (int m = 0; m < XM; m++) {
                    const float2 xv = *(const float2*)(xj + 8 * m);
                    ca = ref_term_fma<L2>(xv.x, yv[b][m].x, ca);
                    cb = ref_term_fma<L2>(xv.y, yv[b][m].y, cb);
                }
            } else {
#pragma unroll
                for (int m = 0; m < XM; m++) {
                    const float2 xv = *(const float2*)(xj + 8 * m);
                    const float ta = ref_term_fma<L2>(xv.x, yv[b][m].x, ca);
                    const float tb = ref_term_fma<L2>(xv.y, yv[b][m].y, cb);
                    ca = m < nm ? ta : ca;
                    cb = m < nm ? tb : cb;
                }
            }
            ca += __shfl_xor(ca, 2);
            cb += __shfl_xor(cb, 2);
            ca += __shfl_xor(ca, 1);
            cb += __shfl_xor(cb, 1);
            float r = ca + cb;
            if (n8 < d) {
                const float* y = yr[b];
                int i = n8;
                if (d - n8 >= 4) {
                    const float e0 = ref_term<L2>(xq[n8], y[n8]), e1 = ref_term<L2>(xq[n8 + 1], y[n8 + 1]);
                    const float e2 = ref_term<L2>(xq[n8 + 2], y[n8 + 2]);
                    const float e3 = ref_term<L2>(xq[n8 + 3], y[n8 + 3]);
                    r = r + ((e0 + e2) + (e1 + e3));
                    i += 4;
                }
                for (; i < d; i++) r = ref_term_fma<L2>(xq[i], y[i], r);
            }
            const float got = __shfl(r, 4 * (lane & 15));
            if ((lane >> 4) == p) out = got;
        }
    }
    return out;
}

// ref_rows64_4lane_pb with 8 lanes per row and 8 rows per pass: lane j of a
// row owns the reference's partial sum c_j (dims 8m + j); x_j = c_j + c_{j+4}
// by a lane swap, then (x0 + x2) + (x1 + x3) (ref_arith.h order), then the
// epilogue dims.  XM row floats per lane and pass (half of the 4-lane form's
// registers), one memory round trip per pass.
template <bool L2, int XM>
__device__ __forceinline__ float ref_rows64_8lane(const float* xr, const float* __restrict__ xq,
                                                  const float* __restrict__ codes, int ldc, int d,
                                                  uint32_t grow, int nv, int lane) {
    const int g = lane >> 3, j = lane & 7;
    const int n8 = d & ~7, nm = n8 >> 3;
    const int npass = (nv + 7) >> 3;
    float out = 0.f;
#pragma unroll 1
    for (int p = 0; p < npass; p++) {
        const uint32_t rg = __shfl(grow, (8 * p + g) & 63);
        const bool rv = 8 * p + g < nv;
        const float* yr = codes + (int64_t)(rv ? rg : 0u) * ldc;
        float yv[XM];
#pragma unroll
        for (int m = 0; m < XM; m++) yv[m] = m < nm ? yr[8 * m + j] : 0.f;
        float c = 0.f;
#pragma unroll
        for (int m = 0; m < XM; m++) {
            const float t = ref_term_fma<L2>(xr[8 * m + j], yv[m], c);
            c = m < nm ? t : c;
        }
        const float x = c + __shfl_xor(c, 4);   // x_j = c_j + c_{j+4}
        const float y = x + __shfl_xor(x, 2);   // x0 + x2, x1 + x3
        float r = y + __shfl_xor(y, 1);         // (x0 + x2) + (x1 + x3)
        if (n8 < d) {
            int i = n8;
            if (d - n8 >= 4) {
                const float e0 = ref_term<L2>(xq[n8], yr[n8]), e1 = ref_term<L2>(xq[n8 + 1], yr[n8 + 1]);
                const float e2 = ref_term<L2>(xq[n8 + 2], yr[n8 + 2]);
                const float e3 = ref_term<L2>(xq[n8 + 3], yr[n8 + 3]);
                r = r + ((e0 + e2) + (e1 + e3));
                i += 4;
            }
            for (; i < d; i++) r = ref_term_fma<L2>(xq[i], yr[i], r);
        }
        const float got = __shfl(r, 8 * (lane & 7));
        if ((lane >> 3) == p) out = got;
    }
    return out;
}

}  // namespace kern
}  // namespace faiss_amd
