// bf3.h — shared pieces of the bf16x3 MFMA filters (IVF-Flat list scan and
// coarse quantizer).
//
// Every f32 operand is split x = xh + xl (+ xr) with xh = bf16(x),
// xl = bf16(x - xh), |xr| <= 2^-16 |x|; <x,y> ~ xh.yh + xh.yl + xl.yh on
// v_mfma_f32_32x32x16_bf16 (products exact in f32, f32 accumulation).
//   |ip_approx - ip| <= (3.1 * 2^-16 + 3 d u) sum |x_i y_i|,   u = 2^-24.
// Callers turn that into a certified margin (bf3_coef) and re-rank the
// candidates the margin cannot separate with the exact f32 evaluation.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "wave_select.h"

namespace faiss_amd {
namespace kern {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BQ = 64;    // queries per work item (IVF-PQ filter)
constexpr int FQ = 128;   // queries per work item (IVF-Flat filter)
constexpr int BV = 64;    // database rows per tile
constexpr int BDM = 128;  // max padded dim (multiple of 16)

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Per-thread sorted queue of the KT smallest 32-bit keys (branchless).
template <int KT>
struct ThreadQueue32 {
    uint32_t q[KT];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int i = 0; i < KT; i++) q[i] = 0xffffffffu;
    }
    // q[i] <- median(q[i-1], c, q[i]) (= max(q[i-1], min(c, q[i])) on a sorted
    // queue): one v_med3_u32 per slot
    __device__ __forceinline__ void push(uint32_t c) {
#pragma unroll
        for (int i = KT - 1; i > 0; i--) q[i] = med3_u32(q[i - 1], c, q[i]);
        q[0] = min(c, q[0]);
    }
};

// 32-bit candidate keys: the approx value with its low `obits` bits replaced
// by the thread-local candidate ordinal.  L2 approx values are clamped at 0
// (the exact distance is >= 0 and max(0, .) is 1-Lipschitz, so the
// certification bound still holds) and their raw bits are already ordered;
// IP keys (-ip) use the sign-folded ordering.  decode_lo / decode_hi bracket
// the approx value whatever the ordinal.
template <bool L2>
__device__ __forceinline__ uint32_t key_encode(float a, uint32_t lowmask, uint32_t ord) {
    const uint32_t bits = L2 ? __float_as_uint(fmaxf(a, 0.f)) : ordered_f32(a);
    return (bits & ~lowmask) | ord;
}
// key_encode in two steps for the filters' inner loop: the clamped / folded
// value bits, then the ordinal inserted by one v_bfi_b32 (ord < 2^obits)
template <bool L2>
__device__ __forceinline__ uint32_t key_bits(float a) {
    return L2 ? __float_as_uint(fmaxf(a, 0.f)) : ordered_f32(a);
}
__device__ __forceinline__ uint32_t key_insert(uint32_t bits, uint32_t lowmask, uint32_t ord) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(lowmask), "s"(ord), "v"(bits));
    return r;
}
template <bool L2>
__device__ __forceinline__ float key_decode_lo(uint32_t key, uint32_t lowmask) {
    return L2 ? __uint_as_float(key & ~lowmask) : unordered_f32(key & ~lowmask);
}
template <bool L2>
__device__ __forceinline__ float key_decode_hi(uint32_t key, uint32_t lowmask) {
    return L2 ? __uint_as_float(key | lowmask) : unordered_f32(key | lowmask);
}

// Folded L2 keys (fold image, kernels.h split_bf16_stream): the filter's
// accumulator is acc = <x, y> - (|x|^2 + |y|^2) / 2 = -approx / 2, and the key
// is the raw bits of acc with the ordinal in the low bits (one v_bfi_b32).
// Negative floats order by magnitude as unsigned integers, so these keys order
// like the approx.  acc >= 0 (approx <= 0, a near-duplicate of the query) gives
// a pattern below 0x80000000: it sorts before every negative one, and its
// decode is 0 (clamped) for both bounds — a valid bracket, as the approx is
// <= 0 and every distance is >= 0 — so no clamp is needed in the hot loop.  A
// kept pattern below 0x80000000 makes the stream's dropped bound 0, which is
// still a lower bound of everything it dropped.  The decode brackets the
// approx whatever the ordinal: for negative patterns, clearing the low bits
// shrinks the magnitude (lower bound), setting them grows it (upper bound).
__device__ __forceinline__ uint32_t fold_key_bits(float acc) { return __float_as_uint(acc); }
// The fold key is key_insert (an inline-asm v_bfi_b32) applied straight to
// an MFMA result register.  The compiler's hazard recognizer does not see
// inline-asm readers of an MFMA's destination, so the caller must put
// mfma_read_guard() between the MFMA and the first key_insert: 16 wait states
// (the compiler itself pads this read with s_nop 11, i.e. 12) behind a
// scheduling fence.  (Plain C, (bits & ~lowmask) | ord, is hazard-safe but
// compiles to v_and + v_or3: two VALU per candidate instead of one.)
__device__ __forceinline__ void mfma_read_guard() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ float fold_decode_lo(uint32_t key, uint32_t lowmask) {
    return fmaxf(-2.f * __uint_as_float(key & ~lowmask), 0.f);
}
__device__ __forceinline__ float fold_decode_hi(uint32_t key, uint32_t lowmask) {
    return fmaxf(-2.f * __uint_as_float(key | lowmask), 0.f);
}
// key decode of the IVF-Flat filter keys, plain or folded (runtime flag)
template <bool L2>
__device__ __forceinline__ float ivf_decode_lo(uint32_t key, uint32_t lowmask, bool fold) {
    return (L2 && fold) ? fold_decode_lo(key, lowmask) : key_decode_lo<L2>(key, lowmask);
}
template <bool L2>
__device__ __forceinline__ float ivf_decode_hi(uint32_t key, uint32_t lowmask, bool fold) {
    return (L2 && fold) ? fold_decode_hi(key, lowmask) : key_decode_hi<L2>(key, lowmask);
}
// v = h + m + l exactly (three round-to-nearest bf16 parts: the first
// residual has <= 16 significant bits, the second <= 8)
__device__ __forceinline__ void split3_bf16(float v, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)v;
    const float r1 = v - (float)h;
    m = (__bf16)r1;
    l = (__bf16)(r1 - (float)m);
}

__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& h, bf16x8& l) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const __bf16 hb = (__bf16)v[j];
        h[j] = hb;
        l[j] = (__bf16)(v[j] - (float)hb);
    }
}

// The B operand (32 query columns per wave) for one work item: lane holds
// query column `li` dims [16 s + 8 lh, +8) split into hi / lo, and |x|^2
// (any order; margins only).  Rows are read as float4 (a row is readable up
// to roundup(d, 4) <= ldx); dims >= d are zeroed.  qr < 0 (an unused column,
// whose results are discarded) reads row 0.
template <int NS>
__device__ __forceinline__ void query_raw_load(const float* __restrict__ x, int ldx, int d, int qr,
                                               int lh, float4 (&raw)[2 * NS]) {
    const float* xr = x + (int64_t)(qr < 0 ? 0 : qr) * ldx;
    const int d4 = (d + 3) & ~3;
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int kk = 16 * s + 8 * lh + 4 * u;
            // clamped address: every load is unconditional (no branches)
            raw[2 * s + u] = *(const float4*)(xr + min(kk, d4 - 4));
        }
}
template <int NS>
__device__ __forceinline__ void query_frags_from_raw(const float4 (&raw)[2 * NS], int d, int lh,
                                                     bf16x8 (&bh)[NS], bf16x8 (&bl)[NS],
                                                     float& xn) {
    xn = 0.f;
#pragma unroll
    for (int s = 0; s < NS; s++) {
        float v[8] = {raw[2 * s].x,     raw[2 * s].y,     raw[2 * s].z,     raw[2 * s].w,
                      raw[2 * s + 1].x, raw[2 * s + 1].y, raw[2 * s + 1].z, raw[2 * s + 1].w};
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = 16 * s + 8 * lh + j < d ? v[j] : 0.f;  // also kk >= d4
        split8(v, bh[s], bl[s]);
#pragma unroll
        for (int j = 0; j < 8; j++) xn = fmaf(v[j], v[j], xn);
    }
    xn += __shfl_xor(xn, 32);
}
template <int NS>
__device__ __forceinline__ void load_query_frags(const float* __restrict__ x, int ldx, int d,
                                                 int qr, int lh, bf16x8 (&bh)[NS],
                                                 bf16x8 (&bl)[NS], float& xn) {
    float4 raw[2 * NS];
    query_raw_load<NS>(x, ldx, d, qr, lh, raw);
    query_frags_from_raw<NS>(raw, d, lh, bh, bl, xn);
}

// Query image (k_query_prep): per query the B fragments load_query_frags
// builds — bf16 hi then bf16 lo, each 16 NS values in dim order (64 NS bytes
// per query) — and its |x|^2 (same order, same bits).  A filter work group
// then reads its fragments with 2 NS 16-byte loads instead of splitting the
// fp32 row itself (~6 VALU per dim, repeated by every work group that sees
// the query: once per probed list item, once per coarse split).
template <int NS>
__device__ __forceinline__ void load_query_image(const uint8_t* __restrict__ qimg,
                                                 const float* __restrict__ qxn, int qr, int lh,
                                                 bf16x8 (&bh)[NS], bf16x8 (&bl)[NS], float& xn) {
    const int q = qr < 0 ? 0 : qr;
    const uint8_t* row = qimg + (int64_t)q * (64 * NS) + 16 * lh;
#pragma unroll
    for (int s = 0; s < NS; s++) {
        bh[s] = *(const bf16x8*)(row + 32 * s);
        bl[s] = *(const bf16x8*)(row + 32 * NS + 32 * s);
    }
    xn = qxn ? qxn[q] : 0.f;
}

// One 32x32 block: A = 32 database rows (hi/lo image in LDS, this lane's row
// pointer `arow` already offset by 16 * lh bytes), B = the register query
// fragments.  acc[r] = row (r&3)+8(r>>2)+4lh, col li.
template <int NS>
__device__ __forceinline__ floatx16 bf3_block(const uint8_t* arow, const bf16x8 (&bh)[NS],
                                              const bf16x8 (&bl)[NS]) {
    constexpr int DB = 16 * NS;
    bf16x8 ah[NS], al[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        ah[s] = *(const bf16x8*)(arow + 32 * s);
        al[s] = *(const bf16x8*)(arow + 2 * DB + 32 * s);
    }
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < NS; s++) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[s], bh[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bl[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bh[s], acc, 0, 0, 0);
    }
    return acc;
}

// bf16x2: codes' hi part only (A), queries hi + lo (B)
template <int NS>
__device__ __forceinline__ floatx16 bf2_block(const uint8_t* arow, const bf16x8 (&bh)[NS],
                                              const bf16x8 (&bl)[NS]) {
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
    return acc;
}

__device__ __forceinline__ uint32_t cdiv_dev(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// list row of a filter key: thread slot (bi, lh) of its (query, list), tile
// and register index from the ordinal (the 32x32 MFMA block layout)
__device__ __forceinline__ uint32_t ivf_key_row(uint32_t key, uint32_t lowmask, int slot) {
    const uint32_t ord = key & lowmask;
    const uint32_t r = ord & 15u;
    return (ord >> 4) * BV + 32 * (slot >> 1) + 4 * (slot & 1) + 8 * (r >> 2) + (r & 3);
}

// Rows of thread stream `slot` of a list of length len, enumerated as
// e = tile * 16 + register (the filter's visiting order within the stream)
__device__ __forceinline__ int ivf_stream_row(int e, int slot) {
    const int r = e & 15;
    return (e >> 4) * BV + 32 * (slot >> 1) + 4 * (slot & 1) + 8 * (r >> 2) + (r & 3);
}

// padded dim of the bf16 hi/lo images: a multiple of 32 (NS = DB/16 even)
inline int bf3_db(int d) { return (d + 31) / 32 * 32; }

}  // namespace kern
}  // namespace faiss_amd
