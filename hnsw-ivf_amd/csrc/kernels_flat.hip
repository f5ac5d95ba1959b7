// kernels_flat.hip — exact flat distance tiles on fp32 MFMA + wave64 top-k.
//
// Reference behaviour: faiss/utils/distances.cpp:259-342
// (exhaustive_L2sqr_blas_default_impl: dis = ||x||^2 + ||y||^2 - 2 <x,y>,
// clamped at 0) with HeapBlockResultHandler (faiss/impl/ResultHandler.h:187-287)
// selecting the k best per query.  Here the <x,y> contraction runs on
// v_mfma_f32_32x32x2_f32 (exact f32 fma chain, k-ordered) from LDS tiles and
// the selection on a wave64 register queue (wave_select.h).
#include <hip/hip_runtime.h>

#include <cfloat>

#include "common.h"
#include "kernels.h"
#include "ref_arith.h"
#include "wave_select.h"
#include "exact_select.h"

namespace faiss_amd {
namespace kern {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------- norms
// One thread per row, a sequential fma chain over the dims: the evaluation
// order is fixed (j = 0..d-1) so the CPU oracle reproduces it bit for bit.
__global__ __launch_bounds__(256) void k_row_norms(const float* __restrict__ x, int64_t n, int d,
                                                   int ld, float* __restrict__ out) {
    int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (row >= n) return;
    const float* xr = x + row * ld;
    // reference order (fvec_norm_L2sqr, see ref_arith.h)
    const float s = ref_norm(xr, d);
    out[row] = s;
}

// Direct form for query blocks below faiss' BLAS threshold
// (faiss/utils/distances.cpp:170-199, 807-823: nx < 20 uses fvec_L2sqr /
// fvec_inner_product per pair).  One thread per (query, row).
__global__ __launch_bounds__(256) void k_direct_dist(const float* __restrict__ x, int64_t nx,
                                                     int ldx, const float* __restrict__ y,
                                                     int64_t ny, int ldy, int d, int metric_l2,
                                                     float* __restrict__ D, int64_t ldD) {
    GRID_STRIDE(p, nx * ny) {
        const int64_t i = p / ny, j = p - i * ny;
        const float* a = x + i * ldx;
        const float* b = y + j * ldy;
        D[i * ldD + j] = metric_l2 ? ref_l2(a, b, d) : ref_ip(a, b, d);
    }
}

void direct_distances(const float* x, int64_t nx, int ldx, const float* y, int64_t ny, int ldy,
                      int d, int metric_l2, float* D, int64_t ldD, hipStream_t s) {
    if (nx <= 0 || ny <= 0) return;
    FAISS_THROW_IF_NOT(ldx % 4 == 0 && ldy % 4 == 0);
    k_direct_dist<<<stride_grid(nx * ny, 256), dim3(256), 0, s>>>(x, nx, ldx, y, ny, ldy, d,
                                                                 metric_l2, D, ldD);
    HIP_LAUNCH_CHECK();
}

void row_norms(const float* x, int64_t n, int d, int ld, float* out, hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT(ld % 4 == 0);
    k_row_norms<<<kgrid(cdiv(n, 256), 256), dim3(256), 0, s>>>(x, n, d, ld, out);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- GEMM tile
// 256 threads = 4 waves; CTA tile 128 (x rows) x 128 (y rows); each wave
// owns a 64x64 quadrant as 2x2 MFMA 32x32 accumulators.  K staged in chunks of
// 32 dims through LDS with a 33-float row stride (conflict-free column reads).
constexpr int GB = 128;
constexpr int GK = 32;
constexpr int GS = GK + 1;

__global__ __launch_bounds__(256) void k_pairwise(const float* __restrict__ x, int64_t nx, int ldx,
                                                  const float* __restrict__ xn,
                                                  const float* __restrict__ y, int64_t ny, int ldy,
                                                  const float* __restrict__ yn, int dp,
                                                  int metric_l2, float* __restrict__ D,
                                                  int64_t ldD, int tiles_y) {
    __shared__ float As[GB * GS];
    __shared__ float Bs[GB * GS];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int w = t >> 6;
    const int wr = w >> 1, wc = w & 1;
    // XCD-friendly order: consecutive blocks walk the y tiles of one x tile
    const int64_t bx = blockIdx.x / tiles_y;
    const int64_t by = blockIdx.x % tiles_y;
    const int64_t r0 = bx * GB, c0 = by * GB;

    floatx16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[m][n][r] = 0.f;

    for (int k0 = 0; k0 < dp; k0 += GK) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            int e = t + 256 * s;
            int r = e >> 3, c4 = e & 7;
            int kc = k0 + 4 * c4;
            float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
            if (r0 + r < nx && kc < dp) va = *(const float4*)(x + (r0 + r) * ldx + kc);
            if (c0 + r < ny && kc < dp) vb = *(const float4*)(y + (c0 + r) * ldy + kc);
            float* pa = As + r * GS + 4 * c4;
            float* pb = Bs + r * GS + 4 * c4;
            pa[0] = va.x; pa[1] = va.y; pa[2] = va.z; pa[3] = va.w;
            pb[0] = vb.x; pb[1] = vb.y; pb[2] = vb.z; pb[3] = vb.w;
        }
        __syncthreads();
        const int li = lane & 31, lk = lane >> 5;
        const float* a0p = As + (wr * 64 + li) * GS + lk;
        const float* a1p = a0p + 32 * GS;
        const float* b0p = Bs + (wc * 64 + li) * GS + lk;
        const float* b1p = b0p + 32 * GS;
#pragma unroll
        for (int kk = 0; kk < GK; kk += 2) {
            float a0 = a0p[kk], a1 = a1p[kk], b0 = b0p[kk], b1 = b1p[kk];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    const int col_l = lane & 31;
    const int rowh = 4 * (lane >> 5);
#pragma unroll
    for (int m = 0; m < 2; m++) {
#pragma unroll
        for (int n = 0; n < 2; n++) {
            int64_t col = c0 + wc * 64 + n * 32 + col_l;
            if (col >= ny) continue;
            float ynj = metric_l2 ? yn[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int64_t row = r0 + wr * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + rowh;
                if (row < nx) {
                    float ip = acc[m][n][r];
                    float v;
                    if (metric_l2) {
                        v = fmaf(-2.f, ip, xn[row] + ynj);
                        if (v < 0.f) v = 0.f;
                    } else {
                        v = ip;
                    }
                    D[row * ldD + col] = v;
                }
            }
        }
    }
}

void pairwise_distances(const float* x, int64_t nx, int ldx, const float* xn, const float* y,
                        int64_t ny, int ldy, const float* yn, int dp, int metric_l2, float* D,
                        int64_t ldD, hipStream_t s) {
    if (nx <= 0 || ny <= 0) return;
    FAISS_THROW_IF_NOT(ldx % 4 == 0 && ldy % 4 == 0 && dp % 4 == 0);
    int64_t tx = cdiv(nx, GB), ty = cdiv(ny, GB);
    FAISS_THROW_IF_NOT(tx * ty < (1ll << 31));
    k_pairwise<<<kgrid(tx * ty, 256), dim3(256), 0, s>>>(x, nx, ldx, xn, y, ny, ldy, yn, dp,
                                                               metric_l2, D, ldD, (int)ty);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- select
// One wave per row.  Pass 1: every lane keeps the minimum key of its strided
// columns; the K-th smallest lane minimum T0 bounds the K-th smallest key of
// the row (K lanes each hold an element <= T0).  Pass 2: the columns with
// key <= T0 (typically 1-3 K of them) are compacted into LDS and folded into
// the wave queue, so a row costs two streaming passes, one 64-lane sort and a
// couple of merges instead of one sort-merge per 64 columns.
constexpr int SEL_CAP = 512;

__global__ __launch_bounds__(256) void k_select_rows(const float* __restrict__ D, int64_t nx,
                                                     int64_t ny, int64_t ldD, int k,
                                                     int metric_l2, int64_t col0,
                                                     float* __restrict__ out_d,
                                                     int32_t* __restrict__ out_i32,
                                                     int64_t* __restrict__ out_i64, int64_t ldo) {
    __shared__ float bufd[4][SEL_CAP];
    __shared__ int32_t bufi[4][SEL_CAP];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t row = (int64_t)blockIdx.x * 4 + w;
    const bool valid_row = row < nx;  // every wave reaches the barrier below
    ny = valid_row ? ny : 0;
    const float* Dr = D + (valid_row ? row : 0) * ldD;
    auto key_of = [&](int64_t col, float& k1, long long& k2) {
        to_key(metric_l2, Dr[col], (long long)col, k1, k2);
        if (!key_admissible(k1)) {
            k1 = WS_INF;
            k2 = WS_NOID;
        }
    };
    // pass 1
    float md = WS_INF;
    long long mi = WS_NOID;
    for (int64_t c = lane; c < ny; c += 64) {
        float k1;
        long long k2;
        key_of(c, k1, k2);
        if (key_less(k1, k2, md, mi)) {
            md = k1;
            mi = k2;
        }
    }
    wave_sort64(md, mi, lane);
    const float t_d = __shfl(md, k - 1);
    const long long t_i = shfl_ll(mi, k - 1);
    // pass 2: compact keys <= T0
    int count = 0;
    bool overflow = false;
    for (int64_t c0 = 0; c0 < ny; c0 += 64) {
        const int64_t c = c0 + lane;
        float k1 = WS_INF;
        long long k2 = WS_NOID;
        if (c < ny) key_of(c, k1, k2);
        const bool pass = k2 != WS_NOID && !key_less(t_d, t_i, k1, k2);
        const unsigned long long m = __ballot(pass);
        if (m) {
            const int pos = count + __popcll(m & ((1ull << lane) - 1ull));
            if (pass && pos < SEL_CAP) {
                bufd[w][pos] = k1;
                bufi[w][pos] = (int32_t)c;
            }
            count += __popcll(m);
        }
    }
    if (count > SEL_CAP) overflow = true;
    __syncthreads();  // one wave per region; also orders the LDS writes
    float qd = WS_INF;
    long long qi = WS_NOID;
    float thr_d = WS_INF;
    long long thr_i = WS_NOID;
    if (!overflow) {
        for (int b0 = 0; b0 < count; b0 += 64) {
            float k1 = WS_INF;
            long long k2 = WS_NOID;
            if (b0 + lane < count) {
                k1 = bufd[w][b0 + lane];
                const long long col = bufi[w][b0 + lane];
                k2 = metric_l2 ? col : -col;
            }
            wave_offer(qd, qi, k1, k2, thr_d, thr_i, k, lane);
        }
    } else {
        for (int64_t c0 = 0; c0 < ny; c0 += 64) {
            const int64_t c = c0 + lane;
            float k1 = WS_INF;
            long long k2 = WS_NOID;
            if (c < ny) key_of(c, k1, k2);
            wave_offer(qd, qi, k1, k2, thr_d, thr_i, k, lane);
        }
    }
    if (valid_row && lane < k) {
        float dis;
        long long id;
        from_key(metric_l2, qd, qi, dis, id);
        if (id >= 0) id += col0;
        if (out_d) out_d[row * ldo + lane] = dis;
        if (out_i32) out_i32[row * ldo + lane] = (int32_t)id;
        if (out_i64) out_i64[row * ldo + lane] = id;
    }
}

void select_rows(const float* D, int64_t nx, int64_t ny, int64_t ldD, int k, int metric_l2,
                 int64_t col0, float* out_d, int32_t* out_i32, int64_t* out_i64, int64_t ldo,
                 hipStream_t s) {
    if (nx <= 0) return;
    FAISS_THROW_IF_NOT_MSG(k >= 1 && k <= kMaxK, "k must be in [1, 64] on this path");
    k_select_rows<<<kgrid(cdiv(nx, 4), 256), dim3(256), 0, s>>>(
            D, nx, ny, ldD, k, metric_l2, col0, out_d, out_i32, out_i64, ldo);
    HIP_LAUNCH_CHECK();
}

// Inner-product rows whose k-th value is tied with a column that was not
// selected: the lexicographic (-ip, -j) choice of k_select_rows differs from
// the reference heap (CMin, strict admission, columns arriving in id
// order), so such rows are re-selected with the arrival-order rule
// (exact_select.h).  One wave per row; rows without a boundary tie exit
// after one counting pass.
struct RowStream {
    const float* row;
    int64_t ny;
    int lane;
    template <class F>
    __device__ __forceinline__ void for_each(F f) const {
        for (int64_t j0 = 0; j0 < ny; j0 += 64) {
            const int64_t j = j0 + lane;
            float k1 = WS_INF;
            long long k2 = WS_NOID;
            bool ok = j < ny;
            if (ok) {
                to_key(0, row[j], (long long)j, k1, k2);
                ok = key_admissible(k1);
            }
            f(ok, k1, k2, (long long)j);
        }
    }
};

template <class OutIdx>
__global__ __launch_bounds__(256) void k_select_fix_ip(const float* __restrict__ D, int64_t nx,
                                                       int64_t ny, int64_t ldD, int k,
                                                       float* __restrict__ out_d,
                                                       OutIdx* __restrict__ out_i, int64_t ldo) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= nx) return;
    const float v = out_d[r * ldo + k - 1];
    if ((int64_t)out_i[r * ldo + k - 1] < 0) return;  // fewer than k results: no boundary
    const float* row = D + r * ldD;
    int cnt = 0;
    for (int64_t j0 = 0; j0 < ny; j0 += 64) {
        const int64_t j = j0 + lane;
        cnt += __popcll(__ballot(j < ny && row[j] == v));
    }
    const int in = __popcll(__ballot(lane < k && out_d[r * ldo + (lane < k ? lane : 0)] == v));
    if (cnt <= in) return;
    RowStream st{row, ny, lane};
    exact_topk_resolve(st, k, 0, lane, true, out_d + r * ldo, out_i + r * ldo);
}

void select_fix_ip(const float* D, int64_t nx, int64_t ny, int64_t ldD, int k, float* out_d,
                   int32_t* out_i32, int64_t* out_i64, int64_t ldo, hipStream_t s) {
    if (nx <= 0) return;
    const dim3 g((unsigned)cdiv(nx, 4)), b(256);
    if (out_i32)
        k_select_fix_ip<int32_t><<<g, b, 0, s>>>(D, nx, ny, ldD, k, out_d, out_i32, ldo);
    else
        k_select_fix_ip<int64_t><<<g, b, 0, s>>>(D, nx, ny, ldD, k, out_d, out_i64, ldo);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- merge
// Shard merge with faiss merge_knn_results ordering (faiss/utils/Heap.cpp:
// 159-230): key (dis, shard, position) for L2; (-dis, nshard-1-shard, pos)
// for IP (a CMax heap pops the larger shard id first on ties).  Inputs
// [nshard][n][kin]; a shard's list ends at its first label < 0.
__global__ __launch_bounds__(256) void k_merge_shards(const float* __restrict__ all_d,
                                                      const int64_t* __restrict__ all_i,
                                                      int64_t n, int kin, int nshard, int k,
                                                      int metric_l2, float* __restrict__ out_d,
                                                      int64_t* __restrict__ out_i) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    float qd = WS_INF;
    long long qi = WS_NOID;
    float thr_d = WS_INF;
    long long thr_i = WS_NOID;
    const int total = nshard * kin;
    const int64_t stride = n * (int64_t)kin;
    for (int c = 0; c < total; c += 64) {
        int e = c + lane;
        float k1 = WS_INF;
        long long k2 = WS_NOID;
        if (e < total) {
            int sh = e / kin, p = e % kin;
            int64_t off = sh * stride + row * kin;
            // valid only if no earlier slot of this shard is empty
            bool ok = true;
            for (int pp = 0; pp <= p; pp++)
                if (all_i[off + pp] < 0) { ok = false; break; }
            if (ok) {
                float dis = all_d[off + p];
                k1 = metric_l2 ? dis : -dis;
                int so = metric_l2 ? sh : (nshard - 1 - sh);
                k2 = (long long)so * kin + p;
            }
        }
        wave_offer(qd, qi, k1, k2, thr_d, thr_i, k, lane);
    }
    if (lane < k) {
        float dis;
        long long lab;
        if (qi == WS_NOID) {
            dis = metric_l2 ? FLT_MAX : -FLT_MAX;
            lab = -1;
        } else {
            int so = (int)(qi / kin), p = (int)(qi % kin);
            int sh = metric_l2 ? so : (nshard - 1 - so);
            int64_t off = sh * stride + row * kin + p;
            dis = all_d[off];
            lab = all_i[off];
        }
        out_d[row * k + lane] = dis;
        out_i[row * k + lane] = lab;
    }
}

void merge_rows(const float* cand_d, const int64_t* cand_i, int64_t n, int nin_x_kin, int k,
                int metric_l2, float* out_d, int64_t* out_i, hipStream_t s) {
    // nin_x_kin is encoded by the caller as nshard * 65536 + kin
    int nshard = nin_x_kin >> 16, kin = nin_x_kin & 0xffff;
    if (n <= 0) return;
    if (k > kMaxK) {
        merge_rows_general(cand_d, cand_i, n, nshard, kin, k, metric_l2, out_d, out_i, s);
        return;
    }
    k_merge_shards<<<kgrid(cdiv(n, 4), 256), dim3(256), 0, s>>>(
            cand_d, cand_i, n, kin, nshard, k, metric_l2, out_d, out_i);
    HIP_LAUNCH_CHECK();
}

}  // namespace kern
}  // namespace faiss_amd

namespace faiss_amd {
namespace kern {
// faiss/IndexShardsIVF.cpp translate_labels: labels >= 0 get += offset
__global__ void k_translate_labels(int64_t* __restrict__ lab, int64_t n, int64_t off) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && lab[i] >= 0) lab[i] += off;
}
void translate_labels(int64_t* labels, int64_t n, int64_t offset, hipStream_t s) {
    if (n <= 0 || offset == 0) return;
    k_translate_labels<<<kgrid(cdiv(n, 256), 256), dim3(256), 0, s>>>(labels, n, offset);
    HIP_LAUNCH_CHECK();
}
}  // namespace kern
}  // namespace faiss_amd
