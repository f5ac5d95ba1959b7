// kernels_range.hip — IVF-Flat range search (reference
// faiss/IndexIVF.cpp:1203-1400 range_search / range_search_preassigned with
// IVFFlatScanner::scan_codes_range, faiss/IndexIVFFlat.cpp:181-201).
//
// One 64-lane wave per (query, probe).  Lanes take 64 consecutive rows of the
// probed list, evaluate the distance in the reference's fp32 order
// (ref_arith.h) and test it against the radius with the reference's strict
// comparison (L2: dis < radius, IP: dis > radius).  Pass 1 counts the hits of
// each (query, probe); the host turns the counts into offsets (probe order
// within a query = the reference's result order); pass 2 re-evaluates and
// writes the hits in row order by ballot prefix counts.  Distances are
// recomputed rather than stored so pass 1 writes 4 B per (query, probe).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "ref_arith.h"

namespace faiss_amd {
namespace kern {

namespace {
template <bool L2, bool FILL>
__global__ __launch_bounds__(64) void k_ivf_range(
        const float* __restrict__ x, int ldx, const int32_t* __restrict__ assign, int np,
        const float* __restrict__ codes, int ldc, const int64_t* __restrict__ ids,
        const uint32_t* __restrict__ list_off, const uint32_t* __restrict__ list_len, int nlist,
        int d, float radius, const uint8_t* __restrict__ selm, uint32_t* __restrict__ counts,
        const uint64_t* __restrict__ offsets, float* __restrict__ outD,
        int64_t* __restrict__ outI, int64_t npairs) {
    const int lane = threadIdx.x;
    // one wave per (query, probe), block-strided over the n np pairs
    for (int64_t qp = blockIdx.x; qp < npairs; qp += gridDim.x) {
        const int64_t q = qp / np;
        const int32_t key = assign[qp];
        uint32_t cnt = 0;
        if (key >= 0 && key < nlist) {
            const uint32_t off = list_off[key], len = list_len[key];
            const float* xq = x + q * (int64_t)ldx;
            const uint64_t base = FILL ? offsets[qp] : 0;
            const uint64_t below = (1ull << lane) - 1ull;
            for (uint32_t r0 = 0; r0 < len; r0 += 64) {
                const uint32_t r = r0 + lane;
                bool hit = false;
                float dis = 0.f;
                if (r < len) {
                    const uint64_t row = (uint64_t)off + r;
                    if (!selm || selm[row]) {
                        dis = ref_dist<L2>(xq, codes + row * (uint64_t)ldc, d);
                        hit = L2 ? (dis < radius) : (radius < dis);
                    }
                }
                const uint64_t m = __ballot(hit);
                if (FILL && hit) {
                    const uint64_t o = base + cnt + (uint32_t)__popcll(m & below);
                    outD[o] = dis;
                    // ids == nullptr: store_pairs, lo_build(list_no, offset)
                    outI[o] = ids ? ids[(uint64_t)off + r] : (((int64_t)key << 32) | (int64_t)r);
                }
                cnt += (uint32_t)__popcll(m);
            }
        }
        if (!FILL && lane == 0) counts[qp] = cnt;
    }
}
}  // namespace

void ivf_range_flat(const float* x, int64_t n, int ldx, const int32_t* assign, int np,
                    const float* codes, int ldc, const int64_t* ids, const uint32_t* list_off,
                    const uint32_t* list_len, int nlist, int d, int metric_l2, float radius,
                    const uint8_t* selm, uint32_t* counts, const uint64_t* offsets, float* outD,
                    int64_t* outI, hipStream_t s) {
    if (n <= 0 || np <= 0) return;
    const dim3 grid((unsigned)std::min<int64_t>(n * np, 65536)), block(64);
    const bool fill = offsets != nullptr;
#define RANGE_LAUNCH(L2, F)                                                                       \
    hipLaunchKernelGGL((k_ivf_range<L2, F>), grid, block, 0, s, x, ldx, assign, np, codes, ldc,  \
                       ids, list_off, list_len, nlist, d, radius, selm, counts, offsets, outD,    \
                       outI, n * np)
    if (metric_l2) {
        if (fill) RANGE_LAUNCH(true, true); else RANGE_LAUNCH(true, false);
    } else {
        if (fill) RANGE_LAUNCH(false, true); else RANGE_LAUNCH(false, false);
    }
#undef RANGE_LAUNCH
    HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace faiss_amd
