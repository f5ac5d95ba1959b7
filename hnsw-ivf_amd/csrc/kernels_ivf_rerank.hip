// kernels_ivf_rerank.hip — the IVF-Flat certified exact re-rank launches
// (the kernels are in ivf_rerank.h; the IVF-PQ instantiations compile in
// kernels_ivfpq_rerank*.hip).
#include "ivf_rerank.h"

namespace faiss_amd {
namespace kern {

// ---------------------------------------------------------------- host
void ivf_flat_rerank(const uint32_t* keys, const ProbeRec* recs, const float* x, int ldx,
                     const float* codes, int ldc, const int64_t* ids, int d, int64_t n,
                     int nprobe, int KE, int obits, int k, int metric_l2, const uint8_t* sel,
                     uint32_t* stats, float* D, int64_t* I, KernelTimes* kt, hipStream_t s,
                     unsigned long long* qdone, int fold) {
    if (n <= 0) return;
    const bool l2 = metric_l2 != 0;
    const bool fk = fold != 0;
    {
        ScopedKernelTimer tm(kt, "ivf_rerank", 0.0, s);
        const int E = nprobe * KE;
        const int V = E <= 128 ? 2 : E <= 256 ? 4 : E <= 512 ? 8 : E <= 1024 ? 16 : 32;
        // FAISS_AMD_RERANK_TRACE=<file>: per-query wave timestamps (profiling)
        static unsigned long long* trace_buf = nullptr;
        static int64_t trace_n = 0;
        const char* tr = getenv("FAISS_AMD_RERANK_TRACE");
        unsigned long long* trace = nullptr;
        if (tr) {
            if (trace_n < n) {
                if (trace_buf) HIP_CHECK(hipFree(trace_buf));
                HIP_CHECK(hipMalloc(&trace_buf, 64 * n));
                trace_n = n;
            }
            trace = trace_buf;
        }
#define LAUNCH_B(L2V, VV)                                                                      \
    k_ivf_rerank<L2V, VV><<<kgrid(cdiv(n, RR_W), 64 * RR_W), dim3(64 * RR_W), 0, s>>>(           \
            keys, recs, x, ldx, codes, ldc, ids, d, n, nprobe, KE / 4, obits, k, D, I, stats,   \
            trace, PQArgs{}, sel, qdone, fk ? 1 : 0)
#define DISPATCH_V(L2V)                      \
    do {                                     \
        if (V == 2) LAUNCH_B(L2V, 2);        \
        else if (V == 4) LAUNCH_B(L2V, 4);   \
        else if (V == 8) LAUNCH_B(L2V, 8);   \
        else if (V == 16) LAUNCH_B(L2V, 16); \
        else LAUNCH_B(L2V, 32);              \
    } while (0)
#define LAUNCH_W(L2V, KEV)                                                                     \
    k_ivf_rerank_wide<L2V, KEV><<<kgrid(n, 64), dim3(64), 0, s>>>(                          \
            keys, recs, x, ldx, codes, ldc, ids, d, n, nprobe, obits, k, D, I, stats, PQArgs{},  \
            sel, qdone, fk ? 1 : 0)
#define DISPATCH_W(L2V)                      \
    do {                                     \
        if (KE == 8) LAUNCH_W(L2V, 8);       \
        else if (KE == 16) LAUNCH_W(L2V, 16); \
        else LAUNCH_W(L2V, 32);              \
    } while (0)
        if (nprobe > 64) {  // probes walked in chunks of 64 (k_ivf_rerank_wide)
            if (l2) DISPATCH_W(true);
            else DISPATCH_W(false);
        } else if (l2) DISPATCH_V(true);
        else DISPATCH_V(false);
        HIP_LAUNCH_CHECK();
#undef DISPATCH_W
#undef LAUNCH_W
        if (trace) {
            std::vector<unsigned long long> h(8 * n);
            HIP_CHECK(hipMemcpyAsync(h.data(), trace, 64 * n, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            if (FILE* f = fopen(tr, "wb")) {
                fwrite(h.data(), 64, n, f);
                fclose(f);
            }
        }
#undef DISPATCH_V
#undef LAUNCH_B
    }
}

}  // namespace kern
}  // namespace faiss_amd
