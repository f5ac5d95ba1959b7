// kernels_ivfpq_rerank_d2.hip — the IVF-PQ re-rank kernels for dsub = 2
// (ivf_rerank.h; a translation unit of their own so the PQ instantiations
// compile in parallel)
#include "ivf_rerank.h"

namespace faiss_amd {
namespace kern {
template void ivfpq_rerank_ds<2>(const uint32_t*, const ProbeRec*, const float*, int, int,
                                   const int64_t*, const PQArgs&, int64_t, int, int, int, int,
                                   const uint8_t*, float*, int64_t*, uint32_t*, hipStream_t,
                                   unsigned long long*, int);
}  // namespace kern
}  // namespace faiss_amd
