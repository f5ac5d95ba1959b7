// kernels_ivfpq_rerank.hip — the IVF-PQ re-rank dispatch: the Flat re-rank's
// certified candidate selection with the reference LUT arithmetic as the
// exact evaluator (pq_exact, ivf_rerank.h); one translation unit per
// sub-quantizer width (kernels_ivfpq_rerank_d<DS>.hip)
#include "ivf_rerank.h"

namespace faiss_amd {
namespace kern {

extern template void ivfpq_rerank_ds<2>(const uint32_t*, const ProbeRec*, const float*, int, int,
                                        const int64_t*, const PQArgs&, int64_t, int, int, int,
                                        int, const uint8_t*, float*, int64_t*, uint32_t*,
                                        hipStream_t, unsigned long long*, int);
extern template void ivfpq_rerank_ds<4>(const uint32_t*, const ProbeRec*, const float*, int, int,
                                        const int64_t*, const PQArgs&, int64_t, int, int, int,
                                        int, const uint8_t*, float*, int64_t*, uint32_t*,
                                        hipStream_t, unsigned long long*, int);
extern template void ivfpq_rerank_ds<8>(const uint32_t*, const ProbeRec*, const float*, int, int,
                                        const int64_t*, const PQArgs&, int64_t, int, int, int,
                                        int, const uint8_t*, float*, int64_t*, uint32_t*,
                                        hipStream_t, unsigned long long*, int);

void ivfpq_rerank(const uint32_t* keys, const ProbeRec* recs, const float* x, int ldx, int d,
                  const int64_t* ids, const PQArgs& pa, int dsub, int64_t n, int nprobe, int KT,
                  int obits, int k, const uint8_t* sel, float* D, int64_t* I, uint32_t* stats,
                  hipStream_t s, unsigned long long* qdone, int fold) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT(d <= BDM && d % 4 == 0);
    FAISS_THROW_IF_NOT(nprobe <= kMaxNprobeFilter);
    FAISS_THROW_IF_NOT_MSG(dsub == 2 || dsub == 4 || dsub == 8,
                           "ivfpq_rerank: dsub must be 2, 4 or 8");
    if (dsub == 2)
        ivfpq_rerank_ds<2>(keys, recs, x, ldx, d, ids, pa, n, nprobe, KT, obits, k, sel, D, I,
                           stats, s, qdone, fold);
    else if (dsub == 4)
        ivfpq_rerank_ds<4>(keys, recs, x, ldx, d, ids, pa, n, nprobe, KT, obits, k, sel, D, I,
                           stats, s, qdone, fold);
    else
        ivfpq_rerank_ds<8>(keys, recs, x, ldx, d, ids, pa, n, nprobe, KT, obits, k, sel, D, I,
                           stats, s, qdone, fold);
}

}  // namespace kern
}  // namespace faiss_amd
