// exact_select.h — wave-level exact top-k with the reference's tie semantics.
//
// The reference scan (faiss/IndexIVFFlat.cpp:155-179 via
// faiss/IndexIVF.cpp:595-631) pushes candidates into a bounded heap in
// arrival order (probe rank, then list row) with STRICT admission on the
// distance (`C::cmp(simi[0], dis)`, faiss/utils/Heap.h:52-78 cmp vs cmp2) and
// evicts the heap top by (distance, id) (heap_replace_top, Heap.h:112-149).
// For candidates that do not tie with the k-th distance v this equals the
// lexicographic top-k by key (L2: (dis, id); IP: (-ip, -id)).  When the k-th
// key value v is shared by more candidates than fit, the survivors among the
// tied ones are a function of arrival order:
//   S      = the first k arrivals among candidates with key <= v,
//   kept   = the m = k - #{key < v} tied members of S with the smallest key2
//            (L2: smallest ids — the CMax top evicts the largest id first;
//             IP: largest ids — CMin evicts the smallest id first).
// Proof sketch: before the k-th arrival with key <= v the heap top is > v, so
// every such candidate is admitted; afterwards tied ones are rejected and each
// later strictly-better arrival evicts the tied member with the largest key2.
//
// exact_topk_resolve() takes a Stream with
//     template <class F> void for_each(F f)  // f(ok, k1, k2, rank) per lane,
//                                            // wave-uniform iteration
// and writes the reference result for one query (one wave).  Streams are
// re-iterated only when a tie crosses the k boundary (rare), so they
// recompute exact distances rather than caching them.
#pragma once

#include "wave_select.h"

namespace faiss_amd {
namespace kern {

template <class Stream, class OutIdx = int64_t>
__device__ __forceinline__ void exact_topk_resolve(Stream& st, int k, int metric_l2, int lane,
                                                   bool write, float* __restrict__ Dq,
                                                   OutIdx* __restrict__ Iq) {
    // pass A: lexicographic top-(k+1) (the extra slot detects a boundary tie)
    const int K1 = k < 64 ? k + 1 : 64;
    float fd = WS_INF, td = WS_INF;
    long long fi = WS_NOID, ti = WS_NOID;
    st.for_each([&](bool ok, float k1, long long k2, long long) {
        wave_offer(fd, fi, ok ? k1 : WS_INF, ok ? k2 : WS_NOID, td, ti, K1, lane);
    });
    const float v = __shfl(fd, k - 1);
    const long long vi = shfl_ll(fi, k - 1);
    bool amb = false;
    if (vi != WS_NOID) {
        if (k < 64) {
            const float nd = __shfl(fd, k);
            const long long ni = shfl_ll(fi, k);
            amb = ni != WS_NOID && nd == v;
        } else {
            int cnt = 0;
            st.for_each([&](bool ok, float k1, long long, long long) {
                cnt += __popcll(__ballot(ok && k1 == v));
            });
            amb = cnt > __popcll(__ballot(lane < k && fd == v));
        }
    }
    float od = fd;
    long long oi = fi;
    if (amb) {
        const int a = __popcll(__ballot(lane < k && fd < v));
        const int m = k - a;
        // pass C: arrival rank of the k-th candidate with key <= v
        float cd = WS_INF;
        long long ci = WS_NOID;
        td = WS_INF;
        ti = WS_NOID;
        st.for_each([&](bool ok, float k1, long long, long long rank) {
            const bool in = ok && k1 <= v;
            wave_offer(cd, ci, in ? 0.f : WS_INF, in ? rank : WS_NOID, td, ti, k, lane);
        });
        const long long R = shfl_ll(ci, k - 1);
        // pass D: the m tied members of S with the smallest key2
        float dd = WS_INF;
        long long di = WS_NOID;
        td = WS_INF;
        ti = WS_NOID;
        st.for_each([&](bool ok, float k1, long long k2, long long rank) {
            const bool in = ok && k1 == v && rank <= R;
            wave_offer(dd, di, in ? 0.f : WS_INF, in ? k2 : WS_NOID, td, ti, m, lane);
        });
        const long long tk = shfl_ll(di, lane >= a ? lane - a : 0);
        if (lane >= a) {
            od = v;
            oi = tk;
        }
    }
    if (write && lane < k) {
        float dis;
        long long id;
        from_key(metric_l2, od, oi, dis, id);
        Dq[lane] = dis;
        Iq[lane] = (OutIdx)id;
    }
}

}  // namespace kern
}  // namespace faiss_amd
