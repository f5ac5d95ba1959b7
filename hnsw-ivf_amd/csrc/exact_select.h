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

// Fast path for a query whose whole candidate set fits NB 64-lane batches
// (candidate 64 b + lane < ns holds key (k1[b], k2[b]); the others are
// ignored): each candidate's rank by (k1, k2) (ties in both broken by
// position, as duplicate (dist, id) pairs are kept twice by the reference
// heap) from a broadcast loop, no sorting network.  Returns false and writes
// nothing when the k-th key value is shared past the k boundary (the
// arrival-order rule then needs exact_topk_resolve).
template <int NB, class OutIdx = int64_t>
__device__ __forceinline__ bool exact_topk_small(float (&k1)[NB], long long (&k2)[NB], int ns,
                                                 int k, int metric_l2, int lane, bool write,
                                                 float* __restrict__ Dq,
                                                 OutIdx* __restrict__ Iq) {
    int rank[NB], eq[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        rank[b] = 0;
        eq[b] = 0;
        if (64 * b + lane >= ns) {
            k1[b] = WS_INF;
            k2[b] = WS_NOID;
        }
    }
    // rank by k1 alone (one broadcast per candidate); equal k1 values (rare:
    // exact distance ties, or the +inf padding) are counted and, when any
    // real candidate shares its k1, ranked again by (k1, k2, position)
#pragma unroll
    for (int bb = 0; bb < NB; bb++) {
        const int nj = min(64, ns - 64 * bb);
        for (int j = 0; j < nj; j++) {
            const float a1 = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(k1[bb]), j));
#pragma unroll
            for (int b = 0; b < NB; b++) {
                if (64 * b < ns) {  // uniform: batches past ns hold nothing
                    rank[b] += a1 < k1[b] ? 1 : 0;
                    eq[b] += a1 == k1[b] ? 1 : 0;
                }
            }
        }
    }
    bool ties = false;
#pragma unroll
    for (int b = 0; b < NB; b++)
        ties |= __ballot(64 * b + lane < ns && eq[b] > 1 && k1[b] < WS_INF) != 0ull;
    if (ties) {
#pragma unroll
        for (int b = 0; b < NB; b++) rank[b] = 0;
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            const int nj = min(64, ns - 64 * bb);
            for (int j = 0; j < nj; j++) {
                const float a1 =
                        __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(k1[bb]), j));
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)(k2[bb] & 0xffffffffLL), j);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(k2[bb] >> 32), j);
                const long long a2 = (long long)(((unsigned long long)hi << 32) | lo);
                const int pj = 64 * bb + j;
#pragma unroll
                for (int b = 0; b < NB; b++) {
                    if (64 * b < ns) {
                        const bool before =
                                a1 < k1[b] ||
                                (a1 == k1[b] && (a2 < k2[b] || (a2 == k2[b] && pj < 64 * b + lane)));
                        rank[b] += before ? 1 : 0;
                    }
                }
            }
        }
    } else {
        // distinct k1 among real candidates; the +inf padding (all k1 equal)
        // only ever fills output slots with (FLT_MAX / -FLT_MAX, -1), so its
        // order among itself is immaterial: break it by position
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            if (64 * bb < ns) {
                const unsigned long long inf_m = __ballot(64 * bb + lane < ns && k1[bb] == WS_INF);
#pragma unroll
                for (int b = 0; b < NB; b++) {
                    // +inf candidates before this one in position order
                    if (64 * b < ns && k1[b] == WS_INF) {
                        if (bb < b) rank[b] += __popcll(inf_m);
                        else if (bb == b) rank[b] += __popcll(inf_m & ((1ull << lane) - 1ull));
                    }
                }
            }
        }
    }
    // boundary tie: the key at rank k has the k1 of the key at rank k - 1
    float v1 = WS_INF, n1 = WS_INF;
    long long n2 = WS_NOID;
    bool hv = false, hn = false;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const bool cand = 64 * b + lane < ns;
        const unsigned long long mv = __ballot(cand && rank[b] == k - 1);
        const unsigned long long mn = __ballot(cand && rank[b] == k);
        if (mv) {
            hv = true;
            v1 = __shfl(k1[b], __ffsll((long long)mv) - 1);
        }
        if (mn) {
            hn = true;
            const int ln = __ffsll((long long)mn) - 1;
            n1 = __shfl(k1[b], ln);
            n2 = shfl_ll(k2[b], ln);
        }
    }
    if (hv && hn && n2 != WS_NOID && n1 == v1) return false;
    if (write) {
#pragma unroll
        for (int b = 0; b < NB; b++) {
            if (64 * b + lane < ns && rank[b] < k) {
                float dis;
                long long id;
                from_key(metric_l2, k1[b], k2[b], dis, id);
                Dq[rank[b]] = dis;
                Iq[rank[b]] = (OutIdx)id;
            }
        }
        if (lane >= ns && lane < k) {  // fewer than k candidates: padding slots
            float dis;
            long long id;
            from_key(metric_l2, WS_INF, WS_NOID, dis, id);
            Dq[lane] = dis;
            Iq[lane] = (OutIdx)id;
        }
    }
    return true;
}

}  // namespace kern
}  // namespace faiss_amd
