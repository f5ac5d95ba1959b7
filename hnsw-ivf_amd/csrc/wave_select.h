// wave_select.h — wave64 k-selection primitives (device side).
//
// Reference semantics being reproduced (faiss/utils/Heap.h:112-149,421-450,
// faiss/utils/ordered_key_value.h:42-80, faiss/impl/ResultHandler.h:263-278):
// a bounded max-heap with strict admission `dis < heap[0]` whose top is the
// largest (dis, id) pair.  When candidates arrive in increasing id order
// (coarse quantizer rows, one inverted list added in order) this keeps exactly
// the k smallest (dis, id) pairs, so the wave queue below orders by the key
// (k1, k2) lexicographically: L2 uses (dis, id); inner product uses (-ip, -id)
// (a CMin heap keeps the largest (ip, id)).
//
// Layout: a wave-wide sorted queue, lane i holds the i-th smallest key.  The
// queue always keeps 64 keys (only the first K are reported); a batch of 64
// candidates (one per lane) is folded in with a 64-lane bitonic sort followed
// by a bitonic merge against the reversed queue.  Batches with no candidate
// below the K-th key are rejected with a single ballot.
#pragma once

#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

namespace faiss_amd {

#define WS_INF __builtin_inff()
#define WS_NOID ((long long)0x7fffffffffffffffLL)

__device__ __forceinline__ bool key_less(float ad, long long ai, float bd, long long bi) {
    return ad < bd || (ad == bd && ai < bi);
}

__device__ __forceinline__ long long shfl_xor_ll(long long v, int m) {
    int lo = __shfl_xor((int)(v & 0xffffffffLL), m);
    int hi = __shfl_xor((int)(v >> 32), m);
    return ((long long)hi << 32) | (unsigned int)lo;
}
__device__ __forceinline__ long long shfl_ll(long long v, int src) {
    int lo = __shfl((int)(v & 0xffffffffLL), src);
    int hi = __shfl((int)(v >> 32), src);
    return ((long long)hi << 32) | (unsigned int)lo;
}

// compare-exchange with the lane at distance `m`; this lane keeps the min
// when take_min, else the max.
__device__ __forceinline__ void cas_lane(float& d, long long& i, int m, bool take_min) {
    float od = __shfl_xor(d, m);
    long long oi = shfl_xor_ll(i, m);
    bool other_less = key_less(od, oi, d, i);
    bool self_less = key_less(d, i, od, oi);
    bool swap = take_min ? other_less : self_less;
    if (swap) {
        d = od;
        i = oi;
    }
}

// ascending bitonic sort of 64 keys, one per lane
__device__ __forceinline__ void wave_sort64(float& d, long long& i, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            bool up = (lane & k) == 0;
            bool lower = (lane & j) == 0;
            cas_lane(d, i, j, lower == up);
        }
    }
}

// merge a sorted batch (cd,ci) into the sorted queue (qd,qi), keeping the 64
// smallest keys, sorted ascending.
__device__ __forceinline__ void wave_merge64(float& qd, long long& qi, float cd, long long ci,
                                             int lane) {
    float rd = __shfl(cd, 63 - lane);
    long long ri = shfl_ll(ci, 63 - lane);
    if (key_less(rd, ri, qd, qi)) {
        qd = rd;
        qi = ri;
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) cas_lane(qd, qi, j, (lane & j) == 0);
}

// Offer one candidate per lane.  thr_d/thr_i hold the K-th key (wave
// uniform) and are refreshed when the queue changes.
__device__ __forceinline__ void wave_offer(float& qd, long long& qi, float cd, long long ci,
                                           float& thr_d, long long& thr_i, int K, int lane) {
    bool pass = key_less(cd, ci, thr_d, thr_i);
    if (__ballot(pass) == 0ull) return;
    if (!pass) {
        cd = WS_INF;
        ci = WS_NOID;
    }
    wave_sort64(cd, ci, lane);
    wave_merge64(qd, qi, cd, ci, lane);
    thr_d = __shfl(qd, K - 1);
    thr_i = shfl_ll(qi, K - 1);
}

// Same as wave_offer, threshold re-derived from the queue (saves registers
// when a wave keeps many queues).
__device__ __forceinline__ void wave_offer_q(float& qd, long long& qi, float cd, long long ci,
                                             int K, int lane) {
    float thr_d = __shfl(qd, K - 1);
    long long thr_i = shfl_ll(qi, K - 1);
    bool pass = key_less(cd, ci, thr_d, thr_i);
    if (__ballot(pass) == 0ull) return;
    if (!pass) {
        cd = WS_INF;
        ci = WS_NOID;
    }
    wave_sort64(cd, ci, lane);
    wave_merge64(qd, qi, cd, ci, lane);
}

// internal key <-> (distance, label) for the two metrics
__device__ __forceinline__ void to_key(int metric_l2, float dis, long long id, float& k1,
                                       long long& k2) {
    if (metric_l2) {
        k1 = dis;
        k2 = id;
    } else {
        k1 = -dis;
        k2 = -id;
    }
}
// admissible: the reference heap starts at neutral() (FLT_MAX / -FLT_MAX)
// with strict comparison, so only keys strictly below FLT_MAX can enter.
__device__ __forceinline__ bool key_admissible(float k1) { return k1 < FLT_MAX; }

__device__ __forceinline__ void from_key(int metric_l2, float k1, long long k2, float& dis,
                                         long long& id) {
    if (k2 == WS_NOID) {
        dis = metric_l2 ? FLT_MAX : -FLT_MAX;
        id = -1;
    } else if (metric_l2) {
        dis = k1;
        id = k2;
    } else {
        dis = -k1;
        id = -k2;
    }
}

}  // namespace faiss_amd

namespace faiss_amd {
// ---------------------------------------------------------------------------
// Per-thread sorted queue of KQ 64-bit keys (ascending).  key = ordered
// float bits << 32 | tie-breaker, so one unsigned compare orders (dist, tie).
// Used where many candidates per query stream through a few threads (the
// list-centric scan): a candidate costs one compare unless it enters the
// queue; entering costs KQ predicated moves.  The union of the per-thread
// top-k sets of a query contains its top-k, so k <= KQ entries per thread
// suffice.
// (branch-free xor forms: negative floats flip every bit, others the sign)
__device__ __forceinline__ uint32_t ordered_f32(float f) {
    const uint32_t u = __float_as_uint(f);
    return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
}
__device__ __forceinline__ float unordered_f32(uint32_t u) {
    return __uint_as_float(u ^ (~(uint32_t)((int32_t)u >> 31) | 0x80000000u));
}

template <int KQ>
struct ThreadQueue {
    unsigned long long q[KQ];
    unsigned long long thr;  // q[k-1]
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int i = 0; i < KQ; i++) q[i] = ~0ull;
        thr = ~0ull;
    }
    __device__ __forceinline__ void push(unsigned long long c, int k) {
        if (c < thr) {
#pragma unroll
            for (int i = KQ - 1; i > 0; i--) {
                unsigned long long prev = q[i - 1];
                q[i] = c < prev ? prev : (c < q[i] ? c : q[i]);
            }
            q[0] = c < q[0] ? c : q[0];
            unsigned long long t = q[0];
#pragma unroll
            for (int i = 1; i < KQ; i++) t = (i == k - 1) ? q[i] : t;
            thr = t;
        }
    }
};
}  // namespace faiss_amd

namespace faiss_amd {
// k-th smallest (1-based k) of the V*64 values held V per lane, by a radix
// descent on the ordered bit patterns: every step is V compares whose
// ballots are popcounted on the scalar unit — no cross-lane shuffles.  +inf
// (or NaN-free padding) sorts last; fewer than k finite values give +inf.
//
// The descent starts below the bits every finite value shares (wave min /
// max of the patterns: c2's keys span one or two binades, so ~8 of the 32
// steps are skipped) and, with LOWB > 0, stops at bit LOWB and returns the
// top of the 2^LOWB-pattern bucket holding the k-th value: an upper bound
// >= the k-th smallest, above it by < 2^(LOWB - 23) relative.  The re-ranks'
// thresholds (T, U) only need such a bound (a larger U admits more exact
// candidates, never fewer), so they take LOWB = 12 (2^-11: ~10 steps left
// instead of 32; r05 PMC: the 32-step descents were ~40 % of the re-ranks'
// SALU).
template <int V, int LOWB = 0>
__device__ __forceinline__ float wave_kth_smallest(const float (&v)[V], int k) {
    constexpr uint32_t ORD_INF = 0xff800000u;  // ordered_f32(+inf)
    uint32_t key[V];
    uint32_t lo = 0xffffffffu, hi = 0u;
    int nfin = 0;
#pragma unroll
    for (int i = 0; i < V; i++) {
        key[i] = ordered_f32(v[i]);
        const bool fin = key[i] < ORD_INF;
        nfin += __popcll(__ballot(fin));
        lo = min(lo, key[i]);
        hi = max(hi, fin ? key[i] : 0u);
    }
    if (nfin < k) return WS_INF;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, m));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, m));
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    const uint32_t diff = lo ^ hi;  // the k-th value lies in [lo, hi]
    if (diff == 0u) return unordered_f32(lo);
    const int hb = 31 - __builtin_clz(diff);
    uint32_t prefix = hb == 31 ? 0u : lo & ~((2u << hb) - 1u);
    for (int bit = hb; bit >= LOWB; bit--) {
        const uint32_t cand = prefix | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < V; i++) cnt += __popcll(__ballot(key[i] < cand));
        if (cnt < k) prefix = cand;
    }
    if constexpr (LOWB > 0) prefix = min(prefix | ((1u << LOWB) - 1u), ORD_INF);
    return unordered_f32(prefix);
}
}  // namespace faiss_amd
