// kernels_exact.hip — the general exact IVF scan and the exact top-k select.
//
// Serves every geometry the MFMA filters do not (k up to kMaxKExact = 2048,
// nprobe up to nlist, any d, IVF-PQ with any M / dsub, inner product,
// store_pairs) with the reference's results bit for bit:
//
//  1. k_ex_offsets: per query, the candidate offset of each probe
//     (probe rank order; max_codes prefixes; skipped keys contribute 0).
//  2. k_ex_flat / k_ex_pq: every candidate row of every probe gets its exact
//     distance in the reference's fp32 order (ref_arith.h, pq_ref.h) and is
//     stored in arrival order as a 32-bit order-preserving key + its arena row.
//     Rows outside the IDSelector and distances the reference heap can never
//     admit (!(dis < FLT_MAX) for L2, !(dis > -FLT_MAX) for IP, NaN) get the
//     SKIP key: for the reference they never arrive
//     (faiss/IndexIVFFlat.cpp:155-179, faiss/IndexIVFPQ.cpp:760-778 with the
//     strict C::cmp(heap[0], dis) admission).
//  3. k_ex_select: per query, the reference heap's result without a heap:
//     a 4 x 8-bit radix select finds the k-th smallest key v, an ordered pass
//     collects the keys < v and the tied keys == v among the first k arrivals
//     with key <= v, the tied ones are cut to the k - #{key < v} smallest
//     labels (IP: largest), and a bitonic sort in LDS gives heap_reorder's
//     order (L2: ascending (dis, label); IP: descending).  The arrival-order
//     rule is derived in exact_select.h.
// The same select serves dense distance rows (coarse quantizer with large
// nprobe), where arrival order = column order and label = column.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>

#include "common.h"
#include "kernels.h"
#include "pq_ref.h"
#include "ref_arith.h"
#include "wave_select.h"

namespace faiss_amd {
namespace kern {

namespace {

constexpr uint32_t EX_SKIP = 0xffffffffu;

__device__ __forceinline__ uint32_t ex_key(float dis, bool l2) {
    if (l2) return dis < FLT_MAX ? ordered_f32(dis) : EX_SKIP;
    return dis > -FLT_MAX ? ~ordered_f32(dis) : EX_SKIP;
}
__device__ __forceinline__ float ex_dis(uint32_t key, bool l2) {
    return l2 ? unordered_f32(key) : unordered_f32(~key);
}

// ---------------------------------------------------------------- offsets
__global__ __launch_bounds__(256) void k_ex_offsets(const int32_t* __restrict__ assign, int64_t n,
                                                    int np, const uint32_t* __restrict__ list_len,
                                                    int nlist, const uint32_t* __restrict__ lim,
                                                    uint32_t* __restrict__ eoff,
                                                    uint32_t* __restrict__ total) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    uint32_t run = 0;
    for (int p = 0; p < np; p++) {
        const int64_t e = q * np + p;
        const int32_t key = assign[e];
        eoff[e] = run;
        if (key >= 0 && key < nlist) run += lim ? lim[e] : list_len[key];
    }
    total[q] = run;
}

// ---------------------------------------------------------------- Flat
// one wave per (query, probe); thread per row, fvec_L2sqr / fvec_inner_product
// order (ref_arith.h) against the query in LDS
template <bool L2>
__global__ __launch_bounds__(64) void k_ex_flat(const float* __restrict__ x, int ldx, int d, int np,
                                                const int32_t* __restrict__ assign,
                                                const uint32_t* __restrict__ lim,
                                                const uint32_t* __restrict__ list_off,
                                                const uint32_t* __restrict__ list_len, int nlist,
                                                const float* __restrict__ codes, int ldc,
                                                const uint8_t* __restrict__ sel,
                                                const uint32_t* __restrict__ eoff, int64_t cap,
                                                uint32_t* __restrict__ okeys,
                                                uint32_t* __restrict__ orows, int64_t e0) {
    extern __shared__ float xs[];  // [ldx]
    const int64_t e = e0 + blockIdx.x;
    const int64_t q = e / np;
    const int32_t key = assign[e];
    if (key < 0 || key >= nlist) return;
    const uint32_t len = lim ? lim[e] : list_len[key];
    if (len == 0) return;
    for (int i = threadIdx.x; i < ldx; i += 64) xs[i] = x[q * ldx + i];
    __syncthreads();
    const uint32_t off = list_off[key];
    const int64_t base = q * cap + eoff[e];
    for (uint32_t r = threadIdx.x; r < len; r += 64) {
        const uint32_t row = off + r;
        uint32_t k = EX_SKIP;
        if (!sel || sel[row]) k = ex_key(ref_dist<L2>(xs, codes + (int64_t)row * ldc, d), L2);
        okeys[base + r] = k;
        orows[base + r] = row;
    }
}

// ---------------------------------------------------------------- PQ
// The (query, probe) table in LDS with the reference arithmetic (QueryTables,
// faiss/IndexIVFPQ.cpp:545-700): lut [M * 256] | xs [ldx] | rs [ldx] | dis0.
// 256 threads; returns dis0 (all threads, after the barrier).
template <bool L2>
__device__ __forceinline__ float ex_pq_tables(const float* __restrict__ xq, int ldx, int d,
                                              int32_t key, float cd, const ExactPQ& pq,
                                              float* lut) {
    const int M = pq.M, dsub = pq.dsub;
    float* xs = lut + M * 256;
    float* rs = xs + ldx;
    float* sd0 = rs + ldx;
    const int tid = threadIdx.x;
    const float* yc = pq.cent + (int64_t)key * pq.ldcent;
    for (int i = tid; i < ldx; i += 256) {
        const float v = xq[i];
        xs[i] = v;
        rs[i] = i < d ? v - yc[i] : 0.f;  // Index::compute_residual (faiss/Index.cpp:107-112)
    }
    __syncthreads();
    if (tid == 0) {
        float d0 = 0.f;
        if (pq.by_residual) {
            if (!L2)  // precompute_list_tables_IP: <x, y_C> (faiss/IndexIVFPQ.cpp:612-628)
                d0 = ref_dist_s<false>(xs, yc, d);
            else if (pq.table1)
                d0 = cd;
        }
        *sd0 = d0;
    }
    for (int ent = tid; ent < M * 256; ent += 256) {
        const int m = ent >> 8;
        const float* c = pq.pq_cent + (int64_t)ent * dsub;
        float v;
        if (!L2 || !pq.by_residual) {
            // IP table of x (init_query_IP) / distance table of x (not by residual)
            v = ny_entry<L2>(xs + m * dsub, c, dsub);
        } else if (pq.table1) {
            const float P = fmaf(2.f, ny_entry<false>(yc + m * dsub, c, dsub),
                                 ref_dist_s<false>(c, c, dsub));
            v = fmaf(-2.f, ny_entry<false>(xs + m * dsub, c, dsub), P);
        } else {
            v = ny_entry<true>(rs + m * dsub, c, dsub);
        }
        lut[ent] = v;
    }
    __syncthreads();
    return *sd0;
}

__device__ __forceinline__ float ex_pq_code(const float* lut, int M, const uint8_t* code) {
    return pq_code_sum(M, [&](int m) { return lut[m * 256 + code[m]]; });
}

// one 256-thread workgroup per (query, probe): tables, then a thread per row
// sums its code in the distance_four_codes order.
template <bool L2>
__global__ __launch_bounds__(256) void k_ex_pq(const float* __restrict__ x, int ldx, int d, int np,
                                               const int32_t* __restrict__ assign,
                                               const float* __restrict__ cdis,
                                               const uint32_t* __restrict__ lim,
                                               const uint32_t* __restrict__ list_off,
                                               const uint32_t* __restrict__ list_len, int nlist,
                                               ExactPQ pq, const uint8_t* __restrict__ sel,
                                               const uint32_t* __restrict__ eoff, int64_t cap,
                                               uint32_t* __restrict__ okeys,
                                               uint32_t* __restrict__ orows, int64_t e0) {
    extern __shared__ float lut[];
    const int64_t e = e0 + blockIdx.x;
    const int64_t q = e / np;
    const int32_t key = assign[e];
    if (key < 0 || key >= nlist) return;
    const uint32_t len = lim ? lim[e] : list_len[key];
    if (len == 0) return;
    const float d0 =
            ex_pq_tables<L2>(x + q * ldx, ldx, d, key, cdis ? cdis[e] : 0.f, pq, lut);
    const uint32_t off = list_off[key];
    const int64_t base = q * cap + eoff[e];
    for (uint32_t r = threadIdx.x; r < len; r += 256) {
        const uint32_t row = off + r;
        uint32_t k = EX_SKIP;
        if (!sel || sel[row])
            k = ex_key(d0 + ex_pq_code(lut, pq.M, pq.codes + (int64_t)row * pq.cs), L2);
        okeys[base + r] = k;
        orows[base + r] = row;
    }
}

// IVF-PQ range scan, any geometry / metric (faiss/IndexIVFPQ.cpp:1254-1279
// scan_codes_range with RangeSearchResults :780-799: kept when
// C::cmp(radius, dis)).  Workgroup per (query, probe); pass 1 counts, pass 2
// writes the hits in row order at offsets[qp] (ordered block prefix).
template <bool L2, bool FILL>
__global__ __launch_bounds__(256) void k_ex_pq_range(
        const float* __restrict__ x, int ldx, int d, int np, const int32_t* __restrict__ assign,
        const float* __restrict__ cdis, const uint32_t* __restrict__ list_off,
        const uint32_t* __restrict__ list_len, int nlist, ExactPQ pq, float radius,
        const uint8_t* __restrict__ sel, const int64_t* __restrict__ ids,
        const uint32_t* __restrict__ row_list, int store_pairs, uint32_t* __restrict__ counts,
        const uint64_t* __restrict__ offsets, float* __restrict__ outD,
        int64_t* __restrict__ outI, int64_t e0) {
    extern __shared__ float lut[];
    __shared__ uint32_t wsum[4];
    const int64_t e = e0 + blockIdx.x;
    const int64_t q = e / np;
    const int32_t key = assign[e];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t cnt = 0;
    if (key >= 0 && key < nlist && list_len[key] > 0) {
        const uint32_t len = list_len[key], off = list_off[key];
        const float d0 =
                ex_pq_tables<L2>(x + q * ldx, ldx, d, key, cdis ? cdis[e] : 0.f, pq, lut);
        const uint64_t base = FILL ? offsets[e] : 0;
        for (uint32_t r0 = 0; r0 < len; r0 += 256) {
            const uint32_t r = r0 + tid;
            bool hit = false;
            float dis = 0.f;
            if (r < len && (!sel || sel[off + r])) {
                dis = d0 + ex_pq_code(lut, pq.M, pq.codes + (int64_t)(off + r) * pq.cs);
                hit = L2 ? dis < radius : dis > radius;
            }
            const uint64_t bm = __ballot(hit);
            if (lane == 0) wsum[wid] = (uint32_t)__popcll(bm);
            __syncthreads();
            uint32_t bpre = 0, btot = 0;
#pragma unroll
            for (int w = 0; w < 4; w++) {
                bpre += w < wid ? wsum[w] : 0u;
                btot += wsum[w];
            }
            if (FILL && hit) {
                const uint64_t o =
                        base + cnt + bpre + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
                outD[o] = dis;
                const uint32_t row = off + r;
                outI[o] = store_pairs ? (((int64_t)key << 32) | (int64_t)r) : ids[row];
            }
            cnt += btot;
            __syncthreads();
        }
    }
    if (!FILL && tid == 0) counts[e] = cnt;
}

// ---------------------------------------------------------------- select
struct SrcIVF {
    const uint32_t* keys;
    const uint32_t* rows;
    const uint32_t* total;
    int64_t cap;
    const int64_t* ids;
    const uint32_t* row_list;
    const uint32_t* list_off;
    int store_pairs;
    unsigned long long* qdone;  // per query: completion stamp (search_stats), or nullptr
    __device__ int64_t count(int64_t q) const { return total[q]; }
    __device__ void done(int64_t q) const {
        if (qdone) qdone[q] = __builtin_amdgcn_s_memrealtime();
    }
    __device__ uint32_t key(int64_t q, int64_t i) const { return keys[q * cap + i]; }
    __device__ int64_t label(int64_t q, int64_t i) const {
        const uint32_t row = rows[q * cap + i];
        if (store_pairs) {  // lo_build(list_no, offset) (faiss/invlists/InvertedLists.h)
            const uint32_t l = row_list[row];
            return ((int64_t)l << 32) | (int64_t)(row - list_off[l]);
        }
        return ids[row];
    }
};

struct SrcDense {
    const float* D;
    int64_t ldD, ny, col0;
    int l2;
    __device__ int64_t count(int64_t) const { return ny; }
    __device__ uint32_t key(int64_t q, int64_t i) const { return ex_key(D[q * ldD + i], l2); }
    __device__ int64_t label(int64_t, int64_t i) const { return col0 + i; }
    __device__ void done(int64_t) const {}
};

// GS: the collection arrays in global scratch (gs_words 64-bit words per
// query) instead of LDS — k beyond what one work group's LDS holds
template <class Src, class OutIdx, bool GS = false>
__global__ __launch_bounds__(256) void k_ex_select(Src src, int k, int l2, float* __restrict__ D,
                                                   OutIdx* __restrict__ I, int64_t ldo,
                                                   unsigned long long* __restrict__ gs = nullptr,
                                                   int64_t gs_words = 0) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t sh_b, sh_kk, sh_all, nlt, neq;
    extern __shared__ unsigned long long smem[];
    const int KS = k <= 1 ? 1 : 1 << (32 - __clz(k - 1));  // pow2 >= k
    unsigned long long* arr = GS ? gs + (int64_t)blockIdx.x * gs_words : smem;
    int64_t* oid = (int64_t*)arr;                           // [KS]
    int64_t* eqid = oid + KS;                               // [k]
    uint32_t* okey = (uint32_t*)(eqid + k);                 // [KS]
    const int64_t q = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t C = src.count(q);
    if (tid == 0) {
        sh_all = 0;
        nlt = 0;
        neq = 0;
    }
    // ---- radix select of the k-th smallest key
    uint32_t prefix = 0, kk = (uint32_t)k;
    bool all = false;
    for (int shift = 24; shift >= 0; shift -= 8) {
        hist[tid] = 0;
        __syncthreads();
        const uint32_t hmask = shift == 24 ? 0u : (0xffffffffu << (shift + 8));
        for (int64_t i = tid; i < C; i += 256) {
            const uint32_t key = src.key(q, i);
            if ((key & hmask) == (prefix & hmask)) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t cum = 0;
            int b = 0;
            for (; b < 256; b++) {
                if (cum + hist[b] >= kk) break;
                cum += hist[b];
            }
            if (b == 256) {
                sh_all = 1;
            } else {
                sh_b = (uint32_t)b;
                sh_kk = kk - cum;
            }
        }
        __syncthreads();
        if (sh_all) {
            all = true;
            break;
        }
        prefix |= sh_b << shift;
        kk = sh_kk;
    }
    const uint32_t vkey = prefix;
    if (!all && vkey == EX_SKIP) all = true;  // fewer than k admissible candidates
    // ---- ordered collection
    const uint32_t want_lt = all ? 0u : (uint32_t)k - kk;
    int64_t run_le = 0;
    for (int64_t c0 = 0; c0 < C; c0 += 256) {
        const int64_t i = c0 + tid;
        const uint32_t key = i < C ? src.key(q, i) : EX_SKIP;
        if (all) {
            if (key != EX_SKIP) {
                const uint32_t slot = atomicAdd(&nlt, 1u);
                okey[slot] = key;
                oid[slot] = src.label(q, i);
            }
            continue;
        }
        const bool lt = key < vkey, eq = key == vkey;
        const uint64_t bm = __ballot(lt || eq);
        const uint32_t wpre = (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wid] = (uint32_t)__popcll(bm);
        __syncthreads();
        uint32_t bpre = 0, btot = 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            bpre += w < wid ? wsum[w] : 0u;
            btot += wsum[w];
        }
        const int64_t rank = run_le + bpre + wpre;
        if (lt) {
            const uint32_t slot = atomicAdd(&nlt, 1u);
            okey[slot] = key;
            oid[slot] = src.label(q, i);
        } else if (eq && rank < k) {
            const uint32_t slot = atomicAdd(&neq, 1u);
            eqid[slot] = src.label(q, i);
        }
        run_le += btot;
        __syncthreads();
        if (nlt == want_lt && run_le >= k) break;  // block-uniform
    }
    __syncthreads();
    // ---- tied candidates: the kk smallest labels (IP: largest)
    const uint32_t n_lt = nlt, n_eq = neq;
    uint32_t K = n_lt;
    if (!all) {
        for (uint32_t t = tid; t < n_eq; t += 256) {
            const int64_t my = eqid[t];
            uint32_t r = 0;
            for (uint32_t j = 0; j < n_eq; j++) {
                const int64_t o = eqid[j];
                r += (l2 ? o < my : o > my) || (o == my && j < t);
            }
            if (r < kk) {
                okey[n_lt + r] = vkey;
                oid[n_lt + r] = my;
            }
        }
        K = n_lt + kk;
    }
    // ---- heap_reorder order: bitonic sort of (key, label) in LDS
    const int64_t pad_id = l2 ? LLONG_MAX : LLONG_MIN;
    for (int t = tid; t < KS; t += 256)
        if ((uint32_t)t >= K) {
            okey[t] = EX_SKIP;
            oid[t] = pad_id;
        }
    __syncthreads();
    for (int size = 2; size <= KS; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < KS / 2; t += 256) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint32_t ka = okey[lo], kb = okey[hi];
                const int64_t ia = oid[lo], ib = oid[hi];
                const bool a_first = ka < kb || (ka == kb && (l2 ? ia < ib : ia > ib));
                if (a_first != up) {
                    okey[lo] = kb;
                    okey[hi] = ka;
                    oid[lo] = ib;
                    oid[hi] = ia;
                }
            }
            __syncthreads();
        }
    for (int t = tid; t < k; t += 256) {
        const bool ok = (uint32_t)t < K;
        D[q * ldo + t] = ok ? ex_dis(okey[t], l2) : (l2 ? FLT_MAX : -FLT_MAX);
        I[q * ldo + t] = ok ? (OutIdx)oid[t] : (OutIdx)-1;
    }
    if (tid == 0) src.done(q);
}

size_t select_lds(int k) {
    const size_t KS = k <= 1 ? 1 : (size_t)1 << (32 - __builtin_clz((unsigned)k - 1));
    return KS * (sizeof(int64_t) + sizeof(uint32_t)) + (size_t)k * sizeof(int64_t);
}

}  // namespace

// (query, probe) work groups per launch of the k_ex_* scans: 2^20 x 256
// work-items stays far inside a dispatch's 32-bit count (common.h kgrid)
constexpr int64_t kExEntriesPerLaunch = (int64_t)1 << 20;

// A query's candidate slot holds every row of its probes: np * max_list_len.
// (Not clamped to the arena size: a caller-supplied assignment may name a list
// twice, and the reference then scans it twice.)
int64_t ivf_exact_chunk(int64_t n, int np, uint32_t max_list_len, int64_t* cap_out) {
    const int64_t cap = std::max<int64_t>(1, (int64_t)np * max_list_len);
    *cap_out = cap;
    const int64_t budget = (int64_t)1 << 30;  // bytes of keys + rows per chunk
    return std::max<int64_t>(1, std::min<int64_t>(n, budget / (cap * 8)));
}

void ivf_exact_search(const ExactScanArgs& a, uint32_t* eoff, uint32_t* total, uint32_t* keys,
                      uint32_t* rows, int64_t cap, float* D, int64_t* I, hipStream_t s) {
    if (a.n <= 0) return;
    FAISS_THROW_IF_NOT_FMT(a.k >= 1 && a.k <= kMaxKExact, "k = %d must be in [1, %d]", a.k,
                           kMaxKExact);
    k_ex_offsets<<<kgrid(cdiv(a.n, 256), 256), dim3(256), 0, s>>>(
            a.assign, a.n, a.np, a.list_len, a.nlist, a.lim, eoff, total);
    HIP_LAUNCH_CHECK();
    const int64_t entries = a.n * (int64_t)a.np;
    FAISS_THROW_IF_NOT(entries < ((int64_t)1 << 31));
    if (a.pq.M > 0) {
        const size_t lds = sizeof(float) * ((size_t)a.pq.M * 256 + 2 * (size_t)a.ldx + 1);
        FAISS_THROW_IF_NOT_FMT(lds <= 160 * 1024, "IVF-PQ table of M = %d does not fit in LDS",
                               a.pq.M);
        const void* kfn = a.l2 ? (const void*)k_ex_pq<true> : (const void*)k_ex_pq<false>;
        if (lds > 64 * 1024)
            HIP_CHECK(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)lds));
#define EXPQ(L2)                                                                             \
    k_ex_pq<L2><<<kgrid(ne, 256), dim3(256), lds, s>>>(                                     \
            a.x, a.ldx, a.d, a.np, a.assign, a.cdis, a.lim, a.list_off, a.list_len, a.nlist, \
            a.pq, a.sel, eoff, cap, keys, rows, e0)
        for (int64_t e0 = 0; e0 < entries; e0 += kExEntriesPerLaunch) {
            const int64_t ne = std::min(kExEntriesPerLaunch, entries - e0);
            if (a.l2)
                EXPQ(true);
            else
                EXPQ(false);
        }
#undef EXPQ
    } else {
        const size_t lds = sizeof(float) * a.ldx;
        for (int64_t e0 = 0; e0 < entries; e0 += kExEntriesPerLaunch) {
            const int64_t ne = std::min(kExEntriesPerLaunch, entries - e0);
            if (a.l2)
                k_ex_flat<true><<<kgrid(ne, 64), dim3(64), lds, s>>>(
                        a.x, a.ldx, a.d, a.np, a.assign, a.lim, a.list_off, a.list_len,
                        a.nlist, a.codes, a.ldc, a.sel, eoff, cap, keys, rows, e0);
            else
                k_ex_flat<false><<<kgrid(ne, 64), dim3(64), lds, s>>>(
                        a.x, a.ldx, a.d, a.np, a.assign, a.lim, a.list_off, a.list_len,
                        a.nlist, a.codes, a.ldc, a.sel, eoff, cap, keys, rows, e0);
        }
    }
    HIP_LAUNCH_CHECK();
    SrcIVF src{keys, rows, total, cap, a.ids, a.row_list, a.list_off, a.store_pairs, a.qdone};
    k_ex_select<SrcIVF, int64_t><<<kgrid(a.n, 256), dim3(256), select_lds(a.k), s>>>(
            src, a.k, a.l2, D, I, a.k);
    HIP_LAUNCH_CHECK();
}

void ivfpq_range_exact(const ExactScanArgs& a, float radius, uint32_t* counts,
                       const uint64_t* offsets, float* outD, int64_t* outI, hipStream_t s) {
    if (a.n <= 0 || a.np <= 0) return;
    const int64_t entries = a.n * (int64_t)a.np;
    FAISS_THROW_IF_NOT(entries < ((int64_t)1 << 31) && a.pq.M > 0);
    const size_t lds = sizeof(float) * ((size_t)a.pq.M * 256 + 2 * (size_t)a.ldx + 1);
    FAISS_THROW_IF_NOT_FMT(lds <= 160 * 1024, "IVF-PQ table of M = %d does not fit in LDS",
                           a.pq.M);
#define EXR(L2, F)                                                                            \
    do {                                                                                      \
        if (lds > 64 * 1024)                                                                  \
            HIP_CHECK(hipFuncSetAttribute((const void*)k_ex_pq_range<L2, F>,                  \
                                          hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                          (int)lds));                                         \
        for (int64_t e0 = 0; e0 < entries; e0 += kExEntriesPerLaunch)                        \
            k_ex_pq_range<L2, F>                                                              \
                    <<<kgrid(std::min(kExEntriesPerLaunch, entries - e0), 256), dim3(256), lds, \
                       s>>>(a.x, a.ldx, a.d, a.np, a.assign, a.cdis, a.list_off, a.list_len,  \
                            a.nlist, a.pq, radius, a.sel, a.ids, a.row_list, a.store_pairs,   \
                            counts, offsets, outD, outI, e0);                                 \
    } while (0)
    if (a.l2) {
        if (offsets) EXR(true, true);
        else EXR(true, false);
    } else {
        if (offsets) EXR(false, true);
        else EXR(false, false);
    }
#undef EXR
    HIP_LAUNCH_CHECK();
}

// merge_knn_results (faiss/utils/Heap.cpp:159-230) for any k: per query the
// heap over the shard heads is a scan of the heads, (dis, shard) with the
// lower shard first for L2 (CMin) and the higher shard first for IP (CMax);
// a shard's list ends at its first label < 0.  Thread per query, positions in
// LDS.  Inputs [nshard][n][kin].
constexpr int MG_T = 64, MG_MAXS = 256;
__global__ __launch_bounds__(MG_T) void k_merge_general(const float* __restrict__ all_d,
                                                        const int64_t* __restrict__ all_i,
                                                        int64_t n, int kin, int nshard, int k,
                                                        int l2, float* __restrict__ out_d,
                                                        int64_t* __restrict__ out_i) {
    __shared__ uint16_t pos[MG_T * MG_MAXS];
    const int64_t q = (int64_t)blockIdx.x * MG_T + threadIdx.x;
    if (q >= n) return;
    uint16_t* p = pos + threadIdx.x * MG_MAXS;
    for (int s = 0; s < nshard; s++) p[s] = 0;
    const int64_t stride = n * (int64_t)kin;
    int j = 0;
    for (; j < k; j++) {
        int bs = -1;
        float bv = 0.f;
        for (int s = 0; s < nshard; s++) {
            if (p[s] >= kin) continue;
            const int64_t o = s * stride + q * kin + p[s];
            if (all_i[o] < 0) continue;
            const float v = all_d[o];
            if (bs < 0 || (l2 ? (v < bv) : (v > bv)) || (v == bv && !l2)) {
                bs = s;
                bv = v;
            }
        }
        if (bs < 0) break;
        const int64_t o = bs * stride + q * kin + p[bs];
        out_d[q * k + j] = bv;
        out_i[q * k + j] = all_i[o];
        p[bs]++;
    }
    for (; j < k; j++) {
        out_d[q * k + j] = l2 ? FLT_MAX : -FLT_MAX;
        out_i[q * k + j] = -1;
    }
}

void merge_rows_general(const float* cand_d, const int64_t* cand_i, int64_t n, int nshard,
                        int kin, int k, int metric_l2, float* out_d, int64_t* out_i,
                        hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT_FMT(nshard >= 1 && nshard <= MG_MAXS, "nshard = %d must be in [1, %d]",
                           nshard, MG_MAXS);
    FAISS_THROW_IF_NOT(kin >= 1 && kin <= 65535 && k >= 1);
    k_merge_general<<<kgrid(cdiv(n, MG_T), MG_T), dim3(MG_T), 0, s>>>(
            cand_d, cand_i, n, kin, nshard, k, metric_l2, out_d, out_i);
    HIP_LAUNCH_CHECK();
}

template <class OutIdx>
void select_rows_exact(const float* Dt, int64_t nx, int64_t ny, int64_t ldD, int k, int metric_l2,
                       int64_t col0, float* out_d, OutIdx* out_i, int64_t ldo, hipStream_t s,
                       DeviceBuffer* scratch) {
    if (nx <= 0) return;
    FAISS_THROW_IF_NOT_FMT(k >= 1, "k = %d must be >= 1", k);
    if (k <= kMaxKExact) {
        SrcDense src{Dt, ldD, ny, col0, metric_l2};
        k_ex_select<SrcDense, OutIdx><<<kgrid(nx, 256), dim3(256), select_lds(k), s>>>(
                src, k, metric_l2, out_d, out_i, ldo);
        HIP_LAUNCH_CHECK();
        return;
    }
    // k > kMaxKExact (e.g. nprobe in the thousands): the same select with its
    // arrays in global scratch, queries in chunks of a 256 MiB scratch
    FAISS_THROW_IF_NOT_MSG(scratch, "select_rows_exact: k > 2048 needs a scratch buffer");
    const int64_t words = (int64_t)cdiv(select_lds(k), sizeof(unsigned long long));
    const int64_t qc = std::max<int64_t>(1, std::min<int64_t>(nx, ((int64_t)256 << 20) / (8 * words)));
    scratch->reserve((size_t)qc * words * 8);
    for (int64_t q0 = 0; q0 < nx; q0 += qc) {
        const int64_t nq = std::min(qc, nx - q0);
        SrcDense src{Dt + q0 * ldD, ldD, ny, col0, metric_l2};
        k_ex_select<SrcDense, OutIdx, true><<<kgrid(nq, 256), dim3(256), 0, s>>>(
                src, k, metric_l2, out_d + q0 * ldo, out_i + q0 * ldo, ldo,
                scratch->as<unsigned long long>(), words);
        HIP_LAUNCH_CHECK();
    }
}
template void select_rows_exact<int32_t>(const float*, int64_t, int64_t, int64_t, int, int,
                                         int64_t, float*, int32_t*, int64_t, hipStream_t,
                                         DeviceBuffer*);
template void select_rows_exact<int64_t>(const float*, int64_t, int64_t, int64_t, int, int,
                                         int64_t, float*, int64_t*, int64_t, hipStream_t,
                                         DeviceBuffer*);

}  // namespace kern
}  // namespace faiss_amd
