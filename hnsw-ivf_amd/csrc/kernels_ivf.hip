// kernels_ivf.hip — list-centric batched IVF-Flat scan for gfx950.
//
// Reference hot loop: faiss/IndexIVFFlat.cpp:155-179 (IVFFlatScanner::
// scan_codes: for each code, dis = fvec_L2sqr(x, y, d); heap_replace_top on
// strict improvement) driven per query by faiss/IndexIVF.cpp:595-631.
//
// MI355X design: instead of streaming every probed list once per query (the
// CPU order, ~4 MB/query at nlist 4096 nprobe 32), the (query, list) pairs of
// the whole batch are bucketed by list.  A workgroup owns one list and up to
// 64 of the queries probing it: the list is read from HBM once per 64 queries,
// tiles of 64 queries x 64 codes live in LDS, and each thread computes a 4x4
// micro-tile of exact sum (x-y)^2 (same arithmetic as the reference, not the
// norm expansion).  Each wave then folds its 16 queries' distance rows into
// wave64 top-k queues and the per-(query, list) top-k is written out; a
// second kernel merges the nprobe partial lists of each query.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cfloat>

#include "common.h"
#include "kernels.h"
#include "ref_arith.h"
#include "wave_select.h"

namespace faiss_amd {
namespace kern {

// ---------------------------------------------------------------- bucketing
// counts per list; the value returned by the atomic is the entry's slot in
// its bucket, so the fill needs no second round of atomics
__global__ void k_bucket_count(const int32_t* __restrict__ assign, int64_t total,
                               const uint32_t* __restrict__ list_len, int nlist,
                               uint32_t* __restrict__ counts, uint32_t* __restrict__ pos) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    int l = assign[e];
    if (l >= 0 && l < nlist && list_len[l] > 0) pos[e] = atomicAdd(&counts[l], 1u);
}

// Same with a block-local LDS histogram (nlist <= BC_MAXL): BC_PER entries
// per thread take their slot from an LDS atomic, then one global atomic per
// non-empty bin reserves the block's range of each bucket.
constexpr int BC_PER = 16;
constexpr int BC_MAXL = 16384;
__global__ __launch_bounds__(1024) void k_bucket_count_lds(const int32_t* __restrict__ assign,
                                                           int64_t total,
                                                           const uint32_t* __restrict__ list_len,
                                                           int nlist, uint32_t* __restrict__ counts,
                                                           uint32_t* __restrict__ pos) {
    extern __shared__ uint32_t hist[];  // [min(nlist, BC_MAXL)]
    const int t = threadIdx.x;
    // lists [lbase, lbase + nl) of this block row (nlist > BC_MAXL: one row
    // of blocks per range, each reading every entry)
    const int lbase = (int)blockIdx.y * BC_MAXL;
    const int nl = min(BC_MAXL, nlist - lbase);
    for (int i = t; i < nl; i += 1024) hist[i] = 0u;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * 1024 * BC_PER;
    int ll[BC_PER];
    uint32_t lp[BC_PER];
#pragma unroll
    for (int j = 0; j < BC_PER; j++) {
        const int64_t e = base + (int64_t)j * 1024 + t;
        int l = -1;
        if (e < total) {
            l = assign[e];
            if (!(l >= 0 && l < nlist && list_len[l] > 0)) l = -1;
        }
        l = (l >= lbase && l < lbase + nl) ? l - lbase : -1;
        ll[j] = l;
        lp[j] = l >= 0 ? atomicAdd(&hist[l], 1u) : 0u;
    }
    __syncthreads();
    for (int i = t; i < nl; i += 1024) {
        const uint32_t c = hist[i];
        if (c) hist[i] = atomicAdd(&counts[lbase + i], c);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < BC_PER; j++) {
        const int64_t e = base + (int64_t)j * 1024 + t;
        if (ll[j] >= 0) pos[e] = hist[ll[j]] + lp[j];
    }
}

// single-workgroup exclusive scan of counts -> bucket_off, ceil(counts/QT)
// -> item_off; per work item its list when asked.  Chunks of 4096 lists:
// 4 consecutive counts per thread, shuffle scan per wave, 16 wave totals
// through LDS; a running carry between chunks.
__global__ __launch_bounds__(1024) void k_bucket_scan(const uint32_t* __restrict__ counts,
                                                      int nlist, int QT,
                                                      uint32_t* __restrict__ bucket_off,
                                                      uint32_t* __restrict__ item_off,
                                                      uint32_t* __restrict__ item_list,
                                                      uint32_t* __restrict__ zero_next) {
    __shared__ uint32_t wb[16], wi[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t carry_b = 0, carry_i = 0;
    for (int c0 = 0; c0 < nlist; c0 += 4096) {
        const int l0 = c0 + 4 * t;
        uint32_t c[4], n[4];
        uint32_t sb = 0, si = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            c[j] = l0 + j < nlist ? counts[l0 + j] : 0u;
            if (zero_next && l0 + j < nlist) zero_next[l0 + j] = 0u;
            n[j] = (c[j] + QT - 1) / QT;
            sb += c[j];
            si += n[j];
        }
        // inclusive wave scan of the thread sums
        uint32_t ib = sb, ii = si;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t vb = __shfl_up(ib, off), vi = __shfl_up(ii, off);
            if (lane >= off) {
                ib += vb;
                ii += vi;
            }
        }
        if (lane == 63) {
            wb[w] = ib;
            wi[w] = ii;
        }
        __syncthreads();
        uint32_t pb = carry_b, pi = carry_i, tb = 0, ti = 0;
#pragma unroll
        for (int v = 0; v < 16; v++) {
            pb += v < w ? wb[v] : 0u;
            pi += v < w ? wi[v] : 0u;
            tb += wb[v];
            ti += wi[v];
        }
        __syncthreads();  // wb / wi are rewritten by the next chunk
        uint32_t rb = pb + ib - sb, ri = pi + ii - si;  // exclusive prefix of this thread
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (l0 + j < nlist) {
                bucket_off[l0 + j] = rb;
                item_off[l0 + j] = ri;
                if (item_list)
                    for (uint32_t i = 0; i < n[j]; i++) item_list[ri + i] = (uint32_t)(l0 + j);
            }
            rb += c[j];
            ri += n[j];
        }
        carry_b += tb;
        carry_i += ti;
    }
    if (t == 0) {
        bucket_off[nlist] = carry_b;
        item_off[nlist] = carry_i;
    }
}

__global__ void k_bucket_fill(const int32_t* __restrict__ assign, int64_t total,
                              const uint32_t* __restrict__ list_len, int nlist, int QT,
                              const uint32_t* __restrict__ bucket_off,
                              const uint32_t* __restrict__ item_off,
                              const uint32_t* __restrict__ pos, uint32_t* __restrict__ entries,
                              uint32_t* __restrict__ item_entries, ItemDesc* __restrict__ item_desc,
                              const uint32_t* __restrict__ counts,
                              const uint32_t* __restrict__ list_off,
                              uint32_t* __restrict__ mkeys, ProbeRec* __restrict__ mrecs,
                              int ke) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    int l = assign[e];
    if (l >= 0 && l < nlist && list_len[l] > 0) {
        const uint32_t p = pos[e];
        if (item_entries) {
            const uint32_t item = item_off[l] + p / QT;
            item_entries[item * QT + p % QT] = (uint32_t)e;
            if (p % QT == 0) {  // the item's first entry writes its descriptor
                ItemDesc dsc;
                dsc.l = (uint32_t)l;
                dsc.nq = min((uint32_t)QT, counts[l] - p);
                dsc.len = list_len[l];
                dsc.off = list_off[l];
                item_desc[item] = dsc;
            }
        } else {
            entries[bucket_off[l] + p] = (uint32_t)e;
        }
    } else if (mkeys) {
        for (int i = 0; i < ke; i++) mkeys[e * ke + i] = 0xffffffffu;
        ProbeRec pr;
        for (int i = 0; i < 4; i++) pr.pb[i] = WS_INF;
        pr.mmax = 0.f;
        pr.off = 0u;
        pr.len = 0u;
        pr.pad = 0u;
        mrecs[e] = pr;
    }
}

// grid-stride partial counts per thread, one atomic pair per work-group
__global__ __launch_bounds__(256) void k_ivf_visit_stats(const int32_t* __restrict__ assign,
                                                         int64_t total,
                                                         const uint32_t* __restrict__ list_len,
                                                         int nlist,
                                                         const uint32_t* __restrict__ lim,
                                                         unsigned long long* __restrict__ stats) {
    unsigned long long nv = 0, nd = 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int l = assign[e];
        uint32_t len = 0;
        if (l >= 0 && l < nlist) len = lim ? lim[e] : list_len[l];
        nv += len > 0 ? 1 : 0;
        nd += len;
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        nv += __shfl_xor(nv, m);
        nd += __shfl_xor(nd, m);
    }
    __shared__ unsigned long long red[2][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = nv;
        red[1][w] = nd;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        const unsigned long long b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        if (a) {
            atomicAdd(&stats[0], a);
            atomicAdd(&stats[1], b);
        }
    }
}

void ivf_visit_stats(const int32_t* assign, int64_t total, const uint32_t* list_len, int nlist,
                     const uint32_t* lim, unsigned long long* stats, hipStream_t s) {
    if (total <= 0) return;
    const int64_t grid = std::min<int64_t>(cdiv(total, 256), 1024);
    k_ivf_visit_stats<<<dim3((unsigned)grid), dim3(256), 0, s>>>(assign, total, list_len, nlist,
                                                                 lim, stats);
    HIP_LAUNCH_CHECK();
}

// one thread per query: faiss/IndexIVF.cpp:609-622 (nscan, list_size_max)
__global__ void k_probe_limits(const int32_t* __restrict__ assign, int64_t n, int nprobe,
                               const uint32_t* __restrict__ list_len, int nlist,
                               int64_t max_codes, int32_t* __restrict__ assign_out,
                               uint32_t* __restrict__ lim) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    int64_t nscan = 0;
    for (int r = 0; r < nprobe; r++) {
        const int64_t e = q * nprobe + r;
        const int l = assign[e];
        const bool ok = l >= 0 && l < nlist && nscan < max_codes;
        const uint32_t len = ok ? list_len[l] : 0u;
        const uint32_t take = (uint32_t)min((int64_t)len, max_codes - nscan);
        assign_out[e] = ok ? l : -1;
        lim[e] = take;
        nscan += take;
    }
}

void probe_limits(const int32_t* assign, int64_t n, int nprobe, const uint32_t* list_len,
                  int nlist, int64_t max_codes, int32_t* assign_out, uint32_t* lim,
                  hipStream_t s) {
    if (n <= 0) return;
    k_probe_limits<<<dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s>>>(
            assign, n, nprobe, list_len, nlist, max_codes, assign_out, lim);
    HIP_LAUNCH_CHECK();
}

void ivf_bucket(const int32_t* assign, int64_t n, int nprobe, const uint32_t* list_len,
                const uint32_t* list_off, int nlist, int QT, IVFBuckets b, hipStream_t s) {
    int64_t total = n * nprobe;
    FAISS_THROW_IF_NOT_MSG(total < (1ll << 32), "n * nprobe must fit in 32 bits");
    if (!b.counts_next) HIP_CHECK(hipMemsetAsync(b.counts, 0, sizeof(uint32_t) * nlist, s));
    if (total > 0) {
        const int nr = (int)cdiv(nlist, BC_MAXL);  // list ranges (LDS histogram each)
        k_bucket_count_lds<<<dim3((unsigned)cdiv(total, 1024 * BC_PER), (unsigned)nr), dim3(1024),
                             sizeof(uint32_t) * std::min(nlist, BC_MAXL), s>>>(
                assign, total, list_len, nlist, b.counts, b.cursor);
        HIP_LAUNCH_CHECK();
    }
    k_bucket_scan<<<dim3(1), dim3(1024), 0, s>>>(b.counts, nlist, QT, b.bucket_off, b.item_off,
                                                 b.item_list, b.counts_next);
    HIP_LAUNCH_CHECK();
    if (total > 0) {
        k_bucket_fill<<<dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s>>>(
                assign, total, list_len, nlist, QT, b.bucket_off, b.item_off, b.cursor, b.entries,
                b.item_entries, b.item_desc, b.counts, list_off, b.mark_keys, b.mark_recs,
                b.mark_ke);
        HIP_LAUNCH_CHECK();
    }
}

// ---------------------------------------------------------------- scan
constexpr int SQT = 64;   // queries per work item
constexpr int SVT = 32;   // codes per tile (8 reference-order partial sums per pair)
constexpr int SDC = 128;  // dims per LDS chunk
constexpr int SSD = SDC + 4;  // LDS row stride (floats): 528 B, 16-B aligned

// KQ > 0: thread-queue selection (4 threads per query, k <= KQ);
// KQ == 0: wave64 bitonic queues (16 queries per wave, any k <= 64).
template <bool L2, int KQ>
__global__ __launch_bounds__(256, 2) void k_ivf_flat_scan(
        const float* __restrict__ x, int ldx, const float* __restrict__ codes, int ldc,
        const int64_t* __restrict__ ids, const uint32_t* __restrict__ list_off,
        const uint32_t* __restrict__ list_len, int nlist, int dp, int dp_true, int nprobe,
        int k, const uint32_t* __restrict__ bucket_off, const uint32_t* __restrict__ item_off,
        const uint32_t* __restrict__ entries, const uint32_t* __restrict__ lim,
        const uint8_t* __restrict__ sel, float* __restrict__ part_k1,
        long long* __restrict__ part_k2) {
    // one array: the end-of-kernel queue merge reuses it (64 KB at KQ=32)
    __shared__ __attribute__((aligned(16))) float smem_xy[(SQT + 64) * SSD];
    float* Xs = smem_xy;
    float* Ys = smem_xy + SQT * SSD;
    __shared__ long long ids_s[64];
    __shared__ uint32_t ent_s[SQT];
    __shared__ int32_t qrow_s[SQT];
    __shared__ int32_t qlim_s[SQT];  // rows of the list scanned for each query

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int w = t >> 6;
    // XCD-aware order: blocks b and b+8 share an XCD (dispatch round-robin),
    // so groups of 4 consecutive work items (chunks of the same list) are
    // placed on one XCD and re-read the list from its L2.  Bijective on the
    // grid (a multiple of 32); affects speed only.
    const uint32_t xcd = blockIdx.x & 7u, rest = blockIdx.x >> 3;
    const uint32_t item = 4u * ((rest >> 2) * 8u + xcd) + (rest & 3u);
    const uint32_t total_items = item_off[nlist];
    if (item >= total_items) return;
    // list owning this item: largest l with item_off[l] <= item
    int lo = 0, hi = nlist;
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (item_off[mid] <= item) lo = mid; else hi = mid;
    }
    const int l = lo;
    const uint32_t chunk = item - item_off[l];
    const uint32_t qb = bucket_off[l] + chunk * SQT;
    const int nQ = (int)min((uint32_t)SQT, bucket_off[l + 1] - qb);
    const int len = (int)list_len[l];
    if (t < SQT) {
        uint32_t e = t < nQ ? entries[qb + t] : 0u;
        ent_s[t] = e;
        qrow_s[t] = t < nQ ? (int32_t)(e / (uint32_t)nprobe) : -1;
        qlim_s[t] = lim && t < nQ ? (int32_t)lim[e] : len;
    }
    const int64_t row0 = list_off[l];
    __syncthreads();

    const bool one_chunk = dp <= SDC;
    auto load_x = [&](int dc) {
        const int dl = min(SDC, dp - dc);
        for (int e = t; e < SQT * (SDC / 4); e += 256) {
            int r = e >> 5, c4 = e & 31;
            int kc = 4 * c4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            int qr = qrow_s[r];
            if (qr >= 0 && kc < dl) v = *(const float4*)(x + (int64_t)qr * ldx + dc + kc);
            *(float4*)(Xs + r * SSD + kc) = v;
        }
    };
    if (one_chunk) load_x(0);

    // selection state
    constexpr int NQW = KQ > 0 ? 1 : 16;  // wave path: 16 queues per lane
    float qd[NQW];
    long long qi[NQW];
    ThreadQueue<(KQ > 0 ? KQ : 1)> tq;
    if constexpr (KQ > 0) {
        tq.init();
    } else {
#pragma unroll
        for (int qq = 0; qq < NQW; qq++) {
            qd[qq] = WS_INF;
            qi[qq] = WS_NOID;
        }
    }
    const int qg = t >> 4, vg = t & 15;

    // register prefetch of the next code tile (d <= 128): its HBM latency
    // overlaps the current tile's compute and selection
    float4 pf[SVT * (SDC / 4) / 256];
    auto fetch = [&](int v0n) {
        const int nvn = min(SVT, len - v0n);
#pragma unroll
        for (int s = 0; s < SVT * (SDC / 4) / 256; s++) {
            const int e = t + 256 * s;
            const int r = e >> 5, kc = 4 * (e & 31);
            pf[s] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r < nvn && kc < dp)
                pf[s] = *(const float4*)(codes + (row0 + v0n + r) * (int64_t)ldc + kc);
        }
    };
    if (one_chunk && len > 0) fetch(0);

    // dims evaluated in the reference order (ref_arith.h): lanes over
    // i < n8, then the 4-term epilogue and the tail in the last chunk
    const int d = dp_true;
    const int n8 = d & ~7;
    for (int v0 = 0; v0 < len; v0 += SVT) {
        const int nv = min(SVT, len - v0);
        RefAcc8 acc[4][2];
        float res[4][2];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) acc[i][j].init();

        for (int dc = 0; dc < dp; dc += SDC) {
            const int dl = min(SDC, dp - dc);
            if (one_chunk) {
#pragma unroll
                for (int s = 0; s < SVT * (SDC / 4) / 256; s++) {
                    const int e = t + 256 * s;
                    *(float4*)(Ys + (e >> 5) * SSD + 4 * (e & 31)) = pf[s];
                }
                __syncthreads();
                if (v0 + SVT < len) fetch(v0 + SVT);
            } else {
                load_x(dc);
                for (int e = t; e < SVT * (SDC / 4); e += 256) {
                    int r = e >> 5, c4 = e & 31;
                    int kc = 4 * c4;
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (r < nv && kc < dl)
                        v = *(const float4*)(codes + (row0 + v0 + r) * (int64_t)ldc + dc + kc);
                    *(float4*)(Ys + r * SSD + kc) = v;
                }
                __syncthreads();
            }
            const int dmain = min(dl, max(0, n8 - dc));
            for (int dd = 0; dd < dmain; dd += 8) {
                float4 xa[4][2], yb[2][2];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    xa[i][0] = *(const float4*)(Xs + (qg + 16 * i) * SSD + dd);
                    xa[i][1] = *(const float4*)(Xs + (qg + 16 * i) * SSD + dd + 4);
                }
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    yb[j][0] = *(const float4*)(Ys + (vg + 16 * j) * SSD + dd);
                    yb[j][1] = *(const float4*)(Ys + (vg + 16 * j) * SSD + dd + 4);
                }
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        float* c = acc[i][j].c;
                        c[0] = ref_term_fma<L2>(xa[i][0].x, yb[j][0].x, c[0]);
                        c[1] = ref_term_fma<L2>(xa[i][0].y, yb[j][0].y, c[1]);
                        c[2] = ref_term_fma<L2>(xa[i][0].z, yb[j][0].z, c[2]);
                        c[3] = ref_term_fma<L2>(xa[i][0].w, yb[j][0].w, c[3]);
                        c[4] = ref_term_fma<L2>(xa[i][1].x, yb[j][1].x, c[4]);
                        c[5] = ref_term_fma<L2>(xa[i][1].y, yb[j][1].y, c[5]);
                        c[6] = ref_term_fma<L2>(xa[i][1].z, yb[j][1].z, c[6]);
                        c[7] = ref_term_fma<L2>(xa[i][1].w, yb[j][1].w, c[7]);
                    }
            }
            if (dc + dl >= dp) {
                // last chunk: reduce, epilogue, tail (dims n8 .. d-1 are here)
                const int e0 = n8 - dc;
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const float* xr = Xs + (qg + 16 * i) * SSD;
                        const float* yr = Ys + (vg + 16 * j) * SSD;
                        float r = acc[i][j].reduce();
                        int ii = e0;
                        if (d - n8 >= 4) {
                            const float t0 = ref_term<L2>(xr[e0], yr[e0]);
                            const float t1 = ref_term<L2>(xr[e0 + 1], yr[e0 + 1]);
                            const float t2 = ref_term<L2>(xr[e0 + 2], yr[e0 + 2]);
                            const float t3 = ref_term<L2>(xr[e0 + 3], yr[e0 + 3]);
                            r = r + ((t0 + t2) + (t1 + t3));
                            ii += 4;
                        }
                        for (; ii < d - dc; ii++) r = ref_term_fma<L2>(xr[ii], yr[ii], r);
                        res[i][j] = r;
                    }
            }
            __syncthreads();
        }
        // distance tile -> LDS (aliases the Y tile)
        float* Ds = Ys;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) Ds[(qg + 16 * i) * (SVT + 1) + vg + 16 * j] = res[i][j];
        if constexpr (KQ == 0) {
            if (t < SVT) ids_s[t] = t < nv ? (long long)ids[row0 + v0 + t] : 0ll;
        }
        __syncthreads();
        if constexpr (KQ > 0) {
            // thread (q = t>>2, s = t&3) owns codes s, s+4, ... of query q
            const int q = t >> 2, s4 = t & 3;
            if (q < nQ) {
                const int nvq = min(nv, qlim_s[q] - v0);
#pragma unroll 4
                for (int j = s4; j < nvq; j += 4) {
                    if (sel && !sel[row0 + v0 + j]) continue;  // IDSelector (use_sel)
                    float dis = Ds[q * (SVT + 1) + j];
                    float k1 = L2 ? dis : -dis;
                    if (k1 < FLT_MAX) {
                        const uint32_t r = (uint32_t)(v0 + j);
                        unsigned long long key =
                                ((unsigned long long)ordered_f32(k1) << 32) | (L2 ? r : ~r);
                        tq.push(key, k);
                    }
                }
            }
        } else {
            // wave w owns queries w*16 .. w*16+15
            const bool lane_ok = lane < nv && (!sel || sel[row0 + v0 + lane]);
            const long long my_id = ids_s[lane];
#pragma unroll
            for (int qq = 0; qq < NQW; qq++) {
                const int q = w * 16 + qq;
                if (q < nQ) {
                    float dis = Ds[q * (SVT + 1) + lane];
                    float k1;
                    long long k2;
                    to_key(L2 ? 1 : 0, dis, my_id, k1, k2);
                    if (!lane_ok || v0 + lane >= qlim_s[q] || !key_admissible(k1)) {
                        k1 = WS_INF;
                        k2 = WS_NOID;
                    }
                    wave_offer_q(qd[qq], qi[qq], k1, k2, k, lane);
                }
            }
        }
        __syncthreads();
    }
    if constexpr (KQ > 0) {
        // merge the 4 thread queues of each query through LDS
        unsigned long long* M = (unsigned long long*)Xs;  // [64][4][KQ] fits Xs+Ys
        const int q = t >> 2, s4 = t & 3;
#pragma unroll
        for (int i = 0; i < KQ; i++) M[(q * 4 + s4) * KQ + i] = tq.q[i];
        __syncthreads();
        if (t < nQ) {
            const unsigned long long* Mq = M + t * 4 * KQ;
            int p0 = 0, p1 = 0, p2 = 0, p3 = 0;
            const int64_t e = ent_s[t];
            for (int j = 0; j < k; j++) {
                unsigned long long h0 = p0 < KQ ? Mq[p0] : ~0ull;
                unsigned long long h1 = p1 < KQ ? Mq[KQ + p1] : ~0ull;
                unsigned long long h2 = p2 < KQ ? Mq[2 * KQ + p2] : ~0ull;
                unsigned long long h3 = p3 < KQ ? Mq[3 * KQ + p3] : ~0ull;
                unsigned long long m01 = h0 < h1 ? h0 : h1, m23 = h2 < h3 ? h2 : h3;
                unsigned long long m = m01 < m23 ? m01 : m23;
                if (m == h0) p0++;
                else if (m == h1) p1++;
                else if (m == h2) p2++;
                else p3++;
                float k1 = WS_INF;
                long long k2 = WS_NOID;
                if (m != ~0ull) {
                    k1 = unordered_f32((uint32_t)(m >> 32));
                    uint32_t r = (uint32_t)m;
                    if (!L2) r = ~r;
                    const long long id = ids[row0 + r];
                    k2 = L2 ? id : -id;
                }
                part_k1[e * k + j] = k1;
                part_k2[e * k + j] = k2;
            }
        }
    } else {
#pragma unroll
        for (int qq = 0; qq < NQW; qq++) {
            const int q = w * 16 + qq;
            if (q < nQ && lane < k) {
                const int64_t e = ent_s[q];
                part_k1[e * k + lane] = qd[qq];
                part_k2[e * k + lane] = qi[qq];
            }
        }
    }
}

template <int KQ>
static void launch_scan(bool l2, int64_t grid, hipStream_t s, const float* x, int ldx,
                        const float* codes, int ldc, const int64_t* ids, const uint32_t* list_off,
                        const uint32_t* list_len, int nlist, int dp, int d, int nprobe, int k,
                        IVFBuckets b, float* pk1, long long* pk2) {
    if (l2)
        k_ivf_flat_scan<true, KQ><<<dim3((unsigned)grid), dim3(256), 0, s>>>(
                x, ldx, codes, ldc, ids, list_off, list_len, nlist, dp, d, nprobe, k, b.bucket_off,
                b.item_off, b.entries, b.lim, b.sel, pk1, pk2);
    else
        k_ivf_flat_scan<false, KQ><<<dim3((unsigned)grid), dim3(256), 0, s>>>(
                x, ldx, codes, ldc, ids, list_off, list_len, nlist, dp, d, nprobe, k, b.bucket_off,
                b.item_off, b.entries, b.lim, b.sel, pk1, pk2);
}

void ivf_flat_scan(const float* x, int ldx, const float* codes, int ldc, const int64_t* ids,
                   const uint32_t* list_off, const uint32_t* list_len, int nlist, int dp, int d,
                   int64_t n, int nprobe, int k, int metric_l2, IVFBuckets b, int64_t max_items,
                   float* part_k1, long long* part_k2, hipStream_t s) {
    if (n <= 0) return;
    FAISS_THROW_IF_NOT_MSG(k >= 1 && k <= kMaxK, "k must be in [1, 64] on this path");
    FAISS_THROW_IF_NOT(ldx % 4 == 0 && ldc % 4 == 0 && dp % 4 == 0);
    FAISS_THROW_IF_NOT(max_items < (1ll << 31));
    const bool l2 = metric_l2 != 0;
    max_items = (int64_t)roundup((size_t)max_items, 32);  // XCD remap needs a multiple of 32
    if (k <= 10)
        launch_scan<10>(l2, max_items, s, x, ldx, codes, ldc, ids, list_off, list_len, nlist, dp,
                        d, nprobe, k, b, part_k1, part_k2);
    else if (k <= 16)
        launch_scan<16>(l2, max_items, s, x, ldx, codes, ldc, ids, list_off, list_len, nlist, dp,
                        d, nprobe, k, b, part_k1, part_k2);
    else
        launch_scan<0>(l2, max_items, s, x, ldx, codes, ldc, ids, list_off, list_len, nlist, dp,
                       d, nprobe, k, b, part_k1, part_k2);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- merge
// Per query: lexicographic top-k of the nprobe per-list partial top-k.  A
// boundary tie (the (k+1)-th merged key, or the last key of a full per-list
// partial, equal to the k-th value) flags the query for the exact re-scan.
__global__ __launch_bounds__(256) void k_ivf_merge(const float* __restrict__ part_k1,
                                                   const long long* __restrict__ part_k2,
                                                   const int32_t* __restrict__ assign,
                                                   const uint32_t* __restrict__ list_len,
                                                   int64_t n, int nprobe, int nlist, int k,
                                                   int metric_l2, float* __restrict__ D,
                                                   int64_t* __restrict__ I,
                                                   uint32_t* __restrict__ flags) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= n) return;
    const int K1 = k < 64 ? k + 1 : 64;
    float qd = WS_INF;
    long long qi = WS_NOID;
    float thr_d = WS_INF;
    long long thr_i = WS_NOID;
    const int total = nprobe * k;
    for (int c = 0; c < total; c += 64) {
        int e = c + lane;
        float k1 = WS_INF;
        long long k2 = WS_NOID;
        if (e < total) {
            int r = e / k;
            int lst = assign[q * nprobe + r];
            if (lst >= 0 && lst < nlist && list_len[lst] > 0) {
                int64_t p = (q * nprobe) * (int64_t)k + e;
                k1 = part_k1[p];
                k2 = part_k2[p];
            }
        }
        wave_offer(qd, qi, k1, k2, thr_d, thr_i, K1, lane);
    }
    const float v = __shfl(qd, k - 1);
    const long long vi = shfl_ll(qi, k - 1);
    bool amb = false;
    if (vi != WS_NOID) {
        int cnt = 0;
        bool tail = false;
        for (int c = 0; c < total; c += 64) {
            int e = c + lane;
            bool eq = false;
            if (e < total) {
                int lst = assign[q * nprobe + e / k];
                if (lst >= 0 && lst < nlist && list_len[lst] > 0) {
                    int64_t p = (q * nprobe) * (int64_t)k + e;
                    eq = part_k2[p] != WS_NOID && part_k1[p] == v;
                    if (eq && e % k == k - 1) tail = true;
                }
            }
            cnt += __popcll(__ballot(eq));
        }
        amb = __ballot(tail) != 0ull || cnt > __popcll(__ballot(lane < k && qd == v));
    }
    if (lane < k) {
        float dis;
        long long id;
        from_key(metric_l2, qd, qi, dis, id);
        D[q * k + lane] = dis;
        I[q * k + lane] = id;
    }
    if (lane == 0) flags[q] = amb ? 1u : 0u;
}

void ivf_merge(const float* part_k1, const long long* part_k2, const int32_t* assign,
               const uint32_t* list_len, int nlist, int64_t n, int nprobe, int k, int metric_l2,
               float* D, int64_t* I, uint32_t* flags, hipStream_t s) {
    if (n <= 0) return;
    k_ivf_merge<<<dim3((unsigned)cdiv(n, 4)), dim3(256), 0, s>>>(
            part_k1, part_k2, assign, list_len, n, nprobe, nlist, k, metric_l2, D, I, flags);
    HIP_LAUNCH_CHECK();
}

}  // namespace kern
}  // namespace faiss_amd
