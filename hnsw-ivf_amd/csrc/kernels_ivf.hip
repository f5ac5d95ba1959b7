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

#include <cstdlib>
#include <cstring>

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
constexpr int BC_MAXL = 16384;       // lists per range in 64 KB of LDS
constexpr int BC_MAXL_BIG = 32768;   // 128 KB (a work group may hold 160 KB on gfx950)
template <int BC_PER>
__global__ __launch_bounds__(1024) void k_bucket_count_lds(const int32_t* __restrict__ assign,
                                                           int64_t total,
                                                           const uint32_t* __restrict__ list_len,
                                                           int nlist, uint32_t* __restrict__ counts,
                                                           uint32_t* __restrict__ pos, int maxl) {
    extern __shared__ uint32_t hist[];  // [min(nlist, maxl)]
    const int t = threadIdx.x;
    // lists [lbase, lbase + nl) of this block row (nlist > maxl: one row of
    // blocks per range, each reading every entry)
    const int lbase = (int)blockIdx.y * maxl;
    const int nl = min(maxl, nlist - lbase);
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
// -> item_off; per work item its list when asked.  E consecutive counts per
// thread (E = nlist / 1024 rounded up to a power of two, at most 64): every
// count of a chunk of 1024 E lists is loaded at once (one round trip — c5's
// 65536 lists in one chunk instead of sixteen), thread sums, shuffle scan per
// wave, 16 wave totals through LDS; a running carry between chunks.
template <int E>
__global__ __launch_bounds__(1024) void k_bucket_scan(const uint32_t* counts,
                                                      int nlist, int QT,
                                                      uint32_t* __restrict__ bucket_off,
                                                      uint32_t* __restrict__ item_off,
                                                      uint32_t* __restrict__ item_list,
                                                      uint32_t* zero_next,
                                                      uint32_t* __restrict__ item_ctr,
                                                      const uint32_t* __restrict__ perm) {
    __shared__ uint32_t wb[16], wi[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    constexpr int CH = 1024 * E;
    static_assert(E % 4 == 0, "E counts per thread as uint4 groups");
    // items of a bucket of c entries: ceil(c / QT), a shift when QT is a power
    // of two (every caller's), else a division
    const int qs = (QT & (QT - 1)) == 0 ? __builtin_ctz((unsigned)QT) : -1;
    auto nitems = [&](uint32_t c) -> uint32_t {
        return qs >= 0 ? (c + (uint32_t)QT - 1u) >> qs : (c + (uint32_t)QT - 1u) / (uint32_t)QT;
    };
    // prefix of the thread sums (v[] per thread) over the work group: returns
    // this thread's exclusive prefix and the chunk total
    auto block_scan = [&](uint32_t sb, uint32_t si, uint32_t& pb, uint32_t& pi, uint32_t& tb,
                          uint32_t& ti) {
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
        pb = 0;
        pi = 0;
        tb = 0;
        ti = 0;
#pragma unroll
        for (int v = 0; v < 16; v++) {
            pb += v < w ? wb[v] : 0u;
            pi += v < w ? wi[v] : 0u;
            tb += wb[v];
            ti += wi[v];
        }
        __syncthreads();  // wb / wi are rewritten by the next chunk
        pb += ib - sb;
        pi += ii - si;
    };
    uint32_t carry_b = 0, carry_i = 0;
    for (int c0 = 0; c0 < nlist; c0 += CH) {
        const int l0 = c0 + E * t;
        uint32_t c[E];
        uint32_t sb = 0, si = 0;
        const bool full = l0 + E <= nlist;  // this thread's E lists exist (uint4 access)
        if (full) {
#pragma unroll
            for (int v = 0; v < E / 4; v++) {
                const uint4 c4 = *(const uint4*)(counts + l0 + 4 * v);
                c[4 * v] = c4.x;
                c[4 * v + 1] = c4.y;
                c[4 * v + 2] = c4.z;
                c[4 * v + 3] = c4.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < E; j++) c[j] = l0 + j < nlist ? counts[l0 + j] : 0u;
        }
        // zero_next == counts: each count is cleared once read (the fill
        // takes the bucket sizes from bucket_off)
        if (zero_next) {
            if (full) {
#pragma unroll
                for (int v = 0; v < E / 4; v++)
                    *(uint4*)(zero_next + l0 + 4 * v) = make_uint4(0u, 0u, 0u, 0u);
            } else {
                for (int j = 0; j < E && l0 + j < nlist; j++) zero_next[l0 + j] = 0u;
            }
        }
#pragma unroll
        for (int j = 0; j < E; j++) {
            sb += c[j];
            si += nitems(c[j]);
        }
        uint32_t pb, pi, tb, ti;
        block_scan(sb, si, pb, pi, tb, ti);
        uint32_t rb = carry_b + pb, ri = carry_i + pi;  // exclusive prefix of this thread
        uint32_t ob[E], oi[E];
#pragma unroll
        for (int j = 0; j < E; j++) {
            ob[j] = rb;
            oi[j] = ri;
            rb += c[j];
            ri += nitems(c[j]);
        }
        if (full) {
#pragma unroll
            for (int v = 0; v < E / 4; v++) {
                *(uint4*)(bucket_off + l0 + 4 * v) =
                        make_uint4(ob[4 * v], ob[4 * v + 1], ob[4 * v + 2], ob[4 * v + 3]);
                *(uint4*)(item_off + l0 + 4 * v) =
                        make_uint4(oi[4 * v], oi[4 * v + 1], oi[4 * v + 2], oi[4 * v + 3]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < E; j++) {
                if (l0 + j < nlist) {
                    bucket_off[l0 + j] = ob[j];
                    item_off[l0 + j] = oi[j];
                }
            }
        }
        if (item_list) {  // rare (item_list users); a second walk keeps the first lean
            ri = carry_i + pi;
            for (int j = 0; j < E && l0 + j < nlist; j++) {
                const uint32_t nj = nitems(c[j]);
                for (uint32_t i = 0; i < nj; i++) item_list[ri + i] = (uint32_t)(l0 + j);
                ri += nj;
            }
        }
        carry_b += tb;
        carry_i += ti;
    }
    if (t == 0) {
        bucket_off[nlist] = carry_b;
        item_off[nlist] = carry_i;
        if (item_ctr) *item_ctr = 0u;  // the persistent filter's work counter
    }
    if (!perm) return;
    // items renumbered in perm order (bucket sizes from bucket_off: the counts
    // are cleared); the bucket_off stores above are this work group's own
    __threadfence_block();
    __syncthreads();
    carry_i = 0;
    for (int c0 = 0; c0 < nlist; c0 += CH) {
        const int i0 = c0 + E * t;
        int ls[E];
        uint32_t n[E], si = 0;
        if (i0 + E <= nlist) {
#pragma unroll
            for (int v = 0; v < E / 4; v++) {
                const uint4 p4 = *(const uint4*)(perm + i0 + 4 * v);
                ls[4 * v] = (int)p4.x;
                ls[4 * v + 1] = (int)p4.y;
                ls[4 * v + 2] = (int)p4.z;
                ls[4 * v + 3] = (int)p4.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < E; j++) ls[j] = i0 + j < nlist ? (int)perm[i0 + j] : -1;
        }
#pragma unroll
        for (int j = 0; j < E; j++) {
            n[j] = ls[j] >= 0 ? nitems(bucket_off[ls[j] + 1] - bucket_off[ls[j]]) : 0u;
            si += n[j];
        }
        uint32_t pb, pi, tb, ti;
        block_scan(0u, si, pb, pi, tb, ti);
        uint32_t ri = carry_i + pi;
#pragma unroll
        for (int j = 0; j < E; j++) {
            if (ls[j] >= 0) item_off[ls[j]] = ri;
            ri += n[j];
        }
        if (item_list) {  // rare (item_list users); a second walk keeps the first lean
            ri = carry_i + pi;
            for (int j = 0; j < E; j++) {
                for (uint32_t i = 0; i < n[j]; i++) item_list[ri + i] = (uint32_t)ls[j];
                ri += n[j];
            }
        }
        carry_i += ti;
    }
}

// The scan of k_bucket_scan over many work groups (nlist > 8192; c5: 65536
// lists, where the single work group's chunks and its gathers of the
// permuted counts took 133 us).  Part: each group scans its 4096 E-runs of
// counts (bucket sizes, and work items in list order or, with perm, in perm
// order — the counts gathered through perm) into local exclusive prefixes
// and writes its three totals; fix: each group adds the totals of the groups
// before it, clears its counts (counts_next) and the last one writes the
// ends and the work counter.
template <int E>
__global__ __launch_bounds__(1024) void k_bucket_scan_part(const uint32_t* __restrict__ counts,
                                                           int nlist, int QT,
                                                           uint32_t* __restrict__ bucket_off,
                                                           uint32_t* __restrict__ item_off,
                                                           const uint32_t* __restrict__ perm,
                                                           uint32_t* __restrict__ tot) {
    __shared__ uint32_t wb[16], wi[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int qs = (QT & (QT - 1)) == 0 ? __builtin_ctz((unsigned)QT) : -1;
    auto nitems = [&](uint32_t c) -> uint32_t {
        return qs >= 0 ? (c + (uint32_t)QT - 1u) >> qs : (c + (uint32_t)QT - 1u) / (uint32_t)QT;
    };
    auto block_scan = [&](uint32_t sb, uint32_t si, uint32_t& pb, uint32_t& pi, uint32_t& tb,
                          uint32_t& ti) {
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
        pb = pi = tb = ti = 0u;
#pragma unroll
        for (int v = 0; v < 16; v++) {
            pb += v < w ? wb[v] : 0u;
            pi += v < w ? wi[v] : 0u;
            tb += wb[v];
            ti += wi[v];
        }
        __syncthreads();
        pb += ib - sb;
        pi += ii - si;
    };
    const int l0 = (int)blockIdx.x * 1024 * E + E * t;
    uint32_t c[E], sb = 0u, si = 0u;
#pragma unroll
    for (int j = 0; j < E; j++) {
        c[j] = l0 + j < nlist ? counts[l0 + j] : 0u;
        sb += c[j];
        si += nitems(c[j]);
    }
    uint32_t pb, pi, tb, ti;
    block_scan(sb, si, pb, pi, tb, ti);
#pragma unroll
    for (int j = 0; j < E; j++) {
        if (l0 + j < nlist) {
            bucket_off[l0 + j] = pb;
            if (!perm) item_off[l0 + j] = pi;
        }
        pb += c[j];
        pi += nitems(c[j]);
    }
    uint32_t tp = 0u;
    if (perm) {
        int ls[E];
        uint32_t nj[E], sp = 0u;
#pragma unroll
        for (int j = 0; j < E; j++) {
            ls[j] = l0 + j < nlist ? (int)perm[l0 + j] : -1;
            nj[j] = ls[j] >= 0 ? nitems(counts[ls[j]]) : 0u;
            sp += nj[j];
        }
        uint32_t pp, dummy, tdummy;
        block_scan(sp, 0u, pp, dummy, tp, tdummy);
#pragma unroll
        for (int j = 0; j < E; j++) {
            if (ls[j] >= 0) item_off[ls[j]] = pp;
            pp += nj[j];
        }
    }
    if (t == 0) {
        tot[3 * blockIdx.x] = tb;
        tot[3 * blockIdx.x + 1] = ti;
        tot[3 * blockIdx.x + 2] = tp;
    }
}
template <int E>
__global__ __launch_bounds__(1024) void k_bucket_scan_fix(int nlist, uint32_t* __restrict__ bucket_off,
                                                          uint32_t* __restrict__ item_off,
                                                          const uint32_t* __restrict__ perm,
                                                          const uint32_t* __restrict__ tot,
                                                          uint32_t* __restrict__ zero_next,
                                                          uint32_t* __restrict__ item_ctr) {
    const int t = threadIdx.x, b = (int)blockIdx.x;
    uint32_t ob = 0u, oi = 0u;
    for (int v = 0; v < b; v++) {
        ob += tot[3 * v];
        oi += tot[3 * v + (perm ? 2 : 1)];
    }
    const int l0 = b * 1024 * E + E * t;
#pragma unroll
    for (int j = 0; j < E; j++) {
        if (l0 + j < nlist) {
            bucket_off[l0 + j] += ob;
            item_off[perm ? (int)perm[l0 + j] : l0 + j] += oi;
            if (zero_next) zero_next[l0 + j] = 0u;
        }
    }
    if (b == (int)gridDim.x - 1 && t == 0) {
        bucket_off[nlist] = ob + tot[3 * b];
        item_off[nlist] = oi + tot[3 * b + (perm ? 2 : 1)];
        if (item_ctr) *item_ctr = 0u;
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
                dsc.nq = min((uint32_t)QT, bucket_off[l + 1] - bucket_off[l] - p);
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

__global__ void k_stamp(unsigned long long* out) { *out = __builtin_amdgcn_s_memrealtime(); }
void device_stamp(unsigned long long* out, hipStream_t s) {
    k_stamp<<<dim3(1), dim3(1), 0, s>>>(out);
    HIP_LAUNCH_CHECK();
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
    k_ivf_visit_stats<<<kgrid(grid, 256), dim3(256), 0, s>>>(assign, total, list_len, nlist,
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
    k_probe_limits<<<kgrid(cdiv(n, 256), 256), dim3(256), 0, s>>>(
            assign, n, nprobe, list_len, nlist, max_codes, assign_out, lim);
    HIP_LAUNCH_CHECK();
}

void ivf_bucket(const int32_t* assign, int64_t n, int nprobe, const uint32_t* list_len,
                const uint32_t* list_off, int nlist, int QT, IVFBuckets b, hipStream_t s) {
    int64_t total = n * nprobe;
    FAISS_THROW_IF_NOT_MSG(total < (1ll << 32), "n * nprobe must fit in 32 bits");
    if (!b.counts_next) HIP_CHECK(hipMemsetAsync(b.counts, 0, sizeof(uint32_t) * nlist, s));
    if (total > 0) {
        // entries per thread: enough work groups to spread the histogram
        // merge's global atomics over the chip (FAISS_AMD_BC_PER: tuning)
        // (c2, 4096 lists: 4 -> 7.6 us, 16 -> 12.9 us; c5, 65536 lists in 4
        // LDS ranges that each read every entry: 16 -> 162 us, 4 -> 233 us,
        // one global atomic per entry 254 us)
        const char* pe = getenv("FAISS_AMD_BC_PER");
        const int per = pe ? atoi(pe) : nlist > BC_MAXL ? 16 : 4;
        {
        // beyond 16384 lists: 32768-list ranges in 128 KB of LDS (half the
        // passes over the entries; FAISS_AMD_BC_BIG=0: 64 KB ranges)
        const char* be = getenv("FAISS_AMD_BC_BIG");
        const int maxl = nlist > BC_MAXL && !(be && !strcmp(be, "0")) ? BC_MAXL_BIG : BC_MAXL;
        const int nr2 = (int)cdiv(nlist, maxl);
        const size_t lds = sizeof(uint32_t) * std::min(nlist, maxl);
#define BCL(P)                                                                              \
    do {                                                                                    \
        if (lds > 65536)                                                                    \
            HIP_CHECK(hipFuncSetAttribute((const void*)k_bucket_count_lds<P>,               \
                                          hipFuncAttributeMaxDynamicSharedMemorySize,       \
                                          (int)lds));                                       \
        k_bucket_count_lds<P><<<dim3((unsigned)cdiv(total, 1024 * P), (unsigned)nr2),       \
                                dim3(1024), lds, s>>>(assign, total, list_len, nlist,       \
                                                      b.counts, b.cursor, maxl);            \
    } while (0)
        if (per >= 16) BCL(16);
        else if (per >= 8) BCL(8);
        else if (per >= 4) BCL(4);
        else if (per >= 2) BCL(2);
        else BCL(1);
#undef BCL
        HIP_LAUNCH_CHECK();
        }
    }
    // beyond 8192 lists (and up to 64 groups of 4096): the scan over many
    // work groups, its block totals after the work counter (b.scan_tmp);
    // FAISS_AMD_SCAN_PAR=0: the single-group scan
    const char* pp = getenv("FAISS_AMD_SCAN_PAR");
    const int nbs = (int)cdiv(nlist, 4096);
    if (nlist > 8192 && nbs <= 64 && b.scan_tmp && !b.item_list && !(pp && !strcmp(pp, "0"))) {
        k_bucket_scan_part<4><<<dim3((unsigned)nbs), dim3(1024), 0, s>>>(
                b.counts, nlist, QT, b.bucket_off, b.item_off, b.perm, b.scan_tmp);
        HIP_LAUNCH_CHECK();
        k_bucket_scan_fix<4><<<dim3((unsigned)nbs), dim3(1024), 0, s>>>(
                nlist, b.bucket_off, b.item_off, b.perm, b.scan_tmp, b.counts_next, b.item_ctr);
        HIP_LAUNCH_CHECK();
    } else {
#define BSCAN(E)                                                                            \
    k_bucket_scan<E><<<dim3(1), dim3(1024), 0, s>>>(b.counts, nlist, QT, b.bucket_off,         \
                                                    b.item_off, b.item_list, b.counts_next,    \
                                                    b.item_ctr, b.perm)
    // counts per thread: 4 up to 4096 lists, else 16 (FAISS_AMD_SCAN_E: tuning)
    const char* se = getenv("FAISS_AMD_SCAN_E");
    const int E = se ? atoi(se) : nlist <= 4096 ? 4 : 16;
    if (E >= 16) BSCAN(16);
    else if (E >= 8) BSCAN(8);
    else BSCAN(4);
#undef BSCAN
    HIP_LAUNCH_CHECK();
    }
    if (total > 0) {
        k_bucket_fill<<<kgrid(cdiv(total, 256), 256), dim3(256), 0, s>>>(
                assign, total, list_len, nlist, QT, b.bucket_off, b.item_off, b.cursor, b.entries,
                b.item_entries, b.item_desc, b.counts, list_off, b.mark_keys, b.mark_recs,
                b.mark_ke);
        HIP_LAUNCH_CHECK();
    }
}


}  // namespace kern
}  // namespace faiss_amd
