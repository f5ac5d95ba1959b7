// kernels.h — host-side launchers of the gfx950 kernels.
//
// Data layout conventions (HBM):
//  * vectors are row-major f32 with a leading dimension `ld` that is a
//    multiple of 4 floats (16 B) and zero padded beyond d, so every row is
//    16-B aligned and dims can be streamed as float4.
//  * coarse assignments are int32 list numbers ([n][nprobe], -1 = none).
//  * inverted lists live in one arena: list l occupies rows
//    [list_off[l], list_off[l] + list_len[l]) of `codes` (row = code_size
//    bytes) and of `ids` (int64).  list_off is aligned to 16 rows.
#pragma once

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>

#include "common.h"

namespace faiss_amd {
namespace kern {

constexpr int kMaxK = 64;  // largest k / nprobe served by the wave queues
// largest nprobe of the list-centric MFMA filters + certified re-rank (one
// probe record per lane up to 64, k_ivf_rerank_wide's 64-probe chunks beyond)
constexpr int kMaxNprobeFilter = 2048;
constexpr int kMaxKExact = 2048;  // largest k of the general exact path (faiss GPU's limit,
                                  // faiss/gpu/utils/DeviceDefs.cuh:28)

// out[i] = sum_j x[i*ld + j]^2, j < d
void row_norms(const float* x, int64_t n, int d, int ld, float* out, hipStream_t s);

// Distance tile on fp32 MFMA (v_mfma_f32_32x32x2_f32):
//   L2: D[i][j] = max(0, fma(-2, <x_i, y_j>, xn[i] + yn[j]))
//   IP: D[i][j] = <x_i, y_j>
// reference: faiss/utils/distances.cpp:259-342 (exhaustive_L2sqr_blas)
void pairwise_distances(const float* x, int64_t nx, int ldx, const float* xn,
                        const float* y, int64_t ny, int ldy, const float* yn, int dp,
                        int metric_l2, float* D, int64_t ldD, hipStream_t s);

// Direct per-pair distances in the reference order (faiss' path for query
// blocks below distance_compute_blas_threshold = 20)
void direct_distances(const float* x, int64_t nx, int ldx, const float* y, int64_t ny, int ldy,
                      int d, int metric_l2, float* D, int64_t ldD, hipStream_t s);

// Coarse top-k on bf16x3 MFMA + certified exact re-rank (kernels_coarse.hip);
// identical results to pairwise_distances + select_rows for blocks of >= 20
// queries.  plan.ok == false: not eligible (fall back to the f32 tile path).
struct CoarsePlan {
    bool ok = false;
    int nsplit = 0, split_len = 0, kt = 0, obits = 0, entries = 0;  // entries per query
};
CoarsePlan coarse_bf3_plan(int64_t n, int nlist, int d, int k);
void coarse_bf3_knn(const CoarsePlan& p, const float* x, int64_t n, int ldx, const float* xnorm,
                    const float* cent, int ldc, const void* cbf, const float* cnorm,
                    const float* cnmax, int nlist, int d, int k, int metric_l2, uint32_t* keys,
                    float* pbs, float* D, int32_t* I32, int64_t* I64, hipStream_t s,
                    const void* cst = nullptr, const void* qimg = nullptr,
                    KernelTimes* kt = nullptr,
                    int fold = 0);  // cst is the fold image (L2)
// Query preparation for the MFMA filters (one launch): the reference-order
// norms ref_norms[i] = fvec_norm_L2sqr(x_i) (skipped when null) and the query
// image of bf3.h load_query_image — qimg [n][64 NS] bytes (NS = bf3_db(d)/16)
// and qxn [n] (skipped when null).  d <= BDM.
void query_prep(const float* x, int64_t n, int ldx, int d, float* ref_norms, void* qimg,
                float* qxn, hipStream_t s);
inline size_t query_image_bytes(int64_t n, int d) {
    return (size_t)std::max<int64_t>(n, 1) * 4 * ((d + 31) / 32 * 32);
}
// the streamed coarse filter's image of the centroids: per row bf16 hi | lo
// (bf3_db(d) dims each) | a 16-byte tail, padded to 64 rows.  fold = 0: the
// tail is the fp32 norm (+inf for padding rows) + 12 zero bytes; fold = 1
// (L2): the bias A-fragment {-|c|^2/2 in three bf16 parts, 1, 1, 1, 0, 0}
// (padding rows -inf, 0, 0, 1, 1, 1, 0, 0), as split_bf16_stream's
void coarse_stream_image(const float* codes, int64_t rows, int d, int ldc, const float* norms,
                         void* out, hipStream_t s, int fold = 0);
size_t coarse_stream_image_bytes(int64_t rows, int d);
void array_max(const float* a, int64_t n, float* out, hipStream_t s);

// k smallest (L2) / largest (IP) per row of D, ties by column index,
// reference faiss/impl/ResultHandler.h:187-287 (HeapBlockResultHandler).
// Outputs are sorted; missing slots are (+-FLT_MAX, -1).  Either of out_i32 /
// out_i64 may be null.  `col0` is added to output column indices.
void select_rows(const float* D, int64_t nx, int64_t ny, int64_t ldD, int k, int metric_l2,
                 int64_t col0, float* out_d, int32_t* out_i32, int64_t* out_i64,
                 int64_t ldo, hipStream_t s);

// Inner product only: re-select rows whose k-th value ties with an unselected
// column using the reference heap's arrival-order rule (col0 == 0 tables).
void select_fix_ip(const float* D, int64_t nx, int64_t ny, int64_t ldD, int k, float* out_d,
                   int32_t* out_i32, int64_t* out_i64, int64_t ldo, hipStream_t s);

// Merge `nin` sorted candidate tables per row: cand_d/cand_i [n][nin*kin]
// (already final (dis,label) form, label -1 = empty) -> [n][k].
void merge_rows(const float* cand_d, const int64_t* cand_i, int64_t n, int nin_x_kin, int k,
                int metric_l2, float* out_d, int64_t* out_i, hipStream_t s);

// merge_knn_results for any k (kernels_exact.hip), inputs [nshard][n][kin]
void merge_rows_general(const float* cand_d, const int64_t* cand_i, int64_t n, int nshard,
                        int kin, int k, int metric_l2, float* out_d, int64_t* out_i,
                        hipStream_t s);

// labels >= 0 get += offset (faiss/IndexShardsIVF.cpp translate_labels)
void translate_labels(int64_t* labels, int64_t n, int64_t offset, hipStream_t s);

// ---------------- IVF list-centric batching ----------------
// Work item = (list, chunk of <= QT queries probing it).
// Per (query, probe) record of the IVF-Flat MFMA filter, read by the re-rank:
// per thread stream (4 per (query, list)) a lower bound of every candidate it
// dropped (+inf: none dropped / empty probe), the list's largest
// certification margin, and the list's arena geometry.
struct alignas(16) ProbeRec {
    float pb[4];
    float mmax;
    uint32_t off;
    uint32_t len;
    uint32_t pad;
};

// work item of the list-centric IVF scans: list, queries in the item, list
// length and arena offset
struct alignas(16) ItemDesc {
    uint32_t l, nq, len, off;
};

struct IVFBuckets {
    uint32_t* counts;      // [nlist]
    uint32_t* bucket_off;  // [nlist + 1]
    uint32_t* item_off;    // [nlist + 1]
    uint32_t* cursor;      // [n * nprobe]: slot of each entry in its bucket
    uint32_t* entries;     // [n * nprobe], entry = q * nprobe + rank
    uint32_t* item_list = nullptr;  // [max_items]: list of each work item
    uint32_t* item_ctr = nullptr;   // [1]: zeroed by the scan (persistent filter's counter)
    uint32_t* scan_tmp = nullptr;   // [3 * 64]: the many-group scan's block totals
    // optional: lists by decreasing length; work items are numbered in this
    // order (longest first: the filters' launch order, so the long items do
    // not start last and set the kernel's tail)
    const uint32_t* perm = nullptr;
    // optional (MFMA filter path): per work item its descriptor and its
    // entries at a fixed stride of QT (so a work item's first loads do not
    // depend on each other)
    ItemDesc* item_desc = nullptr;         // [max_items]
    uint32_t* item_entries = nullptr;      // [max_items * QT]
    // optional (MFMA filter path): entries whose list is invalid or empty get
    // empty partials (part ~0, pub / pbound +inf), so the re-rank reads every
    // entry without consulting the assignment
    uint32_t* mark_keys = nullptr;
    ProbeRec* mark_recs = nullptr;
    int mark_ke = 0;
    // optional: the count array the scan clears after reading it (== counts:
    // self-cleaning).  When set, `counts` is already zero (the previous
    // call's scan cleared it), so no memset is launched.
    uint32_t* counts_next = nullptr;
    // optional (max_codes): rows of each entry's list that are scanned (a
    // prefix; probe_limits), nullptr = whole lists
    const uint32_t* lim = nullptr;
    // optional (IDSelector): arena-row membership mask, nullptr = every row
    const uint8_t* sel = nullptr;
};
// max_codes (faiss/IndexIVF.cpp:595-631, scan_one_list :546-550): per query,
// probes in coarse order; the probe that reaches max_codes is cut to the rows
// still allowed and the later ones are dropped (assign_out -1).  lim[e] = rows
// of entry e scanned (0 for dropped / empty / invalid probes).
void probe_limits(const int32_t* assign, int64_t n, int nprobe, const uint32_t* list_len,
                  int nlist, int64_t max_codes, int32_t* assign_out, uint32_t* lim,
                  hipStream_t s);
void ivf_bucket(const int32_t* assign, int64_t n, int nprobe, const uint32_t* list_len,
                const uint32_t* list_off, int nlist, int QT, IVFBuckets b, hipStream_t s);
// the certified exact re-rank of the IVF-Flat filter's keys / probe records
// (kernels_ivf_rerank.hip; one wave per query, probes in chunks of 64 past
// nprobe 64); ivf_flat_scan_mfma calls it after the filter
void ivf_flat_rerank(const uint32_t* keys, const ProbeRec* recs, const float* x, int ldx,
                     const float* codes, int ldc, const int64_t* ids, int d, int64_t n,
                     int nprobe, int KE, int obits, int k, int metric_l2, const uint8_t* sel,
                     uint32_t* stats, float* D, int64_t* I, KernelTimes* kt, hipStream_t s,
                     unsigned long long* qdone, int fold);
// IVF-PQ list-centric MFMA filter + exact re-rank (kernels_pq_mfma.hip)
struct PQArgs {
    const float* pq_cent = nullptr;  // [M][256][dsub] fp32
    const float* cent = nullptr;     // coarse centroids [nlist][ldcent]
    int ldcent = 0;
    const float* cdis = nullptr;     // coarse distances [n][nprobe] (table 1 dis0)
    const uint8_t* codes = nullptr;  // arena codes, cs bytes per row
    int cs = 0;
    int M = 0;
    int table1 = 0;  // use_precomputed_table == 1 (else table 0, by residual)
};
struct RerankSel {  // IDSelector mask of the arena rows (nullptr = all)
    const uint8_t* sel = nullptr;
};
bool ivfpq_mfma_eligible(int d, int M, int k, int nprobe);
double ivfpq_mfma_coef(int d, int M);
// bf16 decode table ([M][256][dsub] bf16) and per-row |y_R|, |y_R - bf16(y_R)|
void pq_decode_prep(const float* pq_cent, int M, int dsub, const uint8_t* codes, int cs,
                    int64_t rows, void* dec, float* rnorm, float* rres, hipStream_t s);
void ivfpq_filter(const float* x, int ldx, int d, int M, const void* dec, const uint8_t* codes,
                  const float* terms, const float* cdis, const float* cnorm, const float* lrmax,
                  const float* lRmax, int nlist, int64_t n, int nprobe, int k, int obits,
                  const IVFBuckets& b, int64_t max_items, uint32_t* keys, ProbeRec* recs,
                  int* kt_out, hipStream_t s,
                  const void* qimg = nullptr, const float* qxn = nullptr);
// |x_q - c_l|^2 in fvec_L2sqr order for the (query, probe) pairs of assign
// (0 where l < 0): IVF-PQ table-0 filters key on the true coarse distance
void pair_l2(const float* x, int ldx, const float* cent, int ldc, int d, const int32_t* assign,
             int64_t n, int np, float* out, hipStream_t s);
// fold: the keys are folded (ivfpq_stream_filter)
void ivfpq_rerank(const uint32_t* keys, const ProbeRec* recs, const float* x, int ldx, int d,
                  const int64_t* ids, const PQArgs& pa, int dsub, int64_t n, int nprobe, int KT,
                  int obits, int k, const uint8_t* sel, float* D, int64_t* I, uint32_t* stats,
                  hipStream_t s, unsigned long long* qdone = nullptr, int fold = 0);
// PQ stream image (kernels_ivf_mfma.hip k_pq_stream_image): per arena row
// 2 DB + 16 bytes, DB = bf3_db_host(d): bf16 of the decoded residual, then
// the folded bias fragment of -term / 2
void pq_stream_image(const uint8_t* codes, int cs, int64_t rows, int d, int dsub,
                     const float* pq_cent, const float* terms, const uint32_t* row_list, int DB,
                     void* out, hipStream_t s);
bool ivfpq_stream_eligible(int d, int M, int k, int nprobe);
double ivfpq_fold_coef(int d, int M);
// the IVF-Flat streamed filter over the PQ stream image: keys + probe records
// in the k_ivfpq_filter_w format (folded keys; the re-rank takes fold = 1)
void ivfpq_stream_filter(const float* x, int ldx, int d, int M, const void* pcbs,
                         const float* cdis, const float* cnorm, const float* lrmax,
                         const float* lRmax, int nlist, int64_t n, int nprobe, int k, int obits,
                         const IVFBuckets& b, int64_t max_items, uint32_t* keys, ProbeRec* recs,
                         int* kt_out, hipStream_t s, const void* qimg, const float* qxn);
// the device clock (s_memrealtime) into *out, in stream order
void device_stamp(unsigned long long* out, hipStream_t s);

// ---------------- general exact path (kernels_exact.hip) ----------------
// IVF-PQ tables of the exact scan (QueryTables semantics)
struct ExactPQ {
    int M = 0, dsub = 0;
    int by_residual = 1;
    int table1 = 0;                  // use_precomputed_table == 1 (L2 by residual)
    const float* pq_cent = nullptr;  // [M][256][dsub]
    const float* cent = nullptr;     // coarse centroids [nlist][ldcent] fp32
    int ldcent = 0;
    const uint8_t* codes = nullptr;  // arena codes
    int cs = 0;                      // code stride (bytes)
};
struct ExactScanArgs {
    unsigned long long* qdone = nullptr;  // per query completion stamps (search_stats)
    const float* x = nullptr;  // [n][ldx] queries of the chunk
    int ldx = 0, d = 0;
    int64_t n = 0;
    int np = 0, k = 0, l2 = 1;
    const int32_t* assign = nullptr;  // [n][np]
    const float* cdis = nullptr;      // [n][np] (PQ table 1: dis0)
    const uint32_t* list_off = nullptr;
    const uint32_t* list_len = nullptr;
    int nlist = 0;
    const uint32_t* lim = nullptr;  // max_codes prefixes (nullptr: whole lists)
    const uint8_t* sel = nullptr;   // IDSelector row mask (nullptr: all)
    const int64_t* ids = nullptr;
    const uint32_t* row_list = nullptr;  // store_pairs: list of each arena row
    int store_pairs = 0;
    const float* codes = nullptr;  // IVF-Flat arena [rows][ldc]
    int ldc = 0;
    ExactPQ pq;  // pq.M > 0: IVF-PQ
};
// candidates per query (cap) and queries per chunk for a 1 GiB scratch
int64_t ivf_exact_chunk(int64_t n, int np, uint32_t max_list_len, int64_t* cap_out);
// eoff [n*np], total [n], keys / rows [n*cap] scratch
void ivf_exact_search(const ExactScanArgs& a, uint32_t* eoff, uint32_t* total, uint32_t* keys,
                      uint32_t* rows, int64_t cap, float* D, int64_t* I, hipStream_t s);
// IVF-PQ range scan of any geometry / metric (same contract as ivfpq_range;
// a.x / a.assign / a.cdis / a.sel / a.ids / a.row_list / a.store_pairs used)
void ivfpq_range_exact(const ExactScanArgs& a, float radius, uint32_t* counts,
                       const uint64_t* offsets, float* outD, int64_t* outI, hipStream_t s);
// exact top-k (reference heap semantics, label = col0 + column) of dense rows;
// k > kMaxKExact runs with global scratch (required then)
template <class OutIdx>
void select_rows_exact(const float* D, int64_t nx, int64_t ny, int64_t ldD, int k, int metric_l2,
                       int64_t col0, float* out_d, OutIdx* out_i, int64_t ldo, hipStream_t s,
                       DeviceBuffer* scratch = nullptr);

// IndexIVFStats counters of a batch (faiss/IndexIVF.cpp:1184-1198):
// stats[0] += non-empty lists visited, stats[1] += codes scanned (device)
void ivf_visit_stats(const int32_t* assign, int64_t total, const uint32_t* list_len, int nlist,
                     const uint32_t* lim, unsigned long long* stats, hipStream_t s);
// list starts (and list extents) in the arena are aligned to this many rows
// (one filter tile), padding rows zero with row_list == ~0
constexpr int ARENA_ALIGN = 64;
// padding rows (row_list == ~0) get +inf in v (the streamed filter's norms)
void pad_rows_inf(float* v, const uint32_t* row_list, int64_t rows, hipStream_t s);
// queries per work item of the IVF-Flat MFMA filter (bf3.h FQ)
constexpr int IVF_FLAT_QT = 128;
// upper bound on the number of work items (grid size without a host sync)
inline int64_t ivf_max_items(int64_t n, int nprobe, int nlist, int QT) {
    return (n * nprobe + QT - 1) / QT + nlist;
}

// bf16x3-MFMA filter + certified exact re-rank (kernels_ivf_mfma.hip);
// results are identical to the general exact scan (ivf_exact_search).
// ivf_mfma_kq = entries kept per (query, list); 0 = not eligible
// (k > 32 or roundup(d, 16) > 128).
// kt_min: at least that many keys per thread stream (2, 4 or 8; 0: by k)
int ivf_mfma_kq(int k, int d, int nprobe = 0, int kt_min = 0);
int ivf_bf3_obits(uint32_t max_list_len);
// padded dim of the bf16 hi/lo images (multiple of 32)
constexpr int BDM_HOST = 128;  // bf3.h BDM: max padded dim of the MFMA paths
inline int bf3_db_host(int d) { return (d + 31) / 32 * 32; }  // ordinal bits of the 32-bit keys
double ivf_bf3_coef(int d);                // margin coefficient
double ivf_bf2_coef(int d);
double ivf_bf2f_coef(int d);  // bf16x2 with the norms folded into the MFMA (fold image)
double ivf_bf3f_coef(int d);  // bf16x3, norms folded (coarse fold image)
// |y - bf16(y)| per row (bf16x2 filter margins)
void row_resnorm_bf16(const float* codes, int64_t rows, int d, int ldc, float* out,
                      hipStream_t s);
// f32 arena [rows][ldc] -> bf16 hi/lo arena [rows][2 * roundup(d, 16)]
void split_bf16(const float* codes, int64_t rows, int d, int ldc, int DB, void* out,
                hipStream_t s);
void ivf_list_ynmax(const float* yn, const uint32_t* list_off, const uint32_t* list_len,
                    int nlist, float* out, hipStream_t s);
void ivf_flat_scan_mfma(const float* x, int ldx, const float* codes, int ldc, const void* cbf,
                        const int64_t* ids, const float* ynorm, const float* ynmax,
                        const float* rres, const float* rmax,
                        const uint32_t* list_off, const uint32_t* list_len, int nlist, int d,
                        int obits, int64_t n, int nprobe, int k, int metric_l2, IVFBuckets b,
                        int64_t max_items, uint32_t* keys, ProbeRec* recs, uint32_t* stats,
                        float* D, int64_t* I, KernelTimes* kt, hipStream_t s,
                        int list_align = 16, const void* cbs = nullptr,
                        void* qscratch = nullptr,  // query_image_bytes(n, d) + 4 n bytes
                        bool qready = false,  // qscratch already holds x's image
                        unsigned long long* qdone = nullptr,
                        int fold = 0,
                        // ivf_mfma_kq's: keys per thread stream
                        int kt_min = 0);  // cbs is the fold image (split_bf16_stream fold = 1)
// stream image of the arena for the streamed filter: per row bf16(code) (DB
// dims) + a 16-byte tail = 2 DB + 16 bytes.  fold = 0: the tail is the fp32
// norm (+inf for padding rows) + 12 zero bytes; fold = 1 (L2): the tail is the
// row's bias A-fragment {bf16 split of -|y|^2/2 in three parts, 1, 1, 1, 0, 0}
// (padding rows: -inf, 0, 0, 1, 1, 1, 0, 0), so one extra MFMA k-step adds
// -(|x|^2 + |y|^2)/2 to <x, y> and the accumulator is -approx/2 directly.
void split_bf16_stream(const float* codes, int64_t rows, int d, int ldc, int DB,
                       const float* ynorm, const uint32_t* row_list, void* out, hipStream_t s,
                       int fold = 0);
// ---------------- IVF-PQ ----------------
// term[v] = sum_m (||c_{m,code}||^2 + 2 <yC_m, c_{m,code}>) for every arena row
void ivfpq_terms(const uint8_t* codes, const uint32_t* row_list, int64_t nrows,
                 const float* centroids, int ldcent, const float* pq_centroids, int M, int ksub,
                 int dsub, float* terms, hipStream_t s);

// PQ encoding: codes[i][m] = argmin_j ||r_im - c_mj||^2 (first minimum)
// residual r = x - centroid[assign[i]] when centroids != null.
void pq_encode(const float* x, int ldx, int64_t n, const int32_t* assign,
               const float* centroids, int ldcent, const float* pq_centroids, int M, int ksub,
               int dsub, uint8_t* codes, hipStream_t s);

// ---------------- HNSW (one wavefront per query) ----------------
struct HNSWDevice {
    const float* storage;     // [ntotal][ld]
    const float* norms;       // unused (reserved)
    int ld;
    int d;
    const int32_t* levels;    // [ntotal] (level+1 as in faiss)
    const uint64_t* offsets;  // [ntotal+1]
    const int32_t* neighbors;
    const int32_t* cum_nb;    // cum_nneighbor_per_level
    // level-0 neighbours of node v at nb0[v * nb0_stride + j] (a regular copy
    // of the level-0 slices of `neighbors`, so a level-0 hop needs no offsets
    // load); null: read them through offsets
    const int32_t* nb0;
    int nb0_stride;
    // int8 image of the rows for the level-0 prefilter (L2, d <= 128; null:
    // none): q8 [ntotal][128] codes, q8p [ntotal] {o, s, ey, B2}, q8q1
    // [ntotal] sum of the codes (IndexHNSW::sync_device, kernels_hnsw.hip)
    const uint8_t* q8;
    const float* q8p;
    const float* q8q1;
    int nlevels_cum;
    int entry_point;
    int max_level;
    int ntotal;
};
// reference faiss/impl/HNSW.cpp:943-996 (HNSW::search), :852-924 (greedy),
// :605-741 (search_from_candidates), :1096-1342 (MinimaxHeap)
// flags: [n] scratch; queries where an exact distance tie makes the batched
// form unsafe are redone by the sequential kernel (nullptr: no check).
// max(efSearch, k) <= 64: the register kernel (k_hnsw_exact_reg) for every
// query (FAISS_AMD_HNSW=batched: the batched kernel + re-runs); max(efSearch,
// k) > 128 or k > 64: the sequential LDS kernel, with its heaps in
// heap_scratch (hnsw_heap_scratch_words per query) when they exceed the LDS.
void hnsw_search(const HNSWDevice& g, const float* x, int ldx, int64_t n, int k, int efSearch,
                 float* D, int64_t* I, int32_t* I32, uint32_t* visited_scratch,
                 int64_t visited_words_per_query, unsigned long long* stats, uint32_t* flags,
                 hipStream_t s, KernelTimes* kt = nullptr,
                 bool defer = false, float* heap_scratch = nullptr,
                 uint64_t* replay_log = nullptr, int64_t replay_cap = 0,
                 void* arrival_log = nullptr, size_t arrival_log_bytes = 0);
// the register kernel's CandSet update log (64-bit entries per query in
// replay_log): a query whose candidate set meets a layout-dependent decision
// continues from a replayed heap instead of searching level 0 again; a query
// whose log would exceed it searches again.  replay_cap (<= kHnswReplayCap,
// the per-query stride of replay_log) bounds the entries a query may log.
// stats[6..8] count the register kernel's continuations: replayed, searched
// again (log overflowed or absent), log found corrupt (searched again; 0
// unless a bug)
constexpr int64_t kHnswReplayCap = 1024;
constexpr int kHnswStatsWords = 9;
// 32-bit words of global heap scratch per query (0: the heaps fit the LDS)
size_t hnsw_heap_scratch_words(int k, int efSearch, int ld);
// a per-query visited bitmap of vwords words lives in global scratch (for
// some kernel this search may run) rather than the LDS
bool hnsw_visited_scratch_needed(int ld, int k, int efSearch, int64_t vwords);
// the register kernel serves max(efSearch, k) <= 64
bool hnsw_register_eligible(int k, int efSearch);
// the batched kernel (and its tie re-runs) runs for these parameters
bool hnsw_uses_batched(int k, int efSearch);  // leave the flagged queries to the caller
// 128 < max(efSearch, k) <= kHnswWideMaxEf: the wide kernel (k_hnsw_wide,
// candidate set sorted in the LDS) + sequential re-runs of its flagged queries
constexpr int kHnswWideMaxEf = 4096;
bool hnsw_uses_wide(int k, int efSearch);
// flagged queries (flags[q] != 0) -> idx[0 .. *count) (count zeroed first)
void hnsw_flag_compact(const uint32_t* flags, int64_t n, uint32_t* idx, uint32_t* count,
                       hipStream_t s);
// the reference-exact sequential search of the listed queries x[qidx[i]],
// results in compact rows i of D / I32
void hnsw_exact_listed(const HNSWDevice& g, const float* x, int ldx, const uint32_t* qidx,
                       int64_t nf, int k, int efSearch, float* D, int32_t* I32,
                       uint32_t* visited_scratch, int64_t vwords, unsigned long long* stats,
                       hipStream_t s, void* arrival_log = nullptr, size_t arrival_log_bytes = 0);
// bytes of the sequential kernel's arrival-log pool (k_hnsw_exact without
// the result heap) worth providing for n queries of an ntotal-node graph
size_t hnsw_arrival_log_bytes(int64_t n, int64_t ntotal);
// rows: out[i] = in[idx[i]] (d floats, strides ldi / ldo); scatter of
// packed rows of row_words 32-bit words: dst row idx[i] = src row i
void gather_rows(const float* in, int ldi, const uint32_t* idx, int64_t n, int d, float* out,
                 int ldo, hipStream_t s);
void scatter_rows(const void* src, int row_words, const uint32_t* idx, int64_t n, void* dst,
                  hipStream_t s);

// IVF-Flat range search (kernels_range.hip): one wave per (query, probe).
// offsets == nullptr: counts[q*np+p] = hits (dis < radius for L2, > for IP,
// selector rows only); else the hits are written at offsets[q*np+p] in row
// order.  Grid = n*np workgroups (n*np < 2^31).
void ivf_range_flat(const float* x, int64_t n, int ldx, const int32_t* assign, int np,
                    const float* codes, int ldc, const int64_t* ids, const uint32_t* list_off,
                    const uint32_t* list_len, int nlist, int d, int metric_l2, float radius,
                    const uint8_t* selm, uint32_t* counts, const uint64_t* offsets, float* outD,
                    int64_t* outI, hipStream_t s);

}  // namespace kern
}  // namespace faiss_amd
