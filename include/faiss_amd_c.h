/*
 * faiss_amd_c.h — C-ABI of the MI355X-native batched IVF search path.
 *
 * This is the drop-in boundary.  Every `faiss_*` entry point below carries the
 * exact name, argument meaning, ownership rule and return-code convention of
 * the reference's C API (Quaternijkon/hnsw-ivf = Faiss 1.10.0, `c_api/`), so a
 * program linked against the reference `libfaiss_c` relinks against
 * `libfaiss_amd.so` unchanged.  Each declaration cites the
 * reference declaration it replaces.
 *
 * Return codes (reference c_api/error_c.h:19-32, c_api/macros_impl.h:22-56):
 *    0 OK, -1 unknown exception, -2 FaissException, -4 std::exception.
 * The message of the last failure on the calling thread is available from
 * faiss_get_last_error() (reference c_api/error_impl.cpp:15-26).
 *
 * All host-side pointers (x, distances, labels) are owned by the caller.
 * `faiss_amd_*` entry points are extensions with no reference counterpart:
 * they take DEVICE pointers (already resident in HBM) and an optional
 * hipStream_t (passed as void*; NULL = the index's own stream) so that
 * benchmarks and multi-GPU drivers can keep data in HBM.
 */
#ifndef FAISS_AMD_C_H
#define FAISS_AMD_C_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int64_t faiss_idx_t; /* reference c_api/faiss_c.h:17 */
typedef faiss_idx_t idx_t;   /* reference c_api/faiss_c.h:18 */

/* reference c_api/Index_c.h:27-40 */
typedef enum FaissMetricType {
    METRIC_INNER_PRODUCT = 0,
    METRIC_L2 = 1,
} FaissMetricType;

/* reference c_api/error_c.h:19-32 */
typedef enum FaissErrorCode {
    OK = 0,
    UNKNOWN_EXCEPT = -1,
    FAISS_EXCEPT = -2,
    STD_EXCEPT = -4
} FaissErrorCode;

/* Opaque handles.  As in the reference, every index handle is usable as a
 * FaissIndex* (reference c_api/faiss_c.h:28-40, FAISS_DECLARE_CLASS). */
typedef struct FaissIndex_H FaissIndex;
typedef struct FaissIndex_H FaissIndexFlat;
typedef struct FaissIndex_H FaissIndexFlatL2;
typedef struct FaissIndex_H FaissIndexFlatIP;
typedef struct FaissIndex_H FaissIndexIVF;
typedef struct FaissIndex_H FaissIndexIVFFlat;
typedef struct FaissIndex_H FaissIndexIVFPQ;
typedef struct FaissIndex_H FaissIndexHNSW;
typedef struct FaissIndex_H FaissIndexShardsIVF;
typedef struct FaissSearchParameters_H FaissSearchParameters;
typedef struct FaissSearchParameters_H FaissSearchParametersIVF;
typedef struct FaissParameterSpace_H FaissParameterSpace;

/* ---------------- errors ---------------- */
/* reference c_api/error_c.h:35 */
const char* faiss_get_last_error(void);

/* ---------------- Index (reference c_api/Index_c.h) ---------------- */
void faiss_Index_free(FaissIndex* obj);                     /* Index_c.h:50 */
int faiss_Index_d(const FaissIndex*);                       /* Index_c.h:53 */
int faiss_Index_is_trained(const FaissIndex*);              /* Index_c.h:56 */
idx_t faiss_Index_ntotal(const FaissIndex*);                /* Index_c.h:59 */
FaissMetricType faiss_Index_metric_type(const FaissIndex*); /* Index_c.h:62 */
int faiss_Index_verbose(const FaissIndex*);                 /* Index_c.h:64 */
void faiss_Index_set_verbose(FaissIndex*, int);             /* Index_c.h:64 */

/* Index_c.h:72 */
int faiss_Index_train(FaissIndex* index, idx_t n, const float* x);
/* Index_c.h:82 */
int faiss_Index_add(FaissIndex* index, idx_t n, const float* x);
/* Index_c.h:92-96 */
int faiss_Index_add_with_ids(
        FaissIndex* index,
        idx_t n,
        const float* x,
        const idx_t* xids);
/* Index_c.h:108-114 — the hot path: D/I on the host, ascending (dist,id) for
 * L2, descending for IP, unfilled slots = (+FLT_MAX,-1) / (-FLT_MAX,-1). */
int faiss_Index_search(
        const FaissIndex* index,
        idx_t n,
        const float* x,
        idx_t k,
        float* distances,
        idx_t* labels);
/* Index_c.h:128-135 (params may be a FaissSearchParametersIVF) */
int faiss_Index_search_with_params(
        const FaissIndex* index,
        idx_t n,
        const float* x,
        idx_t k,
        const FaissSearchParameters* params,
        float* distances,
        idx_t* labels);
/* Index_c.h:172 */
int faiss_Index_reset(FaissIndex* index);
/* Index_c.h:121-126: labels [n][k] of the k nearest (the search without the
 * distances) */
int faiss_Index_assign(FaissIndex* index, idx_t n, const float* x, idx_t* labels, idx_t k);
/* Index_c.h:196-205 (IndexFlat / IndexIVFFlat / IndexHNSWFlat storage) */
int faiss_Index_reconstruct(const FaissIndex* index, idx_t key, float* recons);
int faiss_Index_reconstruct_n(const FaissIndex* index, idx_t i0, idx_t ni, float* recons);

/* ---------------- SearchParametersIVF (c_api/IndexIVF_c.h:22-35) -------- */
int faiss_SearchParametersIVF_new(FaissSearchParametersIVF** p_sp);
int faiss_SearchParametersIVF_new_with(
        FaissSearchParametersIVF** p_sp,
        void* sel, /* FaissIDSelector* or NULL (borrowed) */
        size_t nprobe,
        size_t max_codes);
void faiss_SearchParametersIVF_free(FaissSearchParametersIVF* obj);
/* IndexIVF_c.h:27 (FAISS_DECLARE_SEARCH_PARAMETERS_DOWNCAST): every search
 * parameter object here carries the IVF fields, so the cast always succeeds */
FaissSearchParametersIVF* faiss_SearchParametersIVF_cast(FaissSearchParameters* sp);

/* ---------------- IDSelector (c_api/impl/AuxIndexStructures_c.h:50-110,
 * c_api/Index_c.h:44-46).  Membership as faiss/impl/IDSelector.cpp; the IVF
 * searches evaluate it on the GPU for every arena row and skip non-members
 * (faiss/IndexIVFFlat.cpp:165-167).  Selectors passed to another selector or
 * to search parameters are borrowed, not owned. */
typedef struct FaissIDSelector_H FaissIDSelector;
typedef struct FaissIDSelector_H FaissIDSelectorRange;
typedef struct FaissIDSelector_H FaissIDSelectorBatch;
typedef struct FaissIDSelector_H FaissIDSelectorBitmap;
typedef struct FaissIDSelector_H FaissIDSelectorNot;
typedef struct FaissIDSelector_H FaissIDSelectorAnd;
typedef struct FaissIDSelector_H FaissIDSelectorOr;
typedef struct FaissIDSelector_H FaissIDSelectorXOr;
int faiss_SearchParameters_new(FaissSearchParameters** p_sp, FaissIDSelector* sel);
void faiss_SearchParameters_free(FaissSearchParameters* obj);
int faiss_IDSelector_is_member(const FaissIDSelector* sel, idx_t id);
void faiss_IDSelector_free(FaissIDSelector* sel);
/* AuxIndexStructures_c.h:62-78 (FAISS_DECLARE_DESTRUCTOR / GETTER) */
void faiss_IDSelectorRange_free(FaissIDSelectorRange* sel);
idx_t faiss_IDSelectorRange_imin(const FaissIDSelectorRange* sel);
idx_t faiss_IDSelectorRange_imax(const FaissIDSelectorRange* sel);
void faiss_IDSelectorBitmap_free(FaissIDSelectorBitmap* sel);
int faiss_IDSelectorRange_new(FaissIDSelectorRange** p_sel, idx_t imin, idx_t imax);
int faiss_IDSelectorBatch_new(FaissIDSelectorBatch** p_sel, size_t n, const idx_t* indices);
/* extension: faiss::IDSelectorArray (faiss/impl/IDSelector.h:54-66), ids borrowed */
int faiss_amd_IDSelectorArray_new(FaissIDSelector** p_sel, size_t n, const idx_t* ids);
int faiss_IDSelectorBitmap_new(FaissIDSelectorBitmap** p_sel, size_t n, const uint8_t* bitmap);
int faiss_IDSelectorNot_new(FaissIDSelectorNot** p_sel, const FaissIDSelector* sel);
int faiss_IDSelectorAnd_new(FaissIDSelectorAnd** p_sel, const FaissIDSelector* lhs_sel,
                            const FaissIDSelector* rhs_sel);
int faiss_IDSelectorOr_new(FaissIDSelectorOr** p_sel, const FaissIDSelector* lhs_sel,
                           const FaissIDSelector* rhs_sel);
int faiss_IDSelectorXOr_new(FaissIDSelectorXOr** p_sel, const FaissIDSelector* lhs_sel,
                            const FaissIDSelector* rhs_sel);
size_t faiss_SearchParametersIVF_nprobe(const FaissSearchParametersIVF*);
void faiss_SearchParametersIVF_set_nprobe(FaissSearchParametersIVF*, size_t);
/* c_api/IndexIVF_c.h:35 (FAISS_DECLARE_GETTER_SETTER max_codes); 0 = unlimited */
size_t faiss_SearchParametersIVF_max_codes(const FaissSearchParametersIVF*);
void faiss_SearchParametersIVF_set_max_codes(FaissSearchParametersIVF*, size_t);
/* extension: IndexIVF::max_codes / parallel_mode (faiss/IndexIVF.h:200-214;
 * the reference C API has no binding; ParameterSpace "max_codes" sets the
 * former, faiss/AutoTune.cpp:530-535).  parallel_mode 0 and 3 run here. */
size_t faiss_amd_IndexIVF_max_codes(const FaissIndexIVF*);
void faiss_amd_IndexIVF_set_max_codes(FaissIndexIVF*, size_t);
int faiss_amd_IndexIVF_parallel_mode(const FaissIndexIVF*);
void faiss_amd_IndexIVF_set_parallel_mode(FaissIndexIVF*, int);
/* extension: efSearch of an HNSW coarse quantizer for this call, 0 = keep
 * (reference SearchParametersIVF::quantizer_params -> SearchParametersHNSW,
 * faiss/IndexIVF.h:77-85, faiss/impl/HNSW.h:46-52) */
void faiss_amd_SearchParametersIVF_set_quantizer_efSearch(
        FaissSearchParametersIVF*,
        int);

/* ---------------- IndexFlat (c_api/IndexFlat_c.h) ---------------- */
/* IndexFlat_c.h:28-31 */
int faiss_IndexFlat_new_with(FaissIndexFlat** p_index, idx_t d, FaissMetricType metric);
/* IndexFlat_c.h:87 */
int faiss_IndexFlatL2_new_with(FaissIndexFlatL2** p_index, idx_t d);
/* IndexFlat_c.h:77 */
int faiss_IndexFlatIP_new_with(FaissIndexFlat** p_index, idx_t d);
/* IndexFlat_c.h:40: pointer to the host mirror of xb (d*ntotal floats) */
void faiss_IndexFlat_xb(FaissIndexFlat* index, float** p_xb, size_t* p_size);
/* IndexFlat_c.h:24-26, 71-93: default constructors (d = 0), destructors and
 * FAISS_DECLARE_INDEX_DOWNCAST (NULL when the index is not of that type) */
int faiss_IndexFlat_new(FaissIndexFlat** p_index);
int faiss_IndexFlatIP_new(FaissIndexFlatIP** p_index);
int faiss_IndexFlatL2_new(FaissIndexFlatL2** p_index);
void faiss_IndexFlat_free(FaissIndexFlat* obj);
void faiss_IndexFlatIP_free(FaissIndexFlatIP* obj);
void faiss_IndexFlatL2_free(FaissIndexFlatL2* obj);
FaissIndexFlat* faiss_IndexFlat_cast(FaissIndex* index);
FaissIndexFlatIP* faiss_IndexFlatIP_cast(FaissIndex* index);
FaissIndexFlatL2* faiss_IndexFlatL2_cast(FaissIndex* index);

/* ---------------- IndexIVF (c_api/IndexIVF_c.h) ---------------- */
size_t faiss_IndexIVF_nlist(const FaissIndexIVF*);              /* :59 */
size_t faiss_IndexIVF_nprobe(const FaissIndexIVF*);             /* :61 */
void faiss_IndexIVF_set_nprobe(FaissIndexIVF*, size_t);         /* :61 */
FaissIndex* faiss_IndexIVF_quantizer(const FaissIndexIVF*);     /* :63 */
int faiss_IndexIVF_own_fields(const FaissIndexIVF*);            /* :72 */
void faiss_IndexIVF_set_own_fields(FaissIndexIVF*, int);        /* :72 */
/* IndexIVF_c.h:112-121: assign/centroid_dis are [n*nprobe] host arrays */
int faiss_IndexIVF_search_preassigned(
        const FaissIndexIVF* index,
        idx_t n,
        const float* x,
        idx_t k,
        const idx_t* assign,
        const float* centroid_dis,
        float* distances,
        idx_t* labels,
        int store_pairs);
/* IndexIVF_c.h:123 */
size_t faiss_IndexIVF_get_list_size(const FaissIndexIVF* index, size_t list_no);
/* IndexIVF_c.h:46-52, 141: destructor, downcast, list-size imbalance
 * (faiss/invlists/InvertedLists.cpp imbalance_factor: nlist * sum(size^2) /
 * sum(size)^2) */
void faiss_IndexIVF_free(FaissIndexIVF* obj);
FaissIndexIVF* faiss_IndexIVF_cast(FaissIndex* index);
double faiss_IndexIVF_imbalance_factor(const FaissIndexIVF* index);
/* IndexIVF_c.h:151-155 */
void faiss_IndexIVF_invlists_get_ids(
        const FaissIndexIVF* index,
        size_t list_no,
        idx_t* invlist);
/* extension: copy the list's codes (list_size * code_size bytes) */
void faiss_amd_IndexIVF_invlists_get_codes(
        const FaissIndexIVF* index,
        size_t list_no,
        uint8_t* codes);
/* extension: code size in bytes of one stored vector */
size_t faiss_amd_IndexIVF_code_size(const FaissIndexIVF* index);

/* reference IndexIVF_c.h:162-178 (global stats, like indexIVF_stats) */
typedef struct FaissIndexIVFStats {
    size_t nq;
    size_t nlist;
    size_t ndis;
    size_t nheap_updates;
    double quantization_time;
    double search_time;
} FaissIndexIVFStats;
void faiss_IndexIVFStats_reset(FaissIndexIVFStats* stats);
FaissIndexIVFStats* faiss_get_indexIVF_stats(void);

/* reference faiss/IndexIVF.h:28-32 — this fork's per-query latency record
 * (microseconds).  GPU semantics: quantization_us = coarse-stage wall time / n
 * (the reference's amortisation over a slice; the batch is one slice),
 * list_scan_us = wall time of the batched scan stage, total = their sum. */
typedef struct FaissQueryLatencyStats {
    double total_us;
    double quantization_us;
    double list_scan_us;
} FaissQueryLatencyStats;
/* extension, replaces IndexIVF::search_stats (faiss/IndexIVF.h:329-337,
 * faiss/IndexIVF.cpp:725-867; the reference C API has no binding for it).
 * params may be NULL or a FaissSearchParametersIVF; per_query_stats may be
 * NULL or [n].  Updates indexIVF_stats nq / nlist / ndis. */
int faiss_amd_IndexIVF_search_stats(
        const FaissIndexIVF* index,
        idx_t n,
        const float* x,
        idx_t k,
        const FaissSearchParameters* params,
        float* distances,
        idx_t* labels,
        FaissQueryLatencyStats* per_query_stats);
/* extension, replaces IndexIVF::search_preassigned_stats
 * (faiss/IndexIVF.h:306-317): sets list_scan_us of each query; ivf_stats NULL
 * = the global indexIVF_stats */
int faiss_amd_IndexIVF_search_preassigned_stats(
        const FaissIndexIVF* index,
        idx_t n,
        const float* x,
        idx_t k,
        const idx_t* assign,
        const float* centroid_dis,
        float* distances,
        idx_t* labels,
        int store_pairs,
        const FaissSearchParameters* params,
        FaissIndexIVFStats* ivf_stats,
        FaissQueryLatencyStats* per_query_stats);

/* ---------------- IndexIVFFlat (c_api/IndexIVFFlat_c.h) ---------------- */
/* IndexIVFFlat_c.h:47-51 */
int faiss_IndexIVFFlat_new_with(
        FaissIndexIVFFlat** p_index,
        FaissIndex* quantizer,
        size_t d,
        size_t nlist);
/* IndexIVFFlat_c.h:53-58 */
int faiss_IndexIVFFlat_new_with_metric(
        FaissIndexIVFFlat** p_index,
        FaissIndex* quantizer,
        size_t d,
        size_t nlist,
        FaissMetricType metric);

/* IndexIVFFlat_c.h:25-45: constructor without arguments (an empty index
 * whose quantizer is set by reading), destructor, downcast and the IndexIVF
 * getters under the IndexIVFFlat name */
int faiss_IndexIVFFlat_new(FaissIndexIVFFlat** p_index);
void faiss_IndexIVFFlat_free(FaissIndexIVFFlat* obj);
FaissIndexIVFFlat* faiss_IndexIVFFlat_cast(FaissIndex* index);
size_t faiss_IndexIVFFlat_nlist(const FaissIndexIVFFlat*);
size_t faiss_IndexIVFFlat_nprobe(const FaissIndexIVFFlat*);
void faiss_IndexIVFFlat_set_nprobe(FaissIndexIVFFlat*, size_t);
FaissIndex* faiss_IndexIVFFlat_quantizer(const FaissIndexIVFFlat*);
int faiss_IndexIVFFlat_own_fields(const FaissIndexIVFFlat*);
void faiss_IndexIVFFlat_set_own_fields(FaissIndexIVFFlat*, int);

/* ---------------- IndexIVFPQ (no reference C binding; mirrors the C++
 * constructor faiss/IndexIVFPQ.h:IndexIVFPQ(quantizer,d,nlist,M,nbits)) --- */
int faiss_amd_IndexIVFPQ_new_with(
        FaissIndexIVFPQ** p_index,
        FaissIndex* quantizer,
        size_t d,
        size_t nlist,
        size_t M,
        size_t nbits,
        FaissMetricType metric);
/* pointer to the PQ centroids [M][ksub][dsub] (host) */
void faiss_amd_IndexIVFPQ_pq_centroids(
        FaissIndexIVFPQ* index,
        float** p_centroids,
        size_t* p_size);
/* M, nbits, by_residual, use_precomputed_table */
int faiss_amd_IndexIVFPQ_info(
        const FaissIndexIVFPQ* index,
        size_t* M,
        size_t* nbits,
        int* by_residual,
        int* use_precomputed_table);
/* faiss IndexIVFPQ::use_precomputed_table (faiss/IndexIVFPQ.h:41-47): the
 * table the reference's scanner would use (0 or 1); selects the exact
 * arithmetic of the GPU re-rank.  0 is always valid, 1 needs by_residual L2 */
int faiss_amd_IndexIVFPQ_set_use_precomputed_table(FaissIndexIVFPQ* index, int v);

/* ---------------- IndexHNSWFlat (C++ faiss/IndexHNSW.h:IndexHNSWFlat) ---- */
int faiss_amd_IndexHNSWFlat_new_with(
        FaissIndexHNSW** p_index,
        int d,
        int M,
        FaissMetricType metric);
int faiss_amd_IndexHNSW_efSearch(const FaissIndexHNSW*);
void faiss_amd_IndexHNSW_set_efSearch(FaissIndexHNSW*, int);
int faiss_amd_IndexHNSW_efConstruction(const FaissIndexHNSW*);
void faiss_amd_IndexHNSW_set_efConstruction(FaissIndexHNSW*, int);
/* the flat storage index of an IndexHNSW (owned by it) */
FaissIndex* faiss_amd_IndexHNSW_storage(const FaissIndexHNSW* index);
/* extension, replaces IndexHNSW::search_stats (faiss/IndexHNSW.h:68-76,
 * faiss/IndexHNSW.cpp:345-366): total_us = list_scan_us = the batch's
 * traversal time, quantization_us = 0 */
int faiss_amd_IndexHNSW_search_stats(
        const FaissIndexHNSW* index,
        idx_t n,
        const float* x,
        idx_t k,
        const FaissSearchParameters* params,
        float* distances,
        idx_t* labels,
        FaissQueryLatencyStats* per_query_stats);
/* faiss/impl/HNSW.h:234-253 — the global hnsw_stats (faiss.cvar.hnsw_stats
 * in the reference's Python tests).  Device-API searches are folded in at the
 * next synchronous call or by faiss_amd_fold_device_stats(index). */
typedef struct FaissHNSWStats {
    size_t n1;
    size_t n2;
    size_t ndis;
    size_t nhops;
} FaissHNSWStats;
FaissHNSWStats* faiss_amd_get_hnsw_stats(void);
void faiss_amd_HNSWStats_reset(void);
/* Not in the reference (diagnostic, the bench's byte count): rows the GPU
 * HNSW kernels read — fp32 rows, and int8-image rows of the register kernel's
 * level-0 prefilter — since the last faiss_amd_HNSWStats_reset. */
void faiss_amd_get_hnsw_row_stats(uint64_t* fp32_rows, uint64_t* q8_rows);
/* Not in the reference (diagnostic): queries of the register HNSW kernel that
 * met a layout-dependent decision and continued from the replayed update log,
 * that searched level 0 again because their log overflowed, and whose log was
 * found corrupt (searched again; must stay 0) — since the last reset. */
void faiss_amd_get_hnsw_replay_stats(uint64_t* replayed, uint64_t* searched_again,
                                     uint64_t* replay_bad);
int faiss_amd_fold_device_stats(const FaissIndex* index);
/* faiss::TimeoutCallback::reset / InterruptCallback::clear_instance
 * (faiss/impl/AuxIndexStructures.h:135-170, C++ only in the reference; here
 * for C / ctypes callers and tests): seconds >= 0 installs a timeout callback
 * (a host search polled after it fires throws "computation interrupted"),
 * seconds < 0 removes the installed callback. */
void faiss_amd_set_interrupt_timeout(double seconds);
/* graph export for tests: levels[ntotal], offsets[ntotal+1], neighbors[],
 * cum_nneighbor_per_level[]; pass NULL to query sizes only */
int faiss_amd_IndexHNSW_graph(
        const FaissIndexHNSW* index,
        int* entry_point,
        int* max_level,
        size_t* n_neighbors,
        size_t* n_cum,
        const int32_t** levels,
        const size_t** offsets,
        const int32_t** neighbors,
        const int32_t** cum_nneighbor_per_level);

/* ---------------- IndexShardsIVF (faiss/IndexShardsIVF.h:19-40) -------- */
/* A set of IVF shards sharing one coarse quantizer; search = one coarse pass
 * then search_preassigned on every shard then merge_knn_results. */
int faiss_amd_IndexShardsIVF_new(
        FaissIndexShardsIVF** p_index,
        FaissIndex* quantizer,
        size_t nlist,
        int threaded,
        int successive_ids);
int faiss_amd_IndexShardsIVF_add_shard(FaissIndexShardsIVF* index, FaissIndex* shard);
int faiss_amd_IndexShardsIVF_count(const FaissIndexShardsIVF* index);
/* borrowed pointer to shard i (owned by the shards index or the caller) */
int faiss_amd_IndexShardsIVF_shard(const FaissIndexShardsIVF* index, int i,
                                   FaissIndex** p_shard);
/* faiss/IndexIVF.h:393-402 IndexIVF::copy_subset_to
 * (faiss/invlists/InvertedLists.cpp:91-175): append to dst the entries of src
 * selected by subset_type 0 = ids in [a1, a2), 1 = id % a1 == a2,
 * 2 = element range [a1, a2) of the running total, 3 = fraction a2 / a1 of
 * every list, 4 = lists [a1, a2).  Host lists; n_added may be NULL. */
int faiss_amd_IndexIVF_copy_subset_to(
        const FaissIndex* src,
        FaissIndex* dst,
        int subset_type,
        idx_t a1,
        idx_t a2,
        size_t* n_added);
/* faiss/gpu/GpuCloner.cpp:283-420 (ToGpuClonerMultiple::clone_Index_to_shards
 * of an IVF index): nshard copies of src, shard i on devices[i] (NULL: src's
 * device) holding shard_type 1 (id % nshard == i), 2 (id range) or 4 (list
 * range).  Shards on several devices are searched over RCCL.  The result owns
 * its shards; free it with faiss_Index_free. */
int faiss_amd_index_ivf_to_shards(
        const FaissIndex* src,
        int nshard,
        int shard_type,
        const int* devices,
        FaissIndexShardsIVF** p_index);

/* ---------------- range search (c_api/impl/AuxIndexStructures_c.h:20-50,
 * c_api/Index_c.h:148-153, c_api/IndexIVF_c.h range_search_preassigned) ----
 * Results of query i: labels/distances[lims[i], lims[i+1]) in the reference's
 * scan order (probe order, then list order).  IndexIVFFlat only. */
typedef struct FaissRangeSearchResult_H FaissRangeSearchResult;
int faiss_RangeSearchResult_new(FaissRangeSearchResult** p_rsr, idx_t nq);
void faiss_RangeSearchResult_free(FaissRangeSearchResult* obj);
size_t faiss_RangeSearchResult_nq(const FaissRangeSearchResult* rsr);
size_t faiss_RangeSearchResult_buffer_size(const FaissRangeSearchResult* rsr);
void faiss_RangeSearchResult_lims(FaissRangeSearchResult* rsr, size_t** lims);
void faiss_RangeSearchResult_labels(FaissRangeSearchResult* rsr, idx_t** labels,
                                    float** distances);
int faiss_Index_range_search(const FaissIndex* index, idx_t n, const float* x, float radius,
                             FaissRangeSearchResult* result);
int faiss_amd_Index_range_search_with_params(const FaissIndex* index, idx_t n, const float* x,
                                             float radius, const FaissSearchParameters* params,
                                             FaissRangeSearchResult* result);
int faiss_IndexIVF_range_search_preassigned(const FaissIndexIVF* index, idx_t n,
                                            const float* x, float radius, const idx_t* assign,
                                            const float* centroid_dis,
                                            FaissRangeSearchResult* result);

/* ---------------- I/O (c_api/index_io_c.h) ---------------- */
int faiss_write_index(const FaissIndex* idx, FILE* f);                   /* :28 */
int faiss_write_index_fname(const FaissIndex* idx, const char* fname);   /* :33 */
int faiss_read_index(FILE* f, int io_flags, FaissIndex** p_out);         /* :41 */
int faiss_read_index_fname(const char* fname, int io_flags, FaissIndex** p_out); /* :46 */
/* faiss/index_io.h:37-64 flags: IO_FLAG_MMAP (8 | 0x646f0000) maps the index
 * file's `ilar` lists (faiss/invlists/OnDiskInvertedLists.cpp:759-800);
 * `ilod` lists are always mapped from their data file (:706-757),
 * IO_FLAG_ONDISK_SAME_DIR (4) looks for it next to the index file. */
/* IVF index with its lists in a separate OnDiskInvertedLists data file: the
 * reference's OnDiskInvertedLists + replace_invlists + write_index
 * (faiss/invlists/OnDiskInvertedLists.cpp:683-704). */
int faiss_amd_write_index_ondisk(const FaissIndex* idx, const char* fname,
                                 const char* lists_fname);

/* c_api/clone_index_c.h:23 (faiss/clone_index.cpp): a deep copy of the
 * index, made through the serialized form (write_index + read_index), on the
 * calling thread's device */
int faiss_clone_index(const FaissIndex* idx, FaissIndex** p_out);

/* ---------------- factory / tuning ---------------- */
/* c_api/index_factory_c.h:24-28; supports "Flat", "IVF<n>,Flat",
 * "IVF<n>,PQ<M>[x<nbits>][np]", "IVF<n>_HNSW<M>,Flat|PQ..", "HNSW<M>[,Flat]" */
int faiss_index_factory(
        FaissIndex** p_index,
        int d,
        const char* description,
        FaissMetricType metric);
/* c_api/AutoTune_c.h:36,63 — "nprobe", "efSearch", "quantizer_efSearch" */
int faiss_ParameterSpace_new(FaissParameterSpace** space);
void faiss_ParameterSpace_free(FaissParameterSpace* space);
int faiss_ParameterSpace_set_index_parameter(
        const FaissParameterSpace*,
        FaissIndex*,
        const char*,
        double);

/* ---------------- merge (faiss/utils/Heap.cpp:159-230) ---------------- */
/* merge nshard sorted result tables [nshard][n][k] into [n][k] (L2: keep
 * smallest; IP: keep largest; ties -> lower shard index). Host pointers. */
int faiss_amd_merge_knn_results(
        size_t n,
        size_t k,
        int nshard,
        const float* all_distances,
        const idx_t* all_labels,
        float* distances,
        idx_t* labels,
        FaissMetricType metric);

/* extension: dynamic type of a handle ("IndexFlat", "IndexIVFFlat",
 * "IndexIVFPQ", "IndexHNSWFlat", "IndexShardsIVF", "Index") */
const char* faiss_amd_Index_type(const FaissIndex* index);

/* ---------------- device-resident extensions (no reference counterpart) */
/* number of visible HIP devices (fails loudly: -4 when the HIP runtime
 * cannot be initialised) */
int faiss_amd_device_count(int* count);
/* select the device an index is created on (default 0) for this thread */
int faiss_amd_set_device(int device);
/* ensure all host-side index data is uploaded to HBM */
int faiss_amd_Index_sync_device(FaissIndex* index);
/* search with x / distances / labels in HBM (device pointers) on `stream` */
int faiss_amd_Index_search_device(
        const FaissIndex* index,
        idx_t n,
        const float* x_dev,
        idx_t k,
        float* distances_dev,
        idx_t* labels_dev,
        void* stream);
/* search_preassigned with device pointers; assign_dev is int32 [n*nprobe]
 * (list numbers, -1 = skip), centroid_dis_dev f32 [n*nprobe].  A query's
 * probes name distinct lists here (the coarse quantizer's output does); the
 * host entry point faiss_IndexIVF_search_preassigned also accepts a list
 * named twice and then returns the reference's duplicated entries. */
int faiss_amd_IndexIVF_search_preassigned_device(
        const FaissIndexIVF* index,
        idx_t n,
        const float* x_dev,
        idx_t k,
        int nprobe,
        const int32_t* assign_dev,
        const float* centroid_dis_dev,
        float* distances_dev,
        idx_t* labels_dev,
        void* stream);
/* coarse quantization only (device): top-nprobe lists per query */
int faiss_amd_IndexIVF_quantize_device(
        const FaissIndexIVF* index,
        idx_t n,
        const float* x_dev,
        int nprobe,
        float* coarse_dis_dev,
        int32_t* assign_dev,
        void* stream);
/* device-side merge of nshard result tables (same semantics as
 * faiss_amd_merge_knn_results) */
int faiss_amd_merge_knn_results_device(
        size_t n,
        size_t k,
        int nshard,
        const float* all_distances_dev,
        const idx_t* all_labels_dev,
        float* distances_dev,
        idx_t* labels_dev,
        FaissMetricType metric,
        void* stream);
/* extension: emulate a reference run on t OpenMP threads (IndexIVF::search
 * quantizes min(t, n) slices, each in the form its size selects,
 * faiss/IndexIVF.cpp:359-368); default 1 */
int faiss_amd_set_search_slices(int t);
/* timing of the dominant kernel in the last search on this index: number of
 * launches and summed milliseconds (HIP events, only when enabled) */
int faiss_amd_set_kernel_timing(int enable);
/* time only the kernel stage of this name (NULL or "": every stage) */
int faiss_amd_set_kernel_timing_filter(const char* name);
int faiss_amd_last_kernel_times(
        const FaissIndex* index,
        int* n_kernels,
        char* names,      /* n_kernels * 32 chars */
        double* millis,   /* n_kernels */
        double* units);   /* n_kernels: work units (bytes or flops) */

int faiss_amd_reset_kernel_times(FaissIndex* index);
/* diagnostic (tests): copy HBM arena rows [row0, row0 + n) of an IVF index to
 * host `out`: what = 0 the code rows, 1 the row -> list table (uint32, ~0 =
 * padding row), 2 the MFMA filter's stream image (IVF-Flat; IVF-PQ when built
 * with FAISS_AMD_PQ_FILTER=image).  *row_bytes = bytes per row, *rows = arena
 * rows (either may be NULL); out = NULL only queries them. */
int faiss_amd_IndexIVF_debug_rows(const FaissIndex* index, int what, int64_t row0, int64_t n,
                                  void* out, size_t* row_bytes, int64_t* rows);
/* faiss::float_rand (faiss/utils/random.cpp:95-112), bit-exact restatement:
 * the synthetic inputs of the benchmark are regenerated on the GPU box */
int faiss_amd_float_rand(float* x, size_t n, int64_t seed);
/* extension: rows row0, row0 + step, ... (nout of them) of the float_rand
 * stream of n_rows * d floats viewed as [n_rows][d] (shards of the large
 * synthetic sets without materialising them) */
int faiss_amd_float_rand_rows(float* out, int64_t n_rows, int d, int64_t seed, int64_t row0,
                              int64_t step, int64_t nout);

#ifdef __cplusplus
}
#endif

#endif /* FAISS_AMD_C_H */
