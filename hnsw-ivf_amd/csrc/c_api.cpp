// c_api.cpp — the extern "C" boundary (include/faiss_amd_c.h).
//
// Conventions restated from the reference C API: every entry point returns
// 0 / -2 (FaissException) / -4 (std::exception) / -1 (other), and stores the
// message in a thread-local slot read by faiss_get_last_error()
// (reference c_api/macros_impl.h:22-56, c_api/error_impl.cpp:15-26).
#include <cmath>
#include <limits>
#include <cstring>
#include <string>

#include "../../include/faiss_amd.h"
#include "../../include/faiss_amd_c.h"
#include "kernels.h"

using namespace faiss_amd;

namespace faiss_amd {
void set_current_device(int d);
}

namespace {
thread_local std::string g_last_error;

struct SearchParamsC {
    SearchParametersIVF ivf;
    SearchParametersHNSW hnsw;
    bool has_q = false;
    SearchParamsC() { ivf.nprobe = 1; }
};

inline Index* IX(FaissIndex* p) { return reinterpret_cast<Index*>(p); }
inline const Index* IX(const FaissIndex* p) { return reinterpret_cast<const Index*>(p); }
inline FaissIndex* FX(Index* p) { return reinterpret_cast<FaissIndex*>(p); }

IndexIVF* IVF(FaissIndex* p) {
    auto r = dynamic_cast<IndexIVF*>(IX(p));
    FAISS_THROW_IF_NOT_MSG(r, "index is not an IndexIVF");
    return r;
}
const IndexIVF* IVF(const FaissIndex* p) {
    auto r = dynamic_cast<const IndexIVF*>(IX(p));
    FAISS_THROW_IF_NOT_MSG(r, "index is not an IndexIVF");
    return r;
}
}  // namespace

#define C_TRY try {
#define C_CATCH                                   \
    }                                             \
    catch (FaissException & e) {                  \
        g_last_error = e.what();                  \
        return -2;                                \
    }                                             \
    catch (std::exception & e) {                  \
        g_last_error = e.what();                  \
        return -4;                                \
    }                                             \
    catch (...) {                                 \
        g_last_error = "Unknown error";           \
        return -1;                                \
    }                                             \
    return 0;

extern "C" {

const char* faiss_get_last_error(void) { return g_last_error.c_str(); }

void faiss_Index_free(FaissIndex* obj) { delete IX(obj); }
int faiss_Index_d(const FaissIndex* i) { return IX(i)->d; }
int faiss_Index_is_trained(const FaissIndex* i) { return IX(i)->is_trained ? 1 : 0; }
idx_t faiss_Index_ntotal(const FaissIndex* i) { return IX(i)->ntotal; }
FaissMetricType faiss_Index_metric_type(const FaissIndex* i) {
    return (FaissMetricType)IX(i)->metric_type;
}
int faiss_Index_verbose(const FaissIndex* i) { return IX(i)->verbose ? 1 : 0; }
void faiss_Index_set_verbose(FaissIndex* i, int v) { IX(i)->verbose = v != 0; }

int faiss_Index_train(FaissIndex* index, idx_t n, const float* x) {
    C_TRY IX(index)->train(n, x);
    C_CATCH
}
int faiss_Index_add(FaissIndex* index, idx_t n, const float* x) {
    C_TRY IX(index)->add(n, x);
    C_CATCH
}
int faiss_Index_add_with_ids(FaissIndex* index, idx_t n, const float* x, const idx_t* xids) {
    C_TRY IX(index)->add_with_ids(n, x, xids);
    C_CATCH
}
int faiss_Index_search(const FaissIndex* index, idx_t n, const float* x, idx_t k,
                       float* distances, idx_t* labels) {
    C_TRY IX(index)->search(n, x, k, distances, labels, nullptr);
    C_CATCH
}

static const SearchParameters* resolve_params(const FaissSearchParameters* p) {
    if (!p) return nullptr;
    auto sp = reinterpret_cast<const SearchParamsC*>(p);
    return &sp->ivf;
}

int faiss_Index_search_with_params(const FaissIndex* index, idx_t n, const float* x, idx_t k,
                                   const FaissSearchParameters* params, float* distances,
                                   idx_t* labels) {
    C_TRY IX(index)->search(n, x, k, distances, labels, resolve_params(params));
    C_CATCH
}
int faiss_Index_reset(FaissIndex* index) {
    C_TRY IX(index)->reset();
    C_CATCH
}
// faiss/Index.cpp:38-43 (assign = search with the distances discarded)
int faiss_Index_assign(FaissIndex* index, idx_t n, const float* x, idx_t* labels, idx_t k) {
    C_TRY std::vector<float> D((size_t)n * k);
    IX(index)->search(n, x, k, D.data(), labels, nullptr);
    C_CATCH
}
int faiss_Index_reconstruct(const FaissIndex* index, idx_t key, float* recons) {
    C_TRY IX(index)->reconstruct(key, recons);
    C_CATCH
}
// faiss/Index.cpp:50-55
int faiss_Index_reconstruct_n(const FaissIndex* index, idx_t i0, idx_t ni, float* recons) {
    C_TRY const Index* ix = IX(index);
    for (idx_t i = 0; i < ni; i++) ix->reconstruct(i0 + i, recons + (size_t)i * ix->d);
    C_CATCH
}

// ---------------- SearchParametersIVF
int faiss_SearchParametersIVF_new(FaissSearchParametersIVF** p_sp) {
    C_TRY* p_sp = reinterpret_cast<FaissSearchParametersIVF*>(new SearchParamsC());
    C_CATCH
}
int faiss_SearchParametersIVF_new_with(FaissSearchParametersIVF** p_sp, void* sel, size_t nprobe,
                                       size_t max_codes) {
    C_TRY auto sp = new SearchParamsC();
    sp->ivf.sel = reinterpret_cast<IDSelector*>(sel);
    sp->ivf.nprobe = nprobe;
    sp->ivf.max_codes = max_codes;
    *p_sp = reinterpret_cast<FaissSearchParametersIVF*>(sp);
    C_CATCH
}
// ---------------- IDSelector (c_api/impl/AuxIndexStructures_c.h:50-110)
int faiss_SearchParameters_new(FaissSearchParameters** p_sp, FaissIDSelector* sel) {
    C_TRY auto sp = new SearchParamsC();
    sp->ivf.sel = reinterpret_cast<IDSelector*>(sel);
    sp->ivf.nprobe = 0;  // 0 = the index's own nprobe (plain SearchParameters)
    *p_sp = reinterpret_cast<FaissSearchParameters*>(sp);
    C_CATCH
}
void faiss_SearchParameters_free(FaissSearchParameters* obj) {
    delete reinterpret_cast<SearchParamsC*>(obj);
}
static IDSelector* SEL(FaissIDSelector* p) { return reinterpret_cast<IDSelector*>(p); }
static const IDSelector* SEL(const FaissIDSelector* p) {
    return reinterpret_cast<const IDSelector*>(p);
}
int faiss_IDSelector_is_member(const FaissIDSelector* sel, idx_t id) {
    return SEL(sel)->is_member(id) ? 1 : 0;
}
void faiss_IDSelector_free(FaissIDSelector* sel) { delete SEL(sel); }
void faiss_IDSelectorRange_free(FaissIDSelectorRange* sel) { delete SEL(sel); }
void faiss_IDSelectorBitmap_free(FaissIDSelectorBitmap* sel) { delete SEL(sel); }
idx_t faiss_IDSelectorRange_imin(const FaissIDSelectorRange* sel) {
    auto r = dynamic_cast<const IDSelectorRange*>(SEL(sel));
    return r ? r->imin : 0;
}
idx_t faiss_IDSelectorRange_imax(const FaissIDSelectorRange* sel) {
    auto r = dynamic_cast<const IDSelectorRange*>(SEL(sel));
    return r ? r->imax : 0;
}
int faiss_IDSelectorRange_new(FaissIDSelectorRange** p_sel, idx_t imin, idx_t imax) {
    C_TRY* p_sel = reinterpret_cast<FaissIDSelectorRange*>(new IDSelectorRange(imin, imax));
    C_CATCH
}
int faiss_IDSelectorBatch_new(FaissIDSelectorBatch** p_sel, size_t n, const idx_t* indices) {
    C_TRY* p_sel = reinterpret_cast<FaissIDSelectorBatch*>(new IDSelectorBatch(n, indices));
    C_CATCH
}
int faiss_amd_IDSelectorArray_new(FaissIDSelector** p_sel, size_t n, const idx_t* ids) {
    C_TRY* p_sel = reinterpret_cast<FaissIDSelector*>(new IDSelectorArray(n, ids));
    C_CATCH
}
int faiss_IDSelectorBitmap_new(FaissIDSelectorBitmap** p_sel, size_t n, const uint8_t* bitmap) {
    C_TRY* p_sel = reinterpret_cast<FaissIDSelectorBitmap*>(new IDSelectorBitmap(n, bitmap));
    C_CATCH
}
int faiss_IDSelectorNot_new(FaissIDSelectorNot** p_sel, const FaissIDSelector* sel) {
    C_TRY* p_sel = reinterpret_cast<FaissIDSelectorNot*>(new IDSelectorNot(SEL(sel)));
    C_CATCH
}
static int sel_binary(FaissIDSelector** p, const FaissIDSelector* a, const FaissIDSelector* b,
                      int op) {
    C_TRY* p = reinterpret_cast<FaissIDSelector*>(new IDSelectorBinary(SEL(a), SEL(b), op));
    C_CATCH
}
int faiss_IDSelectorAnd_new(FaissIDSelectorAnd** p_sel, const FaissIDSelector* lhs,
                            const FaissIDSelector* rhs) {
    return sel_binary(reinterpret_cast<FaissIDSelector**>(p_sel), lhs, rhs, 0);
}
int faiss_IDSelectorOr_new(FaissIDSelectorOr** p_sel, const FaissIDSelector* lhs,
                           const FaissIDSelector* rhs) {
    return sel_binary(reinterpret_cast<FaissIDSelector**>(p_sel), lhs, rhs, 1);
}
int faiss_IDSelectorXOr_new(FaissIDSelectorXOr** p_sel, const FaissIDSelector* lhs,
                            const FaissIDSelector* rhs) {
    return sel_binary(reinterpret_cast<FaissIDSelector**>(p_sel), lhs, rhs, 2);
}

void faiss_SearchParametersIVF_free(FaissSearchParametersIVF* obj) {
    delete reinterpret_cast<SearchParamsC*>(obj);
}
FaissSearchParametersIVF* faiss_SearchParametersIVF_cast(FaissSearchParameters* sp) {
    return reinterpret_cast<FaissSearchParametersIVF*>(sp);
}
size_t faiss_SearchParametersIVF_nprobe(const FaissSearchParametersIVF* p) {
    return reinterpret_cast<const SearchParamsC*>(p)->ivf.nprobe;
}
void faiss_SearchParametersIVF_set_nprobe(FaissSearchParametersIVF* p, size_t v) {
    reinterpret_cast<SearchParamsC*>(p)->ivf.nprobe = v;
}
size_t faiss_SearchParametersIVF_max_codes(const FaissSearchParametersIVF* p) {
    return reinterpret_cast<const SearchParamsC*>(p)->ivf.max_codes;
}
void faiss_SearchParametersIVF_set_max_codes(FaissSearchParametersIVF* p, size_t v) {
    reinterpret_cast<SearchParamsC*>(p)->ivf.max_codes = v;
}
size_t faiss_amd_IndexIVF_max_codes(const FaissIndexIVF* index) { return IVF(index)->max_codes; }
void faiss_amd_IndexIVF_set_max_codes(FaissIndexIVF* index, size_t v) {
    IVF(index)->max_codes = v;
}
int faiss_amd_IndexIVF_parallel_mode(const FaissIndexIVF* index) {
    return IVF(index)->parallel_mode;
}
void faiss_amd_IndexIVF_set_parallel_mode(FaissIndexIVF* index, int v) {
    IVF(index)->parallel_mode = v;
}
void faiss_amd_SearchParametersIVF_set_quantizer_efSearch(FaissSearchParametersIVF* p, int ef) {
    auto sp = reinterpret_cast<SearchParamsC*>(p);
    if (ef > 0) {
        sp->hnsw.efSearch = ef;
        sp->ivf.quantizer_params = &sp->hnsw;
    } else {
        sp->ivf.quantizer_params = nullptr;
    }
}

// ---------------- IndexFlat
int faiss_IndexFlat_new_with(FaissIndexFlat** p_index, idx_t d, FaissMetricType metric) {
    C_TRY* p_index = FX(new IndexFlat(d, (MetricType)metric));
    C_CATCH
}
int faiss_IndexFlatL2_new_with(FaissIndexFlatL2** p_index, idx_t d) {
    C_TRY* p_index = FX(new IndexFlatL2(d));
    C_CATCH
}
int faiss_IndexFlatIP_new_with(FaissIndexFlat** p_index, idx_t d) {
    C_TRY* p_index = FX(new IndexFlatIP(d));
    C_CATCH
}
int faiss_IndexFlat_new(FaissIndexFlat** p_index) {
    C_TRY* p_index = FX(new IndexFlat());
    C_CATCH
}
int faiss_IndexFlatIP_new(FaissIndexFlatIP** p_index) {
    C_TRY* p_index = FX(new IndexFlatIP(0));
    C_CATCH
}
int faiss_IndexFlatL2_new(FaissIndexFlatL2** p_index) {
    C_TRY* p_index = FX(new IndexFlatL2(0));
    C_CATCH
}
void faiss_IndexFlat_free(FaissIndexFlat* obj) { delete IX(obj); }
void faiss_IndexFlatIP_free(FaissIndexFlatIP* obj) { delete IX(obj); }
void faiss_IndexFlatL2_free(FaissIndexFlatL2* obj) { delete IX(obj); }
// FAISS_DECLARE_INDEX_DOWNCAST (c_api/macros_impl.h:93-100): dynamic_cast
FaissIndexFlat* faiss_IndexFlat_cast(FaissIndex* index) {
    return dynamic_cast<IndexFlat*>(IX(index)) ? index : nullptr;
}
FaissIndexFlatIP* faiss_IndexFlatIP_cast(FaissIndex* index) {
    auto f = dynamic_cast<IndexFlat*>(IX(index));
    return f && f->metric_type == faiss_amd::METRIC_INNER_PRODUCT ? index : nullptr;
}
FaissIndexFlatL2* faiss_IndexFlatL2_cast(FaissIndex* index) {
    auto f = dynamic_cast<IndexFlat*>(IX(index));
    return f && f->metric_type == faiss_amd::METRIC_L2 ? index : nullptr;
}
void faiss_IndexFlat_xb(FaissIndexFlat* index, float** p_xb, size_t* p_size) {
    auto f = dynamic_cast<IndexFlat*>(IX(index));
    if (!f) {
        *p_xb = nullptr;
        *p_size = 0;
        return;
    }
    *p_xb = f->xb.data();
    *p_size = f->xb.size();
}

// ---------------- IndexIVF (getters never throw: 0 / no-op on a wrong type)
static const IndexIVF* IVFc(const FaissIndexIVF* i) { return dynamic_cast<const IndexIVF*>(IX(i)); }
static IndexIVF* IVFm(FaissIndexIVF* i) { return dynamic_cast<IndexIVF*>(IX(i)); }
const char* faiss_amd_Index_type(const FaissIndex* i) {
    const Index* x = IX(i);
    if (dynamic_cast<const IndexShardsIVF*>(x)) return "IndexShardsIVF";
    if (dynamic_cast<const IndexIVFPQ*>(x)) return "IndexIVFPQ";
    if (dynamic_cast<const IndexIVFFlat*>(x)) return "IndexIVFFlat";
    if (dynamic_cast<const IndexHNSW*>(x)) return "IndexHNSWFlat";
    if (dynamic_cast<const IndexFlat*>(x)) return "IndexFlat";
    return "Index";
}
size_t faiss_IndexIVF_nlist(const FaissIndexIVF* i) {
    if (auto s = dynamic_cast<const IndexShardsIVF*>(IX(i))) return s->nlist;
    auto v = IVFc(i);
    return v ? v->nlist : 0;
}
size_t faiss_IndexIVF_nprobe(const FaissIndexIVF* i) {
    if (auto s = dynamic_cast<const IndexShardsIVF*>(IX(i))) return s->nprobe;
    auto v = IVFc(i);
    return v ? v->nprobe : 0;
}
void faiss_IndexIVF_set_nprobe(FaissIndexIVF* i, size_t v) {
    if (auto s = dynamic_cast<IndexShardsIVF*>(IX(i))) {
        s->nprobe = v;
        for (auto* sh : s->shards) sh->nprobe = v;
        return;
    }
    if (auto x = IVFm(i)) x->nprobe = v;
}
FaissIndex* faiss_IndexIVF_quantizer(const FaissIndexIVF* i) {
    if (auto s = dynamic_cast<const IndexShardsIVF*>(IX(i))) return FX(s->quantizer);
    auto v = IVFc(i);
    return v ? FX(v->quantizer) : nullptr;
}
int faiss_IndexIVF_own_fields(const FaissIndexIVF* i) {
    auto v = IVFc(i);
    return v && v->own_fields ? 1 : 0;
}
void faiss_IndexIVF_set_own_fields(FaissIndexIVF* i, int v) {
    if (auto x = IVFm(i)) x->own_fields = v != 0;
}

void faiss_IndexIVF_free(FaissIndexIVF* obj) { delete IX(obj); }
FaissIndexIVF* faiss_IndexIVF_cast(FaissIndex* index) {
    return dynamic_cast<IndexIVF*>(IX(index)) ? index : nullptr;
}
double faiss_IndexIVF_imbalance_factor(const FaissIndexIVF* index) {
    auto v = IVFc(index);
    if (!v) return 0.0;
    double tot = 0.0, uf = 0.0;
    for (size_t l = 0; l < v->nlist; l++) {
        const double sz = (double)v->get_list_size(l);
        tot += sz;
        uf += sz * sz;
    }
    return tot > 0 ? uf * (double)v->nlist / (tot * tot) : 0.0;
}

int faiss_IndexIVF_search_preassigned(const FaissIndexIVF* index, idx_t n, const float* x,
                                      idx_t k, const idx_t* assign, const float* centroid_dis,
                                      float* distances, idx_t* labels, int store_pairs) {
    C_TRY IVF(index)->search_preassigned(n, x, k, assign, centroid_dis, distances, labels,
                                         store_pairs != 0, nullptr);
    C_CATCH
}
size_t faiss_IndexIVF_get_list_size(const FaissIndexIVF* index, size_t list_no) {
    auto v = IVFc(index);
    return v && list_no < v->nlist ? v->get_list_size(list_no) : 0;
}
void faiss_IndexIVF_invlists_get_ids(const FaissIndexIVF* index, size_t list_no, idx_t* out) {
    auto v = IVFc(index);
    if (!v || list_no >= v->nlist) return;
    const size_t n = v->invlists->list_size(list_no);
    if (n) memcpy(out, v->invlists->get_ids(list_no), sizeof(idx_t) * n);
}
void faiss_amd_IndexIVF_invlists_get_codes(const FaissIndexIVF* index, size_t list_no,
                                           uint8_t* codes) {
    auto v = IVFc(index);
    if (!v || list_no >= v->nlist) return;
    const size_t n = v->invlists->list_size(list_no) * v->invlists->code_size;
    if (n) memcpy(codes, v->invlists->get_codes(list_no), n);
}
size_t faiss_amd_IndexIVF_code_size(const FaissIndexIVF* index) {
    auto v = IVFc(index);
    return v ? v->code_size : 0;
}

// IndexIVFStats is layout-identical to FaissIndexIVFStats (static_assert
// below), so the C struct aliases the global like the reference C API does
static_assert(sizeof(FaissIndexIVFStats) == sizeof(IndexIVFStats), "stats layout");
static_assert(sizeof(FaissQueryLatencyStats) == sizeof(QueryLatencyStats), "latency layout");
static_assert(sizeof(FaissHNSWStats) == sizeof(HNSWStats), "hnsw stats layout");
void faiss_IndexIVFStats_reset(FaissIndexIVFStats* stats) {
    reinterpret_cast<IndexIVFStats*>(stats)->reset();
}
FaissIndexIVFStats* faiss_get_indexIVF_stats(void) {
    return reinterpret_cast<FaissIndexIVFStats*>(&indexIVF_stats);
}

int faiss_amd_IndexIVF_search_stats(const FaissIndexIVF* index, idx_t n, const float* x,
                                    idx_t k, const FaissSearchParameters* params,
                                    float* distances, idx_t* labels,
                                    FaissQueryLatencyStats* per_query_stats) {
    C_TRY IVF(index)->search_stats(n, x, k, distances, labels, resolve_params(params),
                                   reinterpret_cast<QueryLatencyStats*>(per_query_stats));
    C_CATCH
}

int faiss_amd_IndexIVF_search_preassigned_stats(
        const FaissIndexIVF* index, idx_t n, const float* x, idx_t k, const idx_t* assign,
        const float* centroid_dis, float* distances, idx_t* labels, int store_pairs,
        const FaissSearchParameters* params, FaissIndexIVFStats* ivf_stats,
        FaissQueryLatencyStats* per_query_stats) {
    C_TRY const SearchParametersIVF* p = nullptr;
    if (params) {
        p = dynamic_cast<const SearchParametersIVF*>(resolve_params(params));
        FAISS_THROW_IF_NOT_MSG(p, "IndexIVF params have incorrect type");
    }
    IVF(index)->search_preassigned_stats(n, x, k, assign, centroid_dis, distances, labels,
                                         store_pairs != 0, p,
                                         reinterpret_cast<IndexIVFStats*>(ivf_stats),
                                         reinterpret_cast<QueryLatencyStats*>(per_query_stats));
    C_CATCH
}

// ---------------- IndexIVFFlat
int faiss_IndexIVFFlat_new_with(FaissIndexIVFFlat** p_index, FaissIndex* quantizer, size_t d,
                                size_t nlist) {
    C_TRY* p_index = FX(new IndexIVFFlat(IX(quantizer), d, nlist, faiss_amd::METRIC_L2));
    C_CATCH
}
int faiss_IndexIVFFlat_new_with_metric(FaissIndexIVFFlat** p_index, FaissIndex* quantizer,
                                       size_t d, size_t nlist, FaissMetricType metric) {
    C_TRY* p_index = FX(new IndexIVFFlat(IX(quantizer), d, nlist, (MetricType)metric));
    C_CATCH
}

// default construction (IndexIVFFlat_c.h:34): no vectors, no lists; the
// library's IndexIVF always has a quantizer, so it owns an empty IndexFlatL2
int faiss_IndexIVFFlat_new(FaissIndexIVFFlat** p_index) {
    C_TRY auto q = new IndexFlatL2(0);
    auto ix = new IndexIVFFlat(q, 0, 0, faiss_amd::METRIC_L2);
    ix->own_fields = true;
    *p_index = FX(ix);
    C_CATCH
}
void faiss_IndexIVFFlat_free(FaissIndexIVFFlat* obj) { delete IX(obj); }
FaissIndexIVFFlat* faiss_IndexIVFFlat_cast(FaissIndex* index) {
    return dynamic_cast<IndexIVFFlat*>(IX(index)) ? index : nullptr;
}
size_t faiss_IndexIVFFlat_nlist(const FaissIndexIVFFlat* i) { return faiss_IndexIVF_nlist(i); }
size_t faiss_IndexIVFFlat_nprobe(const FaissIndexIVFFlat* i) { return faiss_IndexIVF_nprobe(i); }
void faiss_IndexIVFFlat_set_nprobe(FaissIndexIVFFlat* i, size_t v) {
    faiss_IndexIVF_set_nprobe(i, v);
}
FaissIndex* faiss_IndexIVFFlat_quantizer(const FaissIndexIVFFlat* i) {
    return faiss_IndexIVF_quantizer(i);
}
int faiss_IndexIVFFlat_own_fields(const FaissIndexIVFFlat* i) { return faiss_IndexIVF_own_fields(i); }
void faiss_IndexIVFFlat_set_own_fields(FaissIndexIVFFlat* i, int v) {
    faiss_IndexIVF_set_own_fields(i, v);
}

// ---------------- IndexIVFPQ
int faiss_amd_IndexIVFPQ_new_with(FaissIndexIVFPQ** p_index, FaissIndex* quantizer, size_t d,
                                  size_t nlist, size_t M, size_t nbits, FaissMetricType metric) {
    C_TRY* p_index = FX(new IndexIVFPQ(IX(quantizer), d, nlist, M, nbits, (MetricType)metric));
    C_CATCH
}
void faiss_amd_IndexIVFPQ_pq_centroids(FaissIndexIVFPQ* index, float** p, size_t* n) {
    auto pq = dynamic_cast<IndexIVFPQ*>(IX(index));
    if (!pq) {
        *p = nullptr;
        *n = 0;
        return;
    }
    *p = pq->pq.centroids.data();
    *n = pq->pq.centroids.size();
}
int faiss_amd_IndexIVFPQ_info(const FaissIndexIVFPQ* index, size_t* M, size_t* nbits,
                              int* by_residual, int* use_precomputed_table) {
    C_TRY auto pq = dynamic_cast<const IndexIVFPQ*>(IX(index));
    FAISS_THROW_IF_NOT_MSG(pq, "not an IndexIVFPQ");
    *M = pq->pq.M;
    *nbits = pq->pq.nbits;
    *by_residual = pq->by_residual ? 1 : 0;
    *use_precomputed_table = pq->use_precomputed_table;
    C_CATCH
}
int faiss_amd_IndexIVFPQ_set_use_precomputed_table(FaissIndexIVFPQ* index, int v) {
    C_TRY auto pq = dynamic_cast<IndexIVFPQ*>(IX(index));
    FAISS_THROW_IF_NOT_MSG(pq, "not an IndexIVFPQ");
    FAISS_THROW_IF_NOT_MSG(v == 0 || (v == 1 && pq->by_residual && pq->metric_type == faiss_amd::METRIC_L2),
                           "use_precomputed_table: 0, or 1 for by-residual L2");
    pq->use_precomputed_table = v;
    C_CATCH
}

// ---------------- IndexHNSW
int faiss_amd_IndexHNSWFlat_new_with(FaissIndexHNSW** p_index, int d, int M,
                                     FaissMetricType metric) {
    C_TRY* p_index = FX(new IndexHNSWFlat(d, M, (MetricType)metric));
    C_CATCH
}
static IndexHNSW* HN(const FaissIndexHNSW* p) {
    auto h = dynamic_cast<IndexHNSW*>(const_cast<Index*>(IX(p)));
    FAISS_THROW_IF_NOT_MSG(h, "not an IndexHNSW");
    return h;
}
static IndexHNSW* HNnt(const FaissIndexHNSW* p) {
    return dynamic_cast<IndexHNSW*>(const_cast<Index*>(IX(p)));
}
int faiss_amd_IndexHNSW_efSearch(const FaissIndexHNSW* p) {
    auto h = HNnt(p);
    return h ? h->hnsw.efSearch : 0;
}
void faiss_amd_IndexHNSW_set_efSearch(FaissIndexHNSW* p, int v) {
    if (auto h = HNnt(p)) h->hnsw.efSearch = v;
}
int faiss_amd_IndexHNSW_efConstruction(const FaissIndexHNSW* p) {
    auto h = HNnt(p);
    return h ? h->hnsw.efConstruction : 0;
}
void faiss_amd_IndexHNSW_set_efConstruction(FaissIndexHNSW* p, int v) {
    if (auto h = HNnt(p)) h->hnsw.efConstruction = v;
}
FaissIndex* faiss_amd_IndexHNSW_storage(const FaissIndexHNSW* p) {
    auto h = HNnt(p);
    return h ? FX(h->storage) : nullptr;
}
int faiss_amd_IndexHNSW_search_stats(const FaissIndexHNSW* p, idx_t n, const float* x, idx_t k,
                                     const FaissSearchParameters* params, float* distances,
                                     idx_t* labels, FaissQueryLatencyStats* per_query_stats) {
    C_TRY auto h = HNnt(p);
    FAISS_THROW_IF_NOT_MSG(h, "index is not an IndexHNSW");
    // the efSearch set with faiss_amd_SearchParametersIVF_set_quantizer_efSearch
    const SearchParameters* sp = nullptr;
    if (params) {
        auto c = reinterpret_cast<const SearchParamsC*>(params);
        if (c->ivf.quantizer_params) sp = &c->hnsw;
    }
    h->search_stats(n, x, k, distances, labels, sp,
                    reinterpret_cast<QueryLatencyStats*>(per_query_stats));
    C_CATCH
}
FaissHNSWStats* faiss_amd_get_hnsw_stats(void) {
    return reinterpret_cast<FaissHNSWStats*>(&hnsw_stats);
}
void faiss_amd_HNSWStats_reset(void) {
    hnsw_stats.reset();
    hnsw_row_stats = HNSWRowStats();
}
void faiss_amd_get_hnsw_row_stats(uint64_t* fp32_rows, uint64_t* q8_rows) {
    if (fp32_rows) *fp32_rows = hnsw_row_stats.fp32_rows;
    if (q8_rows) *q8_rows = hnsw_row_stats.q8_rows;
}
void faiss_amd_get_hnsw_replay_stats(uint64_t* replayed, uint64_t* searched_again,
                                     uint64_t* replay_bad) {
    if (replayed) *replayed = hnsw_row_stats.replayed;
    if (searched_again) *searched_again = hnsw_row_stats.searched_again;
    if (replay_bad) *replay_bad = hnsw_row_stats.replay_bad;
}
void faiss_amd_set_interrupt_timeout(double seconds) {
    if (seconds < 0) InterruptCallback::clear_instance();
    else TimeoutCallback::reset(seconds);
}
int faiss_amd_fold_device_stats(const FaissIndex* index) {
    C_TRY auto ix = IX(index);
    ix->fold_device_stats();
    if (auto v = dynamic_cast<const IndexIVF*>(ix)) v->quantizer->fold_device_stats();
    C_CATCH
}
int faiss_amd_IndexHNSW_graph(const FaissIndexHNSW* p, int* entry_point, int* max_level,
                              size_t* n_neighbors, size_t* n_cum, const int32_t** levels,
                              const size_t** offsets, const int32_t** neighbors,
                              const int32_t** cum) {
    C_TRY auto h = HN(p);
    *entry_point = h->hnsw.entry_point;
    *max_level = h->hnsw.max_level;
    *n_neighbors = h->hnsw.neighbors.size();
    *n_cum = h->hnsw.cum_nneighbor_per_level.size();
    if (levels) *levels = h->hnsw.levels.data();
    if (offsets) *offsets = h->hnsw.offsets.data();
    if (neighbors) *neighbors = h->hnsw.neighbors.data();
    if (cum) *cum = h->hnsw.cum_nneighbor_per_level.data();
    C_CATCH
}

// ---------------- shards
int faiss_amd_IndexShardsIVF_new(FaissIndexShardsIVF** p_index, FaissIndex* quantizer,
                                 size_t nlist, int threaded, int successive_ids) {
    C_TRY* p_index =
            FX(new IndexShardsIVF(IX(quantizer), nlist, threaded != 0, successive_ids != 0));
    C_CATCH
}
int faiss_amd_IndexShardsIVF_add_shard(FaissIndexShardsIVF* index, FaissIndex* shard) {
    C_TRY auto s = dynamic_cast<IndexShardsIVF*>(IX(index));
    FAISS_THROW_IF_NOT_MSG(s, "not an IndexShardsIVF");
    auto iv = dynamic_cast<IndexIVF*>(IX(shard));
    FAISS_THROW_IF_NOT_MSG(iv, "shard is not an IndexIVF");
    s->add_shard(iv);
    C_CATCH
}
int faiss_amd_IndexShardsIVF_count(const FaissIndexShardsIVF* index) {
    auto s = dynamic_cast<const IndexShardsIVF*>(IX(index));
    return s ? (int)s->shards.size() : 0;
}
int faiss_amd_IndexShardsIVF_shard(const FaissIndexShardsIVF* index, int i, FaissIndex** p_shard) {
    C_TRY auto s = dynamic_cast<const IndexShardsIVF*>(IX(index));
    FAISS_THROW_IF_NOT_MSG(s, "not an IndexShardsIVF");
    FAISS_THROW_IF_NOT(i >= 0 && i < (int)s->shards.size());
    *p_shard = FX(s->shards[i]);
    C_CATCH
}
int faiss_amd_IndexIVF_copy_subset_to(const FaissIndex* src, FaissIndex* dst, int subset_type,
                                      idx_t a1, idx_t a2, size_t* n_added) {
    C_TRY auto a = dynamic_cast<const IndexIVF*>(IX(src));
    auto b = dynamic_cast<IndexIVF*>(IX(dst));
    FAISS_THROW_IF_NOT_MSG(a && b, "copy_subset_to: both indexes must be IndexIVF");
    const size_t n = ivf_copy_subset_to(a, b, subset_type, a1, a2);
    if (n_added) *n_added = n;
    C_CATCH
}
int faiss_amd_index_ivf_to_shards(const FaissIndex* src, int nshard, int shard_type,
                                  const int* devices, FaissIndexShardsIVF** p_index) {
    C_TRY auto a = dynamic_cast<const IndexIVF*>(IX(src));
    FAISS_THROW_IF_NOT_MSG(a, "index_ivf_to_shards: not an IndexIVF");
    *p_index = FX(index_ivf_to_shards(a, nshard, shard_type, devices));
    C_CATCH
}

// ---------------- range search
static RangeSearchResult* RSR(FaissRangeSearchResult* p) {
    return reinterpret_cast<RangeSearchResult*>(p);
}
int faiss_RangeSearchResult_new(FaissRangeSearchResult** p_rsr, idx_t nq) {
    C_TRY FAISS_THROW_IF_NOT(nq >= 0);
    *p_rsr = reinterpret_cast<FaissRangeSearchResult*>(new RangeSearchResult((size_t)nq));
    C_CATCH
}
void faiss_RangeSearchResult_free(FaissRangeSearchResult* obj) { delete RSR(obj); }
size_t faiss_RangeSearchResult_nq(const FaissRangeSearchResult* rsr) {
    return reinterpret_cast<const RangeSearchResult*>(rsr)->nq;
}
size_t faiss_RangeSearchResult_buffer_size(const FaissRangeSearchResult* rsr) {
    return reinterpret_cast<const RangeSearchResult*>(rsr)->buffer_size();
}
void faiss_RangeSearchResult_lims(FaissRangeSearchResult* rsr, size_t** lims) {
    *lims = RSR(rsr)->lims.data();
}
void faiss_RangeSearchResult_labels(FaissRangeSearchResult* rsr, idx_t** labels,
                                    float** distances) {
    *labels = RSR(rsr)->labels.data();
    *distances = RSR(rsr)->distances.data();
}
int faiss_Index_range_search(const FaissIndex* index, idx_t n, const float* x, float radius,
                             FaissRangeSearchResult* result) {
    C_TRY IX(index)->range_search(n, x, radius, RSR(result), nullptr);
    C_CATCH
}
int faiss_amd_Index_range_search_with_params(const FaissIndex* index, idx_t n, const float* x,
                                             float radius, const FaissSearchParameters* params,
                                             FaissRangeSearchResult* result) {
    C_TRY IX(index)->range_search(n, x, radius, RSR(result), resolve_params(params));
    C_CATCH
}
int faiss_IndexIVF_range_search_preassigned(const FaissIndexIVF* index, idx_t n,
                                            const float* x, float radius, const idx_t* assign,
                                            const float* centroid_dis,
                                            FaissRangeSearchResult* result) {
    C_TRY auto v = IVFc(index);
    FAISS_THROW_IF_NOT_MSG(v, "index is not an IndexIVF");
    v->range_search_preassigned(n, x, radius, assign, centroid_dis, RSR(result));
    C_CATCH
}

// ---------------- I/O
int faiss_write_index(const FaissIndex* idx, FILE* f) {
    C_TRY write_index(IX(idx), f);
    C_CATCH
}
int faiss_write_index_fname(const FaissIndex* idx, const char* fname) {
    C_TRY write_index(IX(idx), fname);
    C_CATCH
}
int faiss_amd_write_index_ondisk(const FaissIndex* idx, const char* fname,
                                 const char* lists_fname) {
    C_TRY write_index_ondisk(IX(idx), fname, lists_fname);
    C_CATCH
}
int faiss_read_index(FILE* f, int io_flags, FaissIndex** p_out) {
    C_TRY* p_out = FX(read_index(f, io_flags));
    C_CATCH
}
int faiss_read_index_fname(const char* fname, int io_flags, FaissIndex** p_out) {
    C_TRY* p_out = FX(read_index(fname, io_flags));
    C_CATCH
}
// faiss/clone_index.cpp (Cloner::clone_Index): a deep copy.  Every index
// type of this library round-trips its on-disk form byte for byte, so the
// copy goes through it (an anonymous temporary file)
int faiss_clone_index(const FaissIndex* idx, FaissIndex** p_out) {
    C_TRY FILE* f = tmpfile();
    FAISS_THROW_IF_NOT_MSG(f, "clone_index: no temporary file");
    std::unique_ptr<FILE, int (*)(FILE*)> guard(f, fclose);
    write_index(IX(idx), f);
    FAISS_THROW_IF_NOT(fflush(f) == 0);
    rewind(f);
    *p_out = FX(read_index(f, 0));
    C_CATCH
}

// ---------------- factory / parameter space
int faiss_index_factory(FaissIndex** p_index, int d, const char* description,
                        FaissMetricType metric) {
    C_TRY* p_index = FX(index_factory(d, description, (MetricType)metric));
    C_CATCH
}
struct FaissParameterSpace_H {
    int dummy;
};
int faiss_ParameterSpace_new(FaissParameterSpace** space) {
    C_TRY* space = new FaissParameterSpace_H();
    C_CATCH
}
void faiss_ParameterSpace_free(FaissParameterSpace* space) { delete space; }
int faiss_ParameterSpace_set_index_parameter(const FaissParameterSpace*, FaissIndex* index,
                                             const char* name, double val) {
    // faiss/AutoTune.cpp:468-557 subset
    C_TRY std::string n(name);
    Index* ix = IX(index);
    if (n == "nprobe") {
        if (auto s = dynamic_cast<IndexShardsIVF*>(ix)) {
            s->nprobe = (size_t)val;
            for (auto* sh : s->shards) sh->nprobe = (size_t)val;
        } else {
            IVF(index)->nprobe = (size_t)val;
        }
    } else if (n == "efSearch") {
        auto h = dynamic_cast<IndexHNSW*>(ix);
        FAISS_THROW_IF_NOT_MSG(h, "efSearch needs an IndexHNSW");
        h->hnsw.efSearch = (int)val;
    } else if (n == "quantizer_efSearch") {
        Index* q = nullptr;
        if (auto s = dynamic_cast<IndexShardsIVF*>(ix)) q = s->quantizer;
        else q = IVF(index)->quantizer;
        auto h = dynamic_cast<IndexHNSW*>(q);
        FAISS_THROW_IF_NOT_MSG(h, "quantizer is not an IndexHNSW");
        h->hnsw.efSearch = (int)val;
    } else if (n == "max_codes") {
        // faiss/AutoTune.cpp:530-535
        const size_t mc = std::isfinite(val) ? (size_t)val : 0;
        if (auto s = dynamic_cast<IndexShardsIVF*>(ix)) {
            for (auto* sh : s->shards) sh->max_codes = mc;
        } else {
            IVF(index)->max_codes = mc;
        }
    } else {
        FAISS_THROW_MSG("ParameterSpace::set_index_parameter: unknown parameter " + n);
    }
    C_CATCH
}

// ---------------- merge
int faiss_amd_merge_knn_results(size_t n, size_t k, int nshard, const float* all_d,
                                const idx_t* all_l, float* d, idx_t* l, FaissMetricType metric) {
    C_TRY merge_knn_results(n, k, nshard, all_d, all_l, d, l, (MetricType)metric);
    C_CATCH
}

// ---------------- device extensions
int faiss_amd_device_count(int* count) {
    C_TRY int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    C_CATCH
}
int faiss_amd_set_device(int device) {
    C_TRY ensure_hip();
    set_current_device(device);
    C_CATCH
}
int faiss_amd_Index_sync_device(FaissIndex* index) {
    C_TRY ensure_hip();
    int prev = 0;
    HIP_CHECK(hipGetDevice(&prev));
    HIP_CHECK(hipSetDevice(IX(index)->device));
    IX(index)->sync_device();
    HIP_CHECK(hipSetDevice(prev));
    C_CATCH
}

static hipStream_t pick_stream(const Index* ix, void* stream) {
    return stream ? (hipStream_t)stream : ix->stream();
}

static int ldx_of(const Index* ix) { return (int)roundup((size_t)ix->d, 4); }

int faiss_amd_Index_search_device(const FaissIndex* index, idx_t n, const float* x_dev, idx_t k,
                                  float* d_dev, idx_t* l_dev, void* stream) {
    C_TRY const Index* ix = IX(index);
    FAISS_THROW_IF_NOT_MSG(ix->d % 4 == 0, "device entry points need d % 4 == 0");
    ensure_hip();
    ix->sync_device();
    ix->search_device(n, x_dev, ldx_of(ix), k, d_dev, l_dev, nullptr, pick_stream(ix, stream));
    C_CATCH
}
int faiss_amd_IndexIVF_search_preassigned_device(const FaissIndexIVF* index, idx_t n,
                                                 const float* x_dev, idx_t k, int nprobe,
                                                 const int32_t* assign_dev,
                                                 const float* cdis_dev, float* d_dev,
                                                 idx_t* l_dev, void* stream) {
    C_TRY const IndexIVF* ix = IVF(index);
    FAISS_THROW_IF_NOT_MSG(ix->d % 4 == 0, "device entry points need d % 4 == 0");
    FAISS_THROW_IF_NOT(nprobe > 0 && (size_t)nprobe <= ix->nlist);
    ensure_hip();
    ix->sync_device();
    ix->search_preassigned_device_ordered(n, x_dev, ldx_of(ix), k, nprobe, assign_dev, cdis_dev,
                                          d_dev, l_dev, pick_stream(ix, stream));
    C_CATCH
}
int faiss_amd_IndexIVF_quantize_device(const FaissIndexIVF* index, idx_t n, const float* x_dev,
                                       int nprobe, float* cdis_dev, int32_t* assign_dev,
                                       void* stream) {
    C_TRY const IndexIVF* ix = IVF(index);
    FAISS_THROW_IF_NOT_MSG(ix->d % 4 == 0, "device entry points need d % 4 == 0");
    ensure_hip();
    ix->sync_device();
    ix->quantize_device(n, x_dev, ldx_of(ix), nprobe, cdis_dev, assign_dev, nullptr,
                        pick_stream(ix, stream));
    C_CATCH
}
int faiss_amd_merge_knn_results_device(size_t n, size_t k, int nshard, const float* all_d,
                                       const idx_t* all_l, float* d, idx_t* l,
                                       FaissMetricType metric, void* stream) {
    C_TRY ensure_hip();
    FAISS_THROW_IF_NOT(nshard > 0 && nshard < 32768 && k >= 1 &&
                       k <= (size_t)kern::kMaxKExact);
    kern::merge_rows(all_d, all_l, (int64_t)n, (nshard << 16) | (int)k, (int)k,
                     metric == ::METRIC_L2, d, l, (hipStream_t)stream);
    C_CATCH
}
int faiss_amd_set_search_slices(int t) {
    C_TRY set_search_slices(t);
    C_CATCH
}
int faiss_amd_set_kernel_timing(int enable) {
    C_TRY set_kernel_timing_enabled(enable != 0);
    C_CATCH
}
int faiss_amd_set_kernel_timing_filter(const char* name) {
    C_TRY set_kernel_timing_filter(name);
    C_CATCH
}
namespace {
// KernelTimes::resolve, leaving no HIP error behind: a pair whose events
// never completed a record (a failed launch) reads NaN, and the error its
// query returned is cleared rather than left for the caller's next check
void resolve_times(KernelTimes* t) {
    for (; t->resolved < t->e0.size(); t->resolved++) {
        float ms = 0;
        hipError_t e = hipEventSynchronize(t->e1[t->resolved]);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, t->e0[t->resolved], t->e1[t->resolved]);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            ms = std::numeric_limits<float>::quiet_NaN();
        }
        t->millis.push_back(ms);
    }
}
}  // namespace

int faiss_amd_last_kernel_times(const FaissIndex* index, int* n_kernels, char* names,
                                double* millis, double* units) {
    C_TRY const Index* ix = IX(index);
    std::vector<KernelTimes*> all{&ix->ktimes};
    if (auto ivf = dynamic_cast<const IndexIVF*>(ix)) all.push_back(&ivf->quantizer->ktimes);
    if (auto sh = dynamic_cast<const IndexShardsIVF*>(ix)) {
        all.push_back(&sh->quantizer->ktimes);
        for (auto* s : sh->shards) all.push_back(&s->ktimes);
    }
    int cnt = 0;
    for (auto t : all) {
        resolve_times(t);
        cnt += (int)t->names.size();
    }
    if (names && millis) {
        int i = 0;
        for (auto t : all)
            for (size_t j = 0; j < t->names.size() && i < *n_kernels; j++, i++) {
                strncpy(names + 32 * i, t->names[j].c_str(), 31);
                names[32 * i + 31] = 0;
                millis[i] = t->millis[j];
                if (units) units[i] = t->units[j];
            }
    }
    *n_kernels = cnt;
    C_CATCH
}
int faiss_amd_IndexIVF_debug_rows(const FaissIndex* index, int what, int64_t row0, int64_t n,
                                  void* out, size_t* row_bytes, int64_t* rows) {
    C_TRY IVF(index)->debug_rows(what, row0, n, out, row_bytes, rows);
    C_CATCH
}

int faiss_amd_reset_kernel_times(FaissIndex* index) {
    C_TRY Index* ix = IX(index);
    ix->ktimes.clear();
    if (auto ivf = dynamic_cast<IndexIVF*>(ix)) ivf->quantizer->ktimes.clear();
    if (auto sh = dynamic_cast<IndexShardsIVF*>(ix)) {
        sh->quantizer->ktimes.clear();
        for (auto* s : sh->shards) s->ktimes.clear();
    }
    C_CATCH
}
int faiss_amd_float_rand(float* x, size_t n, int64_t seed) {
    C_TRY float_rand(x, n, seed);
    C_CATCH
}
int faiss_amd_float_rand_rows(float* out, int64_t n_rows, int d, int64_t seed, int64_t row0,
                              int64_t step, int64_t nout) {
    C_TRY float_rand_rows(out, n_rows, d, seed, row0, step, nout);
    C_CATCH
}

}  // extern "C"
