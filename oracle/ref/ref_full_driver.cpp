// ref_full_driver.cpp — C entry points over the reference's CPU library
// (oracle/ref/Makefile `full`: the FAISS_SRC list compiled in place from
// /root/reference, MKL as BLAS).  TEST INFRASTRUCTURE ONLY: generates the
// reference-run fixtures under tests/golden (reference-written index files and
// the D/I of reference searches over them) and is the `cpu_baseline` of
// bench.py (kind "reference").  Never linked into the product.
//
// Every entry point is a thin call into the reference's own classes:
//   faiss::index_factory / read_index / write_index (faiss/index_factory.cpp,
//   faiss/impl/index_read.cpp, faiss/impl/index_write.cpp),
//   Index::train / add / search, IndexIVF::search_preassigned,
//   IndexIVF::range_search, IndexIVF::encode_vectors, quantizer->search,
//   merge_knn_results.
#include <faiss/IndexFlat.h>
#include <faiss/IndexHNSW.h>
#include <faiss/IndexIVF.h>
#include <faiss/IndexIVFFlat.h>
#include <faiss/IndexIVFPQ.h>
#include <faiss/impl/AuxIndexStructures.h>
#include <faiss/impl/HNSW.h>
#include <faiss/impl/IDSelector.h>
#include <faiss/index_factory.h>
#include <faiss/index_io.h>
#include <faiss/utils/distances.h>

#include <omp.h>

#include <cstdint>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

using faiss::idx_t;

namespace faiss {
extern size_t precomputed_table_max_bytes;
}

namespace {
thread_local std::string g_err;

template <class F>
int guarded(F&& f) {
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

faiss::IndexIVF* ivf_of(void* h) {
    auto* ivf = dynamic_cast<faiss::IndexIVF*>((faiss::Index*)h);
    if (!ivf) throw std::runtime_error("not an IndexIVF");
    return ivf;
}
}  // namespace

extern "C" {

const char* reff_last_error() { return g_err.c_str(); }

void reff_set_threads(int nt) { omp_set_num_threads(nt); }

void* reff_index_factory(int d, const char* desc, int metric_l2) {
    faiss::Index* r = nullptr;
    guarded([&] {
        r = faiss::index_factory(d, desc,
                                 metric_l2 ? faiss::METRIC_L2 : faiss::METRIC_INNER_PRODUCT);
    });
    return r;
}

void* reff_read_index(const char* fname, int io_flags) {
    faiss::Index* r = nullptr;
    guarded([&] { r = faiss::read_index(fname, io_flags); });
    return r;
}

int reff_write_index(void* h, const char* fname) {
    return guarded([&] { faiss::write_index((faiss::Index*)h, fname); });
}

void reff_free(void* h) { delete (faiss::Index*)h; }

int reff_train(void* h, int64_t n, const float* x) {
    return guarded([&] { ((faiss::Index*)h)->train(n, x); });
}

int reff_add(void* h, int64_t n, const float* x, const int64_t* ids) {
    return guarded([&] {
        if (ids)
            ((faiss::Index*)h)->add_with_ids(n, x, ids);
        else
            ((faiss::Index*)h)->add(n, x);
    });
}

// out: d, ntotal, metric(1=L2), nlist, nprobe, code_size, pq_M, pq_nbits,
//      by_residual, use_precomputed_table
int reff_info(void* h, int64_t* out) {
    return guarded([&] {
        auto* idx = (faiss::Index*)h;
        for (int i = 0; i < 10; i++) out[i] = -1;
        out[0] = idx->d;
        out[1] = idx->ntotal;
        out[2] = idx->metric_type == faiss::METRIC_L2;
        if (auto* ivf = dynamic_cast<faiss::IndexIVF*>(idx)) {
            out[3] = ivf->nlist;
            out[4] = ivf->nprobe;
            out[5] = ivf->code_size;
            out[8] = ivf->by_residual;
        }
        if (auto* pq = dynamic_cast<faiss::IndexIVFPQ*>(idx)) {
            out[6] = pq->pq.M;
            out[7] = pq->pq.nbits;
            out[9] = pq->use_precomputed_table;
        }
    });
}

int reff_set_nprobe(void* h, int64_t nprobe) {
    return guarded([&] { ivf_of(h)->nprobe = nprobe; });
}

int reff_set_parallel_mode(void* h, int pmode) {
    return guarded([&] { ivf_of(h)->parallel_mode = pmode; });
}

int reff_set_quantizer_efsearch(void* h, int ef) {
    return guarded([&] {
        auto* q = dynamic_cast<faiss::IndexHNSW*>(ivf_of(h)->quantizer);
        if (!q) throw std::runtime_error("quantizer is not HNSW");
        q->hnsw.efSearch = ef;
    });
}

int reff_set_hnsw_efsearch(void* h, int ef) {
    return guarded([&] {
        auto* q = dynamic_cast<faiss::IndexHNSW*>((faiss::Index*)h);
        if (!q) throw std::runtime_error("not an IndexHNSW");
        q->hnsw.efSearch = ef;
    });
}

// faiss::precomputed_table_max_bytes (faiss/IndexIVFPQ.cpp:332)
void reff_set_precomputed_table_max_bytes(uint64_t b) { faiss::precomputed_table_max_bytes = b; }

// use_precomputed_table := t, then IndexIVFPQ::precompute_table()
int reff_ivfpq_set_table(void* h, int t) {
    return guarded([&] {
        auto* pq = dynamic_cast<faiss::IndexIVFPQ*>((faiss::Index*)h);
        if (!pq) throw std::runtime_error("not an IndexIVFPQ");
        pq->use_precomputed_table = t;
        pq->precompute_table();
    });
}

int reff_search(void* h, int64_t n, const float* x, int64_t k, float* D, int64_t* I) {
    return guarded([&] { ((faiss::Index*)h)->search(n, x, k, D, I); });
}

int reff_search_params(void* h, int64_t n, const float* x, int64_t k, int64_t nprobe,
                       int64_t max_codes, const int64_t* sel_ids, int64_t nsel, float* D,
                       int64_t* I) {
    return guarded([&] {
        faiss::SearchParametersIVF sp;
        sp.nprobe = nprobe;
        sp.max_codes = max_codes;
        faiss::IDSelectorBatch* sel = nullptr;
        if (sel_ids) sp.sel = sel = new faiss::IDSelectorBatch(nsel, sel_ids);
        ((faiss::Index*)h)->search(n, x, k, D, I, &sp);
        delete sel;
    });
}

int reff_quantizer_search(void* h, int64_t n, const float* x, int64_t nprobe, float* Dq,
                          int64_t* Iq) {
    return guarded([&] { ivf_of(h)->quantizer->search(n, x, nprobe, Dq, Iq); });
}

int reff_search_preassigned(void* h, int64_t n, const float* x, int64_t k, int64_t nprobe,
                            const int64_t* keys, const float* cdis, int store_pairs, float* D,
                            int64_t* I) {
    return guarded([&] {
        faiss::SearchParametersIVF sp;
        sp.nprobe = nprobe;
        ivf_of(h)->search_preassigned(n, x, k, keys, cdis, D, I, store_pairs != 0, &sp);
    });
}

// Range search: returns a handle to a RangeSearchResult; reff_range_copy
// copies lims[n+1], D/I[lims[n]] out and frees it.
void* reff_range_search(void* h, int64_t n, const float* x, float radius, int64_t nprobe) {
    faiss::RangeSearchResult* r = nullptr;
    guarded([&] {
        faiss::SearchParametersIVF sp;
        sp.nprobe = nprobe;
        r = new faiss::RangeSearchResult(n);
        ((faiss::Index*)h)->range_search(n, x, radius, r, &sp);
    });
    return r;
}
int64_t reff_range_total(void* r) {
    auto* rr = (faiss::RangeSearchResult*)r;
    return (int64_t)rr->lims[rr->nq];
}
void reff_range_copy(void* r, int64_t* lims, float* D, int64_t* I) {
    auto* rr = (faiss::RangeSearchResult*)r;
    for (size_t i = 0; i <= rr->nq; i++) lims[i] = (int64_t)rr->lims[i];
    const size_t tot = rr->lims[rr->nq];
    if (tot) {
        memcpy(D, rr->distances, sizeof(float) * tot);
        for (size_t i = 0; i < tot; i++) I[i] = rr->labels[i];
    }
    delete rr;
}

// Add-path pieces: coarse assignment (quantizer->assign) and the list codes
// (IndexIVF::encode_vectors without list numbers).
int reff_assign(void* h, int64_t n, const float* x, int64_t* list_nos) {
    return guarded([&] { ivf_of(h)->quantizer->assign(n, x, list_nos); });
}
int reff_encode_vectors(void* h, int64_t n, const float* x, const int64_t* list_nos,
                        uint8_t* codes) {
    return guarded([&] { ivf_of(h)->encode_vectors(n, x, list_nos, codes, false); });
}

int64_t reff_list_size(void* h, int64_t l) { return ivf_of(h)->invlists->list_size(l); }
int reff_list_copy(void* h, int64_t l, uint8_t* codes, int64_t* ids) {
    return guarded([&] {
        auto* il = ivf_of(h)->invlists;
        const size_t n = il->list_size(l);
        faiss::InvertedLists::ScopedCodes c(il, l);
        faiss::InvertedLists::ScopedIds i(il, l);
        memcpy(codes, c.get(), n * il->code_size);
        memcpy(ids, i.get(), n * sizeof(idx_t));
    });
}

}  // extern "C"
