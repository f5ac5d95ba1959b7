// ref_driver.cpp — C entry points over reference sources compiled in place
// (oracle/ref/Makefile builds faiss/utils/random.cpp, faiss/utils/Heap.cpp,
// faiss/utils/distances_simd.cpp, faiss/impl/HNSW.cpp and their small
// dependencies straight from /root/reference with the reference's own AVX2
// flags).  TEST INFRASTRUCTURE ONLY: used to generate tests/golden fixtures
// and to pin oracle/oracle.c; never linked into the product.
//
// Only loops that live in reference files which cannot be built here (they
// pull in BLAS: IndexIVF.cpp / IndexIVFFlat.cpp / distances.cpp) are
// restated below, and they restate them with the reference's own heap and
// distance primitives:
//   * the IVF-Flat scan loop, faiss/IndexIVFFlat.cpp:155-179 (scan_codes)
//     driven by faiss/IndexIVF.cpp:595-631 (probe order, skip key < 0);
//   * the direct coarse search used for slices below the BLAS threshold,
//     faiss/utils/distances.cpp:170-199 (exhaustive_L2sqr_seq).
#include <faiss/impl/AuxIndexStructures.h>
#include <faiss/impl/DistanceComputer.h>
#include <faiss/impl/HNSW.h>
#include <faiss/impl/ResultHandler.h>
#include <faiss/utils/Heap.h>
#include <faiss/utils/distances.h>
#include <faiss/utils/random.h>

#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

using faiss::idx_t;

extern "C" {

void ref_float_rand(float* x, size_t n, int64_t seed) { faiss::float_rand(x, n, seed); }

// out[i] = fvec_L2sqr / fvec_inner_product(x, y + i*d, d)
void ref_fvec_batch(const float* x, const float* y, size_t d, size_t ny, int metric_l2,
                    float* out) {
    for (size_t i = 0; i < ny; i++)
        out[i] = metric_l2 ? faiss::fvec_L2sqr(x, y + i * d, d)
                           : faiss::fvec_inner_product(x, y + i * d, d);
}

void ref_fvec_norms(const float* x, size_t d, size_t n, float* out) {
    for (size_t i = 0; i < n; i++) out[i] = faiss::fvec_norm_L2sqr(x + i * d, d);
}

// out[i] for 4 rows at a time through fvec_L2sqr_batch_4 (the HNSW
// DistanceComputer path, faiss/IndexFlat.cpp:143-170); ny % 4 == 0
void ref_fvec_batch4(const float* x, const float* y, size_t d, size_t ny, float* out) {
    for (size_t i = 0; i + 4 <= ny; i += 4)
        faiss::fvec_L2sqr_batch_4(x, y + i * d, y + (i + 1) * d, y + (i + 2) * d,
                                  y + (i + 3) * d, d, out[i], out[i + 1], out[i + 2],
                                  out[i + 3]);
}

// Stream (dis[i], ids[i]) in order through the reference's result heap with
// the IVF scanner's admission test; D/I [k] sorted like heap_reorder.
void ref_heap_stream(const float* dis, const int64_t* ids, size_t n, size_t k, int metric_l2,
                     float* D, int64_t* I) {
    if (metric_l2) {
        using C = faiss::CMax<float, idx_t>;
        faiss::heap_heapify<C>(k, D, I);
        for (size_t i = 0; i < n; i++)
            if (C::cmp(D[0], dis[i])) faiss::heap_replace_top<C>(k, D, I, dis[i], ids[i]);
        faiss::heap_reorder<C>(k, D, I);
    } else {
        using C = faiss::CMin<float, idx_t>;
        faiss::heap_heapify<C>(k, D, I);
        for (size_t i = 0; i < n; i++)
            if (C::cmp(D[0], dis[i])) faiss::heap_replace_top<C>(k, D, I, dis[i], ids[i]);
        faiss::heap_reorder<C>(k, D, I);
    }
}

// Direct coarse search (slice below the BLAS threshold): top-k of
// fvec_L2sqr / fvec_inner_product over ny rows.
void ref_knn_direct(const float* x, size_t nx, const float* y, size_t ny, size_t d, size_t k,
                    int metric_l2, float* D, int64_t* I) {
    std::vector<float> dis(ny);
    std::vector<int64_t> ids(ny);
    for (size_t j = 0; j < ny; j++) ids[j] = (int64_t)j;
    for (size_t i = 0; i < nx; i++) {
        ref_fvec_batch(x + i * d, y, d, ny, metric_l2, dis.data());
        ref_heap_stream(dis.data(), ids.data(), ny, k, metric_l2, D + i * k, I + i * k);
    }
}

// IVF-Flat search_preassigned for one query: lists in probe order.
//   codes: all vectors [ntotal][d]; list_off/list_len index them; ids per row
void ref_ivf_flat_query(const float* x, size_t d, const float* codes, const int64_t* ids,
                        const int64_t* list_off, const int64_t* list_len, const int64_t* assign,
                        size_t nprobe, size_t k, int metric_l2, float* D, int64_t* I) {
    std::vector<float> dis;
    std::vector<int64_t> cid;
    for (size_t r = 0; r < nprobe; r++) {
        const int64_t key = assign[r];
        if (key < 0) continue;
        const int64_t n = list_len[key];
        for (int64_t j = 0; j < n; j++) {
            const int64_t row = list_off[key] + j;
            dis.push_back(metric_l2 ? faiss::fvec_L2sqr(x, codes + row * d, d)
                                    : faiss::fvec_inner_product(x, codes + row * d, d));
            cid.push_back(ids[row]);
        }
    }
    ref_heap_stream(dis.data(), cid.data(), dis.size(), k, metric_l2, D, I);
}

// merge_knn_results<int64_t, CMin/CMax<float,int>> (faiss/utils/Heap.cpp:159-230)
void ref_merge_knn_results(size_t n, size_t k, int nshard, const float* all_D,
                           const int64_t* all_I, float* D, int64_t* I, int metric_l2) {
    if (metric_l2)
        faiss::merge_knn_results<idx_t, faiss::CMin<float, int>>(n, k, nshard, all_D, all_I, D,
                                                                 I);
    else
        faiss::merge_knn_results<idx_t, faiss::CMax<float, int>>(n, k, nshard, all_D, all_I, D,
                                                                 I);
}

// HNSW::search (faiss/impl/HNSW.cpp:943-996) on a flat L2 storage; the
// distance computer mirrors IndexFlat's FlatL2Dis (faiss/IndexFlat.cpp:111-170).
struct FlatL2Dis : faiss::DistanceComputer {
    const float* xb;
    size_t d;
    const float* q = nullptr;
    FlatL2Dis(const float* xb, size_t d) : xb(xb), d(d) {}
    void set_query(const float* x) override { q = x; }
    float operator()(idx_t i) override { return faiss::fvec_L2sqr(q, xb + i * d, d); }
    float symmetric_dis(idx_t i, idx_t j) override {
        return faiss::fvec_L2sqr(xb + j * d, xb + i * d, d);
    }
    void distances_batch_4(const idx_t i0, const idx_t i1, const idx_t i2, const idx_t i3,
                           float& d0, float& d1, float& d2, float& d3) override {
        float a = 0, b = 0, c = 0, e = 0;
        faiss::fvec_L2sqr_batch_4(q, xb + i0 * d, xb + i1 * d, xb + i2 * d, xb + i3 * d, d, a,
                                  b, c, e);
        d0 = a;
        d1 = b;
        d2 = c;
        d3 = e;
    }
};

void ref_hnsw_search(const float* xb, size_t nb, size_t d, const int32_t* levels,
                     const uint64_t* offsets, size_t n_offsets, const int32_t* neighbors,
                     size_t n_neighbors, const int32_t* cum_nneighbor_per_level,
                     size_t n_cum, int32_t entry_point, int32_t max_level, int ef_search,
                     const float* xq, size_t nq, size_t k, float* D, int64_t* I,
                     uint64_t* stats /* n1, n2, ndis, nhops summed (HNSWStats), or NULL */) {
    faiss::HNSW h;
    h.levels.assign(levels, levels + nb);
    h.offsets.assign(offsets, offsets + n_offsets);
    h.neighbors.resize(n_neighbors);
    memcpy(h.neighbors.data(), neighbors, sizeof(int32_t) * n_neighbors);
    h.cum_nneighbor_per_level.assign(cum_nneighbor_per_level, cum_nneighbor_per_level + n_cum);
    h.entry_point = entry_point;
    h.max_level = max_level;
    h.efSearch = ef_search;
    FlatL2Dis dis(xb, d);
    faiss::VisitedTable vt(nb);
    faiss::HeapBlockResultHandler<faiss::HNSW::C> bres(nq, D, I, k);
    faiss::HeapBlockResultHandler<faiss::HNSW::C>::SingleResultHandler res(bres);
    faiss::HNSWStats tot;
    for (size_t i = 0; i < nq; i++) {
        res.begin(i);
        dis.set_query(xq + i * d);
        tot.combine(h.search(dis, res, vt, nullptr));
        res.end();
        vt.advance();
    }
    if (stats) {
        stats[0] = tot.n1;
        stats[1] = tot.n2;
        stats[2] = tot.ndis;
        stats[3] = tot.nhops;
    }
}

// ---- HNSW graph construction: faiss/IndexHNSW.cpp:68-230 (hnsw_add_vertices)
// restated serially (the reference runs a level in parallel above 100
// vertices, which makes its graph thread-schedule dependent; with one thread
// it is this loop) over the reference's HNSW::prepare_level_tab and
// HNSW::add_with_locks.
void* ref_hnsw_build(const float* xb, size_t n, size_t d, int M, int ef_construction) {
    faiss::HNSW* h = new faiss::HNSW(M);
    h->efConstruction = ef_construction;
    if (n == 0) return h;
    h->prepare_level_tab(n, false);
    std::vector<omp_lock_t> locks(n);
    for (size_t i = 0; i < n; i++) omp_init_lock(&locks[i]);
    std::vector<int> hist, order(n);
    for (size_t i = 0; i < n; i++) {
        const int lv = h->levels[i] - 1;
        while (lv >= (int)hist.size()) hist.push_back(0);
        hist[lv]++;
    }
    std::vector<int> offs(hist.size() + 1, 0);
    for (size_t i = 0; i + 1 < hist.size(); i++) offs[i + 1] = offs[i] + hist[i];
    for (size_t i = 0; i < n; i++) order[offs[h->levels[i] - 1]++] = (int)i;
    faiss::RandomGenerator rng2(789);
    FlatL2Dis dis(xb, d);
    int i1 = (int)n;
    for (int lv = (int)hist.size() - 1; lv >= 0; lv--) {
        const int i0 = i1 - hist[lv];
        for (int j = i0; j < i1; j++) std::swap(order[j], order[j + rng2.rand_int(i1 - j)]);
        faiss::VisitedTable vt(n);
        for (int i = i0; i < i1; i++) {
            const int pt = order[i];
            dis.set_query(xb + (size_t)pt * d);
            h->add_with_locks(dis, lv, pt, locks, vt, false);
        }
        i1 = i0;
    }
    for (size_t i = 0; i < n; i++) omp_destroy_lock(&locks[i]);
    return h;
}

void ref_hnsw_sizes(void* hp, int64_t* out /* n, n_offsets, n_neighbors, n_cum, entry, max_level */) {
    const faiss::HNSW* h = (const faiss::HNSW*)hp;
    out[0] = (int64_t)h->levels.size();
    out[1] = (int64_t)h->offsets.size();
    out[2] = (int64_t)h->neighbors.size();
    out[3] = (int64_t)h->cum_nneighbor_per_level.size();
    out[4] = h->entry_point;
    out[5] = h->max_level;
}

void ref_hnsw_copy(void* hp, int32_t* levels, uint64_t* offsets, int32_t* neighbors,
                   int32_t* cum, double* probas, int64_t n_probas) {
    const faiss::HNSW* h = (const faiss::HNSW*)hp;
    std::copy(h->levels.begin(), h->levels.end(), levels);
    for (size_t i = 0; i < h->offsets.size(); i++) offsets[i] = h->offsets[i];
    std::copy(h->neighbors.begin(), h->neighbors.end(), neighbors);
    std::copy(h->cum_nneighbor_per_level.begin(), h->cum_nneighbor_per_level.end(), cum);
    for (int64_t i = 0; i < n_probas && i < (int64_t)h->assign_probas.size(); i++)
        probas[i] = h->assign_probas[i];
}

void ref_hnsw_free(void* hp) { delete (faiss::HNSW*)hp; }

}  // extern "C"
