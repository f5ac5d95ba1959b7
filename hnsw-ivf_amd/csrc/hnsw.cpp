// hnsw.cpp — HNSW graph (host build) and IndexHNSW(Flat) with GPU search.
//
// Graph construction restates faiss/impl/HNSW.cpp (set_default_probas :62-75,
// random_level :51-60, prepare_level_tab :210-235, shrink_neighbor_list
// :237-270, add_link :300-335, search_neighbors_to_add :340-490,
// add_links_starting_from :492-527, add_with_locks :533-575) and the vertex
// ordering of faiss/IndexHNSW.cpp:68-230 (hnsw_add_vertices), run serially so
// the graph is deterministic.  It is index building, not the search path; the
// search runs on the GPU (kernels_hnsw.hip).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <queue>

#include "../../include/faiss_amd.h"
#include "kernels.h"

namespace faiss_amd {

namespace {
struct DevGuard2 {
    int prev = 0;
    explicit DevGuard2(int dev) {
        ensure_hip();
        HIP_CHECK(hipGetDevice(&prev));
        if (prev != dev) HIP_CHECK(hipSetDevice(dev));
    }
    ~DevGuard2() {
        int cur = 0;
        hipGetDevice(&cur);
        if (cur != prev) hipSetDevice(prev);
    }
};

// fvec_L2sqr in the reference's evaluation order (see ref_arith.h: 8 fma
// lanes, (j,j+4),(j,j+2),(0,1) reduction, 4-term epilogue, fma tail)
inline float l2_seq(const float* a, const float* b, int d) {
    float c[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int n8 = d & ~7;
    for (int i = 0; i < n8; i += 8)
        for (int j = 0; j < 8; j++) {
            const float t = a[i + j] - b[i + j];
            c[j] = std::fma(t, t, c[j]);
        }
    const float x0 = c[0] + c[4], x1 = c[1] + c[5], x2 = c[2] + c[6], x3 = c[3] + c[7];
    float r = (x0 + x2) + (x1 + x3);
    int i = n8;
    if (d - n8 >= 4) {
        float e[4];
        for (int j = 0; j < 4; j++) {
            const float t = a[n8 + j] - b[n8 + j];
            e[j] = t * t;
        }
        r = r + ((e[0] + e[2]) + (e[1] + e[3]));
        i += 4;
    }
    for (; i < d; i++) {
        const float t = a[i] - b[i];
        r = std::fma(t, t, r);
    }
    return r;
}

struct NodeDistCloser {  // faiss/impl/HNSW.h NodeDistCloser
    float d;
    int id;
    NodeDistCloser(float d_, int i) : d(d_), id(i) {}
    bool operator<(const NodeDistCloser& o) const { return d < o.d; }
};
struct NodeDistFarther {
    float d;
    int id;
    NodeDistFarther(float d_, int i) : d(d_), id(i) {}
    bool operator<(const NodeDistFarther& o) const { return d > o.d; }
};

struct Builder {
    HNSW& h;
    const float* xb;
    int d;
    std::vector<uint8_t> visited;
    Builder(HNSW& h_, const float* xb_, int d_, size_t n) : h(h_), xb(xb_), d(d_), visited(n, 0) {}
    float dis(const float* q, int id) const { return l2_seq(q, xb + (size_t)id * d, d); }
    float sym(int a, int b) const { return l2_seq(xb + (size_t)a * d, xb + (size_t)b * d, d); }

    void greedy(const float* q, int level, int& nearest, float& d_nearest) {
        for (;;) {
            int prev = nearest;
            size_t b, e;
            h.neighbor_range(nearest, level, &b, &e);
            for (size_t j = b; j < e; j++) {
                int v = h.neighbors[j];
                if (v < 0) break;
                float dv = dis(q, v);
                if (dv < d_nearest) {
                    nearest = v;
                    d_nearest = dv;
                }
            }
            if (nearest == prev) return;
        }
    }

    void shrink(std::priority_queue<NodeDistFarther>& input, std::vector<NodeDistFarther>& output,
                int max_size) {
        while (!input.empty()) {
            NodeDistFarther v1 = input.top();
            input.pop();
            bool good = true;
            for (const auto& v2 : output) {
                if (sym(v2.id, v1.id) < v1.d) {
                    good = false;
                    break;
                }
            }
            if (good) {
                output.push_back(v1);
                if ((int)output.size() >= max_size) return;
            }
        }
    }
    void shrink_closer(std::priority_queue<NodeDistCloser>& rs1, int max_size) {
        if ((int)rs1.size() < max_size) return;
        std::priority_queue<NodeDistFarther> rs;
        std::vector<NodeDistFarther> ret;
        while (!rs1.empty()) {
            rs.emplace(rs1.top().d, rs1.top().id);
            rs1.pop();
        }
        shrink(rs, ret, max_size);
        for (const auto& c : ret) rs1.emplace(c.d, c.id);
    }
    void add_link(int src, int dest, int level) {
        size_t b, e;
        h.neighbor_range(src, level, &b, &e);
        if (h.neighbors[e - 1] == -1) {
            size_t i = e;
            while (i > b) {
                if (h.neighbors[i - 1] != -1) break;
                i--;
            }
            h.neighbors[i] = dest;
            return;
        }
        std::priority_queue<NodeDistCloser> rs;
        rs.emplace(sym(src, dest), dest);
        for (size_t i = b; i < e; i++) {
            int ng = h.neighbors[i];
            rs.emplace(sym(src, ng), ng);
        }
        shrink_closer(rs, (int)(e - b));
        size_t i = b;
        while (!rs.empty()) {
            h.neighbors[i++] = rs.top().id;
            rs.pop();
        }
        while (i < e) h.neighbors[i++] = -1;
    }
    void search_to_add(const float* q, std::priority_queue<NodeDistCloser>& results, int entry,
                       float d_entry, int level) {
        std::priority_queue<NodeDistFarther> cand;
        cand.emplace(d_entry, entry);
        results.emplace(d_entry, entry);
        std::vector<int> touched;
        visited[entry] = 1;
        touched.push_back(entry);
        while (!cand.empty()) {
            const NodeDistFarther cur = cand.top();
            if (cur.d > results.top().d) break;
            cand.pop();
            size_t b, e;
            h.neighbor_range(cur.id, level, &b, &e);
            for (size_t j = b; j < e; j++) {
                int v = h.neighbors[j];
                if (v < 0) break;
                if (visited[v]) continue;
                visited[v] = 1;
                touched.push_back(v);
                float dv = dis(q, v);
                if ((int)results.size() < h.efConstruction || results.top().d > dv) {
                    results.emplace(dv, v);
                    cand.emplace(dv, v);
                    if ((int)results.size() > h.efConstruction) results.pop();
                }
            }
        }
        for (int v : touched) visited[v] = 0;
    }
    void add_links_from(const float* q, int pt, int nearest, float d_nearest, int level) {
        std::priority_queue<NodeDistCloser> targets;
        search_to_add(q, targets, nearest, d_nearest, level);
        shrink_closer(targets, h.nb_neighbors(level));
        std::vector<int> to_add;
        while (!targets.empty()) {
            int other = targets.top().id;
            add_link(pt, other, level);
            to_add.push_back(other);
            targets.pop();
        }
        for (int other : to_add) add_link(other, pt, level);
    }
    void add_point(int pt, int pt_level) {
        const float* q = xb + (size_t)pt * d;
        int nearest = h.entry_point;
        if (nearest == -1) {
            h.max_level = pt_level;
            h.entry_point = pt;
            return;
        }
        int level = h.max_level;
        float d_nearest = dis(q, nearest);
        for (; level > pt_level; level--) greedy(q, level, nearest, d_nearest);
        for (; level >= 0; level--) add_links_from(q, pt, nearest, d_nearest, level);
        if (pt_level > h.max_level) {
            h.max_level = pt_level;
            h.entry_point = pt;
        }
    }
};
}  // namespace

// ---------------------------------------------------------------- HNSW
HNSW::HNSW(int M) {
    set_default_probas(M, 1.0f / logf((float)M));
    offsets.push_back(0);
}
void HNSW::set_default_probas(int M, float levelMult) {
    int nn = 0;
    cum_nneighbor_per_level.push_back(0);
    for (int level = 0;; level++) {
        float proba = expf(-level / levelMult) * (1 - expf(-1 / levelMult));
        if (proba < 1e-9) break;
        assign_probas.push_back(proba);
        nn += level == 0 ? M * 2 : M;
        cum_nneighbor_per_level.push_back(nn);
    }
}
int HNSW::nb_neighbors(int l) const {
    return cum_nneighbor_per_level[l + 1] - cum_nneighbor_per_level[l];
}
int HNSW::cum_nb_neighbors(int l) const { return cum_nneighbor_per_level[l]; }
void HNSW::neighbor_range(idx_t no, int l, size_t* b, size_t* e) const {
    size_t o = offsets[no];
    *b = o + cum_nb_neighbors(l);
    *e = o + cum_nb_neighbors(l + 1);
}
int HNSW::random_level(std::mt19937& rng) const {
    double f = rng() / float(std::mt19937::max());
    for (int level = 0; level < (int)assign_probas.size(); level++) {
        if (f < assign_probas[level]) return level;
        f -= assign_probas[level];
    }
    return (int)assign_probas.size() - 1;
}

// ---------------------------------------------------------------- IndexHNSW
IndexHNSW::IndexHNSW(IndexFlat* st, int M)
        : Index(st ? st->d : 0, st ? st->metric_type : METRIC_L2), hnsw(M), storage(st) {
    is_trained = true;
    if (st) device = st->device;
}
IndexHNSW::~IndexHNSW() {
    if (side_) (void)hipStreamSynchronize(side_);
    if (ev_split_) (void)hipEventDestroy(ev_split_);
    if (ev_exact_) (void)hipEventDestroy(ev_exact_);
    if (side_) (void)hipStreamDestroy(side_);
    if (h_fcnt_) (void)hipHostFree(h_fcnt_);
    if (own_fields) delete storage;
}
IndexHNSWFlat::IndexHNSWFlat(int d_, int M, MetricType metric)
        : IndexHNSW(new IndexFlat(d_, metric), M) {
    own_fields = true;
    FAISS_THROW_IF_NOT_MSG(metric == METRIC_L2, "HNSW inner product not supported on GPU");
}

void IndexHNSW::add(idx_t n, const float* x) {
    // faiss/IndexHNSW.cpp:386-397 + hnsw_add_vertices (:68-230)
    FAISS_THROW_IF_NOT_MSG(storage, "Please use IndexHNSWFlat (or variants)");
    const idx_t n0 = ntotal;
    storage->add(n, x);
    ntotal = storage->ntotal;
    if (n == 0) return;
    // prepare_level_tab
    std::mt19937 rng(12345);
    for (idx_t i = 0; i < (idx_t)hnsw.levels.size(); i++) rng();  // keep stream position
    int max_level2 = 0;
    for (idx_t i = 0; i < n; i++) {
        int pl = hnsw.random_level(rng);
        hnsw.levels.push_back(pl + 1);
    }
    for (idx_t i = 0; i < n; i++) {
        int pl = hnsw.levels[n0 + i] - 1;
        max_level2 = std::max(max_level2, pl);
        hnsw.offsets.push_back(hnsw.offsets.back() + hnsw.cum_nb_neighbors(pl + 1));
    }
    hnsw.neighbors.resize(hnsw.offsets.back(), -1);
    // order: by level, highest first, shuffled within a level (rng2 = 789)
    std::vector<int> hist;
    std::vector<int> order(n);
    for (idx_t i = 0; i < n; i++) {
        int pl = hnsw.levels[n0 + i] - 1;
        while (pl >= (int)hist.size()) hist.push_back(0);
        hist[pl]++;
    }
    std::vector<int> offs(hist.size() + 1, 0);
    for (size_t i = 0; i + 1 < hist.size(); i++) offs[i + 1] = offs[i] + hist[i];
    for (idx_t i = 0; i < n; i++) {
        int pl = hnsw.levels[n0 + i] - 1;
        order[offs[pl]++] = (int)(n0 + i);
    }
    std::mt19937 rng2(789);
    Builder bld(hnsw, storage->xb.data(), d, ntotal);
    int i1 = (int)n;
    for (int pl = (int)hist.size() - 1; pl >= 0; pl--) {
        int i0 = i1 - hist[pl];
        for (int j = i0; j < i1; j++) std::swap(order[j], order[j + rng2() % (i1 - j)]);
        for (int j = i0; j < i1; j++) bld.add_point(order[j], hnsw.levels[order[j]] - 1);
        i1 = i0;
    }
    version_++;
    std::lock_guard<std::recursive_mutex> g(mu_);
    dirty_ = true;
}

void IndexHNSW::reset() {
    hnsw = HNSW((int)(hnsw.cum_nneighbor_per_level.size() > 1 ? hnsw.nb_neighbors(1) : 32));
    storage->reset();
    ntotal = 0;
    version_++;
    std::lock_guard<std::recursive_mutex> g(mu_);
    dirty_ = true;
}

void IndexHNSW::reconstruct(idx_t key, float* recons) const { storage->reconstruct(key, recons); }

void IndexHNSW::sync_device() const {
    storage->sync_device();
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (!dirty_) return;
    DevGuard2 dg(device);
    hipStream_t s = stream();
    FAISS_THROW_IF_NOT_MSG(hnsw.nb_neighbors(0) <= 64 &&
                                   (hnsw.cum_nneighbor_per_level.size() < 3 ||
                                    hnsw.nb_neighbors(1) <= 64),
                           "HNSW M > 32 not supported on this path");
    const size_t nl = std::max<size_t>(hnsw.levels.size(), 1);
    d_levels_.reserve(sizeof(int32_t) * nl);
    d_offsets_.reserve(sizeof(uint64_t) * (nl + 1));
    d_neighbors_.reserve(sizeof(int32_t) * std::max<size_t>(hnsw.neighbors.size(), 1));
    d_cum_.reserve(sizeof(int32_t) * hnsw.cum_nneighbor_per_level.size() + 8);
    std::vector<uint64_t> offs(hnsw.offsets.begin(), hnsw.offsets.end());
    if (!hnsw.levels.empty())
        HIP_CHECK(hipMemcpyAsync(d_levels_.ptr, hnsw.levels.data(),
                                 sizeof(int32_t) * hnsw.levels.size(), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_offsets_.ptr, offs.data(), sizeof(uint64_t) * offs.size(),
                             hipMemcpyHostToDevice, s));
    if (!hnsw.neighbors.empty())
        HIP_CHECK(hipMemcpyAsync(d_neighbors_.ptr, hnsw.neighbors.data(),
                                 sizeof(int32_t) * hnsw.neighbors.size(), hipMemcpyHostToDevice,
                                 s));
    HIP_CHECK(hipMemcpyAsync(d_cum_.ptr, hnsw.cum_nneighbor_per_level.data(),
                             sizeof(int32_t) * hnsw.cum_nneighbor_per_level.size(),
                             hipMemcpyHostToDevice, s));
    // regular level-0 table [ntotal][nb_neighbors(0)] (a copy of each node's
    // level-0 slice): the level-0 hop then loads its neighbour ids without
    // first loading offsets[v].  Kept when it costs at most 1 GiB of HBM.
    std::vector<int32_t> nb0;
    const size_t c0 = hnsw.cum_nneighbor_per_level.size() >= 2 ? (size_t)hnsw.nb_neighbors(0) : 0;
    nb0_stride_ = 0;
    if (c0 > 0 && !hnsw.levels.empty() &&
        hnsw.levels.size() * c0 * sizeof(int32_t) <= ((size_t)1 << 30)) {
        const size_t nn = hnsw.levels.size();
        const size_t b0 = (size_t)hnsw.cum_nneighbor_per_level[0];
        nb0.resize(nn * c0);
        for (size_t v = 0; v < nn; v++)
            memcpy(&nb0[v * c0], &hnsw.neighbors[hnsw.offsets[v] + b0], c0 * sizeof(int32_t));
        d_nb0_.reserve(sizeof(int32_t) * nb0.size());
        HIP_CHECK(hipMemcpyAsync(d_nb0_.ptr, nb0.data(), sizeof(int32_t) * nb0.size(),
                                 hipMemcpyHostToDevice, s));
        nb0_stride_ = (int)c0;
    }
    // int8 row image for the register kernel's level-0 prefilter: per row
    // y, o = min y, s = (max y - min y) / 255, q = round((y - o) / s), and
    // with yq = s q + o (exact real): ey >= |y - yq|, B2 = |yq|^2, Q1 = sum q.
    // A fresh neighbour whose certified lower bound on its distance
    // (kernels_hnsw.hip q8_filter) reaches both heaps' bounds cannot enter
    // either, so only the others' fp32 rows are read.  FAISS_AMD_HNSW_Q8=0: off.
    std::vector<uint8_t> q8;
    std::vector<float> q8p, q8q1;
    const char* q8env = getenv("FAISS_AMD_HNSW_Q8");
    q8_ = metric_type == METRIC_L2 && d <= 128 && nb0_stride_ > 0 && ntotal > 0 &&
          !(q8env && !strcmp(q8env, "0"));
    if (q8_) {
        const size_t nn = (size_t)ntotal;
        q8.assign(nn * 128, 0);
        q8p.assign(nn * 4, 0.f);
        q8q1.assign(nn, 0.f);
        const float* xb = storage->xb.data();
        for (size_t v = 0; v < nn; v++) {
            const float* y = xb + v * d;
            float mn = y[0], mx = y[0];
            for (int i = 1; i < d; i++) {
                mn = std::min(mn, y[i]);
                mx = std::max(mx, y[i]);
            }
            float sc = (float)(((double)mx - (double)mn) / 255.0);
            if (!(sc > 0.f) || !std::isfinite(sc)) sc = 1.f;
            double e2 = 0, b2 = 0, q1 = 0;
            for (int i = 0; i < d; i++) {
                const double t = std::nearbyint(((double)y[i] - (double)mn) / (double)sc);
                const int q = (int)std::min(255.0, std::max(0.0, t));
                const double yq = (double)sc * q + (double)mn;
                e2 += ((double)y[i] - yq) * ((double)y[i] - yq);
                b2 += yq * yq;
                q1 += q;
                q8[v * 128 + i] = (uint8_t)q;
            }
            // ey rounded up (fp32 above the double value)
            const double ey = std::sqrt(e2) * (1.0 + 1e-9) + 1e-12 * std::sqrt(b2) + 1e-30;
            float eyf = (float)ey;
            if ((double)eyf < ey) eyf = std::nextafter(eyf, INFINITY);
            q8p[v * 4 + 0] = mn;
            q8p[v * 4 + 1] = sc;
            q8p[v * 4 + 2] = eyf;
            q8p[v * 4 + 3] = (float)b2;
            q8q1[v] = (float)q1;
        }
        d_q8_.reserve(q8.size());
        d_q8p_.reserve(sizeof(float) * q8p.size());
        d_q8q1_.reserve(sizeof(float) * q8q1.size());
        HIP_CHECK(hipMemcpyAsync(d_q8_.ptr, q8.data(), q8.size(), hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(d_q8p_.ptr, q8p.data(), sizeof(float) * q8p.size(),
                                 hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(d_q8q1_.ptr, q8q1.data(), sizeof(float) * q8q1.size(),
                                 hipMemcpyHostToDevice, s));
    }
    HIP_CHECK(hipStreamSynchronize(s));
    dirty_ = false;
}

template <class OutIdx>
void IndexHNSW::hnsw_device(idx_t n, const float* x, int ldx, int k, float* distances,
                            OutIdx* labels, const SearchParameters* params, hipStream_t s,
                            bool defer) const {
    // faiss/IndexHNSW.cpp:246-343 (hnsw_search)
    FAISS_THROW_IF_NOT(k > 0);
    int efSearch = hnsw.efSearch;
    if (params) {
        auto p = dynamic_cast<const SearchParametersHNSW*>(params);
        FAISS_THROW_IF_NOT_MSG(p, "params type invalid");
        efSearch = p->efSearch;
    }
    sync_device();
    std::lock_guard<std::recursive_mutex> g(mu_);
    order_.enter(s);
    kern::HNSWDevice gd;
    gd.storage = storage->device_vectors();
    gd.norms = nullptr;
    gd.ld = ld();
    gd.d = d;
    gd.levels = d_levels_.as<int32_t>();
    gd.offsets = d_offsets_.as<uint64_t>();
    gd.neighbors = d_neighbors_.as<int32_t>();
    gd.cum_nb = d_cum_.as<int32_t>();
    gd.nb0 = nb0_stride_ > 0 ? d_nb0_.as<int32_t>() : nullptr;
    gd.nb0_stride = nb0_stride_;
    gd.q8 = q8_ ? d_q8_.as<uint8_t>() : nullptr;
    gd.q8p = q8_ ? d_q8p_.as<float>() : nullptr;
    gd.q8q1 = q8_ ? d_q8q1_.as<float>() : nullptr;
    gd.nlevels_cum = (int)hnsw.cum_nneighbor_per_level.size();
    gd.entry_point = ntotal > 0 ? hnsw.entry_point : -1;
    gd.max_level = hnsw.max_level;
    gd.ntotal = (int)ntotal;
    const int64_t vwords = (int64_t)cdiv(std::max<idx_t>(ntotal, 1), 32);
    constexpr bool i32 = sizeof(OutIdx) == 4;
    split_.active = false;
    if (!d_stats_.ptr) {
        d_stats_.reserve(kern::kHnswStatsWords * sizeof(unsigned long long));
        HIP_CHECK(hipMemsetAsync(d_stats_.ptr, 0, kern::kHnswStatsWords * sizeof(unsigned long long),
                                 s));
    }
    // queries per launch: the per-query visited bitmaps that do not fit in
    // LDS, and heaps beyond it (max(efSearch, k) in the thousands), live in
    // scratch kept under 256 MiB each (chunks of the batch)
    const size_t hw = kern::hnsw_heap_scratch_words(k, efSearch, ld());
    const bool scratch = kern::hnsw_visited_scratch_needed(ld(), k, efSearch, vwords);
    idx_t qc = n;
    if (scratch)
        qc = std::min<idx_t>(qc, std::max<idx_t>(1, (idx_t)(((size_t)256 << 20) /
                                                            ((size_t)vwords * 4))));
    if (hw) qc = std::min<idx_t>(qc, std::max<idx_t>(1, (idx_t)(((size_t)256 << 20) / (hw * 4))));
    // the register kernel's replay logs (kHnswReplayCap entries per query)
    // (FAISS_AMD_HNSW_REPLAY=0: none; such queries search level 0 again — A/B)
    const char* renv = getenv("FAISS_AMD_HNSW_REPLAY");
    const bool rlog = kern::hnsw_register_eligible(k, efSearch) &&
                      !kern::hnsw_uses_batched(k, efSearch) && !(renv && !strcmp(renv, "0"));
    // FAISS_AMD_HNSW_REPLAY_CAP=<entries>: a smaller log per query (tests: the
    // overflow path)
    int64_t rcap = kern::kHnswReplayCap;
    if (const char* cenv = getenv("FAISS_AMD_HNSW_REPLAY_CAP"))
        rcap = std::max<int64_t>(1, std::min<int64_t>(atoll(cenv), kern::kHnswReplayCap));
    if (rlog)
        qc = std::min<idx_t>(qc, (idx_t)(((size_t)256 << 20) / (8 * kern::kHnswReplayCap)));
    qc = std::max<idx_t>(qc, 1);
    if (rlog) s_rlog_.reserve(8 * (size_t)kern::kHnswReplayCap * qc);
    if (scratch) s_visited_.reserve(sizeof(uint32_t) * vwords * qc);
    if (hw) s_heaps_.reserve(sizeof(float) * hw * qc);
    // the sequential kernel's arrival logs (k_hnsw_exact without the result
    // heap) for the queries it serves: every query past the batched / wide
    // kernels' range, else their flagged ones (a pool; the rest keep the heap)
    const size_t alb = kern::hnsw_arrival_log_bytes(qc, ntotal);
    s_alog_.reserve(alb);
    s_flags_.reserve(sizeof(uint32_t) * std::max<idx_t>(qc, 1));
    // defer (split_begin): one chunk, the batched kernel in use
    defer = defer && !scratch && !hw && i32 && kern::hnsw_uses_batched(k, efSearch);
    for (idx_t q0 = 0; q0 < n; q0 += qc) {
        const idx_t nq = std::min(qc, n - q0);
        kern::hnsw_search(gd, x + q0 * ldx, ldx, nq, k, efSearch, distances + q0 * k,
                          i32 ? nullptr : (int64_t*)labels + q0 * k,
                          i32 ? (int32_t*)labels + q0 * k : nullptr, s_visited_.as<uint32_t>(),
                          vwords, d_stats_.as<unsigned long long>(), s_flags_.as<uint32_t>(), s,
                          &ktimes, defer, hw ? s_heaps_.as<float>() : nullptr,
                          rlog ? s_rlog_.as<uint64_t>() : nullptr, rlog ? rcap : 0, s_alog_.ptr,
                          alb);
    }
    if (!defer) {
        order_.leave(s);
        return;
    }
    // the flagged queries -> compact list, count read back (pinned)
    if (!h_fcnt_) HIP_CHECK(hipHostMalloc((void**)&h_fcnt_, sizeof(uint32_t), hipHostMallocDefault));
    if (!ev_split_) HIP_CHECK(hipEventCreateWithFlags(&ev_split_, hipEventDisableTiming));
    s_fidx_.reserve(sizeof(uint32_t) * std::max<idx_t>(n, 1));
    s_fcnt_.reserve(sizeof(uint32_t));
    kern::hnsw_flag_compact(s_flags_.as<uint32_t>(), n, s_fidx_.as<uint32_t>(),
                            s_fcnt_.as<uint32_t>(), s);
    HIP_CHECK(hipMemcpyAsync(h_fcnt_, s_fcnt_.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipEventRecord(ev_split_, s));
    split_.active = true;
    split_.n = n;
    split_.x = x;
    split_.ldx = ldx;
    split_.k = k;
    split_.efSearch = efSearch;
    split_.s = s;
}

bool IndexHNSW::split_begin(idx_t n, const float* x, int ldx, int k, float* distances,
                            int32_t* labels, const SearchParameters* params,
                            hipStream_t s) const {
    DevGuard2 dg(device);
    mu_.lock();  // held until split_release when a split is returned
    try {
        hnsw_device<int32_t>(n, x, ldx, k, distances, labels, params, s, true);
    } catch (...) {
        split_.active = false;
        mu_.unlock();
        throw;
    }
    if (!split_.active) mu_.unlock();
    return split_.active;
}

void IndexHNSW::split_release() const {
    // the caller's stream has joined the re-runs (split_finish's `done`) and
    // queued its last read of the split scratch
    order_.leave(split_.s);
    split_.active = false;
    mu_.unlock();
}

IndexHNSW::Split IndexHNSW::split_finish() const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    FAISS_THROW_IF_NOT_MSG(split_.active, "split_finish without split_begin");
    DevGuard2 dg(device);
    HIP_CHECK(hipEventSynchronize(ev_split_));
    Split r;
    r.nf = (idx_t)*h_fcnt_;
    if (r.nf == 0) return r;
    if (!side_) HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    if (!ev_exact_) HIP_CHECK(hipEventCreateWithFlags(&ev_exact_, hipEventDisableTiming));
    const int k = split_.k;
    s_fD_.reserve(sizeof(float) * r.nf * k);
    s_fI_.reserve(sizeof(int32_t) * r.nf * k);
    kern::HNSWDevice gd;
    gd.storage = storage->device_vectors();
    gd.norms = nullptr;
    gd.ld = ld();
    gd.d = d;
    gd.levels = d_levels_.as<int32_t>();
    gd.offsets = d_offsets_.as<uint64_t>();
    gd.neighbors = d_neighbors_.as<int32_t>();
    gd.cum_nb = d_cum_.as<int32_t>();
    gd.nb0 = nb0_stride_ > 0 ? d_nb0_.as<int32_t>() : nullptr;
    gd.nb0_stride = nb0_stride_;
    gd.q8 = q8_ ? d_q8_.as<uint8_t>() : nullptr;
    gd.q8p = q8_ ? d_q8p_.as<float>() : nullptr;
    gd.q8q1 = q8_ ? d_q8q1_.as<float>() : nullptr;
    gd.nlevels_cum = (int)hnsw.cum_nneighbor_per_level.size();
    gd.entry_point = ntotal > 0 ? hnsw.entry_point : -1;
    gd.max_level = hnsw.max_level;
    gd.ntotal = (int)ntotal;
    const int64_t vwords = (int64_t)cdiv(std::max<idx_t>(ntotal, 1), 32);
    HIP_CHECK(hipStreamWaitEvent(side_, ev_split_, 0));
    {
        ScopedKernelTimer tm(&ktimes, "hnsw_exact", 0.0, side_);
        const size_t alb = kern::hnsw_arrival_log_bytes(r.nf, ntotal);
        s_alog_.reserve(alb);
        kern::hnsw_exact_listed(gd, split_.x, split_.ldx, s_fidx_.as<uint32_t>(), r.nf, k,
                                split_.efSearch, s_fD_.as<float>(), s_fI_.as<int32_t>(),
                                nullptr, vwords, d_stats_.as<unsigned long long>(), side_,
                                s_alog_.ptr, alb);
    }
    HIP_CHECK(hipEventRecord(ev_exact_, side_));
    r.idx = s_fidx_.as<uint32_t>();
    r.D = s_fD_.as<float>();
    r.I = s_fI_.as<int32_t>();
    r.done = ev_exact_;
    return r;
}

// HNSWStats counted by the kernel -> the host global (faiss::hnsw_stats)
void IndexHNSW::fold_device_stats() const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (!d_stats_.ptr) return;
    DevGuard2 dg(device);
    hipStream_t s = stream();
    unsigned long long st[kern::kHnswStatsWords];
    HIP_CHECK(hipMemcpyAsync(st, d_stats_.ptr, sizeof(st), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemsetAsync(d_stats_.ptr, 0, sizeof(st), s));
    HIP_CHECK(hipStreamSynchronize(s));
    HNSWStats add;
    add.n1 = st[0];
    add.n2 = st[1];
    add.ndis = st[2];
    add.nhops = st[3];
    hnsw_stats.combine(add);
    hnsw_row_stats.fp32_rows += st[4];
    hnsw_row_stats.q8_rows += st[5];
    hnsw_row_stats.replayed += st[6];
    hnsw_row_stats.searched_again += st[7];
    hnsw_row_stats.replay_bad += st[8];
}

void IndexHNSW::search_stats(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                             const SearchParameters* params,
                             QueryLatencyStats* per_query_stats) const {
    // faiss/IndexHNSW.cpp:345-366 + hnsw_search (:246-343)
    FAISS_THROW_IF_NOT(k > 0);
    if (per_query_stats) memset(per_query_stats, 0, sizeof(QueryLatencyStats) * n);
    if (n == 0) return;
    DevGuard2 dg(device);
    sync_device();
    hipStream_t s = stream();
    const int ldx = ld();
    DeviceBuffer bx, bd, bi;
    bx.reserve(sizeof(float) * n * ldx);
    bd.reserve(sizeof(float) * n * k);
    bi.reserve(sizeof(idx_t) * n * k);
    if (ldx != d) HIP_CHECK(hipMemsetAsync(bx.ptr, 0, sizeof(float) * n * ldx, s));
    HIP_CHECK(hipMemcpy2DAsync(bx.ptr, sizeof(float) * ldx, x, sizeof(float) * d,
                               sizeof(float) * d, n, hipMemcpyHostToDevice, s));
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipEventRecord(e0, s));
    hnsw_device<idx_t>(n, bx.as<float>(), ldx, (int)k, bd.as<float>(), bi.as<idx_t>(), params, s);
    HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipMemcpyAsync(distances, bd.ptr, sizeof(float) * n * k, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(labels, bi.ptr, sizeof(idx_t) * n * k, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    fold_device_stats();
    InterruptCallback::check();  // faiss/IndexHNSW.cpp:315 (one device pass)
    if (per_query_stats) {
        // no quantization phase; the batch's traversal time is each query's
        for (idx_t i = 0; i < n; i++) {
            per_query_stats[i].total_us = ms * 1e3;
            per_query_stats[i].list_scan_us = ms * 1e3;
        }
    }
}

void IndexHNSW::search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                              idx_t* labels, const SearchParameters* params,
                              hipStream_t s) const {
    FAISS_THROW_IF_NOT_MSG(!params || !params->sel,
                           "IDSelector is supported by the IVF indexes only on this path");
    DevGuard2 dg(device);
    hnsw_device<idx_t>(n, x, ldx, (int)k, distances, labels, params, s);
}

void IndexHNSW::assign_device(idx_t n, const float* x, int ldx, int k, float* distances,
                              int32_t* labels, const SearchParameters* params,
                              hipStream_t s) const {
    DevGuard2 dg(device);
    hnsw_device<int32_t>(n, x, ldx, k, distances, labels, params, s);
}

}  // namespace faiss_amd
