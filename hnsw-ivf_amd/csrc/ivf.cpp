// ivf.cpp — IndexIVF / IndexIVFFlat / IndexIVFPQ / IndexShardsIVF host side.
//
// Reference: faiss/IndexIVF.cpp:303-397 (search), :399-723
// (search_preassigned), :187-285 (add), faiss/IndexIVFFlat.cpp,
// faiss/IndexIVFPQ.cpp, faiss/IndexShardsIVF.cpp:88-245.
#include <unistd.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cinttypes>
#include <cstring>

#include "../../include/faiss_amd.h"
#include "kernels.h"

namespace faiss_amd {

namespace {
struct DevGuard {
    int prev = 0;
    explicit DevGuard(int dev) {
        ensure_hip();
        HIP_CHECK(hipGetDevice(&prev));
        if (prev != dev) HIP_CHECK(hipSetDevice(dev));
    }
    ~DevGuard() {
        int cur = 0;
        hipGetDevice(&cur);
        if (cur != prev) hipSetDevice(prev);
    }
};
}  // namespace

// ---------------------------------------------------------------- invlists
ArrayInvertedLists::ArrayInvertedLists(size_t nl, size_t cs) : nlist(nl), code_size(cs) {
    codes.resize(nl);
    ids.resize(nl);
}
void ArrayInvertedLists::materialize() {
    if (!map) return;
    for (size_t l = 0; l < nlist; l++) {
        const size_t n = map_sizes[l];
        codes[l].assign(map_codes[l], map_codes[l] + n * code_size);
        ids[l].assign(map_ids[l], map_ids[l] + n);
    }
    map.reset();
    map_ondisk = false;
    ondisk_lists.clear();
    ondisk_slots.clear();
    map_codes.clear();
    map_ids.clear();
    map_sizes.clear();
}
void ArrayInvertedLists::add_entries(size_t l, size_t n, const idx_t* ids_in,
                                     const uint8_t* codes_in) {
    FAISS_THROW_IF_NOT(l < nlist);
    materialize();
    ids[l].insert(ids[l].end(), ids_in, ids_in + n);
    codes[l].insert(codes[l].end(), codes_in, codes_in + n * code_size);
}
void ArrayInvertedLists::reset() {
    map.reset();
    map_ondisk = false;
    ondisk_lists.clear();
    ondisk_slots.clear();
    map_codes.clear();
    map_ids.clear();
    map_sizes.clear();
    for (size_t l = 0; l < nlist; l++) {
        codes[l].clear();
        ids[l].clear();
    }
}

// ---------------------------------------------------------------- IndexIVF
IndexIVF::IndexIVF(Index* q, size_t d_, size_t nl, size_t cs, MetricType metric)
        : Index(d_, metric), quantizer(q), nlist(nl), code_size(cs) {
    FAISS_THROW_IF_NOT(q != nullptr);
    FAISS_THROW_IF_NOT((size_t)q->d == d_);
    is_trained = q->is_trained && (size_t)q->ntotal == nlist;
    invlists = std::make_unique<ArrayInvertedLists>(nlist, code_size);
    device = q->device;
}

IndexIVF::~IndexIVF() {
    for (auto& gr : graphs_) gr.clear();
    for (hipEvent_t e : pipe_ev_) (void)hipEventDestroy(e);
    if (pipe_s_) (void)hipStreamDestroy(pipe_s_);
    for (hipEvent_t e : host_ev_) (void)hipEventDestroy(e);
    if (host_cs_) (void)hipStreamDestroy(host_cs_);
    if (own_fields) delete quantizer;
}

int IndexIVF::device_code_stride() const {
    // IVF-Flat keeps 16-B aligned float rows; PQ keeps 4-B aligned code rows
    return (int)roundup(code_size, 4);
}

void IndexIVF::debug_rows(int what, idx_t row0, idx_t n, void* out, size_t* row_bytes,
                          idx_t* rows) const {
    sync_device();
    std::lock_guard<std::recursive_mutex> g(mu_);
    DevGuard dg(device);
    const void* base = nullptr;
    size_t rb = 0;
    if (what == 0) {
        base = d_codes_.ptr;
        rb = device_code_stride();
    } else if (what == 1) {
        base = d_row_list_.ptr;
        rb = sizeof(uint32_t);
    } else if (what == 2) {
        base = stream_image(&rb);
    }
    FAISS_THROW_IF_NOT_MSG(base && rb > 0, "debug_rows: this index has no such buffer");
    if (row_bytes) *row_bytes = rb;
    if (rows) *rows = (idx_t)arena_rows_;
    if (!out || n <= 0) return;
    FAISS_THROW_IF_NOT(row0 >= 0 && row0 + n <= (idx_t)arena_rows_);
    hipStream_t s = stream();
    HIP_CHECK(hipMemcpyAsync(out, (const uint8_t*)base + (size_t)row0 * rb, (size_t)n * rb,
                             hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
}

void IndexIVF::train(idx_t n, const float* x) {
    // faiss/IndexIVF.cpp:1221-1260 (train) + Level1Quantizer::train_q1
    if (quantizer->is_trained && (size_t)quantizer->ntotal == nlist) {
        if (verbose) fprintf(stderr, "IVF quantizer does not need training\n");
    } else {
        std::vector<float> cent((size_t)nlist * d);
        kmeans_train(d, n, x, (int)nlist, niter, 1234, cent.data(), device, verbose);
        quantizer->reset();
        quantizer->train(nlist, cent.data());
        quantizer->add(nlist, cent.data());
        quantizer->is_trained = true;
    }
    FAISS_THROW_IF_NOT((size_t)quantizer->ntotal == nlist);
    // train the encoder on (a subset of) the assigned training vectors
    std::vector<idx_t> assign(n);
    std::vector<float> dis(n);
    if (by_residual || dynamic_cast<IndexIVFPQ*>(this)) {
        quantizer->search(n, x, 1, dis.data(), assign.data());
        train_encoder(n, x, assign.data());
    }
    is_trained = true;
}

void IndexIVF::add(idx_t n, const float* x) { add_with_ids(n, x, nullptr); }

void IndexIVF::add_with_ids(idx_t n, const float* x, const idx_t* xids) {
    FAISS_THROW_IF_NOT(is_trained);
    const idx_t bs = 1 << 20;
    std::vector<idx_t> assign;
    std::vector<float> dis;
    std::vector<uint8_t> codes;
    for (idx_t i0 = 0; i0 < n; i0 += bs) {
        idx_t nb = std::min(bs, n - i0);
        assign.resize(nb);
        dis.resize(nb);
        codes.resize((size_t)nb * code_size);
        const float* xb = x + (size_t)i0 * d;
        quantizer->search(nb, xb, 1, dis.data(), assign.data());
        encode_vectors(nb, xb, assign.data(), codes.data());
        for (idx_t i = 0; i < nb; i++) {
            idx_t l = assign[i];
            if (l < 0) continue;
            idx_t id = xids ? xids[i0 + i] : ntotal + i0 + i;
            invlists->add_entries(l, 1, &id, codes.data() + (size_t)i * code_size);
        }
    }
    ntotal += n;
    std::lock_guard<std::recursive_mutex> g(mu_);
    dirty_ = true;
}

void IndexIVF::reset() {
    invlists->reset();
    ntotal = 0;
    std::lock_guard<std::recursive_mutex> g(mu_);
    dirty_ = true;
}

// Arena upload: lists packed contiguously, each list start and extent aligned
// to ARENA_ALIGN (64) rows = one filter tile; rows padded to the device
// stride; ids / owning list per row (~0 for padding rows).
void IndexIVF::sync_device() const {
    quantizer->sync_device();
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (!dirty_) return;
    DevGuard dg(device);
    hipStream_t s = stream();
    const size_t stride = device_code_stride();
    const bool flat = dynamic_cast<const IndexIVFFlat*>(this) != nullptr;
    const size_t dstride = flat ? sizeof(float) * roundup((size_t)d, 4) : stride;
    std::vector<uint32_t> off(nlist + 1), len(nlist);
    size_t rows = 0;
    for (size_t l = 0; l < nlist; l++) {
        off[l] = (uint32_t)rows;
        len[l] = (uint32_t)invlists->list_size(l);
        rows += roundup(len[l], kern::ARENA_ALIGN);
        FAISS_THROW_IF_NOT_MSG(rows < (1ull << 32), "arena larger than 2^32 rows");
    }
    off[nlist] = (uint32_t)rows;
    arena_rows_ = rows;
    max_list_len_ = nlist ? *std::max_element(len.begin(), len.end()) : 0;
    const size_t code_bytes = std::max<size_t>(rows, 1) * dstride;
    std::vector<idx_t> hi(std::max<size_t>(rows, 1), -1);
    std::vector<uint32_t> hl(std::max<size_t>(rows, 1), 0xffffffffu);
    for (size_t l = 0; l < nlist; l++) {
        const size_t n = len[l];
        for (size_t i = 0; i < n; i++) hl[off[l] + i] = (uint32_t)l;
        if (n) memcpy(hi.data() + off[l], invlists->get_ids(l), sizeof(idx_t) * n);
    }
    // + tail padding: the re-rank reads BDM floats from any row start
    d_codes_.reserve(code_bytes + sizeof(float) * kern::BDM_HOST);
    d_ids_.reserve(sizeof(idx_t) * hi.size());
    d_row_list_.reserve(sizeof(uint32_t) * hl.size());
    d_list_off_.reserve(sizeof(uint32_t) * (nlist + 1));
    d_list_len_.reserve(sizeof(uint32_t) * std::max<size_t>(nlist, 1));
    // Codes: packed arena order into two pinned staging buffers, each copied
    // to HBM while the other fills (no whole-arena host image; mapped lists
    // are read from the page cache exactly once).
    {
        const size_t cap = std::max<size_t>(dstride, std::min<size_t>(code_bytes, 64u << 20) /
                                                         dstride * dstride);
        uint8_t* buf[2] = {nullptr, nullptr};
        hipEvent_t ev[2];
        for (int b = 0; b < 2; b++) {
            HIP_CHECK(hipHostMalloc((void**)&buf[b], cap, hipHostMallocDefault));
            HIP_CHECK(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
        }
        int cur = 0;
        size_t fill = 0, dev_pos = 0, pending[2] = {0, 0};
        auto flush = [&]() {
            if (!fill) return;
            HIP_CHECK(hipMemcpyAsync((uint8_t*)d_codes_.ptr + dev_pos, buf[cur], fill,
                                     hipMemcpyHostToDevice, s));
            HIP_CHECK(hipEventRecord(ev[cur], s));
            pending[cur] = 1;
            dev_pos += fill;
            fill = 0;
            cur ^= 1;
            if (pending[cur]) HIP_CHECK(hipEventSynchronize(ev[cur]));
            pending[cur] = 0;
        };
        auto put_rows = [&](const uint8_t* src, size_t nrows) {  // src == nullptr: zero rows
            while (nrows) {
                const size_t take = std::min(nrows, (cap - fill) / dstride);
                uint8_t* dst = buf[cur] + fill;
                if (src && dstride == code_size) {
                    memcpy(dst, src, take * code_size);
                } else {
                    memset(dst, 0, take * dstride);
                    if (src)
                        for (size_t i = 0; i < take; i++)
                            memcpy(dst + i * dstride, src + i * code_size, code_size);
                }
                if (src) src += take * code_size;
                fill += take * dstride;
                nrows -= take;
                if (fill + dstride > cap) flush();
            }
        };
        for (size_t l = 0; l < nlist; l++) {
            put_rows(invlists->get_codes(l), len[l]);
            put_rows(nullptr, roundup(len[l], kern::ARENA_ALIGN) - len[l]);
        }
        if (rows == 0) put_rows(nullptr, 1);
        flush();
        HIP_CHECK(hipStreamSynchronize(s));
        for (int b = 0; b < 2; b++) {
            HIP_CHECK(hipEventDestroy(ev[b]));
            HIP_CHECK(hipHostFree(buf[b]));
        }
    }
    HIP_CHECK(hipMemcpyAsync(d_ids_.ptr, hi.data(), sizeof(idx_t) * hi.size(),
                             hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_row_list_.ptr, hl.data(), sizeof(uint32_t) * hl.size(),
                             hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_list_off_.ptr, off.data(), sizeof(uint32_t) * (nlist + 1),
                             hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_list_len_.ptr, len.data(), sizeof(uint32_t) * nlist,
                             hipMemcpyHostToDevice, s));
    {
        // work items longest list first (kern::IVFBuckets::perm)
        std::vector<uint32_t> perm(nlist);
        for (size_t l = 0; l < nlist; l++) perm[l] = (uint32_t)l;
        std::stable_sort(perm.begin(), perm.end(),
                         [&](uint32_t a, uint32_t b) { return len[a] > len[b]; });
        d_list_perm_.reserve(sizeof(uint32_t) * std::max<size_t>(nlist, 1));
        HIP_CHECK(hipMemcpyAsync(d_list_perm_.ptr, perm.data(), sizeof(uint32_t) * nlist,
                                 hipMemcpyHostToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));  // perm is a host temporary
    }
    upload_extra();
    HIP_CHECK(hipStreamSynchronize(s));
    dirty_ = false;
    version_++;  // (the content uploaded may differ from what a captured graph saw)
}

uint32_t* IndexIVF::bucket_counts(hipStream_t s, uint32_t** next) const {
    // nlist counters, zero between calls: the scan clears each count once it
    // has read it (self-cleaning, so a captured step can be replayed).  A
    // (re)allocation starts them at zero; they are (re)zeroed as well when
    // the previous call did not reach flip_counts() (an exception between
    // the two left them dirty) or ran on another stream (whose scan may still
    // be clearing them)
    const size_t need = sizeof(uint32_t) * std::max<size_t>(nlist, 1);
    const bool fresh = !s_counts_.ptr || s_counts_.bytes < need;
    if (fresh || counts_pending_ || s != counts_stream_) {
        if (!fresh && s != counts_stream_ && counts_stream_valid_)
            HIP_CHECK(hipStreamSynchronize(counts_stream_));
        s_counts_.reserve(need);
        HIP_CHECK(hipMemsetAsync(s_counts_.ptr, 0, need, s));
        counts_parity_ = 0;
    }
    counts_stream_ = s;
    counts_stream_valid_ = true;
    counts_pending_ = true;  // until flip_counts()
    uint32_t* base = s_counts_.as<uint32_t>();
    *next = base;  // cleared by the scan that reads them
    return base;
}

namespace {
std::atomic<int> g_search_slices{1};
// [i n / nt, (i + 1) n / nt): the reference's slice bounds (IndexIVF.cpp:367-368)
bool slices_mixed(idx_t n, int nt) {
    // slice sizes are floor(n / nt) or that + 1: one form unless they straddle 20
    const idx_t lo = n / nt, hi = (n + nt - 1) / nt;
    return lo < 20 && hi >= 20;
}
}  // namespace
void set_search_slices(int t) {
    FAISS_THROW_IF_NOT_MSG(t >= 1, "set_search_slices: t must be >= 1");
    g_search_slices = t;
}
int get_search_slices() { return g_search_slices; }

void IndexIVF::quantize_device(idx_t n, const float* x, int ldx, int np, float* coarse_dis,
                               int32_t* assign, const SearchParameters* qparams,
                               hipStream_t s) const {
    const int nt = (int)std::min<idx_t>(g_search_slices, std::max<idx_t>(n, 1));
    if (nt <= 1) {
        quantizer->assign_device(n, x, ldx, np, coarse_dis, assign, qparams, s);
        return;
    }
    if (!slices_mixed(n, nt)) {
        // every slice takes the form of its size: one call with that size
        quantizer->assign_device_slice(n, x, ldx, np, coarse_dis, assign, qparams, s, n / nt);
        return;
    }
    for (int i = 0; i < nt; i++) {
        const idx_t a = (idx_t)i * n / nt, b = (idx_t)(i + 1) * n / nt;
        if (b > a)
            quantizer->assign_device_slice(b - a, x + a * ldx, ldx, np, coarse_dis + a * np,
                                           assign + a * np, qparams, s, b - a);
    }
}

// queries per chunk: bounds the partial-result scratch to ~1 GiB (the
// list-centric Flat scan keeps per-(query, probe) partials; the query-centric
// PQ scan keeps none)
idx_t IndexIVF::search_chunk(idx_t n, size_t np, idx_t k) const {
    const bool pq = dynamic_cast<const IndexIVFPQ*>(this) != nullptr;
    // Flat: direct-scan partials (k keys + ids per probe) or filter keys;
    // PQ: filter keys (<= 32 per probe) + probe records + buckets
    const size_t per_q = pq ? np * (32 * 4 + 32 + 16) + 16
                            : np * (size_t)std::max<idx_t>(k, 32) * 12 + np * 16;
    idx_t qchunk = std::max<idx_t>(1, (idx_t)(((size_t)4 << 30) / per_q));
    return std::max<idx_t>(1, std::min<idx_t>(qchunk, n));
}

namespace {
// faiss/IndexIVF.cpp:445-460, 595-704: parallel_mode 0 / 3 are query-parallel
// scans of one heap per query; 1 / 2 split a query's probes across threads
// and merge the per-thread heaps, which gives the same distances (the
// reference's own test, tests/test_index_accuracy.py:47-60, asserts equal D).
// The GPU computes every mode as mode 0.  PARALLEL_MODE_NO_HEAP_INIT (1024)
// accumulates into the caller's arrays and is not offered.
void check_parallel_mode(int pm) {
    FAISS_THROW_IF_NOT_FMT(pm >= 0 && pm <= 3,
                           "parallel_mode %d not supported on the GPU path (0-3 are)", pm);
}
}  // namespace

const int32_t* IndexIVF::apply_max_codes(idx_t n, int np, const int32_t* assign,
                                         size_t max_codes, const uint32_t** lim,
                                         hipStream_t s) const {
    *lim = nullptr;
    if (max_codes == 0 || n <= 0) return assign;  // 0 = unlimited (IndexIVF.cpp:452-454)
    std::lock_guard<std::recursive_mutex> g(mu_);
    s_lim_.reserve(sizeof(uint32_t) * n * np);
    s_alim_.reserve(sizeof(int32_t) * n * np);
    kern::probe_limits(assign, n, np, d_list_len_.as<uint32_t>(), (int)nlist,
                       (int64_t)std::min<size_t>(max_codes, (size_t)INT64_MAX),
                       s_alim_.as<int32_t>(), s_lim_.as<uint32_t>(), s);
    *lim = s_lim_.as<uint32_t>();
    return s_alim_.as<int32_t>();
}

const uint8_t* IndexIVF::apply_selector(const SearchParameters* params, hipStream_t s) const {
    if (!params || !params->sel) return nullptr;
    std::lock_guard<std::recursive_mutex> g(mu_);
    const int64_t rows = std::max<int64_t>((int64_t)arena_rows_, 1);
    s_selmask_.reserve((size_t)rows + 16);
    HIP_CHECK(hipMemsetAsync(s_selmask_.ptr, 0, (size_t)rows + 16, s));
    params->sel->mark_device(d_ids_.as<int64_t>(), (int64_t)arena_rows_, s_selmask_.as<uint8_t>(),
                             s);
    return s_selmask_.as<uint8_t>();
}

void IndexIVF::SearchGraph::clear() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    exec = nullptr;
    graph = nullptr;
    tsinks.clear();
    tnames.clear();
    tunits.clear();
    tnodes.clear();
    key.clear();
    seen = 0;
    failed = false;
    used = 0;
}

namespace {
// every FAISS_AMD_* switch, in the graph key (they steer host-side choices
// a captured graph would freeze)
std::string amd_env_key() {
    std::string r;
    for (char** e = ::environ; e && *e; e++)
        if (!strncmp(*e, "FAISS_AMD_", 10)) {
            r += *e;
            r += ';';
        }
    return r;
}
}  // namespace

// A search repeated with the same pointers, sizes and settings (a serving
// loop, the bench's steps) runs as one hipGraph: the second identical call
// captures the launches of search_device_eager, later ones replay them, so
// the host issues one launch instead of ~15 (c1 / c2: the kernels are short
// enough for launch gaps to matter).  The key holds everything the eager
// path reads on the host — sizes, pointers, stream, settings, the index and
// quantizer contents, FAISS_AMD_* switches, the kernel-timing state — and
// the DeviceBuffer epoch, so any scratch reallocation anywhere retires the
// graph.  Kernel timing keeps working: the timed stages' event-record nodes
// get fresh events at every replay.
void IndexIVF::search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                             idx_t* labels, const SearchParameters* params_in,
                             hipStream_t s) const {
    const char* genv = getenv("FAISS_AMD_GRAPH");
    std::lock_guard<std::recursive_mutex> g(mu_);
    const auto* qflat = dynamic_cast<const IndexFlat*>(quantizer);
    // (FAISS_AMD_IVF_STATS: the debug counters synchronise inside the scan)
    const bool eligible = !(genv && !strcmp(genv, "0")) && params_in == nullptr && !qdone_ &&
                          !getenv("FAISS_AMD_IVF_STATS") && qflat != nullptr && get_search_slices() <= 1 && n > 0 && !dirty_;
    if (!eligible) {
        search_device_eager(n, x, ldx, k, distances, labels, params_in, s);
        return;
    }
    char buf[512];
    const auto* pq = dynamic_cast<const IndexIVFPQ*>(this);
    snprintf(buf, sizeof(buf), "%lld|%p|%d|%lld|%p|%p|%p|%zu|%zu|%d|%d|%lld|%llu|%p|%llu|%llu|%d|%d|%d",
             (long long)n, (const void*)x, ldx, (long long)k, (void*)distances, (void*)labels,
             (void*)s, nprobe, max_codes, parallel_mode, (int)metric_type, (long long)ntotal,
             (unsigned long long)content_version(), (const void*)quantizer,
             (unsigned long long)quantizer->content_version(),
             (unsigned long long)devbuf_epoch().load(), device, pq ? pq->use_precomputed_table : -1,
             (int)by_residual);
    const std::string key = std::string(buf) + kernel_timing_state() + "|" + amd_env_key();
    SearchGraph* G = nullptr;
    for (auto& e : graphs_)
        if (e.key == key) G = &e;
    if (!G) {
        // a new call: the entry used least recently (or an empty one)
        G = &graphs_[0];
        for (auto& e : graphs_)
            if (e.used < G->used) G = &e;
        G->clear();
        G->key = key;
    }
    SearchGraph& graph_ = *G;
    graph_.used = ++graph_tick_;
    if (graph_.exec) {
        // replay: fresh events at the timed stages' record nodes
        for (size_t i = 0; i < graph_.tnodes.size(); i++) {
            hipEvent_t a, b;
            HIP_CHECK(hipEventCreate(&a));
            HIP_CHECK(hipEventCreate(&b));
            HIP_CHECK(hipGraphExecEventRecordNodeSetEvent(graph_.exec, graph_.tnodes[i].first, a));
            HIP_CHECK(hipGraphExecEventRecordNodeSetEvent(graph_.exec, graph_.tnodes[i].second, b));
            KernelTimes* t = graph_.tsinks[i];
            t->names.push_back(graph_.tnames[i]);
            t->units.push_back(graph_.tunits[i]);
            t->e0.push_back(a);
            t->e1.push_back(b);
        }
        // the graph writes this index's and the quantizer's scratch: wait
        // for their last users on other streams, as the eager path does
        qflat->stream_enter(s);
        order_.enter(s);
        HIP_CHECK(hipGraphLaunch(graph_.exec, s));
        order_.leave(s);
        qflat->stream_leave(s);
        return;
    }
    if (graph_.failed || graph_.seen++ == 0) {
        search_device_eager(n, x, ldx, k, distances, labels, params_in, s);
        return;
    }
    // second identical call: capture it (the stages timed in it are this
    // index's and the quantizer's: sinks[j] from its entry t0s[j] on)
    KernelTimes* sinks[2] = {&ktimes, &quantizer->ktimes};
    const size_t t0s[2] = {ktimes.e0.size(), quantizer->ktimes.e0.size()};
    auto drop_captured = [&] {
        for (int j = 0; j < 2; j++) {
            KernelTimes& t = *sinks[j];
            const size_t t0 = t0s[j];
            t.names.resize(std::min(t.names.size(), t0));
            t.units.resize(std::min(t.units.size(), t0));
            for (size_t i = t0; i < t.e0.size(); i++) {
                (void)hipEventDestroy(t.e0[i]);
                (void)hipEventDestroy(t.e1[i]);
            }
            t.e0.resize(t0);
            t.e1.resize(t0);
        }
    };
    hipGraph_t gr = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();  // (e.g. the legacy default stream)
        graph_.failed = true;
        search_device_eager(n, x, ldx, k, distances, labels, params_in, s);
        return;
    }
    bool ok = true;
    capturing_ = true;
    try {
        search_device_eager(n, x, ldx, k, distances, labels, params_in, s);
    } catch (...) {
        ok = false;
    }
    capturing_ = false;
    hipError_t e = hipStreamEndCapture(s, &gr);
    hipGraphExec_t ex = nullptr;
    if (ok && e == hipSuccess && gr) e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    // the timed stages' record nodes, matched by the events captured into them
    std::vector<std::pair<hipGraphNode_t, hipGraphNode_t>> tn;
    std::vector<KernelTimes*> tsk;
    std::vector<std::string> tnm;
    std::vector<double> tun;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
    for (int j = 0; j < 2; j++)
        for (size_t i = t0s[j]; i < sinks[j]->e0.size(); i++) {
            tn.emplace_back(nullptr, nullptr);
            tsk.push_back(sinks[j]);
            tnm.push_back(sinks[j]->names[i]);
            tun.push_back(sinks[j]->units[i]);
            tev.emplace_back(sinks[j]->e0[i], sinks[j]->e1[i]);
        }
    if (ok && e == hipSuccess && ex) {
        size_t nn = 0;
        e = hipGraphGetNodes(gr, nullptr, &nn);
        std::vector<hipGraphNode_t> nodes(nn);
        if (e == hipSuccess && nn) e = hipGraphGetNodes(gr, nodes.data(), &nn);
        for (size_t j = 0; e == hipSuccess && j < nn; j++) {
            hipGraphNodeType ty;
            if (hipGraphNodeGetType(nodes[j], &ty) != hipSuccess || ty != hipGraphNodeTypeEventRecord)
                continue;
            hipEvent_t ev = nullptr;
            if (hipGraphEventRecordNodeGetEvent(nodes[j], &ev) != hipSuccess) continue;
            for (size_t i = 0; i < tev.size(); i++) {
                if (tev[i].first == ev) tn[i].first = nodes[j];
                if (tev[i].second == ev) tn[i].second = nodes[j];
            }
        }
        for (auto& p : tn)
            if (!p.first || !p.second) e = hipErrorUnknown;
    }
    if (!ok || e != hipSuccess || !ex) {
        // not capturable here: drop the partial capture, run eagerly from now on
        (void)hipGetLastError();
        if (ex) (void)hipGraphExecDestroy(ex);
        if (gr) (void)hipGraphDestroy(gr);
        drop_captured();
        (void)hipGetLastError();
        graph_.failed = true;
        search_device_eager(n, x, ldx, k, distances, labels, params_in, s);
        return;
    }
    graph_.graph = gr;
    graph_.exec = ex;
    graph_.tnodes = tn;
    graph_.tsinks = tsk;
    graph_.tnames = tnm;
    graph_.tunits = tun;
    // the events captured are not recorded by the graph's launches (its
    // nodes hold them only as handles): drop them, and time this first
    // launch through the replay path's fresh events
    drop_captured();
    for (size_t i = 0; i < graph_.tnodes.size(); i++) {
        hipEvent_t a, b;
        HIP_CHECK(hipEventCreate(&a));
        HIP_CHECK(hipEventCreate(&b));
        HIP_CHECK(hipGraphExecEventRecordNodeSetEvent(ex, graph_.tnodes[i].first, a));
        HIP_CHECK(hipGraphExecEventRecordNodeSetEvent(ex, graph_.tnodes[i].second, b));
        KernelTimes* t = graph_.tsinks[i];
        t->names.push_back(graph_.tnames[i]);
        t->units.push_back(graph_.tunits[i]);
        t->e0.push_back(a);
        t->e1.push_back(b);
    }
    HIP_CHECK(hipGraphLaunch(ex, s));
}

void IndexIVF::search_device_eager(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                                   idx_t* labels, const SearchParameters* params_in,
                                   hipStream_t s) const {
    // faiss/IndexIVF.cpp:303-397
    FAISS_THROW_IF_NOT(k > 0);
    const SearchParametersIVF* params = nullptr;
    if (params_in) {
        params = dynamic_cast<const SearchParametersIVF*>(params_in);
        FAISS_THROW_IF_NOT_MSG(params, "IndexIVF params have incorrect type");
    }
    const size_t np = std::min(nlist, params && params->nprobe ? params->nprobe : nprobe);
    FAISS_THROW_IF_NOT(np > 0);
    const size_t mc = params ? params->max_codes : max_codes;
    DevGuard dg(device);
    sync_device();
    const uint8_t* selm = apply_selector(params, s);
    // device API: asynchronous, so indexIVF_stats is maintained by the host
    // entry points (search / search_stats / search_preassigned) only
    const idx_t qchunk = search_chunk(n, np, k);
    std::lock_guard<std::recursive_mutex> g(mu_);
    order_.enter(s);
    s_cd_.reserve(sizeof(float) * qchunk * np);
    s_ci_.reserve(sizeof(int32_t) * qchunk * np);
    // a flat quantizer prepares the query image into this index's scratch, on
    // this stream, and the list filter reads it from there
    const auto* qf = dynamic_cast<const IndexFlat*>(quantizer);
    if (qf && qf->d == d) s_q_.reserve(qf->query_image_size(qchunk));
    for (idx_t q0 = 0; q0 < n; q0 += qchunk) {
        const idx_t nq = std::min(qchunk, n - q0);
        struct Reset {
            const void*& p;
            ~Reset() { p = nullptr; }
        } reset{shared_qimg_};
        const int nt = (int)std::min<idx_t>(get_search_slices(), std::max<idx_t>(nq, 1));
        const bool one_form = nt <= 1 || (nq / nt >= 20);  // the whole batch's BLAS form
        if (qf && qf->d == d && one_form && mc == 0 && !selm &&
            scan_flat_pipelined(nq, x + q0 * ldx, ldx, k, (int)np, distances + q0 * k,
                                labels + q0 * k, s)) {
            continue;
        }
        if (qf && qf->d == d && one_form) {
            if (qf->assign_device_qimg(nq, x + q0 * ldx, ldx, (int)np, s_cd_.as<float>(),
                                       s_ci_.as<int32_t>(), s_q_.ptr, s))
                shared_qimg_ = s_q_.ptr;
        } else if (qf) {
            quantize_device(nq, x + q0 * ldx, ldx, (int)np, s_cd_.as<float>(),
                            s_ci_.as<int32_t>(), params ? params->quantizer_params : nullptr, s);
        } else if (mc == 0 && !selm &&
                   scan_hnsw_pipelined(nq, x + q0 * ldx, ldx, k, (int)np, distances + q0 * k,
                                       labels + q0 * k,
                                       params ? params->quantizer_params : nullptr, s)) {
            continue;
        } else if (mc == 0 && !selm &&
                   scan_hnsw_split(nq, x + q0 * ldx, ldx, k, (int)np, distances + q0 * k,
                                   labels + q0 * k,
                                   params ? params->quantizer_params : nullptr, s)) {
            continue;
        } else {
            quantize_device(nq, x + q0 * ldx, ldx, (int)np, s_cd_.as<float>(),
                            s_ci_.as<int32_t>(), params ? params->quantizer_params : nullptr, s);
        }
        if (paged_marks_ && !capturing_) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            HIP_CHECK(hipEventRecord(e, s));
            paged_marks_->push_back(e);
        }
        const uint32_t* lim = nullptr;
        const int32_t* asg = apply_max_codes(nq, (int)np, s_ci_.as<int32_t>(), mc, &lim, s);
        search_preassigned_device(nq, x + q0 * ldx, ldx, k, (int)np, asg, s_cd_.as<float>(),
                                  distances + q0 * k, labels + q0 * k, s, lim, selm);
    }
    order_.leave(s);
}

// An HNSW quantizer served by the register kernel (max(efSearch, k) <= 64):
// that kernel is latency-bound with one wave per query, and its last waves
// leave most of the GPU idle.  The batch is searched in chunks: chunk c's
// quantizer search runs on pipe_s_ while the caller's stream scans chunk
// c - 1, so the scan fills the idle slots.  Each chunk is an ordinary
// assign + search_preassigned of its queries (results identical).
// FAISS_AMD_HNSW_PIPE=<chunks>; off by default: on c4 (10k queries) the step
// went from 2.50 ms to 3.48 ms with 2 chunks and 4.84 ms with 4 — the HNSW
// waves hold every slot, so the scan's short kernels queue behind them, and
// each chunk pays the HNSW kernel's tail again.
bool IndexIVF::scan_hnsw_pipelined(idx_t nq, const float* x, int ldx, idx_t k, int np,
                                   float* distances, idx_t* labels,
                                   const SearchParameters* qparams, hipStream_t s) const {
    const auto* qh = dynamic_cast<const IndexHNSW*>(quantizer);
    if (!qh || qdone_ || get_search_slices() > 1) return false;
    int ef = qh->hnsw.efSearch;
    if (const auto* hp = dynamic_cast<const SearchParametersHNSW*>(qparams)) ef = hp->efSearch;
    if (!kern::hnsw_register_eligible(np, ef) || kern::hnsw_uses_batched(np, ef)) return false;
    const char* env = getenv("FAISS_AMD_HNSW_PIPE");
    const int P = env ? atoi(env) : 1;  // off: measured slower on c4 (below)
    if (P <= 1 || nq < (idx_t)P * 1024) return false;
    if (!pipe_s_) HIP_CHECK(hipStreamCreateWithFlags(&pipe_s_, hipStreamNonBlocking));
    while ((int)pipe_ev_.size() < P + 1) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        pipe_ev_.push_back(e);
    }
    // the chunks' quantizer searches follow the caller's prior work (x, and
    // the previous readers of the coarse buffers)
    HIP_CHECK(hipEventRecord(pipe_ev_[P], s));
    HIP_CHECK(hipStreamWaitEvent(pipe_s_, pipe_ev_[P], 0));
    for (int c = 0; c < P; c++) {
        const idx_t a = nq * c / P, b = nq * (c + 1) / P;
        float* cd = s_cd_.as<float>() + a * np;
        int32_t* ci = s_ci_.as<int32_t>() + a * np;
        quantizer->assign_device(b - a, x + a * ldx, ldx, np, cd, ci, qparams, pipe_s_);
        HIP_CHECK(hipEventRecord(pipe_ev_[c], pipe_s_));
        HIP_CHECK(hipStreamWaitEvent(s, pipe_ev_[c], 0));
        search_preassigned_device(b - a, x + a * ldx, ldx, k, np, ci, cd, distances + a * k,
                                  labels + a * k, s, nullptr, nullptr);
    }
    return true;
}

// A flat quantizer's batch in P chunks (FAISS_AMD_PIPE=<P>): chunk c's
// coarse search (query image, bf16x3 filter, exact re-rank) on pipe_s_
// overlaps chunk c - 1's list scan on the caller's stream, so the scan's
// latency-bound re-rank shares the CUs with the next chunk's MFMA filter.
// Chunks are whole 128-query blocks of at least 1024 queries, so every
// chunk takes the batch's BLAS form; each chunk's query image lives in its
// own slice of s_q_ (the scan of chunk c reads it while chunk c + 1's is
// written).  Results identical to the one-chunk search.
bool IndexIVF::scan_flat_pipelined(idx_t nq, const float* x, int ldx, idx_t k, int np,
                                   float* distances, idx_t* labels, hipStream_t s) const {
    const auto* qf = dynamic_cast<const IndexFlat*>(quantizer);
    const char* env = getenv("FAISS_AMD_PIPE");
    const int P = env ? atoi(env) : 1;
    if (!qf || qdone_ || P <= 1 || nq < (idx_t)P * 1024) return false;
    if (!pipe_s_) HIP_CHECK(hipStreamCreateWithFlags(&pipe_s_, hipStreamNonBlocking));
    while ((int)pipe_ev_.size() < P + 1) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        pipe_ev_.push_back(e);
    }
    std::vector<idx_t> cut(P + 1);
    for (int c = 0; c < P; c++) cut[c] = std::min<idx_t>(nq, (idx_t)roundup((size_t)(nq * c / P), 128));
    cut[P] = nq;
    size_t tot = 0;
    for (int c = 0; c < P; c++)
        if (cut[c + 1] > cut[c]) tot += roundup(qf->query_image_size(cut[c + 1] - cut[c]), 256);
    s_q_.reserve(tot);
    // the chunks' coarse searches follow the caller's prior work (x, and the
    // previous readers of the coarse buffers and query images)
    HIP_CHECK(hipEventRecord(pipe_ev_[P], s));
    HIP_CHECK(hipStreamWaitEvent(pipe_s_, pipe_ev_[P], 0));
    size_t off = 0;
    for (int c = 0; c < P; c++) {
        const idx_t a = cut[c], b = cut[c + 1];
        if (b <= a) continue;
        float* cd = s_cd_.as<float>() + a * np;
        int32_t* ci = s_ci_.as<int32_t>() + a * np;
        void* qi = (uint8_t*)s_q_.ptr + off;
        off += roundup(qf->query_image_size(b - a), 256);
        const bool img = qf->assign_device_qimg(b - a, x + a * ldx, ldx, np, cd, ci, qi, pipe_s_);
        HIP_CHECK(hipEventRecord(pipe_ev_[c], pipe_s_));
        HIP_CHECK(hipStreamWaitEvent(s, pipe_ev_[c], 0));
        struct Reset {
            const void*& p;
            ~Reset() { p = nullptr; }
        } reset{shared_qimg_};
        shared_qimg_ = img ? qi : nullptr;
        search_preassigned_device(b - a, x + a * ldx, ldx, k, np, ci, cd, distances + a * k,
                                  labels + a * k, s, nullptr, nullptr);
    }
    return true;
}

// An HNSW quantizer re-runs the queries whose batched search met an exact
// distance tie with the reference's sequential algorithm (~0.6 % of c4's
// queries, one wave each for ~1.5 ms).  Here the batched assignment of all
// queries is scanned at once while that re-run proceeds on the quantizer's
// side stream; the re-run queries are then scanned again with their exact
// assignment and their rows replaced (results identical to scanning after
// the full assignment; their first scan is wasted work).  FAISS_AMD_HNSW_DEFER=0
// restores the sequential order.
bool IndexIVF::scan_hnsw_split(idx_t nq, const float* x, int ldx, idx_t k, int np,
                               float* distances, idx_t* labels, const SearchParameters* qparams,
                               hipStream_t s) const {
    const auto* qh = dynamic_cast<const IndexHNSW*>(quantizer);
    const char* env = getenv("FAISS_AMD_HNSW_DEFER");
    if (!qh || qdone_ || (env && !strcmp(env, "0"))) return false;
    if (!qh->split_begin(nq, x, ldx, np, s_cd_.as<float>(), s_ci_.as<int32_t>(), qparams, s)) {
        // not offered: split_begin ran the plain assignment
        search_preassigned_device(nq, x, ldx, k, np, s_ci_.as<int32_t>(), s_cd_.as<float>(),
                                  distances, labels, s, nullptr, nullptr);
        return true;
    }
    IndexHNSW::SplitHold hold{qh};  // the quantizer stays locked to this caller
    search_preassigned_device(nq, x, ldx, k, np, s_ci_.as<int32_t>(), s_cd_.as<float>(),
                              distances, labels, s, nullptr, nullptr);
    const IndexHNSW::Split sp = qh->split_finish();
    if (sp.nf == 0) return true;
    HIP_CHECK(hipStreamWaitEvent(s, sp.done, 0));
    const int l = (int)roundup((size_t)d, 4);
    s_fx_.reserve(sizeof(float) * sp.nf * l);
    s_fDo_.reserve(sizeof(float) * sp.nf * k);
    s_fIo_.reserve(sizeof(idx_t) * sp.nf * k);
    if (l != d) HIP_CHECK(hipMemsetAsync(s_fx_.ptr, 0, sizeof(float) * sp.nf * l, s));
    kern::gather_rows(x, ldx, sp.idx, sp.nf, d, s_fx_.as<float>(), l, s);
    search_preassigned_device(sp.nf, s_fx_.as<float>(), l, k, np, sp.I, sp.D, s_fDo_.as<float>(),
                              s_fIo_.as<idx_t>(), s, nullptr, nullptr);
    kern::scatter_rows(s_fDo_.ptr, (int)k, sp.idx, sp.nf, distances, s);
    kern::scatter_rows(s_fIo_.ptr, 2 * (int)k, sp.idx, sp.nf, labels, s);
    // the exact assignment in the coarse buffers too (their later readers)
    kern::scatter_rows(sp.I, np, sp.idx, sp.nf, s_ci_.ptr, s);
    kern::scatter_rows(sp.D, np, sp.idx, sp.nf, s_cd_.ptr, s);
    return true;
}

void IndexIVF::search_preassigned_device_ordered(idx_t n, const float* x, int ldx, idx_t k,
                                                 int np, const int32_t* assign,
                                                 const float* cdis, float* distances,
                                                 idx_t* labels, hipStream_t s) const {
    DevGuard dg(device);
    sync_device();
    std::lock_guard<std::recursive_mutex> g(mu_);
    order_.enter(s);
    search_preassigned_device(n, x, ldx, k, np, assign, cdis, distances, labels, s);
    order_.leave(s);
}

void IndexIVF::search_preassigned(idx_t n, const float* x, idx_t k, const idx_t* assign,
                                  const float* centroid_dis, float* distances, idx_t* labels,
                                  bool store_pairs, const SearchParametersIVF* params,
                                  IndexIVFStats* stats) const {
    search_preassigned_stats(n, x, k, assign, centroid_dis, distances, labels, store_pairs,
                             params, stats, nullptr);
}

namespace {
// HIP events bracketing the stages of one host call (resolved after the
// final synchronisation, so timing adds no host-device round trip)
struct StageEvents {
    std::vector<hipEvent_t> ev;
    hipEvent_t mark(hipStream_t s) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e));
        HIP_CHECK(hipEventRecord(e, s));
        ev.push_back(e);
        return e;
    }
    static double ms(hipEvent_t a, hipEvent_t b) {
        float t = 0.f;
        HIP_CHECK(hipEventElapsedTime(&t, a, b));
        return t;
    }
    ~StageEvents() {
        for (auto e : ev) (void)hipEventDestroy(e);
    }
};
}  // namespace

void IndexIVF::search_preassigned_stats(idx_t n, const float* x, idx_t k, const idx_t* assign,
                                        const float* centroid_dis, float* distances,
                                        idx_t* labels, bool store_pairs,
                                        const SearchParametersIVF* params,
                                        IndexIVFStats* ivf_stats,
                                        QueryLatencyStats* per_query_stats) const {
    // faiss/IndexIVF.cpp:399-723 / 870-1200 (parallel_mode 0 semantics)
    FAISS_THROW_IF_NOT(k > 0);
    check_parallel_mode(parallel_mode);
    const size_t np = std::min(nlist, params && params->nprobe ? params->nprobe : nprobe);
    FAISS_THROW_IF_NOT(np > 0);
    const size_t mc = params ? params->max_codes : max_codes;
    if (n == 0) return;
    std::vector<int32_t> a32((size_t)n * np);
    for (size_t i = 0; i < (size_t)n * np; i++) {
        idx_t key = assign[i];
        FAISS_THROW_IF_NOT_FMT(key < (idx_t)nlist, "Invalid key=%lld nlist=%zd",
                               (long long)key, nlist);
        a32[i] = (int32_t)(key < 0 ? -1 : key);
    }
    // a caller-supplied assignment may name a list twice for one query; the
    // reference then scans it twice and its heap holds each such vector twice
    // (faiss/IndexIVF.cpp:595-631).  The exact scan reproduces that; the
    // list-centric filter assumes distinct probes.
    bool dup = false;
    {
        std::vector<int32_t> row((size_t)np);
        for (idx_t q = 0; q < n && !dup; q++) {
            std::copy(a32.begin() + q * np, a32.begin() + (q + 1) * np, row.begin());
            std::sort(row.begin(), row.end());
            for (size_t j = 1; j < np && !dup; j++) dup = row[j] >= 0 && row[j] == row[j - 1];
        }
    }
    DevGuard dg(device);
    sync_device();
    hipStream_t s = stream();
    const int ldx = ld();
    // the host entry points' device buffers, kept between calls
    std::lock_guard<std::mutex> hg(host_mu_);
    DeviceBuffer &bx = h_x_, &ba = s_as_, &bc = s_ad_, &bd = h_d_, &bi = h_i_;
    bx.reserve(sizeof(float) * n * ldx);
    ba.reserve(sizeof(int32_t) * n * np);
    bc.reserve(sizeof(float) * n * np);
    bd.reserve(sizeof(float) * n * k);
    bi.reserve(sizeof(idx_t) * n * k);
    if (ldx != d) HIP_CHECK(hipMemsetAsync(bx.ptr, 0, sizeof(float) * n * ldx, s));
    HIP_CHECK(hipMemcpy2DAsync(bx.ptr, sizeof(float) * ldx, x, sizeof(float) * d,
                               sizeof(float) * d, n, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(ba.ptr, a32.data(), sizeof(int32_t) * n * np,
                             hipMemcpyHostToDevice, s));
    if (centroid_dis)
        HIP_CHECK(hipMemcpyAsync(bc.ptr, centroid_dis, sizeof(float) * n * np,
                                 hipMemcpyHostToDevice, s));
    std::lock_guard<std::recursive_mutex> g(mu_);
    s_stats_.reserve(2 * sizeof(unsigned long long));
    HIP_CHECK(hipMemsetAsync(s_stats_.ptr, 0, 2 * sizeof(unsigned long long), s));
    StageEvents ev;
    hipEvent_t e0 = ev.mark(s);
    // per query: the device clock where its result is emitted, against
    // stamps at the scan's start and end (calibrated by e0 / e1)
    struct ResetQ {
        unsigned long long*& p;
        ~ResetQ() { p = nullptr; }
    } reset_q{qdone_};
    if (per_query_stats) {
        s_qdone_.reserve(sizeof(unsigned long long) * n);
        HIP_CHECK(hipMemsetAsync(s_qdone_.ptr, 0, sizeof(unsigned long long) * n, s));
        s_stamps_.reserve(sizeof(unsigned long long) * 2);
        kern::device_stamp(s_stamps_.as<unsigned long long>(), s);
        qdone_ = s_qdone_.as<unsigned long long>();
    }
    const uint32_t* lim = nullptr;
    const int32_t* asg = apply_max_codes(n, (int)np, ba.as<int32_t>(), mc, &lim, s);
    const uint8_t* selm = apply_selector(params, s);
    struct ResetDup {
        bool& f;
        ~ResetDup() { f = false; }
    } reset_dup{dup_probes_};
    dup_probes_ = dup;
    if (!centroid_dis) HIP_CHECK(hipMemsetAsync(bc.ptr, 0, sizeof(float) * n * np, s));
    own_coarse_dis(n, bx.as<float>(), ldx, (int)np, ba.as<int32_t>(), bc.as<float>(), s);
    search_preassigned_device(n, bx.as<float>(), ldx, k, (int)np, asg, bc.as<float>(),
                              bd.as<float>(), bi.as<idx_t>(), s, lim, selm, store_pairs);
    dup_probes_ = false;
    qdone_ = nullptr;
    if (per_query_stats) kern::device_stamp(s_stamps_.as<unsigned long long>() + 1, s);
    hipEvent_t e1 = ev.mark(s);
    kern::ivf_visit_stats(asg, n * (int64_t)np, d_list_len_.as<uint32_t>(), (int)nlist, lim,
                          s_stats_.as<unsigned long long>(), s);
    unsigned long long st[2];
    HIP_CHECK(hipMemcpyAsync(distances, bd.ptr, sizeof(float) * n * k, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(labels, bi.ptr, sizeof(idx_t) * n * k, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(st, s_stats_.ptr, sizeof(st), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    // faiss/IndexIVF.cpp:627, 707-713 (the batch is one device pass here)
    if (InterruptCallback::is_interrupted()) FAISS_THROW_MSG("computation interrupted");
    IndexIVFStats* out = ivf_stats ? ivf_stats : &indexIVF_stats;
    out->nq += n;
    out->nlist += st[0];
    out->ndis += st[1];
    if (per_query_stats) {
        const double scan_us = StageEvents::ms(e0, e1) * 1e3;
        std::vector<unsigned long long> qd((size_t)n), sp(2);
        HIP_CHECK(hipMemcpy(qd.data(), s_qdone_.ptr, sizeof(unsigned long long) * n,
                            hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(sp.data(), s_stamps_.ptr, 2 * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost));
        const double ticks = (double)(sp[1] - sp[0]);
        const double us_per_tick = ticks > 0 ? scan_us / ticks : 0.01;
        for (idx_t i = 0; i < n; i++)
            per_query_stats[i].list_scan_us =
                    qd[i] >= sp[0] ? (double)(qd[i] - sp[0]) * us_per_tick : scan_us;
    }
}

void IndexIVF::search(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                      const SearchParameters* params) const {
    search_host(n, x, k, distances, labels, params, nullptr, true);
}

void IndexIVF::search_stats(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                            const SearchParameters* params,
                            QueryLatencyStats* per_query_stats) const {
    search_host(n, x, k, distances, labels, params, per_query_stats, false);
}

namespace {
// query pages of a host-buffer search: FAISS_AMD_HOST_PAGES=<P> (1 = one
// upload, one graph-replayed search, one download; 0 = the eager host path);
// by default up to 4 pages of >= 25000 queries: a device search of fewer
// queries does not take proportionally less time (c2's index, per call: 10k
// queries 1 page 0.62 ms, 2 pages 0.68; 50k 1.82 / 1.69; 100k 3.44 / 2.85,
// 4 pages 2.89; scripts/exp_host_pages_big.py).  A page
// keeps >= 20 queries, the flat quantizer's batch form
// (faiss/utils/distances.cpp:807-823), so every page computes the batch's
// coarse distances.
int host_pages(idx_t n) {
    const char* e = getenv("FAISS_AMD_HOST_PAGES");
    if (e && atoi(e) <= 0) return 0;
    const idx_t want = e ? atoi(e) : 4;
    const idx_t min_page = e ? 20 : 25000;
    return (int)std::max<idx_t>(1, std::min<idx_t>(want, n / min_page));
}
}  // namespace

// faiss/gpu/GpuIndex.cu:259,307-333 (searchFromCpuPaged_): host queries go
// to the device in pages, each page's upload overlapping the previous page's
// search; here the downloads overlap too.  Page i: upload on host_cs_ ->
// event up[i] -> the index stream waits and runs search_device on the page
// (a hipGraph replay from the third call on: one entry per page), then the
// page's list / distance counts into s_stats_ -> event done[i] -> host_cs_
// waits and downloads the page's results while page i + 1 searches.  The
// results are the whole batch's: every page is scanned exactly as the batch
// would be (per-query work only, the same coarse form).  Taken where the
// device search replays a graph (flat quantizer, no per-call parameters,
// max_codes 0, one slice, FAISS_AMD_GRAPH / FAISS_AMD_PIPE unset) and the
// batch fits one scratch chunk; otherwise false (the eager host path: an
// eager search per page costs more host time than the overlap saves).  One
// page is the upload, the replayed search and the download on two streams.
bool IndexIVF::search_host_paged(idx_t n, const float* x, idx_t k, float* distances,
                                 idx_t* labels, const SearchParameters* params_in,
                                 bool update_times) const {
    const auto* qf = dynamic_cast<const IndexFlat*>(quantizer);
    const char* genv = getenv("FAISS_AMD_GRAPH");
    if (!qf || params_in || max_codes != 0 || get_search_slices() > 1 ||
        (genv && !strcmp(genv, "0")) || getenv("FAISS_AMD_PIPE"))
        return false;
    const int P = host_pages(n);
    if (P < 1) return false;
    const size_t np = std::min(nlist, nprobe);
    if (search_chunk(n, np, k) < n) return false;
    DevGuard dg(device);
    sync_device();
    hipStream_t s = stream();
    const int ldx = ld();
    std::lock_guard<std::mutex> hg(host_mu_);
    std::lock_guard<std::recursive_mutex> g(mu_);
    DeviceBuffer &bx = h_x_, &bd = h_d_, &bi = h_i_;
    bx.reserve(sizeof(float) * n * ldx);
    bd.reserve(sizeof(float) * n * k);
    bi.reserve(sizeof(idx_t) * n * k);
    s_stats_.reserve(2 * sizeof(unsigned long long));
    if (!host_cs_ && P > 1) HIP_CHECK(hipStreamCreateWithFlags(&host_cs_, hipStreamNonBlocking));
    while ((int)host_ev_.size() < 2 * P + 1) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        host_ev_.push_back(e);
    }
    // one page: the copies on the index stream too (nothing to overlap)
    hipStream_t cs = P > 1 ? host_cs_ : s;
    HIP_CHECK(hipMemsetAsync(s_stats_.ptr, 0, 2 * sizeof(unsigned long long), s));
    if (cs != s) {
        // the copy stream writes h_x_ after the index stream's earlier work
        HIP_CHECK(hipEventRecord(host_ev_[2 * P], s));
        HIP_CHECK(hipStreamWaitEvent(cs, host_ev_[2 * P], 0));
    }
    std::vector<idx_t> b(P + 1);
    for (int i = 0; i <= P; i++) b[i] = n * i / P;
    auto h2d = [&](int i) {
        const idx_t r = b[i + 1] - b[i];
        float* dst = bx.as<float>() + b[i] * ldx;
        if (ldx != d) HIP_CHECK(hipMemsetAsync(dst, 0, sizeof(float) * r * ldx, cs));
        HIP_CHECK(hipMemcpy2DAsync(dst, sizeof(float) * ldx, x + b[i] * d, sizeof(float) * d,
                                   sizeof(float) * d, r, hipMemcpyHostToDevice, cs));
        if (cs != s) HIP_CHECK(hipEventRecord(host_ev_[i], cs));
    };
    auto d2h = [&](int i) {
        const idx_t r = b[i + 1] - b[i];
        if (cs != s) HIP_CHECK(hipStreamWaitEvent(cs, host_ev_[P + i], 0));
        HIP_CHECK(hipMemcpyAsync(distances + b[i] * k, bd.as<float>() + b[i] * k,
                                 sizeof(float) * r * k, hipMemcpyDeviceToHost, cs));
        HIP_CHECK(hipMemcpyAsync(labels + b[i] * k, bi.as<idx_t>() + b[i] * k,
                                 sizeof(idx_t) * r * k, hipMemcpyDeviceToHost, cs));
    };
    StageEvents ev;
    std::vector<hipEvent_t> pm, cm, cpage(P, nullptr);
    struct Reset {
        const IndexIVF* ix;
        std::vector<hipEvent_t>& cm;
        ~Reset() {
            ix->paged_marks_ = nullptr;
            for (auto e : cm) (void)hipEventDestroy(e);
        }
    } reset{this, cm};
    paged_marks_ = &cm;
    bool interrupted = false;
    int issued = 0;
    h2d(0);
    for (int i = 0; i < P; i++) {
        // InterruptCallback, polled before each page is queued
        // (faiss/IndexIVF.cpp:627, 707-713)
        if (i > 0 && InterruptCallback::is_interrupted()) {
            interrupted = true;
            break;
        }
        const idx_t r = b[i + 1] - b[i];
        if (cs != s) HIP_CHECK(hipStreamWaitEvent(s, host_ev_[i], 0));
        pm.push_back(ev.mark(s));
        const size_t m0 = cm.size();
        search_device(r, bx.as<float>() + b[i] * ldx, ldx, k, bd.as<float>() + b[i] * k,
                      bi.as<idx_t>() + b[i] * k, nullptr, s);
        if (cm.size() > m0) cpage[i] = cm.back();  // an eager run marked its coarse end
        pm.push_back(ev.mark(s));
        // the page's assignment is in s_ci_ (max_codes 0: the scan's own)
        kern::ivf_visit_stats(s_ci_.as<int32_t>(), r * (int64_t)np, d_list_len_.as<uint32_t>(),
                              (int)nlist, nullptr, s_stats_.as<unsigned long long>(), s);
        if (cs != s) HIP_CHECK(hipEventRecord(host_ev_[P + i], s));
        issued++;
        if (i + 1 < P) h2d(i + 1);
        if (i > 0) d2h(i - 1);
    }
    if (issued) d2h(issued - 1);
    unsigned long long st[2];
    HIP_CHECK(hipMemcpyAsync(st, s_stats_.ptr, sizeof(st), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (cs != s) HIP_CHECK(hipStreamSynchronize(cs));
    if (interrupted || InterruptCallback::is_interrupted()) FAISS_THROW_MSG("computation interrupted");
    quantizer->fold_device_stats();
    // stage times: a page searched eagerly marked its coarse stage's end;
    // a replayed page takes the coarse share of the last marked page
    double qms = 0, sms = 0;
    for (int i = 0; i < issued; i++) {
        const double t = StageEvents::ms(pm[2 * i], pm[2 * i + 1]);
        if (cpage[i] && t > 0) paged_qshare_ = StageEvents::ms(pm[2 * i], cpage[i]) / t;
        qms += t * paged_qshare_;
        sms += t * (1.0 - paged_qshare_);
    }
    indexIVF_stats.nq += n;
    indexIVF_stats.nlist += st[0];
    indexIVF_stats.ndis += st[1];
    if (update_times) {
        indexIVF_stats.quantization_time += qms;
        indexIVF_stats.search_time += qms + sms;
    }
    return true;
}

// faiss/IndexIVF.cpp:303-397 and :725-867 on one slice (the whole batch):
// coarse stage, scan stage, stats.  update_times: search() adds the stage
// times to indexIVF_stats (search_stats() does not, like the reference).
void IndexIVF::search_host(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                           const SearchParameters* params_in,
                           QueryLatencyStats* per_query_stats, bool update_times) const {
    FAISS_THROW_IF_NOT(k > 0);
    if (per_query_stats) memset(per_query_stats, 0, sizeof(QueryLatencyStats) * n);
    const SearchParametersIVF* params = nullptr;
    if (params_in) {
        params = dynamic_cast<const SearchParametersIVF*>(params_in);
        FAISS_THROW_IF_NOT_MSG(params, "IndexIVF params have incorrect type");
    }
    const size_t np = std::min(nlist, params && params->nprobe ? params->nprobe : nprobe);
    FAISS_THROW_IF_NOT(np > 0);
    check_parallel_mode(parallel_mode);
    const size_t mc = params ? params->max_codes : max_codes;
    if (n == 0) return;
    if (!per_query_stats && search_host_paged(n, x, k, distances, labels, params_in, update_times))
        return;
    DevGuard dg(device);
    sync_device();
    hipStream_t s = stream();
    const int ldx = ld();
    std::lock_guard<std::mutex> hg(host_mu_);
    DeviceBuffer &bx = h_x_, &bd = h_d_, &bi = h_i_;
    bx.reserve(sizeof(float) * n * ldx);
    bd.reserve(sizeof(float) * n * k);
    bi.reserve(sizeof(idx_t) * n * k);
    if (ldx != d) HIP_CHECK(hipMemsetAsync(bx.ptr, 0, sizeof(float) * n * ldx, s));
    HIP_CHECK(hipMemcpy2DAsync(bx.ptr, sizeof(float) * ldx, x, sizeof(float) * d,
                               sizeof(float) * d, n, hipMemcpyHostToDevice, s));
    const idx_t qchunk = search_chunk(n, np, k);
    std::lock_guard<std::recursive_mutex> g(mu_);
    s_cd_.reserve(sizeof(float) * qchunk * np);
    s_ci_.reserve(sizeof(int32_t) * qchunk * np);
    s_stats_.reserve(2 * sizeof(unsigned long long));
    HIP_CHECK(hipMemsetAsync(s_stats_.ptr, 0, 2 * sizeof(unsigned long long), s));
    StageEvents ev;
    std::vector<hipEvent_t> marks;
    const uint8_t* selm = apply_selector(params, s);
    // search_stats: device-clock stamps (s_memrealtime) at the batch's first
    // and last stage boundary (their HIP events calibrate the clock), at each
    // chunk's scan start, and per query where its result is emitted
    const idx_t nch = (n + qchunk - 1) / qchunk;
    unsigned long long* stamps = nullptr;
    if (per_query_stats) {
        s_qdone_.reserve(sizeof(unsigned long long) * n);
        HIP_CHECK(hipMemsetAsync(s_qdone_.ptr, 0, sizeof(unsigned long long) * n, s));
        s_stamps_.reserve(sizeof(unsigned long long) * (nch + 2));
        stamps = s_stamps_.as<unsigned long long>();
    }
    struct ResetQ {
        unsigned long long*& p;
        ~ResetQ() { p = nullptr; }
    } reset_q{qdone_};
    // InterruptCallback: polled before each chunk is queued and once the
    // batch is done; when it fires the remaining chunks are not queued and
    // the call throws after draining the queued ones (faiss/IndexIVF.cpp:627,
    // 707-713)
    bool interrupted = false;
    for (idx_t q0 = 0, c = 0; q0 < n; q0 += qchunk, c++) {
        if (c > 0 && InterruptCallback::is_interrupted()) {
            interrupted = true;
            break;
        }
        const idx_t nq = std::min(qchunk, n - q0);
        marks.push_back(ev.mark(s));
        if (stamps && c == 0) kern::device_stamp(stamps, s);
        quantize_device(nq, bx.as<float>() + q0 * ldx, ldx, (int)np, s_cd_.as<float>(),
                        s_ci_.as<int32_t>(), params ? params->quantizer_params : nullptr, s);
        marks.push_back(ev.mark(s));
        if (stamps) {
            kern::device_stamp(stamps + 2 + c, s);
            qdone_ = s_qdone_.as<unsigned long long>() + q0;
        }
        const uint32_t* lim = nullptr;
        const int32_t* asg = apply_max_codes(nq, (int)np, s_ci_.as<int32_t>(), mc, &lim, s);
        search_preassigned_device(nq, bx.as<float>() + q0 * ldx, ldx, k, (int)np, asg,
                                  s_cd_.as<float>(), bd.as<float>() + q0 * k,
                                  bi.as<idx_t>() + q0 * k, s, lim, selm);
        qdone_ = nullptr;
        if (stamps && q0 + nq == n) kern::device_stamp(stamps + 1, s);
        marks.push_back(ev.mark(s));
        kern::ivf_visit_stats(asg, nq * (int64_t)np, d_list_len_.as<uint32_t>(), (int)nlist,
                              lim, s_stats_.as<unsigned long long>(), s);
    }
    unsigned long long st[2];
    HIP_CHECK(hipMemcpyAsync(distances, bd.ptr, sizeof(float) * n * k, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(labels, bi.ptr, sizeof(idx_t) * n * k, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(st, s_stats_.ptr, sizeof(st), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (interrupted || InterruptCallback::is_interrupted()) FAISS_THROW_MSG("computation interrupted");
    quantizer->fold_device_stats();
    double qms = 0, sms = 0;
    for (size_t c = 0; c + 2 < marks.size(); c += 3) {
        qms += StageEvents::ms(marks[c], marks[c + 1]);
        sms += StageEvents::ms(marks[c + 1], marks[c + 2]);
    }
    indexIVF_stats.nq += n;
    indexIVF_stats.nlist += st[0];
    indexIVF_stats.ndis += st[1];
    if (update_times) {
        indexIVF_stats.quantization_time += qms;
        indexIVF_stats.search_time += qms + sms;
    }
    if (per_query_stats) {
        // faiss/IndexIVF.cpp:760-777, 1062-1107: quantization_us is the
        // coarse stage's time amortised over the chunk's queries;
        // list_scan_us runs from the chunk's scan start to the query's
        // result on the device clock (its completion latency in the batch)
        std::vector<unsigned long long> qd((size_t)n), sp((size_t)nch + 2);
        HIP_CHECK(hipMemcpy(qd.data(), s_qdone_.ptr, sizeof(unsigned long long) * n,
                            hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(sp.data(), s_stamps_.ptr, sizeof(unsigned long long) * (nch + 2),
                            hipMemcpyDeviceToHost));
        const double span_us = StageEvents::ms(marks.front(), marks.back()) * 1e3;
        const double ticks = (double)(sp[1] - sp[0]);
        const double us_per_tick = ticks > 0 ? span_us / ticks : 0.01;  // 100 MHz nominal
        for (idx_t q0 = 0, c = 0; q0 < n; q0 += qchunk, c++) {
            const idx_t nq = std::min(qchunk, n - q0);
            const double qus = StageEvents::ms(marks[3 * c], marks[3 * c + 1]) * 1e3 / nq;
            const double sus_all = StageEvents::ms(marks[3 * c + 1], marks[3 * c + 2]) * 1e3;
            for (idx_t i = q0; i < q0 + nq; i++) {
                double sus = qd[i] >= sp[2 + c] ? (double)(qd[i] - sp[2 + c]) * us_per_tick
                                                : sus_all;
                per_query_stats[i].quantization_us = qus;
                per_query_stats[i].list_scan_us = sus;
                per_query_stats[i].total_us = qus + sus;
            }
        }
    }
}

// ---------------------------------------------------------------- IVFFlat
IndexIVFFlat::IndexIVFFlat(Index* q, size_t d_, size_t nl, MetricType metric)
        : IndexIVF(q, d_, nl, sizeof(float) * d_, metric) {
    by_residual = false;  // faiss/IndexIVFFlat.cpp:37-39
}

void IndexIVFFlat::encode_vectors(idx_t n, const float* x, const idx_t*, uint8_t* codes) const {
    memcpy(codes, x, sizeof(float) * n * d);
}

void IndexIVFFlat::reconstruct(idx_t key, float* recons) const {
    for (size_t l = 0; l < nlist; l++) {
        const idx_t* ids = invlists->get_ids(l);
        for (size_t i = 0; i < invlists->list_size(l); i++)
            if (ids[i] == key) {
                memcpy(recons, invlists->get_codes(l) + i * code_size, code_size);
                return;
            }
    }
    FAISS_THROW_MSG("key not found");
}

const void* IndexIVFFlat::stream_image(size_t* row_bytes) const {
    if (!d_cbs_.ptr || arena_rows_ == 0) return nullptr;
    *row_bytes = 2 * (size_t)(kern::bf3_db_host(d) / 2 * 2) + 16;
    return d_cbs_.ptr;
}

void IndexIVFFlat::upload_extra() const {
    hipStream_t s = stream();
    const int l = (int)roundup((size_t)d, 4);
    d_ynorm_.reserve(sizeof(float) * std::max<size_t>(arena_rows_, 1));
    d_ynmax_.reserve(sizeof(float) * std::max<size_t>(nlist, 1));
    if (arena_rows_ > 0) {
        kern::row_norms(d_codes_.as<float>(), arena_rows_, d, l, d_ynorm_.as<float>(), s);
        kern::pad_rows_inf(d_ynorm_.as<float>(), d_row_list_.as<uint32_t>(), arena_rows_, s);
    }
    kern::ivf_list_ynmax(d_ynorm_.as<float>(), d_list_off_.as<uint32_t>(),
                         d_list_len_.as<uint32_t>(), (int)nlist, d_ynmax_.as<float>(), s);
    // bf16 hi/lo image of the arena for the MFMA filter (same bytes as f32)
    if (kern::ivf_mfma_kq(1, d) > 0) {
        const int DB = kern::bf3_db_host(d);
        d_cbf_.reserve(std::max<size_t>(arena_rows_, 1) * 2 * DB * 2);
        kern::split_bf16(d_codes_.as<float>(), arena_rows_, d, l, DB, d_cbf_.ptr, s);
        d_rres_.reserve(sizeof(float) * std::max<size_t>(arena_rows_, 1));
        d_rmax_.reserve(sizeof(float) * std::max<size_t>(nlist, 1));
        kern::row_resnorm_bf16(d_codes_.as<float>(), arena_rows_, d, l, d_rres_.as<float>(), s);
        // the streamed filter's image: bf16 hi + norm per row (2 DB + 16 bytes)
        const int DBs = kern::bf3_db_host(d) / 2 * 2;
        d_cbs_.reserve(std::max<size_t>(arena_rows_, 1) * (2 * (size_t)DBs + 16));
        // L2: the norms enter the filter's MFMA as a bias k-step (fold image;
        // FAISS_AMD_IVF_FOLD=0 keeps the fp32-norm tail and the fma epilogue)
        const char* fenv = getenv("FAISS_AMD_IVF_FOLD");
        fold_ = (metric_type == METRIC_L2 && !(fenv && !strcmp(fenv, "0"))) ? 1 : 0;
        kern::split_bf16_stream(d_codes_.as<float>(), arena_rows_, d, l, DBs,
                                d_ynorm_.as<float>(), d_row_list_.as<uint32_t>(), d_cbs_.ptr, s,
                                fold_);
        kern::ivf_list_ynmax(d_rres_.as<float>(), d_list_off_.as<uint32_t>(),
                             d_list_len_.as<uint32_t>(), (int)nlist, d_rmax_.as<float>(), s);
        size_t mx = 0;
        for (size_t li = 0; li < nlist; li++) mx = std::max(mx, invlists->list_size(li));
        obits_ = kern::ivf_bf3_obits((uint32_t)std::min<size_t>(mx, 0xffffffffu));
    }
}

void IndexIVFFlat::search_preassigned_device(idx_t n, const float* x, int ldx, idx_t k, int np,
                                             const int32_t* assign, const float* cdis,
                                             float* distances, idx_t* labels, hipStream_t s,
                                             const uint32_t* lim, const uint8_t* sel,
                                             bool store_pairs) const {
    if (n <= 0) return;
    sync_device();
    const char* env = getenv("FAISS_AMD_IVF_SCAN");
    int mode = scan_mode;
    if (env && !strcmp(env, "exact")) mode = 1;
    if (env && !strcmp(env, "mfma")) mode = 0;
    // long lists (>= 512 rows on average, nprobe <= 64): 8 keys per filter
    // thread stream, so a stream of ~1/4 of a list rarely drops a key that
    // may reach the top k (c4, 610 rows per list: failing probes 0.029 -> 0
    // per query, overflowing queries 105 -> 0; step 2.29 -> 2.21 ms; c2's
    // 244-row lists measured slower with 8: 0.291 -> 0.311 ms)
    const int ktm = np <= 64 && nlist > 0 && ntotal / (idx_t)nlist >= 512 ? 8 : 0;
    const int KQ = obits_ <= 14 ? kern::ivf_mfma_kq((int)k, d, np, ktm) : 0;
    if (mode != 0 || KQ <= 0 || np > kern::kMaxNprobeFilter || store_pairs || dup_probes_) {
        exact_scan_device(n, x, ldx, k, np, assign, cdis, distances, labels, s, lim, sel,
                          store_pairs);
        return;
    }
    std::lock_guard<std::recursive_mutex> g(mu_);
    const int QT = kern::IVF_FLAT_QT;
    const int l = (int)roundup((size_t)d, 4);
    uint32_t* counts_next = nullptr;
    uint32_t* counts = bucket_counts(s, &counts_next);
    s_cur_.reserve(sizeof(uint32_t) * std::max<idx_t>(n * np, 1));
    s_boff_.reserve(sizeof(uint32_t) * (nlist + 1));
    s_ioff_.reserve(sizeof(uint32_t) * (nlist + 1));
    s_ent_.reserve(sizeof(uint32_t) * n * np);
    kern::IVFBuckets b{counts, s_boff_.as<uint32_t>(), s_ioff_.as<uint32_t>(),
                       s_cur_.as<uint32_t>(), s_ent_.as<uint32_t>()};
    b.counts_next = counts_next;
    b.lim = lim;
    b.sel = sel;
    b.perm = d_list_perm_.as<uint32_t>();
    s_part_.reserve(sizeof(uint32_t) * n * np * KQ);  // raw filter keys
    s_pk2_.reserve(sizeof(kern::ProbeRec) * n * np);  // per-probe records
    b.mark_keys = s_part_.as<uint32_t>();
    b.mark_recs = s_pk2_.as<kern::ProbeRec>();
    b.mark_ke = KQ;
    const int64_t max_items = kern::ivf_max_items(n, np, (int)nlist, QT);
    s_idesc_.reserve(sizeof(kern::ItemDesc) * max_items);
    s_ient_.reserve(sizeof(uint32_t) * max_items * QT);
    b.item_desc = s_idesc_.as<kern::ItemDesc>();
    b.item_entries = s_ient_.as<uint32_t>();
    s_ictr_.reserve(16 + 4 * 3 * 64);
    b.item_ctr = s_ictr_.as<uint32_t>();
    b.scan_tmp = s_ictr_.as<uint32_t>() + 4;
    {
        ScopedKernelTimer tb(&ktimes, "ivf_bucket", 0.0, s);
        kern::ivf_bucket(assign, n, np, d_list_len_.as<uint32_t>(), d_list_off_.as<uint32_t>(),
                         (int)nlist, QT, b, s);
    }
    flip_counts();
    const bool l2 = metric_type == METRIC_L2;
    s_flags_.reserve(sizeof(uint32_t) * std::max<idx_t>(n, 4));
    const bool dbg = getenv("FAISS_AMD_IVF_STATS") != nullptr;
    if (dbg) HIP_CHECK(hipMemsetAsync(s_flags_.ptr, 0, 4 * sizeof(uint32_t), s));
    // query image + |x|^2: the quantizer's when this is search()'s chunk
    const void* qready = shared_qimg_;
    if (!qready) s_q_.reserve(kern::query_image_bytes(n, d) + sizeof(float) * n);
    kern::ivf_flat_scan_mfma(x, ldx, d_codes_.as<float>(), l, d_cbf_.ptr, d_ids_.as<int64_t>(),
                             d_ynorm_.as<float>(), d_ynmax_.as<float>(), d_rres_.as<float>(),
                             d_rmax_.as<float>(), d_list_off_.as<uint32_t>(),
                             d_list_len_.as<uint32_t>(), (int)nlist, d, obits_, n, np, (int)k, l2,
                             b, max_items, s_part_.as<uint32_t>(), s_pk2_.as<kern::ProbeRec>(),
                             dbg ? s_flags_.as<uint32_t>() : nullptr, distances, labels, &ktimes,
                             s, kern::ARENA_ALIGN, d_cbs_.ptr,
                             qready ? const_cast<void*>(qready) : s_q_.ptr, qready != nullptr,
                             qdone_, fold_, ktm);
    if (dbg) {
        uint32_t st[4];
        HIP_CHECK(hipMemcpyAsync(st, s_flags_.ptr, sizeof(st), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        fprintf(stderr,
                "[faiss_amd] ivf mfma scan: nq=%lld survivors/q=%.2f failing probes/q=%.4f "
                "overflow queries=%u general-resolve queries=%u\n",
                (long long)n, st[0] / (double)n, st[1] / (double)n, st[2], st[3]);
    }
}

void IndexIVFFlat::exact_args(void* p) const {
    auto& a = *(kern::ExactScanArgs*)p;
    a.codes = d_codes_.as<float>();
    a.ldc = (int)roundup((size_t)d, 4);
}

// general exact scan: chunks of queries whose candidate keys fit the scratch
void IndexIVF::exact_scan_device(idx_t n, const float* x, int ldx, idx_t k, int np,
                                 const int32_t* assign, const float* cdis, float* distances,
                                 idx_t* labels, hipStream_t s, const uint32_t* lim,
                                 const uint8_t* sel, bool store_pairs) const {
    FAISS_THROW_IF_NOT_FMT(k >= 1 && k <= kern::kMaxKExact, "k = %lld must be in [1, %d]",
                           (long long)k, kern::kMaxKExact);
    std::lock_guard<std::recursive_mutex> g(mu_);
    int64_t cap = 0;
    const idx_t qc = kern::ivf_exact_chunk(n, np, max_list_len_, &cap);
    s_ex_eoff_.reserve(sizeof(uint32_t) * qc * np);
    s_ex_tot_.reserve(sizeof(uint32_t) * qc);
    s_ex_keys_.reserve(sizeof(uint32_t) * qc * cap);
    s_ex_rows_.reserve(sizeof(uint32_t) * qc * cap);
    kern::ExactScanArgs a;
    exact_args(&a);
    a.ldx = ldx;
    a.d = d;
    a.np = np;
    a.k = (int)k;
    a.l2 = metric_type == METRIC_L2;
    a.list_off = d_list_off_.as<uint32_t>();
    a.list_len = d_list_len_.as<uint32_t>();
    a.nlist = (int)nlist;
    a.sel = sel;
    a.ids = d_ids_.as<int64_t>();
    a.row_list = d_row_list_.as<uint32_t>();
    a.store_pairs = store_pairs ? 1 : 0;
    ScopedKernelTimer tm(&ktimes, "ivf_exact_scan", 0.0, s);
    for (idx_t q0 = 0; q0 < n; q0 += qc) {
        a.n = std::min(qc, n - q0);
        a.x = x + q0 * ldx;
        a.assign = assign + q0 * np;
        a.cdis = cdis ? cdis + q0 * np : nullptr;
        a.lim = lim ? lim + q0 * np : nullptr;
        a.qdone = qdone_ ? qdone_ + q0 : nullptr;
        kern::ivf_exact_search(a, s_ex_eoff_.as<uint32_t>(), s_ex_tot_.as<uint32_t>(),
                               s_ex_keys_.as<uint32_t>(), s_ex_rows_.as<uint32_t>(), cap,
                               distances + q0 * k, labels + q0 * k, s);
    }
}

// ---------------------------------------------------------------- PQ
ProductQuantizer::ProductQuantizer(size_t d_, size_t M_, size_t nbits_)
        : d(d_), M(M_), nbits(nbits_) {
    set_derived_values();
}
void ProductQuantizer::set_derived_values() {
    FAISS_THROW_IF_NOT_MSG(M > 0 && d % M == 0,
                           "The dimension of the vector (d) should be a multiple of the number "
                           "of subquantizers (M)");
    dsub = d / M;
    ksub = (size_t)1 << nbits;
    centroids.resize(d * ksub);
}

IndexIVFPQ::IndexIVFPQ(Index* q, size_t d_, size_t nl, size_t M, size_t nbits, MetricType metric)
        : IndexIVF(q, d_, nl, 0, metric), pq(d_, M, nbits) {
    FAISS_THROW_IF_NOT_MSG(nbits == 8, "only nbits = 8 is supported on this path");
    code_size = M;  // (M * nbits + 7) / 8
    invlists = std::make_unique<ArrayInvertedLists>(nlist, code_size);
    by_residual = true;
    is_trained = false;
}

void IndexIVFPQ::train_encoder(idx_t n, const float* x, const idx_t* assign) {
    // faiss/IndexIVFPQ.cpp:61-131: residuals, ProductQuantizer::train per
    // sub-space, then precompute_table()
    const idx_t max_train = (idx_t)pq.ksub * 256;
    const idx_t nt = std::min(n, max_train);
    std::vector<float> resid((size_t)nt * d);
    std::vector<float> c(d);
    for (idx_t i = 0; i < nt; i++) {
        const float* xi = x + (size_t)i * d;
        float* ri = resid.data() + (size_t)i * d;
        if (by_residual && assign[i] >= 0) {
            quantizer->reconstruct(assign[i], c.data());
            for (int j = 0; j < d; j++) ri[j] = xi[j] - c[j];
        } else {
            memcpy(ri, xi, sizeof(float) * d);
        }
    }
    std::vector<float> sub((size_t)nt * pq.dsub), cent(pq.ksub * pq.dsub);
    for (size_t m = 0; m < pq.M; m++) {
        for (idx_t i = 0; i < nt; i++)
            memcpy(sub.data() + (size_t)i * pq.dsub, resid.data() + (size_t)i * d + m * pq.dsub,
                   sizeof(float) * pq.dsub);
        kmeans_train((int)pq.dsub, nt, sub.data(), (int)pq.ksub, 25, 1234 + (int64_t)m,
                     cent.data(), device, false);
        memcpy(pq.centroids.data() + m * pq.ksub * pq.dsub, cent.data(),
               sizeof(float) * pq.ksub * pq.dsub);
    }
    precompute_table();
    std::lock_guard<std::recursive_mutex> g(mu_);
    dirty_ = true;
}

void IndexIVFPQ::precompute_table() {
    // faiss/IndexIVFPQ.cpp:380-406 decision rule (2 GiB limit)
    use_precomputed_table = 0;
    if (metric_type == METRIC_L2 && by_residual) {
        size_t table_size = pq.M * pq.ksub * nlist * sizeof(float);
        use_precomputed_table = table_size > ((size_t)1 << 31) ? 0 : 1;
    }
}

void IndexIVFPQ::encode_vectors(idx_t n, const float* x, const idx_t* list_nos,
                                uint8_t* codes) const {
    if (n <= 0) return;
    DevGuard dg(device);
    hipStream_t s = stream();
    const int ldx = ld();
    const int cs = device_code_stride();
    std::vector<int32_t> a32(n);
    for (idx_t i = 0; i < n; i++) a32[i] = (int32_t)std::max<idx_t>(list_nos[i], 0);
    std::vector<float> cent((size_t)nlist * ldx, 0.f);
    if (by_residual)
        for (size_t l = 0; l < nlist; l++) quantizer->reconstruct(l, cent.data() + l * ldx);
    DeviceBuffer bx, ba, bc, bp, bo;
    bx.reserve(sizeof(float) * n * ldx);
    ba.reserve(sizeof(int32_t) * n);
    bc.reserve(sizeof(float) * cent.size());
    bp.reserve(sizeof(float) * pq.centroids.size());
    bo.reserve((size_t)n * cs);
    if (ldx != d) HIP_CHECK(hipMemsetAsync(bx.ptr, 0, sizeof(float) * n * ldx, s));
    HIP_CHECK(hipMemcpy2DAsync(bx.ptr, sizeof(float) * ldx, x, sizeof(float) * d,
                               sizeof(float) * d, n, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(ba.ptr, a32.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(bc.ptr, cent.data(), sizeof(float) * cent.size(),
                             hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(bp.ptr, pq.centroids.data(), sizeof(float) * pq.centroids.size(),
                             hipMemcpyHostToDevice, s));
    kern::pq_encode(bx.as<float>(), ldx, n, ba.as<int32_t>(),
                    by_residual ? bc.as<float>() : nullptr, ldx, bp.as<float>(), (int)pq.M,
                    (int)pq.ksub, (int)pq.dsub, bo.as<uint8_t>(), s);
    std::vector<uint8_t> hc((size_t)n * cs);
    HIP_CHECK(hipMemcpyAsync(hc.data(), bo.ptr, hc.size(), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    for (idx_t i = 0; i < n; i++) memcpy(codes + (size_t)i * code_size, hc.data() + (size_t)i * cs,
                                         code_size);
}

const void* IndexIVFPQ::stream_image(size_t* row_bytes) const {
    if (!pq_stream_ready_ || !d_pcbs_.ptr) return nullptr;
    *row_bytes = 2 * (size_t)kern::bf3_db_host(d) + 16;
    return d_pcbs_.ptr;
}

void IndexIVFPQ::upload_extra() const {
    hipStream_t s = stream();
    const int ldc = ld();
    std::vector<float> cent((size_t)nlist * ldc, 0.f);
    for (size_t l = 0; l < nlist; l++) quantizer->reconstruct(l, cent.data() + l * ldc);
    d_pq_.reserve(sizeof(float) * pq.centroids.size());
    d_cent_.reserve(sizeof(float) * cent.size());
    d_terms_.reserve(sizeof(float) * std::max<size_t>(arena_rows_, 1));
    HIP_CHECK(hipMemcpyAsync(d_pq_.ptr, pq.centroids.data(), sizeof(float) * pq.centroids.size(),
                             hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_cent_.ptr, cent.data(), sizeof(float) * cent.size(),
                             hipMemcpyHostToDevice, s));
    if (by_residual && arena_rows_ > 0)
        kern::ivfpq_terms(d_codes_.as<uint8_t>(), d_row_list_.as<uint32_t>(), arena_rows_,
                          d_cent_.as<float>(), ldc, d_pq_.as<float>(), (int)pq.M, (int)pq.ksub,
                          (int)pq.dsub, d_terms_.as<float>(), s);
    // list-centric MFMA scan: decode table, row / list norms (any k, nprobe)
    pq_mfma_ready_ = false;
    if (by_residual && metric_type == METRIC_L2 && pq.ksub == 256 &&
        kern::ivfpq_mfma_eligible(d, (int)pq.M, 1, 1) && arena_rows_ > 0) {
        const size_t rows = arena_rows_;
        d_dec_.reserve(sizeof(uint16_t) * pq.centroids.size());
        d_prn_.reserve(sizeof(float) * rows);
        d_prr_.reserve(sizeof(float) * rows);
        d_lRmax_.reserve(sizeof(float) * nlist);
        d_lrmax_.reserve(sizeof(float) * nlist);
        d_cnorm_.reserve(sizeof(float) * nlist);
        kern::pq_decode_prep(d_pq_.as<float>(), (int)pq.M, (int)pq.dsub, d_codes_.as<uint8_t>(),
                             device_code_stride(), (int64_t)rows, d_dec_.ptr, d_prn_.as<float>(),
                             d_prr_.as<float>(), s);
        kern::ivf_list_ynmax(d_prn_.as<float>(), d_list_off_.as<uint32_t>(),
                             d_list_len_.as<uint32_t>(), (int)nlist, d_lRmax_.as<float>(), s);
        kern::ivf_list_ynmax(d_prr_.as<float>(), d_list_off_.as<uint32_t>(),
                             d_list_len_.as<uint32_t>(), (int)nlist, d_lrmax_.as<float>(), s);
        std::vector<float> cn(nlist);
        for (size_t l = 0; l < nlist; l++) {
            double a = 0.0;
            for (int j = 0; j < d; j++) a += (double)cent[l * ldc + j] * cent[l * ldc + j];
            cn[l] = (float)(std::sqrt(a) * (1.0 + 1e-6));
        }
        HIP_CHECK(hipMemcpyAsync(d_cnorm_.ptr, cn.data(), sizeof(float) * nlist,
                                 hipMemcpyHostToDevice, s));
        size_t mx = 0;
        for (size_t li = 0; li < nlist; li++) mx = std::max(mx, invlists->list_size(li));
        pq_obits_ = kern::ivf_bf3_obits((uint32_t)std::min<size_t>(mx, 0xffffffffu));
        pq_mfma_ready_ = pq_obits_ <= 14;
        // the streamed filter's image (by-residual terms in the bias tail):
        // only on request (FAISS_AMD_PQ_FILTER=image at upload) — the default
        // filter gathers the same bf16 values from the codes (4.3-8.5x less
        // HBM per row than the image)
        pq_stream_ready_ = false;
        const char* ienv = getenv("FAISS_AMD_PQ_FILTER");
        d_pcbs_.release();
        // (round 6: no size cap.  The round-5 100M-row wrong keys were the
        // image builder's launch of rows x (DB + 8) work-items, past the
        // dispatch's 32-bit count; it is grid-strided now, common.h kgrid)
        if (pq_mfma_ready_ && ienv && !strcmp(ienv, "image") &&
            kern::ivfpq_stream_eligible(d, (int)pq.M, 1, 1)) {
            const int DB = kern::bf3_db_host(d);
            d_pcbs_.reserve(rows * (2 * (size_t)DB + 16));
            kern::pq_stream_image(d_codes_.as<uint8_t>(), device_code_stride(), (int64_t)rows, d,
                                  (int)pq.dsub, d_pq_.as<float>(), d_terms_.as<float>(),
                                  d_row_list_.as<uint32_t>(), DB, d_pcbs_.ptr, s);
            pq_stream_ready_ = true;
        }
        HIP_CHECK(hipStreamSynchronize(s));  // cn is a host temporary
        // the per-row norms only fed the list maxima: per row the index keeps
        // its codes, id, term and list number (code_size + 16 bytes)
        d_prn_.release();
        d_prr_.release();
    }
}

void IndexIVFPQ::search_preassigned_device(idx_t n, const float* x, int ldx, idx_t k, int np,
                                           const int32_t* assign, const float* centroid_dis,
                                           float* distances, idx_t* labels, hipStream_t s,
                                           const uint32_t* lim, const uint8_t* sel,
                                           bool store_pairs) const {
    if (n <= 0) return;
    sync_device();
    FAISS_THROW_IF_NOT_MSG(centroid_dis || !(by_residual && metric_type == METRIC_L2 &&
                                             use_precomputed_table == 1),
                           "IVF-PQ with precomputed tables needs centroid_dis");
    // list-centric bf16 MFMA filter + exact re-rank in the reference's table
    // arithmetic (default where eligible; FAISS_AMD_PQ_SCAN=exact forces the
    // general exact scan, which serves every other geometry)
    const char* penv = getenv("FAISS_AMD_PQ_SCAN");
    const bool force_exact = penv && !strcmp(penv, "exact");
    if (!force_exact && !store_pairs && !dup_probes_ && pq_mfma_ready_ && metric_type == METRIC_L2 &&
        by_residual && kern::ivfpq_mfma_eligible(d, (int)pq.M, (int)k, np)) {
        std::lock_guard<std::recursive_mutex> g(mu_);
        // the streamed filter over the PQ stream image (default where
        // eligible; FAISS_AMD_PQ_FILTER=decode keeps the in-loop decode filter
        // k_ivfpq_filter_w, which also serves IDSelectors)
        const char* fenv = getenv("FAISS_AMD_PQ_FILTER");
        // filters (both need the query image: the flat quantizer's, or one
        // prepared below for 16-B aligned rows):
        //  * default (and IDSelectors): k_ivfpq_filter_w, the codes streamed
        //    from HBM and each row's A fragments gathered from the decode
        //    table in the LDS (FAISS_AMD_PQ_FILTER=wg: its 4-wave group form);
        //  * image (FAISS_AMD_PQ_FILTER=image both when the index is uploaded
        //    and when it is searched): the streamed Flat filter over a decoded
        //    bf16 image of the residuals (4.3-8.5x the codes' bytes)
        const bool qimg_ok = shared_qimg_ != nullptr || ldx % 4 == 0;
        const bool stream = pq_stream_ready_ && !sel && fenv && !strcmp(fenv, "image") &&
                            qimg_ok && kern::ivfpq_stream_eligible(d, (int)pq.M, (int)k, np);
        const int QT = stream ? kern::IVF_FLAT_QT : 64;
        // folded-bias keys: the image filter and k_ivfpq_filter_w (not its
        // 4-wave group form, FAISS_AMD_PQ_FILTER=wg)
        const bool pq_fold = stream || !(fenv && !strcmp(fenv, "wg"));
        uint32_t* counts_next = nullptr;
        uint32_t* counts = bucket_counts(s, &counts_next);
        s_cur_.reserve(sizeof(uint32_t) * std::max<idx_t>(n * np, 1));
        s_boff_.reserve(sizeof(uint32_t) * (nlist + 1));
        s_ioff_.reserve(sizeof(uint32_t) * (nlist + 1));
        s_ent_.reserve(sizeof(uint32_t) * n * np);
        kern::IVFBuckets b{counts, s_boff_.as<uint32_t>(), s_ioff_.as<uint32_t>(),
                           s_cur_.as<uint32_t>(), s_ent_.as<uint32_t>()};
        s_ictr_.reserve(16 + 4 * 3 * 64);
        b.item_ctr = s_ictr_.as<uint32_t>();  // the PQ filter's work counter
        b.scan_tmp = s_ictr_.as<uint32_t>() + 4;
        b.counts_next = counts_next;
        b.lim = lim;
        b.sel = sel;
        b.perm = d_list_perm_.as<uint32_t>();
        const int KE = kern::ivf_mfma_kq((int)k, d, np);
        s_pkeys_.reserve(sizeof(uint32_t) * n * np * KE);
        s_precs_.reserve(sizeof(kern::ProbeRec) * n * np);
        b.mark_keys = s_pkeys_.as<uint32_t>();
        b.mark_recs = s_precs_.as<kern::ProbeRec>();
        b.mark_ke = KE;
        const int64_t mi = kern::ivf_max_items(n, np, (int)nlist, QT);
        s_idesc_.reserve(sizeof(kern::ItemDesc) * mi);
        s_ient_.reserve(sizeof(uint32_t) * mi * QT);
        b.item_desc = s_idesc_.as<kern::ItemDesc>();
        b.item_entries = s_ient_.as<uint32_t>();
            {
            ScopedKernelTimer tb(&ktimes, "ivf_bucket", 0.0, s);
            kern::ivf_bucket(assign, n, np, d_list_len_.as<uint32_t>(),
                             d_list_off_.as<uint32_t>(), (int)nlist, QT, b, s);
        }
        flip_counts();
        const bool dbg = getenv("FAISS_AMD_IVF_STATS") != nullptr;
        s_pflags_.reserve(4 * sizeof(uint32_t));
        if (dbg) HIP_CHECK(hipMemsetAsync(s_pflags_.ptr, 0, 4 * sizeof(uint32_t), s));
        int KT = 0;
        // query image: the flat quantizer's when this is search()'s chunk,
        // else prepared here (one launch instead of a split per work item)
        const void* qimg = shared_qimg_;
        if (!qimg && ldx % 4 == 0) {
            s_q_.reserve(kern::query_image_bytes(n, d) + sizeof(float) * n);
            kern::query_prep(x, n, ldx, d, nullptr, s_q_.ptr,
                             (float*)((uint8_t*)s_q_.ptr + kern::query_image_bytes(n, d)), s);
            qimg = s_q_.ptr;
        }
        const float* qxn =
                qimg ? (const float*)((const uint8_t*)qimg + kern::query_image_bytes(n, d)) : nullptr;
        {
            ScopedKernelTimer tm(&ktimes, "ivfpq_filter", 0.0, s);
            if (stream)
                kern::ivfpq_stream_filter(x, ldx, d, (int)pq.M, d_pcbs_.ptr, centroid_dis,
                                          d_cnorm_.as<float>(), d_lrmax_.as<float>(),
                                          d_lRmax_.as<float>(), (int)nlist, n, np, (int)k,
                                          pq_obits_, b, mi, s_pkeys_.as<uint32_t>(),
                                          s_precs_.as<kern::ProbeRec>(), &KT, s, qimg, qxn);
            else
                kern::ivfpq_filter(x, ldx, d, (int)pq.M, d_dec_.ptr, d_codes_.as<uint8_t>(),
                                   d_terms_.as<float>(), centroid_dis, d_cnorm_.as<float>(),
                                   d_lrmax_.as<float>(), d_lRmax_.as<float>(), (int)nlist, n, np,
                                   (int)k, pq_obits_, b, mi, s_pkeys_.as<uint32_t>(),
                                   s_precs_.as<kern::ProbeRec>(), &KT, s, qimg, qxn);
        }
        {
            ScopedKernelTimer tm(&ktimes, "ivfpq_rerank", 0.0, s);
            kern::PQArgs pa;
            pa.pq_cent = d_pq_.as<float>();
            pa.cent = d_cent_.as<float>();
            pa.ldcent = ld();
            pa.cdis = centroid_dis;
            pa.codes = d_codes_.as<uint8_t>();
            pa.cs = device_code_stride();
            pa.M = (int)pq.M;
            pa.table1 = use_precomputed_table == 1 ? 1 : 0;
            kern::ivfpq_rerank(s_pkeys_.as<uint32_t>(), s_precs_.as<kern::ProbeRec>(), x, ldx, d,
                               d_ids_.as<int64_t>(), pa, (int)pq.dsub, n, np, KT, pq_obits_,
                               (int)k, sel, distances, labels,
                               dbg ? s_pflags_.as<uint32_t>() : nullptr, s, qdone_,
                               pq_fold ? 1 : 0);
        }
        if (dbg) {
            uint32_t st[4];
            HIP_CHECK(hipMemcpyAsync(st, s_pflags_.ptr, sizeof(st), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            fprintf(stderr,
                    "[faiss_amd] ivfpq mfma scan: nq=%lld survivors/q=%.2f failing streams/q=%.4f "
                    "overflow queries=%u general-resolve queries=%u\n",
                    (long long)n, st[0] / (double)n, st[1] / (double)n, st[2], st[3]);
        }
        return;
    }
    exact_scan_device(n, x, ldx, k, np, assign, centroid_dis, distances, labels, s, lim, sel,
                      store_pairs);
}

void IndexIVFPQ::own_coarse_dis(idx_t n, const float* x, int ldx, int np,
                                const int32_t* assign, float* cdis, hipStream_t s) const {
    // table 0 (faiss/IndexIVFPQ.cpp:634-700) computes |r_m - c|^2 tables and
    // never reads coarse_dis; the list filter's key coarse_dis + term - 2 <x,
    // y_R> needs the true |x - y_C|^2
    if (!(by_residual && metric_type == METRIC_L2 && use_precomputed_table != 1)) return;
    kern::pair_l2(x, ldx, d_cent_.as<float>(), ld(), d, assign, n, np, cdis, s);
}

void IndexIVFPQ::exact_args(void* p) const {
    auto& a = *(kern::ExactScanArgs*)p;
    a.pq.M = (int)pq.M;
    a.pq.dsub = (int)pq.dsub;
    a.pq.by_residual = by_residual ? 1 : 0;
    a.pq.table1 = (metric_type == METRIC_L2 && by_residual && use_precomputed_table == 1) ? 1 : 0;
    a.pq.pq_cent = d_pq_.as<float>();
    a.pq.cent = d_cent_.as<float>();
    a.pq.ldcent = ld();
    a.pq.codes = d_codes_.as<uint8_t>();
    a.pq.cs = device_code_stride();
}

// ---------------------------------------------------------------- shards
void IndexShardsIVF::train(idx_t n, const float* x) {
    // faiss/IndexShardsIVF.cpp:44-86: train the common quantizer, copy to shards
    std::vector<float> cent((size_t)nlist * d);
    if (!(quantizer->is_trained && (size_t)quantizer->ntotal == nlist)) {
        kmeans_train(d, n, x, (int)nlist, 25, 1234, cent.data(), device, verbose);
        quantizer->reset();
        quantizer->add(nlist, cent.data());
        quantizer->is_trained = true;
    }
    for (auto* s : shards) {
        if (!s->is_trained) s->train(n, x);
    }
    is_trained = true;
}

void IndexShardsIVF::add(idx_t n, const float* x) { add_with_ids(n, x, nullptr); }

void IndexShardsIVF::add_with_ids(idx_t n, const float* x, const idx_t* xids) {
    // faiss/IndexShardsIVF.cpp:88-156: contiguous slices per shard
    FAISS_THROW_IF_NOT_MSG(!(successive_ids && xids),
                           "It makes no sense to pass in ids and request them to be shifted");
    if (successive_ids)
        FAISS_THROW_IF_NOT_MSG(ntotal == 0, "when adding to IndexShards with successive_ids, "
                                            "only add() in a single pass is supported");
    const idx_t ns = (idx_t)shards.size();
    FAISS_THROW_IF_NOT(ns > 0);
    std::vector<idx_t> aids;
    const idx_t* ids = xids;
    if (!ids && !successive_ids) {
        aids.resize(n);
        for (idx_t i = 0; i < n; i++) aids[i] = ntotal + i;
        ids = aids.data();
    }
    for (idx_t no = 0; no < ns; no++) {
        idx_t i0 = no * n / ns, i1 = (no + 1) * n / ns;
        shards[no]->add_with_ids(i1 - i0, x + (size_t)i0 * d, ids ? ids + i0 : nullptr);
    }
    ntotal += n;
}

void IndexShardsIVF::reset() {
    for (auto* s : shards) s->reset();
    ntotal = 0;
}

void IndexShardsIVF::search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                                   idx_t* labels, const SearchParameters* params_in,
                                   hipStream_t s) const {
    // faiss/IndexShardsIVF.cpp:158-245
    const SearchParametersIVF* params = dynamic_cast<const SearchParametersIVF*>(params_in);
    const size_t np = std::min(nlist, params && params->nprobe ? params->nprobe : nprobe);
    FAISS_THROW_IF_NOT(np > 0 && k > 0);
    const int ns = (int)shards.size();
    FAISS_THROW_IF_NOT(ns > 0);
    DevGuard dg(device);
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (multi_device()) {
        search_multi(n, x, ldx, k, distances, labels, params, np, s);
        return;
    }
    s_cd_.reserve(sizeof(float) * n * np);
    s_ci_.reserve(sizeof(int32_t) * n * np);
    s_all_d_.reserve(sizeof(float) * ns * n * k);
    s_all_i_.reserve(sizeof(idx_t) * ns * n * k);
    quantizer->assign_device(n, x, ldx, (int)np, s_cd_.as<float>(), s_ci_.as<int32_t>(),
                             params ? params->quantizer_params : nullptr, s);
    idx_t translation = 0;
    for (int no = 0; no < ns; no++) {
        FAISS_THROW_IF_NOT_MSG(shards[no]->nprobe == np || params, "inconsistent nprobe");
        idx_t* li = s_all_i_.as<idx_t>() + (size_t)no * n * k;
        // each shard applies max_codes to its own lists (IndexShardsIVF.cpp:204-213
        // passes the params to every shard's search_preassigned)
        const uint32_t* lim = nullptr;
        const int32_t* asg = shards[no]->apply_max_codes(
                n, (int)np, s_ci_.as<int32_t>(), params ? params->max_codes : shards[no]->max_codes,
                &lim, s);
        const uint8_t* selm = shards[no]->apply_selector(params, s);
        shards[no]->search_preassigned_device(n, x, ldx, k, (int)np, asg, s_cd_.as<float>(),
                                              s_all_d_.as<float>() + (size_t)no * n * k, li, s,
                                              lim, selm);
        if (successive_ids) kern::translate_labels(li, (int64_t)n * k, translation, s);
        translation += shards[no]->ntotal;
    }
    kern::merge_rows(s_all_d_.as<float>(), s_all_i_.as<idx_t>(), n, (ns << 16) | (int)k, (int)k,
                     metric_type == METRIC_L2, distances, labels, s);
    HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace faiss_amd

// ---------------------------------------------------------------- range search
namespace faiss_amd {

void IndexIVF::range_search(idx_t n, const float* x, float radius, RangeSearchResult* result,
                            const SearchParameters* params_in) const {
    // faiss/IndexIVF.cpp:1203-1241
    const SearchParametersIVF* params = nullptr;
    if (params_in) {
        params = dynamic_cast<const SearchParametersIVF*>(params_in);
        FAISS_THROW_IF_NOT_MSG(params, "IndexIVF params have incorrect type");
    }
    FAISS_THROW_IF_NOT(result && result->nq == (size_t)n);
    const size_t np = std::min(nlist, params && params->nprobe ? params->nprobe : nprobe);
    FAISS_THROW_IF_NOT(np > 0);
    check_parallel_mode(parallel_mode);
    result->lims.assign((size_t)n + 1, 0);
    result->labels.clear();
    result->distances.clear();
    if (n == 0) return;
    DevGuard dg(device);
    sync_device();
    hipStream_t s = stream();
    const int ldx = ld();
    DeviceBuffer bx, bcd, bci;
    bx.reserve(sizeof(float) * n * ldx);
    bcd.reserve(sizeof(float) * n * np);
    bci.reserve(sizeof(int32_t) * n * np);
    if (ldx != d) HIP_CHECK(hipMemsetAsync(bx.ptr, 0, sizeof(float) * n * ldx, s));
    HIP_CHECK(hipMemcpy2DAsync(bx.ptr, sizeof(float) * ldx, x, sizeof(float) * d,
                               sizeof(float) * d, n, hipMemcpyHostToDevice, s));
    const auto t0 = std::chrono::steady_clock::now();
    quantize_device(n, bx.as<float>(), ldx, (int)np, bcd.as<float>(), bci.as<int32_t>(),
                    params ? params->quantizer_params : nullptr, s);
    HIP_CHECK(hipStreamSynchronize(s));
    const auto t1 = std::chrono::steady_clock::now();
    indexIVF_stats.quantization_time +=
            std::chrono::duration<double, std::milli>(t1 - t0).count();
    quantizer->fold_device_stats();
    const uint8_t* selm = apply_selector(params, s);
    range_device(n, bx.as<float>(), ldx, (int)np, bci.as<int32_t>(), bcd.as<float>(), radius,
                 selm, result, &indexIVF_stats, s);
    indexIVF_stats.search_time += std::chrono::duration<double, std::milli>(
                                          std::chrono::steady_clock::now() - t1)
                                          .count();
}

void IndexIVF::range_search_preassigned(idx_t n, const float* x, float radius,
                                        const idx_t* assign, const float* centroid_dis,
                                        RangeSearchResult* result, bool store_pairs,
                                        const SearchParametersIVF* params,
                                        IndexIVFStats* stats) const {
    // faiss/IndexIVF.cpp:1243-1400 (parallel_mode 0)
    FAISS_THROW_IF_NOT(result && result->nq == (size_t)n);
    const size_t np = std::min(nlist, params && params->nprobe ? params->nprobe : nprobe);
    FAISS_THROW_IF_NOT(np > 0);
    check_parallel_mode(parallel_mode);
    result->lims.assign((size_t)n + 1, 0);
    result->labels.clear();
    result->distances.clear();
    if (n == 0) return;
    std::vector<int32_t> a32((size_t)n * np);
    for (size_t i = 0; i < a32.size(); i++) {
        const idx_t key = assign[i];
        FAISS_THROW_IF_NOT_FMT(key < (idx_t)nlist, "Invalid key=%" PRId64 " at ik=%zd nlist=%zd\n",
                               (int64_t)key, i % np, nlist);
        a32[i] = key < 0 ? -1 : (int32_t)key;
    }
    DevGuard dg(device);
    sync_device();
    hipStream_t s = stream();
    const int ldx = ld();
    DeviceBuffer bx, bci, bcd;
    bx.reserve(sizeof(float) * n * ldx);
    bci.reserve(sizeof(int32_t) * n * np);
    if (centroid_dis) {
        bcd.reserve(sizeof(float) * n * np);
        HIP_CHECK(hipMemcpyAsync(bcd.ptr, centroid_dis, sizeof(float) * n * np,
                                 hipMemcpyHostToDevice, s));
    }
    if (ldx != d) HIP_CHECK(hipMemsetAsync(bx.ptr, 0, sizeof(float) * n * ldx, s));
    HIP_CHECK(hipMemcpy2DAsync(bx.ptr, sizeof(float) * ldx, x, sizeof(float) * d,
                               sizeof(float) * d, n, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(bci.ptr, a32.data(), sizeof(int32_t) * a32.size(),
                             hipMemcpyHostToDevice, s));
    const uint8_t* selm = apply_selector(params, s);
    range_device(n, bx.as<float>(), ldx, (int)np, bci.as<int32_t>(),
                 centroid_dis ? bcd.as<float>() : nullptr, radius, selm, result,
                 stats ? stats : &indexIVF_stats, s, store_pairs);
}

void IndexIVF::range_launch(const float*, idx_t, int, const int32_t*, const float*, int, float,
                            const uint8_t*, uint32_t*, const uint64_t*, float*, idx_t*, bool,
                            hipStream_t) const {
    FAISS_THROW_MSG("range search not implemented for this type of index");
}

void IndexIVFFlat::range_launch(const float* x, idx_t n, int ldx, const int32_t* assign,
                                const float*, int np, float radius, const uint8_t* selm,
                                uint32_t* counts, const uint64_t* offs, float* D, idx_t* I,
                                bool store_pairs, hipStream_t s) const {
    kern::ivf_range_flat(x, n, ldx, assign, np, d_codes_.as<float>(), ld(),
                         store_pairs ? nullptr : d_ids_.as<int64_t>(), d_list_off_.as<uint32_t>(),
                         d_list_len_.as<uint32_t>(), (int)nlist, d, metric_type == METRIC_L2,
                         radius, selm, counts, offs, D, I, s);
}

void IndexIVFPQ::range_launch(const float* x, idx_t n, int ldx, const int32_t* assign,
                              const float* cdis, int np, float radius, const uint8_t* selm,
                              uint32_t* counts, const uint64_t* offs, float* D, idx_t* I,
                              bool store_pairs, hipStream_t s) const {
    FAISS_THROW_IF_NOT_MSG(cdis || !(metric_type == METRIC_L2 && by_residual &&
                                     use_precomputed_table == 1),
                           "IVF-PQ range search with precomputed tables needs centroid_dis");
    kern::ExactScanArgs a;
    exact_args(&a);
    a.x = x;
    a.ldx = ldx;
    a.d = d;
    a.n = n;
    a.np = np;
    a.l2 = metric_type == METRIC_L2;
    a.assign = assign;
    a.cdis = cdis;
    a.list_off = d_list_off_.as<uint32_t>();
    a.list_len = d_list_len_.as<uint32_t>();
    a.nlist = (int)nlist;
    a.sel = selm;
    a.ids = d_ids_.as<int64_t>();
    a.row_list = d_row_list_.as<uint32_t>();
    a.store_pairs = store_pairs ? 1 : 0;
    kern::ivfpq_range_exact(a, radius, counts, offs, D, I, s);
}

void IndexIVF::range_device(idx_t n, const float* x, int ldx, int np, const int32_t* assign,
                            const float* cdis, float radius, const uint8_t* selm,
                            RangeSearchResult* result, IndexIVFStats* stats, hipStream_t s,
                            bool store_pairs) const {
    // queries per pass: grid n*np < 2^31 and bounded count scratch
    const idx_t qc = std::max<idx_t>(1, std::min<idx_t>(n, ((idx_t)1 << 26) / np));
    std::vector<uint32_t> cnt;
    std::vector<int32_t> hassign;
    std::vector<uint64_t> offs;
    DeviceBuffer bc, bo, bd, bi;
    size_t nlistv = 0, ndis = 0;
    result->lims.assign((size_t)n + 1, 0);
    for (idx_t q0 = 0; q0 < n; q0 += qc) {
        const idx_t nc = std::min(qc, n - q0);
        const size_t m = (size_t)nc * np;
        const int32_t* a = assign + (size_t)q0 * np;
        bc.reserve(sizeof(uint32_t) * m);
        const float* cd = cdis ? cdis + (size_t)q0 * np : nullptr;
        range_launch(x + (size_t)q0 * ldx, nc, ldx, a, cd, np, radius, selm, bc.as<uint32_t>(),
                     nullptr, nullptr, nullptr, store_pairs, s);
        cnt.resize(m);
        hassign.resize(m);
        HIP_CHECK(hipMemcpyAsync(cnt.data(), bc.ptr, sizeof(uint32_t) * m, hipMemcpyDeviceToHost,
                                 s));
        HIP_CHECK(hipMemcpyAsync(hassign.data(), a, sizeof(int32_t) * m, hipMemcpyDeviceToHost,
                                 s));
        HIP_CHECK(hipStreamSynchronize(s));
        // (query, probe) offsets in the reference's order: query-major, probe
        // order within a query (RangeQueryResult per query, :1334-1345)
        offs.resize(m);
        const size_t base = result->labels.size();
        uint64_t tot = 0;
        for (idx_t i = 0; i < nc; i++) {
            result->lims[(size_t)(q0 + i)] = base + tot;
            for (int p = 0; p < np; p++) {
                const size_t j = (size_t)i * np + p;
                offs[j] = tot;
                tot += cnt[j];
                const int32_t key = hassign[j];
                if (key >= 0 && invlists->list_size((size_t)key) > 0) {
                    nlistv++;
                    ndis += invlists->list_size((size_t)key);
                }
            }
        }
        if (tot) {
            bo.reserve(sizeof(uint64_t) * m);
            bd.reserve(sizeof(float) * tot);
            bi.reserve(sizeof(idx_t) * tot);
            HIP_CHECK(hipMemcpyAsync(bo.ptr, offs.data(), sizeof(uint64_t) * m,
                                     hipMemcpyHostToDevice, s));
            range_launch(x + (size_t)q0 * ldx, nc, ldx, a, cd, np, radius, selm, nullptr,
                         bo.as<uint64_t>(), bd.as<float>(), bi.as<int64_t>(), store_pairs, s);
            result->labels.resize(base + tot);
            result->distances.resize(base + tot);
            HIP_CHECK(hipMemcpyAsync(result->distances.data() + base, bd.ptr, sizeof(float) * tot,
                                     hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipMemcpyAsync(result->labels.data() + base, bi.ptr, sizeof(idx_t) * tot,
                                     hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
        }
    }
    result->lims[(size_t)n] = result->labels.size();
    stats->nq += (size_t)n;
    stats->nlist += nlistv;
    stats->ndis += ndis;
}

}  // namespace faiss_amd
