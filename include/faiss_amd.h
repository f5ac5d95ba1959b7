// faiss_amd.h — C++ host API of the MI355X-native IVF search path.
//
// Mirrors the reference faiss::Index hierarchy for the hot path
// (faiss/Index.h:108-181, faiss/IndexFlat.h, faiss/IndexIVF.h:39-587,
// faiss/IndexIVFFlat.h, faiss/IndexIVFPQ.h, faiss/IndexHNSW.h,
// faiss/IndexShardsIVF.h): same class names, method signatures, argument
// meaning and exceptions, in namespace faiss_amd.  Indexes are GPU-resident:
// host mirrors keep the faiss data structures (for I/O and reconstruction),
// HBM holds the search layout.  `search()` takes host pointers and is
// synchronous; `search_device()` takes device pointers and a hipStream_t.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <chrono>
#include <cstdint>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../hnsw-ivf_amd/csrc/common.h"

namespace faiss_amd {

// ---------------------------------------------------------------- selectors
// faiss/impl/IDSelector.h:20-180.  is_member() is the reference predicate;
// mark_device() evaluates it for every arena row on the GPU (mask[r] = 1 when
// ids[r] is a member; ids < 0 are padding rows and never members).
struct IDSelector {
    virtual ~IDSelector() = default;
    virtual bool is_member(idx_t id) const = 0;
    virtual void mark_device(const idx_t* ids, int64_t n, uint8_t* mask,
                             hipStream_t stream) const = 0;
};
struct IDSelectorRange : IDSelector {  // [imin, imax)
    idx_t imin, imax;
    bool assume_sorted;  // reference fast path; same members here
    IDSelectorRange(idx_t imin, idx_t imax, bool assume_sorted = false)
            : imin(imin), imax(imax), assume_sorted(assume_sorted) {}
    bool is_member(idx_t id) const override { return id >= imin && id < imax; }
    void mark_device(const idx_t* ids, int64_t n, uint8_t* mask, hipStream_t s) const override;
};
struct IDSelectorArray : IDSelector {  // the n ids (not owned)
    size_t n;
    const idx_t* ids;
    IDSelectorArray(size_t n, const idx_t* ids) : n(n), ids(ids) {}
    bool is_member(idx_t id) const override;
    void mark_device(const idx_t* ids, int64_t n, uint8_t* mask, hipStream_t s) const override;
};
struct IDSelectorBatch : IDSelector {  // a set of ids (copied)
    std::vector<idx_t> sorted;
    IDSelectorBatch(size_t n, const idx_t* indices);
    bool is_member(idx_t id) const override;
    void mark_device(const idx_t* ids, int64_t n, uint8_t* mask, hipStream_t s) const override;
};
struct IDSelectorBitmap : IDSelector {  // n bytes, bit i of the map (not owned)
    size_t n;
    const uint8_t* bitmap;
    IDSelectorBitmap(size_t n, const uint8_t* bitmap) : n(n), bitmap(bitmap) {}
    bool is_member(idx_t id) const override {
        const uint64_t i = (uint64_t)id;
        return (i >> 3) < n && ((bitmap[i >> 3] >> (i & 7)) & 1);
    }
    void mark_device(const idx_t* ids, int64_t n, uint8_t* mask, hipStream_t s) const override;
};
struct IDSelectorNot : IDSelector {
    const IDSelector* sel;
    explicit IDSelectorNot(const IDSelector* sel) : sel(sel) {}
    bool is_member(idx_t id) const override { return !sel->is_member(id); }
    void mark_device(const idx_t* ids, int64_t n, uint8_t* mask, hipStream_t s) const override;
};
struct IDSelectorBinary : IDSelector {  // And / Or / XOr
    const IDSelector *lhs, *rhs;
    int op;  // 0 and, 1 or, 2 xor
    IDSelectorBinary(const IDSelector* l, const IDSelector* r, int op) : lhs(l), rhs(r), op(op) {}
    bool is_member(idx_t id) const override {
        const bool a = lhs->is_member(id), b = rhs->is_member(id);
        return op == 0 ? (a && b) : op == 1 ? (a || b) : (a != b);
    }
    void mark_device(const idx_t* ids, int64_t n, uint8_t* mask, hipStream_t s) const override;
};

// ---------------------------------------------------------------- params
struct SearchParameters {  // faiss/Index.h:63-70
    IDSelector* sel = nullptr;  // only the vectors whose id is a member
    virtual ~SearchParameters() = default;
};
struct SearchParametersHNSW : SearchParameters {  // faiss/impl/HNSW.h:46-52
    int efSearch = 16;
};
struct SearchParametersIVF : SearchParameters {  // faiss/IndexIVF.h:77-85
    size_t nprobe = 1;
    size_t max_codes = 0;
    SearchParameters* quantizer_params = nullptr;
};

// faiss/IndexIVF.h:567-583.  On the GPU path nheap_updates stays 0 (there is
// no sequential heap); nq / nlist / ndis count exactly what the reference
// counts (non-empty lists visited, codes scanned).
struct IndexIVFStats {
    size_t nq = 0, nlist = 0, ndis = 0, nheap_updates = 0;
    double quantization_time = 0, search_time = 0;
    void reset() { *this = IndexIVFStats(); }
    void add(const IndexIVFStats& o) {
        nq += o.nq;
        nlist += o.nlist;
        ndis += o.ndis;
        nheap_updates += o.nheap_updates;
        quantization_time += o.quantization_time;
        search_time += o.search_time;
    }
};
extern IndexIVFStats indexIVF_stats;

// faiss/IndexIVF.h:28-32 — this fork's per-query latency record filled by
// IndexIVF::search_stats / IndexHNSW::search_stats (microseconds).
// GPU semantics: a batch is one slice, so quantization_us is
// the coarse stage's wall time / n (the reference's amortisation) and
// list_scan_us the wall time of the batched scan stage that produced the
// query's result; total_us = quantization_us + list_scan_us.
struct QueryLatencyStats {
    double total_us = 0.0;
    double quantization_us = 0.0;
    double list_scan_us = 0.0;
};

// faiss/impl/HNSW.h:234-253 (global faiss::hnsw_stats).  Counted on the
// device by the search kernel; folded into the host struct at the end of
// every synchronous host call (device-API searches fold at the next one, or
// at fold_device_stats()).
struct HNSWStats {
    size_t n1 = 0, n2 = 0, ndis = 0, nhops = 0;
    void reset() { n1 = n2 = ndis = nhops = 0; }
    void combine(const HNSWStats& o) {
        n1 += o.n1;
        n2 += o.n2;
        ndis += o.ndis;
        nhops += o.nhops;
    }
};
extern HNSWStats hnsw_stats;
// Not in the reference: rows the GPU HNSW kernels read per distance, for the
// bench's byte count — fp32 rows (every distance computed exactly) and rows
// whose int8 image the register kernel's prefilter read (hnsw_stats.ndis
// counts the distances as the reference does).  Reset with hnsw_stats.
struct HNSWRowStats {
    uint64_t fp32_rows = 0, q8_rows = 0;
    // the register kernel's queries that met a layout-dependent decision:
    // continued from the replayed log / searched level 0 again (log
    // overflowed) / log found corrupt and searched again (0 unless a bug)
    uint64_t replayed = 0, searched_again = 0, replay_bad = 0;
};
extern HNSWRowStats hnsw_row_stats;

// faiss/impl/AuxIndexStructures.h:30-60: results of query i are
// labels/distances[lims[i], lims[i+1]), in the order the scan found them.
struct RangeSearchResult {
    size_t nq = 0;
    std::vector<size_t> lims;
    std::vector<idx_t> labels;
    std::vector<float> distances;
    explicit RangeSearchResult(size_t nq = 0) : nq(nq), lims(nq + 1, 0) {}
    size_t buffer_size() const { return labels.size(); }
};

// faiss/impl/AuxIndexStructures.h:135-170: a callback that long computations
// poll; the one installed in `instance` (if any) is asked want_interrupt().
// Here a host search polls it between its query chunks and once the batch is
// done (a GPU batch is not cut short inside its kernels), and k-means once
// per iteration; a search that sees it fire throws "computation interrupted",
// as IndexIVF::search_preassigned does after its loop (IndexIVF.cpp:627,
// 707-713), and IndexHNSW::search per chunk (IndexHNSW.cpp:315).
struct InterruptCallback {
    virtual bool want_interrupt() = 0;
    virtual ~InterruptCallback() {}
    static std::mutex lock;  // serialises is_interrupted()
    static std::unique_ptr<InterruptCallback> instance;
    static void clear_instance();
    static void check();          // throws "computation interrupted" when it fires
    static bool is_interrupted();  // the same, as a flag
    // iterations between polls for a loop of `flops` per iteration
    static size_t get_period_hint(size_t flops);
};

// fires once, the first poll after `timeout` seconds from set_timeout()
struct TimeoutCallback : InterruptCallback {
    std::chrono::time_point<std::chrono::steady_clock> start;
    double timeout = 0;
    bool want_interrupt() override;
    void set_timeout(double timeout_in_seconds);
    static void reset(double timeout_in_seconds);  // installs a new one as `instance`
};

// ---------------------------------------------------------------- Index
struct Index {
    int d = 0;
    idx_t ntotal = 0;
    bool verbose = false;
    bool is_trained = true;
    MetricType metric_type = METRIC_L2;
    float metric_arg = 0;
    int device = 0;  // HIP device holding the HBM copy

    mutable KernelTimes ktimes;  // dominant-kernel timings of the last search

    explicit Index(idx_t d = 0, MetricType metric = METRIC_L2);
    virtual ~Index();

    virtual void train(idx_t n, const float* x);
    virtual void add(idx_t n, const float* x) = 0;
    virtual void add_with_ids(idx_t n, const float* x, const idx_t* xids);
    // faiss/Index.h:165-171: host pointers, synchronous
    virtual void search(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                        const SearchParameters* params = nullptr) const;
    // device pointers; x rows have leading dimension ldx (multiple of 4)
    virtual void search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                               idx_t* labels, const SearchParameters* params,
                               hipStream_t stream) const = 0;
    // coarse-quantizer entry: top-k as int32 labels (device)
    virtual void assign_device(idx_t n, const float* x, int ldx, int k, float* distances,
                               int32_t* labels, const SearchParameters* params,
                               hipStream_t stream) const;
    // assign_device of n queries that are a slice of a batch of batch_n: the
    // computation form the reference picks by batch size (a flat quantizer's
    // direct form below 20 queries, faiss/utils/distances.cpp:807-823) follows
    // batch_n, so a query split over devices gives the whole batch's result
    virtual void assign_device_slice(idx_t n, const float* x, int ldx, int k, float* distances,
                                     int32_t* labels, const SearchParameters* params,
                                     hipStream_t stream, idx_t batch_n) const {
        assign_device(n, x, ldx, k, distances, labels, params, stream);
    }
    virtual void reset() = 0;
    virtual void reconstruct(idx_t key, float* recons) const;
    // faiss/Index.h:183-196: all vectors with distance < radius (L2) or
    // > radius (IP); only IndexIVFFlat implements it on this path
    virtual void range_search(idx_t n, const float* x, float radius, RangeSearchResult* result,
                              const SearchParameters* params = nullptr) const;
    virtual void sync_device() const {}
    // fold device-side search counters (HNSWStats) into the host globals
    virtual void fold_device_stats() const {}
    // bumped by every add / reset of the index's content and by every upload
    // of changed content to HBM (copies made of it, e.g. IndexShardsIVF's
    // per-rank quantizers, and captured search graphs are rebuilt when it
    // moves); atomic: searches on other threads read it without the lock
    virtual uint64_t content_version() const { return version_.load(); }

    hipStream_t stream() const;
    int ld() const { return (int)roundup((size_t)d, 4); }

   protected:
    // host-pointer entry points: queries and results in HBM, kept between
    // calls (one host call at a time per index)
    mutable std::mutex host_mu_;
    mutable DeviceBuffer h_x_, h_d_, h_i_;
    mutable std::atomic<uint64_t> version_{0};
};

// ---------------------------------------------------------------- flat
// faiss/IndexFlat.h: exhaustive search.  Coarse quantizer of the IVF path.
struct IndexFlat : Index {
    std::vector<float> xb;  // host mirror [ntotal][d] (faiss IndexFlatCodes::codes)

    explicit IndexFlat(idx_t d = 0, MetricType metric = METRIC_L2);
    void add(idx_t n, const float* x) override;
    void search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                       idx_t* labels, const SearchParameters* params,
                       hipStream_t stream) const override;
    void assign_device(idx_t n, const float* x, int ldx, int k, float* distances,
                       int32_t* labels, const SearchParameters* params,
                       hipStream_t stream) const override;
    void reset() override;
    void reconstruct(idx_t key, float* recons) const override;
    void sync_device() const override;

    const float* device_vectors() const;  // [ntotal][ld]
    const float* device_norms() const;
    // assign_device that also leaves the batch's query image (kernels.h
    // query_prep: bf16 fragments, then |x|^2 at byte query_image_bytes(n, d))
    // in the caller's buffer `qimg` (query_image_bytes(n, d) + 4 n bytes), on
    // the caller's stream, so IndexIVF::search hands it to its list filter
    // and a batch is prepared once.  Returns false when the coarse plan does
    // not prepare an image (the buffer is then untouched).
    bool assign_device_qimg(idx_t n, const float* x, int ldx, int k, float* distances,
                            int32_t* labels, void* qimg, hipStream_t stream) const;
    void assign_device_slice(idx_t n, const float* x, int ldx, int k, float* distances,
                             int32_t* labels, const SearchParameters* params, hipStream_t stream,
                             idx_t batch_n) const override;
    // bytes of the query image assign_device_qimg writes for n queries
    size_t query_image_size(idx_t n) const;
    // device order of this quantizer's scratch for work queued on `stream`
    // outside its own entry points (a replayed IVF search graph that writes
    // the quantizer's scratch): enter before queuing, leave after
    void stream_enter(hipStream_t stream) const;
    void stream_leave(hipStream_t stream) const;

   private:
    template <class OutIdx>
    bool knn_device(idx_t n, const float* x, int ldx, int k, float* distances, OutIdx* labels,
                    hipStream_t stream, void* qimg_out = nullptr, idx_t batch_n = -1) const;
    template <class OutIdx>
    bool knn_impl(idx_t n, const float* x, int ldx, int k, float* distances, OutIdx* labels,
                  hipStream_t stream, void* qimg_out, bool direct) const;
    mutable StreamOrder order_;
    mutable DeviceBuffer d_xb_, d_norms_, d_cbf_, d_cnmax_, d_cst_;
    mutable int cfold_ = 0;  // d_cst_ carries folded norm fragments (L2)
    mutable bool dirty_ = true;
    mutable std::recursive_mutex mu_;
    mutable DeviceBuffer s_xn_, s_tile_, s_cand_d_, s_cand_i_, s_qimg_, s_sel_;
    // search with an IDSelector (faiss/IndexFlat.cpp:38-57 ->
    // faiss/utils/distances.cpp:840-935): IDSelectorRange narrows the rows
    // and keeps the batch-size form choice; any other selector takes the
    // direct per-row form over its members (exhaustive_*_seq)
    void search_selected(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                         idx_t* labels, const IDSelector* sel, hipStream_t stream) const;
    mutable DeviceBuffer s_selids_, s_selmask_;  // 0 .. ntotal - 1 (int64) and membership
    mutable idx_t selids_n_ = 0;
};
struct IndexFlatL2 : IndexFlat {
    explicit IndexFlatL2(idx_t d = 0) : IndexFlat(d, METRIC_L2) {}
};
struct IndexFlatIP : IndexFlat {
    explicit IndexFlatIP(idx_t d = 0) : IndexFlat(d, METRIC_INNER_PRODUCT) {}
};

// ---------------------------------------------------------------- HNSW
// faiss/impl/HNSW.h:54-232 graph, faiss/IndexHNSW.h IndexHNSWFlat.
struct HNSW {
    std::vector<double> assign_probas;
    std::vector<int> cum_nneighbor_per_level;
    std::vector<int> levels;
    std::vector<size_t> offsets;
    std::vector<int32_t> neighbors;
    int32_t entry_point = -1;
    int max_level = -1;
    int efConstruction = 40;
    int efSearch = 16;
    bool check_relative_distance = true;
    bool search_bounded_queue = true;

    explicit HNSW(int M = 32);
    void set_default_probas(int M, float levelMult);
    int nb_neighbors(int layer_no) const;
    int cum_nb_neighbors(int layer_no) const;
    void neighbor_range(idx_t no, int layer_no, size_t* begin, size_t* end) const;
    int random_level(std::mt19937& rng) const;
};

struct IndexHNSW : Index {
    HNSW hnsw;
    IndexFlat* storage = nullptr;
    bool own_fields = false;
    IndexHNSW(IndexFlat* storage, int M);
    ~IndexHNSW() override;
    void add(idx_t n, const float* x) override;
    void search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                       idx_t* labels, const SearchParameters* params,
                       hipStream_t stream) const override;
    void assign_device(idx_t n, const float* x, int ldx, int k, float* distances,
                       int32_t* labels, const SearchParameters* params,
                       hipStream_t stream) const override;
    void reset() override;
    void reconstruct(idx_t key, float* recons) const override;
    void sync_device() const override;
    void fold_device_stats() const override;
    uint64_t content_version() const override {
        return version_.load() + (storage ? storage->content_version() : 0);
    }
    // faiss/IndexHNSW.cpp:345-366: search with per-query latency statistics
    // (quantization_us = 0, list_scan_us = total_us, like the reference)
    void search_stats(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                      const SearchParameters* params = nullptr,
                      QueryLatencyStats* per_query_stats = nullptr) const;

    // Coarse assignment with the tie re-runs left to the caller, so it can
    // overlap them with its own work (IndexIVF::search_device): split_begin
    // queues the batched search of n queries (the flagged ones keep the
    // batched result) and a read-back of the flagged count, and returns false
    // when this form is not offered (visited bitmaps beyond LDS, ef > 128 or
    // k > 64: the caller then uses assign_device).  split_finish waits for the
    // count, queues the reference-exact sequential search of the flagged
    // queries on a side stream into compact rows, and returns them; `done` is
    // recorded after it (the caller waits on it before reading D / I).
    struct Split {
        idx_t nf = 0;                  // flagged queries
        const uint32_t* idx = nullptr;  // their query numbers [nf]
        const float* D = nullptr;       // [nf][k] exact coarse distances
        const int32_t* I = nullptr;     // [nf][k] exact assignments
        hipEvent_t done = nullptr;
    };
    // A split in progress holds this quantizer's lock from split_begin (when
    // it returns true) until split_release, so searches of other callers
    // sharing the quantizer wait instead of overwriting its split state;
    // SplitHold releases it on scope exit.
    bool split_begin(idx_t n, const float* x, int ldx, int k, float* distances, int32_t* labels,
                     const SearchParameters* params, hipStream_t stream) const;
    Split split_finish() const;
    void split_release() const;
    struct SplitHold {
        const IndexHNSW* q = nullptr;
        ~SplitHold() {
            if (q) q->split_release();
        }
    };

   private:
    template <class OutIdx>
    void hnsw_device(idx_t n, const float* x, int ldx, int k, float* distances, OutIdx* labels,
                     const SearchParameters* params, hipStream_t stream,
                     bool defer = false) const;
    mutable DeviceBuffer d_levels_, d_offsets_, d_neighbors_, d_cum_, d_nb0_, s_visited_, d_stats_,
            s_flags_, s_fidx_, s_fcnt_, s_fD_, s_fI_, s_heaps_, s_rlog_, d_q8_, d_q8p_, d_q8q1_,
            s_alog_;  // the sequential kernel's arrival-log pool
    mutable bool q8_ = false;  // the int8 level-0 row image is built
    mutable uint32_t* h_fcnt_ = nullptr;  // pinned read-back of the flagged count
    mutable hipEvent_t ev_split_ = nullptr, ev_exact_ = nullptr;
    mutable hipStream_t side_ = nullptr;
    struct SplitState {
        bool active = false;
        idx_t n = 0;
        const float* x = nullptr;
        int ldx = 0, k = 0, efSearch = 0;
        hipStream_t s = nullptr;
    };
    mutable SplitState split_;
    // device order of searches on different streams sharing this index's
    // scratch (a split leaves it at split_release)
    mutable StreamOrder order_;
    mutable int nb0_stride_ = 0;  // level-0 table width (0: not built)
    mutable bool dirty_ = true;
    mutable std::recursive_mutex mu_;
};
struct IndexHNSWFlat : IndexHNSW {
    IndexHNSWFlat(int d = 0, int M = 32, MetricType metric = METRIC_L2);
};

// ---------------------------------------------------------------- IVF
// faiss/invlists/InvertedLists.h:243-275 (ArrayInvertedLists) on the host,
// one contiguous arena in HBM.
// A read-only file mapping (mmap, PROT_READ, MAP_SHARED) that inverted lists
// can point into: `read_index(..., IO_FLAG_MMAP)` on an `ilar` file
// (faiss/invlists/OnDiskInvertedLists.cpp:759-800) and the `ilod` on-disk
// list file (:706-757).  Unmapped when the last list set using it goes.
struct MappedFile {
    const uint8_t* ptr = nullptr;
    size_t size = 0;
    std::string name;
    explicit MappedFile(int fd, const std::string& name);
    ~MappedFile();
};

// faiss/invlists/InvertedLists.h:37-275 (ArrayInvertedLists) with the
// OnDiskInvertedLists read-only case folded in: a list lives either in host
// vectors (codes[l], ids[l]) or, when `map` is set, in the mapped file
// (map_codes[l], map_ids[l], map_sizes[l]).  Mapped lists are streamed
// straight from the mapping through pinned staging buffers into HBM
// (IndexIVF::sync_device); an add on a mapped set first copies it into host
// memory (the reference's mmapped lists are read-only and throw instead).
struct ArrayInvertedLists {
    size_t nlist = 0, code_size = 0;
    std::vector<std::vector<uint8_t>> codes;
    std::vector<std::vector<idx_t>> ids;
    std::shared_ptr<MappedFile> map;
    std::vector<const uint8_t*> map_codes;
    std::vector<const idx_t*> map_ids;
    std::vector<size_t> map_sizes;
    bool map_ondisk = false;  // mapping is an `ilod` data file (written back as `ilod`)
    // `ilod` metadata as read: (size, capacity, offset) per list and the
    // free-slot table (offset, capacity), written back verbatim
    std::vector<size_t> ondisk_lists, ondisk_slots;
    size_t ondisk_totsize = 0;
    ArrayInvertedLists(size_t nlist, size_t code_size);
    bool is_mapped() const { return (bool)map; }
    size_t list_size(size_t l) const { return map ? map_sizes[l] : ids[l].size(); }
    const uint8_t* get_codes(size_t l) const { return map ? map_codes[l] : codes[l].data(); }
    const idx_t* get_ids(size_t l) const { return map ? map_ids[l] : ids[l].data(); }
    void materialize();  // copy mapped lists into host vectors and drop the mapping
    void add_entries(size_t l, size_t n, const idx_t* ids, const uint8_t* codes);
    void reset();
};

struct IndexIVF;
size_t ivf_copy_subset_to(const IndexIVF* src, IndexIVF* dst, int subset_type, idx_t a1,
                          idx_t a2);

struct IndexIVF : Index {
    Index* quantizer = nullptr;
    bool own_fields = false;
    size_t nlist = 0;
    size_t nprobe = 1;
    size_t max_codes = 0;
    size_t code_size = 0;
    bool by_residual = true;
    int niter = 25;  // k-means iterations (faiss ClusteringParameters::niter)
    int parallel_mode = 0;  // faiss/IndexIVF.h:58-62; the GPU path runs mode 0 only
    std::unique_ptr<ArrayInvertedLists> invlists;

    IndexIVF(Index* quantizer, size_t d, size_t nlist, size_t code_size, MetricType metric);
    ~IndexIVF() override;

    void train(idx_t n, const float* x) override;
    void add(idx_t n, const float* x) override;
    void add_with_ids(idx_t n, const float* x, const idx_t* xids) override;
    void search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                       idx_t* labels, const SearchParameters* params,
                       hipStream_t stream) const override;
    // faiss/IndexIVF.cpp:303-397 (host pointers, synchronous): also updates
    // indexIVF_stats (nq, nlist, ndis, quantization_time, search_time)
    void search(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                const SearchParameters* params = nullptr) const override;
    // faiss/IndexIVF.cpp:725-867: search with per-query latency statistics
    void search_stats(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                      const SearchParameters* params = nullptr,
                      QueryLatencyStats* per_query_stats = nullptr) const;
    // faiss/IndexIVF.h:120-130; assign = [n][nprobe] host list numbers
    void search_preassigned(idx_t n, const float* x, idx_t k, const idx_t* assign,
                            const float* centroid_dis, float* distances, idx_t* labels,
                            bool store_pairs, const SearchParametersIVF* params = nullptr,
                            IndexIVFStats* stats = nullptr) const;
    // faiss/IndexIVF.cpp:1203-1241 (coarse nprobe, then the preassigned scan)
    void range_search(idx_t n, const float* x, float radius, RangeSearchResult* result,
                      const SearchParameters* params = nullptr) const override;
    // faiss/IndexIVF.cpp:1243-1400; assign = [n][nprobe] host list numbers
    // (centroid_dis unused by the Flat scanner); parallel_mode 0 order
    void range_search_preassigned(idx_t n, const float* x, float radius, const idx_t* assign,
                                  const float* centroid_dis, RangeSearchResult* result,
                                  bool store_pairs = false,
                                  const SearchParametersIVF* params = nullptr,
                                  IndexIVFStats* stats = nullptr) const;
    // faiss/IndexIVF.cpp:870-1200 (per-query list_scan_us)
    void search_preassigned_stats(idx_t n, const float* x, idx_t k, const idx_t* assign,
                                  const float* centroid_dis, float* distances, idx_t* labels,
                                  bool store_pairs, const SearchParametersIVF* params,
                                  IndexIVFStats* ivf_stats,
                                  QueryLatencyStats* per_query_stats) const;
    // device form (int32 assignments).  lim (optional, max_codes): rows of
    // each (query, probe) list scanned, from apply_max_codes
    // store_pairs: labels are lo_build(list, offset) (faiss/IndexIVF.h:108-118)
    virtual void search_preassigned_device(idx_t n, const float* x, int ldx, idx_t k,
                                           int nprobe, const int32_t* assign,
                                           const float* centroid_dis, float* distances,
                                           idx_t* labels, hipStream_t stream,
                                           const uint32_t* lim = nullptr,
                                           const uint8_t* sel = nullptr,
                                           bool store_pairs = false) const = 0;
    // search_preassigned_device as a public device entry point: calls on
    // different streams are put in device order (they share this index's
    // scratch buffers)
    void search_preassigned_device_ordered(idx_t n, const float* x, int ldx, idx_t k, int nprobe,
                                           const int32_t* assign, const float* centroid_dis,
                                           float* distances, idx_t* labels,
                                           hipStream_t stream) const;
    // range scan of device-resident queries / assignments into host results
    void range_device(idx_t n, const float* x, int ldx, int np, const int32_t* assign,
                      const float* cdis, float radius, const uint8_t* sel,
                      RangeSearchResult* result, IndexIVFStats* stats, hipStream_t s,
                      bool store_pairs = false) const;
    // IDSelector of the call -> arena-row membership mask (index scratch),
    // nullptr when there is none (faiss/IndexIVF.cpp:418-430)
    const uint8_t* apply_selector(const SearchParameters* params, hipStream_t stream) const;
    // max_codes (faiss/IndexIVF.cpp:595-631): per query, the probe prefix
    // scanned before nscan reaches max_codes; returns the assignment with the
    // dropped probes set to -1 and sets *lim (both in index scratch)
    const int32_t* apply_max_codes(idx_t n, int nprobe, const int32_t* assign,
                                   size_t max_codes, const uint32_t** lim,
                                   hipStream_t stream) const;
    void quantize_device(idx_t n, const float* x, int ldx, int nprobe, float* coarse_dis,
                         int32_t* assign, const SearchParameters* qparams,
                         hipStream_t stream) const;
    void reset() override;
    void sync_device() const override;

    virtual void train_encoder(idx_t n, const float* x, const idx_t* assign) {}
    // encode n vectors assigned to lists (host in/out); codes [n][code_size]
    virtual void encode_vectors(idx_t n, const float* x, const idx_t* list_nos,
                                uint8_t* codes) const = 0;
    size_t get_list_size(size_t l) const { return invlists->list_size(l); }
    int device_code_stride() const;  // bytes per arena row
    // diagnostic read-back of HBM arena rows [row0, row0 + n) into host
    // `out` (tests): what = 0 the code rows (device_code_stride() bytes), 1
    // the row -> list table (uint32, ~0 for padding rows), 2 the filter's
    // stream image (IVF-Flat: always; IVF-PQ: when FAISS_AMD_PQ_FILTER=image
    // built it).  *row_bytes = bytes per row, *rows = the arena's rows; out
    // may be null to query them.  Throws when the buffer does not exist.
    void debug_rows(int what, idx_t row0, idx_t n, void* out, size_t* row_bytes,
                    idx_t* rows) const;

   protected:
    virtual void upload_extra() const {}
    // the filter's stream image (debug_rows what = 2): pointer and row bytes,
    // nullptr when this index has none
    virtual const void* stream_image(size_t* row_bytes) const { return nullptr; }
    // search_preassigned with caller coarse distances (device copy cdis,
    // [n][np]): an index whose scan must not trust them rewrites them (IVF-PQ
    // table 0: the reference ignores them, its filter keys on them)
    virtual void own_coarse_dis(idx_t n, const float* x, int ldx, int np, const int32_t* assign,
                                float* cdis, hipStream_t s) const {}
    // general exact scan (kernels_exact.hip): any k <= 2048, any nprobe,
    // store_pairs; the reference's results bit for bit
    void exact_scan_device(idx_t n, const float* x, int ldx, idx_t k, int nprobe,
                           const int32_t* assign, const float* centroid_dis, float* distances,
                           idx_t* labels, hipStream_t stream, const uint32_t* lim,
                           const uint8_t* sel, bool store_pairs) const;
    // the index-type part of the exact scan's arguments (codes / PQ tables)
    virtual void exact_args(void* args) const = 0;
    friend size_t ivf_copy_subset_to(const IndexIVF*, IndexIVF*, int, idx_t, idx_t);
    mutable uint32_t max_list_len_ = 0;
    mutable DeviceBuffer s_ex_eoff_, s_ex_tot_, s_ex_keys_, s_ex_rows_;
    mutable bool dirty_ = true;
    mutable std::recursive_mutex mu_;
    // arena
    mutable DeviceBuffer d_codes_, d_ids_, d_list_off_, d_list_len_, d_row_list_;
    mutable DeviceBuffer d_list_perm_;  // lists by decreasing length (work-item order)
    mutable size_t arena_rows_ = 0;
    // scratch
    mutable DeviceBuffer s_ictr_;
    mutable DeviceBuffer s_x_, s_cd_, s_ci_, s_counts_, s_boff_, s_ioff_, s_cur_, s_ent_,
            s_pk1_, s_pk2_, s_q_;
    // HNSW quantizer: quantize + scan with the tie re-runs overlapped
    // (IndexHNSW::split_begin / split_finish); false = not applicable
    bool scan_hnsw_split(idx_t nq, const float* x, int ldx, idx_t k, int np, float* distances,
                         idx_t* labels, const SearchParameters* qparams, hipStream_t s) const;
    mutable DeviceBuffer s_fx_, s_fDo_, s_fIo_;  // the re-run queries' rows and results
    // HNSW quantizer (register kernel): the batch in chunks, each chunk's
    // quantizer search on pipe_s_ overlapping the previous chunk's scan on the
    // caller's stream; false = not applicable
    bool scan_hnsw_pipelined(idx_t nq, const float* x, int ldx, idx_t k, int np,
                             float* distances, idx_t* labels, const SearchParameters* qparams,
                             hipStream_t s) const;
    // flat quantizer (FAISS_AMD_PIPE=<chunks>): the same overlap, each
    // chunk's query image in its own slice of s_q_
    bool scan_flat_pipelined(idx_t nq, const float* x, int ldx, idx_t k, int np,
                             float* distances, idx_t* labels, hipStream_t s) const;
    mutable hipStream_t pipe_s_ = nullptr;
    mutable std::vector<hipEvent_t> pipe_ev_;
    // search() on host buffers in query pages (faiss/gpu/GpuIndex.cu:307-333):
    // page i + 1's upload on host_cs_ while page i searches on the index
    // stream, page i - 1's results downloaded behind it; false = not applicable
    bool search_host_paged(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                           const SearchParameters* params, bool update_times) const;
    mutable hipStream_t host_cs_ = nullptr;
    mutable std::vector<hipEvent_t> host_ev_;
    // set inside search_host_paged: an eager (not captured) scan marks the
    // end of each chunk's coarse stage there; replays take the coarse share
    // of the page time from the last marked page
    mutable std::vector<hipEvent_t>* paged_marks_ = nullptr;
    mutable double paged_qshare_ = 0.1;
    // search_device replayed from a hipGraph captured on the second identical
    // call (flat quantizer, no parameters); FAISS_AMD_GRAPH=0: off
    void search_device_eager(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                             idx_t* labels, const SearchParameters* params,
                             hipStream_t stream) const;
    struct SearchGraph {
        std::string key;
        int seen = 0;
        bool failed = false;
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        // the event-record nodes of the stages timed at capture (kernel
        // timing; this index's and the quantizer's): each replay records
        // fresh events there, listed in the owner's times (tsinks)
        std::vector<KernelTimes*> tsinks;
        std::vector<std::string> tnames;
        std::vector<double> tunits;
        std::vector<std::pair<hipGraphNode_t, hipGraphNode_t>> tnodes;
        uint64_t used = 0;  // last use (the least recent entry is replaced)
        void clear();
    };
    // one entry per distinct call (a paged host search replays one per page)
    mutable std::array<SearchGraph, 8> graphs_;
    mutable uint64_t graph_tick_ = 0;
    mutable bool capturing_ = false;
    // query image the flat quantizer prepared into s_q_ for the chunk
    // search() is scanning (IndexFlat::assign_device_qimg), null outside it
    mutable const void* shared_qimg_ = nullptr;
    // device order of calls on different streams sharing this index's scratch
    mutable StreamOrder order_;
    // search_stats: per-query completion stamps of the chunk being scanned
    // (device clock, written by the kernel that emits a query's result),
    // null outside such a call
    mutable unsigned long long* qdone_ = nullptr;
    // search_preassigned of a caller assignment naming a list twice for a
    // query: the exact scan (the list-centric filter assumes distinct probes)
    mutable bool dup_probes_ = false;
    mutable DeviceBuffer s_qdone_, s_stamps_;
    mutable DeviceBuffer s_as_, s_ad_, s_stats_, s_ilist_, s_idesc_, s_ient_, s_lim_, s_alim_,
            s_selmask_;
    // bucket counts of this call (zero; the call's scan clears them again);
    // flip_counts() after the bucket kernels are queued
    uint32_t* bucket_counts(hipStream_t s, uint32_t** next) const;
    void flip_counts() const {
        counts_parity_ ^= 1;
        counts_pending_ = false;
    }
    mutable bool counts_pending_ = false, counts_stream_valid_ = false;
    mutable hipStream_t counts_stream_ = nullptr;
    mutable int counts_parity_ = 0;
    // one pass of the range scan (counts when offs == nullptr, else fill);
    // cdis = coarse distances [n][np] on the device (PQ table 1 dis0)
    virtual void range_launch(const float* x, idx_t n, int ldx, const int32_t* assign,
                              const float* cdis, int np, float radius, const uint8_t* sel,
                              uint32_t* counts, const uint64_t* offs, float* D, idx_t* I,
                              bool store_pairs, hipStream_t s) const;

   private:
    idx_t search_chunk(idx_t n, size_t np, idx_t k) const;
    void search_host(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                     const SearchParameters* params, QueryLatencyStats* per_query_stats,
                     bool update_times) const;
};

struct IndexIVFFlat : IndexIVF {
    IndexIVFFlat(Index* quantizer, size_t d, size_t nlist, MetricType metric = METRIC_L2);
    // scan algorithm: 0 = auto (MFMA filter + exact re-rank when eligible),
    // 1 = the general exact scan (kernels_exact.hip).  Both give identical
    // results.
    int scan_mode = 0;
    void encode_vectors(idx_t n, const float* x, const idx_t* list_nos,
                        uint8_t* codes) const override;
    void search_preassigned_device(idx_t n, const float* x, int ldx, idx_t k, int nprobe,
                                   const int32_t* assign, const float* centroid_dis,
                                   float* distances, idx_t* labels, hipStream_t stream,
                                   const uint32_t* lim = nullptr, const uint8_t* sel = nullptr,
                                   bool store_pairs = false) const override;
    void reconstruct(idx_t key, float* recons) const override;

   protected:
    void upload_extra() const override;
    void exact_args(void* args) const override;
    const void* stream_image(size_t* row_bytes) const override;
    // one pass of the range scan (counts when offs == nullptr, else fill);
    // cdis = coarse distances [n][np] on the device (PQ table 1 dis0)
    virtual void range_launch(const float* x, idx_t n, int ldx, const int32_t* assign,
                              const float* cdis, int np, float radius, const uint8_t* sel,
                              uint32_t* counts, const uint64_t* offs, float* D, idx_t* I,
                              bool store_pairs, hipStream_t s) const override;
    mutable DeviceBuffer d_ynorm_, d_ynmax_, d_cbf_, d_cbs_, d_rres_, d_rmax_, s_part_, s_flags_;
    mutable int obits_ = 4;
    mutable int fold_ = 0;  // stream image carries folded norm fragments (L2)
};

// faiss/impl/ProductQuantizer.h:29-186
struct ProductQuantizer {
    size_t d = 0, M = 0, nbits = 8, dsub = 0, ksub = 256;
    std::vector<float> centroids;  // [M][ksub][dsub]
    ProductQuantizer() = default;
    ProductQuantizer(size_t d, size_t M, size_t nbits);
    void set_derived_values();
};

struct IndexIVFPQ : IndexIVF {
    ProductQuantizer pq;
    int use_precomputed_table = 0;  // faiss semantics: 0 / 1 (decided at train/read)
    int polysemous_ht = 0;
    IndexIVFPQ(Index* quantizer, size_t d, size_t nlist, size_t M, size_t nbits,
               MetricType metric = METRIC_L2);
    void train_encoder(idx_t n, const float* x, const idx_t* assign) override;
    void encode_vectors(idx_t n, const float* x, const idx_t* list_nos,
                        uint8_t* codes) const override;
    void search_preassigned_device(idx_t n, const float* x, int ldx, idx_t k, int nprobe,
                                   const int32_t* assign, const float* centroid_dis,
                                   float* distances, idx_t* labels, hipStream_t stream,
                                   const uint32_t* lim = nullptr, const uint8_t* sel = nullptr,
                                   bool store_pairs = false) const override;
    // faiss/IndexIVFPQ.cpp:364-459: choose 0/1 like the reference (the GPU
    // path uses per-code terms either way)
    void precompute_table();

   protected:
    void own_coarse_dis(idx_t n, const float* x, int ldx, int np, const int32_t* assign,
                        float* cdis, hipStream_t s) const override;
    void upload_extra() const override;
    void exact_args(void* args) const override;
    const void* stream_image(size_t* row_bytes) const override;
    // one pass of the range scan (counts when offs == nullptr, else fill);
    // cdis = coarse distances [n][np] on the device (PQ table 1 dis0)
    virtual void range_launch(const float* x, idx_t n, int ldx, const int32_t* assign,
                              const float* cdis, int np, float radius, const uint8_t* sel,
                              uint32_t* counts, const uint64_t* offs, float* D, idx_t* I,
                              bool store_pairs, hipStream_t s) const override;
    mutable DeviceBuffer d_pq_, d_terms_, d_cent_;
    // list-centric MFMA scan (kernels_pq_mfma.hip): bf16 decode table, per
    // row |y_R| and bf16 residual norm, per list maxima, |y_C| per list
    mutable DeviceBuffer d_dec_, d_prn_, d_prr_, d_lRmax_, d_lrmax_, d_cnorm_;
    mutable DeviceBuffer s_pkeys_, s_precs_, s_pflags_;
    mutable int pq_obits_ = 0;
    mutable bool pq_mfma_ready_ = false;
    // PQ stream image (kern::pq_stream_image): the decoded residuals in bf16
    // with the folded bias, what the streamed filter reads (4.3x the codes at
    // M = d / 2: HBM spent to take the decode out of the filter's loop)
    mutable DeviceBuffer d_pcbs_;
    mutable bool pq_stream_ready_ = false;
};

// ---------------------------------------------------------------- shards
// faiss/IndexShardsIVF.h:19-40 — shards sharing one coarse quantizer.
struct IndexShardsIVF : Index {
    Index* quantizer = nullptr;
    size_t nlist = 0;
    bool threaded = false, successive_ids = true;
    std::vector<IndexIVF*> shards;
    // shards (and the quantizer, owned by shard 0) deleted with this object
    // (index_ivf_to_shards)
    bool own_shards = false;
    IndexShardsIVF(Index* quantizer, size_t nlist, bool threaded = false,
                   bool successive_ids = true);
    ~IndexShardsIVF() override;
    // shards may live on other devices than the quantizer: the search then
    // runs as one RCCL communicator over the devices (shards.cpp)
    void add_shard(IndexIVF* idx);
    void add(idx_t n, const float* x) override;
    void add_with_ids(idx_t n, const float* x, const idx_t* xids) override;
    void train(idx_t n, const float* x) override;
    void search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                       idx_t* labels, const SearchParameters* params,
                       hipStream_t stream) const override;
    void reset() override;
    size_t nprobe = 1;

    // true when some shard is on another device than the quantizer (or
    // FAISS_AMD_SHARDS_RCCL=1): search over RCCL
    bool multi_device() const;

   private:
    mutable std::recursive_mutex mu_;
    mutable DeviceBuffer s_x_, s_cd_, s_ci_, s_all_d_, s_all_i_;
    struct MultiDev;
    mutable std::unique_ptr<MultiDev> md_;
    void search_multi(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                      idx_t* labels, const SearchParametersIVF* params, size_t np,
                      hipStream_t s) const;
};

// faiss/invlists/InvertedLists.h:36-43 subset types of copy_subset_to
enum SubsetType {
    SUBSET_TYPE_ID_RANGE = 0,
    SUBSET_TYPE_ID_MOD = 1,
    SUBSET_TYPE_ELEMENT_RANGE = 2,
    SUBSET_TYPE_INVLIST_FRACTION = 3,
    SUBSET_TYPE_INVLIST = 4,
};
// faiss/IndexIVF.cpp:1732-1739 + faiss/invlists/InvertedLists.cpp:91-175:
// append the entries of src selected by (subset_type, a1, a2) to dst's lists
// (same nlist / code_size); returns the number added (dst->ntotal grows)
size_t ivf_copy_subset_to(const IndexIVF* src, IndexIVF* dst, int subset_type, idx_t a1,
                          idx_t a2);
// faiss/gpu/GpuCloner.cpp:283-317 + :319-420 (IVF part of
// clone_Index_to_shards): nshard copies of src with empty lists (through
// write_index / read_index), shard i on devices[i], holding the entries of
// shard_type 1 (id % nshard == i), 2 (ids in [i ntotal / n, (i+1) ntotal / n))
// or 4 (lists [i nlist / n, (i+1) nlist / n)); ids are kept (successive_ids
// false).  The result owns its shards.
IndexShardsIVF* index_ivf_to_shards(const IndexIVF* src, int nshard, int shard_type,
                                    const int* devices);

// ---------------------------------------------------------------- misc
// GPU k-means (faiss/Clustering.h:23-59 defaults); assignment on the GPU
// (fp32 MFMA distance tiles + top-1), centroid update in double on the host.
void kmeans_train(int d, idx_t n, const float* x, int k, int niter, int64_t seed,
                  float* centroids, int device, bool verbose);

// faiss/utils/Heap.cpp:159-230 (host form)
void merge_knn_results(size_t n, size_t k, int nshard, const float* all_distances,
                       const idx_t* all_labels, float* distances, idx_t* labels,
                       MetricType metric);

// faiss/index_io.h
// faiss/index_io.h:37-64
constexpr int IO_FLAG_SKIP_STORAGE = 1;
constexpr int IO_FLAG_READ_ONLY = 2;
constexpr int IO_FLAG_ONDISK_SAME_DIR = 4;
constexpr int IO_FLAG_SKIP_IVF_DATA = 8;
constexpr int IO_FLAG_SKIP_PRECOMPUTE_TABLE = 16;
constexpr int IO_FLAG_PQ_SKIP_SDC_TABLE = 32;
constexpr int IO_FLAG_MMAP = IO_FLAG_SKIP_IVF_DATA | 0x646f0000;
void write_index(const Index* idx, const char* fname);
void write_index(const Index* idx, FILE* f);
Index* read_index(const char* fname, int io_flags = 0);
// IVF index whose inverted lists go to a separate `ilod` data file
// (OnDiskInvertedLists layout, faiss/invlists/OnDiskInvertedLists.cpp:683-704),
// as the reference produces with OnDiskInvertedLists + replace_invlists +
// write_index.
void write_index_ondisk(const Index* idx, const char* fname, const char* lists_fname);
Index* read_index(FILE* f, int io_flags = 0);

// faiss/index_factory.h (subset: Flat, IVFn[_HNSWm],Flat|PQm[xb][np], HNSWm)
Index* index_factory(int d, const char* description, MetricType metric = METRIC_L2);

// The reference's IndexIVF::search cuts a batch into min(omp threads, n)
// slices and quantizes each with the form its size selects (the direct
// fvec_L2sqr form below distance_compute_blas_threshold = 20 queries, else
// the BLAS form; faiss/IndexIVF.cpp:359-368, faiss/utils/distances.cpp:
// 807-823).  set_search_slices(t) makes the IVF searches emulate a reference
// run on t OpenMP threads (default 1: the batch is one slice); results can
// differ between t only by coarse near-ties.
void set_search_slices(int t);
int get_search_slices();

// float_rand (faiss/utils/random.cpp:95-112), bit-exact restatement
void float_rand(float* x, size_t n, int64_t seed);
// selected rows (row0, row0 + step, ...) of float_rand(n_rows * d, seed)
void float_rand_rows(float* out, int64_t n_rows, int d, int64_t seed, int64_t row0, int64_t step,
                     int64_t nout);

}  // namespace faiss_amd
