// core.cpp — device contexts, Index base, IndexFlat (coarse quantizer),
// GPU k-means, host merge_knn_results and the float_rand restatement.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../../include/faiss_amd.h"
#include "kernels.h"

namespace faiss_amd {
namespace kern {
// idselector.hip: D[r][c] = v for every column c whose mask byte is 0
void mask_columns(float* D, int64_t nx, int64_t ny, int64_t ldD, const uint8_t* mask, float v,
                  hipStream_t s);
}  // namespace kern

IndexIVFStats indexIVF_stats;
HNSWStats hnsw_stats;
HNSWRowStats hnsw_row_stats;

// ---------------------------------------------------------------- interrupts
// faiss/impl/AuxIndexStructures.cpp:204-262 (behaviour restated)
std::mutex InterruptCallback::lock;
std::unique_ptr<InterruptCallback> InterruptCallback::instance;

void InterruptCallback::clear_instance() { instance.reset(); }

void InterruptCallback::check() {
    // through is_interrupted(), under the lock (TimeoutCallback fires once)
    if (is_interrupted()) FAISS_THROW_MSG("computation interrupted");
}

bool InterruptCallback::is_interrupted() {
    if (!instance) return false;
    std::lock_guard<std::mutex> g(lock);
    return instance->want_interrupt();
}

size_t InterruptCallback::get_period_hint(size_t flops) {
    if (!instance) return (size_t)1 << 30;  // no callback: never poll
    // a poll every ~100 Mflop of work
    return std::max<size_t>((size_t)100000000 / (flops + 1), 1);
}

bool TimeoutCallback::want_interrupt() {
    if (timeout == 0) return false;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
    if (el <= timeout) return false;
    timeout = 0;  // fires once
    return true;
}

void TimeoutCallback::set_timeout(double timeout_in_seconds) {
    timeout = timeout_in_seconds;
    start = std::chrono::steady_clock::now();
}

void TimeoutCallback::reset(double timeout_in_seconds) {
    auto* tc = new TimeoutCallback();
    InterruptCallback::instance.reset(tc);
    tc->set_timeout(timeout_in_seconds);
}

// ---------------------------------------------------------------- devices
namespace {
std::mutex g_ctx_mu;
std::vector<std::unique_ptr<DeviceContext>> g_ctx;
thread_local int tl_device = 0;
bool g_timing = false;
}  // namespace

void ensure_hip() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        FAISS_THROW_MSG(
                "no usable HIP device: the MI355X IVF search path has no CPU fallback "
                "(hipGetDeviceCount: " +
                std::string(hipGetErrorString(e)) + ")");
    }
}

DeviceContext& device_context(int device) {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    if ((int)g_ctx.size() <= device) g_ctx.resize(device + 1);
    if (!g_ctx[device]) {
        ensure_hip();
        auto c = std::make_unique<DeviceContext>();
        c->device = device;
        int cur = 0;
        HIP_CHECK(hipGetDevice(&cur));
        HIP_CHECK(hipSetDevice(device));
        HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        HIP_CHECK(hipSetDevice(cur));
        g_ctx[device] = std::move(c);
    }
    return *g_ctx[device];
}

int current_device() { return tl_device; }
void set_current_device(int d) { tl_device = d; }
bool kernel_timing_enabled() { return g_timing; }
void set_kernel_timing_enabled(bool b) { g_timing = b; }
namespace {
std::mutex g_timing_mu;
std::string g_timing_only;  // empty: every timed kernel
}  // namespace
void set_kernel_timing_filter(const char* name) {
    std::lock_guard<std::mutex> g(g_timing_mu);
    g_timing_only = name ? name : "";
}
std::string kernel_timing_state() {
    if (!g_timing) return "off";
    std::lock_guard<std::mutex> g(g_timing_mu);
    return "on:" + g_timing_only;
}
bool kernel_timing_wants(const char* name) {
    if (!g_timing) return false;
    std::lock_guard<std::mutex> g(g_timing_mu);
    return g_timing_only.empty() || g_timing_only == name;
}

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int dev) {
        ensure_hip();
        HIP_CHECK(hipGetDevice(&prev));
        if (prev != dev) HIP_CHECK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur = 0;
        hipGetDevice(&cur);
        if (cur != prev) hipSetDevice(prev);
    }
};

// ---------------------------------------------------------------- Index
Index::Index(idx_t d_, MetricType metric) : d((int)d_), metric_type(metric) {
    device = current_device();
}
Index::~Index() = default;

void Index::train(idx_t, const float*) {}

void Index::add_with_ids(idx_t, const float*, const idx_t*) {
    FAISS_THROW_MSG("add_with_ids not implemented for this type of index");
}

void Index::assign_device(idx_t, const float*, int, int, float*, int32_t*,
                          const SearchParameters*, hipStream_t) const {
    FAISS_THROW_MSG("this index cannot be used as a coarse quantizer");
}

void Index::reconstruct(idx_t, float*) const {
    FAISS_THROW_MSG("reconstruct not implemented for this type of index");
}

void Index::range_search(idx_t, const float*, float, RangeSearchResult*,
                         const SearchParameters*) const {
    FAISS_THROW_MSG("range search not implemented for this type of index");  // faiss/Index.cpp:39
}

hipStream_t Index::stream() const { return device_context(device).stream; }

// Host entry: upload (zero-padded rows) into this index's cached device
// buffers, search_device, download.  (HIP stages pageable host memory through
// its own pinned buffers; a pinned caller buffer goes straight to the DMA
// engine.  A staging pipeline of our own measured slower on c2: 0.67 vs 0.61
// ms per 10k-query call.)
void Index::search(idx_t n, const float* x, idx_t k, float* distances, idx_t* labels,
                   const SearchParameters* params) const {
    FAISS_THROW_IF_NOT(k > 0);
    if (n == 0) return;
    DeviceGuard g(device);
    sync_device();
    hipStream_t s = stream();
    const int ldx = ld();
    std::lock_guard<std::mutex> hg(host_mu_);
    h_x_.reserve(sizeof(float) * n * ldx);
    h_d_.reserve(sizeof(float) * n * k);
    h_i_.reserve(sizeof(idx_t) * n * k);
    if (ldx != d) HIP_CHECK(hipMemsetAsync(h_x_.ptr, 0, sizeof(float) * n * ldx, s));
    HIP_CHECK(hipMemcpy2DAsync(h_x_.ptr, sizeof(float) * ldx, x, sizeof(float) * d,
                               sizeof(float) * d, n, hipMemcpyHostToDevice, s));
    search_device(n, h_x_.as<float>(), ldx, k, h_d_.as<float>(), h_i_.as<idx_t>(), params, s);
    HIP_CHECK(hipMemcpyAsync(distances, h_d_.ptr, sizeof(float) * n * k, hipMemcpyDeviceToHost,
                             s));
    HIP_CHECK(hipMemcpyAsync(labels, h_i_.ptr, sizeof(idx_t) * n * k, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    fold_device_stats();
    // IndexHNSW::search polls the interrupt callback (faiss/IndexHNSW.cpp:315;
    // the batch is one device pass); IndexFlat::search does not
    if (dynamic_cast<const IndexHNSW*>(this)) InterruptCallback::check();
}

// ---------------------------------------------------------------- IndexFlat
IndexFlat::IndexFlat(idx_t d_, MetricType metric) : Index(d_, metric) {}

void IndexFlat::add(idx_t n, const float* x) {
    FAISS_THROW_IF_NOT(n >= 0);
    xb.insert(xb.end(), x, x + (size_t)n * d);
    ntotal += n;
    version_++;
    std::lock_guard<std::recursive_mutex> g(mu_);
    dirty_ = true;
}

void IndexFlat::reset() {
    xb.clear();
    ntotal = 0;
    version_++;
    std::lock_guard<std::recursive_mutex> g(mu_);
    dirty_ = true;
}

void IndexFlat::reconstruct(idx_t key, float* recons) const {
    FAISS_THROW_IF_NOT(key >= 0 && key < ntotal);
    memcpy(recons, xb.data() + (size_t)key * d, sizeof(float) * d);
}

void IndexFlat::stream_enter(hipStream_t s) const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    order_.enter(s);
}
void IndexFlat::stream_leave(hipStream_t s) const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    order_.leave(s);
}

void IndexFlat::sync_device() const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (!dirty_) return;
    DeviceGuard dg(device);
    hipStream_t s = stream();
    const int l = ld();
    d_xb_.reserve(sizeof(float) * std::max<idx_t>(ntotal, 1) * l);
    d_norms_.reserve(sizeof(float) * std::max<idx_t>(ntotal, 1));
    if (ntotal > 0) {
        if (l != d) HIP_CHECK(hipMemsetAsync(d_xb_.ptr, 0, sizeof(float) * ntotal * l, s));
        HIP_CHECK(hipMemcpy2DAsync(d_xb_.ptr, sizeof(float) * l, xb.data(), sizeof(float) * d,
                                   sizeof(float) * d, ntotal, hipMemcpyHostToDevice, s));
        kern::row_norms(d_xb_.as<float>(), ntotal, d, l, d_norms_.as<float>(), s);
        // bf16 hi/lo image + largest norm for the bf16x3 coarse filter
        if (kern::bf3_db_host(d) <= 128) {
            const int DB = kern::bf3_db_host(d);
            d_cbf_.reserve((size_t)ntotal * 2 * DB * 2);
            // {max |c|^2, max |c - bf16(c)|}: the coarse filter's margins
            d_cnmax_.reserve(2 * sizeof(float));
            kern::split_bf16(d_xb_.as<float>(), ntotal, d, l, DB, d_cbf_.ptr, s);
            kern::array_max(d_norms_.as<float>(), ntotal, d_cnmax_.as<float>(), s);
            s_tile_.reserve(sizeof(float) * ntotal);
            kern::row_resnorm_bf16(d_xb_.as<float>(), ntotal, d, l, s_tile_.as<float>(), s);
            kern::array_max(s_tile_.as<float>(), ntotal, d_cnmax_.as<float>() + 1, s);
            d_cst_.reserve(kern::coarse_stream_image_bytes(ntotal, d));
            // L2: the norms enter the coarse filter's MFMA as a bias k-step
            // (FAISS_AMD_COARSE_FOLD=0 keeps the fp32-norm tails)
            const char* fenv = getenv("FAISS_AMD_COARSE_FOLD");
            cfold_ = (metric_type == METRIC_L2 && !(fenv && !strcmp(fenv, "0"))) ? 1 : 0;
            kern::coarse_stream_image(d_xb_.as<float>(), ntotal, d, l, d_norms_.as<float>(),
                                      d_cst_.ptr, s, cfold_);
        }
    }
    HIP_CHECK(hipStreamSynchronize(s));
    dirty_ = false;
}

const float* IndexFlat::device_vectors() const {
    sync_device();
    return d_xb_.as<float>();
}
size_t IndexFlat::query_image_size(idx_t n) const {
    return kern::query_image_bytes(n, d) + sizeof(float) * n;
}
const float* IndexFlat::device_norms() const {
    sync_device();
    return d_norms_.as<float>();
}

template <class OutIdx>
bool IndexFlat::knn_device(idx_t n, const float* x, int ldx, int k, float* distances,
                           OutIdx* labels, hipStream_t s, void* qimg_out, idx_t batch_n) const {
    FAISS_THROW_IF_NOT_FMT(k >= 1, "k = %d must be >= 1", k);
    sync_device();
    std::lock_guard<std::recursive_mutex> g(mu_);
    order_.enter(s);
    // faiss/utils/distances.cpp:807-823: batches below
    // distance_compute_blas_threshold (20) take the direct form
    const bool direct = (batch_n >= 0 ? batch_n : n) < 20;
    const bool img = knn_impl<OutIdx>(n, x, ldx, k, distances, labels, s, qimg_out, direct);
    order_.leave(s);
    return img;
}

template <class OutIdx>
bool IndexFlat::knn_impl(idx_t n, const float* x, int ldx, int k, float* distances,
                         OutIdx* labels, hipStream_t s, void* qimg_out, bool direct) const {
    const int l = ld();
    const int metric_l2 = metric_type == METRIC_L2;
    if (k > kern::kMaxK) {
        // large k (e.g. nprobe > 64): whole distance rows in the reference's
        // form (direct below 20 queries, else BLAS form on the fp32 tile) and
        // the exact select with the heap's arrival-order tie rule
        if (metric_l2) {
            s_xn_.reserve(sizeof(float) * std::max<idx_t>(n, 1));
            kern::row_norms(x, n, d, ldx, s_xn_.as<float>(), s);
        }
        const idx_t ny = std::max<idx_t>(ntotal, 1);
        const idx_t qc = std::max<idx_t>(1, std::min<idx_t>(n, ((idx_t)1 << 28) / ny));
        s_tile_.reserve(sizeof(float) * qc * ny);
        ScopedKernelTimer tm(&ktimes, "flat_distance+select_exact", 2.0 * n * ntotal * d, s);
        for (idx_t q0 = 0; q0 < n; q0 += qc) {
            const idx_t nq = std::min(qc, n - q0);
            if (ntotal > 0 && direct)
                kern::direct_distances(x + q0 * ldx, nq, ldx, d_xb_.as<float>(), ntotal, l, d,
                                       metric_l2, s_tile_.as<float>(), ntotal, s);
            else if (ntotal > 0)
                kern::pairwise_distances(x + q0 * ldx, nq, ldx,
                                         metric_l2 ? s_xn_.as<float>() + q0 : nullptr,
                                         d_xb_.as<float>(), ntotal, l, d_norms_.as<float>(), l,
                                         metric_l2, s_tile_.as<float>(), ntotal, s);
            kern::select_rows_exact<OutIdx>(s_tile_.as<float>(), nq, ntotal, ntotal, k,
                                            metric_l2, 0, distances + q0 * k, labels + q0 * k, k,
                                            s, &s_sel_);
        }
        return false;
    }
    constexpr bool i32 = sizeof(OutIdx) == 4;
    int32_t* o32 = i32 ? (int32_t*)labels : nullptr;
    int64_t* o64 = i32 ? nullptr : (int64_t*)labels;
    const idx_t ny = ntotal;
    s_xn_.reserve(sizeof(float) * std::max<idx_t>(n, 1));
    // bf16x3 MFMA filter + certified exact re-rank: identical results to the
    // f32 tile + select below (FAISS_AMD_COARSE=f32 forces the latter)
    const char* cenv = getenv("FAISS_AMD_COARSE");
    const kern::CoarsePlan plan =
            (cenv && !strcmp(cenv, "f32")) || ny > (1 << 20) || d_cbf_.ptr == nullptr || direct
                    ? kern::CoarsePlan{}
                    : kern::coarse_bf3_plan(n, (int)ny, d, k);
    if (plan.ok) {
        // the streamed filter reads prepared query fragments (one launch with
        // the reference-order norms)
        const bool qi = d_cst_.ptr != nullptr && ldx % 4 == 0;
        void* qimg = nullptr;
        if (qi) {
            const size_t ib = kern::query_image_bytes(n, d);
            if (!qimg_out) s_qimg_.reserve(ib + sizeof(float) * n);
            qimg = qimg_out ? qimg_out : s_qimg_.ptr;
            ScopedKernelTimer tq(&ktimes, "query_prep", 0.0, s);
            kern::query_prep(x, n, ldx, d, s_xn_.as<float>(), qimg, (float*)((uint8_t*)qimg + ib),
                             s);
        } else {
            kern::row_norms(x, n, d, ldx, s_xn_.as<float>(), s);
        }
        const size_t per_q = (size_t)plan.entries * 4 + plan.nsplit * 16;
        const idx_t qchunk = std::max<idx_t>(64, (idx_t)(((size_t)256 << 20) / per_q) / 64 * 64);
        const idx_t qc = std::min<idx_t>(qchunk, n);
        s_cand_i_.reserve(sizeof(uint32_t) * qc * plan.entries);  // raw filter keys
        s_tile_.reserve(sizeof(float) * qc * plan.nsplit * 4);    // per-stream dropped bounds
        for (idx_t q0 = 0; q0 < n; q0 += qc) {
            const idx_t nq = std::min(qc, n - q0);
            kern::coarse_bf3_knn(plan, x + q0 * ldx, nq, ldx, s_xn_.as<float>() + q0,
                                 d_xb_.as<float>(), l, d_cbf_.ptr, d_norms_.as<float>(),
                                 d_cnmax_.as<float>(), (int)ny, d, k, metric_l2,
                                 s_cand_i_.as<uint32_t>(), s_tile_.as<float>(), distances + q0 * k,
                                 o32 ? o32 + q0 * k : nullptr, o64 ? o64 + q0 * k : nullptr, s,
                                 d_cst_.ptr,
                                 qi ? (const uint8_t*)qimg + q0 * kern::query_image_bytes(1, d)
                                    : nullptr,
                                 &ktimes, cfold_);
        }
        return qi && qimg_out;
    }
    if (metric_l2) kern::row_norms(x, n, d, ldx, s_xn_.as<float>(), s);
    const idx_t Yc = std::min<idx_t>(std::max<idx_t>(ny, 1), 1 << 20);
    const idx_t nyc = (idx_t)cdiv(std::max<idx_t>(ny, 1), Yc);
    FAISS_THROW_IF_NOT_MSG(!(i32 && nyc > 1), "coarse quantizer larger than 2^20 centroids");
    const size_t tile_budget = (size_t)256 << 20;  // bytes
    idx_t qchunk = std::max<idx_t>(128, (idx_t)(tile_budget / (sizeof(float) * Yc)) / 128 * 128);
    qchunk = std::min<idx_t>(qchunk, n);
    s_tile_.reserve(sizeof(float) * qchunk * Yc);
    if (nyc > 1) {
        s_cand_d_.reserve(sizeof(float) * nyc * qchunk * k);
        s_cand_i_.reserve(sizeof(idx_t) * nyc * qchunk * k);
    }
    double flops = 2.0 * (double)n * (double)ny * (double)d;
    ScopedKernelTimer tm(&ktimes, "flat_distance+select", flops, s);
    for (idx_t q0 = 0; q0 < n; q0 += qchunk) {
        const idx_t nq = std::min(qchunk, n - q0);
        const float* xq = x + q0 * ldx;
        const float* xn = s_xn_.as<float>() + q0;
        if (nyc == 1) {
            // faiss/utils/distances.cpp:807-823: blocks of fewer than
            // distance_compute_blas_threshold (20) queries take the direct form
            if (ny > 0 && direct)
                kern::direct_distances(xq, nq, ldx, d_xb_.as<float>(), ny, l, d, metric_l2,
                                       s_tile_.as<float>(), ny, s);
            else if (ny > 0)
                kern::pairwise_distances(xq, nq, ldx, xn, d_xb_.as<float>(), ny, l,
                                         d_norms_.as<float>(), l, metric_l2,
                                         s_tile_.as<float>(), ny, s);
            kern::select_rows(s_tile_.as<float>(), nq, ny, ny, k, metric_l2, 0,
                              distances + q0 * k, o32 ? o32 + q0 * k : nullptr,
                              o64 ? o64 + q0 * k : nullptr, k, s);
            if (!metric_l2 && ny > 0)
                kern::select_fix_ip(s_tile_.as<float>(), nq, ny, ny, k, distances + q0 * k,
                                    o32 ? o32 + q0 * k : nullptr, o64 ? o64 + q0 * k : nullptr,
                                    k, s);
        } else {
            for (idx_t c = 0; c < nyc; c++) {
                const idx_t y0 = c * Yc, nyy = std::min(Yc, ny - y0);
                if (direct)
                    kern::direct_distances(xq, nq, ldx, d_xb_.as<float>() + y0 * l, nyy, l, d,
                                           metric_l2, s_tile_.as<float>(), nyy, s);
                else
                    kern::pairwise_distances(xq, nq, ldx, xn, d_xb_.as<float>() + y0 * l, nyy,
                                             l, d_norms_.as<float>() + y0, l, metric_l2,
                                             s_tile_.as<float>(), nyy, s);
                kern::select_rows(s_tile_.as<float>(), nq, nyy, nyy, k, metric_l2, y0,
                                  s_cand_d_.as<float>() + c * nq * k, nullptr,
                                  s_cand_i_.as<int64_t>() + c * nq * k, k, s);
            }
            kern::merge_rows(s_cand_d_.as<float>(), s_cand_i_.as<int64_t>(), nq,
                             (int)((nyc << 16) | k), k, metric_l2, distances + q0 * k,
                             o64 + q0 * k, s);
        }
    }
    return false;
}

void IndexFlat::search_device(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                              idx_t* labels, const SearchParameters* params,
                              hipStream_t s) const {
    DeviceGuard g(device);
    if (params && params->sel) {
        search_selected(n, x, ldx, k, distances, labels, params->sel, s);
        return;
    }
    knn_device<idx_t>(n, x, ldx, (int)k, distances, labels, s);
}

void IndexFlat::search_selected(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                                idx_t* labels, const IDSelector* sel, hipStream_t s) const {
    FAISS_THROW_IF_NOT_FMT(k >= 1, "k = %lld must be >= 1", (long long)k);
    if (n <= 0) return;
    sync_device();
    std::lock_guard<std::recursive_mutex> g(mu_);
    order_.enter(s);
    const int l = ld();
    const int metric_l2 = metric_type == METRIC_L2;
    int64_t y0 = 0, ny = ntotal;
    const uint8_t* mask = nullptr;
    // faiss/utils/distances.cpp:807-823: below distance_compute_blas_threshold
    // (20) queries the direct form; with a selector other than a range the
    // direct form always (res.sel)
    bool direct = n < 20;
    if (auto r = dynamic_cast<const IDSelectorRange*>(sel)) {
        // knn_L2sqr / knn_inner_product (:840-935): the rows [imin, imax),
        // labels shifted back by imin, no selector left
        y0 = std::max<idx_t>(r->imin, 0);
        ny = std::max<idx_t>(std::min<idx_t>(r->imax, ntotal) - y0, 0);
        if (ny == 0) y0 = 0;
    } else if (ntotal > 0) {
        // (IDSelectorArray takes this membership form too: the reference's
        // knn_*_by_idx visits the array in its own order, which differs
        // only for an array that lists an id twice or under distance ties)
        direct = true;
        if (selids_n_ != ntotal) {
            std::vector<idx_t> iota((size_t)ntotal);
            for (idx_t i = 0; i < ntotal; i++) iota[(size_t)i] = i;
            s_selids_.reserve(sizeof(idx_t) * ntotal);
            HIP_CHECK(hipMemcpyAsync(s_selids_.ptr, iota.data(), sizeof(idx_t) * ntotal,
                                     hipMemcpyHostToDevice, s));
            HIP_CHECK(hipStreamSynchronize(s));  // (iota is a host temporary)
            selids_n_ = ntotal;
        }
        s_selmask_.reserve((size_t)ntotal);
        sel->mark_device(s_selids_.as<idx_t>(), ntotal, s_selmask_.as<uint8_t>(), s);
        mask = s_selmask_.as<uint8_t>();
    }
    if (metric_l2 && !direct && ny > 0) {
        s_xn_.reserve(sizeof(float) * n);
        kern::row_norms(x, n, d, ldx, s_xn_.as<float>(), s);
    }
    const idx_t qc = std::max<idx_t>(1, std::min<idx_t>(n, ((idx_t)1 << 28) / std::max<idx_t>(ny, 1)));
    s_tile_.reserve(sizeof(float) * qc * std::max<idx_t>(ny, 1));
    float* tile = s_tile_.as<float>();
    for (idx_t q0 = 0; q0 < n; q0 += qc) {
        const idx_t nq = std::min(qc, n - q0);
        if (ny > 0 && direct)
            kern::direct_distances(x + q0 * ldx, nq, ldx, d_xb_.as<float>() + y0 * l, ny, l, d,
                                   metric_l2, tile, ny, s);
        else if (ny > 0)
            kern::pairwise_distances(x + q0 * ldx, nq, ldx, s_xn_.as<float>() + q0,
                                     d_xb_.as<float>() + y0 * l, ny, l,
                                     d_norms_.as<float>() + y0, l, metric_l2, tile, ny, s);
        // non-members never reach the heap: a key the select does not admit
        if (mask && ny > 0)
            kern::mask_columns(tile, nq, ny, ny, mask, metric_l2 ? HUGE_VALF : -HUGE_VALF, s);
        float* Dq = distances + q0 * k;
        idx_t* Iq = labels + q0 * k;
        if (k <= kern::kMaxK) {
            kern::select_rows(tile, nq, ny, ny, (int)k, metric_l2, 0, Dq, nullptr, Iq, k, s);
            if (!metric_l2 && ny > 0)
                kern::select_fix_ip(tile, nq, ny, ny, (int)k, Dq, nullptr, Iq, k, s);
        } else {
            kern::select_rows_exact<idx_t>(tile, nq, ny, ny, (int)k, metric_l2, 0, Dq, Iq, k, s,
                                           &s_sel_);
        }
    }
    if (y0 > 0) kern::translate_labels(labels, n * k, y0, s);
    order_.leave(s);
}

void IndexFlat::assign_device(idx_t n, const float* x, int ldx, int k, float* distances,
                              int32_t* labels, const SearchParameters*, hipStream_t s) const {
    DeviceGuard g(device);
    knn_device<int32_t>(n, x, ldx, k, distances, labels, s);
}

void IndexFlat::assign_device_slice(idx_t n, const float* x, int ldx, int k, float* distances,
                                    int32_t* labels, const SearchParameters*, hipStream_t s,
                                    idx_t batch_n) const {
    DeviceGuard g(device);
    knn_device<int32_t>(n, x, ldx, k, distances, labels, s, nullptr, batch_n);
}

bool IndexFlat::assign_device_qimg(idx_t n, const float* x, int ldx, int k, float* distances,
                                   int32_t* labels, void* qimg, hipStream_t s) const {
    DeviceGuard g(device);
    return knn_device<int32_t>(n, x, ldx, k, distances, labels, s, qimg);
}

// ---------------------------------------------------------------- k-means
// faiss/Clustering.cpp semantics kept where they matter for index quality:
// subsample to 256 points per centroid, random initial centroids, niter
// Lloyd iterations, split_clusters for empty clusters (EPS = 1/1024).
void kmeans_train(int d, idx_t n, const float* x, int k, int niter, int64_t seed,
                  float* centroids, int device, bool verbose) {
    FAISS_THROW_IF_NOT_MSG(n >= k, "Number of training points should be at least as large as "
                                   "number of clusters");
    DeviceGuard g(device);
    std::mt19937 rng((unsigned)seed);
    std::vector<idx_t> perm(n);
    for (idx_t i = 0; i < n; i++) perm[i] = i;
    const idx_t max_pts = (idx_t)k * 256;
    std::vector<float> xs;
    const float* xt = x;
    idx_t nt = n;
    if (n > max_pts) {
        std::shuffle(perm.begin(), perm.end(), rng);
        nt = max_pts;
        xs.resize((size_t)nt * d);
        for (idx_t i = 0; i < nt; i++)
            memcpy(xs.data() + (size_t)i * d, x + (size_t)perm[i] * d, sizeof(float) * d);
        xt = xs.data();
        for (idx_t i = 0; i < nt; i++) perm[i] = i;
        perm.resize(nt);
    }
    std::shuffle(perm.begin(), perm.end(), rng);
    for (int c = 0; c < k; c++)
        memcpy(centroids + (size_t)c * d, xt + (size_t)perm[c] * d, sizeof(float) * d);

    const int ld = (int)roundup((size_t)d, 4);
    hipStream_t s = device_context(device).stream;
    DeviceBuffer bx, bd, bi;
    bx.reserve(sizeof(float) * nt * ld);
    bd.reserve(sizeof(float) * nt);
    bi.reserve(sizeof(int32_t) * nt);
    if (ld != d) HIP_CHECK(hipMemsetAsync(bx.ptr, 0, sizeof(float) * nt * ld, s));
    HIP_CHECK(hipMemcpy2DAsync(bx.ptr, sizeof(float) * ld, xt, sizeof(float) * d,
                               sizeof(float) * d, nt, hipMemcpyHostToDevice, s));
    std::vector<int32_t> assign(nt);
    std::vector<float> dis(nt);
    std::vector<double> sums((size_t)k * d);
    std::vector<idx_t> counts(k);
    IndexFlat cent(d, METRIC_L2);
    cent.device = device;
    for (int it = 0; it < niter; it++) {
        InterruptCallback::check();  // faiss/Clustering.cpp:487
        cent.reset();
        cent.add(k, centroids);
        cent.assign_device(nt, bx.as<float>(), ld, 1, bd.as<float>(), bi.as<int32_t>(), nullptr,
                           s);
        HIP_CHECK(hipMemcpyAsync(assign.data(), bi.ptr, sizeof(int32_t) * nt,
                                 hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipMemcpyAsync(dis.data(), bd.ptr, sizeof(float) * nt, hipMemcpyDeviceToHost,
                                 s));
        HIP_CHECK(hipStreamSynchronize(s));
        std::fill(sums.begin(), sums.end(), 0.0);
        std::fill(counts.begin(), counts.end(), 0);
        double obj = 0;
        for (idx_t i = 0; i < nt; i++) {
            int a = assign[i];
            FAISS_THROW_IF_NOT(a >= 0 && a < k);
            counts[a]++;
            obj += dis[i];
            const float* xi = xt + (size_t)i * d;
            double* sa = sums.data() + (size_t)a * d;
            for (int j = 0; j < d; j++) sa[j] += xi[j];
        }
        for (int c = 0; c < k; c++) {
            if (counts[c] == 0) continue;
            for (int j = 0; j < d; j++)
                centroids[(size_t)c * d + j] = (float)(sums[(size_t)c * d + j] / counts[c]);
        }
        // split_clusters (faiss/Clustering.cpp)
        const float EPS = 1.f / 1024.f;
        std::uniform_real_distribution<float> U(0.f, 1.f);
        for (int ci = 0; ci < k; ci++) {
            if (counts[ci] != 0) continue;
            int cj = 0;
            for (;; cj = (cj + 1) % k) {
                float p = (counts[cj] - 1.0f) / (float)(nt - k);
                if (U(rng) < p) break;
            }
            memcpy(centroids + (size_t)ci * d, centroids + (size_t)cj * d, sizeof(float) * d);
            for (int j = 0; j < d; j++) {
                if (j % 2 == 0) {
                    centroids[(size_t)ci * d + j] *= 1 + EPS;
                    centroids[(size_t)cj * d + j] *= 1 - EPS;
                } else {
                    centroids[(size_t)ci * d + j] *= 1 - EPS;
                    centroids[(size_t)cj * d + j] *= 1 + EPS;
                }
            }
            counts[ci] = counts[cj] / 2;
            counts[cj] -= counts[ci];
        }
        if (verbose) fprintf(stderr, "kmeans iter %d obj %g\n", it, obj);
    }
}

// ---------------------------------------------------------------- merge
// faiss/utils/Heap.cpp:159-230: per query, repeatedly take the best shard
// head (ties -> lower shard for L2, higher shard for IP, as the CMin/CMax
// heap pops them), stop a shard at its first -1, pad with the neutral value.
void merge_knn_results(size_t n, size_t k, int nshard, const float* all_distances,
                       const idx_t* all_labels, float* distances, idx_t* labels,
                       MetricType metric) {
    const size_t stride = n * k;
    const bool l2 = metric == METRIC_L2;
    std::vector<size_t> ptr(nshard);
    for (size_t i = 0; i < n; i++) {
        std::fill(ptr.begin(), ptr.end(), 0);
        size_t j = 0;
        for (; j < k; j++) {
            int best = -1;
            float bd = 0;
            for (int s = 0; s < nshard; s++) {
                size_t p = ptr[s];
                if (p >= k) continue;
                const idx_t lab = all_labels[s * stride + i * k + p];
                if (lab < 0) continue;
                float v = all_distances[s * stride + i * k + p];
                bool better;
                if (best < 0) better = true;
                else if (l2) better = v < bd;           // ties keep the lower shard
                else better = v > bd || v == bd;        // ties move to the higher shard
                if (better) {
                    best = s;
                    bd = v;
                }
            }
            if (best < 0) break;
            distances[i * k + j] = bd;
            labels[i * k + j] = all_labels[best * stride + i * k + ptr[best]];
            ptr[best]++;
        }
        for (; j < k; j++) {
            distances[i * k + j] = l2 ? FLT_MAX : -FLT_MAX;
            labels[i * k + j] = -1;
        }
    }
}

// ---------------------------------------------------------------- float_rand
// faiss/utils/random.cpp:35-53,95-112 — std::mt19937 streams, 1024 blocks.
void float_rand(float* x, size_t n, int64_t seed) {
    const size_t nblock = n < 1024 ? 1 : 1024;
    std::mt19937 rng0((unsigned int)seed);
    int a0 = (int)(rng0() & 0x7fffffff), b0 = (int)(rng0() & 0x7fffffff);
    auto run = [&](int64_t j0, int64_t j1) {
        for (int64_t j = j0; j < j1; j++) {
            std::mt19937 rng((unsigned int)(int64_t)(a0 + j * b0));
            const size_t istart = j * n / nblock;
            const size_t iend = (j + 1) * n / nblock;
            const float mx = (float)std::mt19937::max();
            for (size_t i = istart; i < iend; i++) x[i] = (float)rng() / mx;
        }
    };
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < (1 << 20)) nt = 1;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++) {
        int64_t j0 = (int64_t)nblock * t / nt, j1 = (int64_t)nblock * (t + 1) / nt;
        th.emplace_back(run, j0, j1);
    }
    for (auto& t : th) t.join();
}

// Rows row0, row0 + step, ... (nout of them) of the float_rand(n_rows * d,
// seed) stream viewed as [n_rows][d], without materialising the whole stream
// (the 100M-vector synthetic sets): the same 1024 mt19937 blocks as
// float_rand, each generated once, keeping the selected rows.
void float_rand_rows(float* out, int64_t n_rows, int d, int64_t seed, int64_t row0, int64_t step,
                     int64_t nout) {
    FAISS_THROW_IF_NOT(d > 0 && step > 0 && row0 >= 0);
    FAISS_THROW_IF_NOT(nout >= 0 && (nout == 0 || row0 + (nout - 1) * step < n_rows));
    const size_t n = (size_t)n_rows * d;
    const size_t nblock = n < 1024 ? 1 : 1024;
    std::mt19937 rng0((unsigned int)seed);
    int a0 = (int)(rng0() & 0x7fffffff), b0 = (int)(rng0() & 0x7fffffff);
    auto run = [&](int64_t j0, int64_t j1) {
        for (int64_t j = j0; j < j1; j++) {
            std::mt19937 rng((unsigned int)(int64_t)(a0 + j * b0));
            const size_t istart = j * n / nblock;
            const size_t iend = (j + 1) * n / nblock;
            const float mx = (float)std::mt19937::max();
            for (size_t i = istart; i < iend; i++) {
                const float v = (float)rng() / mx;
                const int64_t r = (int64_t)(i / d);
                if (r < row0 || (r - row0) % step != 0) continue;
                const int64_t o = (r - row0) / step;
                if (o < nout) out[(size_t)o * d + (i - (size_t)r * d)] = v;
            }
        }
    };
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < (1 << 20)) nt = 1;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++) {
        int64_t j0 = (int64_t)nblock * t / nt, j1 = (int64_t)nblock * (t + 1) / nt;
        th.emplace_back(run, j0, j1);
    }
    for (auto& t : th) t.join();
}

}  // namespace faiss_amd
