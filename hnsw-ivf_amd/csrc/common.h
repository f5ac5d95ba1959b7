// common.h — error handling, HIP helpers and device memory for the
// MI355X-native IVF search path.
//
// Error model mirrors the reference: preconditions throw a FaissException
// (reference faiss/impl/FaissAssert.h, faiss/impl/FaissException.h) which the
// C-ABI turns into return code -2 (reference c_api/macros_impl.h:22-56).
#pragma once
#include <algorithm>
#include <atomic>

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace faiss_amd {

using idx_t = int64_t;

enum MetricType { METRIC_INNER_PRODUCT = 0, METRIC_L2 = 1 };

class FaissException : public std::exception {
   public:
    explicit FaissException(const std::string& m) : msg(m) {}
    FaissException(const std::string& m, const char* func, const char* file, int line) {
        char buf[1024];
        snprintf(buf, sizeof(buf), "Error in %s at %s:%d: %s", func, file, line, m.c_str());
        msg = buf;
    }
    const char* what() const noexcept override { return msg.c_str(); }
    std::string msg;
};

#define FAISS_THROW_MSG(MSG) \
    throw ::faiss_amd::FaissException(MSG, __PRETTY_FUNCTION__, __FILE__, __LINE__)

#define FAISS_THROW_IF_NOT(X)                                         \
    do {                                                              \
        if (!(X)) {                                                   \
            FAISS_THROW_MSG("Error: '" #X "' failed");                \
        }                                                             \
    } while (0)

#define FAISS_THROW_IF_NOT_MSG(X, MSG)                                \
    do {                                                              \
        if (!(X)) {                                                   \
            FAISS_THROW_MSG(std::string("Error: '" #X "' failed: ") + (MSG)); \
        }                                                             \
    } while (0)

#define FAISS_THROW_FMT(FMT, ...)                                     \
    do {                                                              \
        char __buf[1024];                                             \
        snprintf(__buf, sizeof(__buf), FMT, __VA_ARGS__);             \
        FAISS_THROW_MSG(__buf);                                       \
    } while (0)

#define FAISS_THROW_IF_NOT_FMT(X, FMT, ...)                           \
    do {                                                              \
        if (!(X)) {                                                   \
            FAISS_THROW_FMT("Error: '" #X "' failed: " FMT, __VA_ARGS__); \
        }                                                             \
    } while (0)

#define HIP_CHECK(expr)                                                            \
    do {                                                                           \
        hipError_t __e = (expr);                                                   \
        if (__e != hipSuccess) {                                                   \
            FAISS_THROW_FMT("HIP error %d (%s) in %s", (int)__e,                   \
                            hipGetErrorString(__e), #expr);                        \
        }                                                                          \
    } while (0)

// Launch check: surfaces launch-configuration errors immediately.
#define HIP_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

inline size_t roundup(size_t a, size_t b) { return (a + b - 1) / b * b; }
inline size_t cdiv(size_t a, size_t b) { return (a + b - 1) / b; }

// Launch geometry.  An AQL dispatch packet counts the work-items of a grid
// dimension (blocks x threads) in 32 bits, so a 1-D launch past 2^32 - 1
// work-items does not fail on its own: the count wraps and the tail of the
// range is never visited (the round-5 100M-row PQ image: rows x (DB + 8)
// ≈ 1.2e10 work-items, most of the image unwritten).  Every launch takes its
// grid from kgrid(), which throws instead; kernels over int64 element counts
// take a bounded grid from stride_grid() and loop (GRID_STRIDE).
inline dim3 kgrid(int64_t blocks, int threads) {
    if (blocks < 1 || (uint64_t)blocks * (uint64_t)threads > 0xffffffffull) {
        FAISS_THROW_FMT("launch of %lld blocks x %d threads is outside the 32-bit work-item "
                        "count of a dispatch",
                        (long long)blocks, threads);
    }
    return dim3((unsigned)blocks);
}
constexpr int64_t kStrideGridMax = 8192;  // 256 CUs x 32 blocks: fills the chip, then loops
inline dim3 stride_grid(int64_t n, int threads) {
    const int64_t b = (int64_t)cdiv((size_t)std::max<int64_t>(n, 1), (size_t)threads);
    return dim3((unsigned)std::min<int64_t>(b, kStrideGridMax));
}
#define GRID_STRIDE(i, n)                                                                  \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)(n);     \
         i += (int64_t)gridDim.x * blockDim.x)

// Owning device buffer (hipMalloc'ed), bound to the device current at alloc.
// bumped by every DeviceBuffer (re)allocation: a captured search graph
// (IndexIVF::search_device) holds raw pointers and is replayed only while
// this has not moved
inline std::atomic<uint64_t>& devbuf_epoch() {
    static std::atomic<uint64_t> e{0};
    return e;
}

struct DeviceBuffer {
    void* ptr = nullptr;
    size_t bytes = 0;
    int device = -1;
    DeviceBuffer() = default;
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    DeviceBuffer(DeviceBuffer&& o) noexcept { *this = std::move(o); }
    DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
        if (this != &o) {
            release();
            ptr = o.ptr; bytes = o.bytes; device = o.device;
            o.ptr = nullptr; o.bytes = 0;
        }
        return *this;
    }
    ~DeviceBuffer() { release(); }
    void release() {
        if (ptr) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            if (device >= 0 && device != cur) (void)hipSetDevice(device);
            (void)hipFree(ptr);
            if (device >= 0 && device != cur) (void)hipSetDevice(cur);
            ptr = nullptr;
            bytes = 0;
        }
    }
    // grow-only reallocation (contents not preserved)
    void reserve(size_t nbytes) {
        if (nbytes <= bytes && ptr) return;
        devbuf_epoch().fetch_add(1, std::memory_order_relaxed);  // (captured graphs go stale)
        release();
        size_t nb = nbytes ? nbytes : 16;
        HIP_CHECK(hipGetDevice(&device));
        HIP_CHECK(hipMalloc(&ptr, nb));
        bytes = nb;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(ptr); }
};

// Per-device resources: one non-blocking stream per device, created lazily.
struct DeviceContext {
    int device = 0;
    hipStream_t stream = nullptr;
};

DeviceContext& device_context(int device);
int current_device();  // device selected by faiss_amd_set_device for this thread
void ensure_hip();     // throws a FaissException when no HIP device is usable

// Device order between calls that share an index's scratch buffers but run
// on different streams: a device entry point calls enter(s) first (s waits
// for the event the previous call recorded on its stream) and leave(s) after
// its last launch.  Same-stream calls are ordered by the stream itself.
struct StreamOrder {
    hipStream_t last = nullptr;
    hipEvent_t ev = nullptr;
    bool valid = false;
    StreamOrder() = default;
    StreamOrder(const StreamOrder&) = delete;
    StreamOrder& operator=(const StreamOrder&) = delete;
    void enter(hipStream_t s) {
        if (valid && last != s) HIP_CHECK(hipStreamWaitEvent(s, ev, 0));
    }
    void leave(hipStream_t s) {
        if (!ev) HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(ev, s));
        last = s;
        valid = true;
    }
    ~StreamOrder() {
        if (ev) (void)hipEventDestroy(ev);
    }
};

// Kernel-time recorder (HIP events) used by bench.py for the roofline line.
// Events are recorded on the launch stream without synchronising; elapsed
// times are resolved lazily when queried.
struct KernelTimes {
    std::vector<std::string> names;
    std::vector<hipEvent_t> e0, e1;
    std::vector<double> units;
    std::vector<double> millis;  // resolved
    size_t resolved = 0;
    void clear() {
        for (auto e : e0) (void)hipEventDestroy(e);
        for (auto e : e1) (void)hipEventDestroy(e);
        names.clear(); e0.clear(); e1.clear(); units.clear(); millis.clear();
        resolved = 0;
    }
    void resolve() {
        for (; resolved < e0.size(); resolved++) {
            float ms = 0;
            (void)hipEventSynchronize(e1[resolved]);
            (void)hipEventElapsedTime(&ms, e0[resolved], e1[resolved]);
            millis.push_back(ms);
        }
    }
    ~KernelTimes() { clear(); }
};
bool kernel_timing_enabled();
void set_kernel_timing_enabled(bool);
// only the kernel stage of this name is timed (nullptr / "": all of them)
void set_kernel_timing_filter(const char* name);
bool kernel_timing_wants(const char* name);
std::string kernel_timing_state();  // "off" / "on:<only>" (graph cache keys)

// Brackets a launch with HIP events when timing is enabled.
struct ScopedKernelTimer {
    KernelTimes* sink;
    hipStream_t stream;
    hipEvent_t a = nullptr, b = nullptr;
    ScopedKernelTimer(KernelTimes* s, const char* name, double units, hipStream_t st)
            : sink(s), stream(st) {
        if (sink && kernel_timing_wants(name)) {
            HIP_CHECK(hipEventCreate(&a));
            HIP_CHECK(hipEventCreate(&b));
            HIP_CHECK(hipEventRecord(a, stream));
            sink->names.push_back(name);
            sink->units.push_back(units);
        }
    }
    ~ScopedKernelTimer() {
        if (a) {
            (void)hipEventRecord(b, stream);
            sink->e0.push_back(a);
            sink->e1.push_back(b);
        }
    }
};

}  // namespace faiss_amd
