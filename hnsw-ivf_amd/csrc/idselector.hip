// idselector.hip — IDSelector membership (faiss/impl/IDSelector.cpp) evaluated
// on the GPU over the inverted-list arena: mask[r] = is_member(ids[r]) for
// every arena row r (padding rows, id < 0, are never members).  The scans
// drop non-members exactly like the reference's `use_sel` branch
// (faiss/IndexIVFFlat.cpp:165-167, faiss/IndexIVFPQ.cpp:777-780): such rows
// are never candidates, while ndis still counts whole lists (scan_one_list
// returns list_size, faiss/IndexIVF.cpp:546-586).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/faiss_amd.h"
#include "common.h"
#include "kernels.h"

namespace faiss_amd {

namespace kern {

__global__ void k_sel_range(const int64_t* __restrict__ ids, int64_t n, int64_t imin,
                            int64_t imax, uint8_t* __restrict__ mask) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t id = ids[r];
    mask[r] = id >= 0 && id >= imin && id < imax ? 1 : 0;
}

// membership in a sorted id array (binary search)
__global__ void k_sel_sorted(const int64_t* __restrict__ ids, int64_t n,
                             const int64_t* __restrict__ set, int64_t m,
                             uint8_t* __restrict__ mask) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t id = ids[r];
    int64_t lo = 0, hi = m;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (set[mid] < id) lo = mid + 1;
        else hi = mid;
    }
    mask[r] = id >= 0 && lo < m && set[lo] == id ? 1 : 0;
}

__global__ void k_sel_bitmap(const int64_t* __restrict__ ids, int64_t n,
                             const uint8_t* __restrict__ bitmap, int64_t nb,
                             uint8_t* __restrict__ mask) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t id = ids[r];
    const uint64_t i = (uint64_t)id;
    mask[r] = id >= 0 && (i >> 3) < (uint64_t)nb ? (bitmap[i >> 3] >> (i & 7)) & 1 : 0;
}

// op 0 and, 1 or, 2 xor, 3 not (a only); padding rows stay 0
__global__ void k_sel_combine(const int64_t* __restrict__ ids, int64_t n, uint8_t* __restrict__ a,
                              const uint8_t* __restrict__ b, int op) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    uint8_t v;
    if (op == 0) v = a[r] & b[r];
    else if (op == 1) v = a[r] | b[r];
    else if (op == 2) v = a[r] ^ b[r];
    else v = a[r] ^ 1;
    a[r] = ids[r] >= 0 ? v : 0;
}

// IndexFlat::search_selected: non-member columns of a distance tile get a
// value the select does not admit
__global__ void k_mask_cols(float* __restrict__ D, int64_t nx, int64_t ny, int64_t ldD,
                            const uint8_t* __restrict__ mask, float v) {
    GRID_STRIDE(i, nx * ny) {
        const int64_t r = i / ny, c = i - r * ny;
        if (!mask[c]) D[r * ldD + c] = v;
    }
}
void mask_columns(float* D, int64_t nx, int64_t ny, int64_t ldD, const uint8_t* mask, float v,
                  hipStream_t s) {
    if (nx <= 0 || ny <= 0) return;
    k_mask_cols<<<stride_grid(nx * ny, 256), dim3(256), 0, s>>>(D, nx, ny, ldD, mask, v);
    HIP_LAUNCH_CHECK();
}

}  // namespace kern

namespace {
dim3 grid_of(int64_t n) { return kgrid(std::max<int64_t>(1, cdiv(n, 256)), 256); }

// device copy of a host array for the duration of one mark_device call
struct DevTmp {
    void* p = nullptr;
    DevTmp(const void* h, size_t bytes, hipStream_t s) {
        HIP_CHECK(hipMalloc(&p, std::max<size_t>(bytes, 8)));
        if (bytes) HIP_CHECK(hipMemcpyAsync(p, h, bytes, hipMemcpyHostToDevice, s));
    }
    ~DevTmp() { (void)hipFree(p); }  // hipFree synchronises the device
};
}  // namespace

void IDSelectorRange::mark_device(const idx_t* ids, int64_t n, uint8_t* mask,
                                  hipStream_t s) const {
    if (n <= 0) return;
    kern::k_sel_range<<<grid_of(n), 256, 0, s>>>(ids, n, imin, imax, mask);
    HIP_LAUNCH_CHECK();
}

bool IDSelectorArray::is_member(idx_t id) const {
    for (size_t i = 0; i < n; i++)
        if (ids[i] == id) return true;
    return false;
}
void IDSelectorArray::mark_device(const idx_t* aids, int64_t na, uint8_t* mask,
                                  hipStream_t s) const {
    if (na <= 0) return;
    std::vector<idx_t> v(ids, ids + n);
    std::sort(v.begin(), v.end());
    DevTmp t(v.data(), sizeof(idx_t) * v.size(), s);
    kern::k_sel_sorted<<<grid_of(na), 256, 0, s>>>(aids, na, (const int64_t*)t.p,
                                                   (int64_t)v.size(), mask);
    HIP_LAUNCH_CHECK();
}

IDSelectorBatch::IDSelectorBatch(size_t n, const idx_t* indices) : sorted(indices, indices + n) {
    std::sort(sorted.begin(), sorted.end());
    sorted.erase(std::unique(sorted.begin(), sorted.end()), sorted.end());
}
bool IDSelectorBatch::is_member(idx_t id) const {
    return std::binary_search(sorted.begin(), sorted.end(), id);
}
void IDSelectorBatch::mark_device(const idx_t* ids, int64_t n, uint8_t* mask,
                                  hipStream_t s) const {
    if (n <= 0) return;
    DevTmp t(sorted.data(), sizeof(idx_t) * sorted.size(), s);
    kern::k_sel_sorted<<<grid_of(n), 256, 0, s>>>(ids, n, (const int64_t*)t.p,
                                                  (int64_t)sorted.size(), mask);
    HIP_LAUNCH_CHECK();
}

void IDSelectorBitmap::mark_device(const idx_t* ids, int64_t na, uint8_t* mask,
                                   hipStream_t s) const {
    if (na <= 0) return;
    DevTmp t(bitmap, n, s);
    kern::k_sel_bitmap<<<grid_of(na), 256, 0, s>>>(ids, na, (const uint8_t*)t.p, (int64_t)n,
                                                   mask);
    HIP_LAUNCH_CHECK();
}

void IDSelectorNot::mark_device(const idx_t* ids, int64_t n, uint8_t* mask,
                                hipStream_t s) const {
    if (n <= 0) return;
    sel->mark_device(ids, n, mask, s);
    kern::k_sel_combine<<<grid_of(n), 256, 0, s>>>(ids, n, mask, nullptr, 3);
    HIP_LAUNCH_CHECK();
}

void IDSelectorBinary::mark_device(const idx_t* ids, int64_t n, uint8_t* mask,
                                   hipStream_t s) const {
    if (n <= 0) return;
    lhs->mark_device(ids, n, mask, s);
    DeviceBuffer tmp;
    tmp.reserve((size_t)n);
    rhs->mark_device(ids, n, tmp.as<uint8_t>(), s);
    kern::k_sel_combine<<<grid_of(n), 256, 0, s>>>(ids, n, mask, tmp.as<uint8_t>(), op);
    HIP_LAUNCH_CHECK();
    HIP_CHECK(hipStreamSynchronize(s));  // tmp is freed on return
}

}  // namespace faiss_amd
