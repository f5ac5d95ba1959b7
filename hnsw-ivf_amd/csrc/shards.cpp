// shards.cpp — IndexShardsIVF across devices (one RCCL communicator in one
// process), the reference's subset copies and the IVF shard cloner.
//
// Reference: faiss/IndexShardsIVF.cpp:158-245 (search = one coarse pass, then
// search_preassigned on every shard, then merge_knn_results),
// faiss/gpu/GpuCloner.cpp:283-420 (clone_Index_to_shards, shard_type 1/2/4),
// faiss/invlists/InvertedLists.cpp:91-175 (copy_subset_to).
//
// Multi-device search, all on device-resident data:
//   rank 0 = the quantizer's device: coarse top-nprobe of the batch;
//   ncclBroadcast of the queries, coarse distances and list numbers to every
//   rank (grouped), each rank runs its shards' search_preassigned_device on its
//   own stream, ncclSend / ncclRecv bring the [n][k] tables to rank 0, which
//   shifts labels (successive_ids) and merges (merge_knn_results order: ties
//   to the lower shard).  xGMI is point to point, so the gather is per-peer
//   send/recv rather than a ring collective.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/faiss_amd.h"
#include "kernels.h"

namespace faiss_amd {

namespace {
struct SDevGuard {
    int prev = 0;
    explicit SDevGuard(int dev) {
        HIP_CHECK(hipGetDevice(&prev));
        if (prev != dev) HIP_CHECK(hipSetDevice(dev));
    }
    ~SDevGuard() {
        int cur = 0;
        hipGetDevice(&cur);
        if (cur != prev) hipSetDevice(prev);
    }
};

#define NCCL_CHECK(call)                                                                    \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        FAISS_THROW_IF_NOT_MSG(r_ == ncclSuccess,                                           \
                               std::string("RCCL error: ") + ncclGetErrorString(r_) + " in " \
                                       #call);                                              \
    } while (0)
}  // namespace

// ---------------------------------------------------------------- subsets
size_t ivf_copy_subset_to(const IndexIVF* src, IndexIVF* dst, int subset_type, idx_t a1,
                          idx_t a2) {
    FAISS_THROW_IF_NOT(src && dst && src != dst);
    const ArrayInvertedLists& il = *src->invlists;
    ArrayInvertedLists& ol = *dst->invlists;
    FAISS_THROW_IF_NOT(il.nlist == ol.nlist);
    FAISS_THROW_IF_NOT(il.code_size == ol.code_size);
    FAISS_THROW_IF_NOT_FMT(subset_type >= 0 && subset_type <= 4, "subset type %d not implemented",
                           subset_type);
    const size_t cs = il.code_size;
    size_t ntotal = 0;
    if (subset_type == SUBSET_TYPE_ELEMENT_RANGE)
        for (size_t l = 0; l < il.nlist; l++) ntotal += il.list_size(l);
    // arguments the reference's loops would index past a list with
    FAISS_THROW_IF_NOT_MSG(subset_type != SUBSET_TYPE_ID_MOD || a1 > 0, "ID_MOD needs a1 > 0");
    FAISS_THROW_IF_NOT_MSG(subset_type != SUBSET_TYPE_ELEMENT_RANGE ||
                                   (0 <= a1 && a1 <= a2 && (size_t)a2 <= ntotal),
                           "ELEMENT_RANGE needs 0 <= a1 <= a2 <= ntotal");
    FAISS_THROW_IF_NOT_MSG(subset_type != SUBSET_TYPE_INVLIST_FRACTION ||
                                   (a1 > 0 && 0 <= a2 && a2 < a1),
                           "INVLIST_FRACTION needs 0 <= a2 < a1");
    size_t accu_n = 0, accu_a1 = 0, accu_a2 = 0, n_added = 0;
    std::vector<idx_t> sid;
    std::vector<uint8_t> scode;
    for (size_t l = 0; l < il.nlist; l++) {
        const size_t n = il.list_size(l);
        const idx_t* ids = il.get_ids(l);
        const uint8_t* codes = il.get_codes(l);
        size_t i1 = 0, i2 = 0;  // a contiguous range, or a filtered list below
        bool filtered = false;
        if (subset_type == SUBSET_TYPE_ID_RANGE || subset_type == SUBSET_TYPE_ID_MOD) {
            sid.clear();
            scode.clear();
            for (size_t i = 0; i < n; i++) {
                const idx_t id = ids[i];
                const bool in = subset_type == SUBSET_TYPE_ID_RANGE ? (a1 <= id && id < a2)
                                                                    : (id % a1 == a2);
                if (in) {
                    sid.push_back(id);
                    scode.insert(scode.end(), codes + i * cs, codes + (i + 1) * cs);
                }
            }
            filtered = true;
        } else if (subset_type == SUBSET_TYPE_ELEMENT_RANGE) {
            // what the running totals allot to a1 and to a2 (InvertedLists.cpp:138-155)
            const size_t next_accu_n = accu_n + n;
            const size_t next_accu_a1 = ntotal ? next_accu_n * a1 / ntotal : 0;
            const size_t next_accu_a2 = ntotal ? next_accu_n * a2 / ntotal : 0;
            i1 = next_accu_a1 - accu_a1;
            i2 = next_accu_a2 - accu_a2;
            accu_n = next_accu_n;
            accu_a1 = next_accu_a1;
            accu_a2 = next_accu_a2;
        } else if (subset_type == SUBSET_TYPE_INVLIST_FRACTION) {
            i1 = n * a2 / a1;
            i2 = n * (a2 + 1) / a1;
        } else {  // SUBSET_TYPE_INVLIST
            if ((idx_t)l >= a1 && (idx_t)l < a2) {
                i1 = 0;
                i2 = n;
            }
        }
        if (filtered) {
            if (!sid.empty()) ol.add_entries(l, sid.size(), sid.data(), scode.data());
            n_added += sid.size();
        } else if (i2 > i1) {
            ol.add_entries(l, i2 - i1, ids + i1, codes + i1 * cs);
            n_added += i2 - i1;
        }
    }
    dst->ntotal += (idx_t)n_added;
    std::lock_guard<std::recursive_mutex> g(dst->mu_);
    dst->dirty_ = true;
    return n_added;
}

// ---------------------------------------------------------------- cloner
namespace {
// an empty copy of src (same quantizer, codebooks and parameters) on `device`
IndexIVF* clone_empty(const IndexIVF* src, int device) {
    char* buf = nullptr;
    size_t len = 0;
    FILE* w = open_memstream(&buf, &len);
    FAISS_THROW_IF_NOT_MSG(w, "open_memstream failed");
    try {
        write_index(src, w);
    } catch (...) {
        fclose(w);
        free(buf);
        throw;
    }
    fclose(w);
    FILE* r = fmemopen(buf, len, "rb");
    if (!r) {
        free(buf);
        FAISS_THROW_MSG("fmemopen failed");
    }
    Index* idx = nullptr;
    try {
        idx = read_index(r, 0);
    } catch (...) {
        fclose(r);
        free(buf);
        throw;
    }
    fclose(r);
    free(buf);
    IndexIVF* ivf = dynamic_cast<IndexIVF*>(idx);
    FAISS_THROW_IF_NOT(ivf);
    ivf->reset();
    ivf->device = device;
    ivf->quantizer->device = device;
    ivf->nprobe = src->nprobe;
    ivf->max_codes = src->max_codes;
    ivf->parallel_mode = src->parallel_mode;
    return ivf;
}
}  // namespace

IndexShardsIVF* index_ivf_to_shards(const IndexIVF* src, int nshard, int shard_type,
                                    const int* devices) {
    FAISS_THROW_IF_NOT(src && nshard >= 1);
    FAISS_THROW_IF_NOT_FMT(shard_type == 1 || shard_type == 2 || shard_type == 4,
                           "shard_type %d not implemented", shard_type);
    std::vector<IndexIVF*> sh;
    try {
        for (int i = 0; i < nshard; i++) {
            IndexIVF* s = clone_empty(src, devices ? devices[i] : src->device);
            sh.push_back(s);
            const idx_t n = nshard, ii = i;
            if (shard_type == 2) {  // GpuCloner.cpp:290-298
                const idx_t i0 = ii * src->ntotal / n, i1 = (ii + 1) * src->ntotal / n;
                ivf_copy_subset_to(src, s, SUBSET_TYPE_ID_RANGE, i0, i1);
            } else if (shard_type == 1) {  // :299-303
                ivf_copy_subset_to(src, s, SUBSET_TYPE_ID_MOD, n, ii);
            } else {  // :304-315
                const idx_t i0 = ii * (idx_t)src->nlist / n, i1 = (ii + 1) * (idx_t)src->nlist / n;
                ivf_copy_subset_to(src, s, SUBSET_TYPE_INVLIST, i0, i1);
            }
        }
    } catch (...) {
        for (auto* s : sh) delete s;
        throw;
    }
    auto* out = new IndexShardsIVF(sh[0]->quantizer, src->nlist, false, false);
    out->own_shards = true;
    out->nprobe = src->nprobe;
    for (auto* s : sh) out->add_shard(s);
    out->is_trained = src->is_trained;
    return out;
}

// ---------------------------------------------------------------- multi-device
struct IndexShardsIVF::MultiDev {
    std::vector<int> devs;        // rank -> device; rank 0 = the quantizer's device
    std::vector<int> shard_rank;  // shard -> rank
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;  // ranks 1.. (rank 0 runs on the caller's stream)
    // per rank: queries, coarse distances / lists; per shard: its [n][k] tables
    std::vector<DeviceBuffer> x, cd, ci, od, oi;
    ~MultiDev() {
        for (size_t r = 0; r < comms.size(); r++) {
            SDevGuard g(devs[r]);
            if (comms[r]) ncclCommDestroy(comms[r]);
            if (r < streams.size() && streams[r]) hipStreamDestroy(streams[r]);
        }
    }
};

IndexShardsIVF::IndexShardsIVF(Index* q, size_t nl, bool th, bool succ)
        : Index(q->d, q->metric_type), quantizer(q), nlist(nl), threaded(th),
          successive_ids(succ) {
    device = q->device;
    is_trained = q->is_trained && (size_t)q->ntotal == nlist;
}

void IndexShardsIVF::add_shard(IndexIVF* idx) {
    FAISS_THROW_IF_NOT(idx && idx->d == d && idx->nlist == nlist);
    // shards on other devices are searched over RCCL (shards.cpp)
    shards.push_back(idx);
    md_.reset();
    ntotal += idx->ntotal;
}

IndexShardsIVF::~IndexShardsIVF() {
    md_.reset();
    if (own_shards) {
        // shard 0 owns the common quantizer (own_fields), delete it last
        for (size_t i = shards.size(); i-- > 0;) delete shards[i];
    }
}

bool IndexShardsIVF::multi_device() const {
    for (auto* s : shards)
        if (s->device != quantizer->device) return true;
    const char* e = getenv("FAISS_AMD_SHARDS_RCCL");
    return e && atoi(e) != 0;
}

void IndexShardsIVF::search_multi(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                                  idx_t* labels, const SearchParametersIVF* params, size_t np,
                                  hipStream_t s) const {
    const int home = quantizer->device;
    const int ns = (int)shards.size();
    if (!md_) {
        auto md = std::make_unique<MultiDev>();
        md->devs.push_back(home);
        for (auto* sh : shards)
            if (std::find(md->devs.begin(), md->devs.end(), sh->device) == md->devs.end())
                md->devs.push_back(sh->device);
        for (auto* sh : shards)
            md->shard_rank.push_back(
                    (int)(std::find(md->devs.begin(), md->devs.end(), sh->device) -
                          md->devs.begin()));
        const int R = (int)md->devs.size();
        md->comms.assign(R, nullptr);
        NCCL_CHECK(ncclCommInitAll(md->comms.data(), R, md->devs.data()));
        md->streams.assign(R, nullptr);
        for (int r = 1; r < R; r++) {
            SDevGuard g(md->devs[r]);
            HIP_CHECK(hipStreamCreateWithFlags(&md->streams[r], hipStreamNonBlocking));
        }
        md->x.resize(R);
        md->cd.resize(R);
        md->ci.resize(R);
        md->od.resize(ns);
        md->oi.resize(ns);
        md_ = std::move(md);
    }
    MultiDev& md = *md_;
    const int R = (int)md.devs.size();
    auto rstream = [&](int r) { return r == 0 ? s : md.streams[r]; };
    const size_t nd = (size_t)n * d, nq = (size_t)n * np, nk = (size_t)n * k;
    // ---- rank 0: contiguous queries and the coarse pass
    {
        SDevGuard g(home);
        md.x[0].reserve(sizeof(float) * std::max<size_t>(nd, 1));
        HIP_CHECK(hipMemcpy2DAsync(md.x[0].ptr, sizeof(float) * d, x, sizeof(float) * ldx,
                                   sizeof(float) * d, n, hipMemcpyDeviceToDevice, s));
        s_cd_.reserve(sizeof(float) * std::max<size_t>(nq, 1));
        s_ci_.reserve(sizeof(int32_t) * std::max<size_t>(nq, 1));
        s_all_d_.reserve(sizeof(float) * ns * std::max<size_t>(nk, 1));
        s_all_i_.reserve(sizeof(idx_t) * ns * std::max<size_t>(nk, 1));
        quantizer->assign_device(n, md.x[0].as<float>(), d, (int)np, s_cd_.as<float>(),
                                 s_ci_.as<int32_t>(), params ? params->quantizer_params : nullptr,
                                 s);
    }
    for (int r = 1; r < R; r++) {
        SDevGuard g(md.devs[r]);
        md.x[r].reserve(sizeof(float) * std::max<size_t>(nd, 1));
        md.cd[r].reserve(sizeof(float) * std::max<size_t>(nq, 1));
        md.ci[r].reserve(sizeof(int32_t) * std::max<size_t>(nq, 1));
    }
    auto xb = [&](int r) { return md.x[r].as<float>(); };
    auto cdb = [&](int r) { return r == 0 ? s_cd_.as<float>() : md.cd[r].as<float>(); };
    auto cib = [&](int r) { return r == 0 ? s_ci_.as<int32_t>() : md.ci[r].as<int32_t>(); };
    // ---- broadcast queries and coarse results from rank 0
    if (R > 1) {
        NCCL_CHECK(ncclGroupStart());
        for (int r = 0; r < R; r++) {
            NCCL_CHECK(ncclBroadcast(xb(0), xb(r), nd, ncclFloat32, 0, md.comms[r], rstream(r)));
            NCCL_CHECK(ncclBroadcast(cdb(0), cdb(r), nq, ncclFloat32, 0, md.comms[r], rstream(r)));
            NCCL_CHECK(ncclBroadcast(cib(0), cib(r), nq, ncclInt32, 0, md.comms[r], rstream(r)));
        }
        NCCL_CHECK(ncclGroupEnd());
    }
    // ---- every shard on its own device and stream
    for (int i = 0; i < ns; i++) {
        const int r = md.shard_rank[i];
        IndexIVF* sh = shards[i];
        SDevGuard g(md.devs[r]);
        FAISS_THROW_IF_NOT_MSG(sh->nprobe == np || params, "inconsistent nprobe");
        float* od;
        idx_t* oi;
        if (r == 0) {
            od = s_all_d_.as<float>() + (size_t)i * nk;
            oi = s_all_i_.as<idx_t>() + (size_t)i * nk;
        } else {
            md.od[i].reserve(sizeof(float) * std::max<size_t>(nk, 1));
            md.oi[i].reserve(sizeof(idx_t) * std::max<size_t>(nk, 1));
            od = md.od[i].as<float>();
            oi = md.oi[i].as<idx_t>();
        }
        const uint32_t* lim = nullptr;
        const int32_t* asg = sh->apply_max_codes(n, (int)np, cib(r),
                                                 params ? params->max_codes : sh->max_codes, &lim,
                                                 rstream(r));
        const uint8_t* selm = sh->apply_selector(params, rstream(r));
        sh->search_preassigned_device(n, xb(r), d, k, (int)np, asg, cdb(r), od, oi, rstream(r),
                                      lim, selm);
    }
    // ---- gather the other ranks' tables on rank 0 (point to point)
    if (R > 1) {
        NCCL_CHECK(ncclGroupStart());
        for (int i = 0; i < ns; i++) {
            const int r = md.shard_rank[i];
            if (r == 0) continue;
            NCCL_CHECK(ncclSend(md.od[i].ptr, nk, ncclFloat32, 0, md.comms[r], rstream(r)));
            NCCL_CHECK(ncclSend(md.oi[i].ptr, nk, ncclInt64, 0, md.comms[r], rstream(r)));
            NCCL_CHECK(ncclRecv(s_all_d_.as<float>() + (size_t)i * nk, nk, ncclFloat32, r,
                                md.comms[0], s));
            NCCL_CHECK(ncclRecv(s_all_i_.as<idx_t>() + (size_t)i * nk, nk, ncclInt64, r,
                                md.comms[0], s));
        }
        NCCL_CHECK(ncclGroupEnd());
    }
    // ---- rank 0: label shift (successive_ids) and merge
    SDevGuard g(home);
    idx_t translation = 0;
    for (int i = 0; i < ns; i++) {
        if (successive_ids)
            kern::translate_labels(s_all_i_.as<idx_t>() + (size_t)i * nk, (int64_t)nk, translation,
                                   s);
        translation += shards[i]->ntotal;
    }
    kern::merge_rows(s_all_d_.as<float>(), s_all_i_.as<idx_t>(), n, (ns << 16) | (int)k, (int)k,
                     metric_type == METRIC_L2, distances, labels, s);
    for (int r = 1; r < R; r++) {
        SDevGuard gr(md.devs[r]);
        HIP_CHECK(hipStreamSynchronize(md.streams[r]));
    }
    HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace faiss_amd
