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
// The exchange between ranks (one rank per device, rank 0 = the quantizer's
// device).  Two transports with the same grouped operations:
//   Rccl: one communicator over the ranks' devices (ncclCommInitAll), the
//         collectives of each group issued between ncclGroupStart / End;
//   Copy: hipMemcpyPeerAsync between the ranks' buffers, ordered by events.
//         Used when ranks share a device (RCCL refuses a communicator with a
//         device twice: the one-GPU rehearsal of the multi-rank composition)
//         or when FAISS_AMD_SHARDS_TRANSPORT=p2p.
// Operations of one group never read what another operation of the group
// writes.
namespace {
struct Exchange {
    std::vector<int> devs;
    std::vector<hipStream_t> streams;  // per rank (rank 0: the caller's stream, per call)
    virtual ~Exchange() = default;
    virtual void group_start() = 0;
    virtual void group_end() = 0;
    virtual void group_abort() noexcept = 0;  // close an open group on an error path
    // bytes from rank root's buf[root] to every other rank's buf[r]
    virtual void bcast(int root, void* const* buf, size_t bytes) = 0;
    // in place: rank r's block r of buf[r] (bytes each) to block r of every rank
    virtual void allgather(void* const* buf, size_t bytes) = 0;
    // bytes from rank src's sbuf to rank dst's rbuf
    virtual void send_recv(int src, const void* sbuf, int dst, void* rbuf, size_t bytes) = 0;
};

struct GroupScope {  // ends the group on every path (an error inside leaves it closed)
    Exchange& x;
    bool open = true;
    explicit GroupScope(Exchange& e) : x(e) { x.group_start(); }
    void end() {
        open = false;
        x.group_end();
    }
    ~GroupScope() {
        if (open) x.group_abort();
    }
};

struct RcclExchange : Exchange {
    std::vector<ncclComm_t> comms;
    explicit RcclExchange(const std::vector<int>& d) {
        devs = d;
        comms.assign(devs.size(), nullptr);
        NCCL_CHECK(ncclCommInitAll(comms.data(), (int)devs.size(), devs.data()));
    }
    ~RcclExchange() override {
        for (size_t r = 0; r < comms.size(); r++) {
            SDevGuard g(devs[r]);
            if (comms[r]) ncclCommDestroy(comms[r]);
        }
    }
    void group_start() override { NCCL_CHECK(ncclGroupStart()); }
    void group_end() override { NCCL_CHECK(ncclGroupEnd()); }
    void group_abort() noexcept override { (void)ncclGroupEnd(); }
    void bcast(int root, void* const* buf, size_t bytes) override {
        for (size_t r = 0; r < devs.size(); r++)
            NCCL_CHECK(ncclBroadcast(buf[root], buf[r], bytes, ncclUint8, root, comms[r],
                                     streams[r]));
    }
    void allgather(void* const* buf, size_t bytes) override {
        for (size_t r = 0; r < devs.size(); r++)
            NCCL_CHECK(ncclAllGather((const uint8_t*)buf[r] + r * bytes, buf[r], bytes,
                                     ncclUint8, comms[r], streams[r]));
    }
    void send_recv(int src, const void* sbuf, int dst, void* rbuf, size_t bytes) override {
        if (!bytes) return;
        if (src == dst) {
            SDevGuard g(devs[src]);
            HIP_CHECK(hipMemcpyAsync(rbuf, sbuf, bytes, hipMemcpyDeviceToDevice, streams[src]));
            return;
        }
        NCCL_CHECK(ncclSend(sbuf, bytes, ncclUint8, dst, comms[src], streams[src]));
        NCCL_CHECK(ncclRecv(rbuf, bytes, ncclUint8, src, comms[dst], streams[dst]));
    }
};

struct CopyExchange : Exchange {
    // ready[r]: rank r's stream reached the group; done[r]: rank r's copies
    std::vector<hipEvent_t> ready, done;
    explicit CopyExchange(const std::vector<int>& d) {
        devs = d;
        ready.assign(devs.size(), nullptr);
        done.assign(devs.size(), nullptr);
        for (size_t r = 0; r < devs.size(); r++) {
            SDevGuard g(devs[r]);
            HIP_CHECK(hipEventCreateWithFlags(&ready[r], hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&done[r], hipEventDisableTiming));
        }
    }
    ~CopyExchange() override {
        for (size_t r = 0; r < devs.size(); r++) {
            SDevGuard g(devs[r]);
            (void)hipEventDestroy(ready[r]);
            (void)hipEventDestroy(done[r]);
        }
    }
    void group_start() override {
        for (size_t r = 0; r < devs.size(); r++) {
            SDevGuard g(devs[r]);
            HIP_CHECK(hipEventRecord(ready[r], streams[r]));
        }
    }
    // every rank's stream waits for every rank's copies (the sources may be
    // rewritten after the group)
    void group_end() override {
        for (size_t r = 0; r < devs.size(); r++) {
            SDevGuard g(devs[r]);
            HIP_CHECK(hipEventRecord(done[r], streams[r]));
        }
        for (size_t r = 0; r < devs.size(); r++) {
            SDevGuard g(devs[r]);
            for (size_t o = 0; o < devs.size(); o++)
                if (o != r) HIP_CHECK(hipStreamWaitEvent(streams[r], done[o], 0));
        }
    }
    void group_abort() noexcept override {}
    // the copy runs on the receiver's stream once the sender reached the group
    void copy(int src, const void* sbuf, int dst, void* rbuf, size_t bytes) {
        if (!bytes) return;
        SDevGuard g(devs[dst]);
        if (src != dst) HIP_CHECK(hipStreamWaitEvent(streams[dst], ready[src], 0));
        HIP_CHECK(hipMemcpyPeerAsync(rbuf, devs[dst], sbuf, devs[src], bytes, streams[dst]));
    }
    void bcast(int root, void* const* buf, size_t bytes) override {
        for (size_t r = 0; r < devs.size(); r++)
            if ((int)r != root) copy(root, buf[root], (int)r, buf[r], bytes);
    }
    void allgather(void* const* buf, size_t bytes) override {
        for (size_t r = 0; r < devs.size(); r++)
            for (size_t o = 0; o < devs.size(); o++)
                if (o != r)
                    copy((int)o, (const uint8_t*)buf[o] + o * bytes, (int)r,
                         (uint8_t*)buf[r] + o * bytes, bytes);
    }
    void send_recv(int src, const void* sbuf, int dst, void* rbuf, size_t bytes) override {
        copy(src, sbuf, dst, rbuf, bytes);
    }
};

// a copy of a quantizer on `device` (its own scratch and stream order), via
// the index I/O
Index* clone_to_device(const Index* src, int device) {
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
    idx->device = device;
    if (auto* h = dynamic_cast<IndexHNSW*>(idx)) {
        if (h->storage) h->storage->device = device;
        h->hnsw.efSearch = dynamic_cast<const IndexHNSW*>(src)->hnsw.efSearch;
    }
    return idx;
}
}  // namespace

struct IndexShardsIVF::MultiDev {
    std::vector<int> devs;        // rank -> device; rank 0 = the quantizer's device
    std::vector<int> shard_rank;  // shard -> rank
    std::unique_ptr<Exchange> xc;
    std::vector<hipStream_t> own;  // ranks 1.. (rank 0 runs on the caller's stream)
    // ranks 1..: a copy of the common quantizer for the rank's query slice
    std::vector<std::unique_ptr<Index>> qrep;
    uint64_t q_version = 0;  // the quantizer's content_version() when copied
    // per rank: padded queries, coarse distances / lists of the whole batch,
    // the rank's slice of every shard's tables and the merged slice
    std::vector<DeviceBuffer> x, cd, ci, sd, si, md, mi;
    // per shard: its [n][k] tables
    std::vector<DeviceBuffer> od, oi;
    ~MultiDev() {
        xc.reset();
        for (size_t r = 1; r < own.size(); r++) {
            SDevGuard g(devs[r]);
            if (own[r]) hipStreamDestroy(own[r]);
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

// faiss/IndexShardsIVF.cpp:158-245 over R ranks (devices).  Per call:
//   1. rank 0 pads the batch to R * S rows (S = ceil(n / R)); broadcast;
//   2. rank r quantizes its slice [r S, r S + S) with its copy of the common
//      quantizer (the form the batch size n decides, assign_device_slice);
//      all-gather of the coarse lists and distances (SURVEY 8e collective 1);
//   3. every shard runs search_preassigned on the whole batch, on its rank;
//   4. rank r receives slice r of every shard's [n][k] tables and merges it
//      (merge_knn_results order: ties to the lower shard);
//   5. the merged slices go to rank 0, into the caller's output.
// Ranks are the distinct devices of the quantizer and the shards, or one per
// shard under FAISS_AMD_SHARDS_RANKS=shard (the one-GPU rehearsal).
void IndexShardsIVF::search_multi(idx_t n, const float* x, int ldx, idx_t k, float* distances,
                                  idx_t* labels, const SearchParametersIVF* params, size_t np,
                                  hipStream_t s) const {
    const int home = quantizer->device;
    const int ns = (int)shards.size();
    // quantizer content changed since the copies were made: rebuild them
    if (md_ && md_->q_version != quantizer->content_version()) md_.reset();
    if (!md_) {
        auto md = std::make_unique<MultiDev>();
        const char* per = getenv("FAISS_AMD_SHARDS_RANKS");
        if (per && !strcmp(per, "shard")) {
            FAISS_THROW_IF_NOT_MSG(shards[0]->device == home,
                                   "FAISS_AMD_SHARDS_RANKS=shard: shard 0 must be on the "
                                   "quantizer's device");
            for (int i = 0; i < ns; i++) {
                md->devs.push_back(shards[i]->device);
                md->shard_rank.push_back(i);
            }
        } else {
            md->devs.push_back(home);
            for (auto* sh : shards)
                if (std::find(md->devs.begin(), md->devs.end(), sh->device) == md->devs.end())
                    md->devs.push_back(sh->device);
            for (auto* sh : shards)
                md->shard_rank.push_back(
                        (int)(std::find(md->devs.begin(), md->devs.end(), sh->device) -
                              md->devs.begin()));
        }
        const int R = (int)md->devs.size();
        std::vector<int> sorted = md->devs;
        std::sort(sorted.begin(), sorted.end());
        const bool distinct = std::unique(sorted.begin(), sorted.end()) == sorted.end();
        const char* tr = getenv("FAISS_AMD_SHARDS_TRANSPORT");
        if (distinct && !(tr && !strcmp(tr, "p2p")))
            md->xc = std::make_unique<RcclExchange>(md->devs);
        else
            md->xc = std::make_unique<CopyExchange>(md->devs);
        md->own.assign(R, nullptr);
        md->qrep.resize(R);
        for (int r = 1; r < R; r++) {
            SDevGuard g(md->devs[r]);
            HIP_CHECK(hipStreamCreateWithFlags(&md->own[r], hipStreamNonBlocking));
            md->qrep[r].reset(clone_to_device(quantizer, md->devs[r]));
        }
        md->q_version = quantizer->content_version();
        for (auto* v : {&md->x, &md->cd, &md->ci, &md->sd, &md->si, &md->md, &md->mi})
            v->resize(R);
        md->od.resize(ns);
        md->oi.resize(ns);
        md_ = std::move(md);
    }
    MultiDev& md = *md_;
    // search-time fields of the quantizer follow the live one on every call
    // (the C API sets efSearch between searches)
    if (auto* hq = dynamic_cast<const IndexHNSW*>(quantizer))
        for (auto& c : md.qrep)
            if (auto* hc = dynamic_cast<IndexHNSW*>(c.get())) {
                hc->hnsw.efSearch = hq->hnsw.efSearch;
                hc->hnsw.check_relative_distance = hq->hnsw.check_relative_distance;
                hc->hnsw.search_bounded_queue = hq->hnsw.search_bounded_queue;
            }
    Exchange& xc = *md.xc;
    const int R = (int)md.devs.size();
    xc.streams = md.own;
    xc.streams[0] = s;
    auto rstream = [&](int r) { return xc.streams[r]; };
    const int ld = (int)roundup((size_t)d, 4);
    const idx_t S = (n + R - 1) / R;  // queries per rank slice
    const size_t npad = (size_t)S * R, nk = (size_t)n * k;
    auto slice_n = [&](int r) { return std::max<idx_t>(0, std::min<idx_t>(S, n - (idx_t)r * S)); };
    for (int r = 0; r < R; r++) {
        SDevGuard g(md.devs[r]);
        md.x[r].reserve(sizeof(float) * std::max<size_t>(npad * ld, 1));
        md.cd[r].reserve(sizeof(float) * std::max<size_t>(npad * np, 1));
        md.ci[r].reserve(sizeof(int32_t) * std::max<size_t>(npad * np, 1));
        const size_t sk = (size_t)ns * std::max<idx_t>(S, 1) * k;
        md.sd[r].reserve(sizeof(float) * sk);
        md.si[r].reserve(sizeof(idx_t) * sk);
        md.md[r].reserve(sizeof(float) * std::max<idx_t>(S, 1) * k);
        md.mi[r].reserve(sizeof(idx_t) * std::max<idx_t>(S, 1) * k);
    }
    // ---- 1. rank 0: the batch, zero padded to npad rows of ld floats
    {
        SDevGuard g(home);
        HIP_CHECK(hipMemsetAsync(md.x[0].ptr, 0, sizeof(float) * npad * ld, s));
        HIP_CHECK(hipMemcpy2DAsync(md.x[0].ptr, sizeof(float) * ld, x, sizeof(float) * ldx,
                                   sizeof(float) * d, n, hipMemcpyDeviceToDevice, s));
    }
    std::vector<void*> xb(R), cdb(R), cib(R);
    for (int r = 0; r < R; r++) {
        xb[r] = md.x[r].ptr;
        cdb[r] = md.cd[r].ptr;
        cib[r] = md.ci[r].ptr;
    }
    if (R > 1) {
        GroupScope gs(xc);
        xc.bcast(0, xb.data(), sizeof(float) * npad * ld);
        gs.end();
    }
    // ---- 2. coarse pass of every rank's slice, all-gathered
    for (int r = 0; r < R; r++) {
        SDevGuard g(md.devs[r]);
        const Index* q = r == 0 ? quantizer : md.qrep[r].get();
        q->assign_device_slice(S, md.x[r].as<float>() + (size_t)r * S * ld, ld, (int)np,
                               md.cd[r].as<float>() + (size_t)r * S * np,
                               md.ci[r].as<int32_t>() + (size_t)r * S * np,
                               params ? params->quantizer_params : nullptr, rstream(r), n);
    }
    if (R > 1) {
        GroupScope gs(xc);
        xc.allgather(cdb.data(), sizeof(float) * S * np);
        xc.allgather(cib.data(), sizeof(int32_t) * S * np);
        gs.end();
    }
    // ---- 3. every shard on its rank, the whole batch
    idx_t translation = 0;
    for (int i = 0; i < ns; i++) {
        const int r = md.shard_rank[i];
        IndexIVF* sh = shards[i];
        SDevGuard g(md.devs[r]);
        FAISS_THROW_IF_NOT_MSG(sh->nprobe == np || params, "inconsistent nprobe");
        md.od[i].reserve(sizeof(float) * std::max<size_t>(nk, 1));
        md.oi[i].reserve(sizeof(idx_t) * std::max<size_t>(nk, 1));
        const uint32_t* lim = nullptr;
        const int32_t* asg = sh->apply_max_codes(n, (int)np, md.ci[r].as<int32_t>(),
                                                 params ? params->max_codes : sh->max_codes, &lim,
                                                 rstream(r));
        const uint8_t* selm = sh->apply_selector(params, rstream(r));
        sh->search_preassigned_device(n, md.x[r].as<float>(), ld, k, (int)np, asg,
                                      md.cd[r].as<float>(), md.od[i].as<float>(),
                                      md.oi[i].as<idx_t>(), rstream(r), lim, selm);
        if (successive_ids)
            kern::translate_labels(md.oi[i].as<idx_t>(), (int64_t)nk, translation, rstream(r));
        translation += sh->ntotal;
    }
    // ---- 4. slice r of every shard's tables to rank r ([ns][slice][k]), merged there
    {
        GroupScope gs(xc);
        for (int i = 0; i < ns; i++)
            for (int r = 0; r < R; r++) {
                const idx_t c = slice_n(r);
                if (c <= 0) continue;
                const size_t o = (size_t)r * S * k, m = (size_t)i * c * k;
                xc.send_recv(md.shard_rank[i], md.od[i].as<float>() + o, r,
                             md.sd[r].as<float>() + m, sizeof(float) * c * k);
                xc.send_recv(md.shard_rank[i], md.oi[i].as<idx_t>() + o, r,
                             md.si[r].as<idx_t>() + m, sizeof(idx_t) * c * k);
            }
        gs.end();
    }
    for (int r = 0; r < R; r++) {
        const idx_t c = slice_n(r);
        if (c <= 0) continue;
        SDevGuard g(md.devs[r]);
        float* od = r == 0 ? distances : md.md[r].as<float>();
        idx_t* oi = r == 0 ? labels : md.mi[r].as<idx_t>();
        kern::merge_rows(md.sd[r].as<float>(), md.si[r].as<idx_t>(), c, (ns << 16) | (int)k,
                         (int)k, metric_type == METRIC_L2, od, oi, rstream(r));
    }
    // ---- 5. merged slices into the caller's output on rank 0
    if (R > 1) {
        GroupScope gs(xc);
        for (int r = 1; r < R; r++) {
            const idx_t c = slice_n(r);
            if (c <= 0) continue;
            xc.send_recv(r, md.md[r].ptr, 0, distances + (size_t)r * S * k,
                         sizeof(float) * c * k);
            xc.send_recv(r, md.mi[r].ptr, 0, labels + (size_t)r * S * k, sizeof(idx_t) * c * k);
        }
        gs.end();
    }
    for (int r = 1; r < R; r++) {
        SDevGuard gr(md.devs[r]);
        HIP_CHECK(hipStreamSynchronize(md.own[r]));
    }
    SDevGuard g(home);
    HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace faiss_amd
