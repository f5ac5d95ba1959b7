// io.cpp — the reference on-disk format for the five index types on the path
// and a subset index_factory.
//
// Format (reference faiss/impl/index_write.cpp, faiss/impl/index_read.cpp):
//   header  = d:i32 ntotal:i64 dummy:i64 dummy:i64 is_trained:u8 metric:i32
//             [metric_arg:f32 if metric > 1]                 (write :79-90)
//   IxF2/IxFI = header, size_t n4, n4*4 bytes of floats       (:396-403)
//   IVF hdr = header, nlist:size_t, nprobe:size_t, nested quantizer,
//             direct map (char type, vector<idx_t>)           (:367-389)
//   IwFl    = IVF hdr, invlists                               (:631-638)
//   IwPQ    = IVF hdr, by_residual:u8, code_size:size_t, PQ (d,M,nbits:size_t,
//             vector<float> centroids), invlists               (:697-705,155-160)
//   ilar    = nlist:size_t, code_size:size_t, "full"+vector<size_t> sizes |
//             "sprs"+vector<size_t>(list,size pairs), then per non-empty list
//             codes then ids                                  (:243-297)
//   IHNf    = header, HNSW (vector<double> assign_probas, vector<int> cum,
//             vector<int> levels, vector<size_t> offsets, vector<i32>
//             neighbors, entry_point:i32, max_level, efConstruction,
//             efSearch:int, dummy int), storage index         (:300-316,760-778)
//   vectors carry a size_t element-count prefix (faiss/impl/io_macros.h:62-67)
//   fourcc = little-endian chars (faiss/impl/io.cpp:237-241)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/faiss_amd.h"

namespace faiss_amd {

MappedFile::MappedFile(int fd, const std::string& nm) : name(nm) {
    struct stat st;
    FAISS_THROW_IF_NOT_MSG(fstat(fd, &st) == 0, std::string("fstat failed: ") + strerror(errno));
    size = (size_t)st.st_size;
    if (size == 0) return;
    void* p = mmap(nullptr, size, PROT_READ, MAP_SHARED, fd, 0);
    FAISS_THROW_IF_NOT_MSG(p != MAP_FAILED, std::string("could not mmap: ") + strerror(errno));
    ptr = (const uint8_t*)p;
}
MappedFile::~MappedFile() {
    if (ptr) munmap((void*)ptr, size);
}

namespace {
uint32_t fourcc(const char* s) {
    return (uint32_t)(uint8_t)s[0] | ((uint32_t)(uint8_t)s[1] << 8) |
           ((uint32_t)(uint8_t)s[2] << 16) | ((uint32_t)(uint8_t)s[3] << 24);
}
std::string fourcc_str(uint32_t h) {
    std::string s(4, ' ');
    for (int i = 0; i < 4; i++) {
        char c = (char)((h >> (8 * i)) & 0xff);
        s[i] = (c >= 32 && c < 127) ? c : '?';
    }
    return s;
}

// A file written next to its target and renamed over it on commit(): saving
// an index back to the file it was mapped from (IO_FLAG_MMAP, or an ilod data
// file) must not truncate the mapping it is reading the lists through (the
// old inode stays alive while mapped).  Removed again when not committed.
// An existing regular file is replaced this way (through a symlink, the file
// it names, keeping its mode), and so is a new name (mode 0666 & ~umask, as
// fopen would create it), so a failed write never leaves a truncated file
// under the final name.  A FIFO, a device such as /dev/stdout, or a directory
// where no temporary can be created is written in place, as fopen(path, "wb")
// would.
struct AtomicFile {
    std::string target, tmp;
    FILE* f = nullptr;
    bool used = false;  // write_index_ondisk: the list data went through this file
    mode_t mode = 0;
    explicit AtomicFile(const std::string& path) : target(path) {
        struct stat st;
        const bool exists = stat(path.c_str(), &st) == 0;
        const bool fresh = !exists && errno == ENOENT;
        if ((exists && S_ISREG(st.st_mode)) || fresh) {
            if (exists) {
                if (char* rp = realpath(path.c_str(), nullptr)) {
                    target = rp;
                    free(rp);
                }
                mode = st.st_mode & 07777;
            } else {
                const mode_t um = umask(0);
                umask(um);
                mode = 0666 & ~um;
            }
            tmp = target + ".tmpXXXXXX";
            const int fd = mkstemp(&tmp[0]);
            if (fd >= 0) {
                f = fdopen(fd, "wb");
                if (!f) {
                    close(fd);
                    unlink(tmp.c_str());
                    FAISS_THROW_MSG("could not open " + path + " for writing");
                }
                return;
            }
            tmp.clear();  // no temporary beside it: write in place
        }
        f = fopen(path.c_str(), "wb");
        FAISS_THROW_IF_NOT_MSG(f, "could not open " + path + " for writing: " + strerror(errno));
    }
    AtomicFile(const AtomicFile&) = delete;
    AtomicFile& operator=(const AtomicFile&) = delete;
    // flush and close; the data is complete (under the temporary name)
    void finish() {
        if (!f) return;
        const bool ok = fflush(f) == 0 && !ferror(f);
        const bool closed = fclose(f) == 0;
        f = nullptr;
        FAISS_THROW_IF_NOT_MSG(ok && closed, "write error on " + target);
    }
    void commit() {
        finish();
        if (tmp.empty()) return;  // written in place
        chmod(tmp.c_str(), mode);  // mkstemp creates 0600: the replaced file's mode
        FAISS_THROW_IF_NOT_MSG(rename(tmp.c_str(), target.c_str()) == 0,
                               "could not rename onto " + target + ": " + strerror(errno));
        tmp.clear();
    }
    ~AtomicFile() {
        if (f) fclose(f);
        if (!tmp.empty()) unlink(tmp.c_str());
    }
};

struct Writer {
    FILE* f;
    const char* ondisk_fname = nullptr;  // write_index_ondisk: lists go to this file
    AtomicFile* ondisk_file = nullptr;   // ... written through this (renamed by the caller)
    void bytes(const void* p, size_t n) {
        if (n && fwrite(p, 1, n, f) != n) FAISS_THROW_MSG("write error");
    }
    template <class T>
    void one(const T& v) { bytes(&v, sizeof(T)); }
    template <class T>
    void vec(const std::vector<T>& v) {
        size_t n = v.size();
        one(n);
        bytes(v.data(), sizeof(T) * n);
    }
};
struct Reader {
    FILE* f;
    std::string name;  // file name when reading from a named file (IO_FLAG_ONDISK_SAME_DIR)
    void bytes(void* p, size_t n) {
        if (n && fread(p, 1, n, f) != n) FAISS_THROW_MSG("read error: truncated index file");
    }
    template <class T>
    T one() {
        T v;
        bytes(&v, sizeof(T));
        return v;
    }
    template <class T>
    void vec(std::vector<T>& v) {
        size_t n = one<size_t>();
        FAISS_THROW_IF_NOT_MSG(n < ((size_t)1 << 40), "corrupt vector size");
        v.resize(n);
        bytes(v.data(), sizeof(T) * n);
    }
};

void write_header(const Index* idx, Writer& w) {
    w.one<int32_t>(idx->d);
    w.one<int64_t>(idx->ntotal);
    int64_t dummy = 1 << 20;
    w.one(dummy);
    w.one(dummy);
    w.one<uint8_t>(idx->is_trained ? 1 : 0);
    w.one<int32_t>((int32_t)idx->metric_type);
    if ((int)idx->metric_type > 1) w.one<float>(idx->metric_arg);
}
struct Header {
    int32_t d;
    int64_t ntotal;
    bool is_trained;
    int32_t metric;
    float metric_arg = 0;
};
Header read_header(Reader& r) {
    Header h;
    h.d = r.one<int32_t>();
    h.ntotal = r.one<int64_t>();
    r.one<int64_t>();
    r.one<int64_t>();
    h.is_trained = r.one<uint8_t>() != 0;
    h.metric = r.one<int32_t>();
    if (h.metric > 1) h.metric_arg = r.one<float>();
    FAISS_THROW_IF_NOT_MSG(h.metric == METRIC_L2 || h.metric == METRIC_INNER_PRODUCT,
                           "only L2 / inner-product indexes are supported");
    return h;
}
void apply_header(Index* idx, const Header& h) {
    idx->d = h.d;
    idx->ntotal = h.ntotal;
    idx->is_trained = h.is_trained;
    idx->metric_type = (MetricType)h.metric;
    idx->metric_arg = h.metric_arg;
}

// `ilod` metadata (faiss/invlists/OnDiskInvertedLists.cpp:683-704): lists as
// (size, capacity, offset) triples, an empty free-slot table, the data file
// name and its size.
void write_ilod(const ArrayInvertedLists* il, Writer& w, const std::string& fname,
                const std::vector<size_t>& lists, size_t totsize) {
    w.one(fourcc("ilod"));
    w.one<size_t>(il->nlist);
    w.one<size_t>(il->code_size);
    w.one<size_t>(il->nlist);
    w.bytes(lists.data(), sizeof(size_t) * lists.size());
    w.one<size_t>(0);
    std::vector<char> fn(fname.begin(), fname.end());
    w.vec(fn);
    w.one<size_t>(totsize);
}

void write_invlists(const ArrayInvertedLists* il, Writer& w) {
    if (w.ondisk_fname) {
        // data file: per non-empty list codes[size*code_size] then ids[size]
        FAISS_THROW_IF_NOT(w.ondisk_file && w.ondisk_file->f);
        w.ondisk_file->used = true;
        Writer dw{w.ondisk_file->f};
        std::vector<size_t> lists(3 * il->nlist, 0);
        size_t o = 0;
        for (size_t l = 0; l < il->nlist; l++) {
            const size_t n = il->list_size(l);
            lists[3 * l] = lists[3 * l + 1] = n;
            lists[3 * l + 2] = o;
            if (!n) continue;
            dw.bytes(il->get_codes(l), n * il->code_size);
            dw.bytes(il->get_ids(l), n * sizeof(idx_t));
            o += n * (il->code_size + sizeof(idx_t));
        }
        w.ondisk_file->finish();
        write_ilod(il, w, w.ondisk_fname, lists, o);
        return;
    }
    if (il->map && il->map_ondisk) {
        // lists still live in an `ilod` data file: write its metadata back
        FAISS_THROW_IF_NOT(il->ondisk_lists.size() == 3 * il->nlist);
        w.one(fourcc("ilod"));
        w.one<size_t>(il->nlist);
        w.one<size_t>(il->code_size);
        w.one<size_t>(il->nlist);
        w.bytes(il->ondisk_lists.data(), sizeof(size_t) * il->ondisk_lists.size());
        w.one<size_t>(il->ondisk_slots.size() / 2);
        w.bytes(il->ondisk_slots.data(), sizeof(size_t) * il->ondisk_slots.size());
        std::vector<char> fn(il->map->name.begin(), il->map->name.end());
        w.vec(fn);
        w.one<size_t>(il->ondisk_totsize);
        return;
    }
    w.one(fourcc("ilar"));
    w.one<size_t>(il->nlist);
    w.one<size_t>(il->code_size);
    size_t n_non0 = 0;
    for (size_t i = 0; i < il->nlist; i++)
        if (il->list_size(i)) n_non0++;
    std::vector<size_t> sizes;
    if (n_non0 > il->nlist / 2) {
        w.one(fourcc("full"));
        for (size_t i = 0; i < il->nlist; i++) sizes.push_back(il->list_size(i));
    } else {
        w.one(fourcc("sprs"));
        for (size_t i = 0; i < il->nlist; i++) {
            if (il->list_size(i)) {
                sizes.push_back(i);
                sizes.push_back(il->list_size(i));
            }
        }
    }
    w.vec(sizes);
    for (size_t i = 0; i < il->nlist; i++) {
        size_t n = il->list_size(i);
        if (n) {
            w.bytes(il->get_codes(i), n * il->code_size);
            w.bytes(il->get_ids(i), n * sizeof(idx_t));
        }
    }
}

// The `ilar` list sizes block (faiss/impl/index_read.cpp:243-297).
std::vector<size_t> read_ilar_sizes(Reader& r, size_t nl) {
    std::vector<size_t> sizes(nl, 0);
    uint32_t lt = r.one<uint32_t>();
    if (lt == fourcc("full")) {
        r.vec(sizes);
        FAISS_THROW_IF_NOT(sizes.size() == nl);
    } else if (lt == fourcc("sprs")) {
        std::vector<size_t> idsz;
        r.vec(idsz);
        for (size_t j = 0; j + 1 < idsz.size(); j += 2) {
            FAISS_THROW_IF_NOT(idsz[j] < nl);
            sizes[idsz[j]] = idsz[j + 1];
        }
    } else {
        FAISS_THROW_MSG("list_type not recognized: " + fourcc_str(lt));
    }
    return sizes;
}

std::string dir_of(const std::string& path) {
    size_t slash = path.find_last_of('/');
    return slash == std::string::npos ? std::string("./") : path.substr(0, slash + 1);
}

void read_invlists(ArrayInvertedLists* il, Reader& r, size_t nlist, size_t code_size,
                   int io_flags) {
    uint32_t h = r.one<uint32_t>();
    if (h == fourcc("ilod")) {
        // OnDiskInvertedLists (faiss/invlists/OnDiskInvertedLists.cpp:706-757):
        // nlist, code_size, vector<List{size,capacity,offset}>, vector<Slot>,
        // vector<char> filename, totsize.  List l = codes[capacity*code_size]
        // then ids[capacity] at `offset` in the data file.
        size_t nl = r.one<size_t>(), cs = r.one<size_t>();
        FAISS_THROW_IF_NOT(nl == nlist && cs == code_size);
        std::vector<size_t> lists;  // 3 size_t per list (POD OnDiskOneList)
        {
            size_t n = r.one<size_t>();
            FAISS_THROW_IF_NOT_MSG(n == nl, "ilod: list table size != nlist");
            lists.resize(3 * n);
            r.bytes(lists.data(), sizeof(size_t) * 3 * n);
        }
        std::vector<size_t> slots;  // 2 size_t per slot (free space, unused here)
        {
            size_t n = r.one<size_t>();
            FAISS_THROW_IF_NOT(n < ((size_t)1 << 40));
            slots.resize(2 * n);
            r.bytes(slots.data(), sizeof(size_t) * 2 * n);
        }
        std::vector<char> fn;
        r.vec(fn);
        std::string filename(fn.begin(), fn.end());
        size_t totsize = r.one<size_t>();
        if (io_flags & IO_FLAG_ONDISK_SAME_DIR) {
            FAISS_THROW_IF_NOT_MSG(!r.name.empty(),
                                   "IO_FLAG_ONDISK_SAME_DIR only supported when reading from file");
            size_t slash = filename.find_last_of('/');
            filename = dir_of(r.name) + (slash == std::string::npos ? filename
                                                                    : filename.substr(slash + 1));
        }
        il->reset();
        // The reference skips do_mmap() under IO_FLAG_SKIP_IVF_DATA (:752) and
        // a later search would dereference a null mapping; here the data file
        // is mapped in every case.
        int fd = open(filename.c_str(), O_RDONLY);
        FAISS_THROW_IF_NOT_MSG(fd >= 0, "could not open on-disk inverted lists " + filename);
        std::shared_ptr<MappedFile> m;
        try {
            m = std::make_shared<MappedFile>(fd, filename);
        } catch (...) {
            close(fd);
            throw;
        }
        close(fd);
        FAISS_THROW_IF_NOT_MSG(m->size >= totsize || totsize == 0,
                               "on-disk inverted lists file shorter than totsize");
        il->map_codes.assign(nl, nullptr);
        il->map_ids.assign(nl, nullptr);
        il->map_sizes.assign(nl, 0);
        for (size_t l = 0; l < nl; l++) {
            const size_t size = lists[3 * l], cap = lists[3 * l + 1], o = lists[3 * l + 2];
            FAISS_THROW_IF_NOT_MSG(size <= cap, "ilod: list size > capacity");
            if (!size) continue;
            // overflow-safe: o + cap * (cs + 8) <= size without wrapping
            FAISS_THROW_IF_NOT_MSG(o <= m->size && cap <= (m->size - o) / (cs + sizeof(idx_t)),
                                   "ilod: list extends past the end of the data file");
            il->map_sizes[l] = size;
            il->map_codes[l] = m->ptr + o;
            il->map_ids[l] = (const idx_t*)(m->ptr + o + cap * cs);
        }
        il->map = m;
        il->map_ondisk = true;
        il->ondisk_lists = std::move(lists);
        il->ondisk_slots = std::move(slots);
        il->ondisk_totsize = totsize;
        return;
    }
    FAISS_THROW_IF_NOT_MSG(h == fourcc("ilar"),
                           "unsupported inverted-list type " + fourcc_str(h));
    size_t nl = r.one<size_t>(), cs = r.one<size_t>();
    FAISS_THROW_IF_NOT(nl == nlist && cs == code_size);
    std::vector<size_t> sizes = read_ilar_sizes(r, nl);
    if (io_flags & IO_FLAG_SKIP_IVF_DATA) {
        // faiss/impl/index_read.cpp:214-225: the hook is chosen by the flag's
        // high 16 bits; only the mmap hook ("ilod", IO_FLAG_MMAP) exists.
        const uint32_t h2 = ((uint32_t)io_flags & 0xffff0000u) | (fourcc("il__") & 0xffffu);
        FAISS_THROW_IF_NOT_MSG(h2 == fourcc("ilod"),
                               "read_InvertedLists: could not load ArrayInvertedLists as " +
                                   fourcc_str(h2));
        // OnDiskInvertedListsIOHook::read_ArrayInvertedLists
        // (faiss/invlists/OnDiskInvertedLists.cpp:759-800): map the whole
        // index file, lists point at their codes/ids, reading resumes after.
        FAISS_THROW_IF_NOT_MSG(r.f, "mmap only supported for File objects");
        long o0 = ftell(r.f);
        FAISS_THROW_IF_NOT_MSG(o0 >= 0, "ftell failed");
        auto m = std::make_shared<MappedFile>(fileno(r.f), r.name);
        size_t o = (size_t)o0;
        il->reset();
        il->map_codes.assign(nl, nullptr);
        il->map_ids.assign(nl, nullptr);
        il->map_sizes = sizes;
        for (size_t i = 0; i < nl; i++) {
            FAISS_THROW_IF_NOT_MSG(o <= m->size && sizes[i] <= (m->size - o) / (cs + sizeof(idx_t)),
                                   "read error: truncated index file");
            const size_t bytes = sizes[i] * (cs + sizeof(idx_t));
            il->map_codes[i] = m->ptr + o;
            il->map_ids[i] = (const idx_t*)(m->ptr + o + sizes[i] * cs);
            o += bytes;
        }
        il->map = m;
        FAISS_THROW_IF_NOT(fseek(r.f, (long)o, SEEK_SET) == 0);
        return;
    }
    for (size_t i = 0; i < nl; i++) {
        il->ids[i].resize(sizes[i]);
        il->codes[i].resize(sizes[i] * cs);
    }
    for (size_t i = 0; i < nl; i++) {
        if (sizes[i]) {
            r.bytes(il->codes[i].data(), sizes[i] * cs);
            r.bytes(il->ids[i].data(), sizes[i] * sizeof(idx_t));
        }
    }
}

void write_index_impl(const Index* idx, Writer& w);

void write_ivf_header(const IndexIVF* ivf, Writer& w) {
    write_header(ivf, w);
    w.one<size_t>(ivf->nlist);
    w.one<size_t>(ivf->nprobe);
    write_index_impl(ivf->quantizer, w);
    w.one<char>(0);  // DirectMap::NoMap
    std::vector<idx_t> empty;
    w.vec(empty);
}

void write_index_impl(const Index* idx, Writer& w) {
    if (idx == nullptr) {
        w.one(fourcc("null"));
    } else if (auto f = dynamic_cast<const IndexFlat*>(idx)) {
        w.one(fourcc(f->metric_type == METRIC_INNER_PRODUCT ? "IxFI" : "IxF2"));
        write_header(f, w);
        size_t n4 = f->xb.size();  // number of 4-byte words
        w.one(n4);
        w.bytes(f->xb.data(), n4 * 4);
    } else if (auto h = dynamic_cast<const IndexHNSW*>(idx)) {
        w.one(fourcc("IHNf"));
        write_header(h, w);
        w.vec(h->hnsw.assign_probas);
        w.vec(h->hnsw.cum_nneighbor_per_level);
        w.vec(h->hnsw.levels);
        w.vec(h->hnsw.offsets);
        w.vec(h->hnsw.neighbors);
        w.one<int32_t>(h->hnsw.entry_point);
        w.one<int32_t>(h->hnsw.max_level);
        w.one<int32_t>(h->hnsw.efConstruction);
        w.one<int32_t>(h->hnsw.efSearch);
        w.one<int32_t>(1);  // deprecated upper_beam
        write_index_impl(h->storage, w);
    } else if (auto fl = dynamic_cast<const IndexIVFFlat*>(idx)) {
        w.one(fourcc("IwFl"));
        write_ivf_header(fl, w);
        write_invlists(fl->invlists.get(), w);
    } else if (auto pq = dynamic_cast<const IndexIVFPQ*>(idx)) {
        w.one(fourcc("IwPQ"));
        write_ivf_header(pq, w);
        w.one<uint8_t>(pq->by_residual ? 1 : 0);
        w.one<size_t>(pq->code_size);
        w.one<size_t>(pq->pq.d);
        w.one<size_t>(pq->pq.M);
        w.one<size_t>(pq->pq.nbits);
        w.vec(pq->pq.centroids);
        write_invlists(pq->invlists.get(), w);
    } else {
        FAISS_THROW_MSG("don't know how to serialize this type of index");
    }
}

Index* read_index_impl(Reader& r, int io_flags) {
    uint32_t h = r.one<uint32_t>();
    if (h == fourcc("null")) return nullptr;
    if (h == fourcc("IxF2") || h == fourcc("IxFI")) {
        Header hd = read_header(r);
        auto f = new IndexFlat(hd.d, (MetricType)hd.metric);
        apply_header(f, hd);
        size_t n4 = r.one<size_t>();
        FAISS_THROW_IF_NOT(n4 == (size_t)hd.ntotal * hd.d);
        f->xb.resize(n4);
        r.bytes(f->xb.data(), n4 * 4);
        return f;
    }
    if (h == fourcc("IHNf")) {
        Header hd = read_header(r);
        auto ix = new IndexHNSW(nullptr, 32);
        apply_header(ix, hd);
        ix->hnsw.assign_probas.clear();
        ix->hnsw.cum_nneighbor_per_level.clear();
        ix->hnsw.offsets.clear();
        r.vec(ix->hnsw.assign_probas);
        r.vec(ix->hnsw.cum_nneighbor_per_level);
        r.vec(ix->hnsw.levels);
        r.vec(ix->hnsw.offsets);
        r.vec(ix->hnsw.neighbors);
        ix->hnsw.entry_point = r.one<int32_t>();
        ix->hnsw.max_level = r.one<int32_t>();
        ix->hnsw.efConstruction = r.one<int32_t>();
        ix->hnsw.efSearch = r.one<int32_t>();
        r.one<int32_t>();
        Index* st = read_index_impl(r, io_flags);
        auto stf = dynamic_cast<IndexFlat*>(st);
        FAISS_THROW_IF_NOT_MSG(stf, "IHNf storage must be a flat index");
        ix->storage = stf;
        ix->own_fields = true;
        ix->device = stf->device;
        return ix;
    }
    if (h == fourcc("IwFl") || h == fourcc("IwPQ")) {
        Header hd = read_header(r);
        size_t nlist = r.one<size_t>();
        size_t nprobe = r.one<size_t>();
        Index* q = read_index_impl(r, io_flags);
        FAISS_THROW_IF_NOT_MSG(q, "IVF index without quantizer");
        char dm = r.one<char>();
        std::vector<idx_t> dmarr;
        r.vec(dmarr);
        FAISS_THROW_IF_NOT_MSG(dm == 0, "direct maps are not supported");
        IndexIVF* ivf;
        if (h == fourcc("IwFl")) {
            ivf = new IndexIVFFlat(q, hd.d, nlist, (MetricType)hd.metric);
        } else {
            bool by_res = r.one<uint8_t>() != 0;
            size_t code_size = r.one<size_t>();
            size_t pd = r.one<size_t>(), M = r.one<size_t>(), nbits = r.one<size_t>();
            FAISS_THROW_IF_NOT(pd == (size_t)hd.d);
            auto pqi = new IndexIVFPQ(q, hd.d, nlist, M, nbits, (MetricType)hd.metric);
            pqi->by_residual = by_res;
            FAISS_THROW_IF_NOT(code_size == pqi->code_size);
            r.vec(pqi->pq.centroids);
            FAISS_THROW_IF_NOT(pqi->pq.centroids.size() == pd * ((size_t)1 << nbits));
            ivf = pqi;
        }
        ivf->own_fields = true;
        apply_header(ivf, hd);
        ivf->nprobe = nprobe;
        read_invlists(ivf->invlists.get(), r, nlist, ivf->code_size, io_flags);
        if (auto pqi = dynamic_cast<IndexIVFPQ*>(ivf)) {
            // faiss/impl/index_read.cpp:510-516
            if (pqi->is_trained && pqi->by_residual) pqi->precompute_table();
        }
        return ivf;
    }
    FAISS_THROW_MSG("Index type " + fourcc_str(h) + " not supported on this path");
}
}  // namespace

void write_index(const Index* idx, FILE* f) {
    Writer w{f};
    write_index_impl(idx, w);
}
void write_index_ondisk(const Index* idx, const char* fname, const char* lists_fname) {
    FAISS_THROW_IF_NOT_MSG(dynamic_cast<const IndexIVF*>(idx),
                           "write_index_ondisk: only IVF indexes have inverted lists");
    // both files are written under temporary names and renamed at the end,
    // so neither truncates a mapping the lists are read from
    AtomicFile df(lists_fname);
    AtomicFile f(fname);
    Writer w{f.f, lists_fname, &df};
    write_index_impl(idx, w);
    f.finish();
    FAISS_THROW_IF_NOT_MSG(df.used, "write_index_ondisk: no inverted lists were written");
    df.commit();
    f.commit();
}
void write_index(const Index* idx, const char* fname) {
    AtomicFile f(fname);
    write_index(idx, f.f);
    f.commit();
}
Index* read_index(FILE* f, int io_flags) {
    Reader r{f, ""};
    return read_index_impl(r, io_flags);
}
Index* read_index(const char* fname, int io_flags) {
    FILE* f = fopen(fname, "rb");
    FAISS_THROW_IF_NOT_MSG(f, std::string("could not open ") + fname + " for reading");
    Index* idx = nullptr;
    try {
        Reader r{f, fname};
        idx = read_index_impl(r, io_flags);
    } catch (...) {
        fclose(f);
        throw;
    }
    fclose(f);
    return idx;
}

// ---------------------------------------------------------------- factory
// faiss/index_factory.cpp:242-345 subset.
Index* index_factory(int d, const char* description, MetricType metric) {
    std::string s(description);
    auto parse_int = [&](size_t& pos) {
        size_t st = pos;
        while (pos < s.size() && isdigit((unsigned char)s[pos])) pos++;
        FAISS_THROW_IF_NOT_MSG(pos > st, "could not parse index_factory string " + s);
        return std::stol(s.substr(st, pos - st));
    };
    if (s == "Flat") return new IndexFlat(d, metric);
    if (s.rfind("HNSW", 0) == 0) {
        size_t pos = 4;
        int M = s.size() > 4 ? (int)parse_int(pos) : 32;
        std::string rest = s.substr(pos);
        FAISS_THROW_IF_NOT_MSG(rest.empty() || rest == ",Flat" || rest == "_Flat",
                               "unsupported HNSW description " + s);
        return new IndexHNSWFlat(d, M, metric);
    }
    FAISS_THROW_IF_NOT_MSG(s.rfind("IVF", 0) == 0, "unsupported index_factory string " + s);
    size_t pos = 3;
    size_t nlist = (size_t)parse_int(pos);
    Index* q = nullptr;
    if (s.compare(pos, 5, "_HNSW") == 0) {
        pos += 5;
        int M = (int)parse_int(pos);
        q = new IndexHNSWFlat(d, M, metric);
    } else if (s.compare(pos, 5, "_Flat") == 0) {
        pos += 5;
        q = new IndexFlat(d, metric);
    } else {
        q = new IndexFlat(d, metric);
    }
    FAISS_THROW_IF_NOT_MSG(pos < s.size() && s[pos] == ',', "unsupported string " + s);
    pos++;
    std::string enc = s.substr(pos);
    IndexIVF* ivf = nullptr;
    try {
        if (enc == "Flat") {
            ivf = new IndexIVFFlat(q, d, nlist, metric);
        } else if (enc.rfind("PQ", 0) == 0) {
            size_t p2 = 2;
            std::string& ss = s;
            (void)ss;
            size_t st = p2;
            while (p2 < enc.size() && isdigit((unsigned char)enc[p2])) p2++;
            size_t M = std::stoul(enc.substr(st, p2 - st));
            size_t nbits = 8;
            if (p2 < enc.size() && enc[p2] == 'x') {
                p2++;
                st = p2;
                while (p2 < enc.size() && isdigit((unsigned char)enc[p2])) p2++;
                nbits = std::stoul(enc.substr(st, p2 - st));
            }
            std::string tail = enc.substr(p2);
            FAISS_THROW_IF_NOT_MSG(tail.empty() || tail == "np", "unsupported PQ spec " + enc);
            ivf = new IndexIVFPQ(q, d, nlist, M, nbits, metric);
        } else {
            FAISS_THROW_MSG("unsupported IVF encoding " + enc);
        }
    } catch (...) {
        delete q;
        throw;
    }
    ivf->own_fields = true;
    return ivf;
}

}  // namespace faiss_amd
