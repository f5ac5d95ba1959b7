// The reference harness's search sequence against the C++ mirror
// (include/faiss_amd.h), as benchmark_hnsw_ivf.cpp:361-390 writes it:
// read_index(fname, IO_FLAG_MMAP), dynamic_cast to IndexIVF, nprobe,
// quantizer hnsw.efSearch, parallel_mode, search_stats.  Same arguments and
// output as harness.c.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "faiss_amd.h"

int main(int argc, char** argv) {
    if (argc != 8) {
        std::fprintf(stderr, "usage: %s index nq k nprobe efSearch seed out\n", argv[0]);
        return 2;
    }
    using namespace faiss_amd;
    const idx_t nq = std::atoll(argv[2]), k = std::atoll(argv[3]);
    try {
        Index* index = read_index(argv[1], IO_FLAG_MMAP);
        auto* ivf = dynamic_cast<IndexIVF*>(index);
        if (!ivf) return 3;
        ivf->nprobe = (size_t)std::atoll(argv[4]);
        if (auto* qh = dynamic_cast<IndexHNSW*>(ivf->quantizer)) qh->hnsw.efSearch = std::atoi(argv[5]);
        ivf->parallel_mode = 0;
        std::vector<float> xq((size_t)nq * index->d), D((size_t)nq * k);
        std::vector<idx_t> I((size_t)nq * k);
        std::vector<QueryLatencyStats> lat((size_t)nq);
        float_rand(xq.data(), xq.size(), std::atoll(argv[6]));
        ivf->search_stats(nq, xq.data(), k, D.data(), I.data(), nullptr, lat.data());
        double mean = 0;
        for (auto& l : lat) mean += l.total_us / 1000.0;
        std::printf("{\"nq\": %lld, \"mean_ms\": %.6f}\n", (long long)nq, mean / nq);
        FILE* f = std::fopen(argv[7], "wb");
        if (!f) return 1;
        std::fwrite(D.data(), sizeof(float), D.size(), f);
        std::fwrite(I.data(), sizeof(idx_t), I.size(), f);
        std::fclose(f);
        delete index;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
