// faiss/impl/faiss_amd_names.h — the library's C++ API under the reference's
// namespace.  The classes of ../../faiss_amd.h (namespace faiss_amd) are the
// faiss:: classes of the hot path (same names, members, signatures and
// exceptions; faiss/Index.h:108-181, faiss/IndexIVF.h:39-587, ...).  This
// header names them in namespace faiss with using-declarations, so code
// written against the reference (`faiss::IndexIVFFlat`, `faiss::read_index`,
// `dynamic_cast<faiss::IndexIVF*>`, `catch (faiss::FaissException&)`)
// compiles unchanged against libfaiss_amd.so; namespace faiss stays open for
// the caller's own declarations.  Every <faiss/...> header of this directory
// includes it, as the reference's headers reach each other transitively.
//
// Building a translation unit against these headers needs the HIP runtime
// headers (the device entry points take hipStream_t):
//   g++ -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I<repo>/include ...
//       -L<repo>/hnsw-ivf_amd/lib -lfaiss_amd -L/opt/rocm/lib -lamdhip64
#pragma once

#include "../../faiss_amd.h"

namespace faiss {

// faiss/MetricType.h:22-44
using faiss_amd::idx_t;
using faiss_amd::MetricType;
using faiss_amd::METRIC_INNER_PRODUCT;
using faiss_amd::METRIC_L2;

// faiss/impl/FaissException.h
using faiss_amd::FaissException;

// faiss/impl/IDSelector.h
using faiss_amd::IDSelector;
using faiss_amd::IDSelectorArray;
using faiss_amd::IDSelectorBatch;
using faiss_amd::IDSelectorBinary;
using faiss_amd::IDSelectorBitmap;
using faiss_amd::IDSelectorNot;
using faiss_amd::IDSelectorRange;

// faiss/Index.h, faiss/impl/AuxIndexStructures.h
using faiss_amd::Index;
using faiss_amd::InterruptCallback;
using faiss_amd::RangeSearchResult;
using faiss_amd::SearchParameters;
using faiss_amd::TimeoutCallback;

// faiss/IndexFlat.h
using faiss_amd::IndexFlat;
using faiss_amd::IndexFlatIP;
using faiss_amd::IndexFlatL2;

// faiss/impl/HNSW.h, faiss/IndexHNSW.h
using faiss_amd::HNSW;
using faiss_amd::hnsw_stats;
using faiss_amd::HNSWStats;
using faiss_amd::IndexHNSW;
using faiss_amd::IndexHNSWFlat;
using faiss_amd::SearchParametersHNSW;

// faiss/invlists/InvertedLists.h
using faiss_amd::ArrayInvertedLists;
using faiss_amd::SubsetType;
using faiss_amd::SUBSET_TYPE_ELEMENT_RANGE;
using faiss_amd::SUBSET_TYPE_ID_MOD;
using faiss_amd::SUBSET_TYPE_ID_RANGE;
using faiss_amd::SUBSET_TYPE_INVLIST;
using faiss_amd::SUBSET_TYPE_INVLIST_FRACTION;

// faiss/IndexIVF.h (this fork's QueryLatencyStats and search_stats included)
using faiss_amd::IndexIVF;
using faiss_amd::indexIVF_stats;
using faiss_amd::IndexIVFStats;
using faiss_amd::QueryLatencyStats;
using faiss_amd::SearchParametersIVF;

// faiss/IndexIVFFlat.h, faiss/IndexIVFPQ.h, faiss/impl/ProductQuantizer.h
using faiss_amd::IndexIVFFlat;
using faiss_amd::IndexIVFPQ;
using faiss_amd::ProductQuantizer;

// faiss/IndexShardsIVF.h
using faiss_amd::IndexShardsIVF;

// faiss/utils/Heap.h (merge_knn_results, host form)
using faiss_amd::merge_knn_results;

// faiss/index_io.h
using faiss_amd::IO_FLAG_MMAP;
using faiss_amd::IO_FLAG_ONDISK_SAME_DIR;
using faiss_amd::IO_FLAG_PQ_SKIP_SDC_TABLE;
using faiss_amd::IO_FLAG_READ_ONLY;
using faiss_amd::IO_FLAG_SKIP_IVF_DATA;
using faiss_amd::IO_FLAG_SKIP_PRECOMPUTE_TABLE;
using faiss_amd::IO_FLAG_SKIP_STORAGE;
using faiss_amd::read_index;
using faiss_amd::write_index;

// faiss/index_factory.h, faiss/utils/random.h
using faiss_amd::float_rand;
using faiss_amd::index_factory;

}  // namespace faiss
