/*
 * faiss_c.h — drop-in for the reference C API header `c_api/faiss_c.h`
 * (Quaternijkon/hnsw-ivf = Faiss 1.10.0).  A C caller of the reference keeps
 * its `#include "faiss_c.h"` (or <faiss/c_api/faiss_c.h>) and links
 * libfaiss_amd.so: the declarations — the common types (idx_t, the opaque Faiss* handles) and the declaration
 * macros, which a caller may use to name further handle types —
 * are this library's, with the reference's names, signatures and return codes
 * (include/faiss_amd_c.h, which cites each reference declaration).
 */
#ifndef FAISS_C_H
#define FAISS_C_H

#include "../../faiss_amd_c.h"

typedef float faiss_component_t;
typedef float faiss_distance_t;

/* the declaration helpers of the reference header, for callers that use
 * them to name their own handle types */
#ifndef FAISS_DECLARE_CLASS
#define FAISS_DECLARE_CLASS(clazz) typedef struct Faiss##clazz##_H Faiss##clazz;
#define FAISS_DECLARE_CLASS_INHERITED(clazz, parent) \
    typedef struct Faiss##parent##_H Faiss##clazz;
#define FAISS_DECLARE_DESTRUCTOR(clazz) void faiss_##clazz##_free(Faiss##clazz* obj);
#define FAISS_DECLARE_GETTER(clazz, ty, name) \
    ty faiss_##clazz##_##name(const Faiss##clazz*);
#define FAISS_DECLARE_SETTER(clazz, ty, name) \
    void faiss_##clazz##_set_##name(Faiss##clazz*, ty);
#define FAISS_DECLARE_GETTER_SETTER(clazz, ty, name) \
    FAISS_DECLARE_GETTER(clazz, ty, name)            \
    FAISS_DECLARE_SETTER(clazz, ty, name)
#define FAISS_DECLARE_INDEX_DOWNCAST(clazz) \
    Faiss##clazz* faiss_##clazz##_cast(FaissIndex*);
#define FAISS_DECLARE_SEARCH_PARAMETERS_DOWNCAST(clazz) \
    Faiss##clazz* faiss_##clazz##_cast(FaissSearchParameters*);
#endif

#endif /* FAISS_C_H */
