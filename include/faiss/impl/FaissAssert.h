// faiss/impl/FaissAssert.h — FaissException and the FAISS_THROW_* macros
// (faiss/impl/FaissAssert.h, faiss/impl/FaissException.h): the library's
// macros throw faiss_amd::FaissException, which is faiss::FaissException.
#pragma once
#include "faiss_amd_names.h"

#ifndef FAISS_ASSERT
#define FAISS_ASSERT(X)                                                              \
    do {                                                                             \
        if (!(X)) {                                                                  \
            fprintf(stderr, "Faiss assertion '%s' failed in %s at %s:%d\n", #X,      \
                    __PRETTY_FUNCTION__, __FILE__, __LINE__);                        \
            abort();                                                                 \
        }                                                                            \
    } while (false)
#endif
#ifndef FAISS_ASSERT_MSG
#define FAISS_ASSERT_MSG(X, MSG)                                                     \
    do {                                                                             \
        if (!(X)) {                                                                  \
            fprintf(stderr, "Faiss assertion '%s' failed in %s at %s:%d; details: " MSG "\n", \
                    #X, __PRETTY_FUNCTION__, __FILE__, __LINE__);                    \
            abort();                                                                 \
        }                                                                            \
    } while (false)
#endif
