/* Test stub (tests/san only): the HIP runtime names pipeline.cpp uses for its pinned host
 * buffers, backed by plain host memory, so the pipeline's host threads (reader ring and
 * gang, deflate pool, ordered writer) build and run under ASan/UBSan/TSan without a GPU. */
#pragma once
#include <stdlib.h>
typedef enum { hipSuccess = 0, hipErrorOutOfMemory = 2 } hipError_t;
#define hipHostMallocDefault 0u
static inline hipError_t hipHostMalloc(void **p, size_t bytes, unsigned flags) {
    (void)flags;
    *p = NULL;
    if (posix_memalign(p, 4096, bytes ? bytes : 1) != 0) return hipErrorOutOfMemory;
    return hipSuccess;
}
static inline hipError_t hipHostFree(void *p) {
    free(p);
    return hipSuccess;
}
#define hipHostRegisterPortable 1u
static inline hipError_t hipHostRegister(void *p, size_t bytes, unsigned flags) {
    (void)p, (void)bytes, (void)flags;
    return hipSuccess;
}
static inline hipError_t hipHostUnregister(void *p) {
    (void)p;
    return hipSuccess;
}
static inline hipError_t hipGetLastError(void) { return hipSuccess; }
