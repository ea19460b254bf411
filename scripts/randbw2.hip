// Random-access roof by allocation kind and load width: does a random load that misses L2
// have to move a 128-byte line?  Independent loads at uniformly random offsets of a buffer
// allocated as
//   cached      hipMalloc (coarse-grained, L2-cached: every miss is a 128 B EA request)
//   uncached    hipExtMallocWithFlags(hipDeviceMallocUncached) (L2 bypass: request = load size?)
//   finegrained hipExtMallocWithFlags(hipDeviceMallocFinegrained)
// with 4, 8 and 16 byte loads, and plain vs nontemporal loads on the cached buffer.
// One JSON line per (kind, width, buffer size).  Profile with rocprofv3 --pmc
// TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum.
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/randbw2.hip -o scripts/randbw2
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

template <typename T, bool NT>
__device__ __forceinline__ uint32_t ld(const T *p) {
    if constexpr (sizeof(T) == 16) {
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        const v4 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p)) : *reinterpret_cast<const v4 *>(p);
        return v.x ^ v.y ^ v.z ^ v.w;
    } else {
        const T v = NT ? __builtin_nontemporal_load(p) : *p;
        return (uint32_t)v ^ (uint32_t)(v >> (sizeof(T) * 4));
    }
}

// each lane: iters rounds of 8 independent loads, each at a random T-aligned offset
template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_rand(const T *buf, uint64_t n, uint32_t iters, uint32_t *sink) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t h = mix(gid + 1);
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; it++) {
        uint32_t v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            h = mix(h + i);
            v[i] = ld<T, NT>(buf + (h & (n - 1)));  // n: power of 2
        }
#pragma unroll
        for (int i = 0; i < 8; i++) acc ^= v[i];
        h ^= acc & 1;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <typename T, bool NT>
int run(const char *kind, const void *buf, uint64_t bytes, uint32_t blocks, uint32_t *sink, hipEvent_t a,
        hipEvent_t b) {
    const uint64_t n = bytes / sizeof(T);
    const uint32_t iters = 32;
    hipLaunchKernelGGL((k_rand<T, NT>), dim3(blocks), dim3(256), 0, 0, (const T *)buf, n, iters, sink);
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 3; r++)
        hipLaunchKernelGGL((k_rand<T, NT>), dim3(blocks), dim3(256), 0, 0, (const T *)buf, n, iters, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double loads = 3.0 * blocks * 256.0 * iters * 8.0;
    printf("{\"test\": \"random_loads\", \"alloc\": \"%s\", \"load_bytes\": %d, \"nontemporal\": %d, "
           "\"buffer_bytes\": %llu, \"g_loads_per_s\": %.2f, \"gb_per_s_at_load_size\": %.1f}\n",
           kind, (int)sizeof(T), (int)NT, (unsigned long long)bytes, loads / ms / 1e6, loads * sizeof(T) / ms / 1e6);
    fflush(stdout);
    return 0;
}

int main(int argc, char **argv) {
    int cus = 0;
    CHECK(hipSetDevice(0));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t big = 4ULL << 30;
    const uint64_t sizes[] = {128ULL << 20, big};
    void *cached, *unc, *fine;
    uint32_t *sink;
    CHECK(hipMalloc(&cached, big));
    CHECK(hipExtMallocWithFlags(&unc, big, hipDeviceMallocUncached));
    CHECK(hipExtMallocWithFlags(&fine, big, hipDeviceMallocFinegrained));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(cached, 1, big));
    CHECK(hipMemset(unc, 1, big));
    CHECK(hipMemset(fine, 1, big));
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const uint32_t blocks = (uint32_t)cus * 8;
    const char *only = argc > 1 ? argv[1] : "";
    for (uint64_t sz : sizes) {
        if (!*only || !strcmp(only, "cached")) {
            if (run<uint32_t, false>("cached", cached, sz, blocks, sink, a, b)) return 1;
            if (run<uint64_t, false>("cached", cached, sz, blocks, sink, a, b)) return 1;
            if (run<uint4, false>("cached", cached, sz, blocks, sink, a, b)) return 1;
            if (run<uint64_t, true>("cached", cached, sz, blocks, sink, a, b)) return 1;
        }
        if (!*only || !strcmp(only, "uncached")) {
            if (run<uint32_t, false>("uncached", unc, sz, blocks, sink, a, b)) return 1;
            if (run<uint64_t, false>("uncached", unc, sz, blocks, sink, a, b)) return 1;
            if (run<uint4, false>("uncached", unc, sz, blocks, sink, a, b)) return 1;
        }
        if (!*only || !strcmp(only, "fine")) {
            if (run<uint64_t, false>("finegrained", fine, sz, blocks, sink, a, b)) return 1;
            if (run<uint4, false>("finegrained", fine, sz, blocks, sink, a, b)) return 1;
        }
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
