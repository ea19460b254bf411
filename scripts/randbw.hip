// Random-access roof of one MI355X: independent 8-byte loads at uniformly random 128-byte
// lines of a buffer of a given size (L2-, Infinity-Cache- and HBM-resident sizes), plus a
// streaming read for reference.  k_ms4 and k_parse4 are bound by random lines, not by
// streaming bytes: this is the yardstick DESIGN.md quotes next to their request rates.
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/randbw.hip -o scripts/randbw
// run:   scripts/randbw            (prints one JSON line per buffer size)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

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

// each lane: iters rounds of 8 independent loads (one per random line)
__global__ __launch_bounds__(256) void k_rand(const uint64_t *buf, uint64_t lines, uint32_t iters, uint64_t *sink) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t h = mix(gid + 1), acc = 0;
    for (uint32_t it = 0; it < iters; it++) {
        uint64_t v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            h = mix(h + i);
            v[i] = buf[(h & (lines - 1)) * 16 + (h >> 60)];  // 8 B at a random offset of a random line (lines: power of 2)
        }
#pragma unroll
        for (int i = 0; i < 8; i++) acc ^= v[i];
        h ^= acc & 1;  // keep the loads live without serialising them
    }
    if (acc == 0x123456789ULL) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_stream(const uint4 *buf, uint64_t n16, uint64_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345u) sink[0] = acc;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipSetDevice(dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t sizes[] = {2ULL << 20, 32ULL << 20, 128ULL << 20, 512ULL << 20, 4ULL << 30};
    uint64_t *buf, *sink;
    CHECK(hipMalloc(&buf, sizes[4]));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 1, sizes[4]));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const uint32_t blocks = (uint32_t)cus * 8, iters = 64;
    for (uint64_t sz : sizes) {
        const uint64_t lines = sz / 128;
        hipLaunchKernelGGL(k_rand, dim3(blocks), dim3(256), 0, 0, buf, lines, iters, sink);
        CHECK(hipEventRecord(a));
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_rand, dim3(blocks), dim3(256), 0, 0, buf, lines, iters, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double loads = 5.0 * blocks * 256.0 * iters * 8.0;
        printf("{\"test\": \"random_8B_loads\", \"buffer_bytes\": %llu, \"g_lines_per_s\": %.2f, "
               "\"gb_per_s_at_128B\": %.1f, \"gb_per_s_at_64B\": %.1f}\n",
               (unsigned long long)sz, loads / ms / 1e6, loads * 128 / ms / 1e6, loads * 64 / ms / 1e6);
    }
    const uint64_t n16 = sizes[4] / 16;
    hipLaunchKernelGGL(k_stream, dim3(blocks * 4), dim3(256), 0, 0, (const uint4 *)buf, n16, sink);
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_stream, dim3(blocks * 4), dim3(256), 0, 0, (const uint4 *)buf, n16, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"test\": \"stream_16B_loads\", \"buffer_bytes\": %llu, \"gb_per_s\": %.1f}\n",
           (unsigned long long)sizes[4], 5.0 * sizes[4] / ms / 1e6);
    CHECK(hipDeviceSynchronize());
    return 0;
}
