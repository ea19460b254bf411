// Host->device paths for a file already in the page cache (e2e ingest experiment):
//   pageable  hipMemcpy from the mmap'd file (the runtime stages it)
//   register  hipHostRegister of the mmap'd file, then hipMemcpy (DMA from page-cache pages)
//   pinned    T threads memcpy the file into hipHostMalloc'd memory, then hipMemcpy
//   parse-like T threads memcpy (the bytes a host parser would touch), no transfer
// usage: hostreg_bw FILE [threads]
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void par_copy(uint8_t *dst, const uint8_t *src, size_t n, int T) {
    std::vector<std::thread> ts;
    for (int t = 0; t < T; t++)
        ts.emplace_back([=] {
            const size_t a = n * t / T, b = n * (t + 1) / T;
            std::memcpy(dst + a, src + a, b - a);
        });
    for (auto &x : ts) x.join();
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const int T = argc > 2 ? atoi(argv[2]) : 16;
    const int fd = open(argv[1], O_RDONLY);
    struct stat st;
    fstat(fd, &st);
    const size_t n = (size_t)st.st_size;
    uint8_t *m = (uint8_t *)mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    volatile uint64_t sink = 0;
    for (size_t i = 0; i < n; i += 4096) sink += m[i];  // fault the mapping in
    void *d = nullptr;
    hipMalloc(&d, n);
    hipDeviceSynchronize();
    double t = now();
    hipMemcpy(d, m, n, hipMemcpyHostToDevice);
    std::printf("{\"path\": \"pageable_h2d\", \"gb_s\": %.2f}\n", n / (now() - t) / 1e9);
    t = now();
    hipError_t e = hipHostRegister(m, n, hipHostRegisterReadOnly);
    const double treg = now() - t;
    if (e == hipSuccess) {
        t = now();
        hipMemcpy(d, m, n, hipMemcpyHostToDevice);
        std::printf("{\"path\": \"registered_h2d\", \"register_gb_s\": %.2f, \"gb_s\": %.2f}\n", n / treg / 1e9,
                    n / (now() - t) / 1e9);
        hipHostUnregister(m);
    } else {
        std::printf("{\"path\": \"registered_h2d\", \"error\": \"%s\"}\n", hipGetErrorString(e));
        (void)hipGetLastError();
    }
    uint8_t *h = nullptr;
    t = now();
    hipHostMalloc((void **)&h, n, hipHostMallocDefault);
    const double tpin = now() - t;
    par_copy(h, m, n, T);  // first touch
    t = now();
    par_copy(h, m, n, T);
    const double tcp = now() - t;
    t = now();
    hipMemcpy(d, h, n, hipMemcpyHostToDevice);
    std::printf("{\"path\": \"pinned\", \"pin_gb_s\": %.2f, \"copy_gb_s\": %.2f, \"threads\": %d, \"h2d_gb_s\": %.2f}\n",
                n / tpin / 1e9, n / tcp / 1e9, T, n / (now() - t) / 1e9);
    hipHostFree(h);
    hipFree(d);
    munmap(m, n);
    close(fd);
    return (int)(sink & 0);
}
