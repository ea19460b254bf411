// Host ingest rates for a plain FASTQ already in the page cache (e2e ingest experiment,
// DESIGN.md "End-to-end"): what the encode reader can feed a GPU-side parse.
//   pin        hipHostMalloc of one slot, and malloc + first touch + hipHostRegister
//   pread      T threads pread the file slot by slot into a pinned slot
//   pread+nl   the same, each thread counting newlines (SSE2) in the piece it just read
//   mmap       T threads read a fresh mapping of the file (page faults included)
// usage: ingest_bw FILE [slot_mb]    (prints one JSON line per measurement)
#include <emmintrin.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static uint64_t count_nl(const uint8_t *p, size_t n) {
    uint64_t c = 0;
    size_t i = 0;
    const __m128i nl = _mm_set1_epi8('\n');
    for (; i + 64 <= n; i += 64) {
        const uint32_t a = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(p + i)), nl));
        const uint32_t b = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(p + i + 16)), nl));
        const uint32_t d = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(p + i + 32)), nl));
        const uint32_t e = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(p + i + 48)), nl));
        c += (uint64_t)__builtin_popcountll((uint64_t)a | (uint64_t)b << 16 | (uint64_t)d << 32 | (uint64_t)e << 48);
    }
    for (; i < n; i++) c += p[i] == '\n';
    return c;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const size_t slot = (argc > 2 ? (size_t)atoi(argv[2]) : 96) << 20;
    if (argc > 3) {  // write N reads of 150 bp first: "@r<i>", bases, "+", quality
        FILE *f = std::fopen(argv[1], "wb");
        uint64_t x = 88172645463325252ull;
        char rec[512];
        for (long i = 0, N = atol(argv[3]); i < N; i++) {
            int p = std::snprintf(rec, 64, "@r%ld\n", i);
            for (int j = 0; j < 150; j++) {
                x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                rec[p++] = "ACGT"[x & 3];
            }
            rec[p++] = '\n', rec[p++] = '+', rec[p++] = '\n';
            std::memset(rec + p, 'I', 150);
            p += 150;
            rec[p++] = '\n';
            std::fwrite(rec, 1, (size_t)p, f);
        }
        std::fclose(f);
    }
    const int fd = open(argv[1], O_RDONLY);
    struct stat st;
    fstat(fd, &st);
    const size_t n = (size_t)st.st_size;
    (void)hipFree(nullptr);
    double t = now();
    uint8_t *pin = nullptr;
    if (hipHostMalloc((void **)&pin, slot, hipHostMallocDefault) != hipSuccess) return 3;
    std::printf("{\"what\": \"hipHostMalloc\", \"mb\": %zu, \"s\": %.4f}\n", slot >> 20, now() - t);
    t = now();
    uint8_t *reg = (uint8_t *)std::aligned_alloc(2u << 20, slot);
    madvise(reg, slot, MADV_HUGEPAGE);
    std::memset(reg, 0, slot);
    const double t_touch = now() - t;
    t = now();
    const hipError_t e = hipHostRegister(reg, slot, hipHostRegisterDefault);
    std::printf("{\"what\": \"malloc+touch+hipHostRegister\", \"mb\": %zu, \"touch_s\": %.4f, \"register_s\": %.4f, \"ok\": %d}\n",
                slot >> 20, t_touch, now() - t, e == hipSuccess);
    if (e == hipSuccess) (void)hipHostUnregister(reg);
    std::free(reg);

    for (int count : {0, 1})
        for (int T : {4, 8, 12, 16}) {
            std::atomic<uint64_t> lines{0};
            t = now();
            for (size_t off = 0; off < n; off += slot) {
                const size_t len = std::min(slot, n - off);
                std::vector<std::thread> th;
                for (int i = 0; i < T; i++)
                    th.emplace_back([&, i] {
                        // 4 MiB pieces dealt round-robin, so each piece is counted while it is hot
                        uint64_t c = 0;
                        for (size_t a = (size_t)i << 22; a < len; a += (size_t)T << 22) {
                            const size_t b = std::min(len, a + (4u << 20));
                            size_t done = 0;
                            while (done < b - a) {
                                const ssize_t r = pread(fd, pin + a + done, b - a - done, (off_t)(off + a + done));
                                if (r <= 0) break;
                                done += (size_t)r;
                            }
                            if (count) c += count_nl(pin + a, b - a);
                        }
                        lines += c;
                    });
                for (auto &x : th) x.join();
            }
            const double s = now() - t;
            std::printf("{\"what\": \"pread%s\", \"threads\": %d, \"gb_s\": %.2f, \"lines\": %llu}\n",
                        count ? "+nl" : "", T, n / s / 1e9, (unsigned long long)lines.load());
        }
    for (int T : {8, 16}) {
        t = now();
        const uint8_t *m = (const uint8_t *)mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
        std::atomic<uint64_t> lines{0};
        std::vector<std::thread> th;
        for (int i = 0; i < T; i++)
            th.emplace_back([&, i] {
                uint64_t c = 0;
                for (size_t a = (size_t)i << 22; a < n; a += (size_t)T << 22) c += count_nl(m + a, std::min(n, a + (4u << 20)) - a);
                lines += c;
            });
        for (auto &x : th) x.join();
        const double s = now() - t;
        munmap((void *)m, n);
        std::printf("{\"what\": \"mmap+nl\", \"threads\": %d, \"gb_s\": %.2f, \"lines\": %llu}\n", T, n / s / 1e9,
                    (unsigned long long)lines.load());
    }
    {
        void *d = nullptr;
        (void)hipMalloc(&d, slot);
        hipStream_t s;
        (void)hipStreamCreate(&s);
        t = now();
        for (int r = 0; r < 10; r++) (void)hipMemcpyAsync(d, pin, slot, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
        std::printf("{\"what\": \"h2d pinned slot\", \"gb_s\": %.2f}\n", 10.0 * slot / (now() - t) / 1e9);
        (void)hipFree(d);
    }
    (void)hipHostFree(pin);
    close(fd);
    return 0;
}
