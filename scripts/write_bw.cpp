// Decode's output bound: how fast can one process put T bytes of text into a fresh regular
// file's page cache, in batches of B bytes (the pipeline's per-batch write)?
//   pwrite1   one pwrite per batch
//   pwriteW   W threads, one pwrite each per batch (the round-5 writer)
//   mmapW     ftruncate per batch, the batch's range mapped shared, W threads populate
//             (MADV_POPULATE_WRITE) and copy their part, munmap
//   odirect1  one O_DIRECT pwrite per batch from a 4 KiB-aligned buffer (no page cache)
// usage: write_bw DIR [total_MB] [batch_MB] [W]    -> one JSON line per mode
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <unistd.h>

#include <cerrno>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    const size_t total = (size_t)(argc > 2 ? atol(argv[2]) : 1600) << 20;
    const size_t batch = (size_t)(argc > 3 ? atol(argv[3]) : 21) << 20;
    const int W = argc > 4 ? atoi(argv[4]) : 8;
    std::vector<uint8_t> src(batch);
    for (size_t i = 0; i < batch; i++) src[i] = (uint8_t)("ACGT\n"[i % 5]);
    struct statfs sf;
    statfs(dir.c_str(), &sf);
    const long page = sysconf(_SC_PAGESIZE);
    // O_DIRECT needs an aligned source: a 4 KiB-aligned copy of the batch
    uint8_t *asrc = nullptr;
    if (posix_memalign((void **)&asrc, 4096, batch) != 0) return 1;
    memcpy(asrc, src.data(), batch);
    const char *modes_env = getenv("WRITE_BW_MODES");
    std::vector<std::string> modes = {"pwrite1", "pwriteW", "mmapW", "mmapW_nopop", "odirect1"};
    if (modes_env) {
        modes.clear();
        for (const char *q = modes_env; *q;) {
            const char *c = strchr(q, ',');
            modes.push_back(c ? std::string(q, c - q) : std::string(q));
            if (!c) break;
            q = c + 1;
        }
    }
    for (const std::string &ms : modes) {
        const char *mode = ms.c_str();
        const std::string path = dir + "/write_bw.out";
        unlink(path.c_str());
        const bool direct = !strcmp(mode, "odirect1");
        const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | (direct ? O_DIRECT : 0), 0644);
        if (fd < 0) {
            printf("{\"mode\": \"%s\", \"ok\": false, \"open_errno\": %d}\n", mode, errno);
            continue;
        }
        const double t0 = now();
        size_t pos = 0;
        bool ok = true;
        while (pos < total && ok) {
            const size_t n = std::min(batch, total - pos);
            if (!strcmp(mode, "pwrite1")) {
                ok = pwrite(fd, src.data(), n, (off_t)pos) == (ssize_t)n;
            } else if (direct) {
                const size_t na = n / 4096 * 4096;  // (the batch size is a multiple of 4 KiB here)
                ok = pwrite(fd, asrc, na, (off_t)pos) == (ssize_t)na;
            } else if (!strcmp(mode, "pwriteW")) {
                std::vector<std::thread> ts;
                std::atomic<bool> good{true};
                for (int w = 0; w < W; w++)
                    ts.emplace_back([&, w] {
                        const size_t a = n * w / W, e = n * (w + 1) / W;
                        if (pwrite(fd, src.data() + a, e - a, (off_t)(pos + a)) != (ssize_t)(e - a)) good = false;
                    });
                for (auto &t : ts) t.join();
                ok = good;
            } else {
                const bool pop = !strcmp(mode, "mmapW");
                if (ftruncate(fd, (off_t)(pos + n)) != 0) {
                    ok = false;
                    break;
                }
                const size_t a0 = pos / page * page, skew = pos - a0;
                uint8_t *m = (uint8_t *)mmap(nullptr, n + skew, PROT_READ | PROT_WRITE, MAP_SHARED, fd, (off_t)a0);
                if (m == MAP_FAILED) {
                    ok = false;
                    break;
                }
                std::vector<std::thread> ts;
                for (int w = 0; w < W; w++)
                    ts.emplace_back([&, w] {
                        size_t a = n * w / W, e = n * (w + 1) / W;
                        if (pop) {
                            const size_t pa = (skew + a) / page * page, pe = (skew + e + page - 1) / page * page;
                            madvise(m + pa, pe - pa, MADV_POPULATE_WRITE);
                        }
                        memcpy(m + skew + a, src.data() + a, e - a);
                    });
                for (auto &t : ts) t.join();
                munmap(m, n + skew);
            }
            pos += n;
        }
        const double t1 = now();
        close(fd);
        const double t2 = now();
        unlink(path.c_str());
        printf("{\"mode\": \"%s\", \"ok\": %s, \"fs_magic\": \"0x%lx\", \"MB\": %zu, \"batch_MB\": %zu, \"threads\": %d, "
               "\"s\": %.4f, \"GB_s\": %.2f, \"close_s\": %.4f}\n",
               mode, ok ? "true" : "false", (unsigned long)sf.f_type, total >> 20, batch >> 20, W, t1 - t0,
               total / (t1 - t0) / 1e9, t2 - t1);
        fflush(stdout);
    }
    return 0;
}
