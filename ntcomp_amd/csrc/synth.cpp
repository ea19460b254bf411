// Seeded synthetic workload of SURVEY.md 8(d): an i.i.d. uniform ACGT genome and 150 bp
// reads with uniform starts, 50 % reverse complemented, i.i.d. substitutions.  Read r
// depends only on (seed, r), so any shard of reads regenerates bit-identically.
#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

#include "../../include/ntcomp_host.h"

namespace {
inline uint64_t splitmix64(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
const uint8_t kBase[4] = {'A', 'C', 'G', 'T'};
}  // namespace

extern "C" int ntc_synth_genome(uint64_t seed, uint64_t length, uint8_t *out) {
    if (!out && length) return NTC_ERR_INVALID_ARG;
    uint64_t s = seed;
    for (uint64_t i = 0; i < length; i += 32) {
        uint64_t x = splitmix64(s);
        for (uint64_t j = 0; j < 32 && i + j < length; j++) out[i + j] = kBase[(x >> (2 * j)) & 3];
    }
    return NTC_OK;
}

// Strain s (0-based) of a collection: the genome with i.i.d. substitutions at rate
// snp_per_million / 1e6; whether position i of strain s mutates, and to which base, depends
// only on (seed, s, i), so strains regenerate identically in any order.
extern "C" int ntc_synth_strains(const uint8_t *genome, uint64_t glen, uint64_t seed, uint32_t n_strains,
                                 uint32_t snp_per_million, uint8_t *out) {
    if ((!genome || !out) && glen && n_strains) return NTC_ERR_INVALID_ARG;
    for (uint32_t st = 0; st < n_strains; st++) {
        uint8_t *o = out + (uint64_t)st * glen;
        for (uint64_t i = 0; i < glen; i++) {
            uint64_t s = seed ^ (0x9E6C63D0676A9A99ULL * ((uint64_t)st + 1)) ^ (0xD6E8FEB86659FD93ULL * (i + 1));
            const uint64_t u = splitmix64(s);
            const uint8_t b0 = genome[i];
            if ((u % 1000000ULL) < snp_per_million) {
                const uint32_t c = b0 == 'A' ? 0 : b0 == 'C' ? 1 : b0 == 'G' ? 2 : 3;
                o[i] = kBase[(c + 1 + (uint32_t)((u >> 32) % 3)) & 3];
            } else {
                o[i] = b0;
            }
        }
    }
    return NTC_OK;
}

extern "C" int ntc_synth_reads(const uint8_t *genome, uint64_t glen, uint64_t seed, uint64_t first_read,
                               uint64_t n_reads, uint32_t read_len, uint32_t err_per_million, int n_threads,
                               uint8_t *out) {
    if (!genome || !out || read_len == 0 || glen < read_len) return NTC_ERR_INVALID_ARG;
    if (n_threads <= 0) n_threads = (int)std::max(1u, std::thread::hardware_concurrency());
    auto work = [&](uint64_t a, uint64_t b) {
        for (uint64_t r = a; r < b; r++) {
            uint64_t s = seed ^ (0xD1B54A32D192ED03ULL * (first_read + r + 1));
            splitmix64(s);
            uint64_t start = splitmix64(s) % (glen - read_len + 1);
            bool rc = splitmix64(s) & 1;
            uint8_t *o = out + r * read_len;
            for (uint32_t j = 0; j < read_len; j++) {
                uint8_t b0 = rc ? genome[start + read_len - 1 - j] : genome[start + j];
                uint32_t c = b0 == 'A' ? 0 : b0 == 'C' ? 1 : b0 == 'G' ? 2 : 3;
                if (rc) c = 3 - c;
                uint64_t u = splitmix64(s);
                if ((u % 1000000ULL) < err_per_million) c = (c + 1 + (uint32_t)((u >> 32) % 3)) & 3;
                o[j] = kBase[c];
            }
        }
    };
    if (n_threads == 1 || n_reads < 4096) {
        work(0, n_reads);
    } else {
        std::vector<std::thread> ts;
        uint64_t chunk = (n_reads + n_threads - 1) / n_threads;
        for (int t = 0; t < n_threads; t++) {
            uint64_t a = t * chunk, b = std::min(n_reads, a + chunk);
            if (a >= b) break;
            ts.emplace_back(work, a, b);
        }
        for (auto &t : ts) t.join();
    }
    return NTC_OK;
}

// Minimizer of each read (bench.py --presort locality experiment): the smallest
// 64-bit-hashed w-mer (2-bit codes, strand as read) of read r = reads[r*L, (r+1)*L).
extern "C" int ntc_minimizer_keys(const uint8_t *reads, uint64_t n_reads, uint32_t read_len, uint32_t w,
                                  int n_threads, uint64_t *keys) {
    if ((!reads || !keys) && n_reads) return NTC_ERR_INVALID_ARG;
    if (w == 0 || w > 32 || read_len < w) return NTC_ERR_INVALID_ARG;
    if (n_threads <= 0) n_threads = (int)std::max(1u, std::thread::hardware_concurrency());
    const uint64_t mask = w == 32 ? ~0ULL : ((1ULL << (2 * w)) - 1);
    auto work = [&](uint64_t a, uint64_t b) {
        for (uint64_t r = a; r < b; r++) {
            const uint8_t *q = reads + r * read_len;
            uint64_t v = 0, best = ~0ULL;
            for (uint32_t j = 0; j < read_len; j++) {
                v = ((v << 2) | (((uint64_t)q[j] >> 1 ^ (uint64_t)q[j] >> 2) & 3)) & mask;
                if (j + 1 >= w) {
                    const uint64_t h = (v * 0x9E3779B97F4A7C15ULL) >> 20;
                    best = h < best ? h : best;
                }
            }
            keys[r] = best;
        }
    };
    std::vector<std::thread> ts;
    const uint64_t chunk = (n_reads + n_threads - 1) / n_threads;
    for (int t = 0; t < n_threads; t++) {
        const uint64_t a = t * chunk, b = std::min(n_reads, a + chunk);
        if (a >= b) break;
        ts.emplace_back(work, a, b);
    }
    for (auto &t : ts) t.join();
    return NTC_OK;
}
