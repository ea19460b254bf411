// Rice parameter of rice_encode (src/encode.rs:62-63), host only: glibc's f64 log / exp /
// log1p, the libm the reference's f64::ln / exp / ln_1p call on Linux.  Shared by the host
// packer (block_codec.cpp) and the GPU packer's host step (pack.hip), so both pick the
// parameter exactly as the reference does.
#pragma once
#include <cmath>
#include <cstdint>

// inv_mean = exp(ln(len) - ln(sum)); dsi-bitstream rice::log2_b(p) =
// ceil(log2(-ln(phi) / ln_1p(-p))) cast `as usize` (NaN, negatives -> 0) [ext, recalled]
static inline int ntc_rice_log2_b(uint64_t n, uint64_t sum) {
    const double inv_mean = std::exp(std::log((double)n) - std::log((double)sum));
    const double phi = (std::sqrt(5.0) + 1.0) / 2.0;
    const double v = std::ceil(std::log2(-std::log(phi) / std::log1p(-inv_mean)));
    if (!(v > 0)) return 0;
    if (v > 63) return 63;
    return (int)v;
}
