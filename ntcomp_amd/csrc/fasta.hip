// Decode output on the GPU: the bases ntc_decode_batch_device left in HBM become the FASTA
// text src/main.rs:203-209 prints, ">seq.{i+1}\n{read}\n" per read, before one D2H copy.
//   k_fasta_sizes  bytes of each read's record (header digits + length + 2 newlines)
//   (scan)         exclusive scan -> byte offsets
//   k_fasta        one wave per read (grid-stride): lanes write the header characters and
//                  copy the read 64 bytes per instruction (coalesced, HBM-bound)
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ntc {

namespace {

__device__ __forceinline__ uint32_t ndigits(uint64_t x) {
    uint32_t d = 1;
    while (x >= 10) {
        x /= 10;
        d++;
    }
    return d;
}

// The offsets are only trusted when the walk left the status clear (~0: capacities held, no
// malformed record); otherwise every size is 0 and k_fasta writes nothing.
__global__ __launch_bounds__(256) void k_fasta_sizes(const uint64_t *offs, uint64_t n, uint64_t first_id,
                                                     const unsigned long long *status, uint64_t *sizes) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    sizes[r] = *status != ~0ull ? 0 : 5 + ndigits(first_id + r) + 1 + (offs[r + 1] - offs[r]) + 1;
}

__global__ __launch_bounds__(256) void k_fasta(const uint8_t *bases, const uint64_t *offs, uint64_t n,
                                               uint64_t first_id, const uint64_t *out_offs, uint64_t out_cap,
                                               uint8_t *out) {
    if (out_offs[n] == 0 || out_offs[n] > out_cap) return;  // a failed walk (sizes 0) or a short buffer
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t o0 = offs[0];
    for (uint64_t r = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); r < n; r += waves) {
        const uint64_t b = offs[r] - o0, len = offs[r + 1] - offs[r];
        uint64_t o = out_offs[r];
        const uint64_t id = first_id + r;
        const uint32_t nd = ndigits(id);
        if (lane < 5 + nd + 1) {
            uint8_t ch;
            if (lane < 5) {
                ch = (uint8_t)">seq."[lane];
            } else if (lane < 5 + nd) {
                uint64_t x = id;
                for (uint32_t t = lane - 5 + 1; t < nd; t++) x /= 10;  // digit lane - 5 from the left
                ch = (uint8_t)('0' + x % 10);
            } else {
                ch = '\n';
            }
            out[o + lane] = ch;
        }
        o += 5 + nd + 1;
        for (uint64_t i = lane; i < len; i += 64) out[o + i] = bases[b + i];
        if (lane == 0) out[o + len] = '\n';
    }
}

}  // namespace

void launch_fasta(const uint8_t *d_bases, const uint64_t *d_offs, uint64_t n, uint64_t first_id,
                  const unsigned long long *d_status, uint64_t *sizes, uint64_t *out_offs, uint64_t *tmp, uint8_t *out,
                  uint64_t out_cap, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_fasta_sizes, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, d_offs, n, first_id,
                       d_status, sizes);
    scan_excl_u64(sizes, n, out_offs, tmp, s);
    const uint64_t blocks = std::min<uint64_t>((n + 3) / 4, 65536);
    hipLaunchKernelGGL(k_fasta, dim3((uint32_t)blocks), dim3(256), 0, s, d_bases, d_offs, n, first_id, out_offs,
                       out_cap, out);
}

}  // namespace ntc
