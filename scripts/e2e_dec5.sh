#!/bin/bash
# Round 5: decode end to end with the streams decoded on the GPU (default) against the host
# decode (NTC_HOST_UNPACK=1), 10 M x 150 bp at k = 91, native CLI, same encoded.dat.
set -e
O=gpurun_out/e2e5
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_dec \
    --reps 3 > $O/plain_gpuunpack.json 2> $O/plain_gpuunpack.err
NTC_HOST_UNPACK=1 timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_dec \
    --keep --reps 3 > $O/plain_hostunpack.json 2> $O/plain_hostunpack.err
rm -rf /tmp/ntc_dec
