#!/bin/bash
# End-to-end encode of compressed FASTQ (10 M x 150 bp) with the native CLI: BGZF and one
# gzip member, the text parsed on the GPU (default, the streamed text path) or on the host.
set -e
mkdir -p gpurun_out/e2e
timeout -k 10 400 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --bgzf --dir /tmp/ntc_bgzf \
    > gpurun_out/e2e/bgzf_auto.json 2> gpurun_out/e2e/bgzf_auto.err
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --bgzf --dir /tmp/ntc_bgzf \
    --keep --host-parse > gpurun_out/e2e/bgzf_hostparse.json 2> gpurun_out/e2e/bgzf_hostparse.err
rm -rf /tmp/ntc_bgzf
timeout -k 10 400 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --dir /tmp/ntc_gz --reps 1 \
    > gpurun_out/e2e/gz_auto.json 2> gpurun_out/e2e/gz_auto.err
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --dir /tmp/ntc_gz --reps 1 \
    --keep --host-parse > gpurun_out/e2e/gz_hostparse.json 2> gpurun_out/e2e/gz_hostparse.err
rm -rf /tmp/ntc_gz
