#!/bin/bash
# End-to-end encode on one box: the native CLI (scripts/e2e_bench.py, plain FASTQ, libdeflate)
# with its defaults (FASTQ parsed on the GPU, 2 encode contexts per GPU), one context, and the
# FASTQ parsed on the host pool; then the native pipeline alone over calls per batch x
# contexts x parse (scripts/pipe_bench.py).
set -e
mkdir -p gpurun_out/e2e
timeout -k 10 400 python -u scripts/e2e_bench.py --reads 10000000 --deflate libdeflate ${E2E_ARGS:-} \
    > gpurun_out/e2e/plain_ld.json 2> gpurun_out/e2e/plain_ld.err
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate libdeflate --keep --contexts-per-gpu 1 \
    > gpurun_out/e2e/plain_ld_1ctx.json 2> gpurun_out/e2e/plain_ld_1ctx.err
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate libdeflate --keep --host-parse \
    > gpurun_out/e2e/plain_ld_hostparse.json 2> gpurun_out/e2e/plain_ld_hostparse.err
timeout -k 10 300 python -u scripts/pipe_bench.py --dir /tmp/ntc_e2e --deflate libdeflate --bpb 4 8 16 \
    --contexts 1 2 --parse gpu host --reps 2 > gpurun_out/e2e/pipe_sweep.jsonl 2> gpurun_out/e2e/pipe_sweep.err
rm -rf /tmp/ntc_e2e
