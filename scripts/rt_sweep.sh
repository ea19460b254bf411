#!/bin/bash
# Encode pipeline (GPU-parsed plain FASTQ, adaptive deflate) over the reader gang's threads
# (NTC_READ_THREADS) x calls per batch x contexts on one GPU (scripts/pipe_bench.py).
set -e
mkdir -p gpurun_out/e2e
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --reps 1 \
    > gpurun_out/e2e/gen.json 2> gpurun_out/e2e/gen.err
for rt in ${RT_LIST:-8 16}; do
  NTC_READ_THREADS=$rt timeout -k 10 200 python -u scripts/pipe_bench.py --dir /tmp/ntc_e2e --deflate adaptive \
    --bpb ${BPB_LIST:-4 8} --contexts ${CTX_LIST:-2 3} --parse gpu --reps 3 | sed "s/^{/{\"read_threads\": $rt, /" \
    >> gpurun_out/e2e/rt_sweep.jsonl
done
rm -rf /tmp/ntc_e2e
