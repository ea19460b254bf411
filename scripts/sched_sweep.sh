#!/bin/bash
# Encode pipeline (GPU-parsed plain FASTQ, 2 contexts, 4 blocks per call) over how host
# threads wait for the device (NTC_DEVICE_SCHEDULE), scripts/pipe_bench.py.
set -e
mkdir -p gpurun_out/e2e
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate libdeflate --reps 1 \
    > gpurun_out/e2e/gen.json 2> gpurun_out/e2e/gen.err
for sc in auto spin yield blocking; do
  NTC_DEVICE_SCHEDULE=$sc timeout -k 10 200 python -u scripts/pipe_bench.py --dir /tmp/ntc_e2e --deflate libdeflate \
    --bpb 4 --contexts 1 2 --parse gpu --reps 3 | sed "s/^{/{\"schedule\": \"$sc\", /" >> gpurun_out/e2e/sched_sweep.jsonl
done
rm -rf /tmp/ntc_e2e
