#!/bin/bash
# End-to-end encode on one box: the native CLI (scripts/e2e_bench.py, plain FASTQ) with its
# defaults (FASTQ parsed on the GPU, 2 encode contexts per GPU, --deflate auto = adaptive),
# then one change at a time (libdeflate everywhere, 1 context, host parse), then the native
# pipeline alone over engines x calls per batch x contexts (scripts/pipe_bench.py).
set -e
mkdir -p gpurun_out/e2e
timeout -k 10 400 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto ${E2E_ARGS:-} \
    > gpurun_out/e2e/plain_auto.json 2> gpurun_out/e2e/plain_auto.err
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate libdeflate --keep \
    > gpurun_out/e2e/plain_ld.json 2> gpurun_out/e2e/plain_ld.err
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --keep --contexts-per-gpu 1 \
    > gpurun_out/e2e/plain_auto_1ctx.json 2> gpurun_out/e2e/plain_auto_1ctx.err
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --keep --host-parse \
    > gpurun_out/e2e/plain_auto_hostparse.json 2> gpurun_out/e2e/plain_auto_hostparse.err
for eng in adaptive libdeflate; do
  timeout -k 10 300 python -u scripts/pipe_bench.py --dir /tmp/ntc_e2e --deflate $eng --bpb 4 8 \
      --contexts 1 2 --parse gpu --reps 2 >> gpurun_out/e2e/pipe_sweep.jsonl 2>> gpurun_out/e2e/pipe_sweep.err
done
for sc in spin yield blocking; do
  NTC_DEVICE_SCHEDULE=$sc timeout -k 10 200 python -u scripts/pipe_bench.py --dir /tmp/ntc_e2e --deflate adaptive \
    --bpb 4 --contexts 2 --parse gpu --reps 3 | sed "s/^{/{\"schedule\": \"$sc\", /" >> gpurun_out/e2e/sched_sweep.jsonl
done
rm -rf /tmp/ntc_e2e
