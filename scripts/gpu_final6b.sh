#!/bin/bash
# Round 6 final, part 2: the bench line with this build's counters, the L31 point with its
# PMC passes (scripts/big_point.sh), a 2-rank rehearsal on the one GPU, end-to-end CLI runs
export TMPDIR=/tmp
O=${O:-gpurun_out/final6}
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_final.json 2> $O/bench_final.err || exit 1
OUT=$O/big timeout -k 10 900 bash scripts/big_point.sh > $O/big.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_2ranks.json 2> $O/bench_2ranks.err || exit 1
O=$O/e2e timeout -k 10 900 bash scripts/gpu_e2e6.sh > $O.e2e.log 2>&1 || exit 1
