#!/bin/bash
# Round 6 A/B: k_pack with 4 (cur) / 8 (C) 16-character chunks per thread against 1 (A):
# the pack tests, then a kernel trace per variant (NTC_GPU_LIB) of the C91 bench, then bench lines
export TMPDIR=/tmp
O=${O:-gpurun_out/ab9}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for v in A cur C; do
  lib=ntcomp_amd/libntcomp_gpu_$v.so; [ $v = cur ] && lib=ntcomp_amd/libntcomp_gpu.so
  NTC_GPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- \
      python3 bench.py --configs encode,c31 --no-cpu --steps 10 --warmup 2 > $O/kt_$v.json 2> $O/kt_$v.err || exit 1
done
OUT=$O/pack CONFIGS=encode,c31 VARIANTS="A cur C" REPS=3 timeout -k 10 600 bash scripts/ab_bench.sh > $O/pack.log 2>&1 || exit 1
