#!/bin/bash
# A/B of library builds on one box: bench.py configs (default strains,encode) for each
# variant in VARIANTS (X = ntcomp_amd/libntcomp_gpu_X.so via NTC_GPU_LIB, "cur" = the in-tree
# library), round-robin, REPS rounds.  Summary: scripts/ab_summary.py $OUT.
set -e
CONFIGS=${CONFIGS:-strains,encode}
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
for i in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-A cur}; do
    lib=ntcomp_amd/libntcomp_gpu_$v.so
    [ "$v" = cur ] && lib=ntcomp_amd/libntcomp_gpu.so
    NTC_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --configs $CONFIGS --no-cpu ${BENCH_ARGS:-} \
        > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err
  done
done
