#!/bin/bash
# alternating A/B of (library, extra bench arguments) pairs:
#   bash scripts/ab_run2.sh <configs> "name|lib|args" ...   (lib "cur" = the in-tree build)
set -e
mkdir -p gpurun_out/ab
CFG=${1:-encode,strains}
shift
for i in 1 2; do
  for spec in "$@"; do
    n="${spec%%|*}"; rest="${spec#*|}"; L="${rest%%|*}"; args="${rest#*|}"
    B="python -u bench.py --configs $CFG --no-cpu --steps 10 --warmup 3 $args"
    if [ "$L" = cur ]; then
      timeout -k 10 300 $B > gpurun_out/ab/$n.$i.json 2> gpurun_out/ab/$n.$i.err
    else
      NTC_GPU_LIB=$L timeout -k 10 300 $B > gpurun_out/ab/$n.$i.json 2> gpurun_out/ab/$n.$i.err
    fi
  done
done
