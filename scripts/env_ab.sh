#!/bin/bash
# A/B of environment settings on one box, alternating: bash scripts/env_ab.sh <configs> "name|VAR=v VAR2=w" ...
# ("name|" = no extra setting).  Output gpurun_out/env_ab/<name>.<i>.json (scripts/ab_summary.py).
set -e
O=gpurun_out/env_ab
mkdir -p $O
CFG=${1:-encode,strains}
shift
for i in 1 2; do
  for spec in "$@"; do
    n="${spec%%|*}"; envs="${spec#*|}"
    env $envs timeout -k 10 300 python -u bench.py --configs $CFG --no-cpu --steps 10 --warmup 3 > $O/$n.$i.json 2> $O/$n.$i.err
  done
done
