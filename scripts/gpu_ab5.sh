#!/bin/bash
# Round 6 A/B: ones_down word pairs in k_parse4 (A = off), C31 + C91 + S91; S91 secondary slots 16 vs 20
export TMPDIR=/tmp
O=${O:-gpurun_out/ab5}
mkdir -p $O
OUT=$O/ones CONFIGS=c31,encode,strains VARIANTS="A cur" REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh > $O/ones.log 2>&1 || exit 1
for i in 1 2 3; do for s in 16 20; do
  timeout -k 10 200 python -u bench.py --configs strains --no-cpu --opt ent_slots=$s > $O/s91_slots${s}_$i.json 2>> $O/s91.err || exit 1
done; done
