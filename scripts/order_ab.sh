#!/bin/bash
# A/B: k_ms4's reads in minimizer order (NTC_READ_ORDER=1) against read order, alternating.
# (The NTC_READ_ORDER build measured slower and was reverted: DESIGN.md §9, profiles/round5/ab_read_order/.)
set -e
O=gpurun_out/order_ab
mkdir -p $O
for i in 1 2; do
  for v in 0 1; do
    NTC_READ_ORDER=$v timeout -k 10 300 python -u bench.py --configs ${CFG:-encode,c31,strains} --steps 10 --warmup 3 --no-cpu \
        > $O/ord$v.$i.json 2> $O/ord$v.$i.err
  done
done
