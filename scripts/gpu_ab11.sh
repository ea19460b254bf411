#!/bin/bash
# Round 6 A/B: C91 / C31 with 3 device calls in flight against 2 (the default)
export TMPDIR=/tmp
O=${O:-gpurun_out/ab11}
mkdir -p $O
for i in 1 2 3; do
  for f in 2 3; do
    timeout -k 10 300 python -u bench.py --configs encode,c31 --no-cpu --inflight $f > $O/f${f}_$i.json 2> $O/f${f}_$i.err || exit 1
  done
done
