#!/bin/bash
# Round 6 A/B: S91 with two device calls in flight (--strain-inflight 2) against one
export TMPDIR=/tmp
O=${O:-gpurun_out/ab10}
mkdir -p $O
for i in 1 2 3; do
  for s in 1 2; do
    timeout -k 10 300 python -u bench.py --configs strains --no-cpu --strain-inflight $s > $O/s${s}_$i.json 2> $O/s${s}_$i.err || exit 1
  done
done
