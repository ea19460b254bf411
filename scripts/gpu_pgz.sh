#!/bin/bash
# Round 6: host side of the gzip encode and the decode writer on the box (no kernels timed):
# host ceilings (GPU stage memoised), THP chunk buffers on/off, then the real CLI end to end.
export TMPDIR=/tmp
O=${O:-gpurun_out/pgz}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/host_ceiling.py --reads 4000000 --threads 8,16 --ctx 2 --reps 3 \
    --out /tmp/ntc_ceiling > $O/ceiling.jsonl 2> $O/ceiling.err || exit 1
for thp in 1 0 1 0; do
  NTC_PGZ_THP=$thp NTC_PIPE_TRACE=1 timeout -k 10 100 tests/san/host_ceiling encode /tmp/ntc_ceiling/idx \
      /tmp/ntc_ceiling/r.fq.gz /tmp/ntc_ceiling/x.dat 16 0 2 2 0 2 >> $O/thp$thp.txt 2>&1 || exit 1
done
rm -rf /tmp/ntc_ceiling
timeout -k 10 500 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --gzip-level 6 \
    --dir /tmp/ntc_gz6 --reps 3 > $O/e2e_gz6.json 2> $O/e2e_gz6.err || exit 1
