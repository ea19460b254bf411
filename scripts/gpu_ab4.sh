#!/bin/bash
# Round 6 A/B: S91 secondary entry slots; pgzip close breakdown and ceilings at 10 M reads
export TMPDIR=/tmp
O=${O:-gpurun_out/ab4}
mkdir -p $O
for s in 12 16 24 12 16 24; do
  timeout -k 10 200 python -u bench.py --configs strains --no-cpu --opt ent_slots=$s > $O/s91_slots$s.json 2>> $O/s91.err || exit 1
done
timeout -k 10 400 python3 -u scripts/host_ceiling.py --reads 10000000 --threads 16 --ctx 2 --reps 2 \
    --out /tmp/ntc_ceiling > $O/ceiling10M.jsonl 2> $O/ceiling10M.err || exit 1
for rt in 8 16; do
  NTC_READ_THREADS=$rt timeout -k 10 100 tests/san/host_ceiling encode /tmp/ntc_ceiling/idx /tmp/ntc_ceiling/r.fq \
      /tmp/ntc_ceiling/x.dat 16 0 2 2 0 2 >> $O/plain_rt$rt.txt 2>&1 || exit 1
done
NTC_PGZ_STATS=1 NTC_PIPE_TRACE=1 timeout -k 10 100 tests/san/host_ceiling encode /tmp/ntc_ceiling/idx \
    /tmp/ntc_ceiling/r.fq.gz /tmp/ntc_ceiling/x.dat 16 0 2 2 0 2 2>&1 | grep -v "^chunk" > $O/pgz_close.txt || exit 1
rm -rf /tmp/ntc_ceiling
