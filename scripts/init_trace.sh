#!/bin/bash
# CLI start-up timeline (NTC_INIT_TRACE): context creation, index preparation and upload, for
# decode and encode of 10 M reads, 3 runs each.
set -e
O=gpurun_out/init_trace
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_i --reps 1 \
    > $O/e2e.json 2> $O/e2e.err
for rep in 1 2 3; do
  rm -f /tmp/ntc_i/dec.fa /tmp/ntc_i/enc2.dat
  NTC_INIT_TRACE=1 timeout -k 10 60 ntcomp_amd/ntcomp decode -i /tmp/ntc_i/idx /tmp/ntc_i/enc.dat --stats > /tmp/ntc_i/dec.fa 2> $O/dec_$rep.txt
  NTC_INIT_TRACE=1 timeout -k 10 60 ntcomp_amd/ntcomp encode -i /tmp/ntc_i/idx /tmp/ntc_i/reads.fq --stats > /tmp/ntc_i/enc2.dat 2> $O/enc_$rep.txt
done
rm -rf /tmp/ntc_i
