#!/bin/bash
# A/B on one box: the CLI's start-up warm-ups (DMA engines, first code objects, workspaces)
# on and off (NTC_NO_WARM=1), 10 M reads, decode and encode process wall clock, alternating.
set -e
O=gpurun_out/warm_ab
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_w --reps 1 \
    > $O/e2e.json 2> $O/e2e.err
for rep in 1 2 3 4; do
  for w in on off; do
    if [ $w = off ]; then export NTC_NO_WARM=1; else unset NTC_NO_WARM; fi
    rm -f /tmp/ntc_w/dec.fa /tmp/ntc_w/enc2.dat
    t0=$(date +%s.%N)
    timeout -k 10 60 ntcomp_amd/ntcomp decode -i /tmp/ntc_w/idx /tmp/ntc_w/enc.dat --stats > /tmp/ntc_w/dec.fa 2> $O/dec_${w}_$rep.txt
    t1=$(date +%s.%N)
    timeout -k 10 60 ntcomp_amd/ntcomp encode -i /tmp/ntc_w/idx /tmp/ntc_w/reads.fq --stats > /tmp/ntc_w/enc2.dat 2> $O/enc_${w}_$rep.txt
    t2=$(date +%s.%N)
    python3 -c "print('wall', round($t1 - $t0, 4))" >> $O/dec_${w}_$rep.txt
    python3 -c "print('wall', round($t2 - $t1, 4))" >> $O/enc_${w}_$rep.txt
  done
done
rm -rf /tmp/ntc_w
