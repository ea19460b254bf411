#!/bin/bash
# Decode / encode first-call costs: the CLI with HIP's deferred code-object loading on
# on (1), off (0: every code object loads at HIP start) and the CLI's own setting (default).
set -e
O=gpurun_out/dec_trace2
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_dt --reps 1 \
    > $O/e2e.json 2> $O/e2e.err
for rep in 1 2 3; do
  for dl in 1 0 default; do
    rm -f /tmp/ntc_dt/dec.fa /tmp/ntc_dt/enc2.dat
    t0=$(date +%s.%N)
    if [ $dl = default ]; then unset HIP_ENABLE_DEFERRED_LOADING; else export HIP_ENABLE_DEFERRED_LOADING=$dl; fi
    NTC_PIPE_TRACE=3 timeout -k 10 60 ntcomp_amd/ntcomp decode \
        -i /tmp/ntc_dt/idx /tmp/ntc_dt/enc.dat --stats > /tmp/ntc_dt/dec.fa 2> $O/dec_dl${dl}_$rep.txt
    t1=$(date +%s.%N)
    python3 -c "print('wall', round($t1 - $t0, 3))" >> $O/dec_dl${dl}_$rep.txt
    timeout -k 10 60 ntcomp_amd/ntcomp encode \
        -i /tmp/ntc_dt/idx /tmp/ntc_dt/reads.fq --stats > /tmp/ntc_dt/enc2.dat 2> $O/enc_dl${dl}_$rep.txt
    t2=$(date +%s.%N)
    python3 -c "print('wall', round($t2 - $t1, 3))" >> $O/enc_dl${dl}_$rep.txt
  done
done
rm -rf /tmp/ntc_dt
