#!/bin/bash
# Decode pipeline timeline (NTC_PIPE_TRACE): the first batches' inflate / unpack / decode /
# write events of one 10 M-read decode, GPU unpack (default) and host unpack.
set -e
O=gpurun_out/dec_trace
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_dt --reps 1 \
    > $O/e2e.json 2> $O/e2e.err
for mode in gpu host; do
  if [ $mode = host ]; then export NTC_HOST_UNPACK=1; else unset NTC_HOST_UNPACK; fi
  for rep in 1 2; do
    rm -f /tmp/ntc_dt/dec.fa
    NTC_PIPE_TRACE=${TRACE_N:-12} timeout -k 10 60 ntcomp_amd/ntcomp decode -i /tmp/ntc_dt/idx /tmp/ntc_dt/enc.dat --stats \
        > /tmp/ntc_dt/dec.fa 2> $O/trace_${mode}_$rep.txt
  done
done
rm -rf /tmp/ntc_dt
