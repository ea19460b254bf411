#!/bin/bash
# Kernel + copy trace of one CLI decode of 10 M reads (the first batches' costs).
set -e
O=gpurun_out/dec_prof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_dp --reps 1 \
    > $O/e2e.json 2> $O/e2e.err
NTC_CLEAN_EXIT=1 NTC_PIPE_TRACE=4 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/prof -o dec --output-format csv -- \
    ntcomp_amd/ntcomp decode -i /tmp/ntc_dp/idx /tmp/ntc_dp/enc.dat --stats > /tmp/ntc_dp/dec.fa 2> $O/dec.err
rm -rf /tmp/ntc_dp
