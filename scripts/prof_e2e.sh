#!/bin/bash
# Kernel + memory-copy trace of one native CLI encode of 10 M plain-FASTQ reads (the GPU
# calls' chain in the encode pipeline: H2D of the text, parse, encode, pack, D2H).
set -e
mkdir -p gpurun_out/prof_e2e
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --reps 1 \
    > gpurun_out/prof_e2e/gen.json 2> gpurun_out/prof_e2e/gen.err
NTC_CLEAN_EXIT=1 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_e2e/trace -o enc \
    --output-format csv -- ./ntcomp_amd/ntcomp encode -i /tmp/ntc_e2e/idx /tmp/ntc_e2e/reads.fq --stats \
    > /tmp/ntc_e2e/x.dat 2> gpurun_out/prof_e2e/enc.err
rm -rf /tmp/ntc_e2e
