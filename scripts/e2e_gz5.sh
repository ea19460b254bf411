#!/bin/bash
# Round 5: end-to-end encode of one-member gzip FASTQ (the reference's own input,
# README.md:30) through the parallel inflater (pgzip.cpp), 10 M x 150 bp, native CLI; the
# encoded.dat must be byte-identical to the one from the plain FASTQ and from --host-parse.
set -e
O=gpurun_out/e2e5
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_plain --reps 2 \
    > $O/plain.json 2> $O/plain.err
for lvl in ${LEVELS:-1 6}; do
  timeout -k 10 500 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --gzip-level $lvl \
      --dir /tmp/ntc_gz$lvl --reps 2 > $O/gz${lvl}.json 2> $O/gz${lvl}.err
  cmp /tmp/ntc_plain/enc.dat /tmp/ntc_gz$lvl/enc.dat && echo "gz$lvl encoded.dat identical to plain" | tee -a $O/cmp.txt
  timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --gzip-level $lvl \
      --dir /tmp/ntc_gz$lvl --keep --host-parse --reps 1 > $O/gz${lvl}_hostparse.json 2> $O/gz${lvl}_hostparse.err
  cmp /tmp/ntc_plain/enc.dat /tmp/ntc_gz$lvl/enc.dat && echo "gz$lvl host-parse encoded.dat identical to plain" | tee -a $O/cmp.txt
  rm -rf /tmp/ntc_gz$lvl
done
rm -rf /tmp/ntc_plain
