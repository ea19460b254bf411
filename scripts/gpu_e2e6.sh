#!/bin/bash
# Round 6: end-to-end CLI (10 M x 150 bp, k = 91) plain / gzip -6 encode and decode, with the
# process's wall-clock timeline (loader, main, exit) from scripts/cli_timeline.py
export TMPDIR=/tmp
O=${O:-gpurun_out/e2e6}
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_plain --reps 3 \
    > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 120 python -u scripts/cli_timeline.py encode /tmp/ntc_plain/idx /tmp/ntc_plain/reads.fq --reps 3 \
    > $O/timeline_plain.jsonl 2>&1 || exit 1
timeout -k 10 120 python -u scripts/cli_timeline.py decode /tmp/ntc_plain/idx /tmp/ntc_plain/enc.dat --reps 3 \
    > $O/timeline_decode.jsonl 2>&1 || exit 1
timeout -k 10 500 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --gzip-level 6 \
    --dir /tmp/ntc_gz6 --reps 3 > $O/gz6.json 2> $O/gz6.err || exit 1
cmp /tmp/ntc_plain/enc.dat /tmp/ntc_gz6/enc.dat && echo "gz6 encoded.dat identical to plain" > $O/cmp.txt
timeout -k 10 120 python -u scripts/cli_timeline.py encode /tmp/ntc_gz6/idx /tmp/ntc_gz6/reads.fq.gz --reps 3 \
    > $O/timeline_gz6.jsonl 2>&1 || exit 1
NTC_PGZ_STATS=1 timeout -k 10 60 ntcomp_amd/ntcomp encode -i /tmp/ntc_gz6/idx /tmp/ntc_gz6/reads.fq.gz --stats \
    2>&1 > /dev/null | grep -v "^chunk" > $O/pgz_stats_gz6.txt || exit 1
rm -rf /tmp/ntc_plain /tmp/ntc_gz6
