#!/bin/bash
# Round 6: the encode's input prefetch (ntc_encode_prefetch while the contexts start) A/B,
# gzip -6 single member and plain FASTQ, alternating; NTC_PREFETCH=0 = no prefetch
export TMPDIR=/tmp
O=${O:-gpurun_out/e2e8}
mkdir -p $O
timeout -k 10 500 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --gzip --gzip-level 6 \
    --dir /tmp/ntc_gz6 --reps 3 > $O/gz6.json 2> $O/gz6.err || exit 1
for i in 1 2; do
  for pf in 0 1; do
    NTC_PREFETCH=$pf timeout -k 10 120 python -u scripts/cli_timeline.py encode /tmp/ntc_gz6/idx \
        /tmp/ntc_gz6/reads.fq.gz --reps 3 >> $O/timeline_gz6_pf$pf.jsonl 2>&1 || exit 1
  done
done
NTC_PREFETCH=1 timeout -k 10 60 ntcomp_amd/ntcomp encode -i /tmp/ntc_gz6/idx /tmp/ntc_gz6/reads.fq.gz > /tmp/pf1.dat || exit 1
NTC_PREFETCH=0 timeout -k 10 60 ntcomp_amd/ntcomp encode -i /tmp/ntc_gz6/idx /tmp/ntc_gz6/reads.fq.gz > /tmp/pf0.dat || exit 1
cmp /tmp/pf1.dat /tmp/pf0.dat && cmp /tmp/pf1.dat /tmp/ntc_gz6/enc.dat && echo "prefetch encoded.dat identical" > $O/cmp.txt
gzip -dc /tmp/ntc_gz6/reads.fq.gz > /tmp/plain.fq || exit 1
rm -f /tmp/pf1.dat /tmp/pf0.dat
for i in 1 2; do
  for pf in 0 1 2; do
    pop=0; [ $pf = 2 ] && pop=1
    NTC_PREFETCH=$(( pf > 0 ? 1 : 0 )) NTC_PREFETCH_POPULATE=$pop timeout -k 10 120 python -u scripts/cli_timeline.py \
        encode /tmp/ntc_gz6/idx /tmp/plain.fq --reps 3 >> $O/timeline_plain_pf$pf.jsonl 2>&1 || exit 1
  done
done
rm -rf /tmp/ntc_gz6 /tmp/plain.fq
