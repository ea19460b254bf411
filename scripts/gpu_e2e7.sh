#!/bin/bash
# Round 6: end-to-end CLI after the decode's one-block first batch and pgzip's early unmaps;
# decode first batch A/B (NTC_FIRST_BATCH_BLOCKS=2 = round 5's batches)
export TMPDIR=/tmp
O=${O:-gpurun_out/e2e7}
mkdir -p $O
O=$O timeout -k 10 900 bash scripts/gpu_e2e6.sh > $O/e2e6.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 10000000 --deflate auto --dir /tmp/ntc_plain --reps 3 \
    > $O/plain_b.json 2> $O/plain_b.err || exit 1
for fb in 2 1 2 1; do
  NTC_FIRST_BATCH_BLOCKS=$fb timeout -k 10 120 python -u scripts/cli_timeline.py decode /tmp/ntc_plain/idx \
      /tmp/ntc_plain/enc.dat --reps 3 >> $O/timeline_decode_fb$fb.jsonl 2>&1 || exit 1
done
rm -rf /tmp/ntc_plain
