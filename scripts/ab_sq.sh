#!/bin/bash
# A/B of bench options with SQ counters (one rocprofv3 --pmc pass per arm; no traces).
set -u
OUT=gpurun_out/ab; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for arm in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --warmup 1 $arm > $OUT/arm$i.json 2> $OUT/arm$i.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-include-regex 'k_ms4|k_parse4|k_pack' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/pmc$i -o pmc --output-format csv -- python3 bench.py --no-cpu --steps 1 --warmup 0 $arm > /dev/null 2> $OUT/pmc$i.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-include-regex 'k_ms4' --pmc FETCH_SIZE -d $OUT/fetch$i -o f --output-format csv -- python3 bench.py --no-cpu --steps 1 --warmup 0 $arm > /dev/null 2> $OUT/fetch$i.err || exit $?
  echo "arm$i [$arm]: $(cat $OUT/arm$i.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step"])')"
done
