#!/bin/bash
# A/B arms with SQ counters (one rocprofv3 --pmc pass per arm; no traces).
# arm = "ENV=val ENV2=val|bench args"  (env part optional; e.g. NTC_GPU_LIB=ntcomp_amd/ab/libX.so)
set -u
OUT=gpurun_out/ab; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for arm in "$@"; do
  i=$((i+1))
  envs=""; args="$arm"
  case "$arm" in *"|"*) envs="${arm%%|*}"; args="${arm#*|}";; esac
  (
    for kv in $envs; do export "$kv"; done
    timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --warmup 1 $args > $OUT/arm$i.json 2> $OUT/arm$i.err || exit $?
    timeout -k 10 300 rocprofv3 --kernel-include-regex 'k_ms4|k_parse4|k_pack' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/pmc$i -o pmc --output-format csv -- python3 bench.py --no-cpu --steps 1 --warmup 0 $args > /dev/null 2> $OUT/pmc$i.err || exit $?
    timeout -k 10 300 rocprofv3 --kernel-include-regex 'k_ms4|k_parse4' --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $OUT/tcc$i -o t --output-format csv -- python3 bench.py --no-cpu --steps 1 --warmup 0 $args > /dev/null 2> $OUT/tcc$i.err || exit $?
  ) || exit $?
  echo "arm$i [$arm]: $(cat $OUT/arm$i.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step"])')"
done
