#!/bin/bash
# k_ms4 / k_parse4 pipeline counters (encode config): address/data unit busy, TCP->L2 latency,
# wave wait and VMEM levels.  One pass per counter group, each within the per-block limits.
#   LIB=ntcomp_amd/libntcomp_gpu.so TAG=cur CFG=encode scripts/pmc_latency.sh
export TMPDIR=/tmp
CFG=${CFG:-encode}
TAG=${TAG:-cur}
OUT=gpurun_out/pmclat
mkdir -p $OUT
B="--configs $CFG --no-cpu --steps 3 --warmup 0 ${OPTS:-}"
run() {
  local name=$1; shift
  NTC_GPU_LIB=${LIB:-} timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k_ms4|k_parse4' --pmc "$@" \
      -d $OUT/${TAG}_$name -o $name --output-format csv -- python3 bench.py $B > $OUT/${TAG}_$name.out 2>&1 || exit 1
}
run ta TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
run tcp TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum
run sq SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VMEM
run rd TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum
