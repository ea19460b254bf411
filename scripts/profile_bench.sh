#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box through gpurun):
#   kt        kernel trace + stats of the default bench command (all configs, as the driver runs it)
#   pmc_*     separate counter passes per workload, each within the per-block slot limits
#             (<= 4 TCC counters, <= 8 SQ, <= 2 GRBM), never combined with other traces.
# Then scripts/pmc_traffic.py turns them into profiles/pmc_traffic.json + a markdown summary.
#   OUT=gpurun_out/prof TAG=r02 scripts/profile_bench.sh
set -u
OUT=${OUT:-gpurun_out/prof}
TAG=${TAG:-r02}
KRE=${KRE:-'k_ms4|k_parse4|k_pack|k_emit4|k_dec_rec|k_dec_tiles'}
BENCH_KT=${BENCH_KT:-"--steps 20 --warmup 5"}
WORKLOADS=${WORKLOADS:-"encode decode c31 strains"}
PASSES=${PASSES:-"kt rd wr misc"}
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { case " $PASSES " in *" $1 "*) return 0;; esac; return 1; }
run() {  # name, limit, bench args, rocprof args...
  local name=$1 secs=$2 bargs=$3; shift 3
  echo "=== $name ($(date +%T))" >&2
  timeout -k 10 "$secs" rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
      python3 bench.py $bargs > "$OUT/$name.stdout" 2> "$OUT/$name.stderr"
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))" >&2
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.stderr" >&2; exit $rc; fi
}
has kt && run kt 600 "$BENCH_KT" --kernel-trace --stats
for w in $WORKLOADS; do
  B="--configs $w --no-cpu --steps 3 --warmup 0"
  has rd && run "pmc_rd_$w" 240 "$B" --kernel-include-regex "$KRE" \
      --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  has wr && run "pmc_wr_$w" 240 "$B" --kernel-include-regex "$KRE" \
      --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_BUBBLE_sum
  has misc && run "pmc_misc_$w" 240 "$B" --kernel-include-regex "$KRE" \
      --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
done
echo "=== done" >&2
