#!/bin/bash
# rocprofv3 evidence for the bench command (run on the GPU box via gpurun).
#   1) kernel trace + stats of the default bench command
#   2) separate PMC passes (FETCH_SIZE / WRITE_SIZE / TCC hit-miss / SQ) -- never combined
#      with sys/runtime traces (gpurun policy; MI355X_MICROARCH.md "rocprofv3 PMC slots")
set -u
OUT=${OUT:-gpurun_out/prof}
MODE=${MODE:-encode}
BENCH="bench.py --mode $MODE"
KRE=${KRE:-'k_encode|k_ms4|k_parse4|k_pack|k_emit4|k_dec_rec|k_dec_reduce|k_dec_apply|k_dec_expand'}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name, limit, rocprof args...
  local name=$1 secs=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$secs" rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
      python3 $BENCH ${BENCH_ARGS:-} > "$OUT/$name.stdout" 2> "$OUT/$name.stderr"
  local rc=$?
  echo "=== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.stderr" >&2; exit $rc; fi
}
PASSES=${PASSES:-"kt fetch write tcc sq grbm"}
has() { case " $PASSES " in *" $1 "*) return 0;; esac; return 1; }
has kt && run kt 420 --kernel-trace --stats
BENCH_ARGS="--no-cpu --steps 2 --warmup 0"
has fetch && run pmc_fetch 300 --kernel-include-regex "$KRE" --pmc FETCH_SIZE
has write && run pmc_write 300 --kernel-include-regex "$KRE" --pmc WRITE_SIZE
has tcc && run pmc_tcc 300 --kernel-include-regex "$KRE" --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
has sq && run pmc_sq 300 --kernel-include-regex "$KRE" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
has grbm && run pmc_grbm 300 --kernel-include-regex "$KRE" --pmc GRBM_GUI_ACTIVE GRBM_COUNT
echo done >&2
