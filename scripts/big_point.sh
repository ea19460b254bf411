#!/bin/bash
# Large-collection throughput point: the 3.0 Gbp / ~177 M-node k = 31
# collection of scripts/big_build.py, 10 M reads encoded in one call, bit-exact on an oracle
# sample and decoded back; then rocprofv3 passes over the same command for k_ms4's requests
# per read (separate PMC passes, never combined with other traces) and its kernel time.
#   OUT=gpurun_out/big scripts/big_point.sh
set -u
OUT=${OUT:-gpurun_out/big}
ARGS=${ARGS:-"--reads 10000000"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/big_build.py $ARGS --reps 3 > "$OUT/point.json" 2> "$OUT/point.err" || exit $?
KRE='k_ms4|k_parse4|k_pack|k_emit4'
timeout -k 10 300 rocprofv3 --kernel-include-regex "$KRE" --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
    TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d "$OUT/pmc_rd" -o pmc_rd --output-format csv -- \
    python3 scripts/big_build.py $ARGS --reps 1 --no-check > "$OUT/pmc_rd.stdout" 2> "$OUT/pmc_rd.stderr" || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex "$KRE" --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    TCC_EA0_RDREQ_DRAM_32B_sum TCC_BUBBLE_sum -d "$OUT/pmc_wr" -o pmc_wr --output-format csv -- \
    python3 scripts/big_build.py $ARGS --reps 1 --no-check > "$OUT/pmc_wr.stdout" 2> "$OUT/pmc_wr.stderr" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 scripts/big_build.py $ARGS --reps 3 --no-check > "$OUT/kt.stdout" 2> "$OUT/kt.stderr" || exit $?
echo "=== done" >&2
