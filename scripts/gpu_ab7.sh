#!/bin/bash
# Round 6 A/B: fused parse + emit (k_parse4e, cur) against k_parse4 + scan + k_emit4 (A); GPU suite first
export TMPDIR=/tmp
O=${O:-gpurun_out/ab7}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
OUT=$O/fused CONFIGS=c31,encode,strains VARIANTS="A cur" REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh > $O/fused.log 2>&1 || exit 1
