#!/bin/bash
# Round 6 A/B: k_parse4 with deferred S loads (cur) against inline (A); GPU parity first
export TMPDIR=/tmp
O=${O:-gpurun_out/ab6}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workspace.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
OUT=$O/defer CONFIGS=c31,encode,strains VARIANTS="A cur" REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh > $O/defer.log 2>&1 || exit 1
