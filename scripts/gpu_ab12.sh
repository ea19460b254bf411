#!/bin/bash
# Round 6 A/B: k_ms4 (non-joint) with the run loop's query-word pair cache at 7 waves (cur)
# against 8 waves without it (A, the default) and 7 waves without it (B); GPU parity first
export TMPDIR=/tmp
O=${O:-gpurun_out/ab12}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workspace.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
OUT=$O/qc CONFIGS=encode,c31 VARIANTS="A B cur" REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh > $O/qc.log 2>&1 || exit 1
