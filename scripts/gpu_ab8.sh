#!/bin/bash
# Round 6 A/B: k_parse4 with a block's reads sorted by entry count (cur: 8 waves, C: 7 waves)
# against batch order (A); GPU parity of cur first
export TMPDIR=/tmp
O=${O:-gpurun_out/ab8}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workspace.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
OUT=$O/sort CONFIGS=c31,encode,strains VARIANTS="A cur C" REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh > $O/sort.log 2>&1 || exit 1
