#!/bin/bash
# Round 6 final check of the committed tree: the GPU suite, smoke and the default bench line
export TMPDIR=/tmp
O=${O:-gpurun_out/final6c}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
