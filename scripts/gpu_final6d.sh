#!/bin/bash
# Round 6 final (query-word cache build): the GPU suite, smoke, the default bench line, then the
# rocprofv3 kernel trace + PMC passes of the same build (scripts/profile_bench.sh)
export TMPDIR=/tmp
O=${O:-gpurun_out/final6d}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_pre.json 2> $O/bench_pre.err || exit 1
OUT=$O/prof TAG=r06 timeout -k 10 900 bash scripts/profile_bench.sh > $O/prof.log 2>&1 || exit 1
