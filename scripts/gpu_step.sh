#!/bin/bash
# Run GPU steps in order; each under its own time limit.  A step that crashes, aborts or
# times out (exit 124/134/137/139 or >128) ends the session: nothing else touches the GPU.
# A plain failure (e.g. pytest rc=1) is recorded and the next step still runs.
# usage: scripts/gpu_step.sh "<seconds>|<name>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  rc=$?
  echo "=== $name rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.out" | sed "s/^/[$name] /"
  if [ $rc -ge 124 ] && [ $rc -ne 0 ]; then
    echo "=== stopping: $name ended with rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
