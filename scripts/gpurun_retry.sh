#!/bin/bash
# gpurun with a retry when the box fails to come up (infrastructure "transient" status or
# exit 3 = no slot).  Never retries a command that ran (its result stands).
for attempt in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | tail -40
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then
    echo "[retry] transient/no-slot (rc=$rc), attempt $attempt; sleeping 40s" >&2
    sleep 40
    continue
  fi
  exit $rc
done
exit 3
