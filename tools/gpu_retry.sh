#!/bin/bash
# Retry a gpurun call (from the main checkout) while the pool has no box (exit 3)
# or the infrastructure reports a transient failure. Never retries a call whose
# command ran (any other status): that result is final.
# usage: bash tools/gpu_retry.sh OUTFILE 'command'
out=$1; shift
for i in $(seq 1 ${RETRIES:-20}); do
  (cd /root/repo && timeout 1700 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@") > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" "$out" && ! grep -q "status=ok" "$out"; then
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
