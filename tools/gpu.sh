#!/bin/bash
# gpurun with retries ONLY for infrastructure-side failures (no box / box lost while being prepared,
# nothing ran, nothing charged).  A command that ran and failed is never retried.
# Usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4; do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun.out 2>&1
  rc=$?
  grep "status=" /tmp/gpurun.out
  if grep -q "status=transient\|backing off" /tmp/gpurun.out || [ $rc -eq 3 ]; then
    sleep 60
    continue
  fi
  tail -n 5 /tmp/gpurun.out | grep -v "^\[gpurun\] status"
  exit $rc
done
exit 3
