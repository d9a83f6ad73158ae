#!/bin/bash
# gpurun with waits for a free box: exit code 3 (no box / slot free: nothing ran, nothing charged) -> wait and
# ask again, up to 10 times; any other outcome (including a failed GPU step) is returned as is.
# usage: scripts/gpu_try.sh <gpurun args...>
for i in $(seq 1 10); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpu_try] no box free (attempt $i); waiting" >&2
  sleep 120
done
exit 3
