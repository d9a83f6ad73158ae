#!/bin/bash
# token-selection geometry sweep on the bench's own timing (time_kernel 2: prep + screening GEMV + rescoring)
# usage: scripts/screen_sweep.sh  -> gpurun_out/screen_sweep.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/screen_sweep.txt
: > $out
for wpc in 8 4 12 16; do
  for ahead in 2 1; do
    LLMI_SCREEN_WPC=$wpc LLMI_SCREEN_AHEAD=$ahead timeout -k 10 200 python bench.py --steps 64 --warmup 4 \
      --no-cpu-baseline > gpurun_out/ss.log 2>&1 || exit $?
    python3 - "$wpc" "$ahead" >> $out <<'PY'
import json, sys
l = [x for x in open("gpurun_out/ss.log") if x.startswith("{")][-1]
d = json.loads(l)
print("wpc", sys.argv[1], "ahead", sys.argv[2], "tok/s", d["value"], "token_selection_us",
      d["kernel_families"]["token_selection"]["us_per_launch"], flush=True)
PY
    tail -1 $out
  done
done
