#!/bin/bash
# A/B of environment settings on the bench (development): alternates the
# settings R rounds, prints value per run.  usage: scripts/ab_env.sh R "ENV=a" "ENV=b" ... -- [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; shift
SETS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for r in $(seq 1 $R); do
  for s in "${SETS[@]}"; do
    env $s timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1 || { echo "FAIL $s"; tail -5 gpurun_out/ab.log; exit 1; }
    python3 - "$s" <<'PY'
import json,sys
l=[x for x in open("gpurun_out/ab.log") if x.startswith("{")][-1]
d=json.loads(l); kf=d.get("kernel_families",{})
print(f"{sys.argv[1]:40s} {d['value']:8.1f} tok/s  " + " ".join(f"{k}={v['us_per_launch']:.2f}" for k,v in kf.items()), flush=True)
PY
  done
done
