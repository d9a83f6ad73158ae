#!/bin/bash
# quick GPU iteration: selected GPU tests, a bench line, an attention-block trace
# usage: scripts/gpu_quick.sh "<pytest -k expr or test files>" [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="$1"; shift
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/quick_tests.log 2>&1
  rc=$?; tail -n 5 gpurun_out/quick_tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/quick_bench.log 2>&1 || exit $?
python - <<'PY'
import json
l=[x for x in open("gpurun_out/quick_bench.log") if x.startswith("{")][-1]
d=json.loads(l); print("value", d["value"], "ms", d["ms_per_step"])
for k,v in d.get("kernel_families",{}).items(): print(" ", k, v["us_per_launch"], v["frac"])
PY
if [ -f llm_inference_amd/libllmi_trace.so ]; then
  rm -f gpurun_out/bt.bin
  LLMI_LIB=llm_inference_amd/libllmi_trace.so LLMI_BLOCK_TRACE=5 LLMI_BLOCK_TRACE_OUT=gpurun_out/bt.bin \
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bt.log 2>&1 || exit $?
  python scripts/block_trace.py gpurun_out/bt.bin 256 128 80 | head -4
fi
