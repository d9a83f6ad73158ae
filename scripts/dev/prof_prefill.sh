#!/bin/bash
# per-GEMM prefill kernel times of several builds (rocprofv3 kernel trace of scripts/prefill_run.py)
# usage: scripts/dev/prof_prefill.sh lib1.so [lib2.so ...]
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in "$@"; do
  n=$(basename "$L" .so)${PP_TAG:-}
  echo "== $L"
  LLMI_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pp_$n -o run -- python3 scripts/prefill_run.py > gpurun_out/pp_$n.log 2>&1
  grep "^prefill" gpurun_out/pp_$n.log | tail -1
  python3 scripts/prefill_trace_summary.py $(find gpurun_out/pp_$n -name '*kernel_trace.csv' | head -1)
done
