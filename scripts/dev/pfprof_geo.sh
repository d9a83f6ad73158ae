#!/bin/bash
# per-GEMM prefill kernel times (rocprofv3 kernel trace of scripts/prefill_run.py) under several environment
# settings (development A/B of the GEMM geometries).  usage: scripts/dev/pfprof_geo.sh "ENV=a" "ENV=b" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
i=0
for e in "$@"; do
  i=$((i+1)); echo "#### $e"
  env $e PP_TAG=_$i scripts/dev/prof_prefill.sh llm_inference_amd/libllmi.so || exit 1
done
