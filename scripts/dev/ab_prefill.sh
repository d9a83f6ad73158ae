#!/bin/bash
# A/B of the batched prefill: the tree's libllmi.so against ab/libllmi_old.so, alternating
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do
  for L in llm_inference_amd/libllmi.so ab/libllmi_old.so; do
    echo "== $L"; LLMI_LIB=$L timeout -k 10 200 python scripts/prefill_run.py ${1:-gemma-3-4b} ${2:-512} 2>&1 | tail -2
  done
done
