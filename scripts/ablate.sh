#!/bin/bash
# In-graph per-family cost by ablation: each LLMI_DUP run launches one kernel
# family twice per token; (ms_per_step - base) is that family's cost per token.
# usage (on the GPU box): bash scripts/ablate.sh  -> gpurun_out/ablate.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ablate.log
: > "$out"
one() {  # label, env...
  local label=$1; shift
  local line
  line=$(env "$@" timeout -k 10 240 python bench.py --steps 128 --warmup 8 --no-cpu-baseline --kernel-reps 1 2>/dev/null | tail -1)
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label FAILED rc=$rc" | tee -a "$out"; exit $rc; fi
  echo "$label $(python -c 'import json,sys; d=json.loads(sys.argv[1]); print(d["ms_per_step"], d["config"]["kernels_per_token"])' "$line")" | tee -a "$out"
}
one fused LLMI_X=0
for k in qkv attn o_proj gate_up down logits; do one "fused+dup:$k" LLMI_DUP=$k; done
one unfused LLMI_NO_FUSE=1
for k in qkv norm gate_up gelu down; do one "unfused+dup:$k" LLMI_NO_FUSE=1 LLMI_DUP=$k; done
echo done | tee -a "$out"
