#!/bin/bash
# bench lines of the other BASELINE configs (one GPU) -> gpurun_out/configs.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
for args in "--config gemma-3-1b" "--config gemma-3-1b --quant q8_0" "--quant q4_k_m" "--config gemma-3-27b --steps 64" \
            "--full-logits" "--prefill 2048" "--exact --steps 32 --warmup 4"; do
  timeout -k 10 400 python bench.py --no-cpu-baseline $args > gpurun_out/cfg.log 2>&1 || { echo "FAIL $args"; tail -3 gpurun_out/cfg.log; exit 1; }
  tail -1 gpurun_out/cfg.log >> gpurun_out/configs.jsonl
  python3 - "$args" <<'PY'
import json,sys
d=json.loads(open("gpurun_out/configs.jsonl").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} {d['value']:8.1f} tok/s  prefill {d['timing_detail'].get('prefill_s')} s  {d['config']['workload'][:60]}", flush=True)
PY
done
