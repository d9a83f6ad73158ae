#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench (+ optional rocprof).  Every GPU
# step has its own time limit; after a fault/abort/timeout nothing else runs.
# usage: scripts/gpu_round.sh [tests] [smoke] [sweep] [ablate] [bench] [prof] [pmc]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
want() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
fatal() {  # exit codes that mean the GPU step crashed / hung
  case "$1" in 124|134|137|139|-6|-11) return 0 ;; *) return 1 ;; esac
}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL in $name: stopping"; exit $rc; fi
  return 0
}
want tests && run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v -rP -p no:cacheprovider --timeout 300 --timeout-method thread
want smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
want sweep && run gemv_sweep 300 scripts/gemv_sweep 200
want ablate && run ablate_run 900 bash scripts/ablate.sh
want bench && run bench 900 python bench.py
if want prof; then  # the timed decode graph itself (hipGraph replay), after a 512-token prefill
  run rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 64 --warmup 4 --prefill 512 --no-cpu-baseline
fi
if want pmc; then  # FETCH_SIZE of the launches the bench line times, 2 reps, at the position it ends on:
  # 784 = the default line (512 + 16 + 256), 537 = the driver's line (512 + 25 decode steps)
  for spec in "784 768 2 14" "537 512 5 20"; do
    set -- $spec
    run pmc_fetch_$1 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$1 -o run -- \
      python3 bench.py --prefill $2 --warmup $3 --steps $4 --no-cpu-baseline
    python3 scripts/pmc_summary.py gpurun_out/pmc_fetch_$1/run_counter_collection.csv \
      gpurun_out/pmc_fetch_summary_$1.json gemma-3-4b/q4_0/pos$1/reps2 68 > gpurun_out/pmc_summary_$1.log 2>&1
  done
fi
echo "== done"
