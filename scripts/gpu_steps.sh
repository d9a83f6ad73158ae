#!/bin/bash
# GPU-box steps, each under its own time limit; after a fault / abort / timeout nothing else runs.
# usage: scripts/gpu_steps.sh 'name|seconds|command' ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($(date +%T)): $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "FATAL in $name: stopping"; exit $rc ;; esac
done
