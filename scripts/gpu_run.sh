#!/bin/bash
# Ad-hoc GPU-box steps with the gpu_round.sh safety rules: each step under its
# own time limit, output to gpurun_out/<name>.log (tail echoed), and nothing
# more on the GPU after a crash / abort / timeout (a failing test does not
# stop later steps).
# usage: scripts/gpu_run.sh 'name|seconds|command' ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%|*}
  rest=${step#*|}
  t=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 12 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "FATAL in $name: stopping"; exit $rc ;; esac
done
echo "== done"
