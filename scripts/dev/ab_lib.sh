#!/bin/bash
# Development: same-box A/B of two builds on the default bench line, alternating (A B A B).
# usage: ab_lib.sh llm_inference_amd/libllmi_<variant>.so [bench args...]
set -u
alt=$1; shift
for i in 1 2; do
  for lib in "" "$alt"; do
    LLMI_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_run.json || exit $?
    echo "${lib:-default} $(grep -o '"value": [0-9.]*' gpurun_out/ab_run.json)"
  done
done
