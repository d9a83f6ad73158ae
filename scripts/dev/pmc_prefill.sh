#!/bin/bash
# SQ counters of the prefill GEMMs (one rocprofv3 --pmc pass per setting; development)
# usage: scripts/dev/pmc_prefill.sh "ENV=a" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1)); echo "#### $e"
  d=/tmp/pmc_pf_$i
  env $e timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $d -o run -- python3 scripts/prefill_run.py gemma-3-4b 512 > gpurun_out/pmc_pf_$i.log 2>&1
  rc=$?
  f=$(find $d -name '*counter_collection.csv' | head -1)
  if [ -z "$f" ]; then echo "rc=$rc, no counter file"; tail -20 gpurun_out/pmc_pf_$i.log; exit 1; fi
  python3 scripts/dev/pmc_kernels.py "$f" gemm
done
