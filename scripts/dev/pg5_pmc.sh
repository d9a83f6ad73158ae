#!/bin/bash
# SQ / TCC counters of the prefill GEMMs (one rocprofv3 --pmc pass per counter group)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
while read -r ctrs; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc/p$i -o run -- \
    python3 scripts/prefill_run.py gemma-3-4b 512 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  python3 scripts/pmc_table.py gpurun_out/pmc/p$i/run_counter_collection.csv --match=gemm
done <<'LIST'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC
SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVES
TCC_HIT_sum TCC_MISS_sum
LIST
echo done
