#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in _x _nodma _nocomp; do
  LLMI_LIB=llm_inference_amd/libllmi$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fl$lib -o run -- \
    python3 scripts/prefill_run.py gemma-3-4b 512 > gpurun_out/fl$lib.log 2>&1 || exit $?
  echo "== $lib"
  python3 - $lib <<'PY'
import csv,sys
rows=[r for r in csv.DictReader(open(f'gpurun_out/fl{sys.argv[1]}/run_kernel_trace.csv')) if 'prefill_gemm' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows]
for k in range(4):
    xs=d[136:][k::4]; r=rows[k]
    print(k, round(sum(xs)/len(xs),1), r['Grid_Size_X'], r['Kernel_Name'][40:100])
PY
done
