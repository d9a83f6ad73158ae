#!/bin/bash
# per-geometry prefill GEMM times (rocprofv3 kernel trace of the 4B 512-token prefill)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for geo in ${GEOS}; do
  LLMI_PG5=$geo timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/geo_$geo -o run -- \
    python3 scripts/prefill_run.py gemma-3-4b 512 > gpurun_out/geo_$geo.log 2>&1 || exit $?
  python3 - $geo <<'PY'
import csv,sys
g=sys.argv[1]
rows=[r for r in csv.DictReader(open(f'gpurun_out/geo_{g}/run_kernel_trace.csv')) if 'prefill_gemm' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows]
print(g, [round(sum(d[136:][k::4])/len(d[136:][k::4]),1) for k in range(4)], rows[0]['Kernel_Name'][40:90])
PY
done
