#!/bin/bash
# prefill GEMM v5 A/B on the GPU box: prefill tests, then 512-token 4B prefill times per geometry / build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_prefill.py -m gpu -x -q -s -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pg5_tests.log 2>&1
rc=$?; grep -E "v5|passed|failed|Error|error" gpurun_out/pg5_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
for lib in "" llm_inference_amd/libllmi_noslp.so llm_inference_amd/libllmi_mix.so; do
  echo "== lib=${lib:-default}"
  LLMI_LIB=$lib timeout -k 10 120 python scripts/prefill_run.py gemma-3-4b 512 2>&1 | tail -1 || exit $?
  for geo in ${GEOS:-}; do
    echo "   geo $geo (all GEMMs)"
    LLMI_LIB=$lib LLMI_PG5=$geo timeout -k 10 120 python scripts/prefill_run.py gemma-3-4b 512 2>&1 | tail -1 || exit $?
  done
done
LLMI_LIB=${PROF_LIB:-} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pg5prof -o run -- \
  python3 scripts/prefill_run.py gemma-3-4b 512 > gpurun_out/pg5prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/pg5prof/run_kernel_trace.csv')) if 'prefill_gemm' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows]
for k in range(4):
    xs=d[136:][k::4]; r=rows[k]
    print(k, round(sum(xs)/len(xs),1), r['Grid_Size_X'], r['Kernel_Name'][40:100])
PY
echo done
