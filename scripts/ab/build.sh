#!/bin/bash
# build the attention A/B tool (development): current k_attn.hip vs scripts/ab/k_attn_old.hip,
# both WITHOUT the phase-trace marks (they cost ~1 us per launch); scripts/ab/attn_trace is the
# traced build of the current version (phase table only).
set -e
cd "$(dirname "$0")/../.."
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Illm_inference_amd/csrc"
$H -c llm_inference_amd/csrc/k_attn.hip -o /tmp/ab_cur.o
$H -DLLMI_ATTN_TRACE -c llm_inference_amd/csrc/k_attn.hip -o /tmp/ab_cur_tr.o
$H -Dllmi=llmi_old -x hip -c scripts/ab/k_attn_old.hip -o /tmp/ab_old.o
$H -c scripts/ab/attn_bench.hip -o /tmp/ab_main.o
$H -DLLMI_ATTN_TRACE -c scripts/ab/attn_bench.hip -o /tmp/ab_main_tr.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/ab_main.o /tmp/ab_cur.o /tmp/ab_old.o -o scripts/ab/attn_bench
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/ab_main_tr.o /tmp/ab_cur_tr.o /tmp/ab_old.o -o scripts/ab/attn_trace
