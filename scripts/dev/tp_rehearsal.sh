#!/bin/bash
# Development: bench.py --gpus 2 with both ranks on the box's one GPU (LLMI_BENCH_ONE_DEVICE=1), the fused
# exchange (default) and the standalone exchange launches (LLMI_TP_FUSED=0); usage: tp_rehearsal.sh CONFIG PORT
set -u
cfg=${1:-gemma-3-4b}
port=${2:-29531}
export LLMI_BENCH_ONE_DEVICE=1
for fused in 1 0; do
  LLMI_TP_FUSED=$fused timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((port + fused)) bench.py --gpus 2 --config "$cfg" --steps 32 --warmup 4 \
    --prefill 64 --no-cpu-baseline || exit $?
done
