"""Summarise a layer-engine phase trace (development).

    LLMI_BLOCK_TRACE_BUILD=1 python -m llm_inference_amd.build --force   # marks compiled in (libllmi_trace.so)
    LLMI_LIB=llm_inference_amd/libllmi_trace.so LLMI_BLOCK_TRACE=<layer> LLMI_BLOCK_TRACE_OUT=f.bin \
        python bench.py --steps 8 --warmup 2 --no-cpu-baseline
    python scripts/engine_trace.py f.bin [n_attention_cus]

Each sync appends one record of 4096 x 8 u64; the engine uses [CU][16] of it.
Phases (wall clock, 100 MHz, us from the first CU's start): 0 start, 1 x in LDS, 2 qkv rows published,
3 q/k/v rows in (attention CUs), 4 attention done (partial / merge published), 5 merged blocks in,
6 o rows published, 7 x2 in LDS, 8 hid published, 9 hid in LDS (+ down weights landed), 10 end;
11 P1's first reduction, 12 qkv products staged, 13 o swept into LDS, 14 gate_up products staged, 15 gate_up rows.
"""
import sys

import numpy as np

NAMES = ["start", "x", "qkv_pub", "qkv_in", "attn_done", "xo_in", "o_pub", "x2", "hid_pub", "hid_in", "end",
         "p1_sum1", "p2_dots", "o_in", "p6_dots", "p6_rows"]
path = sys.argv[1]
na = int(sys.argv[2]) if len(sys.argv) > 2 else 128
raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 4096 * 8)
for rec in raw[-3:]:
    t = rec[: 256 * 16].reshape(256, 16)[:, : len(NAMES)].astype(np.float64)
    t0 = t[:, 0][t[:, 0] > 0].min()
    rel = np.where(t > 0, (t - t0) / 100.0, np.nan)
    print(f"span {np.nanmax(rel):.2f} us")
    for ph in sorted(range(len(NAMES)), key=lambda p: np.nanmean(rel[:, p]) if np.isfinite(rel[:, p]).any() else 1e9):
        name = NAMES[ph]
        v = rel[:, ph] if ph not in (3, 4) else rel[:na, ph]
        if np.isfinite(v).any():
            print(f"  {ph:2d} {name:9s} min {np.nanmin(v):6.2f}  mean {np.nanmean(v):6.2f}  max {np.nanmax(v):6.2f}")
