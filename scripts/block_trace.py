"""Summarise an attention-block phase trace (development).

    LLMI_BLOCK_TRACE_BUILD=1 python -m llm_inference_amd.build --force   # marks compiled in
    LLMI_BLOCK_TRACE=<layer> LLMI_BLOCK_TRACE_OUT=f.bin python bench.py ...
    (layer 1000 + l traces layer l's MLP block)
    python scripts/block_trace.py f.bin NQ NA NO

Each sync appends one record of 4096 work-groups x 8 wall clocks (100 MHz).
Roles by work-group index: [0, NQ) qkv, [NQ, NQ+NA) attention, then NO o.
Phases -- qkv/o: 0 start, 4 wait done (o), [PRO: 5 first norm's operands in, 6 first
reduction done, 7 second reduction done], 1 x in LDS, 2 rows done, 3 end;
attention: 0 start, 1 wait done, 2 rows + prologue done, 3 partial published,
4 merge published (merging work-groups only).  Times in us from the first start.
"""
import sys

import numpy as np

path, nq, na, no = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
names = sys.argv[5].split(",") if len(sys.argv) > 5 else ["qkv", "attn", "o"]  # MLP block: gate_up,-,down
raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 4096, 8)
for rec in raw[-3:]:
    t = rec[: nq + na + no].astype(np.float64)
    t0 = t[:, 0][t[:, 0] > 0].min()
    rel = np.where(t > 0, (t - t0) / 100.0, np.nan)
    print(f"span {np.nanmax(rel):.2f} us")
    for name, a, b in ((names[0], 0, nq), (names[1], nq, nq + na), (names[2], nq + na, nq + na + no)):
        if b <= a:
            continue
        r = rel[a:b]
        cols = []
        for ph in range(8):
            v = r[:, ph]
            if np.isfinite(v).any():
                cols.append(f"p{ph} {np.nanmean(v):6.2f}/{np.nanmax(v):6.2f}")
        print(f"  {name:5s} (mean/max) " + "  ".join(cols))
