"""Per-projection durations of the batched prefill GEMMs from a rocprofv3
kernel trace (dispatch order per layer: qkv, o, gate_up, down).
usage: python scripts/prefill_trace_summary.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "prefill_gemm" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = ["qkv", "o", "gate_up", "down"]
acc = defaultdict(list)
for i, r in enumerate(rows):
    acc[names[i % 4]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for k in names:
    v = acc[k]
    print(f"{k:8s} n={len(v):4d} mean {sum(v) / len(v):8.2f} us  min {min(v):8.2f}")
other = defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    other[r["Kernel_Name"][:60]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, v in sorted(other.items(), key=lambda kv: -kv[1])[:8]:
    print(f"{k:60s} {v:8.2f} ms total")
