"""Per-kernel means of the counters in a rocprofv3 --pmc counter_collection.csv (development).
usage: python scripts/dev/pmc_kernels.py <counter_collection.csv> [kernel-substring ...]"""
import csv
import sys
from collections import defaultdict

path, keys = sys.argv[1], sys.argv[2:]
per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if keys and not any(k in name for k in keys):
        continue
    per[(name, r.get("Dispatch_Id", "0"))][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(list))
for (name, _), cs in per.items():
    for c, v in cs.items():
        agg[name][c].append(v)
for name, cs in sorted(agg.items(), key=lambda kv: -sum(sum(v) for v in kv[1].values())):
    n = len(next(iter(cs.values())))
    print(f"{name[:100]}  ({n} dispatches)")
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.1f}")
