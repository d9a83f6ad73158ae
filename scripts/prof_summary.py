"""Print the top kernels of a rocprofv3 --stats kernel summary (CSV)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6} avg={float(r['AverageNs'])/1e3:8.2f}us "
          f"min={float(r['MinNs'])/1e3:7.2f} max={float(r['MaxNs'])/1e3:8.2f} pct={float(r['TotalDurationNs'])/tot*100:5.1f}")
