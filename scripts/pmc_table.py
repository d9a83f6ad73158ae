"""Mean of every collected counter per kernel from rocprofv3 --pmc CSVs.

usage: python scripts/pmc_table.py <counter_collection.csv> [more.csv ...] [--match SUBSTR]
"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--match")]
match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "")
acc = defaultdict(lambda: defaultdict(list))
for path in args:
    for r in csv.DictReader(open(path)):
        if match and match not in r["Kernel_Name"]:
            continue
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    print(name[:150])
    print("   " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
