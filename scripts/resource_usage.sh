#!/bin/bash
# VGPR / spill / occupancy per kernel of one HIP source (compile-time remarks).
# usage: scripts/resource_usage.sh llm_inference_amd/csrc/k_layer.hip [filter]
src=${1:?source}
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I"$OLDPWD/include" \
  -c "$OLDPWD/$src" -o /tmp/_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys, subprocess
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}; rows.append(cur); continue
    for key in ("VGPRs", "AGPRs", "ScratchSize", "Occupancy", "VGPRs Spill", "SGPRs Spill", "LDS Size"):
        m = re.search(r"\s" + re.escape(key) + r"(?: \[[^\]]*\])?: (\d+)", line)
        if m and cur is not None and key not in cur:
            cur[key] = m.group(1)
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r, d in zip(rows, dem):
    if flt in d:
        print("%-110s vgpr=%s spill=%s occ=%s scratch=%s" % (d[:110], r.get("VGPRs"), r.get("VGPRs Spill"), r.get("Occupancy"), r.get("ScratchSize")))
' "${2:-}"
