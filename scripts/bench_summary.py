"""One line per bench log: tok/s and the kernel families' per-launch microseconds.
usage: python scripts/bench_summary.py gpurun_out/a.log [gpurun_out/b.log ...]"""
import json
import sys

for p in sys.argv[1:]:
    try:
        line = [x for x in open(p) if x.startswith("{")][-1]
    except (OSError, IndexError):
        print(f"{p}: no bench line")
        continue
    d = json.loads(line)
    fam = {k: v["us_per_launch"] for k, v in d.get("kernel_families", {}).items()}
    ex = d.get("exact", {})
    print(f"{p}: {d['value']} tok/s ({d['ms_per_step']} ms)", fam,
          f"exact {ex.get('value')} tok/s prefill {ex.get('prefill_s')} / warm {ex.get('prefill_warm_s')} s" if ex else "",
          f"prefill {d['timing_detail']['prefill_s']} / warm {d['timing_detail'].get('prefill_warm_s')} s")
