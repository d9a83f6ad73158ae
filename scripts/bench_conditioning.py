"""The reference's own conditioning on bench.py's parity inputs (CPU; test infrastructure).

bench.py's fast-path parity bound per position is FAST_ABS + FAST_SPREAD x s_p, with s_p = the reference's distance
from the same computation with f64 attention at position p.  Computing s_p takes two runs of the oracle
restatement (pinned bit for bit to the reference, tests/test_oracle_golden.py) over the bench's 512-token prompt --
minutes of CPU, too long for every bench run -- so it is computed here once per workload and committed as
tests/golden/bench_conditioning.json, keyed like bench.py's parity_key(): model / weights / prompt length.

    python scripts/bench_conditioning.py [--config gemma-3-4b] [--quant q4_0] [--prefill 512] [--threads 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "bench_conditioning.json")


def main():
    import bench
    from llm_inference_amd.gguf import TensorType as TT
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    from oracle.bind import Oracle, build
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="gemma-3-4b")
    p.add_argument("--quant", default="q4_0")
    p.add_argument("--prefill", type=int, default=512)
    p.add_argument("--threads", type=int, default=8)
    a = p.parse_args()
    cfg = CONFIGS[a.config]
    qkw = {"q4_0": {}, "q4_k_m": dict(wtype=TT.Q4_K, wtypes={"v": TT.Q6_K, "down": TT.Q6_K}),
           "q8_0": dict(wtype=TT.Q8_0)}[a.quant]
    g = build_gemma3_gguf(cfg, seed=1234, **qkw)
    prompt = bench.bench_prompt(cfg, a.prefill)
    forced = bench.forced_tokens(cfg.vocab)
    build(ref=False)
    orc = Oracle()
    runs = {}
    for f64 in (False, True):
        t0 = time.time()
        m = orc.model(g, n_threads=a.threads, max_ctx=a.prefill + bench.FORCED + 8, attn_f64=f64)
        lg = [m.forward(prompt, 0)]
        for i, t in enumerate(forced):
            lg.append(m.forward(np.array([t], np.int32), len(prompt) + i))
        runs[f64] = np.stack(lg)
        del m
        print(f"attn_f64={f64}: {time.time() - t0:.0f} s", flush=True)
    spread = [float(np.abs(x - y).max()) for x, y in zip(runs[False], runs[True])]
    d = json.load(open(OUT)) if os.path.exists(OUT) else {}
    d[bench.parity_key(a.config, a.quant, a.prefill)] = {
        "spread_per_position": spread, "max_abs_reference_logit": float(np.abs(runs[False]).max()),
        "reference_argmax": [int(v) for v in runs[False].argmax(1)],
        "how": "max over the vocabulary of |oracle (= reference, bit for bit) - oracle with f64 attention| at each "
               "of the prompt's last position and the FORCED teacher-forced positions (scripts/bench_conditioning.py)"}
    json.dump(d, open(OUT, "w"), indent=1)
    print("spread per position:", [round(s, 4) for s in spread])


if __name__ == "__main__":
    main()
