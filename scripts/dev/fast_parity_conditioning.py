"""Conditioning of the bench's parity positions (CPU, development): the reference restatement (oracle, test
infrastructure) with its f16 attention accumulator against the same with f64 attention, on bench.py's own model
(gemma-3-4b Q4_0 synthetic, seed 1234), prompt (rng 99, 512 tokens) and 8 forced tokens (rng 2024).  A large
difference at a position says the reference's own output there is ill-conditioned (an fp32-class device path
lands anywhere within that spread), bench.py's parity_vs_reference.fast per-position numbers read against it."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402
from oracle.bind import Oracle, build  # noqa: E402


def main():
    cfg = CONFIGS["gemma-3-4b"]
    g = build_gemma3_gguf(cfg, seed=1234)
    rng = np.random.default_rng(99)
    prompt = np.concatenate([[2], rng.integers(4, cfg.vocab, 511)]).astype(np.int32)
    forced = np.random.default_rng(2024).integers(4, cfg.vocab, 8).astype(np.int32)
    build(ref=False)
    orc = Oracle()
    nt = int(os.environ.get("THREADS", "8"))
    out = {}
    for f64 in (False, True):
        t0 = time.time()
        m = orc.model(g, n_threads=nt, max_ctx=544, attn_f64=f64)
        lg = [m.forward(prompt, 0)]
        for i, t in enumerate(forced):
            lg.append(m.forward(np.array([t], np.int32), len(prompt) + i))
        out[f64] = np.stack(lg)
        print(f"attn_f64={f64}: {time.time() - t0:.0f} s", flush=True)
    d = [round(float(np.abs(a - b).max()), 4) for a, b in zip(out[False], out[True])]
    print("per-position max |reference - reference with f64 attention|:", d)
    print("max |reference logit|:", float(np.abs(out[False]).max()))


if __name__ == "__main__":
    main()
