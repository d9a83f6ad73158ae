"""Development probe (GPU): the fast session's logits at the bench's parity positions 0 and 1 (after the 512-token
prompt, then after the first forced token) with the batched prefill and with the token loop (LLMI_NO_PREFILL),
each against the exact-order session (bit-identical to the reference).  Which path moves position 1?"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_inference_amd import _lib  # noqa: E402

_lib.lib()
from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

cfg = CONFIGS["gemma-3-4b"]
g = build_gemma3_gguf(cfg, seed=1234)
rng = np.random.default_rng(99)
prompt = np.concatenate([[2], rng.integers(4, cfg.vocab, 511)]).astype(np.int32)
forced = np.random.default_rng(2024).integers(4, cfg.vocab, 3).astype(np.int32)


def run(exact, no_prefill=False, twice=False):
    if no_prefill:
        os.environ["LLMI_NO_PREFILL"] = "1"
    else:
        os.environ.pop("LLMI_NO_PREFILL", None)
    m = Model(g, exact=exact, max_ctx=600)
    out = [m.forward(prompt, 0)]
    for i, t in enumerate(forced):
        out.append(m.forward(np.array([t], np.int32), len(prompt) + i))
    if twice:  # position 1 again on the same session
        out.append(m.forward(np.array([forced[0]], np.int32), len(prompt)))
    m.close()
    return out


ex = run(True)
for name, kw in [("fast, batched prefill", {}), ("fast, token loop", {"no_prefill": True}),
                 ("fast, batched prefill, pos 1 repeated", {"twice": True})]:
    f = run(False, **kw)
    d = [round(float(np.abs(a - b).max()), 4) for a, b in zip(f[:4], ex[:4])]
    extra = f" repeated pos 1: {float(np.abs(f[4] - ex[1]).max()):.4f}" if kw.get("twice") else ""
    print(f"{name}: per-position max |fast - exact| {d}{extra}", flush=True)
