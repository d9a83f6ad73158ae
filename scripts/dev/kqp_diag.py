"""K-quant batched prefill (int8, Q8_K blocks) vs the token loop on mini-4b, several seeds / lengths (development)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from llm_inference_amd.gguf import TensorType as TT  # noqa: E402
from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

cfg = CONFIGS["mini-4b"]
for seed, n, wt in ((33, 150, "kq"), (33, 20, "kq"), (33, 5, "kq"), (34, 150, "kq"), (33, 150, "q4_0"), (33, 1, "kq")):
    kw = dict(wtype=TT.Q4_K, wtypes={"v": TT.Q6_K, "down": TT.Q6_K}) if wt == "kq" else {}
    g = build_gemma3_gguf(cfg, seed=seed, **kw)
    prompt = np.random.default_rng(6).integers(4, cfg.vocab, n).astype(np.int32)
    os.environ.pop("LLMI_NO_PREFILL", None)
    lp = Model(g, exact=False, max_ctx=256).forward(prompt, 0)
    os.environ["LLMI_NO_PREFILL"] = "1"
    ll = Model(g, exact=False, max_ctx=256).forward(prompt, 0)
    os.environ.pop("LLMI_NO_PREFILL")
    print(f"{wt} seed {seed} n {n}: |prefill - loop| {np.abs(lp - ll).max():.3g}  (|loop| max {np.abs(ll).max():.3g})",
          flush=True)
