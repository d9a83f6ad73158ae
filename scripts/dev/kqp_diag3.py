"""K-quant int8 batched prefill vs the token loop over prompt lengths (development)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from llm_inference_amd.gguf import TensorType as TT  # noqa: E402
from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

cfg = CONFIGS["mini-4b"]
for seed in (33, 35, 36):
    g = build_gemma3_gguf(cfg, seed=seed, wtype=TT.Q4_K, wtypes={"v": TT.Q6_K, "down": TT.Q6_K})
    row = []
    for n in (32, 64, 100, 150, 200):
        prompt = np.random.default_rng(6).integers(4, cfg.vocab, n).astype(np.int32)
        os.environ.pop("LLMI_NO_PREFILL", None)
        lp = Model(g, exact=False, max_ctx=256).forward(prompt, 0)
        os.environ["LLMI_NO_PREFILL"] = "1"
        ll = Model(g, exact=False, max_ctx=256).forward(prompt, 0)
        os.environ["LLMI_NO_FUSE"] = "1"
        lu = Model(g, exact=False, max_ctx=256).forward(prompt, 0)
        os.environ.pop("LLMI_NO_PREFILL")
        os.environ.pop("LLMI_NO_FUSE")
        row.append(f"n{n}: {np.abs(lp - ll).max():.3g} (ctl {np.abs(lu - ll).max():.3g})")
    print(f"seed {seed}: " + "  ".join(row), flush=True)
