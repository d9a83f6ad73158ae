"""Sensitivity control for the K-quant prefill gap (development): the token loop against itself under other
launch layouts (LLMI_NO_BLOCK: three-launch attention; LLMI_NO_FUSE: per-projection GEMVs) on the same input."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from llm_inference_amd.gguf import TensorType as TT  # noqa: E402
from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

cfg = CONFIGS["mini-4b"]
for seed in (33, 34):
    g = build_gemma3_gguf(cfg, seed=seed, wtype=TT.Q4_K, wtypes={"v": TT.Q6_K, "down": TT.Q6_K})
    prompt = np.random.default_rng(6).integers(4, cfg.vocab, 150).astype(np.int32)
    out = {}
    for name, env in (("prefill", {}), ("loop", {"LLMI_NO_PREFILL": "1"}),
                      ("loop_noblock", {"LLMI_NO_PREFILL": "1", "LLMI_NO_BLOCK": "1"}),
                      ("loop_nofuse", {"LLMI_NO_PREFILL": "1", "LLMI_NO_FUSE": "1"})):
        for k in ("LLMI_NO_PREFILL", "LLMI_NO_BLOCK", "LLMI_NO_FUSE"):
            os.environ.pop(k, None)
        os.environ.update(env)
        out[name] = Model(g, exact=False, max_ctx=256).forward(prompt, 0)
    for k in ("LLMI_NO_PREFILL", "LLMI_NO_BLOCK", "LLMI_NO_FUSE"):
        os.environ.pop(k, None)
    ref = out["loop"]
    print(f"seed {seed}: " + "  ".join(f"{k}-loop {np.abs(v - ref).max():.3g}" for k, v in out.items() if k != "loop"),
          flush=True)
