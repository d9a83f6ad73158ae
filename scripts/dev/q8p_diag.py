"""Q8_0 1B mini (embd Q8_0): batched prefill vs token loop vs the f64-attention oracle (development)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from llm_inference_amd.gguf import TensorType as TT  # noqa: E402
from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402
from oracle.bind import Oracle  # noqa: E402  (the checker)

orc = Oracle()
cfg = CONFIGS["mini-1b"]
for seed, embd in ((8, TT.Q8_0), (8, TT.F16), (9, TT.Q8_0), (10, TT.Q8_0)):
    g = build_gemma3_gguf(cfg, seed=seed, wtype=TT.Q8_0, embd_type=embd)
    ideal = orc.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    prompt = np.random.default_rng(4).integers(4, cfg.vocab, 10).astype(np.int32)
    li = ideal.forward(prompt, 0)
    os.environ.pop("LLMI_NO_PREFILL", None)
    lp = Model(g, exact=False, max_ctx=64).forward(prompt, 0)
    os.environ["LLMI_PREFILL_ATTN_V1"] = "1"
    lv = Model(g, exact=False, max_ctx=64).forward(prompt, 0)
    os.environ.pop("LLMI_PREFILL_ATTN_V1")
    print(f"  fp32 vector prefill attention: prefill-ideal {np.abs(lv - li).max():.3g}", flush=True)
    os.environ["LLMI_NO_PREFILL"] = "1"
    ll = Model(g, exact=False, max_ctx=64).forward(prompt, 0)
    os.environ.pop("LLMI_NO_PREFILL")
    print(f"seed {seed} embd {embd}: prefill-ideal {np.abs(lp - li).max():.3g}  loop-ideal {np.abs(ll - li).max():.3g}"
          f"  prefill-loop {np.abs(lp - ll).max():.3g}", flush=True)

