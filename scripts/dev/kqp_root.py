"""Root cause of the K-quant batched-prefill outlier:
mini-4b Q4_K_M, seed 33, 150 prompt tokens.  Every device variant against the
oracle (the reference's arithmetic on the CPU) and the oracle with f64
attention, last token's logits (development)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from llm_inference_amd.gguf import TensorType as TT  # noqa: E402
from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402
from oracle.bind import Oracle  # noqa: E402

cfg = CONFIGS["mini-4b"]
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 33
n = int(sys.argv[2]) if len(sys.argv) > 2 else 150
g = build_gemma3_gguf(cfg, seed=seed, wtype=TT.Q4_K, wtypes={"v": TT.Q6_K, "down": TT.Q6_K})
prompt = np.random.default_rng(6).integers(4, cfg.vocab, n).astype(np.int32)
orc = Oracle()
ref = orc.model(g, n_threads=16, max_ctx=256).forward(prompt, 0)
f64 = orc.model(g, n_threads=16, max_ctx=256, attn_f64=True).forward(prompt, 0)
print(f"seed {seed} n {n}: max|logit| {np.abs(ref).max():.3g}; |oracle - oracle_f64attn| {np.abs(ref - f64).max():.3g}")
variants = {
    "batched (default)": {},
    "token loop (fused)": {"LLMI_NO_PREFILL": "1"},
    "token loop (unfused)": {"LLMI_NO_PREFILL": "1", "LLMI_NO_FUSE": "1"},
}
outs = {}
for name, env in variants.items():
    for k, v in env.items():
        os.environ[k] = v
    m = Model(g, max_ctx=256)
    outs[name] = m.forward(prompt, 0)
    m.close()
    for k in env:
        os.environ.pop(k)
    lg = outs[name]
    print(f"  {name:55s} |.-oracle| {np.abs(lg - ref).max():.4f}  |.-oracle_f64| {np.abs(lg - f64).max():.4f}  "
          f"argmax {int(np.argmax(lg))} (oracle {int(np.argmax(ref))})", flush=True)
