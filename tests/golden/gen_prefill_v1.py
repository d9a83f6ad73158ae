"""Pin of the retired prefill GEMMs (GPU, run once before v1-v4 left the library): the mini-4b logits
after a 200-token batched prefill through GEMM v1 (register-staged 32-row tiles, every output one
fmaf(d_w * d_x, (float)isum, acc) chain in block order) -- the chain GEMM v5 with one K group per output
(LLMI_PG5=big) computes bit for bit.  tests/test_prefill.py::test_prefill_gemm_v5_matches_pinned_v1 holds
v5 to these bits.  Writes tests/golden/prefill_v1_ref.npz (data only).

    LLMI_PREFILL_GEMM=1 python tests/golden/gen_prefill_v1.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402


def case():
    cfg = CONFIGS["mini-4b"]
    g = build_gemma3_gguf(cfg, seed=23)
    prompt = np.random.default_rng(2).integers(4, cfg.vocab, 200).astype(np.int32)
    return g, prompt


def main():
    assert os.environ.get("LLMI_PREFILL_GEMM") == "1", "run with LLMI_PREFILL_GEMM=1 (the v1 GEMM)"
    g, prompt = case()
    m = Model(g, max_ctx=256)
    assert m.info.batched_prefill == 1
    lg = m.forward(prompt, 0)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "prefill_v1_ref.npz")
    np.savez_compressed(out, logits=lg, prompt=prompt)
    print("wrote", out, float(np.abs(lg).max()))


if __name__ == "__main__":
    main()
