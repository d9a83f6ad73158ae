"""Gemma-4 oracle pin: the C restatement
(oracle/llmi_oracle.c, gemma4 branches) is BIT-IDENTICAL to the reference's
own logits recorded by tests/golden/gen_gemma4.py on seeded synthetic
Gemma-4 GGUFs: per-layer token embeddings (F16 and Q6_K tables) + model
projection (model.cpp:568-704), shared KV layers reading an earlier SWA /
global layer's cache (model.cpp:775-777), V RMSNorm (model.cpp:813-829),
the per-layer embedding step and layer output scale (model.cpp:926-977),
attention scale 1 (model.cpp:119-122)."""
import hashlib
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def g4():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "gemma4_ref.npz")))


@pytest.mark.parametrize("case", [0, 1, 2], ids=["tiny4", "tiny4_q6k", "mini4"])
def test_gemma4_oracle_bitwise(oracle, g4, case):
    import gen_gemma4 as gen
    c = gen.CASES[case]
    name = c[0]
    g = gen.build(c)
    assert hashlib.sha256(g.tobytes()).hexdigest().encode() == g4[f"{name}__sha"].tobytes()
    prompt = gen.prompt_of(c)
    assert prompt.tolist() == g4[f"{name}__prompt"].tolist()
    om = oracle.model(g, n_threads=4, max_ctx=64)
    ref_logits, ref_toks = g4[f"{name}__logits"], g4[f"{name}__tokens"]
    lg = om.forward(prompt, 0)
    pos = len(prompt)
    for i in range(len(ref_toks)):
        np.testing.assert_array_equal(lg.view(np.uint32), ref_logits[i].view(np.uint32), err_msg=f"step {i}")
        assert int(np.argmax(lg)) == ref_toks[i]
        if i + 1 < len(ref_toks):
            lg = om.forward([int(ref_toks[i])], pos)
            pos += 1


def test_gemma4_structure():
    """The synthetic file carries the reference's Gemma-4 keys and tensor map:
    shared layers have no K/V projections; per-layer tensors present."""
    from llm_inference_amd.gguf import GGUFFile
    from llm_inference_amd.synthetic import CONFIGS4, build_gemma4_gguf
    cfg = CONFIGS4["tiny4"]
    gf = GGUFFile(build_gemma4_gguf(cfg, seed=1))
    assert gf.metadata["general.architecture"] == "gemma4"
    names = {t.name for t in gf.tensor_infos}
    kv_from = cfg.n_layer - cfg.shared_kv_layers
    for l in range(cfg.n_layer):
        assert (f"blk.{l}.attn_k.weight" in names) == (l < kv_from)
        for t in ("inp_gate", "proj", "post_norm", "layer_output_scale"):
            assert f"blk.{l}.{t}.weight" in names
    assert {"per_layer_token_embd.weight", "per_layer_model_proj.weight", "per_layer_proj_norm.weight"} <= names
