"""Attention block (k_attn.hip): the qkv GEMV, attention and the o GEMV of a
decode layer in ONE launch with in-kernel hand-offs (bs.cnt counters).

Checked against the three-launch fast path (LLMI_NO_BLOCK=1) and the oracle:
  * greedy ids identical, logits within the fast-mode tolerance of
    tests/test_hip_model.py (the o projection reduces its 64 blocks in a
    different lane order in the block: R2 vs R1 rows per wave);
  * determinism: two fresh sessions give bit-identical logits and ids (a
    hand-off race would show up as run-to-run differences);
  * long context (> 1024 keys: several 32-key tiles per split) after a
    batched prefill.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
FAST_VS_REF = 6e-2


def _models(cfg_name, seed, monkeypatch, max_ctx=64):
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=seed)
    blk = Model(g, max_ctx=max_ctx)
    monkeypatch.setenv("LLMI_NO_BLOCK", "1")
    three = Model(g, max_ctx=max_ctx)
    monkeypatch.delenv("LLMI_NO_BLOCK")
    return cfg, g, blk, three


@pytest.mark.parametrize("cfg_name", ["mini-1b", "mini-4b"])
def test_block_matches_three_launches(oracle, cfg_name, monkeypatch):
    cfg, g, blk, three = _models(cfg_name, 21, monkeypatch)
    prompt = np.random.default_rng(9).integers(4, cfg.vocab, 16).astype(np.int32)
    lb = blk.forward(prompt, 0)
    lt = three.forward(prompt, 0)
    np.testing.assert_allclose(lb, lt, atol=FAST_VS_REF, rtol=0)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    np.testing.assert_allclose(lb, ideal.forward(prompt, 0), atol=FAST_VS_REF, rtol=0)
    first = int(np.argmax(lb))
    assert first == int(np.argmax(lt))
    tb = blk.generate(first, len(prompt), 20)
    tt = three.generate(first, len(prompt), 20)
    assert tb.tolist() == tt.tolist()
    # one launch per layer instead of three (qkv, attention, o)
    assert blk.get_info().kernels_per_token == three.get_info().kernels_per_token - 2 * cfg.n_layer
    # step-by-step forward() through the block graph, logits each step
    pos = len(prompt) + 20
    for i in range(4):
        a = blk.forward([int(tb[-1])], pos + i)
        b = three.forward([int(tt[-1])], pos + i)
        np.testing.assert_allclose(a, b, atol=FAST_VS_REF, rtol=0)


def test_block_deterministic(monkeypatch):
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-4b"]
    g = build_gemma3_gguf(cfg, seed=5)
    prompt = np.random.default_rng(1).integers(4, cfg.vocab, 8).astype(np.int32)
    runs = []
    for _ in range(2):
        m = Model(g, max_ctx=256)
        lg = m.forward(prompt, 0)
        toks = m.generate(int(np.argmax(lg)), len(prompt), 96)
        last = m.forward([int(toks[-1])], len(prompt) + 96)
        runs.append((lg, toks, last))
        m.close()
    assert np.array_equal(runs[0][0].view(np.uint32), runs[1][0].view(np.uint32))
    assert runs[0][1].tolist() == runs[1][1].tolist()
    assert np.array_equal(runs[0][2].view(np.uint32), runs[1][2].view(np.uint32))


def test_block_long_context(monkeypatch):
    cfg, g, blk, three = _models("mini-4b", 33, monkeypatch, max_ctx=1536)
    prompt = np.random.default_rng(3).integers(4, cfg.vocab, 1100).astype(np.int32)
    lb = blk.forward(prompt, 0)  # batched prefill (same kernels in both)
    lt = three.forward(prompt, 0)
    assert np.array_equal(lb.view(np.uint32), lt.view(np.uint32))
    first = int(np.argmax(lb))
    tb = blk.generate(first, len(prompt), 8)
    tt = three.generate(first, len(prompt), 8)
    assert tb.tolist() == tt.tolist()
    a = blk.forward([int(tb[-1])], len(prompt) + 8)
    b = three.forward([int(tt[-1])], len(prompt) + 8)
    print(f"long context: max |block - three launches| = {np.abs(a - b).max():.3g}")
    np.testing.assert_allclose(a, b, atol=FAST_VS_REF, rtol=0)
