"""The layer engine (csrc/k_engine.hip): each Gemma-3
decode layer as ONE launch of one 1024-thread work-group per CU.

Opt-in (LLMI_ENGINE=1; measured slower than the default three launches per
layer) and built only into the development variant
(LLMI_VARIANT=engines LLMI_EXTRA_FLAGS=-DLLMI_DEV_ENGINES python -m
llm_inference_amd.build; run these tests with
LLMI_LIB=llm_inference_amd/libllmi_engines.so), never into libllmi.so.  Parity bar (the fast path's,
tests/test_hip_model.py): logits within 6e-2 of the oracle with float64
attention (= the reference's arithmetic with exact attention, pinned to the
reference build), greedy token ids identical to the oracle's.  Against the
three-launch fast path (attention block, gate_up, down) the engine differs only in the summation order of the
projections' block sums and of the norms, so its logits are held to the same
budget and its ids must be identical.  Cases: Gemma-3 1B and 4B layer shapes,
decode positions inside the first key tile, past 32 tiles (a split walks two
tiles, the later one loaded inside the loop), and at tile boundaries.
"""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.environ.get("LLMI_LIB", "").endswith("libllmi_engines.so"),
                                 reason="the engines are in the development variant only (LLMI_LIB=...engines.so)")]
FAST_VS_REF = 6e-2


def _model(g, monkeypatch, engine, **kw):
    from llm_inference_amd.model import Model
    if engine:
        monkeypatch.setenv("LLMI_ENGINE", "1")
    else:
        monkeypatch.delenv("LLMI_ENGINE", raising=False)
    m = Model(g, exact=False, **kw)
    monkeypatch.delenv("LLMI_ENGINE", raising=False)
    return m


@pytest.mark.parametrize("cfg_name", ["mini-1b", "mini-4b"])
def test_engine_selected(cfg_name, monkeypatch):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    g = build_gemma3_gguf(CONFIGS[cfg_name], seed=3)
    on = _model(g, monkeypatch, True, max_ctx=64)
    off = _model(g, monkeypatch, False, max_ctx=64)
    assert on.get_info().layer_engine == 1 and off.get_info().layer_engine == 0
    for m in (on, off):  # the step graph (and its launch count) exists once a decode step ran
        m.forward([5, 6, 7], 0)
        m.forward([8], 3)
    # one launch per layer instead of three
    assert on.get_info().kernels_per_token == off.get_info().kernels_per_token - 2 * CONFIGS[cfg_name].n_layer


@pytest.mark.parametrize("cfg_name", ["mini-1b", "mini-4b"])
def test_engine_decode_vs_oracle(oracle, cfg_name, monkeypatch):
    """Prompt through the batched prefill, then decode steps through the engine, each step's
    logits against the f64-attention oracle on the oracle's own token history; ids identical."""
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=21)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    m = _model(g, monkeypatch, True, max_ctx=64)
    assert m.get_info().layer_engine == 1
    prompt = np.random.default_rng(6).integers(4, cfg.vocab, 11).astype(np.int32)
    ideal.forward(prompt, 0)
    m.forward(prompt, 0)
    tok, pos = int(prompt[-1]) % cfg.vocab, len(prompt)
    worst = 0.0
    for _ in range(10):
        li = ideal.forward([tok], pos)
        lg = m.forward([tok], pos)
        worst = max(worst, float(np.abs(lg - li).max()))
        np.testing.assert_allclose(lg, li, atol=FAST_VS_REF, rtol=0)
        assert int(np.argmax(lg)) == int(np.argmax(li))
        tok, pos = int(np.argmax(li)), pos + 1
    print(f"{cfg_name}: engine vs f64-attention oracle, worst step {worst:.3g}")


@pytest.mark.parametrize("cfg_name", ["mini-1b", "mini-4b"])
def test_engine_greedy_matches_three_launch_path(oracle, cfg_name, monkeypatch):
    """The device-resident greedy loop (hipGraph replays of the engine) against the attention-block
    path and the oracle: 16 tokens, identical ids."""
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=5)
    on = _model(g, monkeypatch, True, max_ctx=64)
    off = _model(g, monkeypatch, False, max_ctx=64)
    om = oracle.model(g, n_threads=8, max_ctx=64)
    prompt = np.random.default_rng(9).integers(4, cfg.vocab, 8).astype(np.int32)
    lo = on.forward(prompt, 0)
    lf = off.forward(prompt, 0)
    ref = om.forward(prompt, 0)
    first = int(np.argmax(ref))
    assert int(np.argmax(lo)) == first == int(np.argmax(lf))
    toks_ref = [first]
    pos = len(prompt)
    for _ in range(15):
        toks_ref.append(int(np.argmax(om.forward([toks_ref[-1]], pos))))
        pos += 1
    a = on.generate(first, len(prompt), 15).tolist()
    b = off.generate(first, len(prompt), 15).tolist()
    assert [first] + a == toks_ref
    assert a == b


@pytest.mark.parametrize("n_prompt", [1023, 1055])
def test_engine_long_context(n_prompt, monkeypatch):
    """Positions past NSPLIT x 32 = 1024 keys: the splits walk a second key tile, loaded inside the
    attention loop (the first is prefetched at launch start), and 1023 puts the first decode key at a
    tile boundary.  Engine vs the attention-block path on the same prefilled cache: logits within the
    fast budget, ids identical."""
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-4b"]
    g = build_gemma3_gguf(cfg, seed=13)
    on = _model(g, monkeypatch, True, max_ctx=2048)
    off = _model(g, monkeypatch, False, max_ctx=2048)
    prompt = np.random.default_rng(3).integers(4, cfg.vocab, n_prompt).astype(np.int32)
    lo = on.forward(prompt, 0)
    lf = off.forward(prompt, 0)
    np.testing.assert_array_equal(lo.view(np.uint32), lf.view(np.uint32))  # same batched prefill on both
    tok, pos = int(np.argmax(lf)), n_prompt
    worst = 0.0
    for _ in range(4):
        a = on.forward([tok], pos)
        b = off.forward([tok], pos)
        worst = max(worst, float(np.abs(a - b).max()))
        np.testing.assert_allclose(a, b, atol=FAST_VS_REF, rtol=0)
        assert int(np.argmax(a)) == int(np.argmax(b))
        tok, pos = int(np.argmax(b)), pos + 1
    print(f"long context {n_prompt}: engine vs attention-block path {worst:.3g}")


def test_engine_time_kernel(monkeypatch):
    """The bench hook for the engine's launch (time_kernel family 6) runs and reports the layer's bytes."""
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-4b"]
    g = build_gemma3_gguf(cfg, seed=2)
    m = _model(g, monkeypatch, True, max_ctx=64)
    m.forward([5, 6, 7], 0)
    us, by = m.time_kernel(6, 3)
    w = 18 / 32 * cfg.n_embd * ((cfg.n_head + 2 * cfg.n_head_kv) * cfg.head_dim + cfg.n_head * cfg.head_dim + 3 * cfg.n_ff)
    assert us > 0 and by >= w
