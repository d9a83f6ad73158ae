"""Device session (whole Gemma-3 forward on the GPU) vs the reference.

Tolerances:
  exact mode (LLMI_EXACT): logits BIT-IDENTICAL to the reference (ModelTest's
    own tolerance is 3e-3, model_test.cpp:422): every op restates the
    reference's arithmetic, glibc's expf/tanhf included (csrc/glibc_math.h).
  fast mode: the attention accumulates P.V in fp32 (split-K), while the
    reference keeps an f16 accumulator rounded at every key (model.cpp:484,
    ops.cpp:1091-1099), itself ~1e-3 away from exact math (the attention
    unit test pins fast attention to float64 math at 2e-5).  Through the
    Q8_0 activation re-quantization of every GEMV input, these ulp-level
    differences are amplified on random-init models: the reference vs the
    same reference with float64 attention differ by up to 3.7e-2 on mini-1b
    (scripts/diag_parts.py).  Fast mode is therefore held, per input, to the
    reference's OWN distance from exact math: |fast - f64-attention oracle|
    <= max(3e-3, 1.5 x |reference - f64-attention oracle|) -- ModelTest's
    3e-3 where the reference is itself exact to that (model_test.gguf:
    fast is 2.4e-7 from the oracle there), and never more than half again the
    reference's own attention-rounding deviation (measured worst: fast 0.033
    vs the reference's 0.037 on the same mini input) -- and vs the reference
    to that budget + |reference - oracle|, with greedy token ids identical.
    Cross-layout checks below (fused vs unfused launches) keep FAST_VS_REF.
  both modes: greedy token ids identical to the reference.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAST_VS_REF = 6e-2  # fused vs unfused fast layouts (reassociation through Q8_0 re-quantization)
REF_TOL = 3e-3  # ModelTest's own tolerance (model_test.cpp:422)


@pytest.fixture(scope="module", params=[True, False], ids=["exact", "fast"])
def exact(request):
    return request.param


def check(got, ref, ideal, exact):
    if exact:  # bit-identical to the reference (glibc's expf/tanhf restated on the device)
        np.testing.assert_array_equal(np.asarray(got).view(np.uint32), np.asarray(ref).view(np.uint32))
    else:
        print(f"fast: vs_ref {np.abs(got - ref).max():.3g} vs_f64attn {np.abs(got - ideal).max():.3g} "
              f"(ref vs f64attn {np.abs(ref - ideal).max():.3g})")
        # the f64-attention restatement is the target, held to the reference's own distance from it on this very
        # input (|ref - ideal|, its f16 accumulator's rounding), floored at ModelTest's 3e-3
        dev = float(np.abs(np.asarray(ref) - ideal).max())
        budget = max(REF_TOL, 1.5 * dev)
        np.testing.assert_allclose(got, ideal, atol=budget, rtol=0)
        np.testing.assert_allclose(got, ref, atol=budget + dev, rtol=0)


def test_model_test_gguf(oracle, golden_models, exact):
    from llm_inference_amd.model import Model
    g = open(os.path.join(ROOT, "tests", "golden", "model_test.gguf"), "rb").read()
    ideal = oracle.model(np.frombuffer(g, np.uint8), n_threads=2, max_ctx=8, attn_f64=True)
    m = Model(g, exact=exact, max_ctx=64)
    l1 = m.forward([1], 0)
    check(l1, golden_models["model_test__l1"], ideal.forward([1], 0), exact)
    if exact:
        for i, v in [(0, 2.9909527), (1, -0.216222), (8, 1.6922607), (9, -2.588623)]:  # model_test.cpp:426-432
            assert abs(l1[i] - v) < 0.003  # ModelTest's own tolerance (model_test.cpp:422)
    nt = int(np.argmax(golden_models["model_test__l1"]))
    assert m.last_argmax == nt
    l2 = m.forward([nt], 1)
    check(l2, golden_models["model_test__l2"], ideal.forward([nt], 1), exact)


def test_tiny_prefill_and_greedy(oracle, golden_models, exact):
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    g = build_gemma3_gguf(CONFIGS["tiny"], seed=7, swa_pattern=[True, False, True])
    ideal = oracle.model(g, n_threads=4, max_ctx=64, attn_f64=True)
    m = Model(g, exact=exact, max_ctx=128)
    prompt = golden_models["tiny__prompt"]
    ref_logits, ref_toks = golden_models["tiny__logits"], golden_models["tiny__tokens"]
    lg = m.forward(prompt, 0)
    check(lg, ref_logits[0], ideal.forward(prompt, 0), exact)
    assert m.last_argmax == ref_toks[0]
    # device-resident greedy loop (no host round trip between tokens)
    toks = m.generate(int(ref_toks[0]), len(prompt), len(ref_toks) - 1)
    assert toks.tolist() == ref_toks[1:].tolist()
    # eager (no graph) forward() path, step by step
    m2 = Model(g, exact=exact, max_ctx=128, use_graph=False)
    m2.forward(prompt, 0)
    pos = len(prompt)
    for i in range(1, len(ref_toks)):
        lg = m2.forward([int(ref_toks[i - 1])], pos)
        check(lg, ref_logits[i], ideal.forward([int(ref_toks[i - 1])], pos), exact)
        pos += 1


@pytest.mark.parametrize("cfg_name", ["mini-1b", "mini-4b"])
def test_mini_models_vs_oracle(oracle, cfg_name, exact):
    """Real Gemma-3 1B/4B layer shapes (2 layers, small vocab): 12-token prompt,
    then 12 greedy tokens; ids identical to the oracle (= reference, pinned)."""
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=3)
    om = oracle.model(g, n_threads=8, max_ctx=64)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    m = Model(g, exact=exact, max_ctx=64)
    prompt = np.random.default_rng(5).integers(4, cfg.vocab, 12).astype(np.int32)
    ref = om.forward(prompt, 0)
    got = m.forward(prompt, 0)
    check(got, ref, ideal.forward(prompt, 0), exact)
    toks_ref = [int(np.argmax(ref))]
    pos = len(prompt)
    for _ in range(11):
        lg = om.forward([toks_ref[-1]], pos)
        pos += 1
        toks_ref.append(int(np.argmax(lg)))
    toks = m.generate(int(np.argmax(got)), len(prompt), 11)
    assert [int(np.argmax(got))] + toks.tolist() == toks_ref


@pytest.mark.parametrize("cfg_name", ["mini-27b", "mini-4b"])
def test_exact_attention_past_a_key_chunk(oracle, cfg_name):
    """The exact attention's accumulate runs its keys in chunks of XA_CH = 1024 (k_exact.hip), each with a branch
    pass that scans the chunk's scores for the running max: a 1100-token prompt crosses a chunk, at head_dim 128
    (mini-27b) and 256 (mini-4b); the logits after it bit-identical to the reference's (round 5: at head_dim 128
    the scan covered 768 keys of a chunk)."""
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=11)
    prompt = np.random.default_rng(17).integers(4, cfg.vocab, 1100).astype(np.int32)
    ref = oracle.model(g, n_threads=16, max_ctx=1152).forward(prompt, 0)
    m = Model(g, exact=True, max_ctx=1152)
    got = m.forward(prompt, 0)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), float(np.abs(got - ref).max())
    m.close()


def test_session_errors():
    from llm_inference_amd._lib import LLMIError
    from llm_inference_amd.model import Model
    with pytest.raises(LLMIError) as ei:
        Model(b"NOPE" + b"\0" * 64)
    assert ei.value.status == "E_GGUF" and "magic" in str(ei.value)
    g = open(os.path.join(ROOT, "tests", "golden", "model_test.gguf"), "rb").read()
    m = Model(g, max_ctx=4)
    with pytest.raises(LLMIError) as ei:
        m.forward([1, 2, 3, 4, 5], 0)
    assert ei.value.status == "E_RANGE"
    with pytest.raises(LLMIError):
        m.forward([10], 0)  # vocab is 10
    # ALiBi (model.cpp:125-128, 492-518), which no Gemma file sets, is refused at load, never silently ignored
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    key = "attention.max_alibi_bias"
    with pytest.raises(LLMIError) as ei:
        Model(build_gemma3_gguf(CONFIGS["tiny"], seed=1, extra_meta={key: 8.0}), max_ctx=16)
    assert ei.value.status == "E_GGUF" and key in str(ei.value)
    Model(build_gemma3_gguf(CONFIGS["tiny"], seed=1, extra_meta={key: 0.0}), max_ctx=16).close()


@pytest.mark.parametrize("path", ["default", "token_loop", "per_op"])
def test_attention_softcap(oracle, golden_models, exact, path, monkeypatch):
    """attention.logit_softcapping (model.cpp:130-133, 511-513) on the tiny model, cap 0.25 (it moves the logits
    by 0.5): the reference's own logits (tests/golden/model_ref.npz tinycap, oracle pinned to them in
    test_oracle_golden.py) -- exact mode bit-identical, fast mode within the module's budget of the f64-attention
    oracle with the same cap -- through the batched prefill (default), the decode launches only (token_loop), and
    the per-projection launches (per_op: no attention block / fused layer launches)."""
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    if path != "default":
        monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    if path == "per_op":
        monkeypatch.setenv("LLMI_NO_FUSE", "1")
        monkeypatch.setenv("LLMI_NO_BLOCK", "1")
    cap = float(golden_models["tinycap__cap"])
    g = build_gemma3_gguf(CONFIGS["tiny"], seed=7, swa_pattern=[True, False, True],
                          extra_meta={"attention.logit_softcapping": cap})
    ideal = oracle.model(g, n_threads=4, max_ctx=64, attn_f64=True)
    m = Model(g, exact=exact, max_ctx=64)
    prompt = golden_models["tiny__prompt"]
    ref_logits, ref_toks = golden_models["tinycap__logits"], golden_models["tinycap__tokens"]
    lg = m.forward(prompt, 0)
    check(lg, ref_logits[0], ideal.forward(prompt, 0), exact)
    pos = len(prompt)
    for i in range(1, len(ref_toks)):
        lg = m.forward([int(ref_toks[i - 1])], pos)
        check(lg, ref_logits[i], ideal.forward([int(ref_toks[i - 1])], pos), exact)
        pos += 1
    m.close()
    m = Model(g, exact=exact, max_ctx=64)
    first = int(np.argmax(m.forward(prompt, 0)))
    assert [first] + m.generate(first, len(prompt), len(ref_toks) - 1).tolist() == ref_toks.tolist()
    m.close()


def test_unfused_fast_path_matches_fused(oracle, monkeypatch):
    """LLMI_NO_FUSE=1 selects the separate norm / GELU launches; both fast
    layouts agree to reassociation noise and give the reference's ids."""
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-4b"]
    g = build_gemma3_gguf(cfg, seed=11)
    prompt = np.random.default_rng(2).integers(4, cfg.vocab, 9).astype(np.int32)
    fused = Model(g, exact=False, max_ctx=64)
    lf = fused.forward(prompt, 0)
    monkeypatch.setenv("LLMI_NO_FUSE", "1")
    plain = Model(g, exact=False, max_ctx=64)
    lp = plain.forward(prompt, 0)
    assert fused.get_info().kernels_per_token < plain.get_info().kernels_per_token
    np.testing.assert_allclose(lf, lp, atol=FAST_VS_REF, rtol=0)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    np.testing.assert_allclose(lf, ideal.forward(prompt, 0), atol=FAST_VS_REF, rtol=0)
    assert int(np.argmax(lf)) == int(np.argmax(lp))


@pytest.mark.parametrize("quant", ["q4_k_m", "q8_0"])
def test_kquant_and_q8_models_vs_oracle(oracle, quant, exact, monkeypatch):
    """BASELINE configs[3]: Gemma-3 4B Q4_K_M (Q4_K projections, Q6_K v/down;
    per-projection path: Q8_K activations, fast K-quant GEMVs) and 1B Q8_0
    layer shapes (fast mode: the fused layer launches with Q8_0 weights) through
    the session, vs the oracle: greedy ids identical, logits within the
    module's tolerances.  The prompt runs through the decode launches (token
    loop); the Q8_0 batched prefill is checked against the same oracle below."""
    from llm_inference_amd.gguf import TensorType as TT
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    if quant == "q4_k_m":
        cfg = CONFIGS["mini-4b"]
        g = build_gemma3_gguf(cfg, seed=8, wtype=TT.Q4_K, wtypes={"v": TT.Q6_K, "down": TT.Q6_K})
    else:
        cfg = CONFIGS["mini-1b"]
        g = build_gemma3_gguf(cfg, seed=8, wtype=TT.Q8_0, embd_type=TT.Q8_0)
    om = oracle.model(g, n_threads=8, max_ctx=64)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    m = Model(g, exact=exact, max_ctx=64)
    prompt = np.random.default_rng(4).integers(4, cfg.vocab, 10).astype(np.int32)
    ref = om.forward(prompt, 0)
    got = m.forward(prompt, 0)
    check(got, ref, ideal.forward(prompt, 0), exact)
    toks_ref = [int(np.argmax(ref))]
    pos = len(prompt)
    for _ in range(6):
        lg = om.forward([toks_ref[-1]], pos)
        pos += 1
        toks_ref.append(int(np.argmax(lg)))
    toks = m.generate(int(np.argmax(got)), len(prompt), 6)
    assert [int(np.argmax(got))] + toks.tolist() == toks_ref


def test_q8_0_fused_matches_unfused(oracle, monkeypatch):
    """Q8_0 weights in the fused layer launch table (k_layer.hip W8 entries:
    half-block units, no zero point) against the per-projection Q8_0 path."""
    from llm_inference_amd.gguf import TensorType as TT
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-1b"]
    g = build_gemma3_gguf(cfg, seed=12, wtype=TT.Q8_0)
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")  # the decode launches on both sides (prefill: tests/test_prefill.py)
    prompt = np.random.default_rng(5).integers(4, cfg.vocab, 9).astype(np.int32)
    fused = Model(g, exact=False, max_ctx=64)
    lf = fused.forward(prompt, 0)
    monkeypatch.setenv("LLMI_NO_FUSE", "1")
    plain = Model(g, exact=False, max_ctx=64)
    lp = plain.forward(prompt, 0)
    assert fused.get_info().kernels_per_token < plain.get_info().kernels_per_token
    np.testing.assert_allclose(lf, lp, atol=FAST_VS_REF, rtol=0)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    np.testing.assert_allclose(lf, ideal.forward(prompt, 0), atol=FAST_VS_REF, rtol=0)
    first = int(np.argmax(lf))
    assert first == int(np.argmax(lp))
    assert fused.generate(first, len(prompt), 8).tolist() == plain.generate(first, len(prompt), 8).tolist()


def test_q8_0_batched_prefill_vs_oracle(oracle):
    """The 1B Q8_0 model of test_kquant_and_q8_models_vs_oracle (Q8_0 token_embd too) through the batched
    prefill: greedy ids identical to the oracle's.  Logits are held to 2 x the fast budget: op by op the prefill
    is exact (embedding Q8_0 blocks bit-identical to the reference's, every GEMM row within 1e-6 of the
    reference's Q8_0 x Q8_0 rows from the device's own inputs: scripts/dev/q8p_diag.py,
    tests/test_fused_ops.py::test_ops_mini1b_q8_0_fused), but on this 2-layer model a one-quantum Q8 rounding
    flip of an activation -- the prefill's norms sum in another order than the decode launches -- moves the
    logits by up to 0.095 (0.091 with the fp32 vector prefill attention, so not the f16 P of the MFMA
    attention); the token loop on the same input is within 4e-6."""
    from llm_inference_amd.gguf import TensorType as TT
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-1b"]
    g = build_gemma3_gguf(cfg, seed=8, wtype=TT.Q8_0, embd_type=TT.Q8_0)
    om = oracle.model(g, n_threads=8, max_ctx=64)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    m = Model(g, exact=False, max_ctx=64)
    assert m.get_info().batched_prefill == 1
    prompt = np.random.default_rng(4).integers(4, cfg.vocab, 10).astype(np.int32)
    ref = om.forward(prompt, 0)
    got = m.forward(prompt, 0)
    d = float(np.abs(got - ideal.forward(prompt, 0)).max())
    print(f"Q8_0 batched prefill vs f64-attention oracle: {d:.3g}")
    assert d <= 2 * FAST_VS_REF
    toks_ref = [int(np.argmax(ref))]
    pos = len(prompt)
    for _ in range(6):
        toks_ref.append(int(np.argmax(om.forward([toks_ref[-1]], pos))))
        pos += 1
    toks = m.generate(int(np.argmax(got)), len(prompt), 6)
    assert [int(np.argmax(got))] + toks.tolist() == toks_ref


@pytest.mark.parametrize("vtype", ["q6_k", "q4_k"])
def test_kquant_fused_matches_unfused(oracle, monkeypatch, vtype):
    """K-quant weights in the fused layer launch table (k_layer.hip kq entries:
    Q4_K / Q6_K rows repacked into 32-element sub-blocks, Q8_K activations
    quantized in the launches' prologues; q|k Q4_K + v Q6_K in one launch)
    against the per-projection K-quant path and the f64-attention oracle."""
    from llm_inference_amd.gguf import TensorType as TT
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-4b"]
    vt = TT.Q6_K if vtype == "q6_k" else TT.Q4_K
    g = build_gemma3_gguf(cfg, seed=17, wtype=TT.Q4_K, wtypes={"v": vt, "down": vt})
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")  # the decode launches on both sides (prefill: tests/test_prefill.py)
    prompt = np.random.default_rng(6).integers(4, cfg.vocab, 9).astype(np.int32)
    fused = Model(g, exact=False, max_ctx=64)
    lf = fused.forward(prompt, 0)
    monkeypatch.setenv("LLMI_NO_FUSE", "1")
    plain = Model(g, exact=False, max_ctx=64)
    lp = plain.forward(prompt, 0)
    print(f"{vtype}: kernels per token fused {fused.get_info().kernels_per_token} vs "
          f"{plain.get_info().kernels_per_token}; |fused - unfused| {float(np.abs(lf - lp).max()):.3g}")
    assert fused.get_info().kernels_per_token < plain.get_info().kernels_per_token
    np.testing.assert_allclose(lf, lp, atol=FAST_VS_REF, rtol=0)
    ideal = oracle.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    np.testing.assert_allclose(lf, ideal.forward(prompt, 0), atol=FAST_VS_REF, rtol=0)
    first = int(np.argmax(lf))
    assert first == int(np.argmax(lp))
    assert fused.generate(first, len(prompt), 8).tolist() == plain.generate(first, len(prompt), 8).tolist()


def test_attention_softcap_exact_engine(oracle):
    """The soft-cap in the exact-order engine (k_exact.hip, taken on real 4B layer shapes): logits and greedy ids
    bit-identical to the oracle with the same cap (the oracle's soft-cap is pinned to the reference's own logits
    in test_oracle_golden.py::test_tiny_model_prefill_decode[tinycap])."""
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-4b"]
    g = build_gemma3_gguf(cfg, seed=3, extra_meta={"attention.logit_softcapping": 0.25})
    plain = oracle.model(build_gemma3_gguf(cfg, seed=3), n_threads=8, max_ctx=64)
    om = oracle.model(g, n_threads=8, max_ctx=64)
    m = Model(g, exact=True, max_ctx=64)
    assert m.get_info().exact_engine == 1
    prompt = np.random.default_rng(5).integers(4, cfg.vocab, 12).astype(np.int32)
    ref = om.forward(prompt, 0)
    assert np.abs(ref - plain.forward(prompt, 0)).max() > 1e-2  # the cap changes this model's logits
    got = m.forward(prompt, 0)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    toks_ref, pos = [int(np.argmax(ref))], len(prompt)
    for _ in range(7):
        toks_ref.append(int(np.argmax(om.forward([toks_ref[-1]], pos))))
        pos += 1
    assert [int(np.argmax(got))] + m.generate(int(np.argmax(got)), len(prompt), 7).tolist() == toks_ref
    m.close()
