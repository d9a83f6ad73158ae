"""The oracle (our CPU restatement) against golden vectors produced by the
reference itself (tests/golden/gen_golden.py) -- bit-exact -- and against the
reference's own published ModelTest numbers (model_test.cpp:422-459)."""
import os

import numpy as np
import pytest

import cases as K
from llm_inference_amd.gguf import TensorType as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


@pytest.mark.parametrize("name,tt,r,c", K.GEMV_CASES, ids=[c[0] for c in K.GEMV_CASES])
def test_gemv_bitexact(oracle, golden_ops, name, tt, r, c):
    w, x = K.gemv_inputs(name, tt, r, c)
    assert K.sha(w, x).encode() == golden_ops[f"gemv__{name}__sha"].tobytes(), "input generator drifted"
    o = oracle.mat_vec_mul(tt, w, r, c, x, n_threads=3)
    np.testing.assert_array_equal(bits(o), bits(golden_ops[f"gemv__{name}__o"]))


@pytest.mark.parametrize("i", range(len(K.QUANT_CASES)))
def test_quantize_bitexact(oracle, golden_ops, i):
    kind, n = K.QUANT_CASES[i]
    x = K.quant_input(kind, n, i)
    y = oracle.quantize_q8_0(x) if kind == "q8_0" else oracle.quantize_q8_k(x)
    np.testing.assert_array_equal(y, golden_ops[f"quant__{kind}_{n}__y"])


@pytest.mark.parametrize("n", K.NORM_CASES)
def test_rms_norm_softmax_bitexact(oracle, golden_ops, n):
    x = K.norm_input(n)
    np.testing.assert_array_equal(bits(oracle.rms_norm(x, float(np.float32(1e-6)))), bits(golden_ops[f"rms__{n}"]))
    np.testing.assert_array_equal(bits(oracle.softmax(x)), bits(golden_ops[f"softmax__{n}"]))


@pytest.mark.parametrize("case", K.ROPE_CASES)
def test_rope_bitexact(oracle, golden_ops, case):
    nt, nh, hd, base, pos = case
    t = K.rope_input(nt, nh, hd)
    got = oracle.rope(t, hd, base, 1.0, pos)
    np.testing.assert_array_equal(bits(got), bits(golden_ops[f"rope__{nt}_{nh}_{hd}_{int(base)}_{pos}"]))


def test_rope_known_answer(oracle):
    # ops_test.cpp:42-62
    t = oracle.rope(np.array([[[1, 2, 3, 4]]], np.float32), 4, 10000.0, 1.0, 1)
    assert abs(t[0, 0, 0] - -1.984111) < 1e-4 and abs(t[0, 0, 2] - 2.462337) < 1e-4


@pytest.mark.parametrize("tt,n", K.DEQ_CASES)
def test_dequantize_bitexact(oracle, golden_ops, tt, n):
    np.testing.assert_array_equal(bits(oracle.dequantize_row(tt, K.deq_input(tt, n), n)),
                                  bits(golden_ops[f"deq__{tt}_{n}"]))


def test_f16_conversions(oracle, golden_ops):
    x = K.f16_input()
    np.testing.assert_array_equal(oracle.f32_to_f16(x), golden_ops["f16__to16"])
    tab = np.array([oracle.lib.orc_f16_to_f32(i) for i in range(65536)], np.float32)
    np.testing.assert_array_equal(tab.view(np.uint32), golden_ops["f16__table"])
    # gguf_test.cpp:63-83 known values
    assert oracle.lib.orc_f16_to_f32(0x3C00) == 1.0 and oracle.lib.orc_f16_to_f32(0x7BFF) == 65504.0
    assert abs(oracle.lib.orc_f16_to_f32(773) - 0.000046) < 1e-6


def test_vec_f16(oracle, golden_ops):
    rng = np.random.default_rng(6000)
    y = rng.standard_normal(256).astype(np.float16).view(np.uint16)
    xv = rng.standard_normal(256).astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(oracle.vec_scale_f16(y, 0.3712), golden_ops["vec__scale"])
    np.testing.assert_array_equal(oracle.vec_mad_f16(y, xv, 0.8123), golden_ops["vec__mad"])


def test_single_block_known_answers(oracle):
    # ops_test.cpp:138-257 (Q4_K 512, Q6_K 256, Q8_0 64, Q5_0 32)
    import struct
    f16 = lambda v: np.float16(v).view(np.uint16)
    q4k = bytearray(144); q4k[0:2] = struct.pack("<H", f16(1.0)); q4k[2:4] = struct.pack("<H", f16(0.0))
    for i in range(4): q4k[4 + i] = 1
    for i in range(8, 12): q4k[4 + i] = 1
    q4k[16:] = bytes([2 | (2 << 4)]) * 128
    assert abs(oracle.mat_vec_mul(T.Q4_K, np.frombuffer(bytes(q4k), np.uint8), 1, 256, np.ones(256, np.float32))[0] - 512) < 1e-3
    q6k = bytearray(210); q6k[:128] = b"\x11" * 128; q6k[128:192] = b"\xaa" * 64; q6k[192:208] = b"\x01" * 16
    q6k[208:210] = struct.pack("<H", f16(1.0))
    assert abs(oracle.mat_vec_mul(T.Q6_K, np.frombuffer(bytes(q6k), np.uint8), 1, 256, np.ones(256, np.float32))[0] - 256) < 1e-3
    q8 = struct.pack("<H", f16(1.0)) + bytes([2]) * 32
    assert abs(oracle.mat_vec_mul(T.Q8_0, np.frombuffer(q8, np.uint8), 1, 32, np.ones(32, np.float32))[0] - 64) < 1e-2
    q5 = struct.pack("<H", f16(1.0)) + b"\xff" * 4 + b"\x11" * 16
    assert abs(oracle.mat_vec_mul(T.Q5_0, np.frombuffer(q5, np.uint8), 1, 32, np.ones(32, np.float32))[0] - 32) < 1e-3


def test_model_test_forward(oracle, golden_models):
    g = open(os.path.join(ROOT, "tests", "golden", "model_test.gguf"), "rb").read()
    from llm_inference_amd.synthetic import build_model_test_gguf
    assert build_model_test_gguf() == g, "ModelTest GGUF builder drifted"
    m = oracle.model(g)
    l1 = m.forward([1], 0)
    np.testing.assert_array_equal(bits(l1), bits(golden_models["model_test__l1"]))
    # the reference's own goldens and tolerance (model_test.cpp:422-432)
    for i, v in [(0, 2.9909527), (1, -0.216222), (8, 1.6922607), (9, -2.588623)]:
        assert abs(l1[i] - v) < 0.003
    assert abs(l1.sum() - 5.2634663581848145) < 0.003
    l2 = m.forward([int(np.argmax(l1))], 1)
    np.testing.assert_array_equal(bits(l2), bits(golden_models["model_test__l2"]))
    for i, v in [(0, 0.6870570), (1, -2.670202), (8, 0.1438203), (9, -0.409215)]:
        assert abs(l2[i] - v) < 0.003
    assert abs(l2.sum() - 2.540453) < 0.003


@pytest.mark.parametrize("case", ["tiny", "tinycap"])
def test_tiny_model_prefill_decode(oracle, golden_models, case):
    """tinycap: the same model with attention.logit_softcapping 0.25 (model.cpp:511-513)."""
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    extra = {"attention.logit_softcapping": float(golden_models["tinycap__cap"])} if case == "tinycap" else None
    g = build_gemma3_gguf(CONFIGS["tiny"], seed=7, swa_pattern=[True, False, True], extra_meta=extra)
    m = oracle.model(g)
    prompt = golden_models["tiny__prompt"]
    ref_logits, ref_toks = golden_models[f"{case}__logits"], golden_models[f"{case}__tokens"]
    lg = m.forward(prompt, 0)
    np.testing.assert_array_equal(bits(lg), bits(ref_logits[0]))
    pos = len(prompt)
    toks = [int(np.argmax(lg))]
    for i in range(1, len(ref_toks)):
        lg = m.forward([toks[-1]], pos)
        pos += 1
        np.testing.assert_array_equal(bits(lg), bits(ref_logits[i]))
        toks.append(int(np.argmax(lg)))
    assert toks == ref_toks.tolist()
