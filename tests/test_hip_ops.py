"""HIP ops through the C ABI (include/llmi.h) vs the golden vectors of the
reference (tests/golden) and the oracle.

Tolerances (stated here):
  * exact kernels (LLMI_EXACT): bit-identical to the reference for GEMV
    (all types), quantize_row_q8_0/_k, rms_norm, rope, scale,
    vec_scale_f16/vec_mad_f16, dequantize.
  * fast GEMV: |o - o_ref| <= 1e-4 * max|o_ref| + 1e-6 (fp32 reassociation of
    the same exact integer block dots).
  * softmax: device expf, rtol 2e-6.
"""
import numpy as np
import pytest

import cases as K
from llm_inference_amd.gguf import TensorType as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from llm_inference_amd import ops as O
    O.init_ops(0)
    return O


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


@pytest.mark.parametrize("name,tt,r,c", K.GEMV_CASES, ids=[c[0] for c in K.GEMV_CASES])
def test_gemv_exact_bitwise(ops, golden_ops, name, tt, r, c):
    w, x = K.gemv_inputs(name, tt, r, c)
    o = ops.mat_vec_mul_raw(tt, w, r, c, x, exact=True)
    np.testing.assert_array_equal(bits(o), bits(golden_ops[f"gemv__{name}__o"]))


@pytest.mark.parametrize("name,tt,r,c", K.GEMV_CASES, ids=[c[0] for c in K.GEMV_CASES])
def test_gemv_fast_tolerance(ops, golden_ops, name, tt, r, c):
    w, x = K.gemv_inputs(name, tt, r, c)
    o = ops.mat_vec_mul_raw(tt, w, r, c, x, exact=False)
    ref = golden_ops[f"gemv__{name}__o"]
    assert np.abs(o - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6


def test_device_weight_reuse(ops, golden_ops):
    name, tt, r, c = K.GEMV_CASES[1]
    w, x = K.gemv_inputs(name, tt, r, c)
    dw = ops.DeviceWeight(tt, w, r, c)
    for _ in range(3):
        np.testing.assert_array_equal(bits(dw(x, exact=True)), bits(golden_ops[f"gemv__{name}__o"]))


@pytest.mark.parametrize("i", range(len(K.QUANT_CASES)))
def test_quantize_bitwise(ops, golden_ops, i):
    kind, n = K.QUANT_CASES[i]
    x = K.quant_input(kind, n, i)
    y = ops.quantize_row_q8_0(x) if kind == "q8_0" else ops.quantize_row_q8_k(x)
    np.testing.assert_array_equal(y, golden_ops[f"quant__{kind}_{n}__y"])


@pytest.mark.parametrize("n", K.NORM_CASES)
def test_rms_norm(ops, golden_ops, n):
    x = K.norm_input(n)
    ref = golden_ops[f"rms__{n}"]
    np.testing.assert_array_equal(bits(ops.rms_norm(None, x, float(np.float32(1e-6)), exact=True)), bits(ref))
    fast = ops.rms_norm(None, x, float(np.float32(1e-6)), exact=False)
    np.testing.assert_allclose(fast, ref, rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("case", K.ROPE_CASES)
def test_rope_bitwise(ops, golden_ops, case):
    nt, nh, hd, base, pos = case
    got = ops.rope(K.rope_input(nt, nh, hd), hd, base, 1.0, pos)
    np.testing.assert_array_equal(bits(got), bits(golden_ops[f"rope__{nt}_{nh}_{hd}_{int(base)}_{pos}"]))


@pytest.mark.parametrize("tt,n", K.DEQ_CASES)
def test_dequantize_bitwise(ops, golden_ops, tt, n):
    np.testing.assert_array_equal(bits(ops.dequantize_row(tt, K.deq_input(tt, n), n)), bits(golden_ops[f"deq__{tt}_{n}"]))


def test_vec_f16_and_scale(ops, golden_ops):
    rng = np.random.default_rng(6000)
    y = rng.standard_normal(256).astype(np.float16).view(np.uint16)
    xv = rng.standard_normal(256).astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(ops.vec_scale_f16(y, 0.3712), golden_ops["vec__scale"])
    np.testing.assert_array_equal(ops.vec_mad_f16(y, xv, 0.8123), golden_ops["vec__mad"])
    t = np.arange(24, dtype=np.float32).reshape(2, 3, 4)
    np.testing.assert_array_equal(ops.scale(t, 0.37), (t * np.float32(0.37)).astype(np.float32))


@pytest.mark.parametrize("n", K.NORM_CASES)
def test_softmax(ops, golden_ops, n):
    np.testing.assert_allclose(ops.softmax(K.norm_input(n)), golden_ops[f"softmax__{n}"], rtol=2e-6, atol=1e-9)


def test_error_behaviour(ops):
    w = np.zeros(18 * 4, np.uint8)
    with pytest.raises(RuntimeError, match="mat_vec_mul_q4_0: input vector size mismatch"):
        ops.mat_vec_mul_raw(T.Q4_0, w, 4, 32, np.zeros(31, np.float32))
    with pytest.raises(RuntimeError, match="unsupported tensor type 3"):
        ops.mat_vec_mul_raw(3, w, 4, 32, np.zeros(32, np.float32))
    with pytest.raises(RuntimeError, match="eps must be > 0"):
        ops.rms_norm(None, np.ones(4, np.float32), 0.0)


def test_known_answers(ops):
    # ops_test.cpp:17-93 analytic checks
    o = ops.rms_norm(None, [1, 2, 3, 4], float(np.float32(1e-5)))
    ss = np.float32(1.0) / np.sqrt(np.float32(7.5) + np.float32(1e-5))
    np.testing.assert_allclose(o, ss * np.array([1, 2, 3, 4], np.float32), atol=1e-6)
    t = ops.rope([[[1, 2, 3, 4]]], 4, 10000.0, 1.0, 1)
    assert abs(t[0, 0, 0] - -1.984111) < 1e-4 and abs(t[0, 0, 2] - 2.462337) < 1e-4
    w = np.array([0x3c00, 0x4000, 0x4200, 0x4400, 0x4500, 0x4600, 0x4700, 0x4800], np.uint16)
    o = ops.mat_vec_mul_fp16(None, w, [0.5] * 4, 2, 4)
    np.testing.assert_allclose(o, [5.0, 13.0], atol=1e-3)


def test_q4_0_large_random_vs_oracle(ops, oracle):
    # full 4B ffn_down shape (2560 x 10240): exact bitwise vs oracle, fast in tolerance
    from llm_inference_amd.synthetic import random_tensor
    w = random_tensor(T.Q4_0, 2560, 10240, seed=11)
    x = np.random.default_rng(12).standard_normal(10240).astype(np.float32)
    ref = oracle.mat_vec_mul(T.Q4_0, w, 2560, 10240, x)
    np.testing.assert_array_equal(bits(ops.mat_vec_mul_raw(T.Q4_0, w, 2560, 10240, x, exact=True)), bits(ref))
    fast = ops.mat_vec_mul_raw(T.Q4_0, w, 2560, 10240, x)
    assert np.abs(fast - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6


@pytest.mark.parametrize("hd,n_head,n_kv,n_keys", [(256, 8, 4, 12), (256, 4, 1, 77), (128, 8, 4, 300),
                                                   (64, 4, 2, 1), (16, 2, 1, 5), (256, 8, 4, 700),
                                                   (128, 4, 2, 64 * 32 * 2 + 37),  # > 1 tile per split
                                                   (256, 8, 1, 300), (256, 16, 2, 1200)])  # GQA 8 (Gemma-4)
def test_attention(ops, oracle, hd, n_head, n_kv, n_keys):
    """exact: the reference algorithm (f16 V accumulator); differs from the
    oracle only via device expf ulps -> <= 2 f16 ulps of the output scale.
    fast: split-K fp32, pinned to the float64-math oracle (atol 2e-5*max)."""
    import ctypes as C
    rng = np.random.default_rng(hd * 1000 + n_keys)
    q = (rng.standard_normal((n_head, hd)) * 0.08).astype(np.float32)
    k = rng.standard_normal((n_kv, n_keys, hd)).astype(np.float16).view(np.uint16)
    v = rng.standard_normal((n_kv, n_keys, hd)).astype(np.float16).view(np.uint16)
    L = oracle.lib
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
    L.orc_attn_head_f64.argtypes = [f32p, u16p, u16p, C.c_size_t, C.c_size_t, f32p]
    ref = np.zeros_like(q)
    ideal = np.zeros_like(q)
    for h in range(n_head):
        g = h // (n_head // n_kv)
        ref[h] = oracle.attn_head(q[h], k[g], v[g])
        L.orc_attn_head_f64(np.ascontiguousarray(q[h]), np.ascontiguousarray(k[g]), np.ascontiguousarray(v[g]),
                            n_keys, hd, ideal[h])
    ex = ops.attention(q, k, v, exact=True)
    fa = ops.attention(q, k, v, exact=False)
    scale = np.abs(ref).max()
    print(f"exact-vs-ref {np.abs(ex - ref).max():.3g}  fast-vs-f64 {np.abs(fa - ideal).max():.3g}  "
          f"ref-vs-f64 {np.abs(ref - ideal).max():.3g}")
    assert np.abs(ex - ref).max() <= 2 * 2.0 ** -10 * scale
    assert np.abs(fa - ideal).max() <= 2e-5 * scale


def test_gelu_mul(ops, oracle):
    rng = np.random.default_rng(77)
    g = (rng.standard_normal(10240) * 3).astype(np.float32)
    u = rng.standard_normal(10240).astype(np.float32)
    np.testing.assert_allclose(ops.gelu_mul(g, u), oracle.gelu_mul(g, u), rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("cols", [128, 384, 1152, 2560, 3840, 5376, 6144])
@pytest.mark.parametrize("rows", [1, 97, 9000])
def test_f16_logits_widths(ops, rows, cols):
    """Fast F16 GEMV (the logits table) at every width class of the pipelined
    row kernel (cols/8 = 64 P + T lanes, T = 0/16/32/48): vs float64 math on
    the same f16-rounded x (ops.cpp:542-551 rounds x to f16), within the fast
    GEMV budget of the module docstring."""
    rng = np.random.default_rng(rows * 7 + cols)
    w = rng.standard_normal((rows, cols)).astype(np.float16)
    x = rng.standard_normal(cols).astype(np.float32)
    o = ops.mat_vec_mul_raw(T.F16, w.view(np.uint16), rows, cols, x, exact=False)
    ref = w.astype(np.float64) @ x.astype(np.float16).astype(np.float64)
    assert np.abs(o - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6


@pytest.mark.parametrize("rows,cols", [(40, 6912), (37, 1152), (3, 32), (260, 2560)])
def test_gemv_q5_0_fast_vs_oracle(ops, oracle, rows, cols):
    """Fast Q5_0 GEMV (k_gemv.hip gemv_q5_0_fast: the Q4_K_M files' fallback type for 1152-wide tensors,
    ops.cpp:840-893) vs the oracle restatement at ragged shapes: the module's fast-GEMV tolerance; the exact
    kernel stays bit-identical."""
    from llm_inference_amd.synthetic import random_tensor
    w = random_tensor(T.Q5_0, rows, cols, seed=rows + cols)
    x = np.random.default_rng(cols).standard_normal(cols).astype(np.float32)
    ref = oracle.mat_vec_mul(T.Q5_0, w, rows, cols, x)
    np.testing.assert_array_equal(bits(ops.mat_vec_mul_raw(T.Q5_0, w, rows, cols, x, exact=True)), bits(ref))
    o = ops.mat_vec_mul_raw(T.Q5_0, w, rows, cols, x, exact=False)
    assert np.abs(o - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6


@pytest.mark.parametrize("rows,cols", [(5, 8), (300, 96), (77, 2560), (40, 8192), (3, 100)])
def test_gemv_bf16_fast_vs_oracle(ops, oracle, rows, cols):
    """Fast BF16 GEMV (k_gemv.hip gemv_bf16_fast: the Gemma-4 per-layer model projection, ops.cpp:895-931) vs the
    oracle at lane-group widths 8..64 (cols 100: not a multiple of 8, the exact kernel): the fast-GEMV tolerance;
    the exact kernel bit-identical."""
    from llm_inference_amd.synthetic import random_tensor
    w = random_tensor(T.BF16, rows, cols, seed=rows * 7 + cols)
    x = np.random.default_rng(cols + 1).standard_normal(cols).astype(np.float32)
    ref = oracle.mat_vec_mul(T.BF16, w, rows, cols, x)
    np.testing.assert_array_equal(bits(ops.mat_vec_mul_raw(T.BF16, w, rows, cols, x, exact=True)), bits(ref))
    o = ops.mat_vec_mul_raw(T.BF16, w, rows, cols, x, exact=False)
    assert np.abs(o - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6


@pytest.mark.gpu
def test_f16_conversion_selftest():
    """The exact attention's f16 V accumulator (k_exact.hip) rounds with the hardware f32 -> f16 conversion:
    over every one of the 2^32 f32 bit patterns it must equal the reference's f32_to_f16 (gguf.cpp:68-95) for
    every non-NaN input."""
    import ctypes as C
    from llm_inference_amd._lib import check, lib
    out = (C.c_ulonglong * 3)()
    check(lib().llmi_selftest(0, C.cast(out, C.c_void_p)))
    print(f"f32->f16: non-NaN mismatches {out[0]}, NaN mismatches {out[1]}")
    assert out[0] == 0, f"first mismatching f32 bits 0x{out[2]:08x}"


@pytest.mark.gpu
def test_speculative_chain_selftest():
    """The exact engine's rms_norm chain (ops.cpp:33-36: sum = fma(x, x, sum) serially) runs speculatively
    (k_exact.hip xl_chain_spec): its result must equal the serial chain's bits on every vector, including
    vectors whose large terms push the true start of a segment outside the candidate window (serial fallback)."""
    import ctypes as C
    from llm_inference_amd._lib import check, lib
    out = (C.c_ulonglong * 3)()
    check(lib().llmi_selftest(1, C.cast(out, C.c_void_p)))
    print(f"speculative chain: {out[0]} mismatches, {out[1]} fallback segments over 8192 x 7 boundaries")
    assert out[0] == 0
    assert out[1] > 0  # the fallback path ran
