"""Op-level parity of the kernels the fast decode graph and the batched
prefill actually launch (VERDICT r1 'What's weak' 3): the attention block
(qkv GEMV with the residual/norm prologue, split attention with q/k norm,
rope and KV append, merge + Q8_0, o GEMV), the gate_up launch (prologue +
GELU epilogue, slab weights), the down launch (QUANT prologue), the final
norm, the logits / screened token, and every prefill_gemm_kernel output
row -- each against the oracle restatement of the reference op computed
from the device's OWN inputs to that launch (tests/oplevel.py states the
per-tensor tolerances and why)."""
import os

import numpy as np
import pytest

from oplevel import OpChecker

pytestmark = pytest.mark.gpu


def _run(oracle, cfg_name, seed, n_prompt, n_decode, max_ctx, monkeypatch=None, env=None, check_prefill=True,
         **gkw):
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    swa = gkw.get("swa_pattern")
    g = build_gemma3_gguf(cfg, seed=seed, **gkw)
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    m = Model(g, max_ctx=max_ctx)
    chk = OpChecker(oracle, g, cfg, max_ctx, swa_pattern=swa)
    prompt = np.random.default_rng(seed).integers(4, cfg.vocab, n_prompt).astype(np.int32)
    taps = m.trace(prompt, 0)
    if check_prefill and m.info.batched_prefill:
        chk.prefill(taps, n_prompt)
    if n_decode < 0:  # prefill GEMMs only (the decode op checks assume Q8_0 activations)
        print(cfg_name, env or "", {k: f"{v:.2e}" for k, v in sorted(chk.report.items())})
        m.close()
        return chk
    tok = int(np.frombuffer([b for n, l, b in taps if n == "token"][-1], np.int32)[0])
    pos = n_prompt
    for _ in range(n_decode):
        tok = chk.decode_step(m.trace([tok], pos, gen=True), pos, gen=True, token=tok)
        pos += 1
    # forward()'s full F16 logits launch as well (not the screened selection)
    chk.decode_step(m.trace([tok], pos), pos, gen=False, token=tok)
    print(cfg_name, env or "", {k: f"{v:.2e}" for k, v in sorted(chk.report.items())})
    m.close()
    return chk


def test_ops_mini4b_block(oracle):
    """Gemma-3 4B layer shapes on the attention-block path, global and local
    rope layers; prefill GEMMs of a 12-token prompt, then 3 decode steps."""
    chk = _run(oracle, "mini-4b", 21, 12, 3, 64, swa_pattern=[True, False])
    assert "gemv_qkv" in chk.report and "prefill_gemm16_gate_up" in chk.report  # the f16 prefill (GEMM v7 / v6)


def test_ops_mini4b_three_launch_attention(oracle, monkeypatch):
    """LLMI_NO_BLOCK=1: standalone PRO/PLAIN layer GEMVs and the split
    attention kernel (the launches the block replaces)."""
    _run(oracle, "mini-4b", 22, 9, 2, 64, monkeypatch, {"LLMI_NO_BLOCK": "1"}, check_prefill=False,
         swa_pattern=[False, True])


def test_ops_mini1b_block(oracle):
    _run(oracle, "mini-1b", 23, 12, 3, 64, swa_pattern=[True, False])


def test_ops_mini4b_int8_prefill(oracle, monkeypatch):
    """The int8 batched prefill (LLMI_PREFILL_F16=0: Q8_0 activation blocks, GEMM v5) op by op: every GEMM row
    against the reference's Q8_0 x Q4_0 rows of the device's own blocks (GEMV tolerance)."""
    chk = _run(oracle, "mini-4b", 21, 12, 1, 64, monkeypatch, {"LLMI_PREFILL_F16": "0"}, swa_pattern=[True, False])
    assert "prefill_gemm_gate_up" in chk.report and "prefill_gemm_down" in chk.report


def test_ops_mini1b_q8_0_fused(oracle):
    """Q8_0 weights in the fused layer launch table (W8 entries) and in the batched prefill (GEMM v5 with the
    Q8_0 blocks as the int8 A operand): every prefill GEMM row against the reference's Q8_0 x Q8_0 rows."""
    from llm_inference_amd.gguf import TensorType as TT
    chk = _run(oracle, "mini-1b", 24, 10, 2, 64, wtype=TT.Q8_0)
    assert "prefill_gemm_qkv" in chk.report and "prefill_gemm_down" in chk.report


def test_ops_mini1b_long_context(oracle):
    """64-key attention tiles (pos + 1 > 32 x 32 splits): 1100-token prefill,
    then decode steps checked op by op at pos 1100-1101."""
    _run(oracle, "mini-1b", 25, 1100, 2, 1200, check_prefill=False)


def test_ops_mini27b_shapes(oracle):
    """Gemma-3 27B layer shapes (5376 / 21504 columns, 32 / 16 heads of 128)."""
    _run(oracle, "mini-27b", 26, 8, 2, 64, swa_pattern=[True, False])


@pytest.mark.parametrize("cfg_name,env", [("mini-4b", {}), ("mini-27b", {}), ("mini-1b", {}),
                                          ("mini-4b", {"LLMI_PG7": "128x64"}), ("mini-4b", {"LLMI_PG6": "1"})])
def test_ops_prefill_f16_gemm(oracle, monkeypatch, cfg_name, env):
    """The default f16 prefill of Q4_0 layers: f16 rows of the dequantized Q8_0 activation blocks scaled per token
    by 2^-s from the norm / attention / GELU producers, GEMM v7 (weights dequantized once per work-group to f16 in
    LDS, v_mfma_f32_32x32x16_f16 over all of K; another tile geometry; GEMM v6 on the same rows): every GEMM output
    row against the exactly dequantized weights times the device's own f16 inputs times the token's 2^s in
    float64 (tests/oplevel.py PREFILL16_RTOL)."""
    chk = _run(oracle, cfg_name, 27, 40, 1, 64, monkeypatch, env)
    assert "prefill_gemm16_gate_up" in chk.report and "prefill_gemm16_down" in chk.report


def test_ops_prefill_kquant_gemm(oracle, monkeypatch):
    """Gemma-3 4B Q4_K_M layer shapes (q, k, o, gate, up Q4_K; v, down Q6_K in the kq layout): the opt-in
    f16 batched prefill (LLMI_PREFILL_F16=1), GEMM v6 dequantizing the K-quant sub-blocks to f16 -- every output
    row against the reference's dequantize_row weights times the device's own f16 inputs in float64."""
    from llm_inference_amd.gguf import TensorType as TT
    chk = _run(oracle, "mini-4b", 29, 24, -1, 64, monkeypatch, {"LLMI_PREFILL_F16": "1"}, wtype=TT.Q4_K,
               wtypes={"v": TT.Q6_K, "down": TT.Q6_K})
    assert "prefill_gemm16_qkv" in chk.report and "prefill_gemm16_down" in chk.report


@pytest.mark.parametrize("vtype", ["q6_k", "q4_k"])
def test_ops_prefill_kquant_int8(oracle, vtype):
    """The default K-quant batched prefill: Q8_K activation blocks from the norm / attention / GELU producers
    (the reference's quantize_row_q8_k, checked block by block: one f32 d per super-block, a +-127 quant in
    each, block sums) and the int8 GEMM's Q4_K / Q6_K variant (i8 MFMA per sub-block, the d sc / dmin m
    scale products on f32 MFMAs) -- every output row against the reference's mat_vec_mul_q4_k / _q6_k of
    those blocks (GEMV tolerance); then 3 decode steps op by op through the FUSED kq launches: the attention
    block (q|k Q4_K + v Q6_K, or all Q4_K, as its qkv role; Q8_K blocks of x from the prologue and of the
    attention output from the merge, checked bit for bit against quantize_row_q8_k; o Q4_K), the slab-major
    Q4_K gate_up with the GELU epilogue and the Q6_K / Q4_K down launch."""
    from llm_inference_amd.gguf import TensorType as TT
    vt = TT.Q6_K if vtype == "q6_k" else TT.Q4_K
    chk = _run(oracle, "mini-4b", 30, 20, 3, 64, wtype=TT.Q4_K, wtypes={"v": vt, "down": vt},
               swa_pattern=[True, False], centered=True)
    assert "prefill_gemm_qkv" in chk.report and "prefill_gemm_down" in chk.report
    assert "gemv_qkv" in chk.report and "gemv_o" in chk.report and "gemv_down" in chk.report
