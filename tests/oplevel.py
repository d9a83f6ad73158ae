"""Op-level parity: every kernel the decode graph (and the batched prefill)
launches, checked against the oracle from the DEVICE's own inputs to that
kernel (Model.trace -> llmi_session_trace), so an error in one fused role
cannot hide behind end-to-end drift.

Reference ops restated by the oracle (oracle/llmi_oracle.c, pinned to the
reference's outputs by tests/test_oracle_golden.py):
  embed + scale      model.cpp:240-344        rms_norm / run_norm  ops.cpp:28-43, model.cpp:346-423
  quantize_row_q8_0  ops.cpp:116-139          Q4_0 / Q8_0 GEMV     ops.cpp:188-451, 787-838
  q/k norm, rope     model.cpp:762-794, ops.cpp:67-95             run_attn  model.cpp:430-566
  GELU * up          model.cpp:885-901        residuals           model.cpp:843-858, 915-924
  F16 logits GEMV    ops.cpp:455-612          argmax              main.cpp:193-194

Tolerances (per tensor, why):
  GEMV outputs       |dev - orc| <= 1e-5 * max|orc|: the int8 block dots are
                     exact; only the f32 sum of nb block terms is reassociated
                     (nb * 2^-24 relative to the term magnitude, far below).
  norms / residuals  rtol 2e-6 of max: the squared-sum tree vs the serial fmaf chain.
  attention          vs the float64 restatement 2e-5 of max x sqrt(keys / 256) (fp32 split-K);
                     vs the reference's f16-accumulator algorithm: that algorithm's
                     own drift from exact math (measured on the same inputs) + 4e-5.
  Q8_0 blocks        bit-identical (same floats in, ops.cpp:116-139 exactly).
"""
from __future__ import annotations

import math
from collections import defaultdict

import numpy as np

from llm_inference_amd.gguf import GGUFFile, TensorType as TT

GEMV_RTOL = 1e-5
NORM_RTOL = 2e-6
ATTN_F64_RTOL = 2e-5
GELU_H = {1152: 32, 2560: 40, 3840: 32, 5376: 32}  # k_layer.hip gate/up interleave group by n_embd


def taps_by_layer(taps):
    """[(name, layer, bytes)] -> {(name, layer): [bytes, ...]} in launch order."""
    d = defaultdict(list)
    for name, layer, b in taps:
        d[(name, layer)].append(b)
    return d


def f32(b):
    return np.frombuffer(b, np.float32)


def granule_values(b):
    """{value, tag} 8-B granules -> the 32-bit values (as float32)."""
    return np.frombuffer(b, np.uint32).reshape(-1, 2)[:, 0].copy().view(np.float32)


def xblocks_to_q8_0(words: np.ndarray) -> np.ndarray:
    """Device XBlock rows (48 B: q[32] | d f32 | nsum8 | pad) -> reference
    BlockQ8_0 rows (34 B: d f16 | q[32], ops.h:89-92); checks nsum8."""
    w = np.ascontiguousarray(words, np.uint32).reshape(-1, 12)
    q = w[:, :8].copy().view(np.int8).reshape(-1, 32)
    d = w[:, 8].copy().view(np.float32)
    d16 = d.astype(np.float16)
    assert np.array_equal(d16.astype(np.float32), d), "XBlock scale is not an f16 value"
    nsum8 = w[:, 9].view(np.int32)
    assert np.array_equal(nsum8, -8 * q.astype(np.int32).sum(1)), "XBlock nsum8 != -8 sum(q)"
    out = np.zeros((w.shape[0], 34), np.uint8)
    out[:, :2] = d16.view(np.uint8).reshape(-1, 2)
    out[:, 2:] = q.view(np.uint8)
    return out.reshape(-1)


def xblocks_q8k_to_f32(words: np.ndarray) -> np.ndarray:
    """Device XBlock rows holding Q8_K quants (q8k_block_quad: d = the super-block's f32 d, nsum8 = the
    block's sum of q) -> x' = d q in f32; the reference's quantize_row_q8_k (ops.cpp:142-178) of x' gives back
    the same quants (its max element is d * (+-127)), so mat_vec_mul(w, x') is the reference's row dot on
    these blocks (to one ulp of d)."""
    w = np.ascontiguousarray(words, np.uint32).reshape(-1, 12)
    q = w[:, :8].copy().view(np.int8).reshape(-1, 32)
    d = w[:, 8].copy().view(np.float32)
    assert np.array_equal(w[:, 9].view(np.int32), q.astype(np.int32).sum(1)), "XBlock nsum8 != sum(q)"
    assert np.array_equal(d.reshape(-1, 8), np.repeat(d.reshape(-1, 8)[:, :1], 8, 1)), "Q8_K d differs in a super-block"
    mx, dsb = np.abs(q.reshape(-1, 256)).max(1), d.reshape(-1, 8)[:, 0]
    bad = np.nonzero((mx < 127) & ((dsb != 0) | (mx != 0)))[0]  # an all-zero x gives d = 0 and zero quants
    assert bad.size == 0, f"Q8_K super-blocks {bad[:8].tolist()} without a +-127 quant (max |q| {mx[bad[:8]].tolist()}, d {dsb[bad[:8]].tolist()})"
    return (d[:, None] * q.astype(np.float32)).astype(np.float32).reshape(-1)


def score_sensitivity(q, kc, vc):
    """First-order bound on the relative change of one head's exact attention output when every score carries
    an fp32-sized error e_t = 2 sqrt(hd) 2^-24 sum_i |q16_i k_ti|: max_i sum_t p_t e_t |v_ti - o_i| / max |o|."""
    q16 = np.asarray(q, np.float32).astype(np.float16).astype(np.float64)
    K = np.asarray(kc).view(np.float16).astype(np.float64)
    V = np.asarray(vc).view(np.float16).astype(np.float64)
    sc = K @ q16
    p = np.exp(sc - sc.max())
    p /= p.sum()
    o = p @ V
    e = 2.0 * math.sqrt(q16.size) * 2.0 ** -24 * (np.abs(K) @ np.abs(q16))
    return float(((p * e)[:, None] * np.abs(V - o[None, :])).sum(0).max() / max(float(np.abs(o).max()), 1e-30))


def rel_err(got, ref):
    return float(np.abs(np.asarray(got, np.float64) - ref).max() / max(float(np.abs(ref).max()), 1e-30))


class Weights:
    """Raw GGUF weights of a synthetic Gemma-3 file, by reference tensor name."""

    def __init__(self, buf: np.ndarray):
        self.g = GGUFFile(buf)

    def raw(self, name):
        t = self.g.tensor(name)
        return (np.frombuffer(self.g.get_tensor_data(t), np.uint8), t.tensor_type,
                int(t.shape[1]) if len(t.shape) > 1 else 1, int(t.shape[0]))

    def f32(self, name):
        return self.raw(name)[0].view(np.float32)

    def qkv(self, l):
        """q|k|v stacked as one weight (the session's fused qkv rows)."""
        parts = [self.raw(f"blk.{l}.attn_{p}.weight") for p in "qkv"]
        return np.concatenate([p[0] for p in parts]), parts[0][1], sum(p[2] for p in parts), parts[0][3]


class OpChecker:
    """Checks one traced decode step (or prefill) op by op; records the
    worst relative error per tensor kind in self.report."""

    def __init__(self, oracle, buf, cfg, max_ctx, threads=16, swa_pattern=None):
        self.orc, self.cfg, self.max_ctx, self.th = oracle, cfg, max_ctx, threads
        self.swa_pattern = swa_pattern
        self.w = Weights(buf)
        self.eps = float(np.float32(cfg.eps))
        self.report = defaultdict(float)

    def note(self, kind, err, tol):
        self.report[kind] = max(self.report[kind], err)
        assert err <= tol, f"{kind}: relative error {err:.3g} > {tol:.1g}"

    def norm(self, x, wname):  # run_norm: rms_norm then a separate multiply by the weight
        return self.orc.rms_norm(x, self.eps) * self.w.f32(wname)

    def gemv(self, w, x):
        data, tt, rows, cols = w
        return self.orc.mat_vec_mul(tt, data, rows, cols, x, self.th)

    def gemv_q8(self, w, xq34):
        data, tt, rows, cols = w
        return self.orc.mat_vec_mul_q8(tt, data, rows, cols, xq34, self.th)

    def swa(self, l):  # model.cpp:723-729: the file's pattern, else 5 local layers per global one
        return bool(self.swa_pattern[l]) if self.swa_pattern is not None else (l % 6) < 5

    def attention(self, l, qkv, kc, vc, pos, attn_dev):
        """q/k norm + rope + scale from the device's q|k|v rows, the device's KV
        cache (its row at pos checked against f16 of the oracle's k/v), then
        every head against both attention restatements."""
        c = self.cfg
        hd, nh, nkv = c.head_dim, c.n_head, c.n_head_kv
        q = qkv[: nh * hd].reshape(nh, hd)
        k = qkv[nh * hd: (nh + nkv) * hd].reshape(nkv, hd)
        v = qkv[(nh + nkv) * hd:].reshape(nkv, hd)
        base = 10000.0 if self.swa(l) else c.rope_base
        qn = np.stack([self.norm(q[h], f"blk.{l}.attn_q_norm.weight") for h in range(nh)])
        kn = np.stack([self.norm(k[h], f"blk.{l}.attn_k_norm.weight") for h in range(nkv)])
        qr = self.orc.rope(qn[None], hd, base, 1.0, pos)[0] * np.float32(1.0 / math.sqrt(hd))
        kr = self.orc.rope(kn[None], hd, base, 1.0, pos)[0]
        kc = kc.reshape(nkv, self.max_ctx, hd)
        vc = vc.reshape(nkv, self.max_ctx, hd)
        k16 = kc[:, pos].view(np.float16).astype(np.float32)
        self.note("kv_append_k", rel_err(k16, kr.astype(np.float16).astype(np.float32)), 2e-3)
        assert np.array_equal(vc[:, pos], v.astype(np.float16).view(np.uint16)), "V row at pos != f16(v)"
        g = nh // nkv
        got = attn_dev.reshape(nh, hd)
        ref64 = np.stack([self.orc.attn_head_f64(qr[h], kc[h // g, : pos + 1], vc[h // g, : pos + 1]) for h in range(nh)])
        refr = np.stack([self.orc.attn_head(qr[h], kc[h // g, : pos + 1], vc[h // g, : pos + 1]) for h in range(nh)])
        # fp32 split-K sums: rounding grows like sqrt(keys) (2e-5 up to 256 keys); plus the first-order effect of
        # fp32 scores (an error of ~2 sqrt(hd) 2^-24 sum_i |q_i k_i| per key, through p_t |v_t - o|): large
        # scores (centered K-quant weights) make the exact softmax itself that sensitive
        sens = max(score_sensitivity(qr[h], kc[h // g, : pos + 1], vc[h // g, : pos + 1]) for h in range(nh))
        self.report["attention_score_sensitivity"] = max(self.report["attention_score_sensitivity"], sens)
        self.note("attention_vs_f64", rel_err(got, ref64), ATTN_F64_RTOL * math.sqrt(max(1.0, (pos + 1) / 256.0)) + sens)
        # the reference's own f16 V accumulator drifts from exact math with the
        # key count (~1e-3 at 256 keys, ~7e-3 at 1100): the fast path may differ
        # from it by that drift plus its own distance to exact math
        ref_drift = rel_err(refr, ref64)
        self.report["reference_attention_drift"] = max(self.report["reference_attention_drift"], ref_drift)
        self.note("attention_vs_reference", rel_err(got, refr), ref_drift * 1.01 + 2 * ATTN_F64_RTOL)

    def q8k_blocks(self, words, x, what):
        """Device XBlocks holding Q8_K quants vs the reference's quantize_row_q8_k of x (ops.cpp:142-178),
        bit for bit: per 256-element super-block the f32 d and the 256 quants; returns x' = d q (f32)."""
        xf = xblocks_q8k_to_f32(words)
        w = np.ascontiguousarray(words, np.uint32).reshape(-1, 12)
        ref = np.frombuffer(self.orc.quantize_q8_k(x), np.uint8).reshape(-1, 292)
        assert np.array_equal(w[:, :8].copy().view(np.int8).reshape(-1, 256), ref[:, 4:260].view(np.int8)), \
            f"{what}: Q8_K quants"
        assert np.array_equal(w[:, 8].copy().view(np.float32).reshape(-1, 8)[:, 0], ref[:, :4].copy().view(np.float32)[:, 0]), \
            f"{what}: Q8_K d"
        return xf

    def decode_step(self, taps, pos, gen, token=None):
        """One traced decode step (llmi_session_trace, n_tokens = 1).  Q4_0 / Q8_0 layers read Q8_0 activation
        blocks; K-quant layers (Q4_K / Q6_K in the kq layout) read Q8_K blocks, checked against the reference's
        quantize_row_q8_k and dotted through the reference's mat_vec_mul_q4_k / _q6_k."""
        c = self.cfg
        E, F = c.n_embd, c.n_ff
        T = taps_by_layer(taps)
        one = lambda n, l: T[(n, l)][-1]
        block = ("qkv_g", 0) in T
        kq = self.w.raw("blk.0.attn_q.weight")[1] in (TT.Q4_K, TT.Q6_K)
        for l in range(c.n_layer):
            x = f32(one("attn_norm", l))
            if l == 0:
                if token is not None:  # embed_tokens + scale_embeddings (model.cpp:240-344), then attn_norm
                    data, tt, rows, cols = self.w.raw("token_embd.weight")
                    row = self.orc.dequantize_row(tt, data[token * (data.size // rows):(token + 1) * (data.size // rows)], cols)
                    emb = row * np.float32(math.sqrt(E))
                    assert np.array_equal(f32(one("inp_scaled", -1)), emb), "embedding row * sqrt(n_embd)"
                self.note("norm", rel_err(x, self.norm(f32(one("inp_scaled", -1)), "blk.0.attn_norm.weight")), NORM_RTOL)
            else:
                r_prev = f32(one("ffn_resid", l - 1))
                y = f32(one("down", l - 1))
                r = r_prev + self.norm(y, f"blk.{l - 1}.post_ffw_norm.weight")
                got_r = f32(one("attn_resid", l))
                self.note("residual", rel_err(got_r, r), NORM_RTOL)
                self.note("norm", rel_err(x, self.norm(got_r, f"blk.{l}.attn_norm.weight")), NORM_RTOL)
            wqkv = self.w.qkv(l)
            qkv = granule_values(one("qkv_g", l)) if block else f32(one("qkv", l))
            if kq:  # q, k, v per tensor (Q4_K_M: q|k Q4_K, v Q6_K); every row's dot is independent of the stacking
                xin = x
                if l == 0 and ("xq", 0) in T:  # layer 0 reads embed_norm's block_q8_K rows (292 B, ops.h:18-23)
                    b = np.frombuffer(one("xq", 0), np.uint8)
                    assert b.size == E // 256 * 292 and np.array_equal(b, self.orc.quantize_q8_k(x)), "embed_norm Q8_K blocks"
                    sb = b.reshape(-1, 292)
                    xin = (sb[:, :4].copy().view(np.float32) * sb[:, 4:260].view(np.int8).astype(np.float32)).reshape(-1)
                ref = np.concatenate([self.gemv(self.w.raw(f"blk.{l}.attn_{p}.weight"), xin) for p in "qkv"])
            elif l == 0 and ("xq", 0) in T:  # layer 0 reads embed_norm's Q8_0 blocks
                xq = xblocks_to_q8_0(np.frombuffer(one("xq", 0), np.uint32))
                assert np.array_equal(xq, self.orc.quantize_q8_0(x)), "embed_norm Q8_0 blocks"
                ref = self.gemv_q8(wqkv, xq)
            else:
                ref = self.gemv(wqkv, x)
            self.note("gemv_qkv", rel_err(qkv, ref), GEMV_RTOL)
            attn = f32(one("attn", l))
            self.attention(l, qkv, np.frombuffer(one("kc", l), np.uint16), np.frombuffer(one("vc", l), np.uint16),
                           pos, attn)
            xo_words = granule_values(one("xo_g", l)).view(np.uint32) if block else np.frombuffer(one("xo", l), np.uint32)
            o = f32(one("o", l))
            if kq:
                xof = self.q8k_blocks(xo_words[: c.n_head * c.head_dim // 32 * 12], attn, f"layer {l}: attention")
                self.note("gemv_o", rel_err(o, self.gemv(self.w.raw(f"blk.{l}.attn_output.weight"), xof)), GEMV_RTOL)
            else:
                xo = xblocks_to_q8_0(xo_words)
                assert np.array_equal(xo, self.orc.quantize_q8_0(attn)), f"layer {l}: attention Q8_0 blocks"
                self.note("gemv_o", rel_err(o, self.gemv_q8(self.w.raw(f"blk.{l}.attn_output.weight"), xo)), GEMV_RTOL)
            r_in = f32(one("attn_resid", l)) if l else f32(one("inp_scaled", -1))
            r2 = r_in + self.norm(o, f"blk.{l}.post_attention_norm.weight")
            got_r2 = f32(one("ffn_resid", l))
            self.note("residual", rel_err(got_r2, r2), NORM_RTOL)
            xf = f32(one("ffn_norm", l))
            self.note("norm", rel_err(xf, self.norm(got_r2, f"blk.{l}.ffn_norm.weight")), NORM_RTOL)
            gate = self.gemv(self.w.raw(f"blk.{l}.ffn_gate.weight"), xf)
            up = self.gemv(self.w.raw(f"blk.{l}.ffn_up.weight"), xf)
            hid = f32(one("hid", l))
            assert np.abs(hid).max() > 0, f"layer {l}: the FFN is dead (GELU output all zero): the check would be vacuous"
            # GELU(g) * u with g, u each within GEMV_RTOL of max: |d hid| <~ (|GELU'| + 1) max|g| max|u| GEMV_RTOL
            err = float(np.abs(hid - self.orc.gelu_mul(gate, up)).max()) / (float(np.abs(gate).max() * np.abs(up).max()) + 1e-30)
            self.note("gemv_gate_up_gelu", err, 3 * GEMV_RTOL)
            d = f32(one("down", l))
            self.note("gemv_down", rel_err(d, self.gemv(self.w.raw(f"blk.{l}.ffn_down.weight"), hid)), GEMV_RTOL)
        rf = f32(one("ffn_resid", c.n_layer - 1)) + self.norm(f32(one("down", c.n_layer - 1)),
                                                              f"blk.{c.n_layer - 1}.post_ffw_norm.weight")
        self.note("residual", rel_err(f32(one("final_resid", -1)), rf), NORM_RTOL)
        xn = f32(one("result_norm", -1))
        self.note("norm", rel_err(xn, self.norm(f32(one("final_resid", -1)), "output_norm.weight")), NORM_RTOL)
        logits = self.gemv(self.w.raw("token_embd.weight"), xn)
        if ("logits", -1) in T:
            self.note("gemv_logits_f16", rel_err(f32(one("logits", -1)), logits), GEMV_RTOL)
        tok = int(np.frombuffer(one("token", -1), np.int32)[0])
        top = np.sort(logits)[-2:]
        if top[1] - top[0] > 1e-5 * abs(top[1]):  # not a near-tie at f32 resolution: the id is determined
            assert tok == int(np.argmax(logits)), f"token {tok} vs oracle argmax {int(np.argmax(logits))}"
        return tok

    def prefill(self, taps, T_tok):
        """Traced batched prefill: every projection GEMM, token by token, from
        the device's own inputs -- Q8_0 blocks (int8 GEMM v5 vs the reference's
        per-token mat_vec_mul rows, GEMV tolerance) or f16 rows (the f16 GEMMs v7 /
        v6 vs the exactly dequantized weights times those f16 values, times the
        token's scale 2^s, in float64: the kernel's weights are f16(d (q - 8)),
        PREFILL16_RTOL).  Each tap's format from its size: the f16 path's last
        layer runs its one remaining token on the int8 path."""
        c = self.cfg
        E, F = c.n_embd, c.n_ff
        D = taps_by_layer(taps)
        H = GELU_H[E]
        xs = max(E, F, c.n_head * c.head_dim) // 32  # activation blocks per token (session pf_xs_)
        row_bytes = len(D[("pf_x_qkv", 0)][-1]) // T_tok
        assert row_bytes in (48 * xs, 64 * xs), f"prefill activation row of {row_bytes} B"
        for l in range(c.n_layer):
            for proj, names, ncols in (("qkv", [f"blk.{l}.attn_{p}.weight" for p in "qkv"], E),
                                       ("o", [f"blk.{l}.attn_output.weight"], c.n_head * c.head_dim),
                                       ("gate_up", None, E),
                                       ("down", [f"blk.{l}.ffn_down.weight"], F)):
                nbytes = len(D[(f"pf_x_{proj}", l)][-1])
                f16_rows = nbytes % (64 * xs) == 0 and (nbytes // (64 * xs) == T_tok or nbytes == 64 * xs)
                if f16_rows and row_bytes == 64 * xs:
                    self._prefill_f16_one(D, l, proj, names, ncols, nbytes // (64 * xs), H)
                else:
                    self._prefill_q8_one(D, l, proj, names, ncols, nbytes // (48 * xs), H)

    def _prefill_q8_one(self, D, l, proj, names, ncols, n_t, H):
        c = self.cfg
        F = c.n_ff
        kq_types = (TT.Q4_K, TT.Q6_K)
        xs = np.frombuffer(D[(f"pf_x_{proj}", l)][-1], np.uint32).reshape(n_t, -1, 12)
        out = f32(D[(f"pf_{proj}", l)][-1]).reshape(n_t, -1)
        ws = [self.w.raw(n) for n in (names or [f"blk.{l}.ffn_gate.weight", f"blk.{l}.ffn_up.weight"])]
        kq = ws[0][1] in kq_types  # Q8_K activation blocks (K-quant layers), else Q8_0
        for t in range(n_t):
            if kq:
                try:
                    xf = xblocks_q8k_to_f32(xs[t, : ncols // 32])
                except AssertionError as e:
                    raise AssertionError(f"layer {l} {proj} token {t}: {e}") from None
                dot = lambda w: self.gemv(w, xf)  # noqa: E731
            else:
                xq = xblocks_to_q8_0(xs[t, : ncols // 32])
                dot = lambda w: self.gemv_q8(w, xq)  # noqa: E731
            if proj == "gate_up":
                g, u = dot(ws[0]), dot(ws[1])
                ref = np.concatenate([np.concatenate([g[k * H:(k + 1) * H], u[k * H:(k + 1) * H]])
                                      for k in range(F // H)])
            else:
                ref = np.concatenate([dot(w) for w in ws])
            self.note(f"prefill_gemm_{proj}", rel_err(out[t, : ref.size], ref), GEMV_RTOL)

    def _prefill_f16_one(self, D, l, proj, names, ncols, n_t, H):
        c = self.cfg
        F = c.n_ff
        x = np.frombuffer(D[(f"pf_x_{proj}", l)][-1], np.float16).reshape(n_t, -1)[:, :ncols].astype(np.float64)
        if (f"pf_xs_{proj}", l) in D:  # the rows' per-token scales 2^s (the attention's rows: none)
            ts = f32(D[(f"pf_xs_{proj}", l)][-1]).astype(np.float64)
            assert ts.size == n_t and np.all(ts > 0) and np.all(np.frexp(ts)[0] == 0.5), "token scales: powers of two"
            x = x * ts[:, None]
        out = f32(D[(f"pf_{proj}", l)][-1]).reshape(n_t, -1)
        if proj == "gate_up":
            g = self.dequant(self.w.raw(f"blk.{l}.ffn_gate.weight"))
            u = self.dequant(self.w.raw(f"blk.{l}.ffn_up.weight"))
            W = np.concatenate([np.concatenate([g[k * H:(k + 1) * H], u[k * H:(k + 1) * H]]) for k in range(F // H)])
        else:
            W = np.concatenate([self.dequant(self.w.raw(n)) for n in names])
        ref = x @ W.T
        for t in range(n_t):
            self.note(f"prefill_gemm16_{proj}", rel_err(out[t, : ref.shape[1]], ref[t]), PREFILL16_RTOL)

    def dequant(self, w):
        """Weight rows -> float64: Q4_0 in numpy, other types through the oracle's dequantize_row."""
        data, tt, rows, cols = w
        if tt == TT.Q4_0:
            return dequant_q4_0(w)
        rb = data.size // rows
        return np.stack([np.asarray(self.orc.dequantize_row(tt, data[i * rb:(i + 1) * rb], cols), np.float64)
                         for i in range(rows)])


PREFILL16_RTOL = 2e-3


def dequant_q4_0(w):
    """Q4_0 rows -> float64 (d * (q - 8); ops.h block layout: f16 d, 16 bytes, element i = low nibble of byte
    i, element i + 16 = high nibble)."""
    data, tt, rows, cols = w
    assert tt == TT.Q4_0, "f16 prefill GEMM check: Q4_0 weights only"
    b = data.reshape(rows, cols // 32, 18)
    d = b[:, :, :2].copy().view(np.float16).astype(np.float64)[:, :, 0]
    qs = b[:, :, 2:]
    q = np.concatenate([qs & 15, qs >> 4], axis=2).astype(np.float64) - 8.0
    return (q * d[:, :, None]).reshape(rows, cols)

