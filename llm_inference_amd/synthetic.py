"""Synthetic Gemma-3 GGUF models and random quantized tensors.

There are no real checkpoints (and no network) in this environment, so the
benchmark and the parity tests run on random-init weights with the exact
architecture/shape of the BASELINE.json configs, written as
real GGUF v3 files that the reference's loader accepts unchanged.

Random block contents follow SURVEY.md section 8(d): Q4_0 nibbles uniform 0..15,
block scale d = fp16(U[0.002, 0.02]).  Everything is seeded (numpy PCG64).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from .gguf import GGUFBuilder, TensorType, row_bytes


# ---------------------------------------------------------------------------
# configs (the 'tiny'/'mini' ones are test-sized)
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class Gemma3Config:
    name: str
    n_layer: int
    n_embd: int
    n_ff: int
    n_head: int
    n_head_kv: int
    head_dim: int
    vocab: int
    rope_base: float = 1000000.0
    eps: float = 1e-6

    @property
    def q_rows(self):
        return self.n_head * self.head_dim

    @property
    def kv_rows(self):
        return self.n_head_kv * self.head_dim


CONFIGS: Dict[str, Gemma3Config] = {
    "gemma-3-1b": Gemma3Config("gemma-3-1b", 26, 1152, 6912, 4, 1, 256, 262144),
    "gemma-3-4b": Gemma3Config("gemma-3-4b", 34, 2560, 10240, 8, 4, 256, 262208),
    "gemma-3-27b": Gemma3Config("gemma-3-27b", 62, 5376, 21504, 32, 16, 128, 262208),
    # reduced shapes for tests (same head/GQA structure, few layers, small vocab)
    "mini-4b": Gemma3Config("mini-4b", 2, 2560, 10240, 8, 4, 256, 4096),
    "mini-1b": Gemma3Config("mini-1b", 2, 1152, 6912, 4, 1, 256, 2048),
    "mini-27b": Gemma3Config("mini-27b", 2, 5376, 21504, 32, 16, 128, 4096),
    "tiny": Gemma3Config("tiny", 3, 256, 512, 4, 2, 64, 512),
}


# ---------------------------------------------------------------------------
# random tensor payloads (GGUF block layouts, ops.h:11-31, 89-102)
# ---------------------------------------------------------------------------
def _f16_bits(x: np.ndarray) -> np.ndarray:
    return np.asarray(x, dtype=np.float32).astype(np.float16).view(np.uint16)


def fill_random(out: np.ndarray, ttype: int, n_rows: int, n_cols: int, rng: np.random.Generator,
                scale_lo: float = 0.002, scale_hi: float = 0.02, centered: bool = False) -> None:
    """Fill ``out`` (uint8 view of exactly the tensor's bytes) with random blocks.
    centered: Q4_0 nibbles uniform on 1..15 (q - 8 symmetric, zero mean, like
    trained weights) instead of 0..15 (mean -0.5: every projection then adds a
    fixed common-mode direction and a deep random model decodes one token
    forever)."""
    if ttype == TensorType.Q4_0:
        blk = out.reshape(-1, 18)
        if centered:
            lo = rng.integers(1, 16, size=(blk.shape[0], 16), dtype=np.uint8)
            hi = rng.integers(1, 16, size=(blk.shape[0], 16), dtype=np.uint8)
            blk[:, 2:] = lo | (hi << 4)
        else:
            blk[:, 2:] = rng.integers(0, 256, size=(blk.shape[0], 16), dtype=np.uint8)
        blk[:, 0:2] = _f16_bits(rng.uniform(scale_lo, scale_hi, blk.shape[0])).view(np.uint8).reshape(-1, 2)
    elif ttype == TensorType.Q8_0:
        blk = out.reshape(-1, 34)
        blk[:, 2:] = rng.integers(-127, 128, size=(blk.shape[0], 32), dtype=np.int8).view(np.uint8)
        blk[:, 0:2] = _f16_bits(rng.uniform(scale_lo, scale_hi, blk.shape[0]) / 8).view(np.uint8).reshape(-1, 2)
    elif ttype == TensorType.Q5_0:
        blk = out.reshape(-1, 22)
        blk[:, 2:] = rng.integers(0, 256, size=(blk.shape[0], 20), dtype=np.uint8)
        blk[:, 0:2] = _f16_bits(rng.uniform(scale_lo, scale_hi, blk.shape[0]) / 2).view(np.uint8).reshape(-1, 2)
    elif ttype == TensorType.Q4_K and centered:
        # w = d sc q - dmin m (ops.cpp:633-641 get_scale_min_k4) with m = sc and dmin = 7.5 d: w = d sc (q - 7.5),
        # zero mean like trained weights (random mins make every projection's output one-signed: a dead FFN)
        blk = out.reshape(-1, 144)
        nb = blk.shape[0]
        blk[:, 16:] = rng.integers(0, 256, size=(nb, 128), dtype=np.uint8)
        sc = rng.integers(1, 64, size=(nb, 8), dtype=np.uint8)
        sb = np.zeros((nb, 12), np.uint8)
        sb[:, 0:4] = sc[:, 0:4] | ((sc[:, 4:8] >> 4) << 6)
        sb[:, 4:8] = sc[:, 0:4] | ((sc[:, 4:8] >> 4) << 6)
        sb[:, 8:12] = (sc[:, 4:8] & 15) | ((sc[:, 4:8] & 15) << 4)
        blk[:, 4:16] = sb
        d = rng.uniform(scale_lo, scale_hi, nb).astype(np.float32) / 64  # d sc ~ Q4_0 scale range
        d16 = d.astype(np.float16)
        blk[:, 0:2] = d16.view(np.uint16).view(np.uint8).reshape(-1, 2)
        blk[:, 2:4] = _f16_bits(d16.astype(np.float32) * 7.5).view(np.uint8).reshape(-1, 2)
    elif ttype == TensorType.Q4_K:
        blk = out.reshape(-1, 144)
        blk[:, 4:] = rng.integers(0, 256, size=(blk.shape[0], 140), dtype=np.uint8)
        blk[:, 0:2] = _f16_bits(rng.uniform(scale_lo, scale_hi, blk.shape[0]) / 16).view(np.uint8).reshape(-1, 2)
        blk[:, 2:4] = _f16_bits(rng.uniform(scale_lo, scale_hi, blk.shape[0]) / 16).view(np.uint8).reshape(-1, 2)
    elif ttype == TensorType.Q6_K:
        blk = out.reshape(-1, 210)
        blk[:, :192] = rng.integers(0, 256, size=(blk.shape[0], 192), dtype=np.uint8)
        blk[:, 192:208] = rng.integers(-64, 64, size=(blk.shape[0], 16), dtype=np.int8).view(np.uint8)
        blk[:, 208:210] = _f16_bits(rng.uniform(scale_lo, scale_hi, blk.shape[0]) / 64).view(np.uint8).reshape(-1, 2)
    elif ttype in (TensorType.F16,):
        # sign | exponent in [7, 11] (|w| ~ 2^-8 .. 2^-4) | random mantissa;
        # centered: [4, 8] (|w| ~ 2^-11 .. 2^-7), so with tied embeddings the
        # token's own row no longer dominates the final state and greedy
        # decoding does not just repeat its input
        bits = rng.integers(0, 1 << 16, size=out.size // 2, dtype=np.uint16)
        e0 = 4 if centered else 7
        exp = (rng.integers(e0, e0 + 5, size=bits.size, dtype=np.uint16) << 10)
        out.view(np.uint16)[:] = (bits & np.uint16(0x83FF)) | exp
    elif ttype == TensorType.BF16:
        v = rng.normal(0, 0.02, size=out.size // 2).astype(np.float32)
        out.view(np.uint16)[:] = (v.view(np.uint32) >> 16).astype(np.uint16)
    elif ttype == TensorType.F32:
        out.view(np.float32)[:] = rng.normal(0, 1, size=out.size // 4).astype(np.float32)
    else:
        raise ValueError(ttype)


def random_tensor(ttype: int, n_rows: int, n_cols: int, seed: int = 0, **kw) -> np.ndarray:
    out = np.zeros(row_bytes(ttype, n_cols) * n_rows, dtype=np.uint8)
    fill_random(out, ttype, n_rows, n_cols, np.random.default_rng(seed), **kw)
    return out


# ---------------------------------------------------------------------------
# synthetic Gemma-3 model
# ---------------------------------------------------------------------------
def build_gemma3_gguf(cfg: Gemma3Config, seed: int = 0, wtype: int = TensorType.Q4_0,
                      embd_type: int = TensorType.F16, wtypes: Optional[Dict[str, int]] = None,
                      swa_pattern: Optional[list] = None, centered: bool = False,
                      pieces: Optional[list] = None, extra_meta: Optional[Dict[str, object]] = None) -> np.ndarray:
    """Random-init Gemma-3 GGUF with the tensor names/shapes model.cpp maps
    (model.cpp:169-238).  Returns the whole file as a uint8 numpy array.
    extra_meta: more metadata keys (without the "gemma3." prefix)."""
    rng = np.random.default_rng(seed)
    b = GGUFBuilder(align_tensors=True)
    a = "gemma3"
    b.add_meta("general.architecture", a)
    b.add_meta(f"{a}.block_count", cfg.n_layer)
    b.add_meta(f"{a}.embedding_length", cfg.n_embd)
    b.add_meta(f"{a}.feed_forward_length", cfg.n_ff)
    b.add_meta(f"{a}.attention.head_count", cfg.n_head)
    b.add_meta(f"{a}.attention.head_count_kv", cfg.n_head_kv)
    b.add_meta(f"{a}.attention.key_length", cfg.head_dim)
    b.add_meta(f"{a}.attention.value_length", cfg.head_dim)
    b.add_meta(f"{a}.attention.layer_norm_rms_epsilon", float(cfg.eps))
    b.add_meta(f"{a}.rope.freq_base", float(cfg.rope_base))
    if swa_pattern is not None:
        b.add_meta(f"{a}.attention.sliding_window_pattern", [bool(x) for x in swa_pattern])
    for k, v in (extra_meta or {}).items():
        b.add_meta(f"{a}.{k}", v)
    toks = ["<pad>", "<eos>", "<bos>", "<unk>"] + [f"t{i}" for i in range(4, cfg.vocab)]
    for i, p in enumerate(pieces or []):  # real vocabulary pieces at ids 4.. (the tokenizer's greedy longest match)
        toks[4 + i] = p
    b.add_meta("tokenizer.ggml.tokens", toks)
    b.add_meta("tokenizer.ggml.bos_token_id", 2)
    b.add_meta("tokenizer.ggml.eos_token_id", 1)

    wt = dict(q=wtype, k=wtype, v=wtype, o=wtype, gate=wtype, up=wtype, down=wtype)
    if wtypes:
        wt.update(wtypes)
    E, F = cfg.n_embd, cfg.n_ff
    specs = [("token_embd.weight", [E, cfg.vocab], embd_type),
             ("output_norm.weight", [E], TensorType.F32)]
    for l in range(cfg.n_layer):
        p = f"blk.{l}."
        specs += [
            (p + "attn_norm.weight", [E], TensorType.F32),
            (p + "attn_q.weight", [E, cfg.q_rows], wt["q"]),
            (p + "attn_k.weight", [E, cfg.kv_rows], wt["k"]),
            (p + "attn_v.weight", [E, cfg.kv_rows], wt["v"]),
            (p + "attn_q_norm.weight", [cfg.head_dim], TensorType.F32),
            (p + "attn_k_norm.weight", [cfg.head_dim], TensorType.F32),
            (p + "attn_output.weight", [cfg.q_rows, E], wt["o"]),
            (p + "post_attention_norm.weight", [E], TensorType.F32),
            (p + "ffn_norm.weight", [E], TensorType.F32),
            (p + "ffn_gate.weight", [E, F], wt["gate"]),
            (p + "ffn_up.weight", [E, F], wt["up"]),
            (p + "ffn_down.weight", [F, E], wt["down"]),
            (p + "post_ffw_norm.weight", [E], TensorType.F32),
        ]
    for name, shape, tt in specs:
        b.add_tensor(name, shape, tt)
    buf, views = b.finalize()
    for name, shape, tt in specs:
        v = views[name]
        if tt == TensorType.F32:  # norm weights (llama.cpp stores Gemma's 1+w)
            v.view(np.float32)[:] = rng.uniform(0.6, 1.4, size=v.size // 4).astype(np.float32)
        else:
            n_rows = shape[1] if len(shape) > 1 else 1
            fill_random(v, tt, n_rows, shape[0], rng, centered=centered)
    return buf


@dataclass(frozen=True)
class Gemma4Config:
    """Gemma-4 structure the reference supports (model.cpp:58-167, 568-704,
    706-980): per-layer token embeddings + their model projection, shared KV
    for the last layers, V RMSNorm, per-layer output scale, attention scale 1,
    separate sliding-window / global head dims."""
    name: str
    n_layer: int
    n_embd: int
    n_ff: int
    n_head: int
    n_head_kv: int
    head_dim: int       # global layers (attention.key_length)
    head_dim_swa: int   # sliding-window layers (attention.key_length_swa)
    n_embd_per_layer: int
    shared_kv_layers: int
    vocab: int
    rope_base: float = 1000000.0
    eps: float = 1e-6


CONFIGS4: Dict[str, Gemma4Config] = {
    "tiny4": Gemma4Config("tiny4", 4, 256, 512, 4, 1, 128, 64, 64, 2, 512),
    "mini4": Gemma4Config("mini4", 6, 1536, 6144, 8, 1, 256, 256, 256, 2, 4096),
}


def build_gemma4_gguf(cfg: Gemma4Config, seed: int = 0, wtype: int = TensorType.Q4_0,
                      ple_type: int = TensorType.BF16, table_type: int = TensorType.F16,
                      swa_pattern: Optional[list] = None, centered: bool = True) -> np.ndarray:
    """Random-init GGUF with the reference's Gemma-4 tensor map
    (model.cpp:169-238): token_embd_per_layer [n_embd_per_layer * n_layer,
    vocab], per_layer_model_proj [n_embd -> n_embd_per_layer * n_layer],
    per_layer_proj_norm; per layer inp_gate / proj (the per-layer embedding
    step) and post_norm, out_scale; no attn_k / attn_v for the shared-KV
    layers (model.cpp:775-777 never reads them)."""
    rng = np.random.default_rng(seed)
    b = GGUFBuilder(align_tensors=True)
    a = "gemma4"
    L, E, F, Ep = cfg.n_layer, cfg.n_embd, cfg.n_ff, cfg.n_embd_per_layer
    pattern = swa_pattern if swa_pattern is not None else [(l % 6) < 5 for l in range(L)]
    b.add_meta("general.architecture", a)
    for k, v in (("block_count", L), ("embedding_length", E), ("feed_forward_length", F),
                 ("attention.head_count", cfg.n_head), ("attention.head_count_kv", cfg.n_head_kv),
                 ("attention.key_length", cfg.head_dim), ("attention.value_length", cfg.head_dim),
                 ("attention.key_length_swa", cfg.head_dim_swa), ("attention.value_length_swa", cfg.head_dim_swa),
                 ("embedding_length_per_layer_input", Ep), ("attention.shared_kv_layers", cfg.shared_kv_layers)):
        b.add_meta(f"{a}.{k}", int(v))
    b.add_meta(f"{a}.attention.layer_norm_rms_epsilon", float(cfg.eps))
    b.add_meta(f"{a}.rope.freq_base", float(cfg.rope_base))
    b.add_meta(f"{a}.attention.sliding_window_pattern", [bool(x) for x in pattern])
    toks = ["<pad>", "<eos>", "<bos>", "<unk>"] + [f"t{i}" for i in range(4, cfg.vocab)]
    b.add_meta("tokenizer.ggml.tokens", toks)
    b.add_meta("tokenizer.ggml.bos_token_id", 2)
    b.add_meta("tokenizer.ggml.eos_token_id", 1)
    kv_from = L - cfg.shared_kv_layers
    specs = [("token_embd.weight", [E, cfg.vocab], TensorType.F16),
             ("output_norm.weight", [E], TensorType.F32),
             ("per_layer_token_embd.weight", [Ep * L, cfg.vocab], table_type),
             ("per_layer_model_proj.weight", [E, Ep * L], ple_type),
             ("per_layer_proj_norm.weight", [Ep], TensorType.F32)]
    for l in range(L):
        p = f"blk.{l}."
        hd = cfg.head_dim_swa if pattern[l] else cfg.head_dim
        specs += [(p + "attn_norm.weight", [E], TensorType.F32),
                  (p + "attn_q.weight", [E, cfg.n_head * hd], wtype)]
        if l < kv_from:
            specs += [(p + "attn_k.weight", [E, cfg.n_head_kv * hd], wtype),
                      (p + "attn_v.weight", [E, cfg.n_head_kv * hd], wtype),
                      (p + "attn_k_norm.weight", [hd], TensorType.F32)]
        specs += [(p + "attn_q_norm.weight", [hd], TensorType.F32),
                  (p + "attn_output.weight", [cfg.n_head * hd, E], wtype),
                  (p + "post_attention_norm.weight", [E], TensorType.F32),
                  (p + "ffn_norm.weight", [E], TensorType.F32),
                  (p + "ffn_gate.weight", [E, F], wtype),
                  (p + "ffn_up.weight", [E, F], wtype),
                  (p + "ffn_down.weight", [F, E], wtype),
                  (p + "post_ffw_norm.weight", [E], TensorType.F32),
                  (p + "inp_gate.weight", [E, Ep], ple_type),
                  (p + "proj.weight", [Ep, E], ple_type),
                  (p + "post_norm.weight", [E], TensorType.F32),
                  (p + "layer_output_scale.weight", [1], TensorType.F32)]
    for name, shape, tt in specs:
        b.add_tensor(name, shape, tt)
    buf, views = b.finalize()
    for name, shape, tt in specs:
        v = views[name]
        if name.endswith("layer_output_scale.weight"):
            v.view(np.float32)[:] = rng.uniform(0.5, 1.0, size=1).astype(np.float32)
        elif tt == TensorType.F32:
            v.view(np.float32)[:] = rng.uniform(0.6, 1.4, size=v.size // 4).astype(np.float32)
        else:
            n_rows = shape[1] if len(shape) > 1 else 1
            fill_random(v, tt, n_rows, shape[0], rng, centered=centered)
    return buf


def bytes_per_token(cfg: Gemma3Config, wtype: int = TensorType.Q4_0,
                    embd_type: int = TensorType.F16) -> Dict[str, int]:
    """Algorithmic HBM bytes of one decode token,
    without the KV term (see kv_bytes_per_position)."""
    E, F = cfg.n_embd, cfg.n_ff
    lin = (row_bytes(wtype, E) * (cfg.q_rows + 2 * cfg.kv_rows + 2 * F) +
           row_bytes(wtype, cfg.q_rows) * E + row_bytes(wtype, F) * E)
    return {"linear": lin * cfg.n_layer, "logits": row_bytes(embd_type, E) * cfg.vocab}


def kv_bytes_per_position(cfg: Gemma3Config) -> int:
    return cfg.n_layer * 2 * cfg.n_head_kv * cfg.head_dim * 2


# ---------------------------------------------------------------------------
# the reference's own ModelTest model (model_test.cpp:81-391), bit-exact
# ---------------------------------------------------------------------------
class _MT19937:
    """std::mt19937 (init_genrand seeding) + libstdc++'s
    uniform_real_distribution<float>(a, b) (generate_canonical<float, 24>)."""

    def __init__(self, seed: int):
        bg = np.random.MT19937()
        bg._legacy_seeding(seed)
        self._bg = bg

    def next_u32(self) -> int:
        return int(self._bg.random_raw())

    def uniform(self, a: float, b: float) -> np.float32:
        f32 = np.float32
        u = f32(self.next_u32()) / f32(4294967296.0)
        if u >= f32(1.0):
            u = np.nextafter(f32(1.0), f32(0.0))
        return u * (f32(b) - f32(a)) + f32(a)


def _trunc_f16(f: np.float32) -> int:
    """model_test.cpp:61-79 (truncating, no subnormals)."""
    x = int(np.float32(f).view(np.uint32))
    sign = (x >> 31) & 1
    exp = ((x >> 23) & 0xFF) - 127
    mant = x & 0x7FFFFF
    if exp > 15:
        return (sign << 15) | (0x1F << 10)
    if exp <= -15:
        return sign << 15
    return (sign << 15) | (((exp + 15) & 0x1F) << 10) | (mant >> 13)


def _test_q4_0(n: int, rng: _MT19937) -> bytes:
    """model_test.cpp:81-123: scale = max|v|/7, lround, interleaved nibbles."""
    out = bytearray()
    for b in range((n + 31) // 32):
        ne = min(32, n - b * 32)
        vals = [np.float32(0.0)] * 32
        mx = np.float32(0.0)
        for i in range(ne):
            vals[i] = rng.uniform(-1.0, 1.0)
            mx = max(mx, np.float32(abs(vals[i])))
        if mx < np.float32(1e-8):
            mx = np.float32(1e-8)
        scale = np.float32(mx / np.float32(7.0))
        out += int(_trunc_f16(scale)).to_bytes(2, "little")
        for i in range(16):
            q = []
            for idx in (2 * i, 2 * i + 1):
                v = 0
                if idx < ne:
                    r = float(np.float32(vals[idx] / scale))
                    v = int(np.floor(abs(r) + 0.5)) * (1 if r >= 0 else -1)  # lround
                q.append(max(-8, min(7, v)))
            out.append(((q[1] + 8) & 0xF) << 4 | ((q[0] + 8) & 0xF))
    return bytes(out)


def build_model_test_gguf() -> bytes:
    """Byte-identical rebuild of ModelTest's in-memory GGUF (model_test.cpp:125-391):
    1 layer, n_embd 32, n_ff 64, 2 heads, 1 KV head, vocab 10, mt19937(12345)."""
    rng = _MT19937(12345)
    E, F, V = 32, 64, 10
    meta = [("general.architecture", "gemma3")]
    meta += [(f"gemma3.{k}", v) for k, v in [("block_count", 1), ("embedding_length", E),
                                            ("feed_forward_length", F), ("attention.head_count", 2),
                                            ("attention.head_count_kv", 1)]]
    meta += [("gemma3.attention.layer_norm_rms_epsilon", 1e-6), ("gemma3.rope.freq_base", 1000000.0),
             ("gemma3.rope.scaling.factor", 1.0)]
    meta += [("tokenizer.ggml.tokens", ["<pad>", "<eos>", "<bos>", "<unk>", "▁", "▁The",
                                        "▁capital", "▁of", "▁Germany", "▁is", ":"]),
             ("tokenizer.ggml.bos_token_id", 2), ("tokenizer.ggml.unknown_token_id", 3)]

    def f32s(n):
        return np.array([rng.uniform(-1.0, 1.0) for _ in range(n)], dtype=np.float32).tobytes()

    te = np.array([_trunc_f16(rng.uniform(-1.0, 1.0)) for _ in range(E * V)], dtype=np.uint16).tobytes()
    out_norm = f32s(E)
    attn_norm = f32s(E)
    qn = f32s(E)
    kn = f32s(E)
    q4 = _test_q4_0(E * E, rng)
    ffn_norm = f32s(E)
    q4f = _test_q4_0(E * F, rng)
    q4d = _test_q4_0(F * E, rng)
    Q, F32_, F16_ = TensorType.Q4_0, TensorType.F32, TensorType.F16
    tensors = [("token_embd.weight", [E, V], F16_, te), ("output_norm.weight", [E], F32_, out_norm),
               ("blk.0.attn_norm.weight", [E], F32_, attn_norm), ("blk.0.attn_q_norm.weight", [E], F32_, qn),
               ("blk.0.attn_k_norm.weight", [E], F32_, kn), ("blk.0.attn_q.weight", [E, E], Q, q4),
               ("blk.0.attn_k.weight", [E, E], Q, q4), ("blk.0.attn_v.weight", [E, E], Q, q4),
               ("blk.0.attn_output.weight", [E, E], Q, q4), ("blk.0.ffn_norm.weight", [E], F32_, ffn_norm),
               ("blk.0.ffn_gate.weight", [E, F], Q, q4f), ("blk.0.ffn_up.weight", [E, F], Q, q4f),
               ("blk.0.ffn_down.weight", [F, E], Q, q4d)]
    from .gguf import write_gguf
    return write_gguf(meta, tensors, align_tensors=False)
