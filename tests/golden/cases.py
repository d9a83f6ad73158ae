"""Deterministic golden-vector CASES shared by gen_golden.py (which runs the
reference itself, oracle/_ref) and the tests (oracle and HIP path).

Each case is (name, kind, params); ``make_inputs`` regenerates the inputs
from a seed with numpy's PCG64 (bit-stable for a given numpy), so only
outputs plus an input hash are committed (tests/golden/*.npz).
Shapes: reduced row counts at the real Gemma-3 n_cols (per-row arithmetic
depends only on n_cols).
"""
from __future__ import annotations

import hashlib

import numpy as np

from llm_inference_amd.gguf import TensorType as T
from llm_inference_amd.synthetic import random_tensor

# (name, ggml type, n_rows, n_cols)
GEMV_CASES = [
    ("q4_0_1152", T.Q4_0, 96, 1152),      # 1B q/gate-like
    ("q4_0_2560", T.Q4_0, 128, 2560),     # 4B q/k/v/gate/up
    ("q4_0_2048", T.Q4_0, 64, 2048),      # 4B attn_output
    ("q4_0_10240", T.Q4_0, 40, 10240),    # 4B ffn_down
    ("q4_0_6912", T.Q4_0, 40, 6912),      # 1B ffn_down
    ("q4_0_5376", T.Q4_0, 40, 5376),      # 27B q/k/v/gate/up
    ("q4_0_96", T.Q4_0, 7, 96),           # ragged tiny: 3 blocks, 7 rows
    ("q4_0_32", T.Q4_0, 5, 32),           # one block per row (ModelTest n_embd)
    ("q4_0_64", T.Q4_0, 9, 64),
    ("q8_0_1152", T.Q8_0, 64, 1152),
    ("q8_0_2560", T.Q8_0, 64, 2560),
    ("q8_0_32", T.Q8_0, 3, 32),
    ("q4_k_2560", T.Q4_K, 64, 2560),
    ("q6_k_2560", T.Q6_K, 64, 2560),
    ("q6_k_10240", T.Q6_K, 24, 10240),
    ("q5_0_1152", T.Q5_0, 64, 1152),
    ("bf16_640", T.BF16, 48, 640),
    ("f16_2560", T.F16, 200, 2560),       # logits-like
    ("f16_1152", T.F16, 130, 1152),
    ("f16_40", T.F16, 9, 40),             # n_cols % 32 != 0 tail path (ops.cpp:581-583)
]

QUANT_CASES = [("q8_0", 32 * 97), ("q8_0", 2560), ("q8_k", 2560), ("q8_k", 256 * 3)]
NORM_CASES = [2560, 256, 1152, 4]
ROPE_CASES = [  # (n_tokens, n_heads, head_dim, base, pos)
    (1, 8, 256, 10000.0, 0), (1, 8, 256, 10000.0, 517), (3, 4, 256, 1000000.0, 41),
    (1, 16, 128, 1000000.0, 4095), (1, 1, 4, 10000.0, 1),
]
DEQ_CASES = [(T.Q4_K, 2560), (T.Q6_K, 2560), (T.Q8_0, 1152), (T.Q5_0, 1152)]


def gemv_inputs(name, ttype, n_rows, n_cols):
    seed = int(hashlib.sha256(name.encode()).hexdigest()[:8], 16)
    w = random_tensor(ttype, n_rows, n_cols, seed=seed)
    x = np.random.default_rng(seed + 1).standard_normal(n_cols).astype(np.float32)
    return w, x


def quant_input(kind, n, k=0):
    rng = np.random.default_rng(1000 + n + k)
    x = (rng.standard_normal(n) * rng.uniform(0.01, 30.0, size=n // 32).repeat(32)).astype(np.float32)
    x[:32] = 0.0            # an all-zero block: d = 0, id = 0 path (ops.cpp:130)
    x[40] = 1e-30           # tiny denormal-ish magnitude
    x[64:96] = -3.0         # constant negative block
    return x


def norm_input(n):
    return (np.random.default_rng(2000 + n).standard_normal(n) * 3).astype(np.float32)


def rope_input(nt, nh, hd):
    return np.random.default_rng(3000 + nt * 100000 + nh * 1000 + hd).standard_normal((nt, nh, hd)).astype(np.float32)


def deq_input(ttype, n):
    return random_tensor(ttype, 1, n, seed=4000 + ttype)


def f16_input(n=4096):
    rng = np.random.default_rng(5000)
    x = np.concatenate([
        rng.standard_normal(n).astype(np.float32) * np.float32(10.0) ** rng.integers(-9, 6, n).astype(np.float32),
        np.array([0.0, -0.0, 65504.0, 65520.0, 1e9, -1e9, 6e-8, 3e-8, 2.98e-8, 1e-40, np.inf, -np.inf], np.float32),
    ]).astype(np.float32)
    return x


def sha(*arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
