"""ctypes bindings for the CHECKERS: oracle/_build/liboracle.so (our CPU
restatement) and oracle/_ref/libllmref.so (the reference itself).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by llm_inference_amd/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libllmref.so")
REF_SRC = "/root/reference"

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


def build(ref: bool = True) -> None:
    """Compile the oracle (and, when the reference sources exist, _ref)."""
    # "dropin": the reference's model.cpp/gguf.cpp with integration/ops_mi355x.cpp
    # in place of ops.cpp (needs llm_inference_amd/libllmi.so built first)
    targets = ["all"] + (["ref", "dropin", "mainloop"] if ref and os.path.isdir(REF_SRC) else [])
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build(ref=False)
        L = self.lib = C.CDLL(path)
        L.orc_f32_to_f16.restype = C.c_uint16
        L.orc_f32_to_f16.argtypes = [C.c_float]
        L.orc_f16_to_f32.restype = C.c_float
        L.orc_f16_to_f32.argtypes = [C.c_uint16]
        L.orc_quantize_row_q8_0.argtypes = [_f32p, C.c_size_t, C.c_void_p]
        L.orc_quantize_row_q8_k.argtypes = [_f32p, C.c_size_t, C.c_void_p]
        L.orc_mat_vec_mul.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t, C.c_size_t, _f32p, _f32p, C.c_int]
        L.orc_mat_vec_mul_q8.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, _f32p, C.c_int]
        L.orc_dequantize_row.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t, _f32p]
        L.orc_rms_norm.argtypes = [_f32p, _f32p, C.c_size_t, C.c_double]
        L.orc_softmax.argtypes = [_f32p, C.c_size_t]
        L.orc_rope.argtypes = [_f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int, C.c_float, C.c_float, C.c_int]
        L.orc_scale.argtypes = [_f32p, C.c_size_t, C.c_float]
        L.orc_vec_scale_f16.argtypes = [_u16p, C.c_size_t, C.c_float]
        L.orc_vec_mad_f16.argtypes = [_u16p, _u16p, C.c_size_t, C.c_float]
        L.orc_gelu_mul.argtypes = [_f32p, _f32p, _f32p, C.c_size_t]
        L.orc_attn_head.argtypes = [_f32p, _u16p, _u16p, C.c_size_t, C.c_size_t, _f32p]
        L.orc_attn_head_f64.argtypes = [_f32p, _u16p, _u16p, C.c_size_t, C.c_size_t, _f32p]
        L.orc_attn_head_cap.argtypes = [_f32p, _u16p, _u16p, C.c_size_t, C.c_size_t, C.c_float, _f32p]
        L.orc_attn_head_f64_cap.argtypes = [_f32p, _u16p, _u16p, C.c_size_t, C.c_size_t, C.c_float, _f32p]
        L.orc_model_create.restype = C.c_void_p
        L.orc_model_create.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int]
        L.orc_model_forward.argtypes = [C.c_void_p, _i32p, C.c_int, C.c_int, _f32p]
        L.orc_model_vocab.argtypes = [C.c_void_p]
        L.orc_model_destroy.argtypes = [C.c_void_p]
        L.orc_model_set_attn_f64.argtypes = [C.c_void_p, C.c_int]
        L.orc_last_error.restype = C.c_char_p

    # --- ops ---
    def f32_to_f16(self, x: np.ndarray) -> np.ndarray:
        return np.array([self.lib.orc_f32_to_f16(float(v)) for v in np.ravel(x)], dtype=np.uint16)

    def quantize_q8_0(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(x.size // 32 * 34, np.uint8)
        self.lib.orc_quantize_row_q8_0(x, x.size, _ptr(y))
        return y

    def quantize_q8_k(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(x.size // 256 * 292, np.uint8)
        self.lib.orc_quantize_row_q8_k(x, x.size, _ptr(y))
        return y

    def mat_vec_mul(self, ttype, w, n_rows, n_cols, x, n_threads=8):
        x = np.ascontiguousarray(x, np.float32)
        w = np.ascontiguousarray(w)
        o = np.zeros(n_rows, np.float32)
        if self.lib.orc_mat_vec_mul(ttype, _ptr(w), n_rows, n_cols, x, o, n_threads) != 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return o

    def mat_vec_mul_q8(self, ttype, w, n_rows, n_cols, xq, n_threads=8):
        """Q4_0/Q8_0 rows x an already-quantized activation (34-B BlockQ8_0 row)."""
        w = np.ascontiguousarray(w)
        xq = np.ascontiguousarray(xq, np.uint8)
        assert xq.size == n_cols // 32 * 34
        o = np.zeros(n_rows, np.float32)
        if self.lib.orc_mat_vec_mul_q8(ttype, _ptr(w), n_rows, n_cols, _ptr(xq), o, n_threads) != 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return o

    def attn_head_f64(self, q, k, v):
        """float64-accumulating restatement (pins the fast path, not the reference)."""
        q = np.ascontiguousarray(q, np.float32)
        out = np.zeros_like(q)
        self.lib.orc_attn_head_f64(q, np.ascontiguousarray(k, np.uint16), np.ascontiguousarray(v, np.uint16),
                                   k.shape[0], q.size, out)
        return out

    def dequantize_row(self, ttype, blocks, n_cols):
        o = np.zeros(n_cols, np.float32)
        b = np.ascontiguousarray(blocks)
        if self.lib.orc_dequantize_row(ttype, _ptr(b), n_cols, o) != 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return o

    def rms_norm(self, x, eps):
        x = np.ascontiguousarray(x, np.float32)
        o = np.zeros_like(x)
        if self.lib.orc_rms_norm(o, x, x.size, eps) != 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return o

    def softmax(self, x):
        x = np.array(x, np.float32)
        self.lib.orc_softmax(x, x.size)
        return x

    def rope(self, t, n_rot, base, scale, pos):
        t = np.array(t, np.float32)
        nt, nh, hd = t.shape
        self.lib.orc_rope(t.reshape(-1), nt, nh, hd, n_rot, base, scale, pos)
        return t

    def vec_scale_f16(self, y, v):
        y = np.array(y, np.uint16)
        self.lib.orc_vec_scale_f16(y, y.size, v)
        return y

    def vec_mad_f16(self, y, x, v):
        y = np.array(y, np.uint16)
        self.lib.orc_vec_mad_f16(y, np.ascontiguousarray(x, np.uint16), y.size, v)
        return y

    def gelu_mul(self, g, u):
        g = np.ascontiguousarray(g, np.float32)
        o = np.zeros_like(g)
        self.lib.orc_gelu_mul(o, g, np.ascontiguousarray(u, np.float32), g.size)
        return o

    def attn_head(self, q, k, v, softcap: float = 0.0):
        q = np.ascontiguousarray(q, np.float32)
        out = np.zeros_like(q)
        self.lib.orc_attn_head_cap(q, np.ascontiguousarray(k, np.uint16), np.ascontiguousarray(v, np.uint16),
                                   k.shape[0], q.size, softcap, out)
        return out

    # --- model ---
    def model(self, gguf: np.ndarray, n_threads: int = 8, max_ctx: int = 1024, attn_f64: bool = False):
        m = OracleModel(self, gguf, n_threads, max_ctx)
        self.lib.orc_model_set_attn_f64(m.h, int(attn_f64))
        return m


class OracleModel:
    def __init__(self, orc: Oracle, gguf, n_threads, max_ctx):
        self.orc = orc
        self.buf = np.ascontiguousarray(np.frombuffer(gguf, np.uint8) if isinstance(gguf, (bytes, bytearray)) else gguf)
        self.h = orc.lib.orc_model_create(_ptr(self.buf), self.buf.size, n_threads, max_ctx)
        if not self.h:
            raise RuntimeError(orc.lib.orc_last_error().decode())
        self.vocab = orc.lib.orc_model_vocab(self.h)

    def forward(self, tokens, pos):
        t = np.ascontiguousarray(tokens, np.int32)
        lg = np.zeros(self.vocab, np.float32)
        if self.orc.lib.orc_model_forward(self.h, t, t.size, pos, lg) != 0:
            raise RuntimeError(self.orc.lib.orc_last_error().decode())
        return lg

    def __del__(self):
        if getattr(self, "h", None):
            self.orc.lib.orc_model_destroy(self.h)
            self.h = None


class Reference:
    """The reference's own code (oracle/_ref/libllmref.so)."""

    def __init__(self, path: str = REF_SO, n_threads: int = 1):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.lib = C.CDLL(path)
        L.ref_init_ops(n_threads)
        L.ref_f32_to_f16.restype = C.c_uint16
        L.ref_f32_to_f16.argtypes = [C.c_float]
        L.ref_f16_to_f32.restype = C.c_float
        L.ref_f16_to_f32.argtypes = [C.c_uint16]
        L.ref_quantize_row_q8_0.argtypes = [_f32p, C.c_size_t, C.c_void_p]
        L.ref_quantize_row_q8_k.argtypes = [_f32p, C.c_size_t, C.c_void_p]
        L.ref_mat_vec_mul.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, _f32p, _f32p]
        L.ref_dequantize_row.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t, _f32p]
        L.ref_rms_norm.argtypes = [_f32p, _f32p, C.c_size_t, C.c_double]
        L.ref_softmax.argtypes = [_f32p, C.c_size_t]
        L.ref_rope.argtypes = [_f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int, C.c_float, C.c_float, C.c_int]
        L.ref_vec_scale_f16.argtypes = [_u16p, C.c_size_t, C.c_float]
        L.ref_vec_mad_f16.argtypes = [_u16p, _u16p, C.c_size_t, C.c_float]
        L.ref_model_create.restype = C.c_void_p
        L.ref_model_create.argtypes = [C.c_void_p, C.c_size_t]
        L.ref_model_forward.argtypes = [C.c_void_p, _i32p, C.c_int, C.c_int, _f32p]
        L.ref_model_destroy.argtypes = [C.c_void_p]
        L.ref_model_tokenize.argtypes = [C.c_void_p, C.c_char_p, C.c_int, _i32p, C.c_int]
        L.ref_last_error.restype = C.c_char_p
        L.ref_gemv_prepare.restype = C.c_void_p
        L.ref_gemv_prepare.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t]
        L.ref_gemv_run.argtypes = [C.c_void_p, _f32p, C.c_void_p]
        L.ref_gemv_free.argtypes = [C.c_void_p]

    def quantize_q8_0(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(x.size // 32 * 34, np.uint8)
        self.lib.ref_quantize_row_q8_0(x, x.size, _ptr(y))
        return y

    def quantize_q8_k(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(x.size // 256 * 292, np.uint8)
        self.lib.ref_quantize_row_q8_k(x, x.size, _ptr(y))
        return y

    def mat_vec_mul(self, ttype, w, n_rows, n_cols, x):
        x = np.ascontiguousarray(x, np.float32)
        w = np.ascontiguousarray(w)
        o = np.zeros(n_rows, np.float32)
        if self.lib.ref_mat_vec_mul(ttype, _ptr(w), w.nbytes, n_rows, n_cols, x, o) != 0:
            raise RuntimeError(self.lib.ref_last_error().decode())
        return o

    def time_gemv(self, ttype, w, n_rows, n_cols, x, reps):
        """Mean seconds of the reference's mat_vec_mul (or mat_vec_mul_fp16 for
        F16) on a weight prepared once (no per-call copies)."""
        import time
        w = np.ascontiguousarray(w)
        h = self.lib.ref_gemv_prepare(ttype, _ptr(w), w.nbytes, n_rows, n_cols)
        if not h:
            raise RuntimeError(self.lib.ref_last_error().decode())
        x = np.ascontiguousarray(x, np.float32)
        self.lib.ref_gemv_run(h, x, None)
        t0 = time.perf_counter()
        for _ in range(reps):
            self.lib.ref_gemv_run(h, x, None)
        dt = (time.perf_counter() - t0) / reps
        self.lib.ref_gemv_free(h)
        return dt

    def dequantize_row(self, ttype, blocks, n_cols):
        o = np.zeros(n_cols, np.float32)
        self.lib.ref_dequantize_row(ttype, _ptr(np.ascontiguousarray(blocks)), n_cols, o)
        return o

    def rms_norm(self, x, eps):
        x = np.ascontiguousarray(x, np.float32)
        o = np.zeros_like(x)
        self.lib.ref_rms_norm(o, x, x.size, eps)
        return o

    def softmax(self, x):
        x = np.array(x, np.float32)
        self.lib.ref_softmax(x, x.size)
        return x

    def rope(self, t, n_rot, base, scale, pos):
        t = np.array(t, np.float32)
        nt, nh, hd = t.shape
        self.lib.ref_rope(t.reshape(-1), nt, nh, hd, n_rot, base, scale, pos)
        return t

    def vec_scale_f16(self, y, v):
        y = np.array(y, np.uint16)
        self.lib.ref_vec_scale_f16(y, y.size, v)
        return y

    def vec_mad_f16(self, y, x, v):
        y = np.array(y, np.uint16)
        self.lib.ref_vec_mad_f16(y, np.ascontiguousarray(x, np.uint16), y.size, v)
        return y

    def model(self, gguf):
        return RefModel(self, gguf)


class RefModel:
    def __init__(self, ref: Reference, gguf):
        self.ref = ref
        self.buf = np.ascontiguousarray(np.frombuffer(gguf, np.uint8) if isinstance(gguf, (bytes, bytearray)) else gguf)
        self.h = ref.lib.ref_model_create(_ptr(self.buf), self.buf.size)
        if not self.h:
            raise RuntimeError(ref.lib.ref_last_error().decode())
        import sys
        sys.path.insert(0, os.path.dirname(HERE))
        from llm_inference_amd.gguf import GGUFFile
        self.vocab = GGUFFile(self.buf).tensor("token_embd.weight").shape[1]

    def forward(self, tokens, pos):
        t = np.ascontiguousarray(tokens, np.int32)
        lg = np.zeros(self.vocab, np.float32)
        if self.ref.lib.ref_model_forward(self.h, t, t.size, pos, lg) < 0:
            raise RuntimeError(self.ref.lib.ref_last_error().decode())
        return lg

    def tokenize(self, prompt: str, chat: bool = False):
        out = np.zeros(4096, np.int32)
        n = self.ref.lib.ref_model_tokenize(self.h, prompt.encode(), int(chat), out, out.size)
        return out[:n].tolist()

    def __del__(self):
        if getattr(self, "h", None):
            self.ref.lib.ref_model_destroy(self.h)
            self.h = None
