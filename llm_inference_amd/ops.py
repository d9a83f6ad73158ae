"""Python mirror of the reference's ops.h surface (ops.h:38-105), executed by
the HIP library through the C ABI (include/llmi.h).

Same names, argument meaning and error behaviour as the reference:
  * ``mat_vec_mul(o, w_tensor, gguf_file, x)`` resizes/fills ``o`` with
    W*x where W is the GGUF tensor (ops.cpp:933-956); a wrong ``len(x)``
    raises RuntimeError("mat_vec_mul_q4_0: input vector size mismatch"),
    an unsupported type RuntimeError("mat_vec_mul: unsupported tensor type N")
    (ops.cpp:196-198, 953-954);
  * ``rms_norm`` with eps <= 0 raises (the reference exit(1)s, ops.cpp:29-32).
Buffers are numpy arrays; everything is synchronous.  ``exact=True`` selects
the bit-exact AVX2-order kernels (LLMI_EXACT).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ._lib import LLMI_EXACT, LLMIError, check, lib, ptr
from .gguf import GGUFFile, TensorInfo, TensorType


def init_ops(device: int = 0) -> None:
    """init_ops(n_threads) (ops.cpp:21-24): selects the HIP device."""
    check(lib().llmi_init_ops(device))


def _f32(x) -> np.ndarray:
    return np.ascontiguousarray(x, dtype=np.float32)


def _fill(o, vals: np.ndarray):
    if o is None:
        return vals
    if isinstance(o, list):
        o[:] = vals.tolist()
        return o
    o.resize(vals.shape, refcheck=False)
    o[...] = vals
    return o


def _raise(e: LLMIError):
    raise RuntimeError(str(e)) from e


def mat_vec_mul_raw(ttype: int, w, n_rows: int, n_cols: int, x, exact: bool = False) -> np.ndarray:
    w = np.ascontiguousarray(np.frombuffer(w, np.uint8) if not isinstance(w, np.ndarray) else w)
    x = _f32(x)
    o = np.zeros(n_rows, np.float32)
    try:
        check(lib().llmi_mat_vec_mul(ttype, ptr(w), n_rows, n_cols, ptr(x), x.size, ptr(o),
                                     LLMI_EXACT if exact else 0))
    except LLMIError as e:
        _raise(e)
    return o


def mat_vec_mul(o, w_tensor: TensorInfo, gguf_file: GGUFFile, x, exact: bool = False):
    """ops.cpp:933-956: n_rows = shape[1], n_cols = shape[0]."""
    if w_tensor.tensor_type == TensorType.F16:  # not in the reference dispatch
        raise RuntimeError(f"mat_vec_mul: unsupported tensor type {w_tensor.tensor_type}")
    w = np.frombuffer(gguf_file.get_tensor_data(w_tensor), np.uint8)
    vals = mat_vec_mul_raw(w_tensor.tensor_type, w, w_tensor.shape[1], w_tensor.shape[0], x, exact)
    return _fill(o, vals)


def mat_vec_mul_fp16(o, w, x, n_rows: int, n_cols: int, exact: bool = False):
    """ops.cpp:455-612 (w: n_rows*n_cols uint16 f16 bits)."""
    w = np.ascontiguousarray(w, np.uint16)
    if len(x) != n_cols:
        raise RuntimeError("mat_vec_mul_fp16: input vector size mismatch")
    if w.size != n_rows * n_cols:
        raise RuntimeError("mat_vec_mul_fp16: weight matrix size mismatch")
    return _fill(o, mat_vec_mul_raw(TensorType.F16, w.view(np.uint8), n_rows, n_cols, x, exact))


def quantize_row_q8_0(x) -> np.ndarray:
    """ops.cpp:116-139 -> 34-byte BlockQ8_0 blocks."""
    x = _f32(x)
    y = np.zeros(x.size // 32 * 34, np.uint8)
    check(lib().llmi_quantize_row_q8_0(ptr(x), x.size, ptr(y)))
    return y


def quantize_row_q8_k(x) -> np.ndarray:
    """ops.cpp:142-178 -> 292-byte block_q8_K blocks."""
    x = _f32(x)
    y = np.zeros(x.size // 256 * 292, np.uint8)
    check(lib().llmi_quantize_row_q8_k(ptr(x), x.size, ptr(y)))
    return y


def dequantize_row(ttype: int, blocks, n_cols: int) -> np.ndarray:
    """dequantize_{q4_k,q6_k,q8_0,q5_0}_row (ops.cpp:958-1082)."""
    b = np.ascontiguousarray(np.frombuffer(blocks, np.uint8) if not isinstance(blocks, np.ndarray) else blocks)
    o = np.zeros(n_cols, np.float32)
    check(lib().llmi_dequantize_row(ttype, ptr(b), n_cols, ptr(o)))
    return o


def rms_norm(o, x, eps: float, exact: bool = False):
    """ops.cpp:28-43."""
    x = _f32(x)
    out = np.zeros_like(x)
    try:
        check(lib().llmi_rms_norm(ptr(out), ptr(x), x.size, float(eps), LLMI_EXACT if exact else 0))
    except LLMIError as e:
        _raise(e)
    return _fill(o, out)


def softmax(x) -> np.ndarray:
    """ops.cpp:45-62 (in place on a copy; returns it)."""
    x = np.array(x, np.float32)
    check(lib().llmi_softmax(ptr(x), x.size))
    return x


def rope(tensor, n_rot: int, rope_freq_base: float, rope_freq_scale: float, pos: int) -> np.ndarray:
    """ops.cpp:67-95; tensor is [n_tokens][n_heads][head_dim]."""
    t = np.array(tensor, np.float32)
    if t.size == 0:
        return t
    nt, nh, hd = t.shape
    check(lib().llmi_rope(ptr(t), nt, nh, hd, n_rot, rope_freq_base, rope_freq_scale, pos))
    return t


def scale(tensor, scale_factor: float) -> np.ndarray:
    """ops.cpp:97-105."""
    t = np.array(tensor, np.float32)
    check(lib().llmi_scale(ptr(t), t.size, scale_factor))
    return t


def vec_scale_f16(y, v: float) -> np.ndarray:
    """ops.cpp:1084-1089 (y: uint16 f16 bits)."""
    y = np.array(y, np.uint16)
    check(lib().llmi_vec_scale_f16(ptr(y), y.size, v))
    return y


def vec_mad_f16(y, x, v: float) -> np.ndarray:
    """ops.cpp:1091-1099."""
    y = np.array(y, np.uint16)
    x = np.ascontiguousarray(x, np.uint16)
    check(lib().llmi_vec_mad_f16(ptr(y), ptr(x), y.size, v))
    return y


def attention(q, k, v, exact: bool = False) -> np.ndarray:
    """Decode attention of Model::run_attn (model.cpp:478-550).
    q: [n_head, hd] f32; k, v: [n_head_kv, n_keys, hd] uint16 f16 bits."""
    q = _f32(q)
    k = np.ascontiguousarray(k, np.uint16)
    v = np.ascontiguousarray(v, np.uint16)
    n_head, hd = q.shape
    n_kv, n_keys, _ = k.shape
    out = np.zeros_like(q)
    check(lib().llmi_attention(ptr(q), ptr(k), ptr(v), n_head, n_kv, n_keys, hd, ptr(out),
                               LLMI_EXACT if exact else 0))
    return out


def gelu_mul(gate, up) -> np.ndarray:
    """GELU(tanh)(gate) * up, model.cpp:892-899."""
    g, u = _f32(gate), _f32(up)
    out = np.zeros_like(g)
    check(lib().llmi_gelu_mul(ptr(g), ptr(u), g.size, ptr(out)))
    return out


class DeviceWeight:
    """A GGUF weight uploaded once (llmi_weight_create); multiply many times."""

    def __init__(self, ttype: int, w, n_rows: int, n_cols: int):
        import ctypes as C
        self.ttype, self.n_rows, self.n_cols = ttype, n_rows, n_cols
        w = np.ascontiguousarray(np.frombuffer(w, np.uint8) if not isinstance(w, np.ndarray) else w)
        h = C.c_void_p()
        check(lib().llmi_weight_create(ttype, ptr(w), n_rows, n_cols, C.byref(h)))
        self.h = h

    def __call__(self, x, exact: bool = False) -> np.ndarray:
        x = _f32(x)
        o = np.zeros(self.n_rows, np.float32)
        check(lib().llmi_weight_mat_vec_mul(self.h, ptr(x), x.size, ptr(o), LLMI_EXACT if exact else 0))
        return o

    def dev(self, x_ptr: int, o_ptr: int, stream: Optional[int] = None, exact: bool = False) -> None:
        check(lib().llmi_weight_mat_vec_mul_dev(self.h, x_ptr, o_ptr, LLMI_EXACT if exact else 0, stream))

    def __del__(self):
        if getattr(self, "h", None):
            lib().llmi_weight_destroy(self.h)
            self.h = None
