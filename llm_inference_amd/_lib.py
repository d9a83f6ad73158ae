"""ctypes binding of include/llmi.h (llm_inference_amd/libllmi.so).

There is deliberately NO fallback: if the HIP library is missing or cannot be
loaded, every op raises.  (The oracle under oracle/ is test infrastructure
and is never imported from this package.)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# LLMI_LIB: an alternate build (development, e.g. the block-trace variant)
LIB_PATH = os.environ.get("LLMI_LIB") or os.path.join(HERE, "libllmi.so")

LLMI_EXACT = 1
LLMI_NO_GRAPH = 2
LLMI_TP_PEER = 4
PEER_HANDLE_BYTES = 64

STATUS = {0: "OK", 1: "E_SIZE", 2: "E_TYPE", 3: "E_ARG", 4: "E_HIP", 5: "E_GGUF", 6: "E_NODEV", 7: "E_RANGE"}


class LLMIError(RuntimeError):
    """A non-zero llmi_status; .code is the status, str() the reference's message."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
        self.status = STATUS.get(code, str(code))


TP_ID_BYTES = 128


class SessionOpts(C.Structure):
    _fields_ = [("device", C.c_int), ("flags", C.c_uint32), ("max_ctx", C.c_int), ("attn_split", C.c_int),
                ("tp_rank", C.c_int), ("tp_size", C.c_int), ("tp_id", C.c_void_p), ("tp_group", C.c_void_p)]


TRACE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_char_p, C.c_int, C.c_void_p, C.c_size_t)


class SessionInfo(C.Structure):
    _fields_ = [("n_layer", C.c_int), ("n_embd", C.c_int), ("n_ff", C.c_int), ("n_head", C.c_int),
                ("n_head_kv", C.c_int), ("head_dim", C.c_int), ("vocab", C.c_int), ("max_ctx", C.c_int),
                ("weight_bytes", C.c_size_t), ("bytes_per_token", C.c_size_t),
                ("kv_bytes_per_pos", C.c_size_t), ("kernels_per_token", C.c_int),
                ("tp_rank", C.c_int), ("tp_size", C.c_int), ("batched_prefill", C.c_int),
                ("screened_logits", C.c_int), ("screen_bytes", C.c_size_t), ("prefill_f16_redo", C.c_int),
                ("layer_engine", C.c_int), ("ffn_engine", C.c_int), ("tp_exchange", C.c_int),
                ("block_slow_waits", C.c_longlong), ("exact_engine", C.c_int), ("exact_batched_prefill", C.c_int),
                ("prefill_gemm", C.c_int)]


_lib = None
_vp, _sz, _u32, _i32, _f32, _f64 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_int32, C.c_float, C.c_double

_SIGS = {
    "llmi_last_error": (C.c_char_p, []),
    "llmi_version": (C.c_int, []),
    "llmi_init_ops": (C.c_int, [C.c_int]),
    "llmi_mat_vec_mul": (C.c_int, [_u32, _vp, _sz, _sz, _vp, _sz, _vp, _u32]),
    "llmi_weight_create": (C.c_int, [_u32, _vp, _sz, _sz, C.POINTER(_vp)]),
    "llmi_weight_mat_vec_mul": (C.c_int, [_vp, _vp, _sz, _vp, _u32]),
    "llmi_weight_mat_vec_mul_dev": (C.c_int, [_vp, _vp, _vp, _u32, _vp]),
    "llmi_weight_destroy": (None, [_vp]),
    "llmi_quantize_row_q8_0": (C.c_int, [_vp, _sz, _vp]),
    "llmi_quantize_row_q8_k": (C.c_int, [_vp, _sz, _vp]),
    "llmi_dequantize_row": (C.c_int, [_u32, _vp, _sz, _vp]),
    "llmi_rms_norm": (C.c_int, [_vp, _vp, _sz, _f64, _u32]),
    "llmi_softmax": (C.c_int, [_vp, _sz]),
    "llmi_rope": (C.c_int, [_vp, _sz, _sz, _sz, C.c_int, _f32, _f32, C.c_int]),
    "llmi_scale": (C.c_int, [_vp, _sz, _f32]),
    "llmi_vec_scale_f16": (C.c_int, [_vp, _sz, _f32]),
    "llmi_vec_mad_f16": (C.c_int, [_vp, _vp, _sz, _f32]),
    "llmi_attention": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int, C.c_int, _vp, _u32]),
    "llmi_gelu_mul": (C.c_int, [_vp, _vp, _sz, _vp]),
    "llmi_session_create":(C.c_int, [_vp, _sz, C.POINTER(SessionOpts), C.POINTER(_vp)]),
    "llmi_session_destroy": (None, [_vp]),
    "llmi_tp_unique_id": (C.c_int, [_vp]),
    "llmi_tp_group_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "llmi_tp_group_destroy": (None, [_vp]),
    "llmi_session_peer_handle": (C.c_int, [_vp, _vp]),
    "llmi_session_peer_connect": (C.c_int, [_vp, _vp]),
    "llmi_session_forward": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _vp, _vp]),
    "llmi_session_generate": (C.c_int, [_vp, _i32, C.c_int, C.c_int, _vp]),
    "llmi_session_dump": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_char_p]),
    "llmi_session_enqueue": (C.c_int, [_vp, _i32, C.c_int, C.c_int]),
    "llmi_session_trace": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _u32, _vp, _vp]),
    "llmi_session_sync": (C.c_int, [_vp, _vp, C.c_int]),
    "llmi_session_get_info": (C.c_int, [_vp, C.POINTER(SessionInfo)]),
    "llmi_session_time_kernel": (C.c_int, [_vp, C.c_int, C.c_int, C.POINTER(_f64), C.POINTER(_f64)]),
    "llmi_selftest": (C.c_int, [C.c_int, _vp]),
}


def lib() -> C.CDLL:
    """Load libllmi.so (raises if it was not built -- no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: build it with `python -m llm_inference_amd.build` "
                              "(HIP, --offload-arch=gfx950); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        raise LLMIError(rc, lib().llmi_last_error().decode(errors="replace"))


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data
