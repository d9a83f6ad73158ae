"""Python mirror of the reference's Model (model.h:72-153) backed by the
device session of include/llmi.h.

    m = Model(gguf_bytes)                 # Model(GGUFFile&)  model.cpp:13-56
    logits = m.forward([tok, ...], pos)   # Model::forward     model.cpp:706-1049
    ids = m.generate(first, pos, n)       # main.cpp:172-224 greedy loop, on device
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from ._lib import LLMI_EXACT, LLMI_NO_GRAPH, SessionInfo, SessionOpts, check, lib, ptr
from .gguf import GGUFFile


class Model:
    def __init__(self, gguf, device: int = 0, exact: bool = False, max_ctx: int = 4096,
                 use_graph: bool = True, attn_split: int = 0):
        buf = gguf if isinstance(gguf, np.ndarray) else np.frombuffer(gguf, np.uint8)
        buf = np.ascontiguousarray(buf)
        opts = SessionOpts(device, (LLMI_EXACT if exact else 0) | (0 if use_graph else LLMI_NO_GRAPH),
                           max_ctx, attn_split)
        h = C.c_void_p()
        check(lib().llmi_session_create(ptr(buf), buf.size, C.byref(opts), C.byref(h)))
        self.h = h
        self.gguf = GGUFFile(buf)  # host-side metadata view (tokenizer etc.)
        self.info = self.get_info()
        self.vocab = self.info.vocab

    def get_info(self) -> SessionInfo:
        info = SessionInfo()
        check(lib().llmi_session_get_info(self.h, C.byref(info)))
        return info

    def forward(self, tokens: Sequence[int], pos: int, want_logits: bool = True):
        t = np.ascontiguousarray(tokens, np.int32)
        lg = np.zeros(self.vocab, np.float32) if want_logits else None
        am = np.zeros(1, np.int32)
        check(lib().llmi_session_forward(self.h, ptr(t), t.size, pos, ptr(lg) if lg is not None else None, ptr(am)))
        self.last_argmax = int(am[0])
        return lg

    def generate(self, first: int, pos: int, n_steps: int) -> np.ndarray:
        out = np.zeros(max(n_steps, 1), np.int32)
        check(lib().llmi_session_generate(self.h, first, pos, n_steps, ptr(out)))
        return out[:n_steps]

    def enqueue(self, first: int, pos: int, n_steps: int) -> None:
        check(lib().llmi_session_enqueue(self.h, first, pos, n_steps))

    def sync(self, n: int = 0) -> Optional[np.ndarray]:
        out = np.zeros(max(n, 1), np.int32)
        check(lib().llmi_session_sync(self.h, ptr(out) if n else None, n))
        return out[:n] if n else None

    def time_kernel(self, which: int, reps: int):
        us, by = C.c_double(), C.c_double()
        check(lib().llmi_session_time_kernel(self.h, which, reps, C.byref(us), C.byref(by)))
        return us.value, by.value

    def close(self):
        if getattr(self, "h", None):
            lib().llmi_session_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()
