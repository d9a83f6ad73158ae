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

from ._lib import (LLMI_EXACT, LLMI_NO_GRAPH, LLMI_TP_PEER, PEER_HANDLE_BYTES, TP_ID_BYTES, TRACE_FN, SessionInfo,
                   SessionOpts, check, lib, ptr)
from .gguf import GGUFFile


def tp_unique_id() -> bytes:
    """A new RCCL communicator id (rank 0 makes it and sends it to the others)."""
    b = C.create_string_buffer(TP_ID_BYTES)
    check(lib().llmi_tp_unique_id(b))
    return b.raw


class TPGroup:
    """Ranks of one tensor-parallel group sharing ONE device (tests: RCCL
    refuses two ranks per GPU).  Each rank's session is driven by its own
    host thread; the all-gathers are the push exchange split around host
    barriers (LLMI_TP_EXCHANGE=copy: device-to-device copies)."""

    def __init__(self, size: int):
        h = C.c_void_p()
        check(lib().llmi_tp_group_create(size, C.byref(h)))
        self.h = h
        self.size = size

    def close(self):
        if getattr(self, "h", None):
            lib().llmi_tp_group_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class Model:
    def __init__(self, gguf, device: int = 0, exact: bool = False, max_ctx: int = 4096,
                 use_graph: bool = True, attn_split: int = 0, tp_rank: int = 0, tp_size: int = 1,
                 tp_id: Optional[bytes] = None, tp_group: Optional["TPGroup"] = None, tp_peer: bool = False):
        """tp_id (RCCL, one process per GPU), tp_group (ranks on one device,
        one host thread each) or tp_peer (one process per GPU, the one-shot
        push exchange: peer_handle() / peer_connect() before the first
        forward) makes this session rank tp_rank of a row-sharded
        tensor-parallel group of tp_size (include/llmi.h)."""
        buf = gguf if isinstance(gguf, np.ndarray) else np.frombuffer(gguf, np.uint8)
        buf = np.ascontiguousarray(buf)
        self._tp_id = C.create_string_buffer(bytes(tp_id), TP_ID_BYTES) if tp_id is not None else None
        if tp_id is not None and len(tp_id) != TP_ID_BYTES:
            raise ValueError(f"tp_id must be {TP_ID_BYTES} bytes")
        self._tp_group = tp_group  # keep the group alive as long as the session
        flags = (LLMI_EXACT if exact else 0) | (0 if use_graph else LLMI_NO_GRAPH) | (LLMI_TP_PEER if tp_peer else 0)
        opts = SessionOpts(device, flags,
                           max_ctx, attn_split, tp_rank, tp_size,
                           C.cast(self._tp_id, C.c_void_p) if self._tp_id is not None else None,
                           tp_group.h.value if tp_group is not None else None)
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

    def dump(self, tokens: Sequence[int], pos: int, path: str) -> None:
        """llmi_session_dump: forward one token at a time, appending the
        reference's --verbose intermediates (print_tensor format) to `path`."""
        t = np.ascontiguousarray(tokens, np.int32)
        check(lib().llmi_session_dump(self.h, ptr(t), t.size, pos, path.encode()))

    def trace(self, tokens: Sequence[int], pos: int, gen: bool = False) -> list:
        """llmi_session_trace: run the launches forward() (or, gen=True, one
        decode-loop step) performs, eagerly, and return what each launch
        produced as [(name, layer, bytes)] in launch order (op-level parity
        tests compare each against the oracle from the device's own inputs)."""
        t = np.ascontiguousarray(tokens, np.int32)
        out = []

        def cb(_user, name, layer, data, nbytes):
            out.append((name.decode(), int(layer), C.string_at(data, nbytes)))

        fn = TRACE_FN(cb)  # kept alive for the duration of the call
        check(lib().llmi_session_trace(self.h, ptr(t), t.size, pos, 1 if gen else 0, fn, None))
        return out

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

    def peer_handle(self) -> bytes:
        """This rank's push-exchange mailbox handle (LLMI_PEER_HANDLE_BYTES)."""
        b = C.create_string_buffer(PEER_HANDLE_BYTES)
        check(lib().llmi_session_peer_handle(self.h, b))
        return b.raw

    def peer_connect(self, handles: Sequence[bytes]) -> None:
        """Every rank's peer_handle(), in rank order."""
        if len(handles) != self.info.tp_size or any(len(h) != PEER_HANDLE_BYTES for h in handles):
            raise ValueError(f"need {self.info.tp_size} handles of {PEER_HANDLE_BYTES} bytes")
        b = C.create_string_buffer(b"".join(handles), PEER_HANDLE_BYTES * len(handles))
        check(lib().llmi_session_peer_connect(self.h, b))

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
