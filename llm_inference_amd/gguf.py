"""GGUF v3 reader/writer -- host-side mirror of the reference's gguf.h/gguf.cpp.

The reader mirrors ``GGUFFile`` (gguf.h:89-121, gguf.cpp:195-304): header,
metadata key/value map, ``TensorInfo`` list, data section aligned to 32 bytes
(gguf.cpp:301-303; ``general.alignment`` is ignored exactly like the
reference).  The writer produces files the reference itself loads; it is used
to build synthetic Gemma-3 models of the BASELINE.json shapes (there are no
real checkpoints in this environment) and the reference's ModelTest model.

Nothing here touches the GPU; the device upload/repack lives in the C++ session
(llm_inference_amd/csrc/session.cpp).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np

GGUF_MAGIC = 0x46554747  # gguf.h:11
GGUF_VERSION = 3         # gguf.h:12


class GGUFType:  # gguf.h:14-28
    UINT8, INT8, UINT16, INT16, UINT32, INT32, FLOAT32, BOOL, STRING, ARRAY, UINT64, INT64, FLOAT64 = range(13)


class TensorType:  # gguf.h:30-46
    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 6
    Q5_1 = 7
    Q8_0 = 8
    Q8_1 = 9
    Q2_K = 10
    Q3_K = 11
    Q4_K = 12
    Q5_K = 13
    Q6_K = 14
    Q8_K = 15
    BF16 = 30


# (elements per block, bytes per block); ops.h:11-31, 89-102
BLOCK = {
    TensorType.F32: (1, 4),
    TensorType.F16: (1, 2),
    TensorType.BF16: (1, 2),
    TensorType.Q4_0: (32, 18),
    TensorType.Q5_0: (32, 22),
    TensorType.Q8_0: (32, 34),
    TensorType.Q4_K: (256, 144),
    TensorType.Q6_K: (256, 210),
}

_TYPE_NAMES = {  # gguf.cpp:358-393
    0: "F32", 1: "F16", 2: "Q4_0", 3: "Q4_1", 6: "Q5_0", 7: "Q5_1", 8: "Q8_0", 9: "Q8_1",
    10: "Q2_K", 11: "Q3_K", 12: "Q4_K", 13: "Q5_K", 14: "Q6_K", 15: "Q8_K", 30: "BF16",
}


def tensor_type_to_string(t: int) -> str:
    """gguf.cpp:358-393 (tensorTypeToString)."""
    return _TYPE_NAMES.get(int(t), f"UNKNOWN ({int(t)})")


def row_bytes(ttype: int, n_cols: int) -> int:
    epb, bpb = BLOCK[ttype]
    if n_cols % epb:
        raise ValueError(f"{tensor_type_to_string(ttype)} row of {n_cols} not a multiple of {epb}")
    return n_cols // epb * bpb


@dataclass
class TensorInfo:  # gguf.h:81-87
    name: str
    shape: List[int]
    tensor_type: int
    tensor_offset: int

    @property
    def total_elements(self) -> int:
        n = 1
        for d in self.shape:
            n *= d
        return n

    @property
    def nbytes(self) -> int:
        return row_bytes(self.tensor_type, self.shape[0]) * (self.total_elements // self.shape[0])


class GGUFFile:
    """Parsed GGUF over a bytes-like buffer (borrowed, like the reference's mmap)."""

    def __init__(self, data):
        self.data = memoryview(data).cast("B")
        self.metadata: Dict[str, object] = {}
        self.tensor_infos: List[TensorInfo] = []
        self._pos = 0
        self._load()

    @classmethod
    def from_path(cls, path: str) -> "GGUFFile":
        return cls(np.memmap(path, dtype=np.uint8, mode="r"))

    # -- reader (gguf.cpp:158-256) --
    def _read(self, fmt: str):
        n = struct.calcsize(fmt)
        if self._pos + n > len(self.data):
            raise ValueError("Read beyond end of file")
        v = struct.unpack_from(fmt, self.data, self._pos)
        self._pos += n
        return v[0] if len(v) == 1 else v

    def _read_str(self) -> str:
        n = self._read("<Q")
        if self._pos + n > len(self.data):
            raise ValueError("String length exceeds file size")
        s = bytes(self.data[self._pos:self._pos + n]).decode("utf-8", errors="surrogateescape")
        self._pos += n
        return s

    _SCALAR = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q", 12: "<d"}

    def _read_value(self, t: int):
        if t in self._SCALAR:
            return self._read(self._SCALAR[t])
        if t == GGUFType.STRING:
            return self._read_str()
        if t == GGUFType.ARRAY:
            et = self._read("<I")
            n = self._read("<Q")
            return [self._read_value(et) for _ in range(n)]
        raise ValueError("Unsupported GGUF value type")

    def _load(self):  # gguf.cpp:274-304
        magic, version, n_tensors, n_kv = self._read("<IIQQ")
        if magic != GGUF_MAGIC:
            raise ValueError("Invalid GGUF magic number")
        self.version = version
        for _ in range(n_kv):
            k = self._read_str()
            t = self._read("<I")
            self.metadata[k] = self._read_value(t)
        for _ in range(n_tensors):
            name = self._read_str()
            nd = self._read("<I")
            shape = [self._read("<Q") for _ in range(nd)]
            tt = self._read("<I")
            off = self._read("<Q")
            self.tensor_infos.append(TensorInfo(name, shape, tt, off))
        self.data_section_start = (self._pos + 31) & ~31

    def get_tensor_data(self, t: TensorInfo) -> memoryview:  # gguf.cpp:354-356
        s = self.data_section_start + t.tensor_offset
        return self.data[s:s + t.nbytes]

    def tensor(self, name: str) -> TensorInfo:
        for t in self.tensor_infos:
            if t.name == name:
                return t
        raise KeyError(name)


# ---------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------
def _pack_str(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def _pack_value(v) -> Tuple[int, bytes]:
    if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], int) and v[0] in GGUFFile._SCALAR:
        return v[0], struct.pack(GGUFFile._SCALAR[v[0]], v[1])
    if isinstance(v, bool):
        return GGUFType.BOOL, struct.pack("<?", v)
    if isinstance(v, int):
        return GGUFType.UINT32, struct.pack("<I", v)
    if isinstance(v, float):
        return GGUFType.FLOAT32, struct.pack("<f", v)
    if isinstance(v, str):
        return GGUFType.STRING, _pack_str(v)
    if isinstance(v, (list, tuple)):
        if not v:
            return GGUFType.ARRAY, struct.pack("<IQ", GGUFType.UINT32, 0)
        et, _ = _pack_value(v[0])
        body = b"".join(_pack_value(e)[1] for e in v)
        return GGUFType.ARRAY, struct.pack("<IQ", et, len(v)) + body
    raise TypeError(type(v))


class GGUFBuilder:
    """Lay out a GGUF v3 file in ONE preallocated numpy buffer.

    ``add_tensor`` records (name, shape, type, nbytes); ``finalize`` writes the
    header and returns (buffer, {name: writable uint8 view of its data}) so
    multi-GB synthetic models are filled in place without extra copies.
    With ``align_tensors`` each tensor's data offset is rounded up to 32 bytes
    (what llama.cpp writes); without it tensors are packed back to back, which
    is what the reference's own test builder does (model_test.cpp:377-384).
    """

    def __init__(self, align_tensors: bool = True):
        self.meta: List[Tuple[str, object]] = []
        self.tensors: List[Tuple[str, List[int], int, int]] = []
        self.align = align_tensors

    def add_meta(self, key: str, value) -> None:
        self.meta.append((key, value))

    def add_tensor(self, name: str, shape: Sequence[int], ttype: int, nbytes: int = -1) -> None:
        if nbytes < 0:
            n = 1
            for d in shape:
                n *= d
            nbytes = row_bytes(ttype, shape[0]) * (n // shape[0])
        self.tensors.append((name, list(shape), ttype, nbytes))

    def finalize(self):
        out = [struct.pack("<IIQQ", GGUF_MAGIC, GGUF_VERSION, len(self.tensors), len(self.meta))]
        for k, v in self.meta:
            t, b = _pack_value(v)
            out.append(_pack_str(k) + struct.pack("<I", t) + b)
        offs, off = [], 0
        for _, _, _, nb in self.tensors:
            if self.align:
                off = (off + 31) & ~31
            offs.append(off)
            off += nb
        for (name, shape, tt, nb), o in zip(self.tensors, offs):
            out.append(_pack_str(name) + struct.pack("<I", len(shape)) +
                       b"".join(struct.pack("<Q", d) for d in shape) + struct.pack("<IQ", tt, o))
        head = b"".join(out)
        start = (len(head) + 31) & ~31
        buf = np.zeros(start + off, dtype=np.uint8)
        buf[:len(head)] = np.frombuffer(head, dtype=np.uint8)
        views = {name: buf[start + o:start + o + nb] for (name, _, _, nb), o in zip(self.tensors, offs)}
        return buf, views


def write_gguf(metadata: Sequence[Tuple[str, object]],
               tensors: Sequence[Tuple[str, Sequence[int], int, bytes]],
               align_tensors: bool = True) -> bytes:
    """Serialize a GGUF v3 file.  ``tensors``: (name, shape, type, raw bytes)."""
    b = GGUFBuilder(align_tensors)
    for k, v in metadata:
        b.add_meta(k, v)
    for name, shape, tt, data in tensors:
        b.add_tensor(name, shape, tt, len(data))
    buf, views = b.finalize()
    for name, _, _, data in tensors:
        views[name][:] = np.frombuffer(bytes(data), dtype=np.uint8)
    return buf.tobytes()
