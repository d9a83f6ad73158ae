"""Build libllmi.so (HIP, gfx950) in-tree with hipcc.

    python -m llm_inference_amd.build [--force]

Every translation unit is compiled with -ffp-contract=off (the numerics
contract of csrc/common.h) for --offload-arch=gfx950 only, in parallel, then
linked into llm_inference_amd/libllmi.so next to this file (git-ignored, but
shipped to the GPU box with the repo snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libllmi.so")
SOURCES = ["k_gemv.hip", "k_layer.hip", "k_elem.hip", "k_attn.hip", "k_session.hip", "k_prefill.hip", "k_logits.hip", "k_exchange.hip", "k_exact.hip", "session.cpp", "collective.cpp", "capi.cpp"]
HEADERS = ["common.h", "kernels.h", "attn.h", "layer_body.h", "session_kernels.h", "session.h", "gguf_reader.h", "collective.h",
           "exact.h", "px.h", "glibc_math.h", "spec_chain.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-result"]
if os.environ.get("LLMI_BLOCK_TRACE_BUILD"):  # development: block-kernel phase clocks (scripts/block_trace.py)
    FLAGS.append("-DLLMI_BLOCK_TRACE")  # into its own objects + libllmi_trace.so (load with LLMI_LIB=...)
    OBJ = os.path.join(HERE, "_build_trace")
    LIB = os.path.join(HERE, "libllmi_trace.so")
# development A/B builds: LLMI_VARIANT=name LLMI_EXTRA_FLAGS="-D..." -> libllmi_<name>.so (load with LLMI_LIB=...)
if os.environ.get("LLMI_VARIANT"):
    FLAGS += os.environ.get("LLMI_EXTRA_FLAGS", "").split()
    OBJ = os.path.join(HERE, "_build_" + os.environ["LLMI_VARIANT"])
    LIB = os.path.join(HERE, "libllmi_" + os.environ["LLMI_VARIANT"] + ".so")


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


# per-file flags: the prefill GEMM's epilogue FMAs stay scalar (packed f32 beside MFMAs costs more issue
# cycles than two v_fmac_f32, MI355X_MICROARCH 'price of one filler beside MFMAs')
FILE_FLAGS = {"k_prefill.hip": ["-fno-slp-vectorize"]}


def _compile(src: str) -> str:
    out = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
    cmd = [HIPCC] + FLAGS + FILE_FLAGS.get(src, []) + ["-x", "hip", "-c", os.path.join(CSRC, src), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
    return out


def build(force: bool = False, jobs: int = 0) -> str:
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS + ["../../include/llmi.h"])
    todo = []
    for s in SOURCES:
        o = os.path.join(OBJ, os.path.splitext(s)[0] + ".o")
        if force or _mtime(o) < max(_mtime(os.path.join(CSRC, s)), hdr_t):
            todo.append(s)
    jobs = jobs or min(len(todo) or 1, os.cpu_count() or 4, 8)
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_compile, todo))
    objs = [os.path.join(OBJ, os.path.splitext(s)[0] + ".o") for s in SOURCES]
    if force or todo or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", LIB] + objs + [
            "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
