"""Record the REFERENCE's --verbose tensor dumps as fixtures (run here, not on
the GPU box): oracle/_ref/libllmref.so (the reference's model.cpp / ops.cpp /
gguf.cpp built by oracle/Makefile) with verbose_g on, stdout captured at the
file-descriptor level while Model::forward runs one token at a time.

  dump_tiny_ref.txt   seeded synthetic 'tiny' Gemma-3 (3 layers, SWA pattern
                      [T, F, T], seed 7): prompt [2, 17, 301], one token per
                      forward (positions 0..2)

    python tests/golden/gen_dumps.py
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.bind import Reference  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

TINY_PROMPT = [2, 17, 301]


def tiny_gguf():
    return build_gemma3_gguf(CONFIGS["tiny"], seed=7, swa_pattern=[True, False, True])


def capture(fn) -> str:
    sys.stdout.flush()
    fd = sys.stdout.fileno()
    saved = os.dup(fd)
    with tempfile.TemporaryFile(mode="w+b") as tmp:
        os.dup2(tmp.fileno(), fd)
        try:
            fn()
        finally:
            os.dup2(saved, fd)
            os.close(saved)
        tmp.seek(0)
        return tmp.read().decode()


def main():
    ref = Reference(n_threads=1)
    ref.lib.ref_set_verbose.argtypes = [np.ctypeslib.ctypes.c_int]
    m = ref.model(tiny_gguf())

    def run():
        ref.lib.ref_set_verbose(1)
        for i, t in enumerate(TINY_PROMPT):
            m.forward([t], i)
        ref.lib.ref_flush()
        ref.lib.ref_set_verbose(0)

    text = capture(run)
    with open(os.path.join(HERE, "dump_tiny_ref.txt"), "w") as f:
        f.write(text)
    print("wrote dump_tiny_ref.txt:", len(text.splitlines()), "lines")


if __name__ == "__main__":
    main()
