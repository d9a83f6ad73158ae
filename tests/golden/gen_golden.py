"""Generate golden fixtures by running the REFERENCE ITSELF.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/gen_golden.py
It loads oracle/_ref/libllmref.so (the reference's ops.cpp/gguf.cpp/model.cpp
compiled with its pinned flags by oracle/Makefile) and records outputs for the
deterministic cases of tests/golden/cases.py:
  ops_ref.npz        op-level outputs (bit patterns) + input hashes
  model_test.gguf    byte-identical rebuild of ModelTest's in-memory GGUF
  model_ref.npz      reference logits / greedy tokens on model_test.gguf and
                     on the seeded synthetic 'tiny' Gemma-3 model, with and
                     without the attention logit soft-cap
No reference source or binary is committed; only these data files.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle.bind import Reference  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf, build_model_test_gguf  # noqa: E402
import cases as K  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SOFTCAP = 0.25


def gen_ops(ref: Reference) -> dict:
    d = {}
    for name, tt, r, c in K.GEMV_CASES:
        w, x = K.gemv_inputs(name, tt, r, c)
        d[f"gemv__{name}__o"] = ref.mat_vec_mul(tt, w, r, c, x)
        d[f"gemv__{name}__sha"] = np.frombuffer(K.sha(w, x).encode(), np.uint8)
    for i, (kind, n) in enumerate(K.QUANT_CASES):
        x = K.quant_input(kind, n, i)
        d[f"quant__{kind}_{n}__y"] = ref.quantize_q8_0(x) if kind == "q8_0" else ref.quantize_q8_k(x)
    for n in K.NORM_CASES:
        x = K.norm_input(n)
        d[f"rms__{n}"] = ref.rms_norm(x, float(np.float32(1e-6)))
        d[f"softmax__{n}"] = ref.softmax(x)
    for (nt, nh, hd, base, pos) in K.ROPE_CASES:
        t = K.rope_input(nt, nh, hd)
        d[f"rope__{nt}_{nh}_{hd}_{int(base)}_{pos}"] = ref.rope(t, hd, base, 1.0, pos)
    for tt, n in K.DEQ_CASES:
        d[f"deq__{tt}_{n}"] = ref.dequantize_row(tt, K.deq_input(tt, n), n)
    x = K.f16_input()
    d["f16__to16"] = np.array([ref.lib.ref_f32_to_f16(float(v)) for v in x], np.uint16)
    tab = np.array([ref.lib.ref_f16_to_f32(i) for i in range(65536)], np.float32)
    d["f16__table"] = tab.view(np.uint32)
    # vec_scale_f16 / vec_mad_f16 (ops.cpp:1084-1099)
    rng = np.random.default_rng(6000)
    y = rng.standard_normal(256).astype(np.float16).view(np.uint16)
    xv = rng.standard_normal(256).astype(np.float16).view(np.uint16)
    d["vec__scale"] = ref.vec_scale_f16(y, 0.3712)
    d["vec__mad"] = ref.vec_mad_f16(y, xv, 0.8123)
    return d


def gen_models(ref: Reference) -> dict:
    d = {}
    g = build_model_test_gguf()
    with open(os.path.join(OUT, "model_test.gguf"), "wb") as f:
        f.write(g)
    m = ref.model(g)
    l1 = m.forward([1], 0)
    l2 = m.forward([int(np.argmax(l1))], 1)
    d["model_test__l1"], d["model_test__l2"] = l1, l2
    # seeded synthetic tiny Gemma-3 (3 layers, incl. a global layer via pattern)
    cfg = CONFIGS["tiny"]
    gt = build_gemma3_gguf(cfg, seed=7, swa_pattern=[True, False, True])
    m = ref.model(gt)
    prompt = np.array([2, 17, 301, 44, 9], np.int32)
    logits = [m.forward(prompt, 0)]
    toks = [int(np.argmax(logits[-1]))]
    pos = len(prompt)
    for _ in range(5):
        logits.append(m.forward([toks[-1]], pos))
        pos += 1
        toks.append(int(np.argmax(logits[-1])))
    d["tiny__prompt"] = prompt
    d["tiny__logits"] = np.stack(logits)
    d["tiny__tokens"] = np.array(toks, np.int32)
    # the same model with the attention logit soft-cap (model.cpp:511-513) set low enough to bend most scores
    gc = build_gemma3_gguf(cfg, seed=7, swa_pattern=[True, False, True],
                           extra_meta={"attention.logit_softcapping": SOFTCAP})
    m = ref.model(gc)
    logits = [m.forward(prompt, 0)]
    toks = [int(np.argmax(logits[-1]))]
    pos = len(prompt)
    for _ in range(5):
        logits.append(m.forward([toks[-1]], pos))
        pos += 1
        toks.append(int(np.argmax(logits[-1])))
    d["tinycap__logits"] = np.stack(logits)
    d["tinycap__tokens"] = np.array(toks, np.int32)
    d["tinycap__cap"] = np.float32(SOFTCAP)
    return d


def main():
    ref = Reference(n_threads=4)
    np.savez_compressed(os.path.join(OUT, "ops_ref.npz"), **gen_ops(ref))
    np.savez_compressed(os.path.join(OUT, "model_ref.npz"), **gen_models(ref))
    print("wrote", os.listdir(OUT))


if __name__ == "__main__":
    main()
