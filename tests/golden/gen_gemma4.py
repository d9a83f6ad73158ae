"""Gemma-4 golden fixtures made by running the
REFERENCE ITSELF (oracle/_ref/libllmref.so, compiled from /root/reference by
oracle/Makefile) on seeded synthetic Gemma-4 GGUFs (synthetic.build_gemma4_gguf):
per-layer token embeddings + model projection (model.cpp:568-704), shared KV
for the last layers (model.cpp:775-777), V RMSNorm (model.cpp:813-829), the
per-layer embedding step and output scale (model.cpp:926-977), attention
scale 1.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/gen_gemma4.py
Writes tests/golden/gemma4_ref.npz with, per case:
  <case>__sha      sha256 of the synthetic GGUF (the test rebuilds and checks it)
  <case>__prompt   prompt ids;  <case>__tokens  the reference's greedy ids
  <case>__logits   every step's full logits (first row: the prompt's last position)
Only data is committed; no reference source or binary.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from llm_inference_amd.gguf import TensorType as TT  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS4, build_gemma4_gguf  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
# (case, config, seed, swa pattern, per-layer table type, prompt length, greedy steps)
CASES = [
    ("tiny4", "tiny4", 21, [True, False, True, False], TT.F16, 6, 10),
    ("tiny4_q6k", "tiny4", 22, [True, False, False, True], TT.Q6_K, 5, 6),
    ("mini4", "mini4", 23, [True, True, True, False, True, False], TT.F16, 9, 8),
]


def build(case):
    _, cfg, seed, pat, ttype, _, _ = case
    return build_gemma4_gguf(CONFIGS4[cfg], seed=seed, swa_pattern=pat, table_type=ttype)


def prompt_of(case):
    _, cfg, seed, _, _, n, _ = case
    rng = np.random.default_rng(seed)
    return np.concatenate([[2], rng.integers(4, CONFIGS4[cfg].vocab, n - 1)]).astype(np.int32)


def run_case(ref, case):
    name, n_steps = case[0], case[6]
    g = build(case)
    m = ref.model(g)
    prompt = prompt_of(case)
    lg = m.forward(prompt, 0)
    toks, logits = [], []
    pos = len(prompt)
    for step in range(n_steps + 1):
        logits.append(lg)
        toks.append(int(np.argmax(lg)))
        if step == n_steps:
            break
        lg = m.forward([toks[-1]], pos)
        pos += 1
    return {f"{name}__sha": np.frombuffer(hashlib.sha256(g.tobytes()).hexdigest().encode(), np.uint8),
            f"{name}__prompt": prompt, f"{name}__tokens": np.array(toks, np.int32),
            f"{name}__logits": np.stack(logits).astype(np.float32)}


def main():
    from oracle.bind import Reference
    ref = Reference(n_threads=os.cpu_count() or 8)
    d = {}
    for c in CASES:
        d.update(run_case(ref, c))
        print(c[0], "tokens", d[f"{c[0]}__tokens"].tolist())
    np.savez_compressed(os.path.join(OUT, "gemma4_ref.npz"), **d)


if __name__ == "__main__":
    main()
