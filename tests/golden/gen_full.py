"""Golden fixtures at the BASELINE model shapes, by running the REFERENCE
ITSELF (oracle/_ref/libllmref.so: the reference's ops.cpp/gguf.cpp/model.cpp
compiled from /root/reference by oracle/Makefile) on seeded synthetic GGUFs.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/gen_full.py
Writes tests/golden/full_ref.npz with, per case:
  <case>__sha       sha256 of the synthetic GGUF bytes (the test rebuilds the
                    file from the same seed and checks it is the same file)
  <case>__prompt    prompt ids;  <case>__tokens  the reference's greedy ids
                    (first = argmax of the prompt's logits, then one per step)
  <case>__top_idx / __top_val  the 16 largest logits of every step
Only data is committed; no reference source or binary.
"""
from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.bind import Reference  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
# (case, config, seed, prompt length, greedy steps): BASELINE configs[2]'s model
# at full depth and vocabulary, and the 1B model of configs[1]; zero-mean
# (centered) Q4_0 weights so the greedy ids depend on the input
CASES = [("g4b", "gemma-3-4b", 4242, 16, 32), ("g1b", "gemma-3-1b", 1111, 16, 32)]
TOPK = 16


def prompt_of(cfg, seed, n):
    return np.concatenate([[2], np.random.default_rng(seed).integers(4, cfg.vocab, n - 1)]).astype(np.int32)


def run_case(ref, case, cfg_name, seed, n_prompt, n_steps):
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=seed, centered=True)
    m = ref.model(g)
    prompt = prompt_of(cfg, seed, n_prompt)
    lg = m.forward(prompt, 0)
    toks, tops_i, tops_v = [], [], []
    pos = n_prompt
    for step in range(n_steps + 1):
        idx = np.argsort(-lg, kind="stable")[:TOPK]
        tops_i.append(idx.astype(np.int32))
        tops_v.append(lg[idx])
        toks.append(int(np.argmax(lg)))
        if step == n_steps:
            break
        lg = m.forward([toks[-1]], pos)
        pos += 1
    return {f"{case}__sha": np.frombuffer(hashlib.sha256(g.tobytes()).hexdigest().encode(), np.uint8),
            f"{case}__prompt": prompt, f"{case}__tokens": np.array(toks, np.int32),
            f"{case}__top_idx": np.stack(tops_i), f"{case}__top_val": np.stack(tops_v)}


def main():
    ref = Reference(n_threads=os.cpu_count() or 8)
    d = {}
    for c in CASES:
        t0 = time.time()
        d.update(run_case(ref, *c))
        print(c[0], "done in", round(time.time() - t0, 1), "s; tokens", d[f"{c[0]}__tokens"].tolist())
    np.savez_compressed(os.path.join(OUT, "full_ref.npz"), **d)


if __name__ == "__main__":
    main()
