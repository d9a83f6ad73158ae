"""Golden fixtures for the BASELINE configs' full depth AND length, by running
the REFERENCE ITSELF (oracle/_ref/libllmref.so: the reference's ops.cpp /
gguf.cpp / model.cpp compiled from /root/reference by oracle/Makefile) on
seeded synthetic GGUFs (VERDICT r2 'Next round' 1 and 2):

  g4b_512  Gemma-3 4B Q4_0 (configs[2]): 34 layers, 262,208 F16 logits rows,
           the 5-local : 1-global sliding-window rope pattern, a 512-token
           prompt, then 64 greedy steps;
  g27b     Gemma-3 27B Q4_0 (configs[4]'s model): 62 layers, 32 / 16 heads of
           128, 21,504 hidden units, an 8-token prompt, then 6 greedy steps;
  g4b_512f the g4b_512 model and prompt, then 64 steps whose INPUTS are seeded
           random ids (a random-init model's free-running greedy ids collapse
           onto a few tokens -- g4b_512 has 4 distinct ids in 65 steps -- while
           every forced step's argmax is a function of a different context:
           the reference's own ids, many distinct ones, at every step).

Run in the build container (needs /root/reference; ~25 GB of host memory for
the 27B file):
    make -C oracle ref && python tests/golden/gen_long.py [case ...]
Writes tests/golden/long_ref.npz with, per case:
  <case>__sha       sha256 of the synthetic GGUF bytes (the test rebuilds the
                    file from the same seed and checks it first)
  <case>__prompt    prompt ids;  <case>__tokens  the reference's greedy ids
                    (first = argmax of the prompt's logits, then one per step)
  <case>__inputs    (forced cases) the ids fed at each step instead of the
                    previous step's argmax
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
TOPK = 16


def swa_4b():
    return [(i % 6) != 5 for i in range(CONFIGS["gemma-3-4b"].n_layer)]


# case -> (config, seed, prompt length, greedy steps, build kwargs)
CASES = {
    "g4b_512": ("gemma-3-4b", 4343, 512, 64, dict(centered=True, swa_pattern=swa_4b())),
    "g27b": ("gemma-3-27b", 2727, 8, 6, dict(centered=True)),
    "g4b_512f": ("gemma-3-4b", 4343, 512, 64, dict(centered=True, swa_pattern=swa_4b())),
}
FORCED = {"g4b_512f"}


def inputs_of(case):
    """The forced cases' step inputs: seeded random ids (step i feeds inputs[i] at position len(prompt) + i)."""
    cfg_name, seed, _, n_steps, _ = CASES[case]
    return np.random.default_rng(seed + 1).integers(4, CONFIGS[cfg_name].vocab, n_steps).astype(np.int32)


def gguf_of(case):
    cfg_name, seed, _, _, kw = CASES[case]
    return build_gemma3_gguf(CONFIGS[cfg_name], seed=seed, **kw)


def prompt_of(case):
    cfg_name, seed, n, _, _ = CASES[case]
    cfg = CONFIGS[cfg_name]
    return np.concatenate([[2], np.random.default_rng(seed).integers(4, cfg.vocab, n - 1)]).astype(np.int32)


def run_case(ref, case):
    n_steps = CASES[case][3]
    g = gguf_of(case)
    sha = hashlib.sha256(g.tobytes()).hexdigest()
    m = ref.model(g)
    prompt = prompt_of(case)
    lg = m.forward(prompt, 0)
    toks, tops_i, tops_v = [], [], []
    pos = len(prompt)
    forced = inputs_of(case) if case in FORCED else None
    for step in range(n_steps + 1):
        idx = np.argsort(-lg, kind="stable")[:TOPK]
        tops_i.append(idx.astype(np.int32))
        tops_v.append(lg[idx])
        toks.append(int(np.argmax(lg)))
        if step == n_steps:
            break
        lg = m.forward([int(forced[step]) if forced is not None else toks[-1]], pos)
        pos += 1
    del m
    out = {f"{case}__sha": np.frombuffer(sha.encode(), np.uint8),
           f"{case}__prompt": prompt, f"{case}__tokens": np.array(toks, np.int32),
           f"{case}__top_idx": np.stack(tops_i), f"{case}__top_val": np.stack(tops_v)}
    if forced is not None:
        out[f"{case}__inputs"] = forced
    return out


def main():
    cases = sys.argv[1:] or list(CASES)
    path = os.path.join(OUT, "long_ref.npz")
    d = dict(np.load(path)) if os.path.exists(path) else {}
    ref = Reference(n_threads=os.cpu_count() or 8)
    for c in cases:
        t0 = time.time()
        d.update(run_case(ref, c))
        print(c, "done in", round(time.time() - t0, 1), "s; tokens", d[f"{c}__tokens"].tolist(), flush=True)
        np.savez_compressed(path, **d)


if __name__ == "__main__":
    main()
