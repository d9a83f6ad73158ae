"""Diagnostics: which fast kernel family moves the logits away from the
float64-attention oracle?  Runs one model per LLMI_EXACT_PARTS setting in a
subprocess (the env var is read at session creation)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, %r)
from llm_inference_amd.model import Model
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
from oracle.bind import Oracle
cfg = CONFIGS[sys.argv[1]]
g = build_gemma3_gguf(cfg, seed=3)
o = Oracle()
ref = o.model(g, n_threads=8, max_ctx=64).forward(np.random.default_rng(5).integers(4, cfg.vocab, 12).astype(np.int32), 0)
ide = o.model(g, n_threads=8, max_ctx=64, attn_f64=True).forward(np.random.default_rng(5).integers(4, cfg.vocab, 12).astype(np.int32), 0)
m = Model(g, exact=False, max_ctx=64)
got = m.forward(np.random.default_rng(5).integers(4, cfg.vocab, 12).astype(np.int32), 0)
print(f"{sys.argv[1]:8s} parts={sys.argv[2]:28s} vs_ref={np.abs(got-ref).max():.4g} vs_f64={np.abs(got-ide).max():.4g} ref_vs_f64={np.abs(ref-ide).max():.4g}")
""" % ROOT

for cfg in ["mini-1b", "mini-4b"]:
    for parts in ["gemv,norm,attn,logits", "", "norm,attn,logits", "gemv,attn,logits", "gemv,norm,logits",
                  "gemv,norm,attn"]:
        env = dict(os.environ, LLMI_EXACT_PARTS=parts)
        r = subprocess.run([sys.executable, "-c", CHILD, cfg, parts or "-"], env=env, capture_output=True, text=True,
                           timeout=300)
        print(r.stdout.strip() or r.stderr[-2000:], flush=True)
