"""Batched prefill of the bench's workload (4B Q4_0, 512 tokens) a few times
(profiling target: rocprofv3 --kernel-trace --stats -- python3 scripts/prefill_run.py)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_amd import _lib  # noqa: E402

_lib.lib()
from llm_inference_amd.model import Model  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "gemma-3-4b"]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
g = build_gemma3_gguf(cfg, seed=1234)
m = Model(g, max_ctx=n + 8)
prompt = np.concatenate([[2], np.random.default_rng(99).integers(4, cfg.vocab, n - 1)]).astype(np.int32)
for i in range(4):
    t0 = time.time()
    m.forward(prompt, 0, want_logits=False)
    print(f"prefill {n} tokens: {(time.time() - t0) * 1e3:.2f} ms", flush=True)
