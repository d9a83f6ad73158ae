"""Development: repeat the mini-1b tp 2 replicated-attention comparison (tests/test_tp.py
test_sharded_attention_block) N times in one process; print each rank's max |logit - whole| per run."""
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_inference_amd.model import Model, TPGroup  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402


def main(cfg_name="mini-1b", tp=2, n=6, np_=40, seed=17):
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=seed)
    prompt = np.random.default_rng(19).integers(4, cfg.vocab, np_).astype(np.int32)
    whole = Model(g, exact=False, max_ctx=64)
    ref = whole.forward(prompt, 0)
    whole.close()
    for it in range(n):
        w2 = Model(g, exact=False, max_ctx=64)
        ref2 = w2.forward(prompt, 0)
        w2.close()
        grp = TPGroup(tp)
        out = [None] * tp

        def rank(r):
            m = Model(g, exact=False, max_ctx=64, tp_rank=r, tp_size=tp, tp_group=grp)
            out[r] = m.forward(prompt, 0)
            m.close()

        th = [threading.Thread(target=rank, args=(r,)) for r in range(tp)]
        [t.start() for t in th]
        [t.join(300) for t in th]
        grp.close()
        print(f"run {it}: whole again {float(np.abs(ref2 - ref).max()):.3g}; ranks "
              + " ".join(f"{float(np.abs(o - ref).max()):.3g}" for o in out), flush=True)


if __name__ == "__main__":
    main(*(int(a) if a.isdigit() else a for a in sys.argv[1:]))
