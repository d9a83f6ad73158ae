"""Development: repeat tests/test_tp.py test_sharded_matches_whole_model (mini-1b, tp 4, rep) N times in one
process; per run print the whole model against its first run, and each rank's max |logit - whole| and whether
its greedy ids match.  usage: LLMI_NO_PREFILL=1 LLMI_NO_BLOCK=1 python scripts/dev/tp_repeat4.py [cfg] [tp] [n]"""
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_inference_amd.model import Model, TPGroup  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402


def main(cfg_name="mini-1b", tp=4, n=10):
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=3)
    prompt = np.random.default_rng(5).integers(4, cfg.vocab, 12).astype(np.int32)
    whole = Model(g, exact=False, max_ctx=64)
    ref = whole.forward(prompt, 0)
    ref_toks = whole.generate(int(np.argmax(ref)), len(prompt), 11)
    whole.close()
    bad = 0
    for it in range(n):
        w2 = Model(g, exact=False, max_ctx=64)
        ref2 = w2.forward(prompt, 0)
        w2.close()
        grp = TPGroup(tp)
        out = [None] * tp

        errs = []

        def rank(r):
            try:
                m = Model(g, exact=False, max_ctx=64, tp_rank=r, tp_size=tp, tp_group=grp)
                lg = m.forward(prompt, 0)
                toks = m.generate(int(np.argmax(lg)), len(prompt), 11)
                out[r] = (lg, toks)
                m.close()
            except Exception as e:  # noqa: BLE001 -- printed below
                errs.append(f"rank {r}: {e}")

        th = [threading.Thread(target=rank, args=(r,)) for r in range(tp)]
        [t.start() for t in th]
        [t.join(300) for t in th]
        grp.close()
        if errs:
            print(f"run {it}: " + " | ".join(errs), flush=True)
            break
        d = [float(np.abs(o[0] - ref).max()) for o in out]
        ids = [o[1].tolist() == ref_toks.tolist() for o in out]
        bad += any(x != 0 for x in d)
        print(f"run {it}: whole again {float(np.abs(ref2 - ref).max()):.3g}; ranks "
              + " ".join(f"{x:.3g}" for x in d) + f"; ids {ids}", flush=True)
    print(f"{bad} of {n} runs differ", flush=True)


if __name__ == "__main__":
    main(*(int(a) if a.isdigit() else a for a in sys.argv[1:]))
