"""Development: characterise the one-GPU tensor-parallel group's wrong-logits failure.

Per run: a whole-model session again, then a TPGroup lifetime whose ranks each run forward(prompt) TWICE (the second
forward overwrites the same KV rows: a persistent corruption -- weights, tables -- repeats, a transient race does not)
and a short greedy decode.  Modes switch the suspects one at a time (the environment is read at session creation):
  default  -- the fused push exchange (the product default)
  copy     -- device-to-device slice copies (no mailbox at all)
  serial   -- the ranks' sessions constructed one at a time (a lock around Model())
  fused0   -- the standalone push-exchange launches (LLMI_TP_FUSED=0)
  ctorbar  -- every rank's session constructed before any rank's first forward (ctorbar0: and LLMI_TP_FUSED=0)
(round 5: the modes that split the three causes of DESIGN.md section 7; the removed A/B builds -- null-stream
initialisation, no deferred frees, a 16 MiB + 64 KiB mailbox -- are recorded there with their counts)
usage: python scripts/dev/tp_diag.py case seconds_per_mode mode[,mode...]
  case: 27b8pf (mini-27b tp 8, 70-token batched prefill) | 4b2dec (mini-4b tp 2, decode kernels only)"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_inference_amd.model import Model, TPGroup  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

CASES = {
    "27b8pf": dict(cfg="mini-27b", tp=8, seed=13, pseed=15, n=70, gen=6, ctx=128, env={"LLMI_NO_BLOCK": "1"}),
    "4b2dec": dict(cfg="mini-4b", tp=2, seed=3, pseed=5, n=12, gen=11, ctx=64,
                   env={"LLMI_NO_BLOCK": "1", "LLMI_NO_PREFILL": "1"}),
    "1b4shard": dict(cfg="mini-1b", tp=4, seed=3, pseed=5, n=12, gen=11, ctx=64,
                     env={"LLMI_NO_BLOCK": "1", "LLMI_NO_PREFILL": "1", "LLMI_TP_HEAD_SHARD": "1"}),
    "1b4dec": dict(cfg="mini-1b", tp=4, seed=3, pseed=5, n=12, gen=11, ctx=64,
                   env={"LLMI_NO_BLOCK": "1", "LLMI_NO_PREFILL": "1"}),
}
MODES = {"default": {}, "copy": {"LLMI_TP_EXCHANGE": "copy"}, "serial": {}, "fused0": {"LLMI_TP_FUSED": "0"},
         "ctorbar": {}, "ctorbar0": {"LLMI_TP_FUSED": "0"}}


def lifetime(g, c, prompt, serial, ctorbar=False):
    grp = TPGroup(c["tp"])
    lock = threading.Lock()
    bar = threading.Barrier(c["tp"])
    out, errs = [None] * c["tp"], []

    def rank(r):
        try:
            kw = dict(exact=False, max_ctx=c["ctx"], tp_rank=r, tp_size=c["tp"], tp_group=grp)
            if serial:
                with lock:
                    m = Model(g, **kw)
            else:
                m = Model(g, **kw)
            if ctorbar:  # every rank's session constructed before any rank's first forward
                bar.wait()
            lg1 = m.forward(prompt, 0)
            lg2 = m.forward(prompt, 0)
            toks = m.generate(int(np.argmax(lg1)), len(prompt), c["gen"])
            out[r] = (lg1, lg2, toks)
            m.close()
        except Exception as e:  # noqa: BLE001 -- printed
            errs.append(f"rank {r}: {e}")

    th = [threading.Thread(target=rank, args=(r,)) for r in range(c["tp"])]
    [t.start() for t in th]
    [t.join(300) for t in th]
    grp.close()
    return out, errs


def main(case, secs, modes):
    c = CASES[case]
    os.environ.setdefault("LLMI_TP_BARRIER_S", "10")
    for k, v in c["env"].items():
        os.environ[k] = v
    cfg = CONFIGS[c["cfg"]]
    g = build_gemma3_gguf(cfg, seed=c["seed"])
    prompt = np.random.default_rng(c["pseed"]).integers(4, cfg.vocab, c["n"]).astype(np.int32)
    whole = Model(g, exact=False, max_ctx=c["ctx"])
    ref = whole.forward(prompt, 0)
    ref_toks = whole.generate(int(np.argmax(ref)), len(prompt), c["gen"])
    whole.close()
    print(f"case {case}: ref logits[:3] {ref[:3]}", flush=True)
    for mode in modes.split(","):
        env = MODES[mode]
        for k, v in env.items():
            os.environ[k] = v
        t0, it, bad = time.time(), 0, 0
        while time.time() - t0 < secs:
            w2 = Model(g, exact=False, max_ctx=c["ctx"])
            ref2 = w2.forward(prompt, 0)
            w2.close()
            out, errs = lifetime(g, c, prompt, mode == "serial", mode.startswith("ctorbar"))
            if errs:
                print(f"{mode} run {it}: ERR " + " | ".join(errs), flush=True)
                bad += 1
                it += 1
                continue
            d1 = [float(np.abs(o[0] - ref).max()) for o in out]
            d2 = [float(np.abs(o[1] - ref).max()) for o in out]
            ids = sum(o[2].tolist() == ref_toks.tolist() for o in out)
            agree = all(np.array_equal(o[0], out[0][0]) for o in out)
            fail = any(d1) or any(d2) or ids != len(out)
            bad += fail
            if fail or it % 5 == 0:
                print(f"{mode} run {it}: whole again {float(np.abs(ref2 - ref).max()):.3g}; fwd1 "
                      + " ".join(f"{x:.3g}" for x in d1) + "; fwd2 " + " ".join(f"{x:.3g}" for x in d2)
                      + f"; ids ok {ids}/{len(out)}; ranks agree {agree}"
                      + (f"; rank0 fwd1[:3] {out[0][0][:3]}" if fail else ""), flush=True)
            it += 1
        print(f"== {mode}: {bad} of {it} runs differ", flush=True)
        for k in env:
            del os.environ[k]


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3])
