"""Development: find the first launch whose output differs in a failing one-GPU tensor-parallel lifetime.

A reference lifetime with the ranks' sessions constructed one at a time (0 failures in 690, tp_diag.py), then
lifetimes with the sessions constructed together; every rank runs llmi_session_trace over the prompt (the token
loop, eager, a host copy of every launch's output).  For a lifetime whose taps differ from the reference: the
first differing tap per rank (token, name, layer), how many elements differ and where.
usage: python scripts/dev/tp_trace_diff.py case lifetimes   (case: as tp_diag.py)"""
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_inference_amd.model import Model, TPGroup  # noqa: E402
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tp_diag import CASES  # noqa: E402


def lifetime(g, c, prompt, serial):
    grp = TPGroup(c["tp"])
    lock = threading.Lock()
    out, errs = [None] * c["tp"], []

    def rank(r):
        try:
            kw = dict(exact=False, max_ctx=c["ctx"], tp_rank=r, tp_size=c["tp"], tp_group=grp)
            if serial:
                with lock:
                    m = Model(g, **kw)
            else:
                m = Model(g, **kw)
            out[r] = m.trace(prompt, 0)
            m.close()
        except Exception as e:  # noqa: BLE001 -- printed
            errs.append(f"rank {r}: {e}")

    th = [threading.Thread(target=rank, args=(r,)) for r in range(c["tp"])]
    [t.start() for t in th]
    [t.join(300) for t in th]
    grp.close()
    return out, errs


def first_diff(ref, got):
    tok = 0
    for i, ((n, l, b), (n2, l2, b2)) in enumerate(zip(ref, got)):
        if n == "token":
            tok += 1
        if (n, l) != (n2, l2):
            return f"tap {i}: launch order differs ({n},{l}) vs ({n2},{l2})"
        if b != b2:
            dt = np.uint8 if len(b) % 4 else np.uint32
            a, z = np.frombuffer(b, dt), np.frombuffer(b2, dt)
            idx = np.nonzero(a != z)[0]
            fa = np.frombuffer(b, np.float32) if len(b) % 4 == 0 else None
            fz = np.frombuffer(b2, np.float32) if len(b2) % 4 == 0 else None
            vals = "" if fa is None else " values ref/got " + " ".join(
                f"{fa[j]:.5g}/{fz[j]:.5g}" for j in idx[:6])
            return (f"token {tok} tap {i} {n} layer {l}: {idx.size} of {a.size} words differ, first at "
                    f"{idx[:8].tolist()}{vals}")
    return None


def main(case, n):
    c = CASES[case]
    for k, v in c["env"].items():
        os.environ[k] = v
    os.environ.setdefault("LLMI_TP_BARRIER_S", "10")
    cfg = CONFIGS[c["cfg"]]
    g = build_gemma3_gguf(cfg, seed=c["seed"])
    prompt = np.random.default_rng(c["pseed"]).integers(4, cfg.vocab, c["n"]).astype(np.int32)
    ref, errs = lifetime(g, c, prompt, True)
    assert not errs, errs
    print(f"reference lifetime: {len(ref[0])} taps per rank", flush=True)
    bad = 0
    for it in range(n):
        out, errs = lifetime(g, c, prompt, False)
        if errs:
            print(f"run {it}: ERR {errs}", flush=True)
            continue
        d = [first_diff(ref[r], out[r]) for r in range(c["tp"])]
        if any(d):
            bad += 1
            print(f"run {it}:", flush=True)
            for r, x in enumerate(d):
                print(f"  rank {r}: {x}", flush=True)
        elif it % 10 == 0:
            print(f"run {it}: identical", flush=True)
    print(f"{bad} of {n} lifetimes differ", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
