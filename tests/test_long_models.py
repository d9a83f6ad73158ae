"""BASELINE configs at full depth AND length, against the REFERENCE ITSELF
(VERDICT r2 'Next round' 1 and 2).  tests/golden/long_ref.npz holds the
greedy ids and top-16 logits of the reference's own Model::forward
(oracle/_ref, built from /root/reference; tests/golden/gen_long.py) on
seeded synthetic GGUFs that the tests rebuild and check by sha256:

  g4b_512  Gemma-3 4B Q4_0 (configs[2]): 34 layers, 262,208 F16 logits rows,
           5 local : 1 global rope layers, 512-token prompt + 64 greedy steps;
  g27b     Gemma-3 27B Q4_0 (configs[4]'s model): 62 layers, 32 / 16 heads of
           128, 8-token prompt + 6 greedy steps;
  g4b_512f the g4b_512 model and prompt, then 64 steps fed seeded random ids
           (a random-init model's greedy ids collapse onto a few tokens --
           g4b_512 has 4 distinct ids -- while every forced step's argmax is
           the reference's over a different context: dozens of distinct ids).

Every step is teacher-forced on the reference's ids (forward() of one token
at the reference's next position), or on the fixture's inputs for the forced
case, so each step's logits are comparable.

Exact mode (LLMI_EXACT): the top-16 logits of EVERY step are the reference's
bits, and the ids are the reference's.

Fast mode: the batched prefill (int8 MFMA GEMMs, MFMA attention) and the fast
decode kernels (fp32 split-K attention, reassociated sums).  Stated bound:
at every step the device's value of each of the reference's top-16 logits is
within TOL_ABS of the reference's, the device's argmax equals the
reference's at every step whose top-2 margin exceeds 2 x the largest error
measured on this run, and the free-running device loop (screened token
selection) reproduces the reference's ids up to the first step whose margin
is below that bound -- no agreement-fraction escape hatch.  27B adds the
tensor-parallel check: a tp 8 group (ranks as threads on one device,
LocalCollective) in the per-model default tp mode reproduces the whole-model
session bit for bit.
"""
import hashlib
import os
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
GOLD = os.path.join(ROOT, "tests", "golden", "long_ref.npz")
# |fast - reference| on the reference's top-16 logits (|logit| ~ 1-3 on these centered models): the fast
# attention's fp32 split-K against the reference's f16 accumulator, amplified through 34 / 62 layers of
# Q8_0 re-quantization (measured: see the printed per-step errors)
TOL_ABS = {"g4b_512": 0.05, "g4b_512f": 0.05, "g27b": 0.07}

pytestmark = pytest.mark.gpu


def _fixture(case):
    import gen_long
    d = np.load(GOLD)
    if f"{case}__sha" not in d.files:
        pytest.skip(f"{case} not in long_ref.npz (tests/golden/gen_long.py {case})")
    g = gen_long.gguf_of(case)
    assert hashlib.sha256(g.tobytes()).hexdigest() == bytes(d[f"{case}__sha"]).decode(), \
        "synthetic GGUF differs from the one the fixture was made from"
    f = {k.split("__")[1]: d[k] for k in d.files if k.startswith(case + "__")}
    assert np.array_equal(f["prompt"], gen_long.prompt_of(case))
    return g, f


def _teacher_forced(m, f):
    """Logits of the prompt and of each step fed the reference's ids (or the forced case's inputs):
    [steps + 1, vocab]."""
    prompt, toks = f["prompt"], f["tokens"]
    feed = f["inputs"] if "inputs" in f else toks[:-1]
    out = [m.forward(prompt, 0)]
    for i in range(len(toks) - 1):
        out.append(m.forward([int(feed[i])], len(prompt) + i))
    return np.stack(out)


def _top(L, f):
    return np.take_along_axis(L, f["top_idx"].astype(np.int64), 1)


@pytest.mark.parametrize("case", ["g4b_512", "g4b_512f", "g27b"])
def test_long_exact(case):
    from llm_inference_amd.model import Model
    g, f = _fixture(case)
    m = Model(g, exact=True, max_ctx=len(f["prompt"]) + len(f["tokens"]) + 8)
    L = _teacher_forced(m, f)
    m.close()
    assert L.argmax(1).tolist() == f["tokens"].tolist()
    got = _top(L, f)
    bad = np.nonzero((got.view(np.uint32) != f["top_val"].view(np.uint32)).any(1))[0]
    print(f"{case} exact: {len(L)} steps ({len(set(f['tokens'].tolist()))} distinct ids), top-16 logits "
          f"bit-identical at {len(L) - bad.size}")
    assert bad.size == 0, f"steps {bad.tolist()[:8]} differ from the reference's bits"


@pytest.mark.parametrize("case", ["g4b_512", "g4b_512f", "g27b"])
def test_long_fast(case):
    from llm_inference_amd.model import Model
    g, f = _fixture(case)
    prompt, toks = f["prompt"], f["tokens"]
    n = len(toks) - 1
    max_ctx = len(prompt) + n + 8
    m = Model(g, max_ctx=max_ctx)
    assert m.info.batched_prefill == 1
    F = _teacher_forced(m, f)
    m.close()
    err = np.abs(_top(F, f) - f["top_val"]).max(1)
    bound = 2.0 * float(err.max())
    tv = f["top_val"]
    margin = tv[:, 0] - tv[:, 1]
    decided = margin > bound
    agree = F.argmax(1) == toks
    print(f"{case} fast: |top-16 logits - reference| per step max {float(err.max()):.3g} mean {float(err.mean()):.3g} "
          f"(|logit| up to {float(np.abs(tv).max()):.3g}); decided steps {int(decided.sum())}/{len(decided)}, "
          f"argmax agreement {int(agree.sum())}/{len(agree)}")
    assert err.max() <= TOL_ABS[case]
    assert agree[decided].all(), "fast argmax differs where the reference's margin exceeds the error bound"
    if "inputs" in f:
        return  # forced inputs: no free-running sequence to compare
    # free-running device loop (screened token selection)
    m2 = Model(g, max_ctx=max_ctx)
    lg = m2.forward(prompt, 0)
    run = [int(np.argmax(lg))] + m2.generate(int(np.argmax(lg)), len(prompt), n).tolist()
    m2.close()
    first_diff = next((i for i in range(len(run)) if run[i] != toks[i]), None)
    print(f"{case} fast free-running ids: identical for {first_diff if first_diff is not None else len(run)} "
          f"of {len(run)} steps")
    if first_diff is not None:
        assert not decided[first_diff], f"free-running ids diverge at a decided step {first_diff}"


def test_27b_tp8_matches_whole_model(monkeypatch):
    """configs[4]'s model at full depth as a tp 8 group (8 ranks as host threads on one device, exchanging over
    the one-shot push all-gather through per-rank mailboxes, LocalCollective: RCCL refuses two ranks per GPU) in
    the per-model default tp mode (head-sharded for 27B, Session::setup_tp), with every rank and the whole model
    pinned to the same per-projection kernels (token loop, no attention block: LLMI_NO_PREFILL / LLMI_NO_BLOCK):
    logits and greedy ids bit-identical to the whole-model session.  The production path (batched prefill,
    default launches) is test_27b_tp8_production_path below."""
    from llm_inference_amd.model import Model, TPGroup
    g, f = _fixture("g27b")
    prompt = f["prompt"]
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    monkeypatch.setenv("LLMI_NO_BLOCK", "1")
    monkeypatch.delenv("LLMI_TP_HEAD_SHARD", raising=False)
    whole = Model(g, max_ctx=32)
    ref = whole.forward(prompt, 0)
    ref_toks = whole.generate(int(np.argmax(ref)), len(prompt), 4)
    whole.close()
    out = _tp8_ranks(g, lambda m: (lambda lg: (lg, m.generate(int(np.argmax(lg)), len(prompt), 4)))(
        m.forward(prompt, 0)))
    for r, (lg, toks) in enumerate(out):
        np.testing.assert_array_equal(lg.view(np.uint32), ref.view(np.uint32), err_msg=f"rank {r} logits")
        assert toks.tolist() == ref_toks.tolist(), f"rank {r} ids"
    print(f"27B tp8 (default mode): 8 ranks bit-identical to the whole model; ids {ref_toks.tolist()}")


def _tp8_ranks(g, body, tp=8, max_ctx=32):
    """body(model) on each of tp ranks (host threads, one TPGroup); the ranks' results in rank order."""
    from llm_inference_amd.model import Model, TPGroup
    grp = TPGroup(tp)
    out, errs = [None] * tp, []

    def rank(r):
        try:
            m = Model(g, max_ctx=max_ctx, tp_rank=r, tp_size=tp, tp_group=grp)
            out[r] = body(m)
            m.close()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append((r, e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(tp)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    grp.close()
    assert not errs, errs
    return out


def test_27b_tp8_exact_matches_reference(monkeypatch):
    """configs[4]'s model at full depth, a tp 8 group in EXACT mode (the exact-order engine, rows sharded): every
    rank's teacher-forced top-16 logits are the REFERENCE's own bits at every step and its argmax the reference's
    ids (a bit-exact path for configs[4])."""
    for k in ("LLMI_NO_PREFILL", "LLMI_NO_BLOCK", "LLMI_TP_HEAD_SHARD"):
        monkeypatch.delenv(k, raising=False)
    g, f = _fixture("g27b")
    max_ctx = len(f["prompt"]) + len(f["tokens"]) + 8

    def body(m):
        assert m.get_info().exact_engine == 1
        return _teacher_forced(m, f)

    out = _tp8_ranks_exact(g, body, max_ctx)
    for r, L in enumerate(out):
        assert L.argmax(1).tolist() == f["tokens"].tolist(), f"rank {r} ids"
        got = _top(L, f)
        bad = np.nonzero((got.view(np.uint32) != f["top_val"].view(np.uint32)).any(1))[0]
        assert bad.size == 0, f"rank {r}: steps {bad.tolist()[:8]} differ from the reference's bits"
    print(f"27B tp8 exact: 8 ranks, {len(out[0])} steps, top-16 logits bit-identical to the reference")


def _tp8_ranks_exact(g, body, max_ctx, tp=8):
    from llm_inference_amd.model import Model, TPGroup
    grp = TPGroup(tp)
    out, errs = [None] * tp, []

    def rank(r):
        try:
            m = Model(g, exact=True, max_ctx=max_ctx, tp_rank=r, tp_size=tp, tp_group=grp)
            out[r] = body(m)
            m.close()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append((r, e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(tp)]
    for t in th:
        t.start()
    for t in th:
        t.join(900)
    grp.close()
    assert not errs, errs
    return out


def test_27b_tp8_production_path(monkeypatch):
    """The tp 8 group on the production path (no switches: the ranks' batched prefill and default decode
    launches) against the REFERENCE's own 62-layer fixture: every rank's teacher-forced top-16 logits within
    TOL_ABS["g27b"] of the reference's, argmax identical at every step whose margin exceeds 2 x the measured
    error, every rank bit-identical to rank 0."""
    for k in ("LLMI_NO_PREFILL", "LLMI_NO_BLOCK", "LLMI_NO_FUSE", "LLMI_TP_HEAD_SHARD"):
        monkeypatch.delenv(k, raising=False)
    g, f = _fixture("g27b")
    out = _tp8_ranks(g, lambda m: (m.get_info().batched_prefill, _teacher_forced(m, f)))
    assert all(bp == 1 for bp, _ in out), "the ranks' prompt must take the batched prefill"
    L = out[0][1]
    for r, (_, Lr) in enumerate(out):
        np.testing.assert_array_equal(Lr.view(np.uint32), L.view(np.uint32), err_msg=f"rank {r} vs rank 0")
    err = np.abs(_top(L, f) - f["top_val"]).max(1)
    tv = f["top_val"]
    decided = tv[:, 0] - tv[:, 1] > 2.0 * float(err.max())
    agree = L.argmax(1) == f["tokens"]
    print(f"27B tp8 production path: |top-16 - reference| max {float(err.max()):.3g}, decided steps "
          f"{int(decided.sum())}/{len(decided)}, argmax agreement {int(agree.sum())}/{len(agree)}")
    assert err.max() <= TOL_ABS["g27b"]
    assert agree[decided].all()
