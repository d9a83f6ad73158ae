"""Greedy token selection by int8 screening + exact f16 rescoring
(csrc/k_logits.hip) against the full F16 logits GEMV.

The decode loop (llmi_session_enqueue / generate) picks each token from the
screened candidates; LLMI_FULL_LOGITS=1 keeps the full GEMV + argmax of
model.cpp:1019-1028 / main.cpp:193-194.  The ids must be identical, ties
(first maximal index wins, std::max_element) included:
  * random Gemma-3 1B/4B layer shapes, 64 greedy tokens;
  * every row duplicated (row i + V/2 == row i): each maximum ties, the lower
    index must win;
  * near-ties (the duplicate nudged by one f16 ulp in one column);
  * all rows equal (every row is a candidate: the worst case).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _embd(g, cfg):
    from llm_inference_amd.gguf import GGUFFile
    f = GGUFFile(g)
    t = f.tensor("token_embd.weight")
    s = f.data_section_start + t.tensor_offset
    return g[s:s + t.nbytes].view(np.float16).reshape(cfg.vocab, cfg.n_embd)


@pytest.fixture(params=[False, True], ids=["fast", "exact"])
def exact(request):
    """fast: rescoring in the fast F16 GEMV's order; exact (the exact-order engine): in the reference's AVX2
    order (ops.cpp:552-585), against the full exact F16 GEMV + argmax."""
    return request.param


def _pair(g, monkeypatch, max_ctx=256, exact=False):
    from llm_inference_amd.model import Model
    scr = Model(g, max_ctx=max_ctx, exact=exact)
    monkeypatch.setenv("LLMI_FULL_LOGITS", "1")
    full = Model(g, max_ctx=max_ctx, exact=exact)
    monkeypatch.delenv("LLMI_FULL_LOGITS")
    assert scr.get_info().screened_logits == 1
    assert full.get_info().screened_logits == 0
    return scr, full


def _run(scr, full, cfg, seed, n=48):
    prompt = np.random.default_rng(seed).integers(4, cfg.vocab, 9).astype(np.int32)
    la = scr.forward(prompt, 0)
    lb = full.forward(prompt, 0)
    assert np.array_equal(la.view(np.uint32), lb.view(np.uint32))  # forward keeps the full GEMV
    first = int(np.argmax(la))
    ta = scr.generate(first, len(prompt), n)
    tb = full.generate(first, len(prompt), n)
    assert ta.tolist() == tb.tolist()
    return ta


@pytest.mark.parametrize("cfg_name", ["mini-1b", "mini-4b"])
def test_screen_ids_match_full_logits(cfg_name, monkeypatch, exact):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=13)
    scr, full = _pair(g, monkeypatch, exact=exact)
    _run(scr, full, cfg, 2, n=64)
    # the screened step's two launches (screening GEMV, rescoring; its prep runs in the final norm launch) replace
    # the one F16 GEMV launch (exact mode: the exact GEMV and its argmax launch), and its token feedback carries
    # the next step's embed_norm (one launch fewer)
    assert scr.get_info().kernels_per_token == full.get_info().kernels_per_token - (1 if exact else 0)


def test_screen_ties_first_index(monkeypatch, exact):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-4b"]
    g = build_gemma3_gguf(cfg, seed=17)
    e = _embd(g, cfg)
    h = cfg.vocab // 2
    e[h:2 * h] = e[:h]  # every row has an exact twin V/2 later
    scr, full = _pair(g, monkeypatch, exact=exact)
    ids = _run(scr, full, cfg, 5)
    assert (ids < h).all()  # the lower index of each tied pair


def test_screen_near_ties(monkeypatch, exact):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-1b"]
    g = build_gemma3_gguf(cfg, seed=19)
    e = _embd(g, cfg)
    h = cfg.vocab // 2
    e[h:2 * h] = e[:h]
    bits = e[h:2 * h].view(np.uint16)
    col = np.random.default_rng(1).integers(0, cfg.n_embd, h)
    bits[np.arange(h), col] += np.uint16(1)  # one f16 ulp in one column of each twin
    scr, full = _pair(g, monkeypatch, exact=exact)
    _run(scr, full, cfg, 7)


def test_screen_all_rows_equal(monkeypatch):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["mini-1b"]
    g = build_gemma3_gguf(cfg, seed=23)
    e = _embd(g, cfg)
    e[1:] = e[0]
    scr, full = _pair(g, monkeypatch, max_ctx=64)
    ids = _run(scr, full, cfg, 3, n=8)
    assert (ids == 0).all()
