"""A session's results must not depend on what it ran before (VERDICT r5 'Next round' 1).

The round-5 driver bench showed the fast path's first forced position 37.2 off the reference after the
decode loop AND Model.time_kernel had run on the same session: time_kernel relaunched the attention blocks
alone, and the block's granule tag was advanced by the NEXT layer's gate_up launch (which time_kernel does
not pair with it), so the next real step's block took the last timed launch's leftover granules for its own.
The block now advances its own tag when its last work-group retires (k_attn.hip block_retire).

Each case runs a session through the bench's sequence -- prompt, greedy decode loop (hipGraph replays),
every kernel family of time_kernel -- and then the parity sequence (the prompt again from position 0, then
teacher-forced single tokens), and requires the logits BIT-IDENTICAL to a fresh session's on the same calls.
The same with only the decode loop before (the folded next-token embedding, the token ring), with the
token loop instead of the batched prefill, and for exact mode.
"""
import numpy as np
import pytest

FORCED = 6


def _gguf(cfg_name, seed):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    return cfg, build_gemma3_gguf(cfg, seed=seed)


def _parity_run(m, prompt, forced):
    out = [m.forward(prompt, 0)]
    for i, t in enumerate(forced):
        out.append(m.forward(np.array([t], np.int32), len(prompt) + i))
    return np.stack(out)


def _history(m, prompt, steps, kernels):
    m.forward(prompt, 0, want_logits=False)
    m.enqueue(m.last_argmax, len(prompt), steps)
    m.sync(steps)
    for which in kernels:
        m.time_kernel(which, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_name,kernels", [
    ("mini-4b", (0, 3, 4, 2, 1, 5)),
    ("mini-4b", ()),
    ("mini-1b", (0, 3, 4, 2, 1)),
    ("mini-27b", (0, 3, 4, 2, 1)),
])
def test_forward_after_decode_loop_and_timing_matches_fresh(cfg_name, kernels):
    from llm_inference_amd.model import Model
    cfg, g = _gguf(cfg_name, 606)
    rng = np.random.default_rng(7)
    prompt = np.concatenate([[2], rng.integers(4, cfg.vocab, 299)]).astype(np.int32)
    forced = rng.integers(4, cfg.vocab, FORCED).astype(np.int32)
    fresh = Model(g, max_ctx=640)
    want = _parity_run(fresh, prompt, forced)
    fresh.close()
    m = Model(g, max_ctx=640)
    _history(m, prompt, 40, kernels)
    got = _parity_run(m, prompt, forced)
    diff = np.abs(got - want).max(1)
    print(f"{cfg_name} kernels {kernels}: max |logits - fresh session| per position {np.round(diff, 5).tolist()}")
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    m.close()


@pytest.mark.gpu
def test_token_loop_after_decode_loop_matches_fresh(monkeypatch):
    """The token loop (no batched prefill) through the step graph after the decode-loop graph ran."""
    from llm_inference_amd.model import Model
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    cfg, g = _gguf("mini-4b", 607)
    rng = np.random.default_rng(8)
    prompt = np.concatenate([[2], rng.integers(4, cfg.vocab, 47)]).astype(np.int32)
    forced = rng.integers(4, cfg.vocab, FORCED).astype(np.int32)
    fresh = Model(g, max_ctx=256)
    want = _parity_run(fresh, prompt, forced)
    fresh.close()
    m = Model(g, max_ctx=256)
    _history(m, prompt, 24, (0, 3, 4, 2))
    got = _parity_run(m, prompt, forced)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    m.close()


@pytest.mark.gpu
def test_exact_after_decode_loop_matches_fresh():
    from llm_inference_amd.model import Model
    cfg, g = _gguf("mini-4b", 608)
    rng = np.random.default_rng(9)
    prompt = np.concatenate([[2], rng.integers(4, cfg.vocab, 39)]).astype(np.int32)
    forced = rng.integers(4, cfg.vocab, FORCED).astype(np.int32)
    fresh = Model(g, exact=True, max_ctx=256)
    want = _parity_run(fresh, prompt, forced)
    fresh.close()
    m = Model(g, exact=True, max_ctx=256)
    _history(m, prompt, 24, ())
    got = _parity_run(m, prompt, forced)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    m.close()


def _mem():
    import ctypes
    from llm_inference_amd import _lib
    out = (ctypes.c_ulonglong * 4)()
    assert _lib.lib().llmi_selftest(2, out) == 0
    return int(out[0]), int(out[1]), int(out[2])


@pytest.mark.gpu
def test_memory_bounded_with_a_long_lived_session():
    """a long-lived session plus sessions created and closed one after another must not grow the
    sessions' device memory (the round-5 graveyard held every closed session's blocks until the LAST session
    ended).  Released blocks are reused; nothing stays held back once no session is being constructed."""
    from llm_inference_amd.model import Model
    cfg, g = _gguf("mini-1b", 609)
    keep = Model(g, max_ctx=128)
    base = None
    for i in range(5):
        m = Model(g, max_ctx=128)
        m.forward(np.array([2, 5, 9], np.int32), 0)
        m.close()
        live, cached, grave = _mem()
        print(f"cycle {i}: allocated {live >> 20} MiB, kept for reuse {cached >> 20} MiB, held back {grave >> 20} MiB")
        assert grave == 0
        base = live if base is None else base
        assert live == base, "device memory grows with every session created and closed"
    keep.close()
