"""Exact mode's batched prompt (VERDICT r5 'Next round' 4): the prompt's tokens before the last run layer by
layer, T at a time (k_exact.hip: xp_norm_kernel, xp_gemm_kernel, the attention kernels' batch form), and the last
one through its decode step.  Every (row, token) keeps the reference's chains (ops.cpp:364-399, model.cpp:430-566),
so the logits must be BIT-IDENTICAL to the token loop's (LLMI_XP_OFF=1), which tests/test_long_models.py and
tests/test_full_models.py pin to the reference's own bits -- at chunk boundaries (LLMI_XP_CHUNK), past a 1024-key
chunk of the accumulate kernel, at head_dim 128 (27B shapes) and for the decode steps that follow.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(g, prompt, forced, monkeypatch, env):
    from llm_inference_amd.model import Model
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m = Model(g, exact=True, max_ctx=len(prompt) + len(forced) + 8)
    assert m.get_info().exact_batched_prefill == (0 if "LLMI_XP_OFF" in env else 1)
    out = [m.forward(prompt, 0)]
    for i, t in enumerate(forced):
        out.append(m.forward(np.array([t], np.int32), len(prompt) + i))
    ids = m.generate(int(np.argmax(out[-1])), len(prompt) + len(forced), 4).tolist()
    m.close()
    for k in env:
        monkeypatch.delenv(k)
    return np.stack(out), ids


@pytest.mark.parametrize("cfg_name,n,chunk", [
    ("mini-4b", 40, None),
    ("mini-4b", 300, "64"),
    ("mini-4b", 1100, None),
    ("mini-1b", 130, "7"),
    ("mini-27b", 1100, "200"),
])
def test_batched_exact_prompt_matches_token_loop(monkeypatch, cfg_name, n, chunk):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=700 + n)
    rng = np.random.default_rng(n)
    prompt = np.concatenate([[2], rng.integers(4, cfg.vocab, n - 1)]).astype(np.int32)
    forced = rng.integers(4, cfg.vocab, 3).astype(np.int32)
    want, ids_want = _run(g, prompt, forced, monkeypatch, {"LLMI_XP_OFF": "1"})
    got, ids_got = _run(g, prompt, forced, monkeypatch, {"LLMI_XP_CHUNK": chunk} if chunk else {})
    diff = np.abs(got - want).max(1)
    print(f"{cfg_name} n={n} chunk={chunk}: max |batched - token loop| per position {diff.tolist()}")
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    assert ids_got == ids_want
