"""The drop-in boundary end to end: the REFERENCE's own model.cpp/gguf.cpp,
compiled unchanged with integration/ops_mi355x.cpp in place of ops.cpp
(oracle/Makefile target `dropin`, output oracle/_ref/dropin_mi355x), runs
Model::forward with every ops.h call served by libllmi.so on the GPU.

Exact mode (the compat layer's default): GEMVs, quantizers, norms, rope and
the f16 attention vector ops are bit-identical to the reference's AVX2
kernels; the remaining arithmetic (attention scores, softmax bookkeeping,
GELU) is the reference's own CPU code.  So the logits must equal the
reference's fixtures (tests/golden/model_ref.npz, recorded from the reference
build) to 1e-5 and the greedy ids exactly.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "dropin_mi355x")


def run(gguf_path, n_decode, prompt):
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/dropin_mi355x not built (needs /root/reference at build time)")
    out = subprocess.run([BIN, gguf_path, str(n_decode)] + [str(int(t)) for t in prompt], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rows = []
    for line in out.stdout.splitlines():
        f = line.split()
        if f[0] == "model":  # several files in one process: a separator line per model
            continue
        assert f[0] == "logits"
        rows.append((int(f[1]), int(f[2]), np.array([float(v) for v in f[3:]], np.float32)))
    return rows


def test_dropin_model_test_gguf(golden_models):
    rows = run(os.path.join(ROOT, "tests", "golden", "model_test.gguf"), 1, [1])
    (p0, a0, l0), (p1, a1, l1) = rows
    np.testing.assert_allclose(l0, golden_models["model_test__l1"], atol=1e-5, rtol=0)
    assert a0 == int(np.argmax(golden_models["model_test__l1"]))
    np.testing.assert_allclose(l1, golden_models["model_test__l2"], atol=1e-5, rtol=0)


def test_dropin_tiny_greedy(golden_models, tmp_path):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    g = build_gemma3_gguf(CONFIGS["tiny"], seed=7, swa_pattern=[True, False, True])
    path = tmp_path / "tiny.gguf"
    path.write_bytes(bytes(g))
    ref_logits, ref_toks = golden_models["tiny__logits"], golden_models["tiny__tokens"]
    rows = run(str(path), len(ref_toks) - 1, golden_models["tiny__prompt"])
    assert [a for _, a, _ in rows] == ref_toks.tolist()
    for i, (_, _, lg) in enumerate(rows):
        np.testing.assert_allclose(lg, ref_logits[i][:16], atol=1e-5, rtol=0)


def test_dropin_two_models_one_process(oracle, tmp_path):
    """Two same-shape GGUFs (different seeds) run one after another in ONE
    process (model_test.cpp:394/410/463 builds several Models from heap
    buffers the same way): the second model's freed-and-reused addresses must
    not serve the first model's cached device weights (ops_mi355x.cpp content
    fingerprint).  Each model's logits equal the oracle's (= the reference's)
    for its own file."""
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS["tiny"]
    paths, models = [], []
    for seed in (7, 8):
        g = build_gemma3_gguf(cfg, seed=seed, swa_pattern=[True, False, True])
        p = tmp_path / f"m{seed}.gguf"
        p.write_bytes(bytes(g))
        paths.append(str(p))
        models.append(oracle.model(g, n_threads=4, max_ctx=64))
    prompt = [2, 17, 301, 44, 9]
    rows = run(",".join(paths), 2, prompt)
    assert len(rows) == 2 * 3
    for mi, om in enumerate(models):
        lg = om.forward(prompt, 0)
        _, a, l0 = rows[3 * mi]
        assert a == int(np.argmax(lg))
        np.testing.assert_allclose(l0, lg[:16], atol=1e-5, rtol=0)


def test_dropin_same_shape_one_block_edited(oracle, tmp_path):
    """Two GGUFs identical except ONE Q4_0 block in the middle of a weight
    (bytes the round-2 sampled fingerprint never read: 64 windows of 64 B).
    Run back to back in one process, the second file's mmap may land at the
    first's address with the same tensor shapes: the compat layer's weight
    cache must see the edit (ops_mi355x.cpp hashes buffers up to 64 MiB
    whole) -- each model's logits equal the oracle's for its own bytes."""
    from llm_inference_amd.gguf import GGUFFile
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    g = np.array(build_gemma3_gguf(CONFIGS["tiny"], seed=7, swa_pattern=[True, False, True]), np.uint8)
    f = GGUFFile(g)
    t = f.tensor("blk.0.ffn_up.weight")
    start = f.data_section_start + t.tensor_offset
    mid = start + (t.nbytes // 2 // 18) * 18 + 37 * 18  # a block boundary off the 64 sampled windows
    g2 = g.copy()
    g2[mid + 2:mid + 18] ^= 0x5A  # the block's nibbles (its f16 scale kept)
    assert not np.array_equal(g, g2)
    paths = []
    for i, gg in enumerate((g, g2)):
        p = tmp_path / f"e{i}.gguf"
        p.write_bytes(gg.tobytes())
        paths.append(str(p))
    prompt = [2, 17, 301, 44, 9]
    rows = run(",".join(paths), 1, prompt)
    assert len(rows) == 2 * 2
    outs = []
    for mi, gg in enumerate((g, g2)):
        lg = oracle.model(gg, n_threads=4, max_ctx=64).forward(prompt, 0)
        _, a, l0 = rows[2 * mi]
        assert a == int(np.argmax(lg))
        np.testing.assert_allclose(l0, lg[:16], atol=1e-5, rtol=0)
        outs.append(lg)
    assert np.abs(outs[0][:16] - outs[1][:16]).max() > 1e-3, "the edit must change the compared logits"
