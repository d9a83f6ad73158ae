"""Layer-by-layer dumps: llmi_session_dump writes the
reference's --verbose intermediates in tensor.h's print_tensor format, and
scripts/compare_dumps.py (the compare_tensors.py counterpart) pairs them
by name and occurrence.

Fixture: tests/golden/dump_tiny_ref.txt, recorded from the reference itself
(oracle/_ref/libllmref.so with verbose_g on, tests/golden/gen_dumps.py) on
the seeded 'tiny' Gemma-3, prompt [2, 17, 301] one token per forward.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "scripts"))
sys.path.insert(0, os.path.join(HERE, "golden"))
from compare_dumps import compare, parse  # noqa: E402

FIXTURE = os.path.join(HERE, "golden", "dump_tiny_ref.txt")
OURS = ["inp_scaled", "attn_norm-{l}", "Qcur-{l}", "Kcur-{l}", "Vcur-{l}", "kqv_out-{l}",
        "attention results (node_30 for MUL_MAT)-{l}", "sa_out-{l}", "ffn_norm-{l}", "ffn_geglu-{l}",
        "ffn_out-{l}", "l_out-{l}", "result_norm", "result_output"]


def _names(n_layer=3):
    out = set()
    for n in OURS:
        out |= {n.format(l=l) for l in range(n_layer)} if "{l}" in n else {n}
    return out


def test_fixture_parses_and_pairs():
    ref = open(FIXTURE).read()
    blocks = parse(ref)
    names = {b["name"] for b in blocks}
    assert _names() <= names  # every tensor the device dump writes is one the reference prints
    q = [b for b in blocks if b["name"] == "Qcur-0"]
    assert len(q) == 3 and q[0]["shape"] == [256, 1, 1, 1] and len(q[0]["values"]) == 6
    assert [b["shape"][0] for b in blocks if b["name"] == "result_output"] == [512] * 3
    rows, only_a, only_b = compare(ref, ref)
    assert rows and all(r[-1] for r in rows) and not only_a and not only_b
    # a perturbed sum is flagged
    bad = ref.replace("sum = " + ref.split("sum = ")[5].split()[0], "sum = 1234.5", 1)
    rows, _, _ = compare(ref, bad)
    assert sum(not r[-1] for r in rows) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [True, False])
def test_session_dump_matches_reference(exact, tmp_path):
    from gen_dumps import TINY_PROMPT, tiny_gguf
    from llm_inference_amd.model import Model
    m = Model(tiny_gguf(), exact=exact, max_ctx=64)
    out = str(tmp_path / "ours.txt")
    m.dump(TINY_PROMPT, 0, out)
    ours = open(out).read()
    blocks = parse(ours)
    assert {b["name"] for b in blocks} == _names()
    assert len(blocks) == len(TINY_PROMPT) * (len(OURS) - 3) * 3 + len(TINY_PROMPT) * 3
    # exact mode: the reference's arithmetic (device expf / tanhf ulps aside);
    # fast mode: reassociated reductions + fp32 split-K attention (model tests' bound)
    tol = 2e-3 if exact else 3e-2
    rows, only_ref, only_ours = compare(open(FIXTURE).read(), ours, tol)
    assert not only_ours
    worst = max(rows, key=lambda r: r[4] / max(1.0, abs(r[2])))
    print(f"{len(rows)} pairs; worst |d sum| {worst[4]:.3g} at {worst[0]}#{worst[1]}; "
          f"max mse {max(r[5] for r in rows):.3g}")
    assert all(r[-1] for r in rows), [r[:5] for r in rows if not r[-1]][:5]
    assert max(r[5] for r in rows) < (1e-6 if exact else 3e-3)  # fast: 7.6e-4 measured
    # the dump's forward equals a plain forward (same session state afterwards)
    m2 = Model(tiny_gguf(), exact=exact, max_ctx=64)
    for i, t in enumerate(TINY_PROMPT):  # the dump's token loop
        l2 = m2.forward([t], i)
    last = [b for b in blocks if b["name"] == "result_output"][-1]
    assert abs(last["sum"] - float(np.float32(l2).sum(dtype=np.float32))) <= 1e-3 * max(1.0, abs(last["sum"]))
