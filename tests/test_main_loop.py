"""The reference's own greedy decode loop (main.cpp:160-224) with the forward
served by the device session (integration/main_mi355x.cpp, built by
`make -C oracle mainloop` from the reference's unchanged GGUFFile / Model /
ops sources): tokenization, chat template, EOS / end-of-turn stop and
std::max_element argmax are the reference's; every forward is
llmi_session_forward (host loop, as main.cpp) or llmi_session_generate
(--device-loop: the argmax fed back on the device).  The printed ids must be
the reference's own (Model::forward on the CPU, oracle/_ref) for the same
prompt: exact mode bit-identical logits -> identical ids; fast mode on the
same file with the reference's margins large enough is checked the same way."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "main_mi355x")
PIECES = ["<start_of_turn>", "<end_of_turn>", "user", "model", "\n", "▁One", "▁sentence", "▁fact",
          "▁about", "▁silicon"]


def run(path, *args):
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/main_mi355x not built (needs /root/reference at build time)")
    out = subprocess.run([BIN, "-m", path] + list(args), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    ids = [ln for ln in out.stdout.splitlines() if ln.startswith("ids:")][0].split()[1:]
    assert "tok/s)" in out.stdout  # main.cpp's summary line
    return [int(t) for t in ids]


def reference_ids(g, prompt, chat, n):
    """main.cpp's loop on the reference itself: tokenize, forward, greedy, EOS stop."""
    from oracle.bind import Reference
    m = Reference(n_threads=4).model(g)
    toks = m.tokenize(prompt, chat)
    lg = m.forward(np.array(toks, np.int32), 0)
    pos, ids = len(toks), []
    for i in range(n):
        t = int(np.argmax(lg))
        if t in (1, 5):  # eos (tokenizer.ggml.eos_token_id) / <end_of_turn> (PIECES[1] at id 5)
            break
        ids.append(t)
        if i < n - 1:
            lg = m.forward(np.array([t], np.int32), pos)
            pos += 1
    return ids


@pytest.fixture(scope="module")
def tiny_file(tmp_path_factory):
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    g = build_gemma3_gguf(CONFIGS["tiny"], seed=17, swa_pattern=[True, False, True], centered=True, pieces=PIECES)
    p = tmp_path_factory.mktemp("m") / "tiny.gguf"
    p.write_bytes(bytes(g))
    return g, str(p)


@pytest.mark.parametrize("chat", [True, False], ids=["chat", "no-cnv"])
@pytest.mark.parametrize("loop", ["host", "device"])
def test_main_loop_exact_matches_reference(tiny_file, chat, loop):
    g, path = tiny_file
    prompt = "One sentence fact about silicon"
    ref = reference_ids(g, prompt, chat, 12)
    args = ["-p", prompt, "-n", "12", "--exact"] + ([] if chat else ["--no-cnv"]) + (["--device-loop"] if loop == "device" else [])
    assert run(path, *args) == ref


def test_main_loop_fast_and_goldens(golden_models, tmp_path):
    """Fast kernels through the same loop: the tiny fixture's reference ids
    (tests/golden/model_ref.npz) from its explicit prompt ids, both loop shapes."""
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    g = build_gemma3_gguf(CONFIGS["tiny"], seed=7, swa_pattern=[True, False, True])
    p = tmp_path / "t.gguf"
    p.write_bytes(bytes(g))
    toks = " ".join(str(int(t)) for t in golden_models["tiny__prompt"])
    ref = golden_models["tiny__tokens"].tolist()
    assert run(str(p), "--tokens", toks, "-n", str(len(ref))) == ref
    assert run(str(p), "--tokens", toks, "-n", str(len(ref)), "--device-loop") == ref
