"""Development diagnostic: exact-mode decode loop (screened token selection) vs the reference's ids on the g1b
full-size fixture; at the first differing step, the step's x16 (llmi_session_trace, decode-loop step) through the
oracle's exact F16 GEMV: the true top-2 and whether the screened token is one of them."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from test_full_models import _fixture  # noqa: E402

from llm_inference_amd.gguf import GGUFFile, TensorType  # noqa: E402
from llm_inference_amd.model import Model  # noqa: E402
from oracle.bind import Oracle  # noqa: E402

os.environ["LLMI_EXACT_SCREEN"] = "1"
cfg, g, f = _fixture("g1b")
prompt, toks = f["prompt"], f["tokens"]
m = Model(g, exact=True, max_ctx=64)
lg = m.forward(prompt, 0)
got = [int(np.argmax(lg))] + m.generate(int(np.argmax(lg)), len(prompt), len(toks) - 1).tolist()
d = next((i for i in range(len(got)) if got[i] != toks[i]), None)
print("screened ids == ref:", d is None, "first diff", d)
if d is not None:
    m2 = Model(g, exact=True, max_ctx=64)
    m2.forward(prompt, 0)
    for i in range(d - 1):
        m2.forward([int(toks[i])], len(prompt) + i)
    tr = m2.trace([int(toks[d - 1])], len(prompt) + d - 1, gen=True)
    names = sorted(set(n for (n, l, b) in tr))
    print("taps", names)
    x16 = [b for (n, l, b) in tr if n == "x16"][-1]
    tok = [b for (n, l, b) in tr if n == "token"][-1]
    x = np.frombuffer(x16, np.float16).astype(np.float32)
    gf = GGUFFile(g)
    t = gf.tensor("token_embd.weight")
    s = gf.data_section_start + t.tensor_offset
    w = g[s:s + t.nbytes]
    o = Oracle()
    L = o.mat_vec_mul(TensorType.F16, w, cfg.vocab, cfg.n_embd, x)
    top = np.argsort(-L)[:4]
    print("traced token", np.frombuffer(tok, np.int32)[0], "ref", toks[d], "got", got[d])
    print("oracle exact top4", top.tolist(), [float(L[i]) for i in top], "margin", float(L[top[0]] - L[top[1]]))
    print("values of ref/got rows", float(L[toks[d]]), float(L[got[d]]))
