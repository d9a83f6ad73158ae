"""Development diagnostic: from the teacher-forced state at position 16 + 9 - k, k decode-loop steps -- does the
k-th step still produce the reference's token 9?"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
os.environ["LLMI_EXACT_SCREEN"] = "1"
from test_full_models import _fixture  # noqa: E402

from llm_inference_amd.model import Model  # noqa: E402

cfg, g, f = _fixture("g1b")
prompt, toks = f["prompt"], f["tokens"]
P = len(prompt)
for k in (6,):
    m = Model(g, exact=True, max_ctx=64, use_graph=False)
    m.forward(prompt, 0)
    for i in range(9 - k):
        m.forward([int(toks[i])], P + i)
    out = m.generate(int(toks[9 - k]), P + 9 - k, k)
    print(os.environ.get("VARIANT"), m.info.exact_engine, m.info.screened_logits, k, "steps: ids", out.tolist(), "ref", toks[10 - k:10].tolist(), "ok", out.tolist() == toks[10 - k:10].tolist())
    m.close()
