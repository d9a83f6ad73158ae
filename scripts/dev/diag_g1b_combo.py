"""Development diagnostic: which part of the exact decode loop departs from the reference's ids on g1b."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from test_full_models import _fixture  # noqa: E402

from llm_inference_amd.model import Model  # noqa: E402

os.environ["LLMI_EXACT_SCREEN"] = "1"
cfg, g, f = _fixture("g1b")
prompt, toks = f["prompt"], f["tokens"]
for env in ({}, {"LLMI_NO_EMBED_FOLD": "1"}, {"LLMI_EXACT_XL": "0"}, {"LLMI_SCREEN_PREP": "1"},
            {"LLMI_EXACT_SERIAL_NORMS": "1"}, {"LLMI_NO_GRAPH_DIAG": "1"}):
    for k in ("LLMI_NO_EMBED_FOLD", "LLMI_EXACT_XL", "LLMI_SCREEN_PREP", "LLMI_EXACT_SERIAL_NORMS"):
        os.environ.pop(k, None)
    os.environ.update({k: v for k, v in env.items() if k != "LLMI_NO_GRAPH_DIAG"})
    m = Model(g, exact=True, max_ctx=64, use_graph="LLMI_NO_GRAPH_DIAG" not in env)
    lg = m.forward(prompt, 0)
    got = [int(np.argmax(lg))] + m.generate(int(np.argmax(lg)), len(prompt), len(toks) - 1).tolist()
    d = next((i for i in range(len(got)) if got[i] != toks[i]), None)
    print(env, "engine", m.info.exact_engine, "screened", m.info.screened_logits, "first diff", d, got[:12])
    m.close()
