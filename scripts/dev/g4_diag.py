"""Gemma-4 fast-path error breakdown (development): oracle vs its f64-attention
variant vs the device session with families of kernels switched to exact."""
import os, sys, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import numpy as np
import gen_gemma4 as gen

case = int(sys.argv[1]) if len(sys.argv) > 1 else 2
if len(sys.argv) > 2:  # child: one session run
    from llm_inference_amd.model import Model
    c = gen.CASES[case]
    g = gen.build(c)
    prompt = gen.prompt_of(c)
    m = Model(g, max_ctx=64)
    np.save(sys.argv[2], m.forward(prompt, 0))
    sys.exit(0)
from oracle.bind import Oracle
orc = Oracle()
c = gen.CASES[case]
g = gen.build(c)
prompt = gen.prompt_of(c)
ref = orc.model(g, n_threads=8, max_ctx=64).forward(prompt, 0)
f64 = orc.model(g, n_threads=8, max_ctx=64, attn_f64=True).forward(prompt, 0)
print("max|L| %.3f  |ref - f64attn| %.4g" % (np.abs(ref).max(), np.abs(ref - f64).max()))
for parts in ["", "attn", "gemv", "norm", "logits", "gemv,norm", "attn,gemv,norm,logits"]:
    env = dict(os.environ)
    if parts:
        env["LLMI_EXACT_PARTS"] = parts
    out = "/tmp/g4_%s.npy" % (parts.replace(",", "_") or "fast")
    subprocess.run([sys.executable, __file__, str(case), out], env=env, check=True)
    lg = np.load(out)
    print("%-24s |dev - ref| %.4g  |dev - f64attn| %.4g" % (parts or "fast", np.abs(lg - ref).max(), np.abs(lg - f64).max()))
