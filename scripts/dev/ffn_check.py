import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from llm_inference_amd.model import Model
from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
from oracle.bind import Oracle
orc = Oracle()
for name in ("mini-4b", "mini-1b"):
    cfg = CONFIGS[name]
    g = build_gemma3_gguf(cfg, seed=21)
    ideal = orc.model(g, n_threads=8, max_ctx=64, attn_f64=True)
    os.environ["LLMI_FFN_ENGINE"] = "1"
    m = Model(g, max_ctx=64)
    os.environ.pop("LLMI_FFN_ENGINE")
    off = Model(g, max_ctx=64)
    print(name, "ffn_engine", m.get_info().ffn_engine, off.get_info().ffn_engine)
    prompt = np.random.default_rng(6).integers(4, cfg.vocab, 11).astype(np.int32)
    ideal.forward(prompt, 0); m.forward(prompt, 0); off.forward(prompt, 0)
    tok, pos = int(prompt[-1]), len(prompt)
    worst = worst_off = 0.0
    for _ in range(10):
        li = ideal.forward([tok], pos); lg = m.forward([tok], pos); lo = off.forward([tok], pos)
        worst = max(worst, float(np.abs(lg - li).max())); worst_off = max(worst_off, float(np.abs(lo - li).max()))
        assert int(np.argmax(lg)) == int(np.argmax(li)), "argmax"
        tok, pos = int(np.argmax(li)), pos + 1
    print(name, "ffn engine vs f64 oracle worst", worst, "three-launch", worst_off)
    assert worst <= 6e-2
    first = int(np.argmax(m.forward(prompt, 0)))
    a = m.generate(first, len(prompt), 12).tolist(); b = off.generate(first, len(prompt), 12).tolist()
    print(name, "greedy equal", a == b)
    assert a == b
print("FFN OK")
