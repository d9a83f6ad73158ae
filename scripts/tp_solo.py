"""Per-rank decode time of a row-sharded group, one rank alone on one GPU
(LLMI_TP_SOLO: the all-gathers are left out), for tp = 1, 2, 4, 8.

    python scripts/tp_solo.py [config ...] [--tp 1 2 4 8] [--steps N] [--no-graph]

The multi-GPU step time is this plus the RCCL all-gathers (4 per layer + the
argmax keys); the difference between this and bench.py --gpus N is the
exchange cost.  Diagnostics only.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["LLMI_TP_SOLO"] = "1"


def main():
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("configs", nargs="*", default=["gemma-3-4b"])
    p.add_argument("--tp", type=int, nargs="*", default=[1, 2, 4, 8])
    p.add_argument("--steps", type=int, default=256)
    p.add_argument("--no-graph", action="store_true", help="eager launches (for rocprofv3)")
    a = p.parse_args()
    from llm_inference_amd import _lib
    _lib.lib()
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    for name in a.configs:
        cfg = CONFIGS[name]
        g = build_gemma3_gguf(cfg, seed=1234)
        for tp in a.tp:
            m = Model(g, max_ctx=1024, tp_rank=0, tp_size=tp, use_graph=not a.no_graph)
            prompt = np.arange(2, 130, dtype=np.int32) % cfg.vocab
            m.forward(prompt, 0, want_logits=False)
            m.enqueue(m.last_argmax, len(prompt), 16)
            m.sync()
            n = a.steps
            t0 = time.perf_counter()
            m.enqueue(m.last_argmax, len(prompt) + 16, n)
            m.sync()
            ms = (time.perf_counter() - t0) * 1e3 / n
            info = m.get_info()
            print(json.dumps({"config": name, "tp": tp, "ms_per_step_rank_only": round(ms, 4),
                              "rank_bytes_per_token": info.bytes_per_token,
                              "kernels_per_token": info.kernels_per_token}), flush=True)
            m.close()


if __name__ == "__main__":
    main()
