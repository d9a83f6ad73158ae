"""Decode benchmark: Gemma-3 4B Q4_0 greedy decode tokens/s on MI355X.

BASELINE.json metric: "decode tokens/sec + achieved HBM GB/s vs roofline,
Gemma-3 4B Q4_0" on configs[2] (4B, 512-token prefill + 256 decode).
A step = one greedy decode token (main.cpp:172-224) of the full model:
embedding, 34 layers (norms, Q4_0 GEMVs, rope, attention over the whole
history, GELU), final norm, F16 logits GEMV, argmax -- all device-resident,
one hipGraph replay per token, the token fed back on the device.

Weights: random-init with the exact gemma-3-4b-it-q4_0 architecture (no
checkpoints offline); prompt: seeded synthetic token ids.

Single process per GPU.  With --gpus N (torchrun) the default is the north
star's row-sharded decode: ONE greedy stream, each rank holding 1/N of every
projection's output rows, slices all-gathered over RCCL after each projection
(include/llmi.h tp_*; "scaling": "strong", value = that stream's tok/s).
--mode replicas instead decodes N independent streams (value = total tok/s,
"scaling": "weak").  Barrier + max-over-ranks timing either way.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=256)
    p.add_argument("--warmup", type=int, default=16)
    p.add_argument("--prefill", type=int, default=512)
    p.add_argument("--config", default="gemma-3-4b")
    p.add_argument("--exact", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--full-logits", action="store_true",
                   help="decode loop: full F16 logits GEMV + argmax instead of int8 screening + exact rescoring")
    p.add_argument("--cpu-decode", type=int, default=24, help="decode tokens in the CPU baseline sample")
    p.add_argument("--kernel-reps", type=int, default=2)
    p.add_argument("--no-graph", action="store_true", help="eager launches (for kernel tracers)")
    p.add_argument("--mode", choices=["tp", "replicas"], default="tp",
                   help="N>1: row-sharded tensor parallel (one stream) or independent replicas")
    p.add_argument("--quant", choices=["q4_0", "q4_k_m", "q8_0"], default="q4_0",
                   help="weight types: q4_0 (headline), q4_k_m (Q4_K + Q6_K v/down), q8_0 (BASELINE configs[3])")
    return p.parse_args()


def pmc_traffic():
    """HBM bytes per launch of the Q4_0 projection family from the committed
    rocprofv3 --pmc FETCH_SIZE pass (profiles/, x2 gfx950 correction; see
    scripts/pmc_summary.py); None when no such profile is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*pmc_fetch*.json")))
    if not files:
        return None, None
    fam = json.load(open(files[-1])).get("q4_0_layer_family", {})
    b = fam.get("hbm_bytes_per_launch")
    return (round(b), os.path.relpath(files[-1], os.path.dirname(os.path.abspath(__file__)))) if b else (None, None)


class Dist:
    def __init__(self, n):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist  # gloo only: the GPU is driven by libllmi, not torch
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def broadcast(self, obj):
        """rank 0's object on every rank (the RCCL unique id)."""
        if self.world == 1:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def cpu_baseline(g, cfg, n_decode: int):
    """The reference's own Model::forward (oracle/_ref, built from its sources)
    on this host's cores; falls back to the oracle restatement ("port")."""
    from oracle import bind
    threads = min(os.cpu_count() or 1, 16)
    kind = "reference"
    try:
        eng = bind.Reference(n_threads=threads)
        m = eng.model(g)
    except Exception:
        kind = "port"
        eng = bind.Oracle()
        m = eng.model(g, n_threads=threads, max_ctx=64)
    prompt = [2] + list(range(100, 107))
    lg = m.forward(np.array(prompt, np.int32), 0)
    tok, pos = int(np.argmax(lg)), len(prompt)
    t0 = time.perf_counter()
    for _ in range(n_decode):
        lg = m.forward(np.array([tok], np.int32), pos)
        tok, pos = int(np.argmax(lg)), pos + 1
    dt = time.perf_counter() - t0
    del m
    return {"value": n_decode / dt, "unit": "tokens/s", "cores": threads, "kind": kind,
            "sample": f"{cfg.name} Q4_0 synthetic GGUF, {len(prompt)}-token prompt then {n_decode} greedy decode "
                      f"tokens via Model::forward (short context: CPU attention cost at pos 512+ not included)"}


def main():
    a = parse()
    if a.full_logits:
        os.environ["LLMI_FULL_LOGITS"] = "1"
    d = Dist(a.gpus)
    # load the HIP library before anything could pull in torch's HIP runtime
    from llm_inference_amd import _lib
    _lib.lib()
    from llm_inference_amd.model import Model, tp_unique_id
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    tp = d.world > 1 and a.mode == "tp"

    cfg = CONFIGS[a.config]
    t0 = time.time()
    from llm_inference_amd.gguf import TensorType as TT
    qkw = {"q4_0": {}, "q4_k_m": dict(wtype=TT.Q4_K, wtypes={"v": TT.Q6_K, "down": TT.Q6_K}),
           "q8_0": dict(wtype=TT.Q8_0)}[a.quant]
    g = build_gemma3_gguf(cfg, seed=1234, **qkw)
    t_build = time.time() - t0
    max_ctx = a.prefill + a.warmup + a.steps + 8
    tp_kw = {}
    if tp:  # one RCCL communicator over the node's GPUs
        tp_kw = dict(tp_rank=d.rank, tp_size=d.world, tp_id=d.broadcast(tp_unique_id() if d.rank == 0 else None))
    m = Model(g, device=d.local if a.gpus > 1 else 0, exact=a.exact, max_ctx=max_ctx, use_graph=not a.no_graph,
              **tp_kw)
    info = m.info
    rng = np.random.default_rng(99 + (0 if tp else d.rank))  # tensor-parallel ranks decode the same stream
    prompt = np.concatenate([[2], rng.integers(4, cfg.vocab, a.prefill - 1)]).astype(np.int32)
    t0 = time.time()
    m.forward(prompt, 0, want_logits=False)
    t_prefill = time.time() - t0
    first = m.last_argmax
    pos = a.prefill
    if a.warmup:
        m.enqueue(first, pos, a.warmup)
        toks = m.sync(a.warmup)
        first, pos = int(toks[-1]), pos + a.warmup
    d.barrier()
    m.sync()
    t0 = time.perf_counter()
    m.enqueue(first, pos, a.steps)
    toks = m.sync(a.steps)
    el = time.perf_counter() - t0
    d.barrier()
    el = d.max(el)
    info = m.get_info()  # kernels_per_token is known once the step graph exists
    value = a.steps * (1 if tp else d.world) / el
    ms = el * 1000.0 / a.steps

    # dominant kernel: the Q4_0 GEMV family (weights swept in decode order, HIP events)
    us, by = m.time_kernel(0, a.kernel_reps)
    us_l, by_l = m.time_kernel(1, 2)
    us_s, by_s = m.time_kernel(2, 8) if info.screened_logits else (0.0, 0.0)
    traffic, traffic_src = pmc_traffic()
    ach = by / (us * 1e-6) / 1e9
    mean_ctx = pos + a.steps / 2
    tok_bytes = info.bytes_per_token + info.kv_bytes_per_pos * mean_ctx
    if info.screened_logits:  # the decode loop streams the int8 screening table instead of the F16 one
        tok_bytes += info.screen_bytes - info.vocab * info.n_embd * 2
    out = {
        "metric": ("decode tokens/sec (Gemma-3 4B Q4_0 shape, greedy)" if (a.config, a.quant) == ("gemma-3-4b", "q4_0")
                   else f"decode tokens/sec ({cfg.name} {a.quant} shape, greedy)"),
        "value": round(value, 3),
        "unit": "tokens/s",
        "n_gpus": d.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong" if tp else "weak",
        "vs_baseline": None,
        "dtype": "q4_0 x q8_0 int8-dot, fp32 accumulate; f16 logits",
        "data": "synthetic (random-init weights of the gemma-3-4b-it-q4_0 architecture, seeded prompt ids)",
        "config": {
            "workload": f"{cfg.name}-{a.quant} greedy decode after a {a.prefill}-token prefill (BASELINE configs[2])",
            "prefill_tokens": a.prefill, "decode_tokens": a.steps, "mode": "exact" if a.exact else "fast",
            "parallelism": (f"tp{d.world} (row-sharded, RCCL all-gather)" if tp else f"replicas{d.world}")
                           if d.world > 1 else "single",
            "kernels_per_token": info.kernels_per_token,
        },
        "hbm": {
            "bytes_per_token": int(tok_bytes),
            # per GPU: this rank's bytes of one token x tokens/s of its stream
            "achieved_GBps": round(tok_bytes * value / (1 if tp else d.world) / 1e9, 1),
            "frac_of_peak": round(tok_bytes * value / (1 if tp else d.world) / 1e9 / PEAK_HBM_GBS, 4),
        },
        "roofline": {
            "kernel": "Q4_0 projection GEMVs of one token in decode order (gemv_q4_0_layer on the fast path: qkv, o, gate_up+GELU, down)",
            "bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": traffic, "traffic_unit": "bytes per launch",
            "traffic_source": traffic_src,
            "us_per_launch": round(us, 3), "bytes_per_launch": int(by),
        },
        "logits_gemv": {"us": round(us_l, 2), "GBps": round(by_l / (us_l * 1e-6) / 1e9, 1)},
        "token_selection": ({"mode": "int8 screening + exact f16 rescoring of the candidates (ids = full F16 GEMV argmax)",
                             "us": round(us_s, 2), "bytes": int(by_s),
                             "GBps": round(by_s / (us_s * 1e-6) / 1e9, 1) if us_s else None}
                            if info.screened_logits else {"mode": "full F16 logits GEMV + argmax"}),
        "timing_detail": {"synthetic_build_s": round(t_build, 1), "prefill_s": round(t_prefill, 4),
                          "prefill_tokens_per_s": round(a.prefill / t_prefill, 1),
                          "prefill_mode": "batched int8-MFMA" if info.batched_prefill else "token loop"},
    }
    if d.rank == 0 and d.world == 1 and not a.no_cpu_baseline:
        m.close()
        try:
            out["cpu_baseline"] = cpu_baseline(g, cfg, a.cpu_decode)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
    if d.rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
