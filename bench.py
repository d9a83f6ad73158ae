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
    p.add_argument("--no-exact", action="store_true",
                   help="skip the exact-mode sub-measurement (the reference's operation order: bit-exact greedy ids)")
    p.add_argument("--full-logits", action="store_true",
                   help="decode loop: full F16 logits GEMV + argmax instead of int8 screening + exact rescoring")
    p.add_argument("--cpu-decode", type=int, default=32, help="decode tokens in the CPU baseline sample")
    p.add_argument("--kernel-reps", type=int, default=2)
    p.add_argument("--no-graph", action="store_true", help="eager launches (for kernel tracers)")
    p.add_argument("--exchange", choices=["push", "rccl"], default="push",
                   help="tp: the one-shot push all-gather over IPC-mapped mailboxes (k_exchange.hip) or RCCL")
    p.add_argument("--mode", choices=["tp", "replicas"], default="tp",
                   help="N>1: row-sharded tensor parallel (one stream) or independent replicas")
    p.add_argument("--quant", choices=["q4_0", "q4_k_m", "q8_0"], default="q4_0",
                   help="weight types: q4_0 (headline), q4_k_m (Q4_K + Q6_K v/down), q8_0 (BASELINE configs[3])")
    return p.parse_args()


def pmc_key(a) -> str:
    """The workload a PMC pass must have run to be quoted for this bench line:
    model, weight types, the position the roofline kernels are timed at
    (prefill + warmup + steps: the attention kernels' KV bytes depend on it)
    and the timing reps (the pass's tail dispatches).  A short pass that ends
    at the same position (e.g. --prefill 768 --warmup 2 --steps 14 for the
    default 512 + 16 + 256) measures the same launches."""
    return f"{a.config}/{a.quant}/pos{a.prefill + a.warmup + a.steps}/reps{a.kernel_reps}"


def pmc_traffic(kernel_substr: str, key: str, kv_bytes_per_key: float = 0.0):
    """HBM bytes per launch of the kernel whose name contains kernel_substr,
    from the newest committed rocprofv3 --pmc FETCH_SIZE pass (profiles/,
    x2 gfx950 correction: scripts/pmc_summary.py) OF THE SAME WORKLOAD (`key`,
    pmc_key), over that pass's last dispatches of the kernel -- the ones the
    bench's roofline timing (Model.time_kernel, after the decode loop) made, at
    the position it reports.  With no pass at this position, the pass of the
    same model / weights / reps nearest in position, its bytes moved by the KV
    history difference (kv_bytes_per_key per key attended: the attention
    block's only position-dependent stream; 0 for the GEMVs and the screening
    table), and the source says so.  (None, None) when no such pass is
    committed."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_fetch*.json")))

    def lookup(d):
        hits = [v for k, v in d.get("kernels", {}).items() if kernel_substr in k]
        if not hits:
            return None
        v = max(hits, key=lambda h: h["dispatches"])
        return v.get("hbm_bytes_tail_mean", v["hbm_bytes_mean"])

    passes = [(f, json.load(open(f))) for f in reversed(files)]
    for f, d in passes:
        if d.get("config") == key:
            t = lookup(d)
            if t is not None:
                return round(t), os.path.relpath(f, ROOT)
    m = re.fullmatch(r"(.*)/pos(\d+)/(reps\d+)", key)
    if m is None:
        return None, None
    best = None
    for f, d in passes:
        mm = re.fullmatch(r"(.*)/pos(\d+)/(reps\d+)", d.get("config") or "")
        if mm is None or (mm.group(1), mm.group(3)) != (m.group(1), m.group(3)):
            continue
        t = lookup(d)
        if t is not None and (best is None or abs(int(mm.group(2)) - int(m.group(2))) < abs(best[0] - int(m.group(2)))):
            best = (int(mm.group(2)), t, f)
    if best is None:
        return None, None
    p0, t, f = best
    delta = (int(m.group(2)) - p0) * kv_bytes_per_key
    return round(t + delta), (f"{os.path.relpath(f, ROOT)} (pass at pos{p0}; "
                              f"{'+' if delta >= 0 else '-'}{abs(delta):.0f} B of KV history to pos{m.group(2)})")


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

    def all_gather(self, obj) -> list:
        """Every rank's object, in rank order (the push exchange's mailbox handles)."""
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def _cpu_model_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    """Host threads this process may use: the CPU affinity, capped at the
    GPU box's per-GPU share (16: the box's nproc counts the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("LLMI_CPU_SHARE", "16"))))


FORCED = 8  # teacher-forced steps after the GPU line's prompt (parity check of exact and fast mode vs the reference)


def bench_prompt(cfg, n: int, offset: int = 0) -> np.ndarray:
    """The GPU line's seeded prompt (BOS then n - 1 ids; offset: a replica's own stream)."""
    rng = np.random.default_rng(99 + offset)
    return np.concatenate([[2], rng.integers(4, cfg.vocab, n - 1)]).astype(np.int32)


def parity_key(config: str, quant: str, prefill: int) -> str:
    """The workload a committed conditioning fixture (tests/golden/bench_conditioning.json) was computed on."""
    return f"{config}/{quant}/prefill{prefill}/forced{FORCED}"


def load_spread(key: str):
    """The reference's own f16-vs-f64-attention spread per parity position for this workload, or None."""
    p = os.path.join(ROOT, "tests", "golden", "bench_conditioning.json")
    try:
        return json.load(open(p)).get(key, {}).get("spread_per_position")
    except (OSError, ValueError):
        return None


def progress(msg: str) -> None:
    """A line on stderr per phase (a run that prints nothing for minutes looks hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def forced_tokens(vocab: int) -> np.ndarray:
    return np.random.default_rng(2024).integers(4, vocab, FORCED).astype(np.int32)


def forced_logits(m, prompt, vocab):
    """Logits after the prompt, then after each of FORCED teacher-forced tokens (positions len(prompt)..): the
    same inputs on the device session and on the reference, so the comparison does not depend on the greedy ids
    a random-init model settles into."""
    out = [m.forward(prompt, 0)]
    for i, t in enumerate(forced_tokens(vocab)):
        out.append(m.forward(np.array([t], np.int32), len(prompt) + i))
    return np.stack(out)


# The fast path's stated parity bound per position p (fp32 reassociation and fp32 split-K attention where the
# reference rounds an f16 accumulator at every key): |fast - reference|_p <= FAST_ABS + FAST_SPREAD x s_p, s_p =
# the reference's own distance from the same computation with f64 attention at p (its conditioning there: the
# oracle with attn_f64 on the same inputs, committed per workload by scripts/bench_conditioning.py -- two oracle
# runs over the 512-token prompt take minutes of CPU).  FAST_ABS is the full-depth 4B budget of tests/test_long_models.py.  And
# wherever the reference's top-2 margin exceeds twice the measured difference, the argmax must be the reference's.
FAST_ABS, FAST_SPREAD = 0.05, 3.0


def parity(ref, got, spread=None, exact=False) -> dict:
    """Device logits vs the reference's at the same FORCED + 1 positions; `ok` False when the mode's stated
    bound is exceeded (exact: every bit; fast: the bound above, where the spread s_p was measured)."""
    same_bits = [bool(np.array_equal(r.view(np.uint32), x.view(np.uint32))) for r, x in zip(ref, got)]
    diff = [float(np.abs(r - x).max()) for r, x in zip(ref, got)]
    srt = np.sort(ref, 1)
    margin = srt[:, -1] - srt[:, -2]
    agree = [int(np.argmax(r)) == int(np.argmax(x)) for r, x in zip(ref, got)]
    out = {"positions": len(ref), "logits_bit_identical": int(sum(same_bits)), "argmax_identical": int(sum(agree)),
           "max_abs_logit_diff": max(diff),
           "max_abs_logit_diff_per_position": [round(d, 4) for d in diff],
           "max_abs_reference_logit": float(np.abs(ref).max()),
           "reference_top2_margin_per_position": [round(float(m), 4) for m in margin]}
    if exact:
        out["bound"] = "bit-identical logits at every position"
        out["ok"] = all(same_bits)
    elif spread is not None:
        bound = [FAST_ABS + FAST_SPREAD * s for s in spread]
        decided = [m > 2.0 * d for m, d in zip(margin, diff)]
        out["reference_f64_attention_spread_per_position"] = [round(s, 4) for s in spread]
        out["bound_per_position"] = [round(b, 4) for b in bound]
        out["bound"] = (f"|fast - reference|_p <= {FAST_ABS} + {FAST_SPREAD} x s_p (s_p: the reference's own "
                        "f16-vs-f64-attention spread at p); argmax = the reference's wherever its top-2 margin "
                        "exceeds twice the difference")
        out["ok"] = all(d <= b for d, b in zip(diff, bound)) and all(a for a, k in zip(agree, decided) if k)
    return out


def cpu_baseline(g, cfg, n_decode: int, mean_ctx=None, ctx_prompt=None):
    """BASELINE.md section 4 on this host: the reference's own Model::forward
    (oracle/_ref, built from its sources) -- or, where the reference is not
    built, the oracle restatement ("port") -- timed on a bounded sample.

    * decode rate at `threads` (this process's CPU share) and at half of it
      (the reference's default is hw/2, main.cpp:12), 8-token prompt then
      n_decode greedy tokens, per-step wall clock;
    * the per-position attention cost from a linear fit of those per-step
      times (the reference's run_attn is single-threaded and O(pos)), and the
      rate extrapolated to the GPU run's mean context;
    * GEMV-only timings at the 4B shapes (mat_vec_mul / mat_vec_mul_fp16);
    * configs[0]: Gemma-3 1B Q4_0, --predict 64;
    * at the GPU line's own context (ctx_prompt: the GPU run's prompt, one untimed Model::forward of it, then
      FORCED timed steps on teacher-forced tokens): a measurement, not the extrapolation; their logits are the
      parity fixture of the GPU line."""
    from oracle import bind
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf, random_tensor
    from llm_inference_amd.gguf import TensorType as TT
    threads = cpu_share()

    def engine(n):
        try:
            return "reference", bind.Reference(n_threads=n)
        except Exception:
            return "port", bind.Oracle()

    def model(eng, kind, gg, n):
        return eng.model(gg) if kind == "reference" else eng.model(gg, n_threads=n, max_ctx=128)

    prompt = [2] + list(range(100, 107))
    out = {"cores": threads, "cpu_model": _cpu_model_name(), "compiler": "g++ -std=c++17 -O2 -DNDEBUG -mavx2 -mfma -mf16c (BUILD:41-53)"}
    runs = {}
    for n in (threads, max(1, threads // 2)):
        progress(f"cpu baseline: decode sample on {n} threads")
        kind, eng = engine(n)
        m = model(eng, kind, g, n)
        lg = m.forward(np.array(prompt, np.int32), 0)
        tok, pos, ids, per = int(np.argmax(lg)), len(prompt), [int(np.argmax(lg))], []
        for _ in range(n_decode):
            t0 = time.perf_counter()
            lg = m.forward(np.array([tok], np.int32), pos)
            per.append(time.perf_counter() - t0)
            tok, pos = int(np.argmax(lg)), pos + 1
            ids.append(tok)
        del m
        runs[n] = (kind, per, ids)
    kind, per, ids = runs[threads]
    per = np.array(per)
    x = np.arange(len(prompt), len(prompt) + len(per))
    slope, icpt = np.polyfit(x, per, 1)
    out.update({
        "value": round(len(per) / per.sum(), 3), "unit": "tokens/s", "kind": kind,
        "sample": f"{cfg.name} synthetic GGUF, {len(prompt)}-token prompt then {len(per)} greedy decode tokens "
                  f"(pos {len(prompt)}-{len(prompt) + len(per) - 1}) via Model::forward on {threads} threads; "
                  f"a SHORT-CONTEXT sample: the reference's single-threaded attention grows with the position, "
                  f"so its rate at the GPU line's mean context is lower (estimated_at_gpu_mean_context)",
        "half_threads": {"threads": max(1, threads // 2),
                         "value": round(len(runs[max(1, threads // 2)][1]) / sum(runs[max(1, threads // 2)][1]), 3)},
        "attention_s_per_position": float(max(slope, 0.0)),
        "step_s_at_pos0": float(icpt),
    })
    if mean_ctx:  # the linear fit extrapolated to the GPU run's mean context (an estimate, not a measurement)
        out["estimated_at_gpu_mean_context"] = {
            "position": int(mean_ctx), "value": round(1.0 / (icpt + max(slope, 0.0) * mean_ctx), 3),
            "unit": "tokens/s", "how": "step time = a + b * pos fitted to the measured per-step times"}
    # (bounded: the reference's T-token forward costs about T decode steps, so it runs when that is <= 40 s here)
    if ctx_prompt is not None and kind == "reference" and len(ctx_prompt) * float(np.median(per)) <= 40.0:
        progress(f"cpu baseline: the GPU line's {len(ctx_prompt)}-token prompt on the reference")
        kind_c, eng_c = engine(threads)
        mc = model(eng_c, kind_c, g, threads)
        t0 = time.perf_counter()
        lg = mc.forward(np.asarray(ctx_prompt, np.int32), 0)
        t_pf = time.perf_counter() - t0
        # FORCED timed steps on teacher-forced tokens (bench.forced_tokens): their logits are the parity fixture
        pos, per_c, ref_lg = len(ctx_prompt), [], [lg.copy()]
        for t in forced_tokens(cfg.vocab):
            t0 = time.perf_counter()
            lg = mc.forward(np.array([t], np.int32), pos)
            per_c.append(time.perf_counter() - t0)
            ref_lg.append(lg.copy())
            pos += 1
        del mc
        out["_ref_forced_logits"] = np.stack(ref_lg)  # (popped before printing)
        out["measured_at_gpu_context"] = {
            "positions": f"{len(ctx_prompt)}-{len(ctx_prompt) + FORCED - 1}", "value": round(FORCED / sum(per_c), 3),
            "unit": "tokens/s", "threads": threads, "prefill_s": round(t_pf, 2),
            "how": f"the GPU line's prompt through one untimed Model::forward, then {FORCED} timed steps on "
                   "teacher-forced tokens (their logits: the parity check of the GPU line)"}
    progress("cpu baseline: GEMV-only timings, configs[0]")
    # GEMV-only (the reference's mat_vec_mul, 4B shapes; BASELINE.md section 4 / SURVEY section 6)
    kind_t, eng = engine(threads)
    gemv = {}
    rng = np.random.default_rng(1)
    for name, tt, rows, cols in (("q4_0 2560->2048", TT.Q4_0, 2048, 2560), ("q4_0 2560->10240", TT.Q4_0, 10240, 2560),
                                 ("q4_0 10240->2560", TT.Q4_0, 2560, 10240), ("f16 2560->262208", TT.F16, 262208, 2560)):
        w = random_tensor(tt, rows, cols, seed=3)
        xv = rng.standard_normal(cols).astype(np.float32)
        reps = 5 if tt == TT.F16 else 50
        if kind_t == "reference":
            dt = eng.time_gemv(tt, w, rows, cols, xv, reps)
        else:
            eng.mat_vec_mul(tt, w, rows, cols, xv, threads)
            t0 = time.perf_counter()
            for _ in range(reps):
                eng.mat_vec_mul(tt, w, rows, cols, xv, threads)
            dt = (time.perf_counter() - t0) / reps
        gemv[name] = {"us": round(dt * 1e6, 1), "GBps": round(w.nbytes / dt / 1e9, 1)}
    out["gemv_only"] = gemv
    # configs[0]: gemma-3-1b Q4_0, --predict 64, on the CPU
    c1 = CONFIGS["gemma-3-1b"]
    g1 = build_gemma3_gguf(c1, seed=1234)
    kind1, eng1 = engine(threads)
    m1 = model(eng1, kind1, g1, threads)
    lg = m1.forward(np.array(prompt, np.int32), 0)
    tok, pos = int(np.argmax(lg)), len(prompt)
    t0 = time.perf_counter()
    for _ in range(63):  # 64 tokens emitted = 63 forwards after the prompt (main.cpp:169-234)
        lg = m1.forward(np.array([tok], np.int32), pos)
        tok, pos = int(np.argmax(lg)), pos + 1
    dt = time.perf_counter() - t0
    del m1
    out["configs0_gemma3_1b_predict64"] = {"value": round(63 / dt, 3), "unit": "tokens/s", "threads": threads,
                                           "kind": kind1}
    return out


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
    # LLMI_BENCH_ONE_DEVICE=1 (development): every rank on device 0 -- the tp path rehearsed on a one-GPU box
    dev = d.local if a.gpus > 1 and not os.environ.get("LLMI_BENCH_ONE_DEVICE") else 0

    def rccl_model():  # one RCCL communicator over the node's GPUs
        tid = d.broadcast(tp_unique_id() if d.rank == 0 else None)
        return Model(g, device=dev, exact=a.exact, max_ctx=max_ctx, use_graph=not a.no_graph, tp_rank=d.rank,
                     tp_size=d.world, tp_id=tid)

    exchange = a.exchange if tp else None
    if not tp:
        m = Model(g, device=dev, exact=a.exact, max_ctx=max_ctx, use_graph=not a.no_graph)
    elif exchange == "rccl":
        m = rccl_model()
    else:  # push: every rank's mailbox handle to every rank; if any rank cannot map them, all fall back to RCCL
        m = Model(g, device=dev, exact=a.exact, max_ctx=max_ctx, use_graph=not a.no_graph, tp_rank=d.rank,
                  tp_size=d.world, tp_peer=True)
        err = None
        try:
            handles = d.all_gather(m.peer_handle())
            m.peer_connect(handles)
        except Exception as e:  # noqa: BLE001 -- reported, then the RCCL exchange
            err = e
        if d.max(1.0 if err is not None else 0.0) > 0:
            print(f"[bench] rank {d.rank}: push exchange unavailable ({err!r}); RCCL instead", file=sys.stderr)
            m.close()
            exchange = "rccl"
            m = rccl_model()
    info = m.info
    prompt = bench_prompt(cfg, a.prefill, 0 if tp else d.rank)  # tensor-parallel ranks decode the same stream
    progress(f"session ready; prefill {a.prefill} tokens")
    t0 = time.time()
    m.forward(prompt, 0, want_logits=False)
    t_prefill = time.time() - t0
    first = m.last_argmax
    pos = a.prefill
    if a.warmup:
        m.enqueue(first, pos, a.warmup)
        toks = m.sync(a.warmup)
        first, pos = int(toks[-1]), pos + a.warmup
    progress(f"prefill {t_prefill:.3f} s; timed decode of {a.steps} steps")
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

    # Per-family kernel time of the timed graph: every family relaunched with
    # its decode-step arguments, one launch per layer in decode order, each
    # timed by events its own dispatch signals (Model.time_kernel); the
    # dominant family by time per token is the roofline kernel.  The attention
    # block reads the KV history at the position the decode loop ended on.
    L = info.n_layer
    fams = {}
    in_graph = {0: True, 3: True, 4: True, 2: bool(info.screened_logits)}
    for name, which, per_tok, kern in (("attention_block", 0, L, "attn_block_kernel"),
                                       ("gate_up", 3, L, "gemv_q4_0_layer"),
                                       ("down", 4, L, "gemv_q4_0_layer"),
                                       ("token_selection", 2, 1, "screen_gemv_kernel")):
        if not in_graph[which]:  # only the families the timed graph launches
            continue
        progress(f"kernel timing: {name}")
        us_f, by_f = m.time_kernel(which, a.kernel_reps if which != 2 else 8)
        if us_f <= 0:
            continue
        fams[name] = {"us_per_launch": round(us_f, 3), "launches_per_token": per_tok,
                      "us_per_token": round(us_f * per_tok, 1), "bytes_per_launch": int(by_f),
                      "GBps": round(by_f / (us_f * 1e-6) / 1e9, 1),
                      "frac": round(by_f / (us_f * 1e-6) / 1e9 / PEAK_HBM_GBS, 4), "kernel": kern}
    us_l, by_l = m.time_kernel(1, 2)
    # the prompt once more on the same session: the prefill warm (prefill_s above is the session's first call, which
    # also pays each prefill kernel's first launch)
    t0 = time.time()
    m.forward(prompt, 0, want_logits=False)
    t_prefill_warm = time.time() - t0
    dom_name = max(fams, key=lambda k: fams[k]["us_per_token"]) if fams else None
    dom = fams.get(dom_name, {})
    kpat = {"attention_block": "attn_block_kernel", "gate_up": "gemv_q4_0_layer<8, 10, 10",
            "down": "gemv_q4_0_layer<1, 10, 5", "token_selection": "screen_gemv_kernel"}.get(dom_name, "-")
    # the attention block's position-dependent stream: K and V rows of every kv head, per key attended
    kv_key = info.kv_bytes_per_pos / L if dom_name == "attention_block" else 0.0
    traffic, traffic_src = pmc_traffic(kpat, pmc_key(a), kv_key)
    # the timed steps decode positions pos .. pos + steps - 1; the step at
    # position p attends to p + 1 keys, so the mean KV history read is
    # pos + (steps + 1) / 2 keys per layer
    mean_ctx = pos + (a.steps + 1) / 2
    # time_kernel runs after the loop: the device position is then pos + steps
    # (the attention block attends to pos + steps + 1 keys there)
    pos_end = pos + a.steps
    tok_bytes = info.bytes_per_token + info.kv_bytes_per_pos * mean_ctx
    if info.screened_logits:  # the decode loop streams the int8 screening table instead of the F16 one
        tok_bytes += info.screen_bytes - info.vocab * info.n_embd * 2
    if a.exact and getattr(info, "exact_engine", 0):
        # exact mode: the exact-order engine's launches are not timed family by family -- the roofline is the
        # whole decode step (its 6 launches per layer + token selection), bytes = what the step streams
        us_step = ms * 1000.0
        dom_name = "exact_step"
        dom = {"us_per_launch": round(us_step, 3), "bytes_per_launch": int(tok_bytes),
               "GBps": round(tok_bytes / (us_step * 1e-6) / 1e9, 1),
               "frac": round(tok_bytes / (us_step * 1e-6) / 1e9 / PEAK_HBM_GBS, 4)}
        traffic, traffic_src = None, None
    # BASELINE.json / SURVEY 8(d) definition: every linear weight + the F16
    # logits table + KV read per token (4B: 3147.4 MB + 139.3 KB x L)
    base_bytes = info.bytes_per_token + info.kv_bytes_per_pos * mean_ctx
    per_gpu = 1 if tp else d.world
    qname = {"q4_0": "Q4_0", "q4_k_m": "Q4_K_M", "q8_0": "Q8_0"}[a.quant]
    base_cfg = {("gemma-3-4b", "q4_0"): "configs[2]", ("gemma-3-1b", "q4_0"): "configs[1]",
                ("gemma-3-4b", "q4_k_m"): "configs[3]", ("gemma-3-1b", "q8_0"): "configs[3]",
                ("gemma-3-27b", "q4_0"): "configs[4]"}.get((a.config, a.quant), "not a BASELINE config")
    dtypes = {"q4_0": "q4_0 x q8_0 int8 dot, fp32 accumulate", "q8_0": "q8_0 x q8_0 int8 dot, fp32 accumulate",
              "q4_k_m": "q4_k/q6_k x q8_k int8 dot, fp32 accumulate"}[a.quant]
    out = {
        "metric": ("decode tokens/sec + achieved HBM GB/s vs roofline, Gemma-3 4B Q4_0"  # BASELINE.json
                   if (a.config, a.quant) == ("gemma-3-4b", "q4_0") else
                   f"decode tokens/sec + achieved HBM GB/s vs roofline, Gemma-3 {cfg.name.split('-')[-1].upper()} {qname}"),
        "value": round(value, 3),
        "unit": "tokens/s",
        "n_gpus": d.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong" if tp else "weak",
        # BASELINE.md's only published figure is a 1B CPU number on unstated
        # hardware, not this metric: no ratio is claimed
        "vs_baseline": None,
        "dtype": dtypes + ("; exact (reference operation order)" if a.exact else "") + "; f16 logits table",
        "data": f"synthetic (random-init weights of the {cfg.name}-it {qname} architecture, seeded prompt ids)",
        "config": {
            "workload": f"{cfg.name}-{a.quant} greedy decode after a {a.prefill}-token prefill "
                        f"(BASELINE {base_cfg})",
            "prefill_tokens": a.prefill, "decode_tokens": a.steps, "mode": "exact" if a.exact else "fast",
            "parallelism": (f"tp{d.world} (row-sharded, " + (("one-shot push all-gather over IPC-mapped mailboxes"
                                                               + (", fused into the decode launches"
                                                                  if info.tp_exchange == 4 else ""))
                                                              if exchange == "push" else "RCCL all-gather") + ")"
                            if tp else f"replicas{d.world}")
                           if d.world > 1 else "single",
            "kernels_per_token": info.kernels_per_token,
            **({"exact_engine": bool(info.exact_engine)} if a.exact else {}),
        },
        "hbm": {
            "bytes_per_token": int(tok_bytes),
            "bytes_definition": "bytes the decode loop streams: weights + KV at the mean position + int8 screening table",
            "achieved_GBps": round(tok_bytes * value / per_gpu / 1e9, 1),
            "frac_of_peak": round(tok_bytes * value / per_gpu / 1e9 / PEAK_HBM_GBS, 4),
            "baseline_bytes_per_token": int(base_bytes),
            "baseline_definition": "BASELINE/SURVEY 8(d): weights + full F16 logits table + KV at the mean position",
            "baseline_achieved_GBps": round(base_bytes * value / per_gpu / 1e9, 1),
            "baseline_frac_of_peak": round(base_bytes * value / per_gpu / 1e9 / PEAK_HBM_GBS, 4),
        },
        "roofline": ({
            "kernel": (f"{dom_name}: the dominant kernel of the timed decode graph by time per token"
                       if dom_name != "exact_step" else
                       "exact_step: the whole exact-mode decode step (6 exact-order launches per layer + token "
                       "selection), per token"),
            "bound": "hbm", "achieved": dom["GBps"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": dom["frac"], "traffic": traffic, "traffic_unit": "HBM bytes per launch (FETCH_SIZE x2)",
            "traffic_source": traffic_src,
            "us_per_launch": dom["us_per_launch"], "bytes_per_launch": dom["bytes_per_launch"],
            "position": pos_end, "keys_attended": pos_end + 1, "pmc_key": pmc_key(a),
        } if dom else None),
        "kernel_families": fams,
        "logits_gemv": {"us": round(us_l, 2), "GBps": round(by_l / (us_l * 1e-6) / 1e9, 1)},
        "token_selection_mode": ("int8 screening + exact f16 rescoring of the candidates (ids = full F16 GEMV argmax)"
                                 if info.screened_logits else "full F16 logits GEMV + argmax"),
        "timing_detail": {"synthetic_build_s": round(t_build, 1), "prefill_s": round(t_prefill, 4),
                          "prefill_tokens_per_s": round(a.prefill / t_prefill, 1),
                          "prefill_warm_s": round(t_prefill_warm, 4),
                          "prefill_mode": ({7: "batched f16-MFMA (GEMM v7 gate_up, v6 qkv / o / down; f16 rows of the "
                                                "dequantized Q8_0 activations)", 6: "batched f16-MFMA (v6, K-quants)",
                                            5: "batched int8-MFMA (GEMM v5, Q8_0 activation blocks)"}
                                           .get(getattr(info, "prefill_gemm", 5), "batched")
                                           if info.batched_prefill else "token loop"),
                          # attention-block hand-off waits (per wave) over 20 us since the session was created
                          # (prefill tail, warmup, timed steps, kernel timing): the spin-wait outlier check
                          "block_slow_waits": m.get_info().block_slow_waits},
    }
    # Exact mode in the same invocation (north_star: "bit-exact token ids for greedy decode"): a second session on
    # the exact-order engine (the reference's operation order), the same prompt, then the
    # same timed decode; its logits on the parity fixture's inputs are checked against the reference's own
    # (cpu_baseline, below).  Single GPU only.
    gpu_forced = {}
    if d.world == 1 and not a.no_cpu_baseline:  # this session's logits on the parity fixture's inputs
        gpu_forced["exact" if a.exact else "fast"] = forced_logits(m, prompt, cfg.vocab)
    if d.world == 1 and not a.exact and not a.no_exact:
        progress("exact-mode session")
        mx = Model(g, device=dev, exact=True, max_ctx=max_ctx, use_graph=not a.no_graph)
        t0 = time.time()
        mx.forward(prompt, 0, want_logits=False)
        t_pf_x = time.time() - t0
        t0 = time.time()
        mx.forward(prompt, 0, want_logits=False)
        t_pf_xw = time.time() - t0
        n_chk = max(a.warmup, 8)  # warmup steps (positions prefill .. prefill + n_chk - 1)
        mx.enqueue(mx.last_argmax, a.prefill, n_chk)
        wt = mx.sync(n_chk)
        mx.sync()
        t0 = time.perf_counter()
        mx.enqueue(int(wt[-1]), a.prefill + n_chk, a.steps)
        mx.sync(a.steps)
        el_x = time.perf_counter() - t0
        xinfo = mx.get_info()
        gpu_forced["exact"] = forced_logits(mx, prompt, cfg.vocab) if not a.no_cpu_baseline else None
        mx.close()
        out["exact"] = {
            "value": round(a.steps / el_x, 3), "unit": "tokens/s", "steps": a.steps,
            "ms_per_step": round(el_x * 1000.0 / a.steps, 4),
            "positions": f"{a.prefill + n_chk}-{a.prefill + n_chk + a.steps - 1}",
            "exact_engine": bool(getattr(xinfo, "exact_engine", 0)), "kernels_per_token": xinfo.kernels_per_token,
            "batched_prefill": bool(getattr(xinfo, "exact_batched_prefill", 0)),
            "prefill_s": round(t_pf_x, 3), "prefill_warm_s": round(t_pf_xw, 3),
            "how": "a second session with LLMI_EXACT (bit-identical to the reference's logits: "
                   "parity_vs_reference.exact), the same prompt, then the same timed decode"}
    parity_ok = True
    if d.rank == 0 and d.world == 1 and not a.no_cpu_baseline:
        m.close()
        try:
            progress("cpu baseline (the reference on the host cores)")
            out["cpu_baseline"] = cpu_baseline(g, cfg, a.cpu_decode, mean_ctx, ctx_prompt=prompt)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
        ref_lg = out["cpu_baseline"].pop("_ref_forced_logits", None)
        key = parity_key(a.config, a.quant, a.prefill)
        spread = load_spread(key)
        if ref_lg is not None:  # device logits vs the reference's own on the same prompt + teacher-forced tokens
            out["parity_vs_reference"] = {
                k: parity(ref_lg, v, spread, exact=(k == "exact")) for k, v in gpu_forced.items() if v is not None}
            out["parity_vs_reference"]["how"] = (
                f"the reference (oracle/_ref: its own ops.cpp / model.cpp) and the device sessions on the GPU line's "
                f"prompt, then {FORCED} teacher-forced tokens, logits compared at each of the {FORCED + 1} positions "
                f"(exact: the reference's operation order, every bit; fast: fp32 reassociation, within `bound`); "
                f"the fast session ran the whole timed decode loop and the kernel timing before, so a result that "
                f"depends on what ran before shows here")
            out["parity_vs_reference"]["conditioning"] = (
                f"tests/golden/bench_conditioning.json[{key}]" if spread is not None else
                f"no committed conditioning for {key}: the fast path is reported, not gated")
            parity_ok = all(v.get("ok", True) for k, v in out["parity_vs_reference"].items() if isinstance(v, dict))
            out["parity_vs_reference"]["ok"] = parity_ok
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    if not parity_ok:  # the line is printed (the record), but a result outside its stated bound fails the run
        print("[bench] parity_vs_reference outside its stated bound", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
