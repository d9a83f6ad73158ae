"""The one-shot push exchange between PROCESSES (include/llmi.h
LLMI_TP_PEER): each rank is its own process with its own session and its own
hardware queues, its mailbox shared through hipIpcGetMemHandle / OpenMemHandle
(handles swapped through the parent, as bench.py swaps them through
torch.distributed), one combined push + gather kernel per all-gather captured
in the token's hipGraph -- the production multi-GPU exchange.  Here both ranks
share the box's single GPU (the kernel does not care whether a peer's mailbox
is local or across xGMI).  Bar: logits and greedy ids bit-identical to the
whole model (row sharding is exact)."""
import multiprocessing as mp

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _int8_prefill(monkeypatch):
    """Tensor-parallel ranks run the batched prefill on the int8 GEMM (tests/test_tp.py), so the whole-model
    sessions compared against them do too (the spawned rank processes inherit the environment)."""
    monkeypatch.setenv("LLMI_PREFILL_F16", "0")


def _peer_ranks(g, size, prompt, n_gen, env):
    from _peer_worker import run
    ctx = mp.get_context("spawn")
    to_parent = ctx.Queue()
    inboxes = [ctx.Queue() for _ in range(size)]
    procs = [ctx.Process(target=run, args=(r, size, bytes(g), prompt, n_gen, env, to_parent, inboxes[r]))
             for r in range(size)]
    for p in procs:
        p.start()
    handles, results, errors = [None] * size, [None] * size, []
    try:
        while sum(h is not None for h in handles) + len(errors) < size:
            r, kind, val = to_parent.get(timeout=240)
            if kind == "handle":
                handles[r] = val
            else:
                errors.append((r, val))
        if not errors:
            for q in inboxes:
                q.put(handles)
        while sum(x is not None for x in results) + len(errors) < size:
            r, kind, val = to_parent.get(timeout=240)
            if kind == "result":
                results[r] = val
            else:
                errors.append((r, val))
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert not errors, errors
    return results


@pytest.mark.parametrize("cfg_name,prefill,mode", [("mini-4b", True, "fused"), ("mini-1b", False, "fused"),
                                                   ("mini-1b", False, "standalone"), ("mini-4b", False, "block")])
def test_peer_push_processes_match_whole_model(cfg_name, prefill, mode, monkeypatch):
    """mode fused (default): the o / GELU / down outputs pushed from the producing launches, read by the consumers
    from their mailboxes (csrc/px.h); standalone (LLMI_TP_FUSED=0): an exchange launch per all-gather; block: the
    fused exchanges around the ranks' attention blocks (replicated attention), against the whole model's block."""
    from llm_inference_amd.model import Model
    from llm_inference_amd.synthetic import CONFIGS, build_gemma3_gguf
    cfg = CONFIGS[cfg_name]
    g = build_gemma3_gguf(cfg, seed=31)
    prompt = np.random.default_rng(37).integers(4, cfg.vocab, 40).astype(np.int32)
    env = {} if mode == "block" else {"LLMI_NO_BLOCK": "1"}  # else the per-projection launches on both sides
    if not prefill:
        env["LLMI_NO_PREFILL"] = "1"  # the prompt token by token through the decode graph's exchanges
    if mode == "standalone":
        env["LLMI_TP_FUSED"] = "0"
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    whole = Model(g, exact=False, max_ctx=128)
    ref = whole.forward(prompt, 0)
    ref_toks = whole.generate(int(np.argmax(ref)), len(prompt), 10)
    whole.close()
    out = _peer_ranks(g, 2, prompt, 10, env)
    for r, (lg, toks, exchange, kpt) in enumerate(out):
        print(f"{cfg_name} peer rank {r} ({mode}): kernels/token {kpt}, max|dlogit| {float(np.abs(lg - ref).max()):.3g}")
        assert exchange == (3 if mode == "standalone" else 4)
        np.testing.assert_array_equal(lg, ref)
        assert toks.tolist() == ref_toks.tolist()
