"""One rank of tests/test_tp_peer.py: a LLMI_TP_PEER session in its own
process, its mailbox handle sent to the parent, every rank's handles back,
then a prompt and a greedy run; results (or the error text) to the parent."""
import os
import traceback

import numpy as np


def run(rank, size, gguf, prompt, n_gen, env, to_parent, from_parent):
    try:
        os.environ.update(env)
        from llm_inference_amd.model import Model
        m = Model(np.frombuffer(gguf, np.uint8), exact=False, max_ctx=128, tp_rank=rank, tp_size=size, tp_peer=True)
        to_parent.put((rank, "handle", m.peer_handle()))
        m.peer_connect(from_parent.get(timeout=120))
        lg = m.forward(prompt, 0)
        toks = m.generate(int(np.argmax(lg)), len(prompt), n_gen)
        info = m.get_info()
        to_parent.put((rank, "result", (lg, toks, info.tp_exchange, info.kernels_per_token)))
        m.close()
    except Exception:  # noqa: BLE001 -- reported to the parent
        to_parent.put((rank, "error", traceback.format_exc()))
