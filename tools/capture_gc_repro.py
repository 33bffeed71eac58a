"""Reproduce (or rule out) the round-4 driver abort: the cyclic GC collecting a
dead engine <-> captured-graph cycle in the middle of another update's capture.

  python tools/capture_gc_repro.py guarded   # the product: mjrl_amd._capture.capture
  python tools/capture_gc_repro.py plain     # capture with torch.cuda.graph only (round 4)

Engine A (c2_swimmer shape) captures a graph, is put in a reference cycle and
dropped; with the collector disabled, so the dead cycle is still there when engine B
captures a TRPO update of the HalfCheetah shape (the driver's failing test).
"plain" runs one collection INSIDE the capture, as an allocation-triggered
collection would; it is expected to abort (SIGABRT) if the hypothesis holds.
"""
import contextlib
import gc
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import mjrl_amd.engine as E  # noqa: E402
from oracle import npg_cpu as O  # noqa: E402
import test_gpu_parity as P  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


@contextlib.contextmanager
def plain_capture(graph, **kw):
    with torch.cuda.graph(graph, **kw):
        gc.collect()          # what an allocation-triggered collection does mid-capture
        yield graph


def engine_with_graph(name, algo, extra):
    c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
    dev = torch.device("cuda:0")
    eng = E.UpdateEngine(int(c["n"]), int(c["m"]), c["hidden_t"], device=dev)
    batch = P.make_batch(c, dev)
    th = torch.from_numpy(c["theta0"].astype(np.float32)).to(dev)
    lam = None if np.isnan(c["gae_lambda"]) else float(c["gae_lambda"])
    args = dict(algo=algo, gamma=float(c["gamma"]), gae_lambda=lam, **extra)
    eng.graphs = True
    for _ in range(3):
        eng.update(batch, th, **args)
    assert eng._gstate.get("graph") is not None
    return eng, batch


def main(mode):
    if mode == "plain":
        E.capture = plain_capture
    gc.disable()
    for i in range(3):
        a, ba = engine_with_graph("c2_swimmer", "npg", dict(n_step_size=0.05))
        a._cycle = a          # a dead cycle holding a captured graph, pinned buffers, events
        a._host_res_keep = ba
        del a, ba
    c = O.load_case(os.path.join(GOLDEN, "c3_trpo_backtrack.npz"))
    kw = O.case_kwargs(c)
    b, _ = engine_with_graph("c3_trpo_backtrack", "trpo", dict(kl_dist=kw["kl_dist"], trpo_verbose=False))
    gc.enable()
    torch.cuda.synchronize()
    print("capture_gc_repro %s: OK (engine B captured and replayed)" % mode, flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "guarded")
