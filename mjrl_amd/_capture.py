"""hipGraph capture with Python's cyclic garbage collector held off.

torch.cuda.graph captures in the "global" error mode: while a stream captures,
a HIP call that is illegal during capture (an event query or synchronisation,
hipFree, a graph destruction, ...) from ANY code in the process invalidates the
capture, and where that code is a C++ destructor the error cannot propagate and
the process aborts.  Python's cyclic GC can run such destructors at any
allocation: a dead cycle holding an old engine's captured graph, its pinned
readback buffers (the host allocator queries their events on free) or its
timing events gets collected in the middle of the next capture.  That is what
aborted the round-4 driver suite (SIGABRT inside the TRPO capture, DESIGN.md
§5).  So every capture in this package goes through `capture`: synchronise,
collect the dead cycles first (their destructors run outside any capture), and
keep the collector off until the capture has ended.
"""
import contextlib
import gc

import torch


@contextlib.contextmanager
def capture(graph, **kwargs):
    """`with capture(g): ...` = `with torch.cuda.graph(g, **kwargs): ...` with
    the cyclic GC collected before and disabled during the capture."""
    torch.cuda.synchronize()
    gc.collect()
    enabled = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph, **kwargs):
            yield graph
    finally:
        if enabled:
            gc.enable()
