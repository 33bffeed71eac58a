"""Host -> HBM staging through a small pinned RING (slots reused as soon as their
H2D copy completed) instead of a batch-sized pinned slab, on the GPU box.  The
question: with ordinary (cached) stores into a ring that fits the L3, do the
conversion's writes and the DMA's reads stay out of DRAM, so that the host
memory traffic is the f64 read alone?  1000 Humanoid paths (3 GB f64 -> 1.5 GB
f32), 16 threads; the batch-slab engine stage timed beside it.
    python tools/ring_probe.py"""
import concurrent.futures as cf
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mjrl_amd import _lib, engine  # noqa: E402

n, P, L = 376, 1000, 1000
nth = engine._host_threads()
rs = np.random.RandomState(0)
paths = [rs.randn(L, n) for _ in range(P)]
SL = _lib.stage_lib()
dev = torch.device("cuda:0")
PB = L * n * 4
d = torch.empty(P * PB, dtype=torch.uint8, device=dev)
ex = cf.ThreadPoolExecutor(nth)
list(ex.map(lambda i: time.sleep(0.01), range(nth)))
cs = torch.cuda.Stream(dev)
print("threads", nth, "avx512", SL.mjrl_host_stage_avx512(), flush=True)


def ring(fn, R, per):
    sb = per * PB
    h = torch.empty(R * sb, dtype=torch.uint8, pin_memory=True)
    hv = h.numpy()
    items = P // per
    done = [threading.Event() for _ in range(items)]
    issued = [threading.Event() for _ in range(items)]
    evs = [None] * items

    def work(k):
        if k >= R:
            issued[k - R].wait()
            evs[k - R].synchronize()
        s = k % R
        dst = hv[s * sb:(s + 1) * sb].view(np.float32)
        for j in range(per):
            fn(paths[k * per + j].ctypes.data, L, n, dst[j * L * n:].ctypes.data, None, None)
        done[k].set()

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    futs = [ex.submit(work, k) for k in range(items)]
    with torch.cuda.stream(cs):
        for k in range(items):
            done[k].wait()
            s = k % R
            d[k * sb:(k + 1) * sb].copy_(h[s * sb:(s + 1) * sb], non_blocking=True)
            e = torch.cuda.Event()
            e.record(cs)
            evs[k] = e
            issued[k].set()
    cs.synchronize()
    dt = time.perf_counter() - t0
    for f in futs:
        f.result()
    return dt


def check(R, per):
    ref = np.concatenate(paths[:8]).astype(np.float32)
    got = d[:8 * PB].cpu().numpy().view(np.float32).reshape(-1, n)
    assert np.array_equal(got, ref), (R, per)


st = engine._STAGING
st._pool = ex
for _ in range(2):
    st.stage("obs", paths, n, np.float32, dev, reuse=True, ranges=True)
ts = []
for _ in range(4):
    torch.cuda.synchronize()
    t = time.perf_counter()
    st.stage("obs", paths, n, np.float32, dev, reuse=True, ranges=True)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
print("engine stage (slab, convert || h2d, ranges): %.1f ms" % (sorted(ts)[1] * 1e3), flush=True)
for name, fn in (("cached", SL.mjrl_host_stage_f64_portable), ("stream", SL.mjrl_host_stage_f64)):
    for R, per in ((8, 1), (16, 1), (32, 1), (64, 1), (16, 4)):
        ring(fn, R, per)
        ts = sorted(ring(fn, R, per) for _ in range(4))
        check(R, per)
        print("ring %-6s %2d slots x %d path (%5.1f MB): %.1f ms  (%.1f GB/s of f32)" % (
            name, R, per, R * per * PB / 2**20, ts[1] * 1e3, P * PB / ts[1] / 1e9), flush=True)
