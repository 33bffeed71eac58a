"""Host -> HBM staging of a 1M-row Humanoid batch on the GPU box's host: the
f64 -> f32 convert-and-range pass alone (portable loop vs the AVX-512 streaming
path), the H2D copy alone, and the pipelined engine stage (conversion || H2D).

    python tools/stage_convert_probe.py [threads] [pin]

pin: "none" (the OS places the threads), "node0" (main thread and workers on
node 0's first physical cores, the data first-touched there), "spread".
"""
import concurrent.futures as cf
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mjrl_amd import _lib, engine  # noqa: E402

n, P, L = 376, 1000, 1000
nth = int(sys.argv[1]) if len(sys.argv) > 1 else engine._host_threads()
pin = sys.argv[2] if len(sys.argv) > 2 else "none"
allowed = sorted(os.sched_getaffinity(0))


def node_cpus(k):
    out = []
    for part in open("/sys/devices/system/node/node%d/cpulist" % k).read().strip().split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return [c for c in out if c in allowed]


cpus = None
if pin == "node0":
    cpus = node_cpus(0)[:nth]
elif pin == "spread":
    c0, c1 = node_cpus(0), node_cpus(1)
    cpus = [c for pair in zip(c0, c1) for c in pair][:nth]
if cpus:
    os.sched_setaffinity(0, {cpus[0]})
rs = np.random.RandomState(0)
paths = [rs.randn(L, n) for _ in range(P)]
R = P * L
SL = _lib.stage_lib()
print("threads %d  avx512 %d  cpus %s" % (nth, SL.mjrl_host_stage_avx512(), sorted(os.sched_getaffinity(0))[:4]))
try:
    nodes = sorted(d for d in os.listdir("/sys/devices/system/node") if d.startswith("node"))
    print("numa nodes", nodes, [open("/sys/devices/system/node/%s/cpulist" % d).read().strip() for d in nodes])
except OSError:
    pass
h = torch.empty(R * n * 4, dtype=torch.uint8, pin_memory=True)
view = h.numpy().view(np.float32).reshape(R, n)
_tid = iter(range(10**6))


def _init():
    if cpus:
        os.sched_setaffinity(0, {cpus[next(_tid) % len(cpus)]})


ex = cf.ThreadPoolExecutor(nth, initializer=_init)
list(ex.map(lambda i: time.sleep(0.01), range(nth)))
if cpus:
    print("pinned to", cpus)


def convert(fn, ranges):
    rng = np.empty((P, 2, n), np.float32)
    rng[:, 0], rng[:, 1] = np.inf, -np.inf

    def f(i):
        a = paths[i]
        lo, hi = (rng[i, 0].ctypes.data, rng[i, 1].ctypes.data) if ranges else (None, None)
        fn(a.ctypes.data, L, n, view[i * L:].ctypes.data, lo, hi)
    list(ex.map(f, range(P)))


ts = []
for _ in range(4):
    t = time.perf_counter()
    list(ex.map(lambda i: float(paths[i].sum()), range(P)))
    ts.append(time.perf_counter() - t)
t = sorted(ts)[1]
print("read-only pass (numpy sum, threads): %.1f ms (%.1f GB/s)" % (t * 1e3, R * n * 8 / t / 1e9), flush=True)
res = {}
for name, fn in (("portable", SL.mjrl_host_stage_f64_portable), ("avx512", SL.mjrl_host_stage_f64),
                 ):
    for ranges in (True, False):
        ts = []
        for _ in range(4):
            t = time.perf_counter()
            convert(fn, ranges)
            ts.append(time.perf_counter() - t)
        t = sorted(ts)[1]
        res[(name, ranges)] = t
        print("convert %-8s ranges=%d: %.1f ms  (%.1f GB/s read + %.1f GB/s written)" % (
            name, ranges, t * 1e3, R * n * 8 / t / 1e9, R * n * 4 / t / 1e9), flush=True)
dev = torch.device("cuda:0")
d = torch.empty(R * n * 4, dtype=torch.uint8, device=dev)
for _ in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    th = time.perf_counter() - t
print("h2d alone %.1f ms (%.1f GB/s)" % (th * 1e3, R * n * 4 / th / 1e9), flush=True)
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
print("engine stage (convert || h2d, ranges): %.1f ms (median of 4)" % (sorted(ts)[1] * 1e3), flush=True)

# the bench's e2e staging call: every slot of a DeviceBatch (obs with ranges, act,
# rewards, offsets, flags) and the device LinearBaseline predict
from mjrl_amd.baselines.linear_baseline import LinearBaseline  # noqa: E402
from mjrl_amd.utils.gym_env import EnvSpec  # noqa: E402
acts = [rs.randn(L, 17) for _ in range(P)]
pd = [dict(observations=o, actions=a, rewards=rs.randn(L), terminated=False) for o, a in zip(paths, acts)]
base = LinearBaseline(EnvSpec(n, 17, L, 1))
base._coeffs = rs.randn(n + 4) * 0.01
for _ in range(2):
    engine.DeviceBatch.from_paths(pd, dev, baseline=base, reuse=True)
ts = []
for _ in range(4):
    torch.cuda.synchronize()
    t = time.perf_counter()
    engine.DeviceBatch.from_paths(pd, dev, baseline=base, reuse=True)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
print("DeviceBatch.from_paths (all slots + device baseline): %.1f ms (median of 4)" % (sorted(ts)[1] * 1e3))
st.trace = tr = []
t0 = time.perf_counter()
engine.DeviceBatch.from_paths(pd, dev, baseline=base, reuse=True)
torch.cuda.synchronize()
st.trace = None
by = {}
for c in tr:
    if c["fill"]:
        d = by.setdefault(c["slot"], [1e9, 0, 0.0])
        d[0] = min(d[0], c["fill"][0] - t0)
        d[1] = max(d[1], c["fill"][1] - t0)
        d[2] += c["fill"][1] - c["fill"][0]
for k, (a, b, busy) in by.items():
    print("  slot %-6s fill span %.1f -> %.1f ms, summed chunk fill %.1f ms" % (k, a * 1e3, b * 1e3, busy * 1e3))
