"""A/B of the host -> HBM staging of a 1M-row Humanoid batch on one box: the
observations, actions and rewards staged slot after slot (_PinnedStaging.stage,
as DeviceBatch.from_paths does); the f64 -> f32 conversion alone and the H2D copy
alone for reference.  (A variant staging all three slots in one chunked pipeline
measured 52 ms against 32.5 ms: profiles/r03f/staging_ab.txt.)"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from mjrl_amd import engine  # noqa: E402

n, m, P, L = 376, 17, 1000, 1000
rs = np.random.RandomState(0)
obs = [rs.randn(L, n) for _ in range(P)]
act = [rs.randn(L, m) for _ in range(P)]
rew = [rs.randn(L) for _ in range(P)]
dev = torch.device("cuda:0")
st = engine._STAGING
print("threads", engine._host_threads(), flush=True)


def sep():
    st.stage("obs", obs, n, np.float32, dev, reuse=True)
    st.stage("act", act, m, np.float32, dev, reuse=True)
    st.stage("rew", rew, 0, np.float64, dev, reuse=True)


for name, fn in (("separate", sep), ("separate", sep)):
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    print("%-9s %s ms (median %.1f)" % (name, " ".join("%.1f" % x for x in ts), sorted(ts)[2]), flush=True)
R = P * L
h = torch.empty(R * n * 4, dtype=torch.uint8, pin_memory=True)
d = torch.empty(R * n * 4, dtype=torch.uint8, device=dev)
for _ in range(3):
    torch.cuda.synchronize(); t = time.perf_counter(); d.copy_(h, non_blocking=True); torch.cuda.synchronize()
    th = time.perf_counter() - t
view = h.numpy().view(np.float32).reshape(R, n)
ex = st.pool()
for _ in range(2):
    t = time.perf_counter()
    list(ex.map(lambda i: np.copyto(view[i * L:(i + 1) * L], obs[i], casting="unsafe"), range(P)))
    tf = time.perf_counter() - t
print("obs alone: f64->f32 fill %.1f ms, H2D %.1f ms (%.1f GB/s)" % (tf * 1e3, th * 1e3, R * n * 4 / th / 1e9))
