"""Where the host -> HBM staging time of a 1M-row Humanoid batch goes: the f64 ->
f32 conversion into pinned memory alone (all staging threads), the H2D copy of
the pinned f32 buffer alone, and the pipelined stage (conversion || H2D) as the
engine runs it, at a few chunk sizes."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from mjrl_amd import engine  # noqa: E402

n, P, L = 376, 1000, 1000
rs = np.random.RandomState(0)
paths = [rs.randn(L, n) for _ in range(P)]
dev = torch.device("cuda:0")
st = engine._STAGING
R = P * L
h = torch.empty(R * n * 4, dtype=torch.uint8, pin_memory=True)
view = h.numpy().view(np.float32).reshape(R, n)
ex = st.pool()
print("threads", engine._host_threads())


def fill_all():
    def f(i):
        np.copyto(view[i * L:(i + 1) * L], paths[i], casting="unsafe")
    list(ex.map(f, range(P)))


for _ in range(2):
    t = time.perf_counter(); fill_all(); tf = time.perf_counter() - t
d = torch.empty(R * n * 4, dtype=torch.uint8, device=dev)
for _ in range(3):
    torch.cuda.synchronize(); t = time.perf_counter(); d.copy_(h, non_blocking=True); torch.cuda.synchronize()
    th = time.perf_counter() - t
print("fill %.1f ms (%.1f GB/s out)  h2d %.1f ms (%.1f GB/s)" % (tf * 1e3, R * n * 4 / tf / 1e9, th * 1e3,
                                                                 R * n * 4 / th / 1e9))
for mb in (16, 32, 64, 128):
    st.CHUNK_BYTES = mb << 20
    ts = []
    for _ in range(3):
        torch.cuda.synchronize(); t = time.perf_counter()
        st.stage("obs", paths, n, np.float32, dev, reuse=True); torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    print("stage chunk %d MB: %.1f ms (median)" % (mb, sorted(ts)[1] * 1e3))
