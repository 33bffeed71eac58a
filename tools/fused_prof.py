"""Phase profile of the fused VPG / FVP kernel (k_fused) on the GPU box.

Needs the profiling build (python -m mjrl_amd.build --prof) and
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so.  Runs FWD and 3 FVPs on a
Swimmer-shaped batch (n 8, m 2, MLP(64, 64); T rows, default 12500) and prints,
per mode, the cycles wave 0 of workgroup 0 spent between consecutive stamps.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mjrl_amd import _lib  # noqa: E402
from mjrl_amd.engine import UpdateEngine  # noqa: E402

NAMES = {0: "loop top", 1: "P1 gemm", 2: "epilogue 1", 3: "P2", 4: "P3", 5: "row pass", 6: "P4", 7: "P5",
         8: "wgrad 2/1", 9: "bias sums", 10: "gW0", 11: "tail puts", 12: "tail barrier"}
NPROF = 24


def read(lib):
    out = (C.c_ulonglong * NPROF)()
    _lib.check(lib.mjrl_debug_kx_prof(out), "mjrl_debug_kx_prof")
    return np.array(out[:NPROF], dtype=np.float64)


def main(T=12500, n=8, m=2):
    lib = _lib.load()
    lib.mjrl_debug_kx_prof.argtypes = [C.c_void_p]
    lib.mjrl_debug_kx_prof.restype = C.c_int
    rs = np.random.RandomState(0)
    eng = UpdateEngine(n, m, (64, 64), device="cuda:0")
    obs = rs.randn(T, n).astype(np.float32)
    act = rs.randn(T, m).astype(np.float32)
    eng.load_rows(obs, act, rs.randn(T))
    d = eng.shape.d
    theta = (rs.randn(d) * 0.05).astype(np.float32)
    th = torch.from_numpy(theta).cuda()
    read(lib)
    eng.forward_pass(th, T)
    torch.cuda.synchronize()
    res = {"FWD": read(lib)}
    v = torch.from_numpy(rs.randn(d).astype(np.float32)).cuda()
    for _ in range(3):
        eng.fvp(v, T=T)
    torch.cuda.synchronize()
    read(lib)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        eng.fvp(v, T=T)
    e1.record()
    torch.cuda.synchronize()
    res["FVP"] = read(lib) / 3
    print("FVP + gather: %.1f us per call (events, includes host launch gaps)" % (e0.elapsed_time(e1) / 3 * 1e3))
    print("cycles per launch (wave 0 of workgroup 0, launches counted: FWD %d, FVP %.0f)"
          % (res["FWD"][17], res["FVP"][17]))
    print("%-16s" % "phase" + "".join("%10s" % k for k in res))
    for i, nm in [(15, "preamble")] + sorted(NAMES.items()) + [(16, "tail stores")]:
        print("%-16s" % nm + "".join("%10.0f" % (r[i] / max(r[17], 1)) for r in res.values()))
    print("%-16s" % "total" + "".join("%10.0f" % (r[list(NAMES) + [15, 16]].sum() / max(r[17], 1))
                                      for r in res.values()))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
