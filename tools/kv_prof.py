"""Phase profile of the pipelined FVP kernel (k_kv, kv.h) on the GPU box.

Needs the profiling build (python -m mjrl_amd.build --prof) and
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so.  Runs FVPs on a Humanoid-shaped
batch and prints the cycles wave 0 of workgroup 0 spent per interval, per tile.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mjrl_amd import _lib  # noqa: E402
from mjrl_amd.engine import UpdateEngine  # noqa: E402

NAMES = ["I1 P2 (+DMA half)", "I1 barrier", "I2 P3+gW2+aload", "I2 DMA wait+bar", "I3 P1a+P4", "I3 gW1",
         "I3 barrier", "I4 P1b+P5", "I4 P6", "I4 -", "I4 barrier", "I1 DMA issue"]
NPROF = 24


def read(lib):
    out = (C.c_ulonglong * NPROF)()
    _lib.check(lib.mjrl_debug_kx_prof(out), "mjrl_debug_kx_prof")
    return np.array(out[:NPROF], dtype=np.float64)


def main(T=1000000, reps=3):
    lib = _lib.load()
    lib.mjrl_debug_kx_prof.argtypes = [C.c_void_p]
    lib.mjrl_debug_kx_prof.restype = C.c_int
    rs = np.random.RandomState(0)
    eng = UpdateEngine(376, 17, (64, 64), device="cuda:0", precision="split")
    obs = rs.randn(T, 376).astype(np.float32)
    act = rs.randn(T, 17).astype(np.float32)
    eng.load_rows(obs, act, rs.randn(T))
    theta = (rs.randn(29410) * 0.05).astype(np.float32)
    th = torch.from_numpy(theta).cuda()
    eng.forward_pass(th, T)
    torch.cuda.synchronize()
    v = torch.from_numpy(rs.randn(29410).astype(np.float32)).cuda()
    eng.fvp(v, T=T)
    torch.cuda.synchronize()
    read(lib)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        eng.fvp(v, T=T)
    e1.record()
    torch.cuda.synchronize()
    r = read(lib) / reps
    tiles = ((T + 31) // 32 + 255) // 256
    print("FVP + gather: %.1f us per call (events), %d tiles per workgroup" % (e0.elapsed_time(e1) / reps * 1e3, tiles))
    print("cycles per tile (wave 0 of workgroup 0):")
    for i, n in enumerate(NAMES):
        print("  %-18s %8.0f" % (n, r[i] / tiles))
    for i, n in ((19, " I4 epilogue"), (20, " I4 images")):
        print("  %-18s %8.0f" % (n, r[i] / tiles))
    print("  %-18s %8.0f" % ("total", (r[:12].sum() + r[18:21].sum()) / tiles))
    print("preamble + prologue %8.0f   tail %8.0f   past-headroom tiles %.1f" % (r[15], r[16], r[12]))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1000000)
