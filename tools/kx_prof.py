"""Phase profile of the all-split K-split kernel (k_kx) on the GPU box.

Needs the profiling build (python -m mjrl_amd.build --prof) and
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so.  Runs FWD, 3 FVPs and EVAL on a
Humanoid-shaped batch and prints, per mode, the cycles wave 0 of workgroup 0
spent between consecutive barriers, per tile.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mjrl_amd import _lib  # noqa: E402
from mjrl_amd.engine import UpdateEngine  # noqa: E402

NAMES = ["publish", "P1 first layer", "P1 fold", "P2", "P3", "row pass", "P4", "P5", "P6 barrier", "loop top",
         "P6 xload", "P6 G0 split", "P6 gW0", "P6 gW1", "P6 gW2+bias"]


NPROF = 24


def read(lib):
    out = (C.c_ulonglong * NPROF)()
    _lib.check(lib.mjrl_debug_kx_prof(out), "mjrl_debug_kx_prof")
    return np.array(out[:NPROF], dtype=np.float64)


def main(T=1000000):
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
    tiles = (T + 31) // 32 // 256 + 1
    read(lib)
    eng.forward_pass(th, T)
    torch.cuda.synchronize()
    res = {"FWD": read(lib)}
    v = torch.from_numpy(rs.randn(29410).astype(np.float32)).cuda()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        eng.fvp(v, T=T)
    e1.record()
    torch.cuda.synchronize()
    res["FVP"] = read(lib) / 3
    print("FVP + gather: %.1f us per call (events)" % (e0.elapsed_time(e1) / 3 * 1e3))
    eng.eval_pass(th, T)
    torch.cuda.synchronize()
    res["EVAL"] = read(lib)
    print("cycles per tile (wave 0 of workgroup 0, ~%d tiles)" % tiles)
    print("%-16s" % "phase" + "".join("%10s" % k for k in res))
    for i, n in enumerate(NAMES):
        print("%-16s" % n + "".join("%10.0f" % (r[i] / tiles) for r in res.values()))
    print("%-16s" % "total" + "".join("%10.0f" % (r[:15].sum() / tiles) for r in res.values()))
    print("per launch (cycles, workgroup 0):")
    for i, n in ((15, "preamble"), (18, " loads issued"), (19, " W0 slice split"), (20, " row scales+bar"),
                 (21, " col scales+bar"), (22, " image stores"), (23, " xhat load+bar"), (16, "tail")):
        print("%-16s" % n + "".join("%10.0f" % (r[i] / max(r[17], 1)) for r in res.values()))
    print("%-16s" % "tile loop" + "".join("%10.0f" % (r[:15].sum() / max(r[17], 1)) for r in res.values()))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1000000)
