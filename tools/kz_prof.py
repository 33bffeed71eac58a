"""Interval profile of the three-role FVP kernel (k_kz, kz.h) on the GPU box.

Needs the profiling build (python -m mjrl_amd.build --prof) and
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so.  Runs FVPs on a Humanoid-shaped
batch and prints, per role (wave 0 of each role in workgroup 0) and interval, the
cycles of work (interval start -> its barrier) and the interval's total (-> the
barrier's release), per period (tile).
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mjrl_amd import _lib  # noqa: E402
from mjrl_amd.engine import UpdateEngine  # noqa: E402

NPROF = 28
ROLES = ["P1 (first layer, next tile)", "P6 (gW0 sums, previous tile; image refill)", "chain (P2 / P3 / P4+gW2 / P5+gW1)"]


def main(T=1000000, reps=3):
    lib = _lib.load()
    lib.mjrl_debug_kz_prof.argtypes = [C.c_void_p]
    lib.mjrl_debug_kz_prof.restype = C.c_int
    out = (C.c_ulonglong * NPROF)()
    rs = np.random.RandomState(0)
    eng = UpdateEngine(376, 17, (64, 64), device="cuda:0", precision="split")
    obs = rs.randn(T, 376).astype(np.float32)
    act = rs.randn(T, 17).astype(np.float32)
    eng.load_rows(obs, act, rs.randn(T))
    th = torch.from_numpy((rs.randn(29410) * 0.05).astype(np.float32)).cuda()
    eng.forward_pass(th, T)
    v = torch.from_numpy(rs.randn(29410).astype(np.float32)).cuda()
    eng.fvp(v, T=T)
    torch.cuda.synchronize()
    lib.mjrl_debug_kz_prof(out)   # clear
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        eng.fvp(v, T=T)
    e1.record()
    torch.cuda.synchronize()
    _lib.check(lib.mjrl_debug_kz_prof(out), "mjrl_debug_kz_prof")
    a = np.array(out[:NPROF], dtype=np.float64)
    per = a[24]
    print("FVP + gather: %.1f us per call (events, profiling build)" % (e0.elapsed_time(e1) / reps * 1e3))
    print("periods per launch (workgroup 0): %.0f" % (per / reps))
    print("cycles per period: work (interval start -> barrier) / total (-> release)")
    print("%-46s %13s %13s %13s %13s %9s" % ("role", "I1", "I2", "I3", "I4", "sum"))
    for r, name in enumerate(ROLES):
        w = a[r * 8:r * 8 + 8:2] / per
        t = a[r * 8 + 1:r * 8 + 8:2] / per
        print("%-46s %s %9.0f" % (name, " ".join("%6.0f/%6.0f" % (w[i], t[i]) for i in range(4)), t.sum()))


if __name__ == "__main__":
    main()
