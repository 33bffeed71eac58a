"""Times mjrl_moments_whiten_small (one workgroup) against mjrl_moments2 x 2 +
mjrl_whiten_moments (three launches) over batch sizes, HIP events over 50
back-to-back calls each (what UpdateEngine.SMALL_MOMENTS_ROWS is set from).
GPU box:  python tools/moments_probe.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mjrl_amd import _lib  # noqa: E402


def run(T, P, reps=50):
    L = _lib.lib()
    dev = torch.device("cuda:0")
    rs = np.random.RandomState(T)
    adv = torch.from_numpy(rs.randn(T)).to(dev)
    pr = torch.from_numpy(rs.randn(P)).to(dev)
    part = torch.zeros(_lib.MOM_SCRATCH, dtype=torch.float64, device=dev)
    st = torch.zeros(64, dtype=torch.float64, device=dev)
    a32 = torch.zeros(T, dtype=torch.float32, device=dev)
    p = lambda k: C.c_void_p(st[k:].data_ptr())   # noqa: E731
    sp = _lib.stream_ptr()

    def small():
        L.mjrl_moments_whiten_small(_lib.ptr(adv), T, _lib.ptr(pr), P, 1e-6, _lib.ptr(a32), None, _lib.ptr(part),
                                    p(0), p(8), p(16), p(24), p(32), sp)

    def three():
        L.mjrl_moments2(_lib.ptr(adv), T, None, _lib.ptr(pr), P, None, _lib.ptr(part), p(0), p(8), sp)
        L.mjrl_moments2(_lib.ptr(adv), T, p(0), _lib.ptr(pr), P, p(8), _lib.ptr(part), p(16), p(24), sp)
        L.mjrl_whiten_moments(_lib.ptr(adv), T, p(0), p(16), 1e-6, _lib.ptr(a32), None, _lib.ptr(part), p(32), sp)

    out = []
    for fn in (small, three):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps * 1e3)
    return out


if __name__ == "__main__":
    for T, P in ((500, 5), (1000, 10), (2000, 10), (4096, 20), (8192, 25), (12500, 25), (32768, 50), (65536, 64)):
        s, t = run(T, P)
        print("T %6d P %4d  one workgroup %7.2f us  three launches %7.2f us" % (T, P, s, t), flush=True)
