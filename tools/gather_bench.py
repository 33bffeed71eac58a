"""Times k_gather (slab fold) on the Humanoid shape: right after an FVP launch,
and re-run on the same (now clean) slabs, to separate the fold from the
write-back of the slabs the FVP kernel just wrote."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mjrl_amd import _lib  # noqa: E402
from mjrl_amd.engine import UpdateEngine  # noqa: E402


def main(T=1000000):
    rs = np.random.RandomState(0)
    eng = UpdateEngine(376, 17, (64, 64), device="cuda:0")
    eng.load_rows(rs.randn(T, 376).astype(np.float32), rs.randn(T, 17).astype(np.float32), rs.randn(T))
    th = torch.from_numpy((rs.randn(29410) * 0.05).astype(np.float32)).cuda()
    eng.forward_pass(th, T)
    L, s = eng.lib, eng.shape
    sp = C.byref(s)
    rows = eng._rows(T, eng.ws["adv32"])
    sc = eng._scratch(T)
    st = _lib.stream_ptr()
    ev = lambda: torch.cuda.Event(enable_timing=True)
    res = {"after_fvp": [], "repeat": [], "fvp": []}
    for _ in range(5):
        e0, e1, e2, e3 = ev(), ev(), ev(), ev()
        e0.record()
        _lib.check(L.mjrl_fvp_accumulate(sp, C.byref(rows), T, _lib.ptr(eng.packed_theta), _lib.ptr(eng.packed_p),
                                         None, None, C.byref(sc), st), "fvp")
        e1.record()
        _lib.check(L.mjrl_gather_grads(sp, C.byref(rows), T, C.byref(sc), 0, None, _lib.ptr(eng.vec["gsum"]), st),
                   "gather")
        e2.record()
        _lib.check(L.mjrl_gather_grads(sp, C.byref(rows), T, C.byref(sc), 0, None, _lib.ptr(eng.vec["gsum"]), st),
                   "gather")
        e3.record()
        torch.cuda.synchronize()
        res["fvp"].append(e0.elapsed_time(e1) * 1e3)
        res["after_fvp"].append(e1.elapsed_time(e2) * 1e3)
        res["repeat"].append(e2.elapsed_time(e3) * 1e3)
    for k, v in res.items():
        print("%-10s us: %s" % (k, " ".join("%.1f" % x for x in v)))


if __name__ == "__main__":
    main()
