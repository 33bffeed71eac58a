"""Times the policy passes of one engine build on the GPU box: FWD (vpg
accumulate), FVP accumulate and EVAL at T rows of the Humanoid shape, HIP events
on the launch stream, median of 20.  MJRL_AMD_LIB selects the library build.
    python tools/fvp_time.py [T] [precision]"""
import os
os.environ.setdefault("MJRL_AMD_ALLOW_ABLATION", "1")   # this tool times ablation builds
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mjrl_amd import _lib  # noqa: E402
from mjrl_amd.engine import UpdateEngine  # noqa: E402


def main(T=1000000, prec="split"):
    rs = np.random.RandomState(0)
    eng = UpdateEngine(376, 17, (64, 64), device="cuda:0", precision=prec)
    eng.load_rows(rs.randn(T, 376).astype(np.float32), rs.randn(T, 17).astype(np.float32), rs.randn(T))
    theta = torch.from_numpy((rs.randn(29410) * 0.05).astype(np.float32)).cuda()
    eng.forward_pass(theta, T)
    L, s = eng.lib, eng.shape
    sp = C.byref(s)
    rows, sc = eng._rows(T, eng.ws["adv32"]), eng._scratch(T)
    _lib.check(L.mjrl_pack_params(sp, _lib.ptr(theta), _lib.ptr(eng.packed_p), 0, -3.0, _lib.stream_ptr()), "pack")
    st = _lib.stream_ptr()
    tn = torch.from_numpy((rs.randn(29410) * 0.05).astype(np.float32)).cuda()
    _lib.check(L.mjrl_pack_params(sp, _lib.ptr(tn), _lib.ptr(eng.packed_new), 1, -3.0, st), "pack")

    def fwd():
        _lib.check(L.mjrl_vpg_accumulate(sp, C.byref(rows), _lib.ptr(eng.packed_theta), None, None, C.byref(sc), st),
                   "vpg")

    def fvp():
        _lib.check(L.mjrl_fvp_accumulate(sp, C.byref(rows), T, _lib.ptr(eng.packed_theta), _lib.ptr(eng.packed_p),
                                         None, None, C.byref(sc), st), "fvp")

    def ev():
        _lib.check(L.mjrl_policy_eval(sp, C.byref(rows), T, _lib.ptr(eng.packed_new), _lib.ptr(eng.packed_theta),
                                      None, None, C.byref(sc), C.c_void_p(eng.stats.data_ptr()), st), "eval")

    out = {}
    for name, f in (("fwd", fwd), ("fvp", fvp), ("eval", ev)):
        for _ in range(3):
            f()
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        out[name] = float(np.median(ts))
    fvp_bytes = 4 * s.np + 4 + 4 * 128
    print("%s T=%d fwd %.3f ms  fvp %.3f ms (%.1f%% of 8 TB/s)  eval %.3f ms" % (
        os.environ.get("MJRL_AMD_LIB", "default"), T, out["fwd"], out["fvp"],
        100 * fvp_bytes * T / (out["fvp"] * 1e-3) / 8e12, out["eval"]))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1000000, sys.argv[2] if len(sys.argv) > 2 else "split")
