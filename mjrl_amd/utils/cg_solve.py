"""Conjugate gradient (API of mjrl/utils/cg_solve.py:3-22) with the vector
arithmetic on the GPU.  `f_Ax` is the caller's operator (numpy in, numpy out, as
in the reference); x, r, p and the dot products / updates live on the device in
fp32 like the reference's fp32 numpy arrays.  x_0 is ignored, as in the
reference.  The NPG update itself uses the fully device-resident CG
(mjrl_cg_init / mjrl_cg_step) with no per-iteration host round trip."""
import ctypes as C

import numpy as np
import torch

from .. import _lib


def cg_solve(f_Ax, b, x_0=None, cg_iters=10, residual_tol=1e-10):
    L = _lib.lib()
    dev = torch.device("cuda")
    st = _lib.stream_ptr()
    b32 = torch.from_numpy(np.ascontiguousarray(b, dtype=np.float32)).to(dev)
    d = int(b32.numel())
    x, r, p, z = (torch.empty(d, dtype=torch.float32, device=dev) for _ in range(4))
    cg = torch.zeros(_lib.CG_STATE, dtype=torch.float32, device=dev)   # MJRL_CG_STATE
    done = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(L.mjrl_cg_init_vec(d, _lib.ptr(b32), _lib.ptr(x), _lib.ptr(r), _lib.ptr(p), _lib.ptr(cg),
                                  _lib.ptr(done), st), "mjrl_cg_init_vec")
    for _ in range(cg_iters):
        zz = f_Ax(p.cpu().numpy())
        z.copy_(torch.from_numpy(np.ascontiguousarray(zz, dtype=np.float32)))
        _lib.check(L.mjrl_cg_update(d, _lib.ptr(z), _lib.ptr(x), _lib.ptr(r), _lib.ptr(p), _lib.ptr(cg),
                                    _lib.ptr(done), float(residual_tol), st), "mjrl_cg_update")
        if int(done.item()):
            break
    return x.cpu().numpy().astype(np.asarray(b).dtype, copy=False)
