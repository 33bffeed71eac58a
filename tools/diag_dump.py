"""Diagnostic (GPU box): dumps the HIP path's VPG, FVPs and CG solution for some
golden cases to gpurun_out/diag_<case>.npz for offline accuracy analysis."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from test_gpu_parity import run_case  # noqa: E402

for name in sys.argv[1:]:
    c, kw, eng, res = run_case(name)
    dev = torch.device("cuda:0")
    damping = kw.get("damping", 1e-4)
    out = dict(g=eng.vec["g"].cpu().numpy(), x=eng.vec["x"].cpu().numpy(),
               theta1=eng.vec["theta_new"].cpu().numpy(), alpha=res["alpha"], kl=res["kl_dist"])
    out["fv"] = eng.fvp(torch.from_numpy(c["hvp_v"]).to(dev), damping=damping).cpu().numpy()
    out["zs"] = np.array([eng.fvp(torch.from_numpy(p.astype(np.float32)).to(dev), damping=damping).cpu().numpy()
                          for p in c["cg_p"]])
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez("gpurun_out/diag_%s.npz" % name, **out)
    print(name, "ok")
