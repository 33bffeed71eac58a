"""Bit-exactness A/B of the row kernels between two library builds (GPU box).

    MJRL_AMD_LIB=<lib A> python tools/fused_exact.py dump a.npz
    MJRL_AMD_LIB=<lib B> python tools/fused_exact.py dump b.npz
    python tools/fused_exact.py compare a.npz b.npz

`dump` runs forward_pass (VPG), two FVPs and an eval_pass on seeded inputs for a
set of policy shapes covering the k_fused instantiations (hidden 32 / 64, MP 16 /
32, one or several 64-column observation chunks, partial last tiles, more tiles
than workgroups) and saves the results; `compare` requires them bit-identical.
A kernel change meant to move only WHERE operands come from (LDS images instead
of L2) must leave every bit unchanged.
"""
import os
import sys

import numpy as np

SHAPES = [  # (n, m, hidden, T)
    (8, 2, (64, 64), 12500),     # Swimmer (c2)
    (8, 2, (64, 64), 64),        # one tile
    (17, 6, (64, 64), 20003),    # HalfCheetah shape, partial last tile
    (17, 6, (32, 32), 9001),
    (100, 6, (64, 64), 7777),    # two observation chunks
    (45, 20, (64, 64), 5000),    # MP 32
    (150, 20, (32, 32), 4001),   # three chunks, MP 32
    (8, 2, (64, 64), 40000),     # more tiles than workgroups
]


UPDATE_CASES = ["c2_swimmer", "c2_constlr", "c2_logstd_clamp", "c2_nogae", "c2_ragged", "c2_hvp_sub", "c2_h48x32",
                "c1_pointmass_mlp32", "c3_halfcheetah_full", "c3_trpo_backtrack", "c4_humanoid", "c4_humanoid_scaled"]


def dump(path):
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from mjrl_amd.engine import UpdateEngine
    out = {}
    for k, (n, m, hid, T) in enumerate(SHAPES):
        rs = np.random.RandomState(100 + k)
        eng = UpdateEngine(n, m, hid, device="cuda:0", precision="f32")
        eng.load_rows(rs.randn(T, n), rs.randn(T, m), rs.randn(T))
        d = eng.shape.d
        theta = torch.from_numpy((rs.randn(d) * 0.1).astype(np.float32)).cuda()
        g = eng.forward_pass(theta, T).cpu().numpy()
        z1 = eng.fvp(torch.from_numpy(rs.randn(d).astype(np.float32)).cuda(), T=T).cpu().numpy()
        z2 = eng.fvp(torch.from_numpy(rs.randn(d).astype(np.float32)).cuda(), T=T).cpu().numpy()
        th2 = theta + torch.from_numpy((rs.randn(d) * 0.01).astype(np.float32)).cuda()
        sur, kl = eng.eval_pass(th2, T)
        out["s%d_g" % k], out["s%d_z1" % k], out["s%d_z2" % k] = g, z1, z2
        out["s%d_ev" % k] = np.array([sur, kl], dtype=np.float32)
        print("shape", (n, m, hid, T), "fused", eng.fused, "|g|", float(np.abs(g).sum()), "|z1|",
              float(np.abs(z1).sum()), flush=True)
    # whole updates on the golden cases (the CG loop, graphs, line searches)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    import test_gpu_parity as TP
    for name in UPDATE_CASES:
        c, kw, eng, res = TP.run_case(name)
        out["u_%s_theta" % name] = eng.vec["theta_new"].cpu().numpy()
        out["u_%s_x" % name] = eng.pvec["x"].cpu().numpy()
        out["u_%s_cg" % name] = eng.cg[:5].cpu().numpy()
        print("update", name, "cg", eng.cg[:5].cpu().numpy(), flush=True)
    np.savez(path, **out)


def compare(pa, pb):
    a, b = np.load(pa), np.load(pb)
    bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
    for k in bad:
        print("DIFF", k, "max abs", float(np.max(np.abs(a[k].astype(np.float64) - b[k]))))
    print("bit-identical: %d / %d arrays" % (len(a.files) - len(bad), len(a.files)))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
