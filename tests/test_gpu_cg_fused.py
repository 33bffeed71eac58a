"""The one-launch CG solve (mjrl_cg_solve_fused, csrc/cgf.h) against the
per-iteration launches it replaces (mjrl_fvp_accumulate + mjrl_gather_cg_z +
mjrl_cg_step_xr_p per iteration, cg_solve.py:9-20 with npg_cg.py:55-74): the same
folds in the same order, so parameters, CG counters and statistics are bit for
bit equal — eager, as a replayed hipGraph, and through the residual_tol break."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
FUSED_CASES = ["c2_swimmer", "c2_ragged", "c1_pointmass_mlp32", "c2_h48x32", "c2_logstd_clamp"]


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _run(name, fused, graphs, residual_tol=1e-10, reps=1):
    from mjrl_amd import engine as E
    from oracle import npg_cpu as O
    c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
    kw = O.case_kwargs(c)
    offs = np.concatenate([[0], np.cumsum(c["lengths"])])
    batch = E.DeviceBatch(_t(c["obs64"]), _t(c["act64"]), _t(c["rewards"]), _t(c["baseline"]), _t(offs),
                          _t(c["terminated"].astype(np.uint8)))
    eng = E.UpdateEngine(int(c["n"]), int(c["m"]), c["hidden_t"], device=DEV)
    if c["transforms"] is not None:
        eng.set_transformations(*c["transforms"])
    eng.graphs = graphs
    args = dict(algo="npg", gamma=float(c["gamma"]), gae_lambda=float(c["gae_lambda"]),
                n_step_size=kw.get("n_step_size", 0.01), residual_tol=residual_tol)
    th0 = _t(c["theta0"].astype(np.float32))
    saved = E.CG_FUSED_SOLVE
    E.CG_FUSED_SOLVE = fused
    try:
        out = []
        for _ in range(reps):
            res = eng.update(batch, th0, **args)
            out.append((res, eng.vec["theta_new"].cpu().numpy().copy(), eng.vec["x"].cpu().numpy().copy()))
    finally:
        E.CG_FUSED_SOLVE = saved
    return eng, out


def test_fused_path_is_taken():
    from mjrl_amd import _lib
    from mjrl_amd.engine import UpdateEngine
    eng = UpdateEngine(8, 2, (64, 64), device=DEV)
    assert int(_lib.lib().mjrl_fused_path(eng.shape)) == 1


@pytest.mark.parametrize("name", FUSED_CASES)
def test_one_launch_cg_bit_identical(name):
    _, (ref,) = _run(name, False, False)
    _, (got,) = _run(name, True, False)
    assert np.array_equal(got[2], ref[2]), "CG solution differs"
    assert np.array_equal(got[1], ref[1]), "parameters differ"
    for k in ("cg_iters", "alpha", "kl_dist", "surr_after", "base_stats"):
        assert got[0][k] == ref[0][k], k


@pytest.mark.parametrize("name", ["c2_swimmer", "c2_ragged"])
def test_one_launch_cg_in_graph_replay(name):
    """Captured (the kernel with its grid barriers inside the update's graph) and
    replayed: the eager loop's result, bit for bit, on every replay."""
    _, (ref,) = _run(name, False, False)
    _, outs = _run(name, True, True, reps=4)
    for res, th, x in outs:
        assert np.array_equal(th, ref[1]) and np.array_equal(x, ref[2])
        assert res["cg_iters"] == ref[0]["cg_iters"]


def test_one_launch_cg_residual_break():
    """residual_tol reached at once (tol above any r.r): the same early exit after
    one iteration (cg_solve.py:19-20), the same iteration count and solution."""
    _, (ref,) = _run("c2_swimmer", False, False, residual_tol=1e30)
    _, (got,) = _run("c2_swimmer", True, False, residual_tol=1e30)
    assert ref[0]["cg_iters"] == 1
    assert got[0]["cg_iters"] == ref[0]["cg_iters"]
    assert np.array_equal(got[2], ref[2]) and np.array_equal(got[1], ref[1])
