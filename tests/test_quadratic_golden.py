"""The QuadraticBaseline fixtures (tests/golden/quad_*.npz, the reference's own
fit / predict, make_golden.py:quad_case) against mjrl_amd's host QuadraticBaseline
(the reference's algorithm restated: features, ridge normal equations, lstsq
retry) on the regenerated inputs: pins the fixtures the device fit is tested
against (tests/test_gpu_quadratic.py)."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", ["quad_point_mass", "quad_swimmer", "quad_halfcheetah"])
def test_host_quadratic_baseline_matches_reference(name):
    from oracle import npg_cpu as O
    from mjrl_amd.baselines.quadratic_baseline import QuadraticBaseline
    from mjrl_amd.utils.gym_env import EnvSpec
    c = O.load_f64obs(os.path.join(GOLD, name + ".npz"))
    n = int(c["n"])
    off = np.concatenate([[0], np.cumsum(c["lengths"])])
    paths = [dict(observations=o, rewards=r, returns=c["returns"][off[i]:off[i + 1]])
             for i, (o, r) in enumerate(zip(c["obs_paths"], c["rew_paths"]))]
    q = QuadraticBaseline(EnvSpec(n, 1, 1000, 1))
    err0 = q.fit(paths[: len(paths) // 2], return_errors=True)
    np.testing.assert_allclose(q._coeffs, c["coeffs0"], rtol=0, atol=1e-12 * np.linalg.norm(c["coeffs0"]))
    np.testing.assert_allclose(err0, c["err0"], rtol=1e-12)
    err1 = q.fit(paths, return_errors=True)
    np.testing.assert_allclose(q._coeffs, c["coeffs1"], rtol=0, atol=1e-12 * np.linalg.norm(c["coeffs1"]))
    np.testing.assert_allclose(err1, c["err1"], rtol=1e-12)
    np.testing.assert_allclose(q.predict(paths[-1]), c["predict_last"], rtol=1e-12, atol=1e-12)
    assert len(q._coeffs) == n + n * (n + 1) // 2 + 5
