"""QuadraticBaseline.fit on the device (mjrl_quadratic_baseline_gram / _residual,
UpdateEngine.fit_quadratic_baseline) against the reference's own fit on
observations that are NOT float32s: tests/golden/quad_*.npz
(make_golden.py:quad_case, the reference's QuadraticBaseline.fit(return_errors=True)
twice, quadratic_baseline.py:40-65).  Point-mass, Swimmer and HalfCheetah widths
(19 / 49 / 175 features: one to three 64-column Gram tiles), ragged and
terminated paths, values past the +-10 clip.

Bars: coefficients within max(1e-10 |c|, 3x the reference's own path-order
spread), error_before / error_after within 1e-9 relative — for float32 rows with
their low halves (the default staging) and for float64 rows."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["quad_point_mass", "quad_swimmer", "quad_halfcheetah"]


def _case(name):
    from oracle import npg_cpu as O
    return O.load_f64obs(os.path.join(GOLD, name + ".npz"))


def _paths(c, m=2, seed=5):
    rs = np.random.RandomState(seed)
    return [dict(observations=o, actions=rs.randn(len(r), m), rewards=r, terminated=bool(t), agent_infos={},
                 env_infos={})
            for o, r, t in zip(c["obs_paths"], c["rew_paths"], c["terminated"])]


def _bound(c, key="coeffs1", spread=None):
    s = float(c["coeffs1_spread"]) if spread is None else spread
    return max(1e-10 * np.linalg.norm(c[key]), 3.0 * s)


@pytest.mark.parametrize("f64", [False, True])
@pytest.mark.parametrize("name", CASES)
def test_device_fit_matches_reference(name, f64):
    from mjrl_amd.baselines.quadratic_baseline import QuadraticBaseline
    from mjrl_amd.engine import DeviceBatch, UpdateEngine
    from mjrl_amd.utils.gym_env import EnvSpec
    c = _case(name)
    n = int(c["n"])
    paths = _paths(c)
    half = len(paths) // 2
    dev = torch.device("cuda:0")
    eng = UpdateEngine(n, 2, (64, 64), device=dev)
    qb = QuadraticBaseline(EnvSpec(n, 2, 1000, 1))
    off = np.concatenate([[0], np.cumsum(c["lengths"])])
    dt = np.float64 if f64 else np.float32
    for sub, key, ekey in ((paths[:half], "coeffs0", "err0"), (paths, "coeffs1", "err1")):
        b = DeviceBatch.from_paths(sub, dev, baseline=None, obs_dtype=dt)
        lo = None if f64 else b.obs_lo(sub, reuse=False)
        assert f64 or lo is not None   # genuinely f64 values: the low halves are staged
        y = torch.from_numpy(np.ascontiguousarray(c["returns"][:off[len(sub)]])).to(dev)
        err = eng.fit_quadratic_baseline(b, qb, returns=y, return_errors=True, obs_lo=lo)
        # the half-path fit's spread is not stored; its conditioning is the full fit's
        assert np.linalg.norm(qb._coeffs - c[key]) <= _bound(c, key), (key, np.linalg.norm(qb._coeffs - c[key]))
        np.testing.assert_allclose(err, c[ekey], rtol=1e-9)


@pytest.mark.parametrize("name", CASES[1:])
def test_agent_fits_quadratic_baseline_on_device(name, monkeypatch):
    """The agent's own route: train_from_samples stages the batch (float32 rows,
    host QuadraticBaseline predictions from the f64 paths), then _fit_baseline
    fits on the device from the rows still in HBM plus their low halves."""
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.quadratic_baseline import QuadraticBaseline
    from mjrl_amd.engine import UpdateEngine
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec

    class _Env:
        env_id = "quad-v0"

    c = _case(name)
    n, m = int(c["n"]), 2
    spec = EnvSpec(n, m, 1000, 1)
    qb = QuadraticBaseline(spec)
    qb._coeffs = c["coeffs0"].copy()
    agent = NPG(_Env(), MLP(spec, hidden_sizes=(64, 64), seed=0), qb, normalized_step_size=0.01, seed=1,
                device="cuda:0")
    calls = []
    orig = UpdateEngine.fit_quadratic_baseline
    monkeypatch.setattr(UpdateEngine, "fit_quadratic_baseline",
                        lambda self, *a, **k: calls.append(1) or orig(self, *a, **k))
    paths = _paths(c, m)
    agent.train_from_samples(paths, float(c["gamma"]), 0.97)
    assert np.array_equal(np.concatenate([p["returns"] for p in paths]), c["returns"])
    err = agent._fit_baseline(paths, return_errors=True)
    assert calls, "the QuadraticBaseline fit did not run on the device"
    assert np.linalg.norm(qb._coeffs - c["coeffs1"]) <= _bound(c)
    np.testing.assert_allclose(err, c["err1"], rtol=1e-9)
