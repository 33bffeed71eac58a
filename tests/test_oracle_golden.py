"""Pins the oracle (oracle/npg_cpu.py) against the reference's own outputs.

The fixtures were produced by running bennevans/mjrl's update code on seeded
synthetic paths (tests/golden/make_golden.py).  Tolerances:
  * returns / advantages / baseline / path-return stats: bit-exact (fp64, same
    operation order as process_samples.py:37-44).
  * whitened advantages: rtol 1e-12 (numpy pairwise sums reordered only in ulps).
  * LL / mean / surrogate / VPG / single FVP: rtol 1e-5 of the vector norm
    (fp32; the reference disagrees with itself across torch thread counts at
    ~5e-7).
  * CG teacher-forced per iteration: rtol 1e-5.
  * end-to-end npg_grad / theta1: norm-relative 1e-3 and cosine >= 0.99999
    (the fp32 CG amplifies reduction-order noise).
"""
import os

import numpy as np
import pytest
import torch

from conftest import golden_cases, GOLDEN
from oracle import npg_cpu as O

CASES = golden_cases()


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def cos(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.dot(b) / (np.linalg.norm(a) * np.linalg.norm(b))


def load(name):
    return O.load_case(os.path.join(GOLDEN, name + ".npz"))


@pytest.mark.parametrize("name", CASES)
def test_returns_advantages_bitexact(name):
    c = load(name)
    lam = None if np.isnan(c["gae_lambda"]) else float(c["gae_lambda"])
    base = O.linear_baseline_predict(c["baseline_coeffs"], c["obs64"], c["lengths"])
    assert np.array_equal(base, c["baseline"])
    ret, adv = O.returns_and_advantages(c["rewards"], c["baseline"], c["lengths"],
                                        c["terminated"].astype(bool), float(c["gamma"]), lam)
    assert np.array_equal(ret, c["returns"])
    assert np.array_equal(adv, c["advantages"])


@pytest.mark.parametrize("name", CASES)
def test_whitening_and_stats(name):
    c = load(name)
    w = O.whiten(c["advantages"])
    np.testing.assert_allclose(w, c["adv_whitened"], rtol=1e-12, atol=1e-12)
    st = O.path_return_stats(c["rewards"], c["lengths"])
    np.testing.assert_allclose(st, c["base_stats"], rtol=1e-12)


@pytest.mark.parametrize("name", CASES)
def test_policy_forward_and_grads(name):
    c = load(name)
    torch.set_num_threads(1)
    pol = O.Policy(int(c["n"]), int(c["m"]), c["hidden_t"], c["theta0"], c["transforms"])
    assert pol.d == c["theta0"].size
    assert list(pol.sizes) == list(c["param_sizes"])
    k = len(c["mean0"])   # regenerated (large) fixtures keep the first rows only
    mu, ll = pol.mean_ll(pol.new, c["obs64"][:k], c["act64"][:k])
    assert nrel(mu.detach().numpy(), c["mean0"]) < 1e-6
    assert nrel(ll.detach().numpy(), c["ll0"]) < 1e-6
    kw = O.case_kwargs(c)
    idx = O.hvp_rows(c)
    fv = pol.fvp(c["obs64"][idx], c["act64"][idx], c["hvp_v"], kw.get("damping", 1e-4))
    assert nrel(fv, c["hvp_out"]) < 1e-5
    if kw["algo"] != "dapg":
        g = pol.flat_vpg(c["obs64"], c["act64"], c["adv_whitened"])
        assert nrel(g, c["vpg_grad"]) < 1e-5


@pytest.mark.parametrize("name", CASES)
def test_cg_teacher_forced(name):
    """Feed the reference's own CG search directions into the oracle FVP."""
    c = load(name)
    torch.set_num_threads(1)
    pol = O.Policy(int(c["n"]), int(c["m"]), c["hidden_t"], c["theta0"], c["transforms"])
    damping = O.case_kwargs(c).get("damping", 1e-4)
    for p, z, idx in zip(c["cg_p"], c["cg_z"], O.cg_rows(c)):
        assert nrel(pol.fvp(c["obs64"][idx], c["act64"][idx], p, damping), z) < 1e-5


@pytest.mark.parametrize("name", CASES)
def test_full_update(name):
    c = load(name)
    torch.set_num_threads(1)
    pol = O.Policy(int(c["n"]), int(c["m"]), c["hidden_t"], c["theta0"], c["transforms"])
    kw = O.case_kwargs(c)
    res = O.update(pol, c["obs64"], c["act64"], c["advantages"], c["rewards"], c["lengths"], **kw)
    assert nrel(res["vpg_grad"], c["cg_b"]) < 1e-5
    assert nrel(res["npg_grad"], c["cg_x"]) < 1e-3
    assert cos(res["npg_grad"], c["cg_x"]) > 0.99999
    assert nrel(res["theta1"], c["theta1"]) < 1e-3
    np.testing.assert_allclose(res["alpha"], c["log_alpha"], rtol=2e-3)
    np.testing.assert_allclose(res["kl_dist"], c["log_kl_dist"], rtol=2e-3, atol=1e-7)
    surr_imp = res["surr_after"] - res["surr_before"]
    np.testing.assert_allclose(surr_imp, c["log_surr_improvement"], rtol=2e-3, atol=1e-7)
    np.testing.assert_allclose(res["base_stats"], c["base_stats"], rtol=1e-12)
    if kw["algo"] == "trpo":
        n_trials = len(c["kl_calls"]) - 1
        assert len(res["trials"]) == n_trials
