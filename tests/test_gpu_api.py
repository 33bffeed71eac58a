"""GPU tests of the drop-in API (mjrl_amd.algos / policies / utils) and of
size-independent properties at full scale.  Fixture tolerances as in
test_gpu_parity.py."""
import os

import ctypes as C

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def load(name):
    from oracle import npg_cpu as O
    return O.load_case(os.path.join(GOLDEN, name + ".npz"))


def paths_of(c, with_adv=True):
    offs = np.concatenate([[0], np.cumsum(c["lengths"])])
    out = []
    for i in range(len(c["lengths"])):
        s = slice(offs[i], offs[i + 1])
        p = dict(observations=c["obs64"][s], actions=c["act64"][s], rewards=c["rewards"][s],
                 terminated=bool(c["terminated"][i]), agent_infos={}, env_infos={})
        if with_adv:
            p["advantages"] = c["advantages"][s]
        out.append(p)
    return out


def make_policy(c):
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.policies.gaussian_linear import LinearPolicy
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(int(c["n"]), int(c["m"]), 1000, 1)
    pol = LinearPolicy(spec, seed=0) if int(c["linear"]) else MLP(spec, hidden_sizes=c["hidden_t"], seed=0)
    if c["transforms"] is not None:
        for mdl in (pol.model, pol.old_model):
            mdl.set_transformations(*c["transforms"])
    pol.set_param_values(c["theta0"], set_new=True, set_old=True)
    return pol, spec


def tol(c, key, floor):
    return max(floor, 3.0 * float(c["spread_" + key]))


def make_agent(name, c, pol, spec):
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.algos.trpo import TRPO
    from mjrl_amd.algos.dapg import DAPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from oracle import npg_cpu as O
    base = LinearBaseline(spec)
    if c["baseline_coeffs"].size:
        base._coeffs = c["baseline_coeffs"]
    kw = O.case_kwargs(c)
    if kw["algo"] == "npg":
        args = {}
        if "kw_normalized_step_size" in c:
            args["normalized_step_size"] = float(c["kw_normalized_step_size"])
        if "kw_const_learn_rate" in c:
            args["const_learn_rate"] = float(c["kw_const_learn_rate"])
        if "kw_hvp_sample_frac" in c:
            args["hvp_sample_frac"] = float(c["kw_hvp_sample_frac"])
        return NPG(None, pol, base, save_logs=True, **args), base
    if kw["algo"] == "trpo":
        return TRPO(None, pol, base, kl_dist=kw["kl_dist"], save_logs=True), base
    offs = np.concatenate([[0], np.cumsum(c["demo_lengths"])])
    demos = [dict(observations=c["demo_obs"][offs[i]:offs[i + 1]].astype(np.float64),
                  actions=c["demo_act"][offs[i]:offs[i + 1]].astype(np.float64))
             for i in range(len(c["demo_lengths"]))]
    return DAPG(None, pol, base, demo_paths=demos, save_logs=True), base


REF_KEYS = {"npg": {"alpha", "delta", "time_vpg", "time_npg", "kl_dist", "surr_improvement", "running_score",
                    "stoc_pol_mean", "stoc_pol_std", "stoc_pol_max", "stoc_pol_min"}}


@pytest.mark.parametrize("name", ["c1_pointmass_linear", "c2_swimmer", "c3_trpo_backtrack", "c4_humanoid",
                                  "c5_door_dapg", "c2_constlr", "c2_hvp_sub"])
def test_train_from_paths(name):
    c = load(name)
    pol, spec = make_policy(c)
    agent, _ = make_agent(name, c, pol, spec)
    if "np_seed" in c:
        np.random.seed(int(c["np_seed"]))
    stats = agent.train_from_paths(paths_of(c))
    np.testing.assert_allclose(stats, c["base_stats"], rtol=1e-12)
    assert nrel(pol.get_param_values(), c["theta1"]) < tol(c, "theta", 1e-3)
    log = agent.logger.get_current_log()
    assert REF_KEYS["npg"] <= set(log) | {"delta", "time_npg"}
    np.testing.assert_allclose(log["alpha"], c["log_alpha"], rtol=tol(c, "alpha", 2e-3))
    np.testing.assert_allclose(log["kl_dist"], c["log_kl_dist"], rtol=tol(c, "kl", 2e-3), atol=1e-7)
    np.testing.assert_allclose(agent.running_score, c["base_stats"][0], rtol=1e-12)
    # the CPU mirror now holds the device result, old == new
    old = np.concatenate([p.data.reshape(-1).numpy() for p in pol.old_params])
    assert np.array_equal(old, pol.get_param_values())


@pytest.mark.parametrize("name", ["c2_ragged", "c2_nogae", "c2_swimmer"])
def test_train_from_samples_fused_gae(name):
    """train_step's path: raw paths + baseline -> GAE on device -> update; the
    returns / baseline / advantages written back into the paths are bit-exact."""
    c = load(name)
    pol, spec = make_policy(c)
    agent, base = make_agent(name, c, pol, spec)
    paths = paths_of(c, with_adv=False)
    lam = None if np.isnan(c["gae_lambda"]) else float(c["gae_lambda"])
    stats = agent.train_from_samples(paths, float(c["gamma"]), lam)
    from oracle import npg_cpu as O
    assert np.array_equal(np.concatenate([p["returns"] for p in paths]), c["returns"])
    # the LinearBaseline prediction now runs on the device (rtol 1e-12 vs numpy's
    # dgemv order); the GAE scan is bit-exact given those predictions
    bl = np.concatenate([p["baseline"] for p in paths])
    np.testing.assert_allclose(bl, c["baseline"], rtol=1e-12, atol=1e-12)
    _, adv_ref = O.returns_and_advantages(c["rewards"], bl, c["lengths"], c["terminated"].astype(bool),
                                          float(c["gamma"]), lam)
    assert np.array_equal(np.concatenate([p["advantages"] for p in paths]), adv_ref)
    np.testing.assert_allclose(np.concatenate([p["advantages"] for p in paths]), c["advantages"], rtol=1e-9,
                               atol=1e-12)
    np.testing.assert_allclose(stats, c["base_stats"], rtol=1e-12)
    assert nrel(pol.get_param_values(), c["theta1"]) < tol(c, "theta", 1e-3)


def test_process_samples_bitexact():
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.utils import process_samples as ps
    from mjrl_amd.utils.gym_env import EnvSpec
    from oracle import npg_cpu as O
    c = load("c2_ragged")
    paths = paths_of(c, with_adv=False)
    base = LinearBaseline(EnvSpec(8, 2, 10, 1))
    base._coeffs = c["baseline_coeffs"]
    ps.compute_returns(paths, float(c["gamma"]))
    ps.compute_advantages(paths, base, float(c["gamma"]), float(c["gae_lambda"]))
    assert np.array_equal(np.concatenate([p["returns"] for p in paths]), c["returns"])
    assert np.array_equal(np.concatenate([p["advantages"] for p in paths]), c["advantages"])
    x = np.random.RandomState(0).randn(37)
    assert np.array_equal(ps.discount_sum(x, 0.9), O.discount_sum(x, 0.9))
    assert np.array_equal(ps.discount_sum(x, 0.9, terminal=2.5), O.discount_sum(x, 0.9, terminal=2.5))
    ps.compute_advantages(paths, base, float(c["gamma"]), float(c["gae_lambda"]), normalize=True)
    a = c["advantages"]
    np.testing.assert_allclose(np.concatenate([p["advantages"] for p in paths]),
                               (a - a.mean()) / (a.std() + 1e-8), rtol=1e-12, atol=1e-12)


def test_cg_solve_generic_matches_reference_semantics():
    from mjrl_amd.utils.cg_solve import cg_solve
    from oracle import npg_cpu as O
    rs = np.random.RandomState(2)
    A = rs.randn(300, 300).astype(np.float32)
    A = (A @ A.T / 300 + np.eye(300, dtype=np.float32)).astype(np.float32)
    b = rs.randn(300).astype(np.float32)
    f = lambda v: (A @ v).astype(np.float32)
    x = cg_solve(f, b, cg_iters=10)
    xr = O.cg_solve(f, b.copy(), iters=10)
    assert x.dtype == np.float32
    assert nrel(x, xr) < 1e-5
    x3 = cg_solve(f, b, cg_iters=300, residual_tol=1e-10)
    assert nrel(A @ x3, b) < 1e-4


def test_single_passes_match_reference():
    """CPI_surrogate / kl_old_new / flat_vpg / HVP called directly (the reference API)."""
    c = load("c2_swimmer")
    pol, spec = make_policy(c)
    agent, _ = make_agent("c2_swimmer", c, pol, spec)
    obs, act = c["obs64"], c["act64"]
    g = agent.flat_vpg(obs, act, c["adv_whitened"])
    assert nrel(g, c["vpg_grad"]) < 1e-5
    hv = agent.HVP(obs, act, c["hvp_v"])
    assert nrel(hv, c["hvp_out"]) < 1e-5
    assert abs(float(agent.kl_old_new(obs, act))) < 1e-7          # old == new
    surr = float(agent.CPI_surrogate(obs, act, c["adv_whitened"]))
    np.testing.assert_allclose(surr, c["surr_calls"][0], atol=1e-7)
    # after moving only the new params, surrogate / KL against the oracle
    from oracle import npg_cpu as O
    pol.set_param_values(c["theta1"], set_new=True, set_old=False)
    ref = O.Policy(8, 2, (64, 64), c["theta0"], None)
    ref.set_params(c["theta1"], set_new=True, set_old=False)
    np.testing.assert_allclose(float(agent.kl_old_new(obs, act)), float(ref.kl(obs, act).detach()), rtol=1e-4)
    np.testing.assert_allclose(float(agent.CPI_surrogate(obs, act, c["adv_whitened"])),
                               float(ref.surrogate(obs, act, c["adv_whitened"]).detach()), rtol=1e-4, atol=1e-7)
    with pytest.raises(ValueError):
        agent.flat_vpg(obs, act, c["adv_whitened"])


# ---------------------------------------------------------------------------
# size-independent properties at full scale (Humanoid shape)
# ---------------------------------------------------------------------------
def _engine_with_rows(T, seed=0):
    from mjrl_amd.engine import UpdateEngine
    rs = np.random.RandomState(seed)
    eng = UpdateEngine(376, 17, (64, 64), device="cuda:0")
    obs = rs.randn(T, 376)
    act = rs.randn(T, 17)
    eng.load_rows(obs, act, rs.randn(T))
    theta = (rs.randn(29410) * 0.05).astype(np.float32)
    theta[-17:] = np.linspace(-1, 0.5, 17)
    th = torch.from_numpy(theta).cuda()
    eng.forward_pass(th, T)
    return eng, rs


@pytest.mark.parametrize("T", [300000])
def test_fvp_properties_full_scale(T):
    eng, rs = _engine_with_rows(T)
    d = 29410
    v = torch.from_numpy(rs.randn(d).astype(np.float32)).cuda()
    w = torch.from_numpy(rs.randn(d).astype(np.float32)).cuda()
    Fv = eng.fvp(v, damping=0.0, T=T).double()
    Fw = eng.fvp(w, damping=0.0, T=T).double()
    # symmetry: w.Fv == v.Fw
    a, b = torch.dot(w.double(), Fv).item(), torch.dot(v.double(), Fw).item()
    assert abs(a - b) / abs(a) < 1e-4
    # positive semi-definite
    assert torch.dot(v.double(), Fv).item() > 0 and torch.dot(w.double(), Fw).item() > 0
    # linearity
    F2 = eng.fvp(2.0 * v - 3.0 * w, damping=0.0, T=T).double()
    assert (torch.norm(F2 - (2 * Fv - 3 * Fw)) / torch.norm(F2)).item() < 1e-5
    # damping adds exactly damping * v
    Fd = eng.fvp(v, damping=0.5, T=T).double()
    assert (torch.norm(Fd - Fv - 0.5 * v.double()) / torch.norm(Fd)).item() < 1e-6


def test_fvp_row_permutation_invariance():
    """Reordering timesteps only reorders sums (the update is path-order invariant)."""
    from mjrl_amd.engine import UpdateEngine
    T = 5000
    rs = np.random.RandomState(3)
    obs, act = rs.randn(T, 376), rs.randn(T, 17)
    theta = (rs.randn(29410) * 0.05).astype(np.float32)
    theta[-17:] = np.linspace(-1, 0.5, 17)
    th = torch.from_numpy(theta).cuda()
    v = torch.from_numpy(rs.randn(29410).astype(np.float32)).cuda()
    eng = UpdateEngine(376, 17, (64, 64), device="cuda:0")
    eng.load_rows(obs, act)
    g1 = eng.forward_pass(th, T).cpu().numpy()
    F1 = eng.fvp(v, damping=0.0, T=T).cpu().numpy()
    perm = np.random.RandomState(9).permutation(T)
    eng.load_rows(obs[perm], act[perm])
    g2 = eng.forward_pass(th, T).cpu().numpy()
    F2 = eng.fvp(v, damping=0.0, T=T).cpu().numpy()
    assert nrel(F1, F2) < 1e-5
    assert nrel(g1, g2) < 1e-5 or np.linalg.norm(g1) < 1e-6


def test_edge_cases_tiny_and_ragged():
    """One path of length 1, paths shorter than a tile, terminated flags, a
    batch smaller than one 64-row tile: against the oracle."""
    from mjrl_amd.engine import UpdateEngine, DeviceBatch
    from oracle import npg_cpu as O
    rs = np.random.RandomState(4)
    for lengths in ([1], [1, 2, 3], [63, 1, 64, 65]):
        lengths = np.array(lengths)
        T = int(lengths.sum())
        n, m = 6, 3
        obs = rs.randn(T, n).astype(np.float32).astype(np.float64)
        act = rs.randn(T, m).astype(np.float32).astype(np.float64)
        rew = rs.randn(T)
        base = rs.randn(T)
        term = (np.arange(len(lengths)) % 2).astype(np.uint8)
        theta = (rs.randn(6 * 32 + 32 + 32 * 32 + 32 + 3 * 32 + 3 + 3) * 0.1).astype(np.float32)
        eng = UpdateEngine(n, m, (32, 32), device="cuda:0")
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
        off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
        b = DeviceBatch(t(obs), t(act), t(rew), t(base), t(off), t(term))
        res = eng.update(b, t(theta), algo="npg", gamma=0.99, gae_lambda=0.95, n_step_size=0.05)
        ret, adv = O.returns_and_advantages(rew, base, lengths, term.astype(bool), 0.99, 0.95)
        assert np.array_equal(eng.ws["adv64"][:T].cpu().numpy(), adv)
        assert np.array_equal(eng.ws["ret"][:T].cpu().numpy(), ret)
        if T < 3:
            continue   # whitening of 1-2 samples is degenerate in the reference too
        pol = O.Policy(n, m, (32, 32), theta.astype(np.float64), None)
        g = pol.flat_vpg(obs, act, O.whiten(adv))
        assert nrel(eng.vec["g"].cpu().numpy(), g) < 1e-5
        np.testing.assert_allclose(res["base_stats"], O.path_return_stats(rew, lengths), rtol=1e-12)


def test_linear_baseline_predict_on_device():
    """a4: LinearBaseline.predict computed on the device from the staged obs."""
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.engine import DeviceBatch
    from mjrl_amd.utils.gym_env import EnvSpec
    c = load("c2_ragged")
    base = LinearBaseline(EnvSpec(8, 2, 10, 1))
    base._coeffs = c["baseline_coeffs"]
    b = DeviceBatch.from_paths(paths_of(c, with_adv=False), torch.device("cuda:0"), baseline=base)
    np.testing.assert_allclose(b.baseline.cpu().numpy(), c["baseline"], rtol=1e-12, atol=1e-12)
    base._coeffs = None
    b = DeviceBatch.from_paths(paths_of(c, with_adv=False), torch.device("cuda:0"), baseline=base)
    assert np.array_equal(b.baseline.cpu().numpy(), np.zeros(c["baseline"].shape))


@pytest.mark.parametrize("use_gae", [1, 0])
@pytest.mark.parametrize("fn", ["mjrl_gae", "mjrl_gae_wave"])
def test_gae_kernel_ragged_many_paths(use_gae, fn):
    """Both GAE kernels (lanes = paths, 8 paths per workgroup and 256-step
    windows: mjrl_gae; one wave per path: mjrl_gae_wave) on 86 ragged paths
    (empty, 1, window +-1, several windows, terminated or not; P not a multiple
    of 8): bit-identical to the oracle's discount_sum chains."""
    from mjrl_amd import _lib
    from oracle import npg_cpu as O
    L = _lib.lib()
    rs = np.random.RandomState(23)
    lengths = np.concatenate([[0, 1, 2, 127, 128, 129, 255, 256, 257, 1000, 0, 3001, 640, 511, 512, 513],
                              rs.randint(1, 700, size=70)])
    T = int(lengths.sum())
    rew = rs.randn(T) * 3.0
    base = rs.randn(T)
    term = (rs.rand(len(lengths)) < 0.5).astype(np.uint8)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    ret = torch.full((T,), np.nan, dtype=torch.float64, device="cuda")
    adv = torch.full((T,), np.nan, dtype=torch.float64, device="cuda")
    pret = torch.full((len(lengths),), np.nan, dtype=torch.float64, device="cuda")
    gamma, lam = 0.99, 0.95
    args = [t(rew), t(base), t(off), t(term)]
    rc = getattr(L, fn)(*[_lib.ptr(a) for a in args], len(lengths), gamma, lam, use_gae, _lib.ptr(ret), _lib.ptr(adv),
                        _lib.ptr(pret), _lib.stream_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    keep = lengths > 0
    m = np.repeat(keep, lengths)
    r_ref, a_ref = O.returns_and_advantages(rew[m], base[m], lengths[keep], term[keep].astype(bool), gamma,
                                            lam if use_gae else None)
    assert np.array_equal(ret.cpu().numpy(), r_ref)
    assert np.array_equal(adv.cpu().numpy(), a_ref)
    pr = pret.cpu().numpy()
    assert np.array_equal(pr[keep], np.array([sum(r) for r in O.split(rew[m], lengths[keep])]))
    assert np.all(pr[~keep] == 0.0)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_gae_kernel_random_lengths(seed):
    """mjrl_gae on random batches (P in [1, 300], lengths in [0, 1200] with exact
    multiples of the 16-step segment and the 256-step window mixed in, random
    termination flags, GAE on and off): bit-identical to the oracle's chains."""
    from mjrl_amd import _lib
    from oracle import npg_cpu as O
    L = _lib.lib()
    rs = np.random.RandomState(100 + seed)
    P = int(rs.randint(1, 301))
    lengths = rs.randint(0, 1201, size=P)
    pick = rs.rand(P)
    lengths[pick < 0.15] = 16 * rs.randint(0, 40, size=int((pick < 0.15).sum()))
    lengths[pick > 0.9] = 256 * rs.randint(1, 5, size=int((pick > 0.9).sum()))
    T = int(lengths.sum())
    rew = rs.randn(T) * 2.0
    base = rs.randn(T)
    term = (rs.rand(P) < 0.5).astype(np.uint8)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    keep = lengths > 0
    m = np.repeat(keep, lengths)
    d_rew, d_base, d_off, d_term = t(rew), t(base), t(off), t(term)   # alive across the launches
    for use_gae in (1, 0):
        ret = torch.full((max(T, 1),), np.nan, dtype=torch.float64, device="cuda")
        adv = torch.full((max(T, 1),), np.nan, dtype=torch.float64, device="cuda")
        pret = torch.full((P,), np.nan, dtype=torch.float64, device="cuda")
        gamma, lam = 0.995, 0.97
        rc = L.mjrl_gae(_lib.ptr(d_rew), _lib.ptr(d_base), _lib.ptr(d_off), _lib.ptr(d_term), P, gamma, lam,
                        use_gae, _lib.ptr(ret), _lib.ptr(adv), _lib.ptr(pret), _lib.stream_ptr())
        assert rc == 0
        torch.cuda.synchronize()
        r_ref, a_ref = O.returns_and_advantages(rew[m], base[m], lengths[keep], term[keep].astype(bool), gamma,
                                                lam if use_gae else None)
        assert np.array_equal(ret.cpu().numpy()[:T], r_ref)
        assert np.array_equal(adv.cpu().numpy()[:T], a_ref)
        pr = pret.cpu().numpy()
        assert np.array_equal(pr[keep], np.array([sum(r) for r in O.split(rew[m], lengths[keep])]))
        assert np.all(pr[~keep] == 0.0)


@pytest.mark.parametrize("use_gae", [1, 0])
def test_gae_kernel_multiwindow_bitexact(use_gae):
    """mjrl_gae through the C-ABI on paths shorter than, equal to and longer
    than the 1024-step LDS window of rounds 1-5 (and an empty path): returns,
    advantages and per-path reward sums bit-identical to the oracle
    (process_samples.py:3-44, npg_cg.py:97)."""
    import ctypes as C
    from mjrl_amd import _lib
    from oracle import npg_cpu as O
    L = _lib.lib()
    rs = np.random.RandomState(11)
    lengths = np.array([1, 7, 1023, 1024, 1025, 0, 2048, 3001, 5, 64, 65])
    T = int(lengths.sum())
    rew = rs.randn(T) * 3.0
    base = rs.randn(T)
    term = (rs.rand(len(lengths)) < 0.5).astype(np.uint8)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    d_rew, d_base, d_off, d_term = t(rew), t(base), t(off), t(term)
    ret = torch.full((T,), np.nan, dtype=torch.float64, device="cuda")
    adv = torch.full((T,), np.nan, dtype=torch.float64, device="cuda")
    pret = torch.full((len(lengths),), np.nan, dtype=torch.float64, device="cuda")
    gamma, lam = 0.995, 0.97
    rc = L.mjrl_gae(_lib.ptr(d_rew), _lib.ptr(d_base), _lib.ptr(d_off), _lib.ptr(d_term), len(lengths), gamma, lam,
                    use_gae, _lib.ptr(ret), _lib.ptr(adv), _lib.ptr(pret), _lib.stream_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    keep = lengths > 0
    m = np.repeat(keep, lengths)
    r_ref, a_ref = O.returns_and_advantages(rew[m], base[m], lengths[keep], term[keep].astype(bool), gamma,
                                            lam if use_gae else None)
    assert np.array_equal(ret.cpu().numpy(), r_ref)
    assert np.array_equal(adv.cpu().numpy(), a_ref)
    pr = pret.cpu().numpy()
    assert np.array_equal(pr[keep], np.array([sum(r) for r in O.split(rew[m], lengths[keep])]))
    assert pr[~keep].tolist() == [0.0]


@pytest.mark.parametrize("use_gae", [1, 0])
def test_gae_scan_kernel(use_gae):
    """mjrl_gae_scan (the wave-shuffle scan form of process_samples.py:21-44) on
    paths shorter than, equal to and longer than its 1024-step window: returns and
    advantages within 1e-12 of each path's largest |value| of the oracle's
    discount_sum, path-return sums within 1e-12 relative; an empty path gives 0;
    the update engine with gae_mode="scan" on a full-size fixture lands on the
    same update as the exact scan."""
    from mjrl_amd import _lib
    from oracle import npg_cpu as O
    L = _lib.lib()
    rs = np.random.RandomState(12)
    lengths = np.array([1, 7, 63, 64, 65, 1023, 1024, 1025, 0, 2048, 3001, 5, 1000])
    T = int(lengths.sum())
    rew = rs.randn(T) * 3.0
    base = rs.randn(T)
    term = (rs.rand(len(lengths)) < 0.5).astype(np.uint8)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    ret = torch.full((T,), np.nan, dtype=torch.float64, device="cuda")
    adv = torch.full((T,), np.nan, dtype=torch.float64, device="cuda")
    pret = torch.full((len(lengths),), np.nan, dtype=torch.float64, device="cuda")
    gamma, lam = 0.995, 0.97
    d = [t(rew), t(base), t(off), t(term)]
    assert L.mjrl_gae_scan(*[_lib.ptr(x) for x in d], len(lengths), gamma, lam, use_gae, _lib.ptr(ret),
                           _lib.ptr(adv), _lib.ptr(pret), _lib.stream_ptr()) == 0
    torch.cuda.synchronize()
    keep = lengths > 0
    m = np.repeat(keep, lengths)
    r_ref, a_ref = O.returns_and_advantages(rew[m], base[m], lengths[keep], term[keep].astype(bool), gamma,
                                            lam if use_gae else None)
    r, a = ret.cpu().numpy(), adv.cpu().numpy()
    for x, y in ((r, r_ref), (a, a_ref)):
        for seg_x, seg_y in zip(O.split(x, lengths[keep]), O.split(y, lengths[keep])):
            assert np.abs(seg_x - seg_y).max() <= 1e-12 * np.abs(seg_y).max() + 1e-300
    pr = pret.cpu().numpy()
    np.testing.assert_allclose(pr[keep], np.array([sum(v) for v in O.split(rew[m], lengths[keep])]), rtol=1e-12)
    assert pr[~keep].tolist() == [0.0]
    # the whole update on the scan: the same as on the exact chain to fp32 noise
    res = {}
    from mjrl_amd.engine import UpdateEngine
    import test_gpu_parity as TP
    for mode in ("serial", "scan"):
        cc, case_kwargs = TP.load("c3_halfcheetah_full")
        kw = case_kwargs(cc)
        eng = UpdateEngine(int(cc["n"]), int(cc["m"]), cc["hidden_t"], device=torch.device("cuda:0"))
        eng.gae_mode = mode
        b = TP.make_batch(cc, torch.device("cuda:0"))
        out = eng.update(b, t(cc["theta0"].astype(np.float32)), algo="trpo", gamma=float(cc["gamma"]),
                         gae_lambda=float(cc["gae_lambda"]), kl_dist=kw["kl_dist"], trpo_verbose=False)
        res[mode] = (eng.vec["theta_new"].cpu().numpy(), out["kl_dist"], eng.ws["adv64"][:b.T].cpu().numpy())
    assert np.abs(res["scan"][2] - res["serial"][2]).max() <= 1e-12 * np.abs(res["serial"][2]).max()
    assert TP.nrel(res["scan"][0], res["serial"][0]) < 1e-5
    np.testing.assert_allclose(res["scan"][1], res["serial"][1], rtol=1e-4)


def test_subsampled_hvp_api():
    """NPG.HVP with hvp_sample_frac < 1 through the drop-in API: the reference's
    np.random.choice draw from numpy's global RNG (npg_cg.py:58-62)."""
    c = load("c2_hvp_sub")
    pol, spec = make_policy(c)
    agent, _ = make_agent("c2_hvp_sub", c, pol, spec)
    np.random.seed(int(c["hvp_np_seed"]))
    hv = agent.HVP(c["obs64"], c["act64"], c["hvp_v"])
    assert nrel(hv, c["hvp_out"]) < 1e-5


def test_linear_baseline_fit_on_device_matches_reference():
    """LinearBaseline.fit (linear_baseline.py:20-44) with the Gram products on the
    device: the reference fixture (ragged paths, +-10 clip, return_errors), then a
    Humanoid-width batch against numpy's F^T F / F^T y."""
    from mjrl_amd.baselines.linear_baseline import LinearBaseline, time_features
    from mjrl_amd.engine import DeviceBatch, UpdateEngine
    from mjrl_amd.utils.gym_env import EnvSpec
    z = np.load(os.path.join(GOLDEN, "baselines.npz"))
    lengths = z["lengths"]
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    n = z["obs"].shape[1]
    T = int(off[-1])
    b = DeviceBatch(t(z["obs"]), t(np.zeros((T, 2))), t(z["rewards"]), t(np.zeros(T)), t(off),
                    t(np.zeros(len(lengths), np.uint8)))
    eng = UpdateEngine(n, 2, (32, 32), device="cuda:0")
    base = LinearBaseline(EnvSpec(n, 2, 30, 1))
    errs = eng.fit_linear_baseline(b, base, returns=t(z["returns"]), return_errors=True)
    np.testing.assert_allclose(base._coeffs, z["lin_coeffs"], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(errs, z["lin_err"], rtol=1e-9)
    pred = np.concatenate([base.predict(dict(observations=z["obs"][off[i]:off[i + 1]],
                                             rewards=z["rewards"][off[i]:off[i + 1]]))
                           for i in range(len(lengths))])
    np.testing.assert_allclose(pred, z["lin_pred"], rtol=1e-9, atol=1e-12)

    # Humanoid width, ragged paths: Gram vs numpy, coefficients vs the host fit
    rs = np.random.RandomState(3)
    lengths = rs.randint(1, 1500, size=40)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    T, n = int(off[-1]), 376
    obs = rs.randn(T, n) * 4.0
    y = rs.randn(T) * 10.0
    b = DeviceBatch(t(obs), t(np.zeros((T, 17))), t(y), t(np.zeros(T)), t(off),
                    t(np.zeros(len(lengths), np.uint8)))
    eng = UpdateEngine(n, 17, (64, 64), device="cuda:0")
    dev = LinearBaseline(EnvSpec(n, 17, 1500, 1))
    eng.fit_linear_baseline(b, dev, returns=t(y))
    paths = [dict(observations=obs[off[i]:off[i + 1]], rewards=y[off[i]:off[i + 1]], returns=y[off[i]:off[i + 1]])
             for i in range(len(lengths))]
    host = LinearBaseline(EnvSpec(n, 17, 1500, 1))
    host.fit(paths)
    F = np.concatenate([time_features(p["observations"]) for p in paths])
    pd, ph = F @ dev._coeffs, F @ host._coeffs
    assert np.linalg.norm(pd - ph) / np.linalg.norm(ph) < 1e-9


def test_train_step_baseline_fit_path():
    """train_step's fit (batch_reinforce.py:93-101) after train_from_samples: the
    device fit from the batch in HBM equals the host LinearBaseline.fit on the
    returns written back into the paths."""
    import copy
    c = load("c2_swimmer")
    pol, spec = make_policy(c)
    agent, base = make_agent("c2_swimmer", c, pol, spec)
    paths = paths_of(c, with_adv=False)
    agent.train_from_samples(paths, float(c["gamma"]), float(c["gae_lambda"]))
    host = copy.deepcopy(base)
    eb, ea = agent._fit_baseline(paths, return_errors=True)
    hb, ha = host.fit(paths, return_errors=True)
    np.testing.assert_allclose([eb, ea], [hb, ha], rtol=1e-9)
    np.testing.assert_allclose(base._coeffs, host._coeffs, rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("name", ["c2_swimmer", "c4_humanoid", "c3_halfcheetah_trpo", "c5_door_dapg"])
def test_graph_replay_matches_eager(name):
    """UpdateEngine.graphs: the second identical update is captured as a hipGraph
    and later ones replay it; the replayed update must equal the eager one bit
    for bit (same kernels, same order, same reductions).  Covers every kernel
    family under capture: k_fused (c2), k_kx (c4), k_rows + k_wgrad_all (c3,
    run as NPG here; its TRPO search is the next test) and k_rows + k_wgrad
    with demo rows (c5, DAPG)."""
    from oracle import npg_cpu as O
    from mjrl_amd.engine import UpdateEngine
    import test_gpu_parity as P
    c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
    kw = O.case_kwargs(c)
    dev = torch.device("cuda:0")
    eng = UpdateEngine(int(c["n"]), int(c["m"]), c["hidden_t"], device=dev)
    if c["transforms"] is not None:
        eng.set_transformations(*c["transforms"])
    batch = P.make_batch(c, dev)
    th = torch.from_numpy(c["theta0"].astype(np.float32)).to(dev)
    lam = None if np.isnan(c["gae_lambda"]) else float(c["gae_lambda"])
    args = dict(algo="npg", gamma=float(c["gamma"]), gae_lambda=lam, n_step_size=0.05)
    if kw["algo"] == "dapg":
        args = dict(algo="dapg", gamma=float(c["gamma"]), gae_lambda=lam, kl_dist=kw["kl_dist"],
                    demo_coef=kw["demo_coef"])
    ref = eng.update(batch, th, graph=False, **args)
    ref_theta = eng.vec["theta_new"].cpu().numpy()
    eng.graphs = True
    outs = []
    for _ in range(4):
        res = eng.update(batch, th, **args)
        outs.append((res, eng.vec["theta_new"].cpu().numpy()))
    assert eng._gstate.get("graph") is not None
    for res, theta in outs:
        assert np.array_equal(theta, ref_theta)
        for k in ("alpha", "kl_dist", "surr_after", "surr_before", "cg_iters"):
            assert res[k] == ref[k], k
        np.testing.assert_array_equal(res["base_stats"], ref["base_stats"])
    # a different theta through the captured input buffer
    th2 = th * 1.01
    eng.update(batch, th2, graph=False, **args)
    ref2 = eng.vec["theta_new"].cpu().numpy()
    eng.update(batch, th2, **args)
    assert np.array_equal(eng.vec["theta_new"].cpu().numpy(), ref2)


@pytest.mark.parametrize("name", ["c3_trpo_backtrack", "c3_halfcheetah_trpo"])
def test_trpo_graph_replay_matches_eager(name):
    """TRPO under UpdateEngine.graphs: everything up to the first evaluation is
    captured and replayed, the KL backtracking (trpo.py:98-124) continues on the
    host after it; the replayed updates (trials included) must equal the eager one
    bit for bit.  c3_trpo_backtrack backtracks several times."""
    from oracle import npg_cpu as O
    from mjrl_amd.engine import UpdateEngine
    import test_gpu_parity as P
    c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
    kw = O.case_kwargs(c)
    assert kw["algo"] == "trpo"
    dev = torch.device("cuda:0")
    eng = UpdateEngine(int(c["n"]), int(c["m"]), c["hidden_t"], device=dev)
    if c["transforms"] is not None:
        eng.set_transformations(*c["transforms"])
    batch = P.make_batch(c, dev)
    th = torch.from_numpy(c["theta0"].astype(np.float32)).to(dev)
    lam = None if np.isnan(c["gae_lambda"]) else float(c["gae_lambda"])
    args = dict(algo="trpo", gamma=float(c["gamma"]), gae_lambda=lam, kl_dist=kw["kl_dist"],
                cg_iters=kw.get("cg_iters", 10), damping=kw.get("damping", 1e-4), trpo_verbose=False)
    ref = eng.update(batch, th, graph=False, **args)
    ref_theta = eng.vec["theta_new"].cpu().numpy()
    eng.graphs = True
    outs = []
    for _ in range(4):
        res = eng.update(batch, th, **args)
        outs.append((res, eng.vec["theta_new"].cpu().numpy()))
    assert eng._gstate.get("graph") is not None
    for res, theta in outs:
        assert np.array_equal(theta, ref_theta)
        assert res["trials"] == ref["trials"]
        for k in ("alpha", "kl_dist", "surr_after", "surr_before", "cg_iters"):
            assert res[k] == ref[k], k


def test_capture_survives_dead_graph_cycles():
    """The round-4 driver abort: the cyclic GC destroying a dead
    engine's captured graph, pinned readback buffers and events while another
    engine captures.  Dead cycles holding captured graphs are left for the
    collector (disabled meanwhile, so they are still there at the capture), then
    a TRPO update of the HalfCheetah shape is captured and replayed: every
    capture goes through mjrl_amd._capture.capture, which collects them first
    and keeps the collector off until the capture ends."""
    import gc
    from oracle import npg_cpu as O
    from mjrl_amd.engine import UpdateEngine
    import test_gpu_parity as P
    dev = torch.device("cuda:0")

    def engine(name, **extra):
        c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
        eng = UpdateEngine(int(c["n"]), int(c["m"]), c["hidden_t"], device=dev)
        batch = P.make_batch(c, dev)
        th = torch.from_numpy(c["theta0"].astype(np.float32)).to(dev)
        lam = None if np.isnan(c["gae_lambda"]) else float(c["gae_lambda"])
        eng.graphs = True
        outs = [eng.update(batch, th, gamma=float(c["gamma"]), gae_lambda=lam, **extra) for _ in range(3)]
        assert eng._gstate.get("graph") is not None
        return eng, outs

    enabled = gc.isenabled()
    gc.disable()
    try:
        for _ in range(2):
            a, _ = engine("c2_swimmer", algo="npg", n_step_size=0.05)
            a._cycle = a
            del a
        kl = O.case_kwargs(O.load_case(os.path.join(GOLDEN, "c3_trpo_backtrack.npz")))["kl_dist"]
        b, outs = engine("c3_trpo_backtrack", algo="trpo", kl_dist=kl, trpo_verbose=False)
    finally:
        if enabled:
            gc.enable()
    assert outs[1]["trials"] == outs[2]["trials"] and outs[1]["alpha"] == outs[2]["alpha"]
    torch.cuda.synchronize()


def test_mlp_baseline_fit_matches_reference():
    """MLPBaseline.fit / predict on the GPU (mlp_baseline.py:59-115) against the
    reference's own CPU fit: same initial weights, same minibatch order (numpy
    global RNG), two fits with the Adam state carried over.  fp32 GEMMs sum in
    another order than the reference's CPU ones and Adam's normalised steps carry
    that difference into the weights (2.1e-4 relative on the predictions measured
    on MI355X after two 2-epoch fits): rtol 1e-3 on the predictions."""
    import pickle
    from mjrl_amd.baselines.mlp_baseline import MLPBaseline
    from mjrl_amd.utils.gym_env import EnvSpec
    z = np.load(os.path.join(GOLDEN, "mlp_baseline.npz"))
    offs = np.concatenate([[0], np.cumsum(z["lengths"])])
    paths = [dict(observations=z["obs"][offs[i]:offs[i + 1]], rewards=z["rewards"][offs[i]:offs[i + 1]],
                  returns=z["returns"][offs[i]:offs[i + 1]]) for i in range(len(z["lengths"]))]
    torch.manual_seed(7)
    b = MLPBaseline(EnvSpec(5, 2, 300, 1), batch_size=64, epochs=2, learn_rate=3e-3)
    for it in range(2):
        np.random.seed(int(z["np_seed%d" % it]))
        err = b.fit(paths, return_errors=True)
        np.testing.assert_allclose(err, z["err%d" % it], rtol=1e-4)
        pred = np.concatenate([b.predict(p) for p in paths])
        np.testing.assert_allclose(pred, z["pred%d" % it], rtol=1e-3, atol=1e-4)
    for k, v in b.model.state_dict().items():
        # single weights next to a ReLU kink move by up to ~2e-3 (Adam's
        # normalised step on a near-zero gradient); each tensor as a whole agrees
        ref = z["final_" + k.replace(".", "_")]
        assert np.linalg.norm(v.numpy() - ref) <= 1e-3 * np.linalg.norm(ref), k
    clone = pickle.loads(pickle.dumps(b))   # CPU state: the fitted weights came back from the device
    np.testing.assert_allclose(np.concatenate([clone.predict(p) for p in paths]), pred, rtol=1e-5, atol=1e-6)


def test_mlp_baseline_device_batch_predict():
    """DeviceBatch.from_paths with an MLPBaseline predicts all rows with one
    device forward; equal to the per-path predict (f64-staged observations)."""
    from mjrl_amd.baselines.mlp_baseline import MLPBaseline
    from mjrl_amd.engine import DeviceBatch
    from mjrl_amd.utils.gym_env import EnvSpec
    rs = np.random.RandomState(3)
    paths = [dict(observations=rs.randn(L, 6) * 5, actions=rs.randn(L, 2), rewards=rs.randn(L))
             for L in (40, 1, 77)]
    torch.manual_seed(0)
    b = MLPBaseline(EnvSpec(6, 2, 100, 1))
    batch = DeviceBatch.from_paths(paths, torch.device("cuda:0"), baseline=b, obs_dtype=np.float64)
    ref = np.concatenate([b.predict(p) for p in paths])
    np.testing.assert_allclose(batch.baseline.cpu().numpy(), ref, rtol=1e-6, atol=1e-7)


def test_bc_on_gpu_matches_reference():
    """BC (behavior_cloning.py:11-68) with its minibatch steps replayed as a
    captured graph on the GPU, against the reference's CPU run: Adam's
    normalised steps carry the GEMM summation-order differences into the
    weights, so the final parameters agree in norm to 1e-3, the logged losses
    to 1e-4."""
    from test_bc_ppo import run_bc
    bc, policy, z = run_bc("cuda:0")
    assert bc.trainer().graphable
    np.testing.assert_allclose(np.array(bc.logger.log["loss"], dtype=np.float64), z["loss"], rtol=1e-4)
    ref = z["final"]
    assert np.linalg.norm(policy.get_param_values() - ref) <= 1e-3 * np.linalg.norm(ref)


def test_bc_train_twice_on_gpu_matches_cpu():
    """A second BC.train() on new expert data (the same trainer, the Adam state
    carried over) replays a graph captured for THAT call's rows, not the first
    call's: the GPU run tracks the CPU-device run of the same sequence."""
    from test_bc_ppo import run_bc
    out = {}
    for dev in ("cpu", "cuda:0"):
        bc, policy, z = run_bc(dev)
        rs = np.random.RandomState(99)
        bc.expert_paths = [dict(observations=p["observations"] * 0.5 + rs.randn(*p["observations"].shape) * 0.1,
                                actions=p["actions"][::-1].copy()) for p in bc.expert_paths]
        np.random.seed(123)
        bc.train()
        out[dev] = (policy.get_param_values(), np.array(bc.logger.log["loss"], dtype=np.float64))
    np.testing.assert_allclose(out["cuda:0"][1], out["cpu"][1], rtol=1e-4)
    ref = out["cpu"][0]
    assert np.linalg.norm(out["cuda:0"][0] - ref) <= 1e-3 * np.linalg.norm(ref)


def test_ppo_on_gpu_matches_reference():
    """PPO.train_from_paths (ppo_clip.py:57-120) twice (the Adam state carries
    over), against the reference run: base_stats exact; parameters in norm to
    1e-3; surrogate improvement and KL (HIP evaluation passes) to the same
    relative level of the step they measure."""
    from mjrl_amd.algos.ppo_clip import PPO
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    z = np.load(os.path.join(GOLDEN, "ppo.npz"))
    policy = MLP(EnvSpec(6, 2, 200, 1), hidden_sizes=(32, 32), seed=3, init_log_std=-0.5)
    np.testing.assert_array_equal(policy.get_param_values(), z["init"])
    ppo = PPO(None, policy, None, clip_coef=0.2, epochs=2, mb_size=64, learn_rate=3e-3, save_logs=True)
    offs = np.concatenate([[0], np.cumsum(z["lengths"])])
    for it in range(2):
        sl = lambda k: [z["%s%d" % (k, it)][offs[i]:offs[i + 1]] for i in range(len(z["lengths"]))]
        paths = [dict(observations=o, actions=a, rewards=r, advantages=v)
                 for o, a, r, v in zip(sl("obs"), sl("act"), sl("rew"), sl("adv"))]
        np.random.seed(int(z["np_seed%d" % it]))
        stats = ppo.train_from_paths(paths)
        np.testing.assert_allclose(stats, z["base_stats%d" % it], rtol=1e-12)
        ref = z["params%d" % it]
        assert np.linalg.norm(policy.get_param_values() - ref) <= 1e-3 * np.linalg.norm(ref), it
        step = np.linalg.norm(ref - (z["init"] if it == 0 else z["params0"]))
        assert abs(ppo.logger.log["kl_dist"][-1] - z["kl_dist%d" % it]) <= 0.05 * abs(z["kl_dist%d" % it]) + 1e-6
        assert abs(ppo.logger.log["surr_improvement"][-1] - z["surr_improvement%d" % it]) <= \
            0.05 * abs(z["surr_improvement%d" % it]) + 1e-5, (it, step)
        np.testing.assert_allclose(ppo.logger.log["running_score"][-1], z["running_score%d" % it], rtol=1e-12)


def test_vectorized_sampler_matches_serial_rollout():
    """sample_paths_vectorized (f3: one mjrl_policy_mean launch per lock-stepped
    step) against base_sampler.do_rollout's serial loop with policy.get_action on
    the CPU (tests/stub_env.py): same trajectory lengths and termination flags,
    observations / actions / rewards to f32 rounding of the mean, and numpy's
    global RNG left where the serial loop leaves it."""
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.samplers.vector_sampler import sample_paths_vectorized
    from mjrl_amd.utils.gym_env import EnvSpec
    from stub_env import StubEnv, serial_rollout
    policy = MLP(EnvSpec(6, 2, 40, 1), hidden_sizes=(48, 32), seed=2, init_log_std=-1.0)
    policy.model.set_transformations(np.full(6, 0.1), np.full(6, 1.5), np.zeros(2), np.full(2, 0.5))
    ref = serial_rollout(13, policy, 1e6, StubEnv, 100)
    after_ref = np.random.rand()
    got = sample_paths_vectorized(13, policy, 1e6, env=StubEnv, pegasus_seed=100, num_envs=5)
    assert np.random.rand() == after_ref
    assert len(got) == 13
    for r, g in zip(ref, got):
        assert g["terminated"] == r["terminated"]
        assert len(g["rewards"]) == len(r["rewards"])
        np.testing.assert_allclose(g["agent_infos"]["mean"], r["mean"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g["observations"], r["observations"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g["actions"], r["actions"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g["rewards"], r["rewards"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g["env_infos"]["norm"], r["norm"], rtol=1e-5, atol=1e-6)
    assert any(r["terminated"] for r in ref) and not all(r["terminated"] for r in ref)


def test_policy_mean_kernel_matches_cpu_forward():
    """mjrl_policy_mean against the CPU MuNet for MLP(64,64) at the Humanoid shape,
    an MLP(128,128) and a linear policy, 1000 rows."""
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.policies.gaussian_linear import LinearPolicy
    from mjrl_amd.samplers.vector_sampler import BatchedPolicy
    from mjrl_amd.utils.gym_env import EnvSpec
    rs = np.random.RandomState(4)
    for pol in (MLP(EnvSpec(376, 17, 10, 1), seed=1), MLP(EnvSpec(17, 6, 10, 1), hidden_sizes=(128, 128), seed=2),
                LinearPolicy(EnvSpec(6, 2, 10, 1), seed=3)):
        th = pol.get_param_values()
        pol.set_param_values(th + 0.1 * rs.randn(th.size).astype(np.float32))
        obs = rs.randn(1000, pol.n) * 2
        bp = BatchedPolicy(pol, "cuda:0")
        with torch.no_grad():
            ref = pol.model(torch.from_numpy(obs).float()).numpy()
        np.testing.assert_allclose(bp.means(obs), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("n", [376, 252, 255])
def test_pack_split_f32_input_matches_f64(n):
    """mjrl_pack_batch_split_f32 (train_step's f32 staging; the 16-byte quad
    kernel when n % 4 == 0) writes the same split rows, row scales and actions
    as the f64-input pack of the same (f32-representable) values."""
    from mjrl_amd.engine import UpdateEngine
    rs = np.random.RandomState(n)
    T, m = 1000, 17
    obs = (rs.randn(T, n) * np.exp(rs.randn(n) * 2)).astype(np.float32)
    act = rs.randn(T, m).astype(np.float32)
    dev = torch.device("cuda:0")
    for tf in (None, (rs.randn(n) * 0.1, rs.rand(n) + 0.5, rs.randn(m), rs.rand(m) + 0.5)):
        outs = []
        for dt in (torch.float64, torch.float32):
            eng = UpdateEngine(n, m, (64, 64), device=dev)
            assert eng.split
            if tf is not None:
                eng.set_transformations(*tf)
            eng._ensure(T, 1)
            o = torch.from_numpy(obs).to(dev, dt)
            a = torch.from_numpy(act).to(dev, dt)
            eng._pack(o, a, T, _lib_stream())
            torch.cuda.synchronize()
            outs.append([eng.ws[k][:T].cpu().clone() for k in ("xs", "xu", "xc", "act32")])
        for x64, x32 in zip(*outs):
            assert torch.equal(x64.view(torch.int16) if x64.dtype == torch.float16 else x64,
                               x32.view(torch.int16) if x32.dtype == torch.float16 else x32)


def _lib_stream():
    from mjrl_amd import _lib
    return _lib.stream_ptr()


@pytest.mark.parametrize("reuse", [False, True])
def test_staged_batch_matches_numpy(reuse):
    """DeviceBatch.from_paths on the GPU: numpy f64 sampler
    paths -> the host convert-and-range pass (AVX-512 streaming path where the CPU
    has it, one native call per chunk of paths) -> pinned slabs -> chunked H2D.
    The staged observations / actions are numpy's f32 cast bit for bit (the
    reference's torch .float() of the concatenation, gaussian_mlp.py:103), rewards,
    offsets and flags exact, the column ranges the f32 min / max; enough paths of
    uneven lengths for many chunks, odd widths for the masked vector tails."""
    from mjrl_amd.engine import DeviceBatch
    rs = np.random.RandomState(7)
    n, m = 45, 7
    lengths = rs.randint(1, 900, size=300)
    paths = [dict(observations=rs.randn(h, n) * np.logspace(-3, 3, n), actions=rs.randn(h, m),
                  rewards=rs.randn(h), terminated=bool(i % 3 == 0)) for i, h in enumerate(lengths)]
    paths[5]["observations"][3, 7] = np.nan
    dev = torch.device("cuda:0")
    for _ in range(2):   # the second call reuses the pinned slabs (and, with reuse, the device slots)
        b = DeviceBatch.from_paths(paths, dev, baseline=None, reuse=reuse)
        torch.cuda.synchronize()
        obs = np.concatenate([p["observations"] for p in paths]).astype(np.float32)
        act = np.concatenate([p["actions"] for p in paths]).astype(np.float32)
        assert np.array_equal(b.obs.cpu().numpy(), obs, equal_nan=True)
        assert np.array_equal(b.act.cpu().numpy(), act)
        assert np.array_equal(b.rewards.cpu().numpy(), np.concatenate([p["rewards"] for p in paths]))
        assert np.array_equal(b.path_off.cpu().numpy(), np.concatenate([[0], np.cumsum(lengths)]))
        assert np.array_equal(b.terminated.cpu().numpy(), np.array([p["terminated"] for p in paths], np.uint8))
        rng = b.obs_range.cpu().numpy()
        np.testing.assert_array_equal(rng[0], np.nanmin(obs, axis=0))
        np.testing.assert_array_equal(rng[1], np.nanmax(obs, axis=0))


