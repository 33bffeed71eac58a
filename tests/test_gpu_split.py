"""GPU tests of the split-f16 first layer (precision='split').

  - the packed rows: (hi + lo) * xu * xc reproduces the f32 xhat of
    mjrl_pack_batch element by element to 2^-23 |xhat| + 2^-38 of the column's
    max, on rows with columns spanning 10^-6 .. 10^3 and with the input
    normalisation;
  - accuracy against fp64 truth: the VPG, the Fisher-vector product and the
    post-step surrogate / KL of the split kernels are compared with an fp64
    evaluation of the same closed forms (torch float64 on the GPU, jvp / vjp of
    the Gaussian-MLP mean) and must be within 1e-6 norm-relative and within 4x
    of the exact-f32 kernels' own error — the split path is an f32-accuracy
    path, not a reduced-precision one.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, M, H = 376, 17, (64, 64)


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _obs(T, rs):
    scales = 10.0 ** rs.uniform(-6, 3, size=N)
    obs = rs.randn(T, N) * scales
    obs[:, :5] = 0.0                     # always-zero columns (Humanoid's cfrc_ext)
    obs[7, :] = 0.0                      # an all-zero row: only the bias column
    return obs


def test_pack_split_roundtrip():
    """The split rows carry the f32 xhat of mjrl_pack_batch to the element bound of
    common.h: |xc xu (hi + lo) - xhat| <= 2^-23 |xhat| + 2^-38 colmax_k, with xc a
    power of two per column (colmax / xc in [1/2, 1)) and xu one per row (the row's
    max |xhat / xc| / xu in [2^14, 2^15))."""
    from mjrl_amd import _lib
    from mjrl_amd.engine import UpdateEngine
    rs = np.random.RandomState(0)
    T = 3000
    obs, act = _obs(T, rs), rs.randn(T, M)
    for transforms in (None, (rs.randn(N) * 5, np.abs(rs.randn(N)) * 10 + 0.1)):
        ef = UpdateEngine(N, M, H, device="cuda:0", precision="f32")
        es = UpdateEngine(N, M, H, device="cuda:0", precision="split")
        for e in (ef, es):
            if transforms is not None:
                e.set_transformations(transforms[0], transforms[1])
            e.load_rows(obs, act)
        x = ef.ws["xhat"][:T].double().cpu().numpy()
        xs = es.ws["xs"][:T].float().double().cpu().numpy()
        xu = es.ws["xu"][:T].double().cpu().numpy()
        xc = es.ws["xc"].double().cpu().numpy()
        np_ = ef.shape.np
        pow2 = lambda a: np.all(np.log2(a) == np.round(np.log2(a)))
        assert pow2(xu) and pow2(xc)
        colmax = np.abs(x).max(0)
        nz = colmax > 0
        assert np.all(colmax[nz] < xc[nz]) and np.all(colmax[nz] >= xc[nz] / 2) and np.all(xc[~nz] == 1)
        assert colmax[N] == 1.0 and xc[N] == 2.0          # the bias column
        y = x / xc[None, :]
        assert np.all(np.abs(y).max(1) / xu >= 2.0 ** 14) and np.all(np.abs(y).max(1) / xu < 2.0 ** 15)
        rec = (xs[:, :np_] + xs[:, np_:]) * xu[:, None] * xc[None, :]
        err = np.abs(rec - x)
        bound = 2.0 ** -23 * np.abs(x) + 2.0 ** -38 * colmax[None, :]
        assert np.all(err <= bound), (err / np.maximum(bound, 1e-300)).max()
        # a [1/2, 1) row block (the round-2 form) breaks that bound on these rows
        assert np.abs(x).max() / np.abs(x[x != 0]).min() > 2.0 ** 30
        assert np.array_equal(es.ws["act32"][:T].cpu().numpy(), ef.ws["act32"][:T].cpu().numpy())
        _lib.load()


def _mu64(theta, X):
    h0, h1 = H
    o = 0

    def take(k, shape):
        nonlocal o
        t = theta[o:o + k].reshape(shape)
        o += k
        return t
    W0 = take(h0 * N, (h0, N)); b0 = take(h0, (h0,))
    W1 = take(h1 * h0, (h1, h0)); b1 = take(h1, (h1,))
    W2 = take(M * h1, (M, h1)); b2 = take(M, (M,))
    return torch.tanh(torch.tanh(X @ W0.T + b0) @ W1.T + b1) @ W2.T + b2


def _truth(obs, act, adv, theta, v, damping):
    """fp64 VPG and F v + damping v (closed forms of SURVEY.md appendix A)."""
    from torch.func import jvp, vjp
    dev = torch.device("cuda:0")
    X = torch.from_numpy(np.float32(obs).astype(np.float64)).to(dev)
    A = torch.from_numpy(np.float32(act).astype(np.float64)).to(dev)
    adv = torch.from_numpy(np.float32(adv).astype(np.float64)).to(dev)
    th = torch.from_numpy(theta.astype(np.float64)).to(dev)
    vv = torch.from_numpy(v.astype(np.float64)).to(dev)
    T = X.shape[0]
    d_mu = th.numel() - M
    ls = th[d_mu:]
    sig2 = torch.exp(2 * ls)
    f = lambda t: _mu64(t, X)
    mu, back = vjp(f, th[:d_mu])
    z = (A - mu) / torch.exp(ls)
    g_mu = back((adv[:, None] * (A - mu) / sig2) / T)[0]
    g_ls = (adv[:, None] * (z * z - 1)).sum(0) / T
    vpg = torch.cat([g_mu, g_ls])
    _, Jv = jvp(f, (th[:d_mu],), (vv[:d_mu],))
    wgt = 2.0 / (2.0 * sig2 + 1e-8)
    Fm = back(wgt * Jv / T)[0]
    c = 4 * sig2 * (2 * sig2 - 1e-8) / (2 * sig2 + 1e-8) ** 2
    Fv = torch.cat([Fm, c * vv[d_mu:]]) + damping * vv
    return vpg.cpu().numpy(), Fv.cpu().numpy()


@pytest.mark.parametrize("T", [40000])
def test_split_accuracy_vs_fp64(T):
    from mjrl_amd.engine import UpdateEngine
    rs = np.random.RandomState(1)
    obs, act, adv = _obs(T, rs) / 50.0, rs.randn(T, M), rs.randn(T)
    theta = (rs.randn(29410) * 0.05).astype(np.float32)
    theta[-M:] = np.linspace(-1.5, 0.5, M)
    v = (rs.randn(29410) * 1e-3).astype(np.float32)
    vpg64, fv64 = _truth(obs, act, adv, theta, v, 1e-4)
    errs = {}
    for prec in ("f32", "split"):
        eng = UpdateEngine(N, M, H, device="cuda:0", precision=prec)
        eng.load_rows(obs, act, adv)
        th = torch.from_numpy(theta).cuda()
        g = eng.forward_pass(th, T).cpu().numpy()
        fv = eng.fvp(torch.from_numpy(v).cuda(), damping=1e-4, T=T).cpu().numpy()
        errs[prec] = (nrel(g, vpg64), nrel(fv, fv64))
    for i, what in enumerate(("vpg", "fvp")):
        e32, esp = errs["f32"][i], errs["split"][i]
        assert esp < 1e-6, (what, errs)
        assert esp < 4 * e32 + 2e-8, (what, errs)


def test_split_eval_matches_f32():
    """Post-step surrogate / KL (the EVAL pass) on both precisions."""
    from mjrl_amd.engine import UpdateEngine
    rs = np.random.RandomState(2)
    T = 20000
    obs, act, adv = rs.randn(T, N), rs.randn(T, M), rs.randn(T)
    theta = (rs.randn(29410) * 0.05).astype(np.float32)
    theta1 = theta + (rs.randn(29410) * 1e-3).astype(np.float32)
    out = {}
    for prec in ("f32", "split"):
        eng = UpdateEngine(N, M, H, device="cuda:0", precision=prec)
        eng.load_rows(obs, act, adv)
        eng.forward_pass(torch.from_numpy(theta).cuda(), T)
        out[prec] = eng.eval_pass(torch.from_numpy(theta1).cuda(), T)
    np.testing.assert_allclose(out["split"][0], out["f32"][0], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(out["split"][1], out["f32"][1], rtol=1e-4, atol=1e-9)


def test_split_accuracy_vs_fp64_bench_workload():
    """The bench's own workload (Humanoid shape, 1,000 paths x 1,000 steps, the
    same seeded synthetic obs / act and the same initial parameters as bench.py):
    VPG and F v of the split-f16 kernels against fp64 truth at the full 1M rows,
    beside the exact-f32 kernels' error on the same data."""
    import bench
    from mjrl_amd.engine import UpdateEngine
    obs, act, _ = bench.make_paths(0, bench.N_PATHS)
    obs = np.concatenate(obs)
    act = np.concatenate(act)
    T = obs.shape[0]
    assert T == 1_000_000
    rs = np.random.RandomState(3)
    adv = rs.randn(T)
    theta = bench.initial_theta()
    v = (rs.randn(theta.size) * 1e-3).astype(np.float32)
    vpg64, fv64 = _truth(obs, act, adv, theta, v, 1e-4)
    errs = {}
    for prec in ("f32", "split"):
        eng = UpdateEngine(N, M, H, device="cuda:0", precision=prec)
        eng.load_rows(obs, act, adv)
        g = eng.forward_pass(torch.from_numpy(theta).cuda(), T).cpu().numpy()
        fv = eng.fvp(torch.from_numpy(v).cuda(), damping=1e-4, T=T).cpu().numpy()
        errs[prec] = (nrel(g, vpg64), nrel(fv, fv64))
        del eng
        torch.cuda.empty_cache()
    print("1M split vs fp64:", errs)
    for i, what in enumerate(("vpg", "fvp")):
        e32, esp = errs["f32"][i], errs["split"][i]
        assert esp < 1e-6, (what, errs)
        assert esp < 4 * e32 + 2e-8, (what, errs)
