"""GPU tests of the row-kernel path (k_rows + the weight-gradient kernels) on the
shapes the fixtures do not cover: every (hidden, padded action width, padded
observation width) combination of k_wgrad_all's instances and of k_wgrad's
fallbacks, against an fp64 evaluation of the same closed forms (torch float64,
jvp / vjp of the Gaussian-MLP mean).  Row counts are not
multiples of the 32-row tiles, so every slice count / empty-slice / zero-tile
path of the slab layout runs.  Tolerance: 1e-5 norm-relative (the exact-f32
kernels' own error is 1e-7 .. 1e-6 against fp64)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _mu64(theta, X, n, m, h):
    h0, h1 = h
    o = 0

    def take(k, shape):
        nonlocal o
        t = theta[o:o + k].reshape(shape)
        o += k
        return t
    W0 = take(h0 * n, (h0, n)); b0 = take(h0, (h0,))
    W1 = take(h1 * h0, (h1, h0)); b1 = take(h1, (h1,))
    W2 = take(m * h1, (m, h1)); b2 = take(m, (m,))
    return torch.tanh(torch.tanh(X @ W0.T + b0) @ W1.T + b1) @ W2.T + b2


def _truth(obs, act, adv, theta, v, damping, n, m, h):
    """fp64 VPG and F v + damping v at old == new (gaussian_mlp.py:100-140,
    npg_cg.py:55-74)."""
    from torch.func import jvp, vjp
    dev = torch.device("cuda:0")
    X = torch.from_numpy(np.float32(obs).astype(np.float64)).to(dev)
    A = torch.from_numpy(np.float32(act).astype(np.float64)).to(dev)
    adv = torch.from_numpy(np.float32(adv).astype(np.float64)).to(dev)
    th = torch.from_numpy(theta.astype(np.float64)).to(dev)
    vv = torch.from_numpy(v.astype(np.float64)).to(dev)
    T = X.shape[0]
    d_mu = th.numel() - m
    ls = th[d_mu:]
    sig2 = torch.exp(2 * ls)
    f = lambda t: _mu64(t, X, n, m, h)
    mu, back = vjp(f, th[:d_mu])
    z = (A - mu) / torch.exp(ls)
    g_mu = back((adv[:, None] * (A - mu) / sig2) / T)[0]
    g_ls = (adv[:, None] * (z * z - 1)).sum(0) / T
    _, Jv = jvp(f, (th[:d_mu],), (vv[:d_mu],))
    Fm = back((2.0 / (2.0 * sig2 + 1e-8)) * Jv / T)[0]
    c = 4 * sig2 * (2 * sig2 - 1e-8) / (2 * sig2 + 1e-8) ** 2
    return torch.cat([g_mu, g_ls]).cpu().numpy(), (torch.cat([Fm, c * vv[d_mu:]]) + damping * vv).cpu().numpy()


@pytest.mark.parametrize("n,m,h,T", [
    (17, 6, (128, 128), 5001),     # HalfCheetah: k_wgrad_all<128, 16, 2> (two prefetch stages)
    (45, 24, (128, 128), 3333),    # Adroit-like: k_wgrad_all<128, 32, 4>
    (100, 20, (128, 128), 1000),   # k_wgrad_all<128, 32, 8>
    (20, 40, (128, 128), 2049),    # k_wgrad_all<128, 64, 2>
    (70, 40, (128, 128), 777),     # 128-wide, 64 actions, np = 80: the k_wgrad fallback
    (15, 40, (32, 32), 4097),      # k_wgrad_all<32, 64, 2>
    (40, 33, (64, 64), 1500),      # k_wgrad_all<64, 64, 4>
    (39, 28, (256, 256), 2001),    # door: 256-wide layers on k_wgrad
    (17, 6, (128, 128), 31),       # a single partial tile, most slices empty
])
def test_rows_path_vs_fp64(n, m, h, T):
    from mjrl_amd.engine import UpdateEngine
    rs = np.random.RandomState(n * 1000 + T)
    obs, act, adv = rs.randn(T, n), rs.randn(T, m), rs.randn(T)
    d = h[0] * n + h[0] + h[1] * h[0] + h[1] + m * h[1] + m + m
    theta = (rs.randn(d) * 0.1).astype(np.float32)
    theta[-m:] = np.linspace(-1.0, 0.3, m)
    v = (rs.randn(d) * 1e-2).astype(np.float32)
    vpg64, fv64 = _truth(obs, act, adv, theta, v, 1e-4, n, m, h)
    eng = UpdateEngine(n, m, h, device="cuda:0", precision="f32")
    assert eng.accumulate_path() == 0
    eng.load_rows(obs, act, adv)
    g = eng.forward_pass(torch.from_numpy(theta).cuda(), T).cpu().numpy()
    fv = eng.fvp(torch.from_numpy(v).cuda(), damping=1e-4, T=T).cpu().numpy()
    assert nrel(g, vpg64) < 1e-5, nrel(g, vpg64)
    assert nrel(fv, fv64) < 1e-5, nrel(fv, fv64)
    # every block of the flat parameter vector, not just the norm (a missing
    # bias column or a dropped strip would hide in the total)
    offs = np.cumsum([0, h[0] * n, h[0], h[1] * h[0], h[1], m * h[1], m, m])
    for a, b in zip(offs[:-1], offs[1:]):
        assert nrel(g[a:b], vpg64[a:b]) < 1e-4, (a, b, nrel(g[a:b], vpg64[a:b]))
        assert nrel(fv[a:b], fv64[a:b]) < 1e-4, (a, b, nrel(fv[a:b], fv64[a:b]))


@pytest.mark.parametrize("n,m,h,T", [
    (8, 2, (64, 64), 12500),       # Swimmer: every weight image in LDS, one observation chunk
    (8, 2, (64, 64), 64),          # one tile
    (8, 2, (64, 64), 40000),       # more tiles than workgroups
    (17, 6, (32, 32), 9001),       # hidden 32, partial last tile
    (45, 20, (64, 64), 5000),      # MP 32: W1 / W2 images, W0 from L2
    (100, 6, (64, 64), 7777),      # two observation chunks (the gW0 re-stream)
    (150, 20, (32, 32), 4001),     # three chunks, MP 32
])
def test_fused_path_vs_fp64(n, m, h, T):
    """The fused persistent kernel (k_fused: weight images in LDS, W1^T / W2^T read
    transposed from them, the slab staged through LDS) against the same fp64
    closed forms, on each of its layout variants."""
    from mjrl_amd.engine import UpdateEngine
    rs = np.random.RandomState(n * 1000 + T)
    obs, act, adv = rs.randn(T, n), rs.randn(T, m), rs.randn(T)
    d = h[0] * n + h[0] + h[1] * h[0] + h[1] + m * h[1] + m + m
    theta = (rs.randn(d) * 0.1).astype(np.float32)
    theta[-m:] = np.linspace(-1.0, 0.3, m)
    v = (rs.randn(d) * 1e-2).astype(np.float32)
    vpg64, fv64 = _truth(obs, act, adv, theta, v, 1e-4, n, m, h)
    eng = UpdateEngine(n, m, h, device="cuda:0", precision="f32")
    assert eng.accumulate_path() == 1
    eng.load_rows(obs, act, adv)
    g = eng.forward_pass(torch.from_numpy(theta).cuda(), T).cpu().numpy()
    fv = eng.fvp(torch.from_numpy(v).cuda(), damping=1e-4, T=T).cpu().numpy()
    assert nrel(g, vpg64) < 1e-5, nrel(g, vpg64)
    assert nrel(fv, fv64) < 1e-5, nrel(fv, fv64)
    offs = np.cumsum([0, h[0] * n, h[0], h[1] * h[0], h[1], m * h[1], m, m])
    for a, b in zip(offs[:-1], offs[1:]):
        assert nrel(g[a:b], vpg64[a:b]) < 1e-4, (a, b, nrel(g[a:b], vpg64[a:b]))
        assert nrel(fv[a:b], fv64[a:b]) < 1e-4, (a, b, nrel(fv[a:b], fv64[a:b]))
