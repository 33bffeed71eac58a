"""GPU tests of the batch assembly fused into the forward pass
(mjrl_policy_vpg_pack, k_kx<.., FWD, true>; engine.FUSED_PACK): the split rows it
writes are the pack's bit for bit (mjrl_pack_batch_split_f32), and a whole update
through it (NPG and TRPO, graph replay included, ragged batches whose row count is
not a multiple of the 32-row tile) gives bit-identical parameters, statistics and
caches to the update with the separate pack.  Batches with an input
normalisation, f64 staging or demo rows outside the forward pass keep the pack."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, M, H = 376, 17, (64, 64)


def _batch(rs, lengths, dtype=np.float32, demos=(), N=N):
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.engine import DeviceBatch
    from mjrl_amd.utils.gym_env import EnvSpec
    scales = 10.0 ** rs.uniform(-4, 2, size=N)
    paths = []
    for h in lengths:
        o = rs.randn(h, N) * scales
        o[:, :3] = 0.0
        paths.append(dict(observations=o, actions=rs.randn(h, M), rewards=rs.randn(h), terminated=bool(h % 2)))
    demo_paths = [dict(observations=rs.randn(h, N) * scales, actions=rs.randn(h, M)) for h in demos]
    base = LinearBaseline(EnvSpec(N, M, max(lengths), 1))
    base._coeffs = rs.randn(N + 4) * 0.01
    return DeviceBatch.from_paths(paths, torch.device("cuda:0"), baseline=base, obs_dtype=dtype,
                                  demo_paths=demo_paths or None), paths


def _run(fused, batch, theta, algo, graph, N=N):
    from mjrl_amd import engine as E
    old = E.FUSED_PACK
    E.FUSED_PACK = fused
    try:
        eng = E.UpdateEngine(N, M, H, device="cuda:0", precision="split")
        eng.graphs = graph
        kw = dict(algo=algo, gamma=0.995, gae_lambda=0.97, cg_iters=10, damping=1e-4, trpo_verbose=False)
        kw.update(dict(n_step_size=0.01) if algo == "npg" else dict(kl_dist=0.01))
        if algo == "dapg":
            kw["demo_coef"] = 0.1
        outs = []
        for _ in range(3 if graph else 1):          # graph: capture, then replays
            out = eng.update(batch, theta, **kw)
            torch.cuda.synchronize()
            outs.append((out, eng.vec["theta_new"].clone()))
        T = batch.T + batch.T_demo
        ws = {k: eng.ws[k][:T].clone() for k in ("xs", "xu", "mu0", "ll0", "a0", "a1")}
        return outs, ws, eng._fused_pack(batch, T, T if algo == "dapg" else batch.T)
    finally:
        E.FUSED_PACK = old


def _same(a, b):
    return np.array_equal(np.atleast_1d(np.asarray(a)).view(np.uint8), np.atleast_1d(np.asarray(b)).view(np.uint8))


@pytest.mark.parametrize("algo,graph,lengths,demos", [
    ("npg", False, (1000, 999, 1, 37, 500), ()),        # 2537 rows: a partial last tile
    ("npg", True, (64,) * 40, ()),
    ("trpo", False, (700, 333, 1000), ()),
    ("dapg", False, (600, 411), (200, 77)),             # demo rows behind the RL rows, in the forward pass
])
def test_fused_pack_update_is_bit_identical(algo, graph, lengths, demos):
    rs = np.random.RandomState(len(lengths))
    batch, _ = _batch(rs, lengths, demos=demos)
    theta = torch.from_numpy((rs.randn(29410) * 0.05).astype(np.float32)).cuda()
    (o1, ws1, f1), (o0, ws0, f0) = _run(True, batch, theta, algo, graph), _run(False, batch, theta, algo, graph)
    assert f1 and not f0
    for k in ws1:
        assert torch.equal(ws1[k].contiguous().view(torch.uint8), ws0[k].contiguous().view(torch.uint8)), k
    for (a, ta), (b, tb) in zip(o1, o0):
        assert torch.equal(ta, tb)
        for k in ("alpha", "gx", "delta", "surr_before", "surr_after", "kl_dist", "base_stats", "cg_iters",
                  "trials"):
            assert _same(np.asarray(a[k], np.float64), np.asarray(b[k], np.float64)), k


@pytest.mark.parametrize("N", [N, 252, 120])   # 384 / 256 / 128 split columns (KG 12 / 8 / 4)
def test_fused_pack_rows_equal_the_pack(N):
    """xs / xu written by the fused forward pass equal mjrl_pack_batch_split_f32's
    (the all-zero leading columns and the bias column included); a batch with an
    input normalisation, or staged in f64, takes the separate pack."""
    from mjrl_amd import engine as E
    rs = np.random.RandomState(7)
    batch, _ = _batch(rs, (300, 5, 411), N=N)
    T = batch.T
    d = E.UpdateEngine(N, M, H, device="cuda:0", precision="split").shape.d
    theta = torch.from_numpy((rs.randn(d) * 0.05).astype(np.float32)).cuda()
    _, ws1, f1 = _run(True, batch, theta, "npg", False, N=N)
    eng = E.UpdateEngine(N, M, H, device="cuda:0", precision="split")
    eng._ensure(T, batch.P)
    from mjrl_amd import _lib
    st = _lib.stream_ptr()
    eng._pack(batch.obs, batch.act, T, st, batch.obs_range)
    torch.cuda.synchronize()
    assert f1
    assert torch.equal(ws1["xs"].view(torch.int16), eng.ws["xs"][:T].view(torch.int16))
    assert torch.equal(ws1["xu"], eng.ws["xu"][:T])
    # not fused: an input normalisation; f64 observations
    eng.set_transformations(rs.randn(N), np.abs(rs.randn(N)) + 0.5)
    assert not eng._fused_pack(batch, T, T)
    b64, _ = _batch(rs, (100, 20), dtype=np.float64, N=N)
    eng2 = E.UpdateEngine(N, M, H, device="cuda:0", precision="split")
    assert not eng2._fused_pack(b64, b64.T, b64.T)
