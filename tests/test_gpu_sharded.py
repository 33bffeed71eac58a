"""The sharded update path on one GPU, through RCCL driven directly
(comm.RcclComm): a one-rank communicator forced onto the sharded schedule runs
exactly what every rank of an N-GPU run executes — the moment records through
ncclAllGather + mjrl_moments_combine, an ncclAllReduce of the VPG sum and of
every FVP sum between the gather and the CG step (mjrl_cg_step1), the surr /
KL sums — and the whole update captured into ONE hipGraph with the RCCL calls
inside (npg_cg.py:84-144, cg_solve.py:3-22 sharded over paths).  RCCL refuses
two ranks on one GPU, so the N-rank exchange itself is rehearsed over gloo
(test_gpu_dist.py, test_dist_gloo.py); here: the device kernels of the sharded
schedule against the unsharded path, the reference, and graph replay against
eager, bit for bit."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _case(name):
    from oracle import npg_cpu as O
    return O.load_case(os.path.join(GOLDEN, name + ".npz"))


def _batch(c):
    from mjrl_amd.engine import DeviceBatch
    obs, act, T_demo = c["obs64"], c["act64"], 0
    if "demo_obs" in c:
        obs = np.concatenate([obs, c["demo_obs"].astype(np.float64)])
        act = np.concatenate([act, c["demo_act"].astype(np.float64)])
        T_demo = c["demo_obs"].shape[0]
    offs = np.concatenate([[0], np.cumsum(c["lengths"])])
    return DeviceBatch(_t(obs), _t(act), _t(c["rewards"]), _t(c["baseline"]), _t(offs),
                       _t(c["terminated"].astype(np.uint8)), T_demo=T_demo)


def _args(c):
    from oracle import npg_cpu as O
    kw = O.case_kwargs(c)
    args = dict(algo=kw["algo"], gamma=float(c["gamma"]), gae_lambda=float(c["gae_lambda"]), trpo_verbose=False)
    if kw["algo"] == "npg":
        args["n_step_size"] = kw.get("n_step_size", 0.01)
    else:
        args["kl_dist"] = kw["kl_dist"]
    if kw["algo"] == "dapg":
        args["demo_coef"] = kw["demo_coef"]
    return args


def _engine(c, comm):
    from mjrl_amd.engine import UpdateEngine
    eng = UpdateEngine(int(c["n"]), int(c["m"]), c["hidden_t"], device=DEV, comm=comm)
    if c["transforms"] is not None:
        eng.set_transformations(*c["transforms"])
    return eng


@pytest.fixture(scope="module")
def rccl():
    from mjrl_amd.comm import RcclComm
    comm = RcclComm.local(DEV)
    yield comm
    comm.close()


def test_rccl_comm_ops(rccl):
    """One-rank RCCL collectives are identities / copies, on the current stream,
    eager and inside a captured graph."""
    x = torch.arange(10, dtype=torch.float32, device=DEV)
    ref = x.clone()
    rccl.allreduce_sum(x)
    rccl.allreduce_max(x)
    rccl.broadcast(x)
    g = torch.zeros(10, dtype=torch.float32, device=DEV)
    rccl.allgather(x, g)
    torch.cuda.synchronize()
    assert torch.equal(x, ref) and torch.equal(g, ref)
    d = torch.arange(6, dtype=torch.float64, device=DEV)
    out = torch.zeros(6, dtype=torch.float64, device=DEV)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        rccl.allreduce_sum(d)
        rccl.allgather(d, out)
    d.copy_(torch.arange(6, dtype=torch.float64, device=DEV) * 3)
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, torch.arange(6, dtype=torch.float64, device=DEV) * 3)


def test_moments_combine_kernel():
    """mjrl_moments_combine against its restatement (oracle.moments_combine) over
    three shards, one of them empty (a rank with no paths)."""
    import ctypes as C
    from mjrl_amd import _lib
    from oracle import npg_cpu as O
    rs = np.random.RandomState(0)
    shards = [rs.standard_normal(1000) * 5 + 2, np.zeros(0), rs.standard_normal(77) - 40]
    recs = np.stack([np.concatenate([O.moments_record(s), O.moments_record(s * 0.5)]) for s in shards])
    g = _t(recs.ravel())
    out = torch.zeros(32, dtype=torch.float64, device=DEV)
    L = _lib.lib()
    _lib.check(L.mjrl_moments_combine(_lib.ptr(g), 3, 32, 2, _lib.ptr(out), _lib.stream_ptr()), "combine")
    o = out.cpu().numpy()
    for j in range(2):
        ref = O.moments_combine(recs[:, 16 * j:16 * j + 16])
        np.testing.assert_allclose(o[16 * j:16 * j + 6], ref[0:6], rtol=1e-15)
        np.testing.assert_allclose(o[16 * j + 8:16 * j + 14], ref[8:14], rtol=1e-13)
    x = np.concatenate(shards)
    np.testing.assert_allclose(np.sqrt(o[9] / o[2]), np.std(x), rtol=1e-12)


@pytest.mark.parametrize("transforms", [False, True])
def test_colscale_range_matches_device_colmax(transforms):
    """Column scales from the host staging pass's ranges (mjrl_obs_colscale_range)
    equal the device column-max pass's (mjrl_obs_colscale_f32) bit for bit."""
    import ctypes as C
    from mjrl_amd import _lib
    from mjrl_amd.engine import host_stage
    rs = np.random.RandomState(7)
    n, T = 376, 5000
    obs = (rs.standard_normal((T, n)) * np.logspace(-6, 3, n)).astype(np.float32)
    obs[:, 11] = 0.0                                   # an all-zero column
    obs[:, 12] = 2.0 ** -20                            # a constant power-of-two column
    s = _lib.make_shape(n, 17, 64, 64)
    ins = isc = None
    if transforms:
        ins = _t((rs.standard_normal(n) * 0.1).astype(np.float32))
        sc = rs.uniform(0.5, 3.0, n).astype(np.float32)
        sc[3] = -1.7                                   # a negative scale: decreasing map
        isc = _t(sc)
    lo, hi = np.full(n, np.inf, np.float32), np.full(n, -np.inf, np.float32)
    view = np.empty_like(obs)
    host_stage([obs[:2000], obs[2000:]], view, np.array([0, 2000, T]), 0, 2, lo, hi)
    L = _lib.lib()
    xa = torch.zeros(s.np, dtype=torch.float32, device=DEV)
    xb = torch.zeros(s.np, dtype=torch.float32, device=DEV)
    st = _lib.stream_ptr()
    od, lod, hid = _t(obs), _t(lo), _t(hi)   # held: a freed temporary's block is reused by the next one
    _lib.check(L.mjrl_obs_colscale_f32(_lib.ptr(od), T, C.byref(s), _lib.ptr(ins), _lib.ptr(isc),
                                       _lib.ptr(xa), st), "colscale")
    _lib.check(L.mjrl_obs_colscale_range(_lib.ptr(lod), _lib.ptr(hid), C.byref(s), _lib.ptr(ins),
                                         _lib.ptr(isc), _lib.ptr(xb), st), "colscale_range")
    a, b = xa.cpu().numpy(), xb.cpu().numpy()
    bad = np.nonzero(a != b)[0]
    assert len(bad) == 0, [(int(k), float(a[k]), float(b[k]), float(lo[k]) if k < n else None,
                            float(hi[k]) if k < n else None, float(np.abs(obs[:, k]).max()) if k < n else None)
                           for k in bad[:8]]


@pytest.mark.parametrize("name", ["c4_humanoid", "c2_ragged", "c5_door_dapg", "c3_halfcheetah_trpo"])
def test_sharded_path_one_rank(rccl, name):
    """The sharded schedule on a one-rank RCCL communicator gives the one-process
    schedule's results bit for bit (mjrl_moments_combine is exact at one rank, and
    the CG iteration after the all-reduce — mjrl_cg_z, mjrl_cg_step_xr_p — is the
    fused gather's arithmetic), within the reference tolerance."""
    from mjrl_amd.comm import LocalComm
    c = _case(name)
    th0 = _t(c["theta0"].astype(np.float32))
    res, th = {}, {}
    for key, comm in (("local", LocalComm()), ("sharded", rccl)):
        eng = _engine(c, comm)
        eng.graphs = False
        res[key] = eng.update(_batch(c), th0, **_args(c))
        th[key] = eng.vec["theta_new"].cpu().numpy()
    assert res["sharded"]["base_stats"] == res["local"]["base_stats"]
    assert res["sharded"]["surr_before"] == res["local"]["surr_before"]
    assert np.array_equal(th["sharded"], th["local"])
    assert res["sharded"]["kl_dist"] == res["local"]["kl_dist"] and res["sharded"]["alpha"] == res["local"]["alpha"]
    tol = max(1e-3, 3 * float(c["spread_theta"]))
    assert np.linalg.norm(th["sharded"] - c["theta1"]) / np.linalg.norm(c["theta1"]) < tol


@pytest.mark.parametrize("name", ["c4_humanoid", "c5_door_dapg"])
def test_sharded_graph_replay_is_bit_identical(rccl, name):
    """The sharded update captured as one hipGraph (RCCL collectives inside) and
    replayed gives the eager sharded update's parameters and statistics bit for
    bit."""
    c = _case(name)
    th0 = _t(c["theta0"].astype(np.float32))
    eng = _engine(c, rccl)
    eng.graphs = True
    b = _batch(c)
    args = _args(c)
    r_eager = eng.update(b, th0, **args)             # eager (first sighting)
    th_eager = eng.vec["theta_new"].cpu().numpy()
    eng.update(b, th0, **args)                       # eager, then captured
    assert eng._gstate.get("graph") is not None, "sharded update was not captured"
    for _ in range(2):
        r = eng.update(b, th0, **args)               # replays
        assert np.array_equal(eng.vec["theta_new"].cpu().numpy(), th_eager)
        assert r["base_stats"] == r_eager["base_stats"]
        assert r["kl_dist"] == r_eager["kl_dist"] and r["alpha"] == r_eager["alpha"]


@pytest.fixture(scope="module")
def torch_nccl():
    """A one-rank torch.distributed group on the nccl (= RCCL) backend in this
    process: the fallback comm of an N-GPU run (MJRL_AMD_COMM=torch: torch's own
    collectives, eager)."""
    import socket
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=DEV)
    try:
        yield dist
    finally:
        from mjrl_amd.comm import release_comms
        release_comms()
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["c4_humanoid", "c3_halfcheetah_trpo"])
def test_sharded_path_torch_collectives_eager(torch_nccl, monkeypatch, name):
    """The escape hatch if the captured RCCL path misbehaves at N > 1:
    MJRL_AMD_COMM=torch selects torch.distributed's collectives on the nccl group
    (comm.DistComm), the sharded schedule runs eager (graphs off), and the update
    equals the one-process update bit for bit."""
    from mjrl_amd.comm import DistComm, LocalComm, _group_comm
    monkeypatch.setenv("MJRL_AMD_COMM", "torch")
    comm = _group_comm()
    assert type(comm) is DistComm and torch_nccl.get_backend() == "nccl"
    comm = DistComm(force_sharded=True)
    c = _case(name)
    th0 = _t(c["theta0"].astype(np.float32))
    res, th = {}, {}
    for key, cm in (("local", LocalComm()), ("torch", comm)):
        eng = _engine(c, cm)
        eng.graphs = False
        res[key] = eng.update(_batch(c), th0, **_args(c))
        th[key] = eng.vec["theta_new"].cpu().numpy()
    assert np.array_equal(th["torch"], th["local"])
    assert res["torch"]["base_stats"] == res["local"]["base_stats"]
    assert res["torch"]["kl_dist"] == res["local"]["kl_dist"] and res["torch"]["alpha"] == res["local"]["alpha"]


def test_rccl_cache_rebuilds_for_a_new_group(torch_nccl, monkeypatch):
    """comm._group_comm's cached RcclComm belongs to the live group: the same
    object while the group lives, a new one for another group object."""
    from mjrl_amd.comm import RcclComm, _group_comm
    monkeypatch.setenv("MJRL_AMD_COMM", "rccl")
    a = _group_comm()
    assert isinstance(a, RcclComm) and _group_comm() is a
    g2 = torch_nccl.new_group([0])
    b = _group_comm(g2)
    assert b is not a and _group_comm(g2) is b


@pytest.mark.parametrize("name", ["c3_trpo_backtrack", "c3_halfcheetah_trpo"])
@pytest.mark.parametrize("graph", [False, True])
def test_trpo_device_line_search_equals_host(name, graph):
    """The device line search (mjrl_trpo_trial + mjrl_policy_eval_if: the first
    trials tested and stepped on the device, no host round trip per trial) against
    the host loop (trpo_device_trials = 0): the same trials (alpha, kl, surr), the
    same parameters and statistics, bit for bit. The full step is evaluated in
    the launch and K device trials follow it, so with K = 1 the backtracking case
    (3 trials) also exercises the host continuation past them."""
    from mjrl_amd.comm import LocalComm
    c = _case(name)
    th0 = _t(c["theta0"].astype(np.float32))
    out = {}
    for K in (0, 1, 2, 4):
        eng = _engine(c, LocalComm())
        eng.trpo_device_trials = K
        eng.graphs = graph
        b = _batch(c)
        for _ in range(3 if graph else 1):   # graph: eager, capture, replay
            r = eng.update(b, th0, **_args(c))
        out[K] = (r, eng.vec["theta_new"].cpu().numpy())
    r0, th_0 = out[0]
    for K in (1, 2, 4):
        r, th = out[K]
        assert r["trials"] == r0["trials"], (K, r["trials"], r0["trials"])
        assert np.array_equal(th, th_0)
        assert r["alpha"] == r0["alpha"] and r["kl_dist"] == r0["kl_dist"] and r["surr_after"] == r0["surr_after"]
    if name == "c3_trpo_backtrack":
        assert len(r0["trials"]) > 2   # past the K = 1 device sequence
