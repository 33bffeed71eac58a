"""train_step orchestration (mjrl/algos/batch_reinforce.py:58-103) on CPU.

The device update is replaced by a stand-in (this container has no GPU; the GPU
version of these checks is tests/test_gpu_train_step.py); everything around it
is the product code: the sampler calls, `seed += N`, the returned
[mean, std, min, max, N], the DataLog keys, the baseline fit — and, on two gloo
ranks, the rank-aware sampling (each rank draws its ceil(N / world) share with
the pegasus seed offset of that share, trajectory_sampler.py:37-45) and the
baseline fitted on the union of the shards.  Samplers: tests/stub_samplers.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import stub_samplers

N_OBS, N_ACT = 5, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Env:
    env_id = "stub-v0"


class _CountingBaseline:
    """A baseline with no sharded fit of its own: fit must see the union."""

    def __init__(self):
        self.seen = None

    def predict(self, path):
        return np.zeros(len(path["rewards"]))

    def fit(self, paths, return_errors=False):
        self.seen = sorted(round(float(p["rewards"][0]), 12) for p in paths)
        if return_errors:
            return 1.0, 0.5


def _stub_update(self, paths, gamma, gae_lambda):
    """Stand-in for the device update (train_from_samples): returns per path, then
    the reference's base_stats over ALL ranks' paths (npg_cg.py:97-102)."""
    from oracle import npg_cpu as O
    for p in paths:
        p["returns"] = O.discount_sum(p["rewards"], gamma)
        p["baseline"] = np.zeros(len(p["rewards"]))
    pr = [float(np.sum(p["rewards"])) for p in paths]
    comm = self.comm()
    if comm.world_size > 1:
        import torch.distributed as dist
        parts = [None] * comm.world_size
        dist.all_gather_object(parts, pr)
        pr = [v for part in parts for v in part]
    self._stub_paths = paths
    return [np.mean(pr), np.std(pr), np.amin(pr), np.amax(pr)]


def _agent(baseline_kind, comm=None):
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.baselines.quadratic_baseline import QuadraticBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(N_OBS, N_ACT, 100, 1)
    pol = MLP(spec, hidden_sizes=(32, 32), seed=0)
    base = {"linear": lambda: LinearBaseline(spec), "quadratic": lambda: QuadraticBaseline(spec),
            "other": _CountingBaseline}[baseline_kind]()
    agent = NPG(_Env(), pol, base, seed=1000, save_logs=True, comm=comm)
    agent.train_from_samples = _stub_update.__get__(agent)
    return agent


def _run_steps(agent, N, mode, num_cpu=1):
    stub_samplers.install()
    out = []
    for _ in range(2):
        stats = agent.train_step(N, sample_mode=mode, gamma=0.99, gae_lambda=0.95, num_cpu=num_cpu)
        seeds = [round(float(p["rewards"][0]), 12) for p in agent._stub_paths]
        coeffs = getattr(agent.baseline, "_coeffs", None)
        out.append(dict(stats=stats, seed=agent.seed, first=seeds, coeffs=None if coeffs is None else coeffs.copy(),
                        seen=getattr(agent.baseline, "seen", None), calls=list(stub_samplers.CALLS),
                        log={k: list(v) for k, v in agent.logger.log.items()}))
        stub_samplers.CALLS.clear()
    return out


def _worker(rank, world, port, kind, N, mode, q, num_cpu=1):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mjrl_amd.comm import DistComm
        q.put((rank, _run_steps(_agent(kind, DistComm()), N, mode, num_cpu)))
    finally:
        dist.destroy_process_group()


def _sharded(kind, N, mode, world=2, num_cpu=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, N, mode, q, num_cpu)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=300)
        out[r] = v
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_train_step_single_process():
    agent = _agent("quadratic")
    res = _run_steps(agent, 6, "trajectories")
    for it, r in enumerate(res):
        assert r["seed"] == 1000 + 6 * (it + 1)                       # seed += N (batch_reinforce.py:84)
        assert len(r["stats"]) == 5 and r["stats"][4] == 6             # [mean, std, min, max, N]
        assert r["calls"] == [("trajectories", 6, 1000 + 6 * it, 1)]
        assert r["coeffs"] is not None
    log = res[-1]["log"]
    for k in ("time_sampling", "time_VF", "VF_error_before", "VF_error_after"):
        assert len(log[k]) == 2, k


@pytest.mark.parametrize("kind", ["linear", "quadratic", "other"])
def test_train_step_sharded_two_ranks(kind):
    N = 7   # ceil(7 / 2) = 4 paths on rank 0 (seed + 0), 3 on rank 1 (seed + 4)
    single = _run_steps(_agent(kind), N, "trajectories")
    out = _sharded(kind, N, "trajectories")
    for it in range(2):
        s = single[it]
        r0, r1 = out[0][it], out[1][it]
        base = 1000 + N * it
        assert r0["calls"] == [("trajectories", 4, base, 1)]
        assert r1["calls"] == [("trajectories", 3, base + 4, 1)]
        assert r0["first"] + r1["first"] == s["first"]                 # the same N paths, split
        assert r0["seed"] == r1["seed"] == s["seed"] == base + N
        np.testing.assert_allclose(r0["stats"], s["stats"], rtol=1e-12)
        assert r0["stats"] == r1["stats"] and r0["stats"][4] == N
        if kind == "other":
            assert r0["seen"] == r1["seen"] == s["seen"]               # fitted on the union
        else:
            np.testing.assert_array_equal(r0["coeffs"], r1["coeffs"])
            np.testing.assert_allclose(r0["coeffs"], s["coeffs"], rtol=1e-6, atol=1e-9)
        for k in ("time_sampling", "time_VF", "VF_error_before", "VF_error_after"):
            assert len(r0["log"][k]) == it + 1
        np.testing.assert_allclose(r0["log"]["VF_error_after"], s["log"]["VF_error_after"], rtol=1e-6)


def test_train_step_sharded_samples_mode():
    N = 250
    out = _sharded("linear", N, "samples")
    starts = []
    for it in range(2):
        base = 1000 + N * it
        assert out[0][it]["calls"] == [("samples", 125, base, 1)]
        assert out[1][it]["calls"] == [("samples", 125, base + 125, 1)]   # rank 1's slot of the window
        assert out[0][it]["seed"] == base + N
        starts += [out[r][it]["calls"][0][2] for r in range(2)]
    # no rank starts where any rank started before (the next iteration's rank 0 vs
    # this one's rank 1 included): no two shards replay the same env resets
    assert len(set(starts)) == len(starts), starts


def test_train_step_sharded_samples_mode_multicore():
    """num_cpu > 1: the reference's multi-core loop advances its seed cumulatively
    (batch_sampler.py:45), so the ranks' calls are interleaved instead
    (BatchREINFORCE._sample_calls): call k of rank r at seed + (2k + r) w, w = 2 x
    ceil(5 / 2) = 6 seeds per call on two cores; every rank draws more than its
    n_r = 125 steps, and no env reset is replayed by two ranks in one batch."""
    N = 250
    out = _sharded("linear", N, "samples", num_cpu=2)
    for it in range(2):
        base = 1000 + N * it
        seeds = {}
        for r in range(2):
            calls = out[r][it]["calls"]
            assert all(c[0] == "trajectories" and c[1] == 5 and c[3] == 2 for c in calls)
            assert [c[2] for c in calls] == [base + (2 * k + r) * 6 for k in range(len(calls))]
            seeds[r] = {c[2] + i for c in calls for i in range(5)}
            # the loop stops on the first call that takes the rank past n_r steps
            h = [min(stub_samplers.HORIZON - (s % 7), 1e6) for s in sorted(seeds[r])]
            assert sum(h) > 125 and sum(h[:-5]) <= 125
        assert not seeds[0] & seeds[1]
        assert out[0][it]["seed"] == out[1][it]["seed"] == base + N
        assert out[0][it]["stats"] == out[1][it]["stats"]


def test_ppo_stays_in_process_with_devices_set(monkeypatch):
    """MJRL_AMD_DEVICES hands NPG / TRPO / DAPG updates to the worker pool; PPO's
    update does not shard (one global minibatch order) and stays in this process."""
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.algos.ppo_clip import PPO
    from mjrl_amd import pool
    monkeypatch.setenv("MJRL_AMD_DEVICES", "0,1")
    started = []
    monkeypatch.setattr(pool, "get_pool", lambda devices, backend=None: started.append(devices) or "pool")
    ppo = PPO.__new__(PPO)
    ppo._comm, ppo._devices = None, None
    assert ppo._pool() is None and not started
    npg = NPG.__new__(NPG)
    npg._comm, npg._devices = None, None
    assert npg._pool() == "pool" and started == [[0, 1]]


def test_dapg_demo_share():
    """Each rank stages its share of the demonstrations (dapg.py:68-70)."""
    from types import SimpleNamespace
    from mjrl_amd.algos.dapg import DAPG
    demos = [dict(observations=np.zeros((L, 3)), actions=np.zeros((L, 1))) for L in (5, 9, 2, 7, 4)]
    got = []
    for r in range(3):
        a = DAPG.__new__(DAPG)
        a.demo_paths, a.lam_0 = demos, 1.0
        a._comm = SimpleNamespace(world_size=3, rank=r)
        got += a._demo_paths()
    assert [len(p["observations"]) for p in got] == [5, 9, 2, 7, 4]
