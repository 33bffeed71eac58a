"""Multi-GPU behind an unchanged, single-process training loop (mjrl_amd/pool.py),
on CPU: the agent gets devices=[0, 0] and the pool's two workers (gloo) run the
update; the loop — train_agent's file I/O (mjrl/utils/train_agent.py:28-88:
mkdir / chdir, policy and baseline pickles, log.csv, results.txt) — runs in this
process only, and parameters, statistics, logs, the baseline fit and the
returns / advantages written back into the paths equal the one-process run.
The device update is a sharding-invariant CPU stand-in (tests/stub_pool_agent.py);
the GPU version is tests/test_gpu_pool.py."""
import os
import pickle

import numpy as np
import pytest

import stub_samplers

N_OBS, N_ACT = 5, 2


class _Env:
    env_id = "stub-v0"


def _loop(tmp, devices, niter=3, N=12):
    """A train_agent-shaped loop (train_agent.py:28-88, evaluation left out)."""
    from stub_pool_agent import StubNPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(N_OBS, N_ACT, 100, 1)
    agent = StubNPG(_Env(), MLP(spec, hidden_sizes=(32, 32), seed=0), LinearBaseline(spec), seed=1000,
                    save_logs=True, devices=devices)
    os.makedirs(tmp, exist_ok=True)
    job = os.path.join(tmp, "job")
    cwd = os.getcwd()
    if not os.path.isdir(job):
        os.mkdir(job)
    os.chdir(job)
    try:
        for d in ("iterations", "logs"):
            if not os.path.isdir(d):
                os.mkdir(d)
        stats = []
        for i in range(niter):
            stats.append(agent.train_step(N=N, sample_mode="trajectories", gamma=0.99, gae_lambda=0.95, num_cpu=1))
            pickle.dump(agent.policy, open("iterations/policy_%i.pickle" % i, "wb"))
            pickle.dump(agent.baseline, open("iterations/baseline_%i.pickle" % i, "wb"))
            agent.logger.save_log("logs/")
            with open("results.txt", "a") as f:
                f.write("%4i %5.2f %5.2f\n" % (i, stats[-1][0], stats[-1][0]))
        paths = [dict(p) for p in stub_samplers.LAST]
    finally:
        os.chdir(cwd)
    return agent, stats, paths, job


@pytest.fixture
def pool_env(monkeypatch):
    stub_samplers.install()
    monkeypatch.setenv("MJRL_AMD_POOL_BACKEND", "gloo")
    yield
    from mjrl_amd import pool
    pool.close_pools()
    stub_samplers.CALLS.clear()


def test_pool_matches_one_process(tmp_path, pool_env):
    a1, s1, p1, j1 = _loop(str(tmp_path / "one"), None)
    a2, s2, p2, j2 = _loop(str(tmp_path / "two"), [0, 0])
    from mjrl_amd import pool
    assert len(pool._POOLS) == 1 and next(iter(pool._POOLS.values())).world == 2
    np.testing.assert_allclose(np.array(s2), np.array(s1), rtol=1e-12)
    np.testing.assert_allclose(a2.policy.get_param_values(), a1.policy.get_param_values(), rtol=1e-6)
    np.testing.assert_allclose(a2.baseline._coeffs, a1.baseline._coeffs, rtol=1e-6, atol=1e-9)
    assert list(a2.logger.log) == list(a1.logger.log)
    for k in a1.logger.log:
        if not k.startswith("time"):
            np.testing.assert_allclose(np.array(a2.logger.log[k], float), np.array(a1.logger.log[k], float),
                                       rtol=1e-6, err_msg=k)
    assert a2.running_score == pytest.approx(a1.running_score, rel=1e-12)
    assert a2.seed == a1.seed == 1000 + 3 * 12
    for x, y in zip(p1, p2):   # written back by the workers into this process's path dicts
        for k in ("returns", "baseline", "advantages"):
            np.testing.assert_allclose(y[k], x[k], rtol=1e-9, atol=1e-12)
    # the loop's files exist once, written by this process
    assert open(os.path.join(j2, "results.txt")).read().count("\n") == 3
    assert sorted(os.listdir(os.path.join(j2, "iterations"))) == sorted(os.listdir(os.path.join(j1, "iterations")))
    # the pickled agent objects carry no pool / device state
    pickle.loads(pickle.dumps(a2.policy))
    b = pickle.loads(pickle.dumps(a2.baseline))
    np.testing.assert_array_equal(b._coeffs, a2.baseline._coeffs)


def test_pool_train_from_paths(pool_env):
    from stub_pool_agent import StubNPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(N_OBS, N_ACT, 100, 1)
    rs = np.random.RandomState(3)
    paths = [dict(observations=rs.randn(h, N_OBS), actions=rs.randn(h, N_ACT), rewards=rs.randn(h),
                  advantages=rs.randn(h)) for h in (7, 30, 12, 3, 25)]
    out = []
    for devices in (None, [0, 0]):
        ag = StubNPG(_Env(), MLP(spec, hidden_sizes=(32, 32), seed=0), LinearBaseline(spec), devices=devices)
        out.append((ag.train_from_paths(paths), ag.policy.get_param_values()))
    np.testing.assert_allclose(out[1][0], out[0][0], rtol=1e-12)
    np.testing.assert_allclose(out[1][1], out[0][1], rtol=1e-6)


def _adv_paths(seed=3):
    rs = np.random.RandomState(seed)
    return [dict(observations=rs.randn(h, N_OBS) * 10 ** rs.uniform(-3, 3, N_OBS), actions=rs.randn(h, N_ACT),
                 rewards=rs.randn(h), advantages=rs.randn(h)) for h in (7, 30, 12, 3, 25)]


def _agent(cls, devices, **kw):
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(N_OBS, N_ACT, 100, 1)
    return cls(_Env(), MLP(spec, hidden_sizes=(32, 32), seed=0), LinearBaseline(spec), devices=devices, **kw)


def test_pool_f32_segments(pool_env):
    """float32 staging: the workers get the batch already converted, with its
    column ranges (the worker-side checks are in StubNPG32), and the update equals
    the one-process one."""
    from stub_pool_agent import StubNPG32
    paths = _adv_paths()
    out = []
    for devices in (None, [0, 0]):
        ag = _agent(StubNPG32, devices)
        if devices is None:
            ag._pre = dict(obs=np.concatenate([p["observations"] for p in paths]).astype(np.float32),
                           act=np.concatenate([p["actions"] for p in paths]).astype(np.float32))
            ag._pre["obs_range"] = (ag._pre["obs"].min(0), ag._pre["obs"].max(0))
        out.append((ag.train_from_paths(paths), ag.policy.get_param_values()))
    np.testing.assert_allclose(out[1][0], out[0][0], rtol=1e-12)
    np.testing.assert_allclose(out[1][1], out[0][1], rtol=1e-6)


def test_fill_shard_layouts():
    """The controller's fill of a segment, read back as the worker reads it."""
    from mjrl_amd.pool import _Layout, _fill_shard, _worker_paths
    paths = _adv_paths(5)
    lengths = np.array([len(p["rewards"]) for p in paths])
    import concurrent.futures as cf
    ex = cf.ThreadPoolExecutor(4)
    for dt, kw in ((np.float64, {}), (np.float32, {}), (np.float64, dict(ex=ex, chunk_rows=20)),
                   (np.float32, dict(ex=ex, chunk_rows=20)),    # one chunk / several chunks in parallel
                   (np.float32, dict(ex=ex, threads=4))):       # the default chunking (two per thread)
        L = _Layout(int(lengths.sum()), len(paths), N_OBS, N_ACT, True, dt)
        buf = bytearray(L.nbytes)
        _fill_shard(buf, L, paths, lengths, **kw)
        got = _worker_paths(L, buf)
        for p, q in zip(paths, got):
            assert q["observations"].dtype == dt
            np.testing.assert_array_equal(q["observations"], p["observations"].astype(dt))
            np.testing.assert_array_equal(q["actions"], p["actions"].astype(dt))
            np.testing.assert_array_equal(q["rewards"], p["rewards"])
            np.testing.assert_array_equal(q["advantages"], p["advantages"])
        if dt == np.float32:
            rng = L.view(buf, "orange").reshape(2, N_OBS)
            allo = np.concatenate([p["observations"] for p in paths]).astype(np.float32)
            np.testing.assert_array_equal(rng[0], allo.min(0))
            np.testing.assert_array_equal(rng[1], allo.max(0))
        assert all(off % 64 == 0 for off, _, _ in L.fields.values())


def test_pool_state_travels_once(pool_env):
    """Attributes whose pickle did not change since the last step stay with the
    workers (hyperparameters, DAPG demos); the policy travels every step."""
    from stub_pool_agent import StubNPG
    from mjrl_amd import pool
    ag = _agent(StubNPG, [0, 0])
    ag.demo_like = np.arange(1000.0)
    paths = _adv_paths()
    ag.train_from_paths(paths)
    p = next(iter(pool._POOLS.values()))
    st = p._state(ag, commit=False)                 # what the next step sends: the update's results
    assert "policy" in st["changed"] and "demo_like" not in st["changed"] and "n_step_size" not in st["changed"]
    p._state(ag)                      # as if sent
    st = p._state(ag, commit=False)   # nothing changed since
    assert not st["changed"] and not st["dropped"]
    ag.policy.set_param_values(ag.policy.get_param_values() + 1.0, set_new=True, set_old=True)
    del ag.demo_like
    st = p._state(ag, commit=False)
    assert set(st["changed"]) == {"policy"} and st["dropped"] == ["demo_like"]
    th = ag.policy.get_param_values()
    ref = _agent(StubNPG, None)
    ref.policy.set_param_values(th, set_new=True, set_old=True)
    ref.running_score = ag.running_score
    # the workers rebuild the agent from their cache + the delta
    np.testing.assert_allclose(ag.train_from_paths(paths), ref.train_from_paths(paths), rtol=1e-12)
    np.testing.assert_allclose(ag.policy.get_param_values(), ref.policy.get_param_values(), rtol=1e-6)


def test_pool_worker_exits_before_connecting(pool_env, monkeypatch):
    """A worker that dies before it connects (e.g. an import error) ends the pool
    start with a RuntimeError instead of an accept() that never returns."""
    import sys
    import time
    from mjrl_amd import pool
    monkeypatch.setattr(sys, "executable", "/bin/false")
    t0 = time.time()
    with pytest.raises(RuntimeError, match="exited before connecting"):
        pool.DevicePool([0, 0], "gloo")
    assert time.time() - t0 < 30


def test_pool_failed_update_is_cleaned_up(pool_env):
    """One rank's update raises while the other waits in the all-reduce: the step
    raises at once, every worker is killed, the segments are unlinked and the
    pool is forgotten; the next step starts a fresh pool."""
    import time
    from multiprocessing import shared_memory
    from stub_pool_agent import FailingNPG, StubNPG
    from mjrl_amd import pool
    paths = _adv_paths()
    ag = _agent(FailingNPG, [0, 0])
    t0 = time.time()
    with pytest.raises(RuntimeError, match="update failed on rank 1"):
        ag.train_from_paths(paths)
    assert time.time() - t0 < 60
    assert not pool._POOLS
    ag2 = _agent(StubNPG, [0, 0])
    ag2.train_from_paths(paths)
    p = next(iter(pool._POOLS.values()))
    assert all(q.poll() is None for q in p._procs)
    names = [s.name for s in p._shm]
    pool.close_pools()
    for nm in names:
        with pytest.raises(FileNotFoundError):
            shared_memory.SharedMemory(name=nm)


def test_resolve_devices(monkeypatch):
    from mjrl_amd.pool import resolve_devices
    monkeypatch.delenv("MJRL_AMD_DEVICES", raising=False)
    assert resolve_devices(None) is None and resolve_devices([3]) is None
    assert resolve_devices(4) == [0, 1, 2, 3] and resolve_devices([2, 5]) == [2, 5]
    monkeypatch.setenv("MJRL_AMD_DEVICES", "0,1,2")
    assert resolve_devices(None) == [0, 1, 2]
    monkeypatch.setenv("MJRL_AMD_DEVICES", "8")
    assert resolve_devices(None) == list(range(8))
