"""Multi-GPU from one controller process on the GPU box (mjrl_amd/pool.py): the
real NPG agent with devices=[0, 0] — two worker processes on the box's one GPU,
gloo carrying the all-reduces (RCCL refuses two ranks on one GPU; the 8-GPU
node uses RCCL over the same code) — inside a train_agent-shaped loop whose
file I/O (mkdir / chdir / pickles / log.csv / results.txt) runs in this process
only.  The pool is started before this process touches the GPU (as a training
script's controller never does); then the same loop runs in-process on one GPU
and the two must agree: statistics to fp64 rounding, parameters and the device
LinearBaseline fit within the sharded-sum tolerance (tests/test_gpu_dist.py)."""
import os
import pickle

import numpy as np
import pytest

import stub_samplers

pytestmark = pytest.mark.gpu


class _Env:
    env_id = "stub-v0"


def _loop(tmp, devices, niter=2, N=120, baseline="linear"):
    import torch
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.baselines.mlp_baseline import MLPBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(8, 2, 100, 1)
    policy = MLP(spec, hidden_sizes=(64, 64), seed=0)
    if baseline == "linear":
        base = LinearBaseline(spec)
    else:
        torch.manual_seed(11)
        base = MLPBaseline(spec, batch_size=64, epochs=2, learn_rate=1e-3)
    agent = NPG(_Env(), policy, base, normalized_step_size=0.05, seed=500, save_logs=True, devices=devices)
    os.makedirs(tmp, exist_ok=True)
    job = os.path.join(tmp, "job")
    cwd = os.getcwd()
    os.mkdir(job)
    os.chdir(job)
    try:
        os.mkdir("iterations")
        os.mkdir("logs")
        stats = []
        for i in range(niter):
            stats.append(agent.train_step(N=N, sample_mode="trajectories", gamma=0.995, gae_lambda=0.97, num_cpu=1))
            pickle.dump(agent.policy, open("iterations/policy_%i.pickle" % i, "wb"))
            pickle.dump(agent.baseline, open("iterations/baseline_%i.pickle" % i, "wb"))
            agent.logger.save_log("logs/")
            with open("results.txt", "a") as f:
                f.write("%4i %5.2f\n" % (i, stats[-1][0]))
        adv = np.concatenate([p["advantages"] for p in stub_samplers.LAST])
    finally:
        os.chdir(cwd)
    return agent, stats, adv, job


def test_pool_npg_two_workers_one_gpu(tmp_path, monkeypatch):
    stub_samplers.install()
    monkeypatch.setenv("MJRL_AMD_POOL_BACKEND", "gloo")
    from mjrl_amd import pool
    try:
        a2, s2, adv2, j2 = _loop(str(tmp_path / "pool"), [0, 0])
        assert len(pool._POOLS) == 1
    finally:
        pool.close_pools()
    a1, s1, adv1, j1 = _loop(str(tmp_path / "one"), None)
    stub_samplers.CALLS.clear()
    np.testing.assert_allclose(np.array(s2), np.array(s1), rtol=1e-10)
    # advantages of the last iteration: its baseline came from an fp64 Gram summed
    # over two shards (all-reduced) against one sum: 1e-11-level differences
    np.testing.assert_allclose(adv2, adv1, rtol=1e-9, atol=1e-9)
    th1, th2 = a1.policy.get_param_values(), a2.policy.get_param_values()
    assert np.linalg.norm(th2 - th1) / np.linalg.norm(th1) < 1e-3
    np.testing.assert_allclose(a2.baseline._coeffs, a1.baseline._coeffs, rtol=1e-6, atol=1e-8)
    assert list(a2.logger.log) == list(a1.logger.log)
    np.testing.assert_allclose(a2.logger.log["kl_dist"], a1.logger.log["kl_dist"], rtol=1e-2)
    assert open(os.path.join(j2, "results.txt")).read().count("\n") == 2


def test_pool_mlp_baseline_matches_in_process(tmp_path, monkeypatch):
    """The pool with an MLPBaseline: its features are built from the
    path observations on the host in f64 (mlp_baseline.py:37-56), so the pool
    ships float64 segments for it (pool._segment_dtype) and the workers fit it
    sharded (fit_sharded: minibatch gradients all-reduced).  Against the same loop
    in-process: the statistics exactly (returns need no baseline), the first
    iteration's advantages exactly (the untrained baseline predicts zeros), then
    the fitted baseline's predictions and the parameters within the sharded-sum
    tolerance of Adam (1e-3, as the MLPBaseline device fit against the reference)."""
    stub_samplers.install()
    monkeypatch.setenv("MJRL_AMD_POOL_BACKEND", "gloo")
    from mjrl_amd import pool
    try:
        a2, s2, adv2, j2 = _loop(str(tmp_path / "pool"), [0, 0], baseline="mlp")
        agent_dtype = pool._segment_dtype(a2)
    finally:
        pool.close_pools()
    assert agent_dtype == np.float64
    a1, s1, adv1, j1 = _loop(str(tmp_path / "one"), None, baseline="mlp")
    stub_samplers.CALLS.clear()
    np.testing.assert_allclose(np.array(s2), np.array(s1), rtol=1e-10)
    rel = np.linalg.norm(adv2 - adv1) / np.linalg.norm(adv1)
    assert rel < 1e-3, rel
    th1, th2 = a1.policy.get_param_values(), a2.policy.get_param_values()
    assert np.linalg.norm(th2 - th1) / np.linalg.norm(th1) < 1e-3
    p = dict(observations=np.random.RandomState(3).randn(50, 8), rewards=np.zeros(50))
    b1, b2 = a1.baseline.predict(p), a2.baseline.predict(p)
    assert np.linalg.norm(b2 - b1) / max(np.linalg.norm(b1), 1e-12) < 1e-3
