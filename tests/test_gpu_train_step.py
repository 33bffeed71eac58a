"""train_step on the GPU (mjrl/algos/batch_reinforce.py:58-103) with the stub
samplers of tests/stub_samplers.py: the real device update and device baseline
fit, on one process and on two ranks (gloo on the box's GPU; RCCL on the
8-GPU node runs the same code).

End-to-end parameters are compared on the linear policy (d = 20: the 10-step CG
converges, so the step is well determined).  For the MLP the comparison stops
at the VPG: its fp32 CG amplifies reduction-order noise on these synthetic
batches (the reference's own spread on the similar c1_pointmass_mlp32 case is
1 %, tests/golden), so theta after the step is not a sound end-to-end check."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import stub_samplers

pytestmark = pytest.mark.gpu
N_OBS, N_ACT, HID, N_PATHS = 8, 2, (32, 32), 40


def nrel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))


class _Env:
    env_id = "stub-v0"


def _agent(comm=None, linear=True):
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.policies.gaussian_linear import LinearPolicy
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(N_OBS, N_ACT, 100, 1)
    pol = LinearPolicy(spec, seed=0) if linear else MLP(spec, hidden_sizes=HID, seed=0)
    return NPG(_Env(), pol, LinearBaseline(spec), normalized_step_size=0.05, seed=500, save_logs=True,
               comm=comm, device="cuda:0")


def _steps(agent, k=2):
    stub_samplers.install()
    out = []
    for _ in range(k):
        th0 = agent.policy.get_param_values()
        coeffs0 = None if agent.baseline._coeffs is None else agent.baseline._coeffs.copy()
        stats = agent.train_step(N_PATHS, gamma=0.99, gae_lambda=0.95, num_cpu=1)
        out.append(dict(stats=stats, seed=agent.seed, theta0=th0, theta=agent.policy.get_param_values(),
                        g=agent.engine().vec["g"].cpu().numpy(),
                        coeffs0=coeffs0, coeffs=agent.baseline._coeffs.copy(),
                        paths=[{k: p[k] for k in ("observations", "actions", "rewards", "terminated", "returns",
                                                  "baseline", "advantages")}
                               for p in stub_samplers.LAST],
                        log={k: list(v) for k, v in agent.logger.log.items()}))
    return out


@pytest.mark.parametrize("linear", [True, False])
def test_train_step_one_gpu_matches_oracle(linear):
    from oracle import npg_cpu as O
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.utils.gym_env import EnvSpec
    res = _steps(_agent(linear=linear))
    for it, r in enumerate(res):
        assert r["seed"] == 500 + N_PATHS * (it + 1)
        assert len(r["stats"]) == 5 and r["stats"][4] == N_PATHS
        paths = r["paths"]
        lengths = np.array([len(p["rewards"]) for p in paths])
        obs = np.concatenate([p["observations"] for p in paths])
        act = np.concatenate([p["actions"] for p in paths])
        rew = np.concatenate([p["rewards"] for p in paths])
        term = np.array([p["terminated"] for p in paths])
        base = O.linear_baseline_predict(r["coeffs0"], obs, lengths)
        ret, adv = O.returns_and_advantages(rew, base, lengths, term, 0.99, 0.95)
        assert np.array_equal(np.concatenate([p["returns"] for p in paths]), ret)   # written back, bit-exact
        # the stub's observations are f64 randn (not float32s): the default f32
        # staging still predicts from the f64 values (1e-12 of the fp64
        # LinearBaseline.predict), and the written-back advantages are the GAE of
        # those predictions bit for bit
        got_base = np.concatenate([p["baseline"] for p in paths])
        if r["coeffs0"] is not None:
            bound = np.concatenate([np.abs(O.linear_baseline_features(o)).dot(np.abs(r["coeffs0"]))
                                    for o in O.split(obs, lengths)])
            assert np.all(np.abs(got_base - base) <= 1e-12 * bound)
        else:
            assert np.array_equal(got_base, base)
        _, adv_given = O.returns_and_advantages(rew, got_base, lengths, term, 0.99, 0.95)
        assert np.array_equal(np.concatenate([p["advantages"] for p in paths]), adv_given)
        np.testing.assert_allclose(r["stats"][:4], O.path_return_stats(rew, lengths), rtol=1e-12)
        pol = O.Policy(N_OBS, N_ACT, None if linear else HID, r["theta0"].astype(np.float64), None)
        ref = O.update(pol, obs, act, adv, rew, lengths, algo="npg", n_step_size=0.05)
        assert nrel(r["g"], ref["vpg_grad"]) < 1e-5, nrel(r["g"], ref["vpg_grad"])
        if linear:
            assert nrel(r["theta"], ref["theta1"]) < 1e-5, nrel(r["theta"], ref["theta1"])
        # the device LinearBaseline fit (all-reduced Gram + the reference's lstsq loop)
        host = LinearBaseline(EnvSpec(N_OBS, N_ACT, 100, 1))
        host.fit([dict(p) for p in paths])
        # the device fit reads the f32-staged rows AND their low halves (the f64 values)
        assert np.linalg.norm(r["coeffs"] - host._coeffs) <= 1e-10 * np.linalg.norm(host._coeffs)
    for k in ("time_sampling", "time_VF", "VF_error_before", "VF_error_after", "alpha", "kl_dist",
              "stoc_pol_mean", "running_score"):
        assert len(res[-1]["log"][k]) == 2, k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mjrl_amd.comm import DistComm
        res = _steps(_agent(DistComm()))
        q.put((rank, [(r["theta"], r["coeffs"], r["stats"], r["seed"], len(r["paths"]), r["g"]) for r in res]))
    finally:
        dist.destroy_process_group()


def test_train_step_two_ranks_equals_one():
    single = _steps(_agent())
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=600)
        out[r] = v
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for it in range(2):
        (th0, c0, st0, sd0, n0, g0), (th1, c1, st1, sd1, n1, g1) = out[0][it], out[1][it]
        assert (n0, n1) == (20, 20)                          # each rank sampled its half
        assert np.array_equal(th0, th1) and np.array_equal(c0, c1)   # replicated state
        assert sd0 == sd1 == single[it]["seed"]
        np.testing.assert_allclose(st0, single[it]["stats"], rtol=1e-10)
        assert nrel(g0, single[it]["g"]) < 1e-5
        assert nrel(th0, single[it]["theta"]) < 1e-5, nrel(th0, single[it]["theta"])
        np.testing.assert_allclose(c0, single[it]["coeffs"], rtol=1e-6, atol=1e-9)


def test_train_from_paths_graph_replay_bitwise():
    """Three train_from_paths iterations with the same path lengths: the engine
    captures the update on the second (graphs = "auto", 6k rows) and replays it on
    the third; the parameters stay bit-identical to an agent running every update
    eagerly (staging buffers and transformation buffers keep their addresses)."""
    import copy
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.zero_baseline import ZeroBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(N_OBS, N_ACT, 100, 1)
    agents = []
    for graphs in ("auto", False):
        pol = MLP(spec, hidden_sizes=(64, 64), seed=1)
        pol.model.set_transformations(np.full(N_OBS, 0.1), np.full(N_OBS, 2.0), np.zeros(N_ACT), np.ones(N_ACT))
        ag = NPG(_Env(), pol, ZeroBaseline(spec), normalized_step_size=0.05, device="cuda:0")
        ag.engine().graphs = graphs
        agents.append(ag)
    for it in range(3):
        rs = np.random.RandomState(it)
        paths = [dict(observations=rs.randn(100, N_OBS), actions=rs.randn(100, N_ACT), rewards=rs.randn(100),
                      advantages=rs.randn(100), terminated=False) for _ in range(60)]
        for ag in agents:
            ag.train_from_paths(copy.deepcopy(paths))
    assert agents[0].engine()._gstate.get("graph") is not None
    assert agents[1].engine()._gstate.get("graph") is None
    np.testing.assert_array_equal(agents[0].policy.get_param_values(), agents[1].policy.get_param_values())


def test_train_step_vector_sampler_matches_reference_sampler():
    """train_step with the opt-in vectorised sampler (agent.sampler = "vector",
    SURVEY.md §8f row f3) against train_step with a reference-style serial
    sampler (base_sampler.do_rollout's loop, tests/stub_env.py) over the same
    environment and seeds: the same trajectories (to f32 rounding of the policy
    mean), hence the same update."""
    import sys
    import types
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    from stub_env import StubEnv, serial_rollout

    def serial(N, policy, T, env_name, seed, num_cpu, **kw):
        ps = serial_rollout(N, policy, T, StubEnv, seed)
        return [dict(observations=p["observations"], actions=p["actions"], rewards=p["rewards"], agent_infos={},
                     env_infos={}, terminated=p["terminated"]) for p in ps]
    mods = {"mjrl": types.ModuleType("mjrl"), "mjrl.samplers": types.ModuleType("mjrl.samplers"),
            "mjrl.samplers.trajectory_sampler": types.ModuleType("mjrl.samplers.trajectory_sampler"),
            "mjrl.samplers.batch_sampler": types.ModuleType("mjrl.samplers.batch_sampler")}
    mods["mjrl.samplers.trajectory_sampler"].sample_paths_parallel = serial
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    try:
        out = []
        for kind in ("reference", "vector"):
            spec = EnvSpec(6, 2, 40, 1)
            agent = NPG(_Env(), MLP(spec, hidden_sizes=(64, 64), seed=3, init_log_std=-1.0), LinearBaseline(spec),
                        normalized_step_size=0.05, seed=200, save_logs=True)
            agent.sampler, agent.env_factory, agent.num_envs = kind, StubEnv, 16
            # one iteration: the next one samples with the updated policy, and f32-level
            # differences of the two updates can move a termination by a step there
            stats = [agent.train_step(N=150, gamma=0.99, gae_lambda=0.95)]
            out.append((stats, agent.policy.get_param_values(), agent.seed))
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    (s_ref, th_ref, seed_ref), (s_vec, th_vec, seed_vec) = out
    assert seed_ref == seed_vec == 200 + 150
    np.testing.assert_allclose(np.array(s_vec), np.array(s_ref), rtol=1e-5)
    assert np.linalg.norm(th_vec - th_ref) / np.linalg.norm(th_ref) < 1e-3
