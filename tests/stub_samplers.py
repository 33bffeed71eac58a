"""Stand-ins for mjrl.samplers.{trajectory_sampler, batch_sampler} (test helper,
written for this repo: MuJoCo / gym are not installed).  Path i of a call with
pegasus seed s is drawn from RandomState(s + i) — the pegasus convention of the
reference samplers (base_sampler.py:37-44 seeds the env with the given seed and
numbers paths from there) — so a split of N paths over workers or ranks with
seed offsets reproduces exactly the paths of the unsplit call."""
import sys
import types

import numpy as np

HORIZON = 100
CALLS = []
LAST = []   # the paths of the last call (the caller's objects: train_step writes returns into them)


def _path(seed, policy, T):
    rs = np.random.RandomState(seed)
    H = int(min(T, HORIZON - (seed % 7)))        # ragged lengths
    n, m = policy.n, policy.m
    obs = rs.randn(H, n)
    act = rs.randn(H, m)
    rew = rs.randn(H)
    a0, info = policy.get_action(obs[0])         # the CPU policy mirror is usable in a sampler
    assert a0.shape == (m,) and "mean" in info
    return dict(observations=obs, actions=act, rewards=rew, agent_infos={}, env_infos={},
                terminated=bool(seed % 3 == 0))


def sample_paths_parallel(N, policy, T=1e6, env_name=None, pegasus_seed=None, num_cpu="max", **kw):
    CALLS.append(("trajectories", N, pegasus_seed, num_cpu))
    base = 0 if pegasus_seed is None else pegasus_seed
    LAST[:] = [_path(base + i, policy, T) for i in range(N)]
    return list(LAST)


def sample_paths(N, policy, T=1e6, env=None, env_name=None, pegasus_seed=None, num_cpu="max",
                 paths_per_call=5, mode="sample"):
    """batch_sampler.sample_paths: whole paths until more than N timesteps
    (batch_sampler.py:39-53, seed advanced by the paths drawn so far)."""
    CALLS.append(("samples", N, pegasus_seed, num_cpu))
    paths, so_far, n_paths = [], 0, 0
    seed = 0 if pegasus_seed is None else pegasus_seed
    while so_far <= N:
        seed += n_paths
        new = [_path(seed + i, policy, T) for i in range(paths_per_call)]
        paths += new
        n_paths += paths_per_call
        so_far += sum(len(p["rewards"]) for p in new)
    return paths


def install():
    """Registers the stubs as mjrl.samplers.trajectory_sampler / batch_sampler."""
    me = sys.modules[__name__]
    mjrl = sys.modules.get("mjrl") or types.ModuleType("mjrl")
    samplers = types.ModuleType("mjrl.samplers")
    traj = types.ModuleType("mjrl.samplers.trajectory_sampler")
    traj.sample_paths_parallel = me.sample_paths_parallel
    batch = types.ModuleType("mjrl.samplers.batch_sampler")
    batch.sample_paths = me.sample_paths
    samplers.trajectory_sampler, samplers.batch_sampler = traj, batch
    mjrl.samplers = samplers
    sys.modules.update({"mjrl": mjrl, "mjrl.samplers": samplers, "mjrl.samplers.trajectory_sampler": traj,
                        "mjrl.samplers.batch_sampler": batch})
