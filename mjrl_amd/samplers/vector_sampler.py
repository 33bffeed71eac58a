"""Vectorised trajectory sampling: N environments stepped
in lock step, the policy's mean action for all of them from one device launch
per step (mjrl_policy_mean, csrc/rollout.hip) instead of N per-observation CPU
forwards (policy.get_action, mjrl/policies/gaussian_mlp.py:92-98).  The
environments (MuJoCo) stay on the CPU.

Each trajectory is the one mjrl/samplers/base_sampler.py:do_rollout (:39-83)
produces for the same pegasus seed: trajectory ep seeds its environment with
seed + ep, draws its action noise exp(log_std) * randn(m) per step from its own
numpy stream seeded with seed + ep (the reference re-seeds numpy's global RNG
per trajectory and draws nothing else from it inside the loop), resets under
that stream (env resets that use the global RNG see the state the reference's
would), stops at done or T = min(T, env.horizon) steps, and is returned in the
sampler wire format (observations, actions, rewards, agent_infos, env_infos,
terminated).  Paths come back in trajectory order; numpy's global RNG is left
as the reference leaves it (the last trajectory's stream).  The mean action is
the f32 MuNet forward (index-order f32 sums: equal to the CPU forward up to f32
rounding).
"""
import ctypes as C

import numpy as np
import torch

from .. import _lib
from ..engine import UpdateEngine


class BatchedPolicy:
    """The policy's mean network on the device for a batch of observations."""

    def __init__(self, policy, device=None):
        if device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("mjrl_amd batched sampling runs the policy forward on the GPU; none is visible")
            device = torch.device("cuda", torch.cuda.current_device())
        self.policy = policy
        self.device = torch.device(device)
        self.eng = UpdateEngine(policy.n, policy.m, policy.hidden, device=self.device,
                                min_log_std=policy.min_log_std)
        self.packed = torch.zeros(self.eng.shape.packed, dtype=torch.float32, device=self.device)
        self.refresh()

    def refresh(self):
        """Re-packs the policy's current (new) parameters and transformations."""
        eng = self.eng
        with torch.cuda.device(self.device):
            eng.set_transformations(*self.policy.transformations())
            theta = torch.from_numpy(np.ascontiguousarray(self.policy.get_param_values(), dtype=np.float32))
            theta = eng._pad(theta.to(self.device), "act")
            _lib.check(eng.lib.mjrl_pack_params(C.byref(eng.shape), _lib.ptr(theta), _lib.ptr(self.packed), 0,
                                                eng.min_log_std, _lib.stream_ptr()), "mjrl_pack_params")
        self.log_std_val = np.float64(self.policy.log_std.data.numpy().ravel())

    def means(self, observations):
        """f32 [N][m] mean actions for observations [N][n] (numpy)."""
        eng = self.eng
        N = int(observations.shape[0])
        with torch.cuda.device(self.device):
            obs = torch.from_numpy(np.ascontiguousarray(observations, dtype=np.float32)).to(self.device)
            out = torch.empty((N, self.policy.m), dtype=torch.float32, device=self.device)
            ins, isc, osh, osc = eng.transforms
            p = lambda t: None if t is None else _lib.ptr(t)
            _lib.check(eng.lib.mjrl_policy_mean(C.byref(eng.shape), _lib.ptr(obs), N, _lib.ptr(self.packed), p(ins),
                                                p(isc), p(osh), p(osc), _lib.ptr(out), _lib.stream_ptr()),
                       "mjrl_policy_mean")
            return out.cpu().numpy()


def _seed_env(env, seed):
    try:
        env.env._seed(seed)
    except AttributeError:
        env.env.seed(seed)


def _stack(dicts):
    """tensor_utils.stack_tensor_dict_list: a list of (nested) dicts -> a dict of arrays."""
    if not dicts:
        return {}
    out = {}
    for k, v in dicts[0].items():
        vals = [d[k] for d in dicts]
        out[k] = _stack(vals) if isinstance(v, dict) else np.array(vals)
    return out


class _Slot:
    __slots__ = ("env", "ep", "rs", "o", "t", "obs", "act", "rew", "ainfo", "einfo", "idx")


def sample_paths_vectorized(N, policy, T=1e6, env=None, env_name=None, pegasus_seed=None, num_envs=64,
                            device=None, sink=None):
    """N trajectories on min(num_envs, N) lock-stepped environments.

    env: an environment factory (called once per slot) or None with env_name
    (mjrl.utils.get_environment, the reference's registry).  sink: a
    samplers.stream_staging.StreamSink (built with nslots >= min(num_envs, N)
    and horizon >= the trajectories' length) that receives every observation /
    action row as it is produced and stages each trajectory to HBM when it ends
    (sink.batch(paths) afterwards), or a factory sink(N, horizon, slots) that
    builds one.  The paths returned are the same either way."""
    if env is None:
        if env_name is None:
            raise ValueError("sample_paths_vectorized needs env (a factory) or env_name")
        from mjrl.utils.get_environment import get_environment
        env = lambda: get_environment(env_name)   # noqa: E731
    if N <= 0:
        return []
    bp = BatchedPolicy(policy, device)
    scale = np.exp(bp.log_std_val)
    m = policy.m
    slots = []
    for _ in range(min(int(num_envs), int(N))):
        s = _Slot()
        s.env = env()
        slots.append(s)
    horizon = min(T, slots[0].env.horizon)
    if callable(sink):   # a factory: sink(N, horizon, slots)
        sink = sink(N, int(horizon), len(slots))
    if sink is not None and (sink.N != N or sink.H < horizon or len(sink.buf) < len(slots)):
        raise ValueError("StreamSink sized for %d paths x %d steps on %d slots; sampling %d x %d on %d"
                         % (sink.N, sink.H, len(sink.buf), N, horizon, len(slots)))
    for i, s in enumerate(slots):
        s.idx = i
    paths = [None] * N
    last_state = [None]
    next_ep = [0]

    def start(s):
        if next_ep[0] >= N:
            s.ep = None
            return
        s.ep = ep = next_ep[0]
        next_ep[0] += 1
        if pegasus_seed is not None:
            _seed_env(s.env, pegasus_seed + ep)
            s.rs = np.random.RandomState(pegasus_seed + ep)
        else:
            s.rs = np.random.RandomState()
        # the reset sees the trajectory's stream as numpy's global RNG (base_sampler.py:48-58)
        saved = np.random.get_state()
        np.random.set_state(s.rs.get_state())
        s.o = s.env.reset()
        s.rs.set_state(np.random.get_state())
        np.random.set_state(saved)
        s.t = 0
        s.obs, s.act, s.rew, s.ainfo, s.einfo = [], [], [], [], []
        if sink is not None:
            sink.begin(s.idx, ep)

    def finish(s, done):
        if sink is not None:
            sink.finish(s.idx, s.t, bool(done))
        paths[s.ep] = dict(observations=np.array(s.obs), actions=np.array(s.act), rewards=np.array(s.rew),
                           agent_infos=_stack(s.ainfo), env_infos=_stack(s.einfo), terminated=done)
        if s.ep == N - 1:
            last_state[0] = s.rs.get_state()
        start(s)

    for s in slots:
        start(s)
    while True:
        live = [s for s in slots if s.ep is not None]
        if not live:
            break
        O = np.stack([np.asarray(s.o, dtype=np.float64).ravel() for s in live])
        means = bp.means(O)
        # every slot's action from its own stream (the draw order within a slot is
        # the reference's), then the environments step
        acts = [mean + scale * s.rs.randn(m) for s, mean in zip(live, means)]
        if sink is not None:
            idx, ts = [s.idx for s in live], [s.t for s in live]
            sink.rows(idx, O, ts)
            sink.actions(idx, np.stack(acts), ts)
        for s, mean, a in zip(live, means, acts):
            next_o, r, done, info = s.env.step(a)
            if sink is not None:
                sink.reward(s.idx, s.t, r)
            s.obs.append(s.o)
            s.act.append(a)
            s.rew.append(r)
            s.ainfo.append({"mean": mean, "log_std": bp.log_std_val, "evaluation": mean})
            s.einfo.append(info)
            s.o = next_o
            s.t += 1
            if done == True or s.t >= horizon:   # noqa: E712 (base_sampler.py:61: done != True)
                finish(s, done)
    if last_state[0] is not None:
        np.random.set_state(last_state[0])
    return paths
