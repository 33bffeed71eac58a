"""A small deterministic environment with the GymEnv surface the samplers use
(reset / step / horizon / env.seed), written for the sampler tests: stable
linear dynamics driven by the action, a quadratic reward, termination when the
state leaves a ball.  Its reset draws from the environment's own seeded stream
and from numpy's global RNG (as some gym resets do), so a sampler that does not
reproduce the reference's per-trajectory global seeding is caught."""
import numpy as np


class _Inner:
    def __init__(self):
        self.rs = np.random.RandomState(0)

    def seed(self, s):
        self.rs = np.random.RandomState(s)


class StubEnv:
    def __init__(self, n=6, m=2, horizon=40, radius=2.5):
        self.env = _Inner()
        self.n, self.m, self.horizon, self.radius = n, m, horizon, radius
        self.B = np.random.RandomState(123).randn(n, m) * 0.3

    def reset(self):
        self.x = self.env.rs.randn(self.n) + 0.01 * np.random.randn(self.n)
        return self.x.copy()

    def step(self, a):
        self.x = 0.9 * self.x + self.B.dot(np.tanh(a))
        r = -float(self.x.dot(self.x))
        done = bool(np.linalg.norm(self.x) > self.radius)
        return self.x.copy(), r, done, {"norm": float(np.linalg.norm(self.x))}


def serial_rollout(N, policy, T, env_fn, pegasus_seed):
    """mjrl/samplers/base_sampler.py:do_rollout's loop restated for the stub
    (per-trajectory global seeding, policy.get_action per step)."""
    env = env_fn()
    T = min(T, env.horizon)
    paths = []
    for ep in range(N):
        seed = pegasus_seed + ep
        env.env.seed(seed)
        np.random.seed(seed)
        obs, act, rew, means, infos = [], [], [], [], []
        o = env.reset()
        done, t = False, 0
        while t < T and done != True:   # noqa: E712
            a, info = policy.get_action(o)
            next_o, r, done, einfo = env.step(a)
            obs.append(o)
            act.append(a)
            rew.append(r)
            means.append(info["mean"])
            infos.append(einfo["norm"])
            o = next_o
            t += 1
        paths.append(dict(observations=np.array(obs), actions=np.array(act), rewards=np.array(rew),
                          mean=np.array(means), norm=np.array(infos), terminated=done))
    return paths
