"""Gaussian MLP policy with the API of mjrl/policies/gaussian_mlp.py:8-182.

The object is the CPU-side policy the reference's samplers pickle into forked
workers (get_action per step, mjrl/samplers/base_sampler.py:64-74), so it keeps
CPU torch modules and pickles to CPU-only state.  The batch update never runs
through these modules: the NPG / TRPO / DAPG classes in mjrl_amd.algos hand the
flat parameters to the gfx950 engine (mjrl_amd.engine) and write the result back
with set_param_values.

Construction consumes the torch / numpy RNGs exactly like the reference (same
modules created in the same order), so MLP(spec, seed=s) starts from the same
parameters as the reference's MLP(spec, seed=s).
"""
import numpy as np
import torch
import torch.nn as nn

LOG_2PI = float(np.log(2 * np.pi))


class MuNet(nn.Module):
    """obs -> normalise -> tanh(fc0) -> tanh(fc1) -> fc2 -> de-normalise
    (gaussian_mlp.py:143-182)."""

    def __init__(self, obs_dim, act_dim, hidden_sizes=(64, 64), in_shift=None, in_scale=None,
                 out_shift=None, out_scale=None):
        super().__init__()
        self.obs_dim, self.act_dim, self.hidden_sizes = obs_dim, act_dim, tuple(hidden_sizes)
        self.set_transformations(in_shift, in_scale, out_shift, out_scale)
        self.fc0 = nn.Linear(obs_dim, hidden_sizes[0])
        self.fc1 = nn.Linear(hidden_sizes[0], hidden_sizes[1])
        self.fc2 = nn.Linear(hidden_sizes[1], act_dim)

    def set_transformations(self, in_shift=None, in_scale=None, out_shift=None, out_scale=None):
        self.transformations = dict(in_shift=in_shift, in_scale=in_scale, out_shift=out_shift, out_scale=out_scale)
        f = lambda v, fill, k: torch.from_numpy(np.float32(v)) if v is not None else torch.full((k,), float(fill))
        self.in_shift = f(in_shift, 0.0, self.obs_dim)
        self.in_scale = f(in_scale, 1.0, self.obs_dim)
        self.out_shift = f(out_shift, 0.0, self.act_dim)
        self.out_scale = f(out_scale, 1.0, self.act_dim)

    def forward(self, x):
        h = (x - self.in_shift) / (self.in_scale + 1e-8)
        h = torch.tanh(self.fc0(h))
        h = torch.tanh(self.fc1(h))
        return self.fc2(h) * self.out_scale + self.out_shift


class _GaussianPolicyBase:
    """Flat-parameter plumbing shared by MLP and LinearPolicy
    (gaussian_mlp.py:59-140, gaussian_linear.py:57-138)."""

    def _finish_init(self, init_log_std, make_model):
        self.model = make_model()
        for p in list(self.model.parameters())[-2:]:   # last layer * 1e-2
            p.data = 1e-2 * p.data
        self.log_std = torch.ones(self.m, requires_grad=True)
        with torch.no_grad():
            self.log_std.mul_(init_log_std)
        self.trainable_params = list(self.model.parameters()) + [self.log_std]
        self.old_model = make_model()
        self.old_log_std = torch.ones(self.m) * init_log_std
        self.old_params = list(self.old_model.parameters()) + [self.old_log_std]
        for dst, src in zip(self.old_params, self.trainable_params):
            dst.data = src.data.clone()
        self.log_std_val = np.float64(self.log_std.data.numpy().ravel())
        self.param_shapes = [tuple(p.data.shape) for p in self.trainable_params]
        self.param_sizes = [int(p.data.numel()) for p in self.trainable_params]
        self.d = int(np.sum(self.param_sizes))
        self.obs_var = torch.randn(self.n)

    # ---- flat parameters -------------------------------------------------
    def get_param_values(self):
        return np.concatenate([p.data.reshape(-1).numpy() for p in self.trainable_params]).copy()

    def _assign(self, params, flat):
        i = 0
        for p, shp, sz in zip(params, self.param_shapes, self.param_sizes):
            p.data = torch.from_numpy(np.asarray(flat[i:i + sz]).reshape(shp)).float()
            i += sz
        params[-1].data = torch.clamp(params[-1].data, self.min_log_std)

    def set_param_values(self, new_params, set_new=True, set_old=True):
        if set_new:
            self._assign(self.trainable_params, new_params)
            self.log_std_val = np.float64(self.log_std.data.numpy().ravel())
        if set_old:
            self._assign(self.old_params, new_params)

    # ---- sampling (CPU, per step, inside sampler workers) ----------------
    def get_action(self, observation):
        o = np.float32(observation.reshape(1, -1))
        with torch.no_grad():
            mean = self.model(torch.from_numpy(o)).numpy().ravel()
        noise = np.exp(self.log_std_val) * np.random.randn(self.m)
        return [mean + noise, {"mean": mean, "log_std": self.log_std_val, "evaluation": mean}]

    # ---- CPU torch distribution API (used by BC / PPO-style callers) ------
    def mean_LL(self, observations, actions, model=None, log_std=None):
        model = self.model if model is None else model
        log_std = self.log_std if log_std is None else log_std
        mean = model(torch.from_numpy(observations).float())
        zs = (torch.from_numpy(actions).float() - mean) / torch.exp(log_std)
        LL = -0.5 * torch.sum(zs ** 2, dim=1) - torch.sum(log_std) - 0.5 * self.m * LOG_2PI
        return mean, LL

    def log_likelihood(self, observations, actions, model=None, log_std=None):
        return self.mean_LL(observations, actions, model, log_std)[1].data.numpy()

    def old_dist_info(self, observations, actions):
        mean, LL = self.mean_LL(observations, actions, self.old_model, self.old_log_std)
        return [LL, mean, self.old_log_std]

    def new_dist_info(self, observations, actions):
        mean, LL = self.mean_LL(observations, actions, self.model, self.log_std)
        return [LL, mean, self.log_std]

    def likelihood_ratio(self, new_dist_info, old_dist_info):
        return torch.exp(new_dist_info[0] - old_dist_info[0])

    def mean_kl(self, new_dist_info, old_dist_info):
        so, sn = torch.exp(old_dist_info[2]), torch.exp(new_dist_info[2])
        num = (old_dist_info[1] - new_dist_info[1]) ** 2 + so ** 2 - sn ** 2
        den = 2 * sn ** 2 + 1e-8
        return torch.mean(torch.sum(num / den + new_dist_info[2] - old_dist_info[2], dim=1))

    # ---- device hand-off ---------------------------------------------------
    @property
    def hidden(self):
        return None

    def transformations(self):
        t = self.model.transformations
        return (t["in_shift"], t["in_scale"], t["out_shift"], t["out_scale"])

    def __getstate__(self):
        # CPU-only state: nothing device-side is ever attached to the policy
        return dict(self.__dict__)


class MLP(_GaussianPolicyBase):
    def __init__(self, env_spec, hidden_sizes=(64, 64), min_log_std=-3, init_log_std=0, seed=None):
        self.n = env_spec.observation_dim
        self.m = env_spec.action_dim
        self.min_log_std = min_log_std
        self.hidden_sizes = tuple(hidden_sizes)
        if seed is not None:
            torch.manual_seed(seed)
            np.random.seed(seed)
        self._finish_init(init_log_std, lambda: MuNet(self.n, self.m, self.hidden_sizes))

    @property
    def hidden(self):
        return self.hidden_sizes
