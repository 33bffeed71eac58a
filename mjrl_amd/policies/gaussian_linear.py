"""Linear Gaussian policy with the API of mjrl/policies/gaussian_linear.py:8-175
(BASELINE config 1: point_mass).  Same CPU-mirror / device hand-off contract as
mjrl_amd.policies.gaussian_mlp.MLP; the engine runs it as the zero-hidden-layer
kernel variant."""
import numpy as np
import torch
import torch.nn as nn

from .gaussian_mlp import _GaussianPolicyBase


class LinearModel(nn.Module):
    def __init__(self, obs_dim, act_dim, in_shift=None, in_scale=None, out_shift=None, out_scale=None):
        super().__init__()
        self.obs_dim, self.act_dim = obs_dim, act_dim
        self.set_transformations(in_shift, in_scale, out_shift, out_scale)
        self.fc0 = nn.Linear(obs_dim, act_dim)

    def set_transformations(self, in_shift=None, in_scale=None, out_shift=None, out_scale=None):
        self.transformations = dict(in_shift=in_shift, in_scale=in_scale, out_shift=out_shift, out_scale=out_scale)
        f = lambda v, fill, k: torch.from_numpy(np.float32(v)) if v is not None else torch.full((k,), float(fill))
        self.in_shift = f(in_shift, 0.0, self.obs_dim)
        self.in_scale = f(in_scale, 1.0, self.obs_dim)
        self.out_shift = f(out_shift, 0.0, self.act_dim)
        self.out_scale = f(out_scale, 1.0, self.act_dim)

    def forward(self, x):
        h = (x - self.in_shift) / (self.in_scale + 1e-8)
        return self.fc0(h) * self.out_scale + self.out_shift


class LinearPolicy(_GaussianPolicyBase):
    def __init__(self, env_spec, min_log_std=-3, init_log_std=0, seed=None):
        self.n = env_spec.observation_dim
        self.m = env_spec.action_dim
        self.min_log_std = min_log_std
        if seed is not None:
            torch.manual_seed(seed)
            np.random.seed(seed)
        self._finish_init(init_log_std, lambda: LinearModel(self.n, self.m))
