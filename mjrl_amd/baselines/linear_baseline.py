"""Linear time-feature value baseline (the input to the GAE scan).

API of mjrl/baselines/linear_baseline.py:4-49: `predict(path)` feeds
compute_advantages; `fit(paths, return_errors)` solves the ridge normal
equations on [clip(obs, +-10), t/1000, (t/1000)^2, (t/1000)^3, 1] features.
This object is the host numpy (fp64) form, used when a caller calls it directly.
Inside the agents both directions run on the GPU from the batch already in HBM:
predict as k_linear_baseline while the paths are staged (engine.DeviceBatch,
C-ABI mjrl_linear_baseline), and fit as the fp64 MFMA Gram of [features,
returns] plus the residual pass (UpdateEngine.fit_linear_baseline, C-ABI
mjrl_linear_baseline_gram / _residual) followed by this class's lstsq retry loop
on the (n+5) x (n+5) system (§8f row f1).
"""
import numpy as np


def time_features(obs, clip=10.0):
    o = np.clip(obs, -clip, clip)
    if o.ndim > 2:
        o = o.reshape(o.shape[0], -1)
    t = (np.arange(o.shape[0]) / 1000.0)[:, None]
    return np.concatenate([o, t, t ** 2, t ** 3, np.ones_like(t)], axis=1)


class LinearBaseline:
    def __init__(self, env_spec, reg_coeff=1e-5):
        self.n = env_spec.observation_dim
        self._reg_coeff = reg_coeff
        self._coeffs = None

    def _features(self, path):
        return time_features(path["observations"])

    def predict(self, path):
        if self._coeffs is None:
            return np.zeros(len(path["rewards"]))
        return self._features(path).dot(self._coeffs)

    def fit(self, paths, return_errors=False):
        F = np.concatenate([self._features(p) for p in paths])
        y = np.concatenate([p["returns"] for p in paths])
        if return_errors:
            pred = F.dot(self._coeffs) if self._coeffs is not None else np.zeros_like(y)
            err_before = np.sum((y - pred) ** 2) / np.sum(y ** 2)
        FtF, Fty = F.T.dot(F), F.T.dot(y)
        reg = self._reg_coeff
        for _ in range(10):   # retry with 10x regularisation on NaN (linear_baseline.py:31-38)
            c = np.linalg.lstsq(FtF + reg * np.identity(F.shape[1]), Fty, rcond=None)[0]
            self._coeffs = c
            if not np.any(np.isnan(c)):
                break
            reg *= 10
        if return_errors:
            err_after = np.sum((y - F.dot(self._coeffs)) ** 2) / np.sum(y ** 2)
            return err_before, err_after
