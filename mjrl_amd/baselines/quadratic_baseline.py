"""Quadratic-feature value baseline (API of mjrl/baselines/quadratic_baseline.py:4-70):
[o/10 (clipped), upper-triangular o_i o_j, 1, t/1000 .. (t/1000)^4] features,
ridge normal equations.  The object and its predict are host numpy; an agent
fits it on the device from the batch in HBM (UpdateEngine.fit_quadratic_baseline,
n <= 64; BatchREINFORCE._fit_baseline), and fit() here is the host path."""
import numpy as np


def quadratic_features(paths, n):
    o = np.concatenate([p["observations"] for p in paths])
    o = np.clip(o, -10, 10) / 10.0
    if o.ndim > 2:
        o = o.reshape(o.shape[0], -1)
    N = o.shape[0]
    iu, ju = np.triu_indices(n)
    feat = np.ones((N, n + len(iu) + 1 + 4))
    feat[:, :n] = o
    feat[:, n:n + len(iu)] = o[:, iu] * o[:, ju]
    k = 0
    for p in paths:
        H = len(p["rewards"])
        t = np.arange(H) / 1000.0
        for j in range(4):
            feat[k:k + H, -4 + j] = t ** (j + 1)
        k += H
    return feat


class QuadraticBaseline:
    def __init__(self, env_spec, reg_coeff=1e-5, obs_dim=None):
        self.n = obs_dim if obs_dim is not None else env_spec.observation_dim
        self._reg_coeff = reg_coeff
        self._coeffs = None

    def _features(self, paths):
        return quadratic_features(paths, self.n)

    def fit(self, paths, return_errors=False):
        F = self._features(paths)
        y = np.concatenate([p["returns"] for p in paths])
        if return_errors:
            pred = F.dot(self._coeffs) if self._coeffs is not None else np.zeros_like(y)
            err_before = np.sum((y - pred) ** 2) / np.sum(y ** 2)
        FtF, Fty = F.T.dot(F), F.T.dot(y)
        reg = self._reg_coeff
        for _ in range(10):
            c = np.linalg.lstsq(FtF + reg * np.identity(F.shape[1]), Fty, rcond=None)[0]
            self._coeffs = c
            if not np.any(np.isnan(c)):
                break
            reg *= 10
        if return_errors:
            err_after = np.sum((y - F.dot(self._coeffs)) ** 2) / np.sum(y ** 2)
            return err_before, err_after

    def predict(self, path):
        if self._coeffs is None:
            return np.zeros(len(path["rewards"]))
        return self._features([path]).dot(self._coeffs)
