"""Zero baseline (API of mjrl/baselines/zero_baseline.py:4-14)."""
import numpy as np


class ZeroBaseline:
    def __init__(self, env_spec, **kwargs):
        self._coeffs = None

    def fit(self, paths, return_errors=False):
        if return_errors:
            return 1.0, 1.0

    def predict(self, path):
        return np.zeros(len(path["rewards"]))
