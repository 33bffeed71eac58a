"""Returns and advantages on the GPU (API of mjrl/utils/process_samples.py:3-44).

compute_returns / compute_advantages take the sampler's path dicts, run the
reverse discounted scans on the device (one lane per path, fp64,
multiply-then-add: bit-identical to the reference's discount_sum) and write
"returns", "baseline" and "advantages" back into each path, as the reference
does.  Inside NPG.train_step the same kernel runs on the already-staged batch
instead (mjrl_amd.algos.batch_reinforce.train_from_samples)."""
import numpy as np

from ..engine import device_returns_advantages


def _cat(paths, key):
    return np.concatenate([np.asarray(p[key], dtype=np.float64) for p in paths]) if paths else np.zeros(0)


def _scatter(paths, key, values):
    i = 0
    for p in paths:
        H = len(p["rewards"])
        p[key] = values[i:i + H]
        i += H


def compute_returns(paths, gamma):
    lengths = [len(p["rewards"]) for p in paths]
    ret, _ = device_returns_advantages(_cat(paths, "rewards"), None, lengths, [False] * len(paths), gamma, None)
    _scatter(paths, "returns", ret)


def compute_advantages(paths, baseline, gamma, gae_lambda=None, normalize=False):
    lengths = [len(p["rewards"]) for p in paths]
    for p in paths:
        p["baseline"] = baseline.predict(p)
    # plain branch (gae_lambda None / outside [0, 1]): returns - baseline, with the
    # returns recomputed by the same kernel that produced path["returns"]
    ret, adv = device_returns_advantages(_cat(paths, "rewards"), _cat(paths, "baseline"), lengths,
                                         [bool(p.get("terminated", False)) for p in paths], gamma, gae_lambda,
                                         normalize=normalize)
    _scatter(paths, "advantages", adv)


def discount_sum(x, gamma, terminal=0.0):
    """y_t = x_t + gamma y_{t+1}, y_H = terminal (process_samples.py:37-44), on the GPU.
    A non-zero terminal folds into the last element exactly as the reference's
    first step does (x[-1] + gamma * terminal)."""
    x = np.array(x, dtype=np.float64, copy=True)
    if len(x) == 0:
        return np.array([])
    if terminal != 0.0:
        x[-1] = x[-1] + gamma * terminal
    ret, _ = device_returns_advantages(x, None, [len(x)], [False], gamma, None)
    return ret
