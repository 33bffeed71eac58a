"""An NPG agent whose device update is replaced by a CPU stand-in (test helper,
written for this repo): the GPU worker pool's protocol and the single-process
training loop around it are exercised on CPU (tests/test_pool.py).  The
stand-in is sharding-invariant: every full-batch quantity is an all-reduced sum,
so N workers reproduce the one-process result."""
import numpy as np
import torch

from mjrl_amd.algos.npg_cg import NPG


class StubNPG(NPG):
    def train_from_samples(self, paths, gamma, gae_lambda):
        from oracle import npg_cpu as O
        for p in paths:
            p["returns"] = O.discount_sum(p["rewards"], gamma)
            p["baseline"] = self.baseline.predict(p)
            p["advantages"] = p["returns"] - p["baseline"]
        return self._stub_update(paths)

    def train_from_paths(self, paths):
        return self._stub_update(paths)

    def _stub_update(self, paths):
        comm = self.comm()
        pr = np.array([float(np.sum(p["rewards"])) for p in paths])
        adv = np.concatenate([p["advantages"] for p in paths])
        s = torch.tensor([pr.sum(), (pr ** 2).sum(), len(pr), adv.sum(), len(adv)], dtype=torch.float64)
        mx = torch.tensor([pr.max(), -pr.min()], dtype=torch.float64)
        comm.allreduce_sum(s)
        comm.allreduce_max(mx)
        s, mx = s.numpy(), mx.numpy()
        mean = s[0] / s[2]
        base_stats = [mean, np.sqrt(max(s[1] / s[2] - mean ** 2, 0.0)), -mx[1], mx[0]]
        self.running_score = mean if self.running_score is None else 0.9 * self.running_score + 0.1 * mean
        theta = self.policy.get_param_values() + np.float32(1e-3 * s[3] / s[4])
        self.policy.set_param_values(theta, set_new=True, set_old=True)
        self.last_update = dict(alpha=float(s[3] / s[4]))
        if self.save_logs:
            self.logger.log_kv("stoc_pol_mean", base_stats[0])
            self.logger.log_kv("alpha", float(s[3] / s[4]))
            self.logger.log_kv("running_score", self.running_score)
            self._log_success(paths)
        return base_stats
