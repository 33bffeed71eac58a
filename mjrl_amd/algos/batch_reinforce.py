"""BatchREINFORCE with the API of mjrl/algos/batch_reinforce.py:22-175; the
per-iteration update runs on the gfx950 engine (mjrl_amd.engine).

train_step keeps the reference's flow (batch_reinforce.py:58-103): sample on
host CPUs with the reference's samplers, returns + GAE, the policy update, then
baseline.fit on the paths.  Here the paths are staged into HBM once; the GAE
scan, the whole update and the statistics run on the GPU; returns / baseline /
advantages are written back into the path dicts for baseline.fit.
"""
import logging
import time as timer

import numpy as np
import torch

from ..engine import DeviceBatch, UpdateEngine
from ..utils.logger import DataLog

logging.disable(logging.CRITICAL)   # as the reference's algos do at import


def _samplers():
    """The reference's host-CPU samplers (MuJoCo stays on the CPU)."""
    try:
        import mjrl.samplers.trajectory_sampler as trajectory_sampler
        import mjrl.samplers.batch_sampler as batch_sampler
    except ImportError as e:   # pragma: no cover - needs the reference + gym + mujoco-py
        raise ImportError("train_step samples with mjrl's samplers (mjrl.samplers.*, gym, mujoco-py); "
                          "install mjrl alongside mjrl_amd, or stage your own paths and call "
                          "train_from_paths") from e
    return trajectory_sampler, batch_sampler


class BatchREINFORCE:
    algo = "vpg"

    def __init__(self, env, policy, baseline, learn_rate=0.01, seed=None, save_logs=False, device=None,
                 comm=None):
        self.env = env
        self.policy = policy
        self.baseline = baseline
        self.alpha = learn_rate
        self.seed = seed
        self.save_logs = save_logs
        self.running_score = None
        if save_logs:
            self.logger = DataLog()
        self._device = device
        self._comm = comm
        self._engine = None

    # ---- device engine (never pickled: agents stay CPU-picklable) -----------
    def __getstate__(self):
        d = dict(self.__dict__)
        d["_engine"] = None
        d["_last_batch"] = None   # device tensors
        return d

    def engine(self):
        if self._engine is None:
            self._engine = UpdateEngine(self.policy.n, self.policy.m, self.policy.hidden, device=self._device,
                                        comm=self._comm, min_log_std=self.policy.min_log_std)
        self._engine.set_transformations(*self.policy.transformations())
        return self._engine

    def _theta(self, old=False):
        params = self.policy.old_params if old else self.policy.trainable_params
        flat = np.concatenate([p.data.reshape(-1).numpy() for p in params]).astype(np.float32)
        return torch.from_numpy(flat).to(self.engine().device)

    def _same_old_new(self):
        return all(torch.equal(a.data, b.data) for a, b in zip(self.policy.old_params, self.policy.trainable_params))

    # ---- single passes (batch_reinforce.py:37-55) -----------------------------
    def CPI_surrogate(self, observations, actions, advantages):
        eng = self.engine()
        T = eng.load_rows(observations, actions, advantages)
        eng.forward_pass(self._theta(old=True), T)
        surr, _ = eng.eval_pass(self._theta(), T)
        return torch.tensor(surr)

    def kl_old_new(self, observations, actions):
        eng = self.engine()
        T = eng.load_rows(observations, actions)
        eng.forward_pass(self._theta(old=True), T)
        _, kl = eng.eval_pass(self._theta(), T)
        return torch.tensor(kl)

    def flat_vpg(self, observations, actions, advantages):
        if not self._same_old_new():
            raise ValueError("flat_vpg on the device path is the gradient at old == new parameters "
                             "(likelihood ratio 1), which is every call site of the reference")
        eng = self.engine()
        T = eng.load_rows(observations, actions, advantages)
        return eng.forward_pass(self._theta(), T).cpu().numpy().copy()

    # ---- one iteration (batch_reinforce.py:58-103) ---------------------------
    def train_step(self, N, sample_mode="trajectories", env_name=None, T=1e6, gamma=0.995, gae_lambda=0.98,
                   num_cpu="max"):
        if env_name is None:
            env_name = self.env.env_id
        if sample_mode != "trajectories" and sample_mode != "samples":
            print("sample_mode in NPG must be either 'trajectories' or 'samples'")
            quit()
        trajectory_sampler, batch_sampler = _samplers()
        ts = timer.time()
        if sample_mode == "trajectories":
            paths = trajectory_sampler.sample_paths_parallel(N, self.policy, T, env_name, self.seed, num_cpu)
        else:
            paths = batch_sampler.sample_paths(N, self.policy, T, env_name=env_name, pegasus_seed=self.seed,
                                               num_cpu=num_cpu)
        if self.save_logs:
            self.logger.log_kv("time_sampling", timer.time() - ts)
        self.seed = self.seed + N if self.seed is not None else self.seed

        eval_statistics = self.train_from_samples(paths, gamma, gae_lambda)
        eval_statistics.append(N)
        if self.save_logs:
            ts = timer.time()
            error_before, error_after = self._fit_baseline(paths, return_errors=True)
            self.logger.log_kv("time_VF", timer.time() - ts)
            self.logger.log_kv("VF_error_before", error_before)
            self.logger.log_kv("VF_error_after", error_after)
        else:
            self._fit_baseline(paths)
        return eval_statistics

    def _fit_baseline(self, paths, return_errors=False):
        """baseline.fit(paths) (batch_reinforce.py:93-101).  A LinearBaseline is
        fitted on the device from the batch still in HBM (its Gram products are
        the T x k work); other baselines fit on the host."""
        batch = getattr(self, "_last_batch", None)
        if batch is not None and type(self.baseline).__name__ == "LinearBaseline" \
                and hasattr(self.baseline, "_reg_coeff") and batch.T == sum(len(p["rewards"]) for p in paths):
            self._last_batch = None
            return self.engine().fit_linear_baseline(batch, self.baseline, return_errors=return_errors)
        return self.baseline.fit(paths, return_errors=return_errors) if return_errors else self.baseline.fit(paths)

    def train_from_samples(self, paths, gamma, gae_lambda):
        """Returns + advantages + update from raw sampled paths with one staging:
        compute_returns / compute_advantages (process_samples.py:3-35) then
        train_from_paths, fused on the device.  Writes returns / baseline /
        advantages into the path dicts like the reference does."""
        eng = self.engine()
        batch = DeviceBatch.from_paths(paths, eng.device, baseline=self.baseline, demo_paths=self._demo_paths())
        ret, adv = eng.returns_advantages(batch, gamma, gae_lambda)
        ret, adv = ret.cpu().numpy(), adv.cpu().numpy()
        base = batch.baseline.cpu().numpy()
        off = np.concatenate([[0], np.cumsum(batch.lengths)])
        for i, p in enumerate(paths):
            p["returns"] = ret[off[i]:off[i + 1]]
            p["baseline"] = base[off[i]:off[i + 1]]
            p["advantages"] = adv[off[i]:off[i + 1]]
        out = self._update(batch, paths, skip_gae=True, gamma=gamma)
        self._last_batch = batch   # obs + returns stay in HBM for the baseline fit
        return out

    def train_from_paths(self, paths):
        eng = self.engine()
        batch = DeviceBatch.from_paths(paths, eng.device, use_advantages=True, demo_paths=self._demo_paths())
        return self._update(batch, paths)

    # ---- hooks for subclasses ---------------------------------------------------
    def _demo_paths(self):
        return None

    def _update_args(self):
        return dict(algo="vpg", learn_rate=self.alpha)

    def _log_update(self, res):
        self.logger.log_kv("alpha", self.alpha)
        self.logger.log_kv("time_vpg", res["time_vpg"])
        self.logger.log_kv("kl_dist", res["kl_dist"])
        self.logger.log_kv("surr_improvement", res["surr_after"] - res["surr_before"])
        self.logger.log_kv("running_score", self.running_score)

    def _update(self, batch, paths, skip_gae=False, gamma=0.995):
        eng = self.engine()
        args = self._update_args()
        res = eng.update(batch, self._theta(), skip_gae=skip_gae, gamma=gamma, gae_lambda=None, **args)
        self.last_update = res
        base_stats = [float(v) for v in res["base_stats"]]
        mean_return = base_stats[0]
        self.running_score = mean_return if self.running_score is None else \
            0.9 * self.running_score + 0.1 * mean_return
        self.policy.set_param_values(eng.vec["theta_new"].cpu().numpy(), set_new=True, set_old=True)
        if self.save_logs:
            self.logger.log_kv("stoc_pol_mean", base_stats[0])
            self.logger.log_kv("stoc_pol_std", base_stats[1])
            self.logger.log_kv("stoc_pol_max", base_stats[3])
            self.logger.log_kv("stoc_pol_min", base_stats[2])
            self._log_update(res)
            self._log_success(paths)
        return base_stats

    def _log_success(self, paths):
        try:
            self.env.env.env.evaluate_success(paths, self.logger)
        except Exception:
            try:
                success_rate = self.env.env.env.evaluate_success(paths)
                self.logger.log_kv("success_rate", success_rate)
            except Exception:
                pass

    def log_rollout_statistics(self, paths):
        path_returns = [sum(p["rewards"]) for p in paths]
        self.logger.log_kv("stoc_pol_mean", np.mean(path_returns))
        self.logger.log_kv("stoc_pol_std", np.std(path_returns))
        self.logger.log_kv("stoc_pol_max", np.amax(path_returns))
        self.logger.log_kv("stoc_pol_min", np.amin(path_returns))
