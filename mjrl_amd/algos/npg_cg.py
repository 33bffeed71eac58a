"""Natural policy gradient (API of mjrl/algos/npg_cg.py:24-165) on the gfx950
engine: VPG, 10 device Fisher-vector products inside a device-side CG, the
normalised step and the post-step surrogate / KL, one host readback."""
import numpy as np
import torch

from .batch_reinforce import BatchREINFORCE, _check_policy
from ..utils.logger import DataLog


class NPG(BatchREINFORCE):
    algo = "npg"

    def __init__(self, env, policy, baseline, normalized_step_size=0.01, const_learn_rate=None,
                 FIM_invert_args={"iters": 10, "damping": 1e-4}, hvp_sample_frac=1.0, seed=None,
                 save_logs=False, kl_dist=None, device=None, comm=None, devices=None):
        self.env = env
        self.policy = policy
        _check_policy(policy)
        self.baseline = baseline
        self.alpha = const_learn_rate
        self.n_step_size = normalized_step_size if kl_dist is None else 2.0 * kl_dist
        self.seed = seed
        self.save_logs = save_logs
        self.FIM_invert_args = FIM_invert_args
        self.hvp_subsample = hvp_sample_frac
        self.running_score = None
        if save_logs:
            self.logger = DataLog()
        self._device = device
        self._comm = comm
        self._engine = None
        self._devices = devices   # several GPUs from this process: mjrl_amd/pool.py

    def HVP(self, observations, actions, vector, regu_coef=None):
        """F v + damping v at the current (old == new) parameters (npg_cg.py:55-74);
        with hvp_sample_frac < 0.99 on np.random.choice(N, int(frac N)) rows drawn
        from numpy's global RNG, as the reference does (npg_cg.py:58-62)."""
        regu_coef = self.FIM_invert_args["damping"] if regu_coef is None else regu_coef
        if self.hvp_subsample is not None and self.hvp_subsample < 0.99:
            num_samples = observations.shape[0]
            rand_idx = np.random.choice(num_samples, size=int(self.hvp_subsample * num_samples))
            observations, actions = observations[rand_idx], actions[rand_idx]
        eng = self.engine()
        T = eng.load_rows(observations, actions)
        eng.forward_pass(self._theta(), T)
        v = torch.from_numpy(np.ascontiguousarray(vector, dtype=np.float32)).to(eng.device)
        return eng.fvp(v, damping=float(regu_coef), T=T).cpu().numpy()

    def build_Hvp_eval(self, inputs, regu_coef=None):
        def eval(v):
            return self.HVP(*(list(inputs) + [v, regu_coef]))
        return eval

    def _update_args(self):
        return dict(algo="npg", n_step_size=self.n_step_size, const_lr=self.alpha,
                    cg_iters=self.FIM_invert_args["iters"], damping=self.FIM_invert_args["damping"],
                    hvp_sample_frac=self.hvp_subsample)

    def _log_update(self, res):
        self.logger.log_kv("alpha", res["alpha"])
        self.logger.log_kv("delta", res["delta"])
        self.logger.log_kv("time_vpg", res["time_vpg"])
        self.logger.log_kv("time_npg", res["time_npg"])
        self.logger.log_kv("kl_dist", res["kl_dist"])
        self.logger.log_kv("surr_improvement", res["surr_after"] - res["surr_before"])
        self.logger.log_kv("running_score", self.running_score)
