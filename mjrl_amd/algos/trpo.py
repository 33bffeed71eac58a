"""TRPO (API of mjrl/algos/trpo.py:25-145): the NPG direction with delta =
2 kl_dist and the KL backtracking line search (alpha *= 0.9 until
KL < kl_dist, alpha = 0 after 100 trials).  Each trial is one device forward
over the batch and one 2-double readback."""
from .npg_cg import NPG
from .batch_reinforce import _check_policy
from ..utils.logger import DataLog


class TRPO(NPG):
    algo = "trpo"

    def __init__(self, env, policy, baseline, kl_dist=0.01, FIM_invert_args={"iters": 10, "damping": 1e-4},
                 hvp_sample_frac=1.0, seed=None, save_logs=False, normalized_step_size=0.01, device=None,
                 comm=None, devices=None):
        self.env = env
        self.policy = policy
        _check_policy(policy)
        self.baseline = baseline
        self.kl_dist = kl_dist if kl_dist is not None else 0.5 * normalized_step_size
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

    def _update_args(self):
        return dict(algo="trpo", kl_dist=self.kl_dist, cg_iters=self.FIM_invert_args["iters"],
                    damping=self.FIM_invert_args["damping"], hvp_sample_frac=self.hvp_subsample)
