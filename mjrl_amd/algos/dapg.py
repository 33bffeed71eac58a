"""DAPG (API of mjrl/algos/dapg.py:26-141): the VPG over RL + demonstration rows
with all_adv = 1e-2 [w / (std(w) + 1e-8); lam_0 lam_1^k], scaled by T_all / T_rl,
the Fisher metric on the RL rows only, delta = 2 kl_dist, no line search.  The
demonstration rows are staged behind the RL rows of the same device batch."""
from .npg_cg import NPG
from .batch_reinforce import _check_policy
from ..utils.logger import DataLog


class DAPG(NPG):
    algo = "dapg"

    def __init__(self, env, policy, baseline, demo_paths=None, normalized_step_size=0.01,
                 FIM_invert_args={"iters": 10, "damping": 1e-4}, hvp_sample_frac=1.0, seed=None, save_logs=False,
                 kl_dist=None, lam_0=1.0, lam_1=0.95, device=None, comm=None, devices=None):
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
        self.demo_paths = demo_paths
        self.lam_0 = lam_0
        self.lam_1 = lam_1
        self.iter_count = 0.0
        if save_logs:
            self.logger = DataLog()
        self._device = device
        self._comm = comm
        self._engine = None
        self._devices = devices   # several GPUs from this process: mjrl_amd/pool.py

    def _use_demos(self):
        return self.demo_paths is not None and self.lam_0 > 0.0

    def _demo_paths(self):
        """The demonstrations this rank stages: all of them on one process, its
        share under several ranks (each demo row enters the all-reduced sum once)."""
        return self._rank_share(self.demo_paths) if self._use_demos() else None

    def _update_args(self):
        args = dict(algo="dapg", kl_dist=self.kl_dist, cg_iters=self.FIM_invert_args["iters"],
                    damping=self.FIM_invert_args["damping"], hvp_sample_frac=self.hvp_subsample)
        if self._use_demos():
            args["demo_coef"] = self.lam_0 * (self.lam_1 ** self.iter_count)   # dapg.py:65
            self.iter_count += 1
        return args
