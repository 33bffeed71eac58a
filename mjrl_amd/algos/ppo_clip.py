"""PPO with the clipped surrogate, API of mjrl/algos/ppo_clip.py:23-120
(SURVEY.md §8f row f4).

train_from_paths keeps the reference's flow: whitened advantages
(adv - mean) / (std + 1e-6), path-return statistics, surr_before, `epochs`
passes of int(N / mb_size) minibatches drawn by np.random.choice from numpy's
global RNG, each an Adam step on -mean(min(LR adv, clip(LR, 1 +- c) adv))
(ppo_clip.py:47-54), then surr_after and the old/new KL, and
set_param_values(new, set_new=True, set_old=True).

Device work: the minibatch steps run on the GPU as replays of one captured step
(algos/_device_sgd.py; the likelihood ratio != 1 gradient the NPG path never
needs), with the old log-likelihoods computed once for all rows when the old
parameters are fixed during the call (see _old_on_device for when they are not).  surr_before / surr_after / kl_dist come
from the HIP engine's forward / evaluation passes (CPI_surrogate, kl_old_new).
train_step is BatchREINFORCE's (device GAE), handing the paths with their
advantages to train_from_paths.  Single process: the minibatch order is global,
so a sharded PPO is not offered (comm must be local).
"""
import time as timer

import numpy as np
import torch

from .batch_reinforce import BatchREINFORCE
from ._device_sgd import DeviceTrainer, choice_batches
from ..utils.logger import DataLog


class PPO(BatchREINFORCE):
    _poolable = False   # the minibatch order is global: one process, even with MJRL_AMD_DEVICES set
    def __init__(self, env, policy, baseline, clip_coef=0.2, epochs=10, mb_size=64, learn_rate=3e-4, seed=0,
                 save_logs=False, device=None, comm=None):
        super().__init__(env, policy, baseline, learn_rate=learn_rate, seed=seed, save_logs=save_logs,
                         device=device, comm=comm)
        self.learn_rate = learn_rate
        self.clip_coef = clip_coef
        self.epochs = epochs
        self.mb_size = mb_size
        if save_logs:
            self.logger = DataLog()
        self.optimizer = torch.optim.Adam(self.policy.trainable_params, lr=learn_rate)
        self._trainer = None

    def __getstate__(self):
        d = super().__getstate__()
        d["_trainer"] = None
        return d

    def trainer(self):
        if self._trainer is None:
            self._trainer = DeviceTrainer(self.policy, self.optimizer, self.engine().device)
        return self._trainer

    def _update(self, batch, paths, skip_gae=False, gamma=0.995):
        # train_step -> train_from_samples: the device GAE wrote the advantages into
        # the path dicts; PPO's own train_from_paths takes it from there
        return self.train_from_paths(paths)

    def _old_on_device(self, tr):
        """The old parameters as the minibatch steps see them.  The reference's
        set_param_values(p, set_new=True, set_old=True) (gaussian_mlp.py:66-89)
        hands the same float32 array to the new and the old parameters, so after
        any previous update they share storage (log_std excepted: its clamp makes a
        new tensor) and the optimizer's in-place steps move the old mean network
        with the new one (the likelihood ratio then only sees the log_std change).
        The same aliasing exists in this package's policy classes; a shared tensor
        is mirrored as the live device parameter (detached: the old branch carries
        no gradient), any other as a frozen copy.  Returns (list, any aliased)."""
        out, aliased = [], False
        for i, (o, n) in enumerate(zip(self.policy.old_params, self.policy.trainable_params)):
            if o.data.data_ptr() == n.data.data_ptr() and o.data.shape == n.data.shape:
                out.append(tr.params[i].detach())
                aliased = True
            else:
                out.append(o.data.to(tr.device))
        return out, aliased

    def train_from_paths(self, paths):
        if self.comm().world_size > 1:
            raise NotImplementedError("PPO's minibatch order is global (ppo_clip.py:89-91): run it in one process")
        observations = np.concatenate([path["observations"] for path in paths])
        actions = np.concatenate([path["actions"] for path in paths])
        advantages = np.concatenate([path["advantages"] for path in paths])
        advantages = (advantages - np.mean(advantages)) / (np.std(advantages) + 1e-6)
        path_returns = [sum(p["rewards"]) for p in paths]
        mean_return = np.mean(path_returns)
        std_return = np.std(path_returns)
        min_return = np.amin(path_returns)
        max_return = np.amax(path_returns)
        base_stats = [mean_return, std_return, min_return, max_return]
        self.running_score = mean_return if self.running_score is None else \
            0.9 * self.running_score + 0.1 * mean_return
        if self.save_logs:
            self.log_rollout_statistics(paths)

        surr_before = float(self.CPI_surrogate(observations, actions, advantages))
        ts = timer.time()
        tr = self.trainer()
        tr.pull()
        dev = tr.device
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(dev)
        O, A, ADV = t(observations), t(actions), t(advantages)   # adv f32 as ppo_clip.py:48
        old_dev, aliased = self._old_on_device(tr)
        c = float(self.clip_coef)
        if not aliased:
            # the old parameters are fixed during the call: LL_old once for all rows
            with torch.no_grad():
                LL_old = tr.log_likelihood(O, A, old_dev)

        def mb_loss(idx):
            adv = ADV.index_select(0, idx)
            o, a = O.index_select(0, idx), A.index_select(0, idx)
            if aliased:
                with torch.no_grad():
                    ll_old = tr.log_likelihood(o, a, old_dev)
            else:
                ll_old = LL_old.index_select(0, idx)
            LR = torch.exp(tr.log_likelihood(o, a) - ll_old)
            LR_clip = torch.clamp(LR, min=1 - c, max=1 + c)
            return -torch.mean(torch.min(LR * adv, LR_clip * adv))

        num_samples = observations.shape[0]
        # the captured step reads this call's O / A / ADV / LL_old: a new key per call
        self._ncall = getattr(self, "_ncall", 0) + 1
        for ep in range(self.epochs):
            tr.epoch(("ppo", self._ncall), mb_loss, choice_batches(num_samples, self.mb_size, dev))
        tr.push()
        params_after_opt = self.policy.get_param_values()
        surr_after = float(self.CPI_surrogate(observations, actions, advantages))
        kl_dist = float(self.kl_old_new(observations, actions))
        self.policy.set_param_values(params_after_opt, set_new=True, set_old=True)
        t_opt = timer.time() - ts
        if self.save_logs:
            self.logger.log_kv("t_opt", t_opt)
            self.logger.log_kv("kl_dist", kl_dist)
            self.logger.log_kv("surr_improvement", surr_after - surr_before)
            self.logger.log_kv("running_score", self.running_score)
            self._log_success(paths)
        return base_stats
