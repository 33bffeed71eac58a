"""Behaviour cloning with the API of mjrl/algos/behavior_cloning.py:11-68
(SURVEY.md §8f row f4): maximum likelihood of the expert actions under the
Gaussian policy, minibatch Adam over policy.trainable_params, the minibatch
steps on the GPU (algos/_device_sgd.py).

Same semantics as the reference: the constructor sets the policy's input /
output transformations from the expert data's mean / std (population std,
behavior_cloning.py:27-35) and builds Adam(trainable_params, lr) unless an
optimizer is given; train() logs epoch / loss / time before every epoch and
once after, draws int(N / batch_size) minibatches of np.random.choice(N,
batch_size) per epoch from numpy's global RNG, and ends with
set_param_values(params, set_new=True, set_old=True) (the log_std clamp).
The expert rows are staged to the device once per train() call.
"""
import logging
import time as timer

import numpy as np
import torch

from ..utils.logger import DataLog
from ._device_sgd import DeviceTrainer, choice_batches, default_device

logging.disable(logging.CRITICAL)


class BC:
    def __init__(self, expert_paths, policy, epochs=5, batch_size=64, lr=1e-3, optimizer=None, device=None):
        self.policy = policy
        self.expert_paths = expert_paths
        self.epochs = epochs
        self.mb_size = batch_size
        self.logger = DataLog()
        observations = np.concatenate([path["observations"] for path in expert_paths])
        actions = np.concatenate([path["actions"] for path in expert_paths])
        in_shift, in_scale = np.mean(observations, axis=0), np.std(observations, axis=0)
        out_shift, out_scale = np.mean(actions, axis=0), np.std(actions, axis=0)
        self.policy.model.set_transformations(in_shift, in_scale, out_shift, out_scale)
        self.policy.old_model.set_transformations(in_shift, in_scale, out_shift, out_scale)
        self.optimizer = torch.optim.Adam(self.policy.trainable_params, lr=lr) if optimizer is None else optimizer
        self._device = device
        self._trainer = None

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_trainer"] = None
        return d

    def trainer(self):
        if self._trainer is None:
            self._trainer = DeviceTrainer(self.policy, self.optimizer, default_device(self._device))
        return self._trainer

    def loss(self, obs, act):
        """-mean(LL) at the current parameters (behavior_cloning.py:39-42), on the
        device; numpy inputs are staged first."""
        tr = self.trainer()
        tr.pull()
        o, a = self._stage(obs, act, tr.device)
        with torch.no_grad():
            return (-torch.mean(tr.log_likelihood(o, a))).cpu()

    @staticmethod
    def _stage(obs, act, dev):
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(dev)
        return t(obs), t(act)

    def train(self):
        observations = np.concatenate([path["observations"] for path in self.expert_paths])
        actions = np.concatenate([path["actions"] for path in self.expert_paths])
        tr = self.trainer()
        tr.pull()
        O, A = self._stage(observations, actions, tr.device)
        num_samples = observations.shape[0]

        def full_loss():
            with torch.no_grad():
                return float((-torch.mean(tr.log_likelihood(O, A))).item())

        def mb_loss(idx):
            return -torch.mean(tr.log_likelihood(O.index_select(0, idx), A.index_select(0, idx)))

        ts = timer.time()
        # the captured step reads this call's O / A: a new key per call (an id() of a
        # freed tensor can come back for the next call's data)
        self._ncall = getattr(self, "_ncall", 0) + 1
        for ep in range(self.epochs):
            self.logger.log_kv("epoch", ep)
            self.logger.log_kv("loss", np.float32(full_loss()))
            self.logger.log_kv("time", timer.time() - ts)
            tr.epoch(("bc", self._ncall), mb_loss,
                     choice_batches(num_samples, self.mb_size, tr.device))
        tr.push()
        params_after_opt = self.policy.get_param_values()
        self.policy.set_param_values(params_after_opt, set_new=True, set_old=True)
        self.logger.log_kv("epoch", self.epochs)
        tr.pull()
        self.logger.log_kv("loss", np.float32(full_loss()))
        self.logger.log_kv("time", timer.time() - ts)
