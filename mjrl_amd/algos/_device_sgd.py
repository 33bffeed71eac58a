"""Minibatch first-order training of a Gaussian policy on the GPU, shared by BC
(behavior_cloning.py) and PPO (ppo_clip.py) — SURVEY.md §8f row f4.

The CPU policy (mjrl_amd.policies.*) and the caller's CPU optimizer over
policy.trainable_params stay the source of truth, exactly the objects the
reference trains (behavior_cloning.py:37, ppo_clip.py:44).  Around a training
call, DeviceTrainer copies the parameters and the optimizer state to the device,
runs every minibatch step there, and copies both back, so pickling, CPU sampling
and a later call (Adam moments carried over, as the reference's optimizer
carries them) see the same state the reference would leave.

A minibatch step — gather the rows named by a device index buffer, the policy
mean (functional form of MuNet / LinearModel, gaussian_mlp.py:143-182), the
loss, backward, the optimizer step — is captured once as a hipGraph and replayed
per minibatch (capturable Adam); the minibatch indices come from numpy's global
RNG in the reference's order, drawn for a whole epoch up front and uploaded in one
copy.  Optimizers without a capturable mode run the same step eagerly.
"""
import numpy as np
import torch
import torch.nn.functional as F

from .._capture import capture

LOG_2PI = float(np.log(2 * np.pi))


def default_device(device=None):
    if device is not None:
        return torch.device(device)
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class DeviceTrainer:
    def __init__(self, policy, optimizer, device=None):
        self.policy = policy
        self.cpu_opt = optimizer
        self.device = default_device(device)
        self.params = [torch.zeros(p.shape, dtype=torch.float32, device=self.device, requires_grad=True)
                       for p in policy.trainable_params]
        self.graphable = self.device.type == "cuda" and "capturable" in optimizer.defaults
        kw = dict(optimizer.defaults)
        if self.graphable:
            kw["capturable"] = True
        self.opt = type(optimizer)(self.params, **kw)
        self._graphs = {}
        self._tf = None

    # ---- CPU <-> device ------------------------------------------------------
    def pull(self):
        """policy params + optimizer state (CPU) -> device."""
        with torch.no_grad():
            for d, c in zip(self.params, self.policy.trainable_params):
                d.copy_(c.data)
        cpu_state = self.cpu_opt.state
        for d, c in zip(self.params, self.policy.trainable_params):
            sc = cpu_state.get(c)
            sd = self.opt.state[d]
            if not sc:
                for v in sd.values():
                    if torch.is_tensor(v):
                        v.zero_()
                continue
            for k, v in sc.items():
                if torch.is_tensor(v):
                    v = v.to(self.device, dtype=torch.float32 if k == "step" else v.dtype)
                    if k in sd and torch.is_tensor(sd[k]) and sd[k].shape == v.shape:
                        sd[k].copy_(v)
                    else:
                        sd[k] = v.clone()
                else:
                    sd[k] = torch.tensor(float(v), dtype=torch.float32, device=self.device) \
                        if k == "step" and self.graphable else v
        for gd, gc in zip(self.opt.param_groups, self.cpu_opt.param_groups):
            for k, v in gc.items():
                if k not in ("params", "capturable", "foreach", "fused", "differentiable"):
                    gd[k] = v
        t = self.policy.model.transformations
        dev = self.device
        f = lambda v, fill, k: torch.from_numpy(np.float32(v)).to(dev) if v is not None else \
            torch.full((k,), float(fill), device=dev)
        tf = (f(t["in_shift"], 0.0, self.policy.n), f(t["in_scale"], 1.0, self.policy.n),
              f(t["out_shift"], 0.0, self.policy.m), f(t["out_scale"], 1.0, self.policy.m))
        if self._tf is None:
            self._tf = tf
        else:
            # copied into the existing buffers: a captured step reads them by address
            for d, s in zip(self._tf, tf):
                d.copy_(s)

    def push(self):
        """device params + optimizer state -> the CPU policy / optimizer (the
        Parameter objects keep their identity: the CPU optimizer stays bound)."""
        with torch.no_grad():
            for d, c in zip(self.params, self.policy.trainable_params):
                c.data.copy_(d.detach().cpu())
        for d, c in zip(self.params, self.policy.trainable_params):
            sd = self.opt.state.get(d)
            if not sd:
                continue
            sc = self.cpu_opt.state[c]
            for k, v in sd.items():
                if torch.is_tensor(v):
                    sc[k] = torch.tensor(float(v.item())) if k == "step" else v.detach().cpu().clone()
                else:
                    sc[k] = v

    # ---- the policy on the device -----------------------------------------------
    def mean(self, obs, params=None):
        """policy.model(obs) for device rows (gaussian_mlp.py:168-182 / gaussian_linear.py)."""
        p = self.params if params is None else params
        ins, isc, osh, osc = self._tf
        h = (obs - ins) / (isc + 1e-8)
        if self.policy.hidden is None:
            out = F.linear(h, p[0], p[1])
        else:
            h = torch.tanh(F.linear(h, p[0], p[1]))
            h = torch.tanh(F.linear(h, p[2], p[3]))
            out = F.linear(h, p[4], p[5])
        return out * osc + osh

    def log_likelihood(self, obs, act, params=None):
        """mean_LL (gaussian_mlp.py:100-108): -0.5 sum z^2 - sum log_std - 0.5 m log 2 pi."""
        p = self.params if params is None else params
        log_std = p[-1]
        zs = (act - self.mean(obs, p)) / torch.exp(log_std)
        return -0.5 * torch.sum(zs ** 2, dim=1) + -torch.sum(log_std) + -0.5 * self.policy.m * LOG_2PI

    # ---- minibatch steps ------------------------------------------------------------
    def epoch(self, key, loss_fn, idx_batches):
        """One pass over idx_batches (device i64 [nmb][mb]): per row of it, the
        step zero_grad -> loss_fn(idx) -> backward -> optimizer step.  `key`
        names the captured graph: a replay re-reads the tensors loss_fn closed
        over at capture, so a caller gives every new set of data a new key."""
        nmb = int(idx_batches.shape[0])
        if nmb == 0:
            return
        mb = int(idx_batches.shape[1])
        g = self._graph(key, loss_fn, mb) if self.graphable else None
        for i in range(nmb):
            if g is not None:
                g[1].copy_(idx_batches[i])
                g[0].replay()
            else:
                self.opt.zero_grad()
                loss_fn(idx_batches[i]).backward()
                self.opt.step()

    def _graph(self, key, loss_fn, mb):
        hyper = tuple((k, v) for g in self.opt.param_groups for k, v in sorted(g.items())
                      if k != "params" and isinstance(v, (int, float, bool, tuple)))
        gkey = (key, mb, hyper)   # hyperparameters are baked into a captured step
        if gkey in self._graphs:
            return self._graphs[gkey]
        self._graphs.clear()   # a graph holds its closure's data buffers: keep only the live one
        dev = self.device
        idx = torch.zeros(mb, dtype=torch.int64, device=dev)

        def body():
            self.opt.zero_grad(set_to_none=False)
            loss_fn(idx).backward()
            self.opt.step()

        # the optimizer state has to exist before capture: one warm-up step on a side
        # stream, then the parameters and state it touched are restored
        saved = [p.detach().clone() for p in self.params]
        saved_state = {p: {k: v.clone() for k, v in self.opt.state[p].items() if torch.is_tensor(v)}
                       for p in self.params if self.opt.state.get(p)}
        try:
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                body()
            torch.cuda.current_stream(dev).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with capture(graph):
                body()
        finally:
            with torch.no_grad():
                for p, v in zip(self.params, saved):
                    p.copy_(v)
                for p in self.params:
                    st = self.opt.state.get(p, {})
                    for k, v in st.items():
                        if torch.is_tensor(v):
                            if p in saved_state and k in saved_state[p]:
                                v.copy_(saved_state[p][k])
                            else:
                                v.zero_()
        self._graphs[gkey] = (graph, idx)
        return self._graphs[gkey]


def choice_batches(num_samples, mb_size, device):
    """int(num_samples / mb_size) draws of np.random.choice(num_samples, mb_size)
    from numpy's global RNG, in the reference's order (behavior_cloning.py:58-59,
    ppo_clip.py:90-91), as one device tensor [nmb][mb]."""
    nmb = int(num_samples / mb_size)
    if nmb == 0:
        return torch.zeros((0, mb_size), dtype=torch.int64, device=device)
    idx = np.stack([np.random.choice(num_samples, size=mb_size) for _ in range(nmb)]).astype(np.int64)
    return torch.from_numpy(idx).to(device)
