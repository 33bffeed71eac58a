"""Sampler-fed staging ("have the samplers fill pinned fp32
per-path slabs ... and overlap the H2D with" the rest of sampling).

The reference concatenates the finished f64 paths (npg_cg.py:87-89) and the
policy casts them to f32 on every forward (gaussian_mlp.py:103); the staging
path of engine.DeviceBatch.from_paths does that conversion once, but only after
sampling has finished, so the update waits for a ~3 GB f64 read and a 1.5 GB
PCIe copy at Humanoid 1M.  StreamSink moves that work INTO the
sampling loop of samplers/vector_sampler.py:

  - every lock step, the observation rows of the live environments go through
    ONE native call (mjrl_host_stage_rows_f64x) straight into their
    trajectories' pinned f32 slabs (one double-buffered slab per environment
    slot), folded into the column ranges, with the LinearBaseline prediction of
    each row computed from its f64 values (the coefficients are fixed while a
    batch is sampled: baseline.fit runs after the update) and the exactness
    flag; the actions likewise (f32);
  - every FLUSH_ROWS steps of a trajectory, its completed rows are copied to HBM
    on the staging copy stream at their fixed position (ep * H + t) of a padded
    device slab, and the rest when it ends, while the environments keep
    stepping (so the last lock step leaves at most FLUSH_ROWS rows a slot to
    copy);
  - rewards and the predictions travel the same way (8 bytes a row each);
  - after sampling, batch() compacts the padded slabs into the contiguous
    layout with one device gather per slot (mjrl_gather_rows; none when every
    trajectory ran the full horizon: the padded slabs are then the batch) and
    stages the path offsets and flags.

The DeviceBatch it returns is bit-identical to DeviceBatch.from_paths on the
same paths (the same f32 rounding, the same per-row prediction arithmetic,
ranges that give the same column scales): tests/test_gpu_stream_staging.py.
What remains after the last environment step is the trajectories' last rows,
the gather, the 1-D slots and the update itself (bench.py e2e_stream).
"""
import ctypes as C

import numpy as np
import torch

from .. import _lib
from ..engine import DeviceBatch, _STAGING, _linear_coeffs


_SLABS = {}


class StreamSink:
    """Receives rows from the vectorised sampler and stages them as they come.

    n, m: observation / action widths; horizon: the longest trajectory; N: the
    number of trajectories; baseline: the agent's value baseline (a
    LinearBaseline's coefficients are used for the predictions, as fixed while
    the batch is sampled); nslots: the sampler's environment slots."""

    NBUF = 2   # slabs per environment slot: a slot starts its next trajectory while the last one's copy runs
    FLUSH_ROWS = 256   # a live trajectory's completed rows leave for HBM in runs of this many

    def __init__(self, n, m, horizon, N, device, baseline=None, nslots=64):
        self.n, self.m, self.H, self.N = int(n), int(m), int(horizon), int(N)
        self.device = torch.device(device)
        self.baseline = baseline
        c = _linear_coeffs(baseline, self.n)
        self.linear = c is not False
        self.coeffs = None if c is False or c is None else np.ascontiguousarray(c, dtype=np.float64)
        self.L = _lib.stage_lib()
        S, B, H = int(nslots), self.NBUF, self.H
        # pinned per-slot slabs, [slot][buf][H][n] f32 observations, [..][m] actions
        # and [..] f64 predictions, kept across batches (a training loop builds one
        # sink per iteration) with the copy events that guard them
        key = (S, B, H, self.n, self.m)
        ent = _SLABS.get(key)
        if ent is None:
            _SLABS.clear()   # one shape at a time
            pin = lambda *shape, dt=torch.float32: torch.empty(shape, dtype=dt, pin_memory=True)   # noqa: E731
            ent = _SLABS[key] = dict(obs=pin(S, B, H, self.n), act=pin(S, B, H, self.m),
                                     rew=pin(S, B, H, dt=torch.float64), pred=pin(S, B, H, dt=torch.float64),
                                     ev=[[None] * B for _ in range(S)])
        self._obs, self._act, self._rew, self._pred, self._ev = (ent[k] for k in ("obs", "act", "rew", "pred", "ev"))
        self.obs_h, self.act_h, self.rew_h, self.pred_h = (t.numpy() for t in (self._obs, self._act, self._rew,
                                                                               self._pred))
        self._row_ptr0 = self.obs_h.ctypes.data
        self.buf = np.zeros(S, np.int64)
        self.ep = np.full(S, -1, np.int64)
        self.copied = np.zeros(S, np.int64)   # rows of the slot's live trajectory already sent
        self.lo = np.full(self.n, np.inf, np.float32)
        self.hi = np.full(self.n, -np.inf, np.float32)
        self.flag = np.zeros(1, np.int32)
        self.lengths = np.zeros(self.N, np.int64)
        self.term = np.zeros(self.N, np.uint8)
        with torch.cuda.device(self.device):
            slot = lambda name, k, dt: _STAGING.device_slot(name, self.N * H * k, dt, self.device)   # noqa: E731
            self.obs_pad = slot("stream_obs", self.n, np.float32).view(self.N * H, self.n)
            self.act_pad = slot("stream_act", self.m, np.float32).view(self.N * H, self.m)
            self.rew_pad = slot("stream_rew", 1, np.float64)
            self.pred_pad = slot("stream_pred", 1, np.float64) if self.coeffs is not None else None
            self.cs = _STAGING._copy_stream(self.device)
            # the padded slabs may still be read by work queued on the current stream
            self.cs.wait_stream(torch.cuda.current_stream(self.device))
        self.done = False

    # ---- sampler side -------------------------------------------------------
    def begin(self, slot, ep):
        """Slot `slot` starts trajectory `ep`: it writes into its other slab, once
        that slab's previous copy has completed."""
        b = (self.buf[slot] + 1) % self.NBUF
        ev = self._ev[slot][b]
        if ev is not None:
            ev.synchronize()
            self._ev[slot][b] = None
        self.buf[slot] = b
        self.ep[slot] = ep
        self.copied[slot] = 0

    def rows(self, slots, obs, t):
        """Observation rows obs [E, n] (f64) of environments `slots` at path
        indices t (the row each trajectory records at this step)."""
        obs = np.ascontiguousarray(obs, dtype=np.float64)
        slots = np.asarray(slots, np.int64)
        t = np.ascontiguousarray(t, dtype=np.int64)
        E = len(slots)
        if E == 0:
            return
        b = self.buf[slots]
        stride_b, stride_s = self.H * self.n * 4, self.NBUF * self.H * self.n * 4
        ptrs = (C.c_void_p * E)(*(self._row_ptr0 + slots * stride_s + b * stride_b + t * self.n * 4).tolist())
        pred = np.empty(E, np.float64) if self.coeffs is not None else None
        _lib.check(self.L.mjrl_host_stage_rows_f64x(
            obs.ctypes.data, E, self.n, ptrs, self.lo.ctypes.data, self.hi.ctypes.data,
            None if pred is None else self.coeffs.ctypes.data, t.ctypes.data, None if pred is None else pred.ctypes.data,
            self.flag.ctypes.data), "mjrl_host_stage_rows_f64x")
        if pred is not None:
            self.pred_h[slots, b, t] = pred
        # row t arriving means rows < t are complete (their actions and rewards were
        # recorded in the previous step): send full runs of them
        due = np.nonzero(t - self.copied[slots] >= self.FLUSH_ROWS)[0]
        for i in due.tolist():
            self._send(int(slots[i]), int(t[i]))

    def actions(self, slots, act, t):
        """Action rows act [E, m] of environments `slots` at path indices t."""
        slots = np.asarray(slots, np.int64)
        self.act_h[slots, self.buf[slots], np.asarray(t, np.int64)] = np.asarray(act, dtype=np.float64)

    def rewards(self, slots, rew, t):
        """Rewards rew [E] (f64) of environments `slots` at path indices t."""
        slots = np.asarray(slots, np.int64)
        self.rew_h[slots, self.buf[slots], np.asarray(t, np.int64)] = np.asarray(rew, dtype=np.float64)

    def reward(self, slot, t, r):
        """One environment's reward at path index t (the sampler's per-step call)."""
        self.rew_h[slot, self.buf[slot], t] = r

    def _send(self, slot, upto):
        """Rows [copied, upto) of slot `slot`'s live trajectory (observations,
        actions, rewards, baseline predictions) to their place in the padded
        device slabs, on the copy stream."""
        ep, b, a = int(self.ep[slot]), int(self.buf[slot]), int(self.copied[slot])
        if upto <= a:
            return
        H = self.H
        with torch.cuda.stream(self.cs):
            self.obs_pad[ep * H + a: ep * H + upto].copy_(self._obs[slot, b, a:upto], non_blocking=True)
            self.act_pad[ep * H + a: ep * H + upto].copy_(self._act[slot, b, a:upto], non_blocking=True)
            self.rew_pad[ep * H + a: ep * H + upto].copy_(self._rew[slot, b, a:upto], non_blocking=True)
            if self.pred_pad is not None:
                self.pred_pad[ep * H + a: ep * H + upto].copy_(self._pred[slot, b, a:upto], non_blocking=True)
        self.copied[slot] = upto

    def finish(self, slot, length, terminated=False):
        """Slot `slot`'s trajectory ended after `length` rows: its rows not sent yet
        leave for HBM now, on the copy stream, while sampling continues."""
        ep, b, Lr = int(self.ep[slot]), int(self.buf[slot]), int(length)
        self.lengths[ep] = Lr
        self.term[ep] = bool(terminated)
        if Lr:
            self._send(slot, Lr)
            ev = torch.cuda.Event()   # covers the trajectory's earlier runs too (one stream, in order)
            ev.record(self.cs)
            self._ev[slot][b] = ev
        self.ep[slot] = -1

    # ---- update side -------------------------------------------------------
    def batch(self, paths, reuse=True):
        """The DeviceBatch of the sampled paths (those this sink received, in
        trajectory order), as DeviceBatch.from_paths would stage them."""
        with torch.cuda.device(self.device):
            return self._batch(paths, reuse)

    def _batch(self, paths, reuse):
        N, H, dev = self.N, self.H, self.device
        lengths = np.array([len(p["rewards"]) for p in paths], dtype=np.int64)
        if len(paths) != N or not np.array_equal(lengths, self.lengths):
            raise ValueError("StreamSink.batch: the paths are not the ones the sink received")
        T = int(lengths.sum())
        cur = torch.cuda.current_stream(dev)
        cur.wait_stream(self.cs)   # every trajectory's copy

        def stage(slot, arrs, ncols, dtype=np.float64):
            return _STAGING.stage(slot, arrs, ncols, dtype, dev, reuse)

        offs = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
        off = stage("off", [offs], 0, np.int64)
        term = stage("term", [self.term], 0, np.uint8)
        orange = stage("orange", [np.stack([self.lo, self.hi])], self.n, np.float32)
        pads = [("obs", self.obs_pad, self.n, np.float32), ("act", self.act_pad, self.m, np.float32),
                ("rew", self.rew_pad, 1, np.float64)] + \
            ([("base", self.pred_pad, 1, np.float64)] if self.pred_pad is not None else [])
        out = {}
        if T == N * H:
            # every trajectory ran the full horizon: the padded slabs are the batch
            for name, pad, k, _ in pads:
                out[name] = pad[:T] if k == 1 else pad.view(-1)[:T * k].view(T, k)
        else:
            # compact: row i of the batch is row ep H + (i - off[ep]) of the slabs, one
            # device gather per slot
            start = torch.from_numpy(np.arange(N, dtype=np.int64) * H - offs[:-1]).to(dev)
            idx = torch.arange(T, dtype=torch.int64, device=dev) + torch.repeat_interleave(
                start, torch.from_numpy(lengths).to(dev), output_size=T)
            L = _lib.lib()
            st = _lib.stream_ptr()
            for name, pad, k, dt in pads:
                dst = _STAGING.device_slot(name, T * k, dt, dev) if reuse else \
                    torch.empty(T * k, dtype=torch.float32 if dt == np.float32 else torch.float64, device=dev)
                if T:
                    _lib.check(L.mjrl_gather_rows(_lib.ptr(pad), k * np.dtype(dt).itemsize, _lib.ptr(idx), T,
                                                  _lib.ptr(dst), st), "mjrl_gather_rows")
                out[name] = dst.view(T, k) if k > 1 else dst
        obs, act, rew = out["obs"], out["act"], out["rew"]
        if self.pred_pad is not None:
            base = out["base"]
        elif not self.linear and self.baseline is not None:
            # another baseline: its own predict per path, as DeviceBatch.from_paths
            # (process_samples.py:23)
            base = stage("base", [self.baseline.predict(p) for p in paths], 0)
        else:
            base = _STAGING.device_slot("base", T, np.float64, dev) if reuse else \
                torch.empty(T, dtype=torch.float64, device=dev)
            base.zero_()
        b = DeviceBatch(obs, act, rew, base, off, term, obs_range=orange)
        b.lengths = lengths
        b.obs_inexact = bool(self.flag[0])
        self.done = True
        return b
