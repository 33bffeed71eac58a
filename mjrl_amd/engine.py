"""Device-side update engine: one NPG / TRPO / DAPG / vanilla-PG update over a
trajectory batch resident in HBM, driven through the C ABI (include/mjrl_amd.h).

Everything between the batch and the host readback at the end is stream-ordered
device work: no host synchronisation inside the CG loop (a device `done` flag
replaces cg_solve's early break, mjrl/utils/cg_solve.py:19-20).  With a
torch.distributed group every rank runs this on its own shard of paths and the
sums listed in mjrl_amd/comm.py are all-reduced (RCCL) between the kernels.

Reference this replaces: mjrl/algos/npg_cg.py:84-165 (NPG.train_from_paths),
mjrl/algos/trpo.py:54-145, mjrl/algos/dapg.py:54-141,
mjrl/algos/batch_reinforce.py:106-164, mjrl/utils/process_samples.py:3-44.
"""
import ctypes as C
import functools
import math
import os

import time

import numpy as np
import torch

from . import _lib
from ._capture import capture
from .comm import LocalComm

# slots (doubles) in the per-update stats buffer; each moments result takes 8 (6
# used).  Layout for the sharded collectives: [0, 32) the advantage / path-return
# moment records all-gathered as one block (mjrl_moments_combine), [32, 40) the
# surr_before moments then the two eval sums (one contiguous all-reduce),
# [40, 56) DAPG's w moments (one all-gathered record).
S_M1, S_M2, S_PM1, S_PM2, S_MS, S_EVAL, S_MW1, S_MW2 = 0, 8, 16, 24, 32, 38, 40, 48
N_STATS = 64


def _thread_safe_predict(baseline):
    """numpy baselines predict in parallel threads; torch-module baselines do not."""
    return type(baseline).__name__ in ("QuadraticBaseline", "ZeroBaseline", "LinearBaseline")


def _linear_coeffs(baseline, n):
    """Coefficients when `baseline` is a LinearBaseline (mjrl's or ours: same
    features, baselines/linear_baseline.py:10-18) — None before its first fit —
    or False when predict must run on the host."""
    if baseline is None or type(baseline).__name__ != "LinearBaseline" or not hasattr(baseline, "_coeffs"):
        return False
    c = baseline._coeffs
    if c is None:
        return None
    return c if len(c) == n + 4 else False


def _host_threads(cap=16):
    """Host threads for staging: the CPUs this process may actually use — its
    affinity set capped by the cgroup CPU quota (a container's affinity can list
    the whole machine while its quota is a fraction of it) — at most `cap` (16
    for one GPU's staging; the pool controller, which converts every GPU's shard,
    passes 16 per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:   # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:   # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota:
        n = min(n, max(1, int(quota)))
    return max(1, min(int(cap), n))


def host_stage(arrs, view, offs, a0, a1, lo=None, hi=None, extras=None):
    """Arrays a0 .. a1 - 1 of `arrs` into their rows offs[i]:offs[i+1] of `view`
    (a pinned host array), converted to view's dtype; with lo / hi (float32 [n])
    the column ranges of what was written are folded in.  f64 / f32 arrays go
    through the native one-pass convert-and-range loop (mjrl_host_stage_* of the
    host-only lib/libmjrl_stage.so: AVX-512 with streaming stores; ctypes
    releases the GIL), anything else through numpy.

    extras (float32 2-D views only): dict(coeffs=f64 [n+4] or None, pred=f64
    host array over the rows of the first `npred` arrays, npred=, flag=int32 [1])
    — the LinearBaseline prediction of every row of arrays < npred, in fp64 from
    the sampler's own values, and flag[0] = 1 when any value is not a float32
    (mjrl_host_stage_paths_f64x).  Sources that are not C-contiguous f64 are
    converted to it first, so the extras always come from the values as given."""
    fns = None
    if view.dtype == np.float32 and view.ndim == 2:
        L = _lib.stage_lib()
        fns = {np.dtype(np.float64): L.mjrl_host_stage_f64, np.dtype(np.float32): L.mjrl_host_stage_f32}
        # the common case, every array of the chunk C-contiguous f64 of the view's
        # width: one native call for the whole chunk
        srcs = [np.asarray(arrs[i]) for i in range(a0, a1)]
        n = view.shape[1]
        if extras is not None:
            srcs = [np.ascontiguousarray(a.reshape(a.shape[0], -1) if a.ndim > 2 else a, dtype=np.float64)
                    for a in srcs]
        if srcs and all(a.dtype == np.float64 and a.ndim == 2 and a.shape[1] == n and a.flags.c_contiguous
                        and a.shape[0] == offs[i + 1] - offs[i] for i, a in zip(range(a0, a1), srcs)):
            k = len(srcs)
            ptrs = (C.c_void_p * k)(*[a.ctypes.data for a in srcs])
            rows = (C.c_int64 * k)(*[a.shape[0] for a in srcs])
            dst = view[offs[a0]:offs[a1]]
            rng = (None if lo is None else lo.ctypes.data, None if hi is None else hi.ctypes.data)
            if dst.shape[0] and extras is None:
                _lib.check(L.mjrl_host_stage_paths_f64(ptrs, rows, k, n, dst.ctypes.data, *rng), "mjrl_host_stage")
            elif dst.shape[0]:
                npred = max(0, min(a1, int(extras["npred"])) - a0)
                c = extras.get("coeffs")
                withp = c is not None and npred > 0
                _lib.check(L.mjrl_host_stage_paths_f64x(
                    ptrs, rows, k, n, dst.ctypes.data, *rng, c.ctypes.data if withp else None,
                    extras["pred"][offs[a0]:].ctypes.data if withp else None, npred if withp else 0,
                    extras["flag"].ctypes.data), "mjrl_host_stage")
            return
        if extras is not None:
            raise ValueError("host_stage extras: observation arrays of a path do not match the staged width %d" % n)
    elif a1 > a0:
        # other slots (1-D rewards / offsets / flags, f64 observations): one
        # numpy concatenate per chunk (a copyto per path cost ~25 us each: 25 ms
        # summed over the 1000 reward arrays of a 1M-row batch)
        srcs = [np.asarray(arrs[i]) for i in range(a0, a1)]
        if all(a.dtype == view.dtype and a.shape[1:] == view.shape[1:] and a.shape[0] == offs[i + 1] - offs[i]
               for i, a in zip(range(a0, a1), srcs)):
            dst = view[offs[a0]:offs[a1]]
            if lo is None and dst.flags.c_contiguous and all(a.flags.c_contiguous for a in srcs):
                # one native call per chunk (ctypes releases the GIL; np.concatenate
                # holds it across the chunk's per-array work)
                k = len(srcs)
                ptrs = (C.c_void_p * k)(*[a.ctypes.data for a in srcs])
                nb = (C.c_int64 * k)(*[a.nbytes for a in srcs])
                _lib.check(_lib.stage_lib().mjrl_host_gather(ptrs, nb, k, dst.ctypes.data), "mjrl_host_gather")
                return
            np.concatenate(srcs, out=dst)
            if lo is not None and view.ndim == 2 and offs[a1] > offs[a0]:
                dst = view[offs[a0]:offs[a1]]
                np.fmin(lo, np.nanmin(dst, axis=0), out=lo)
                np.fmax(hi, np.nanmax(dst, axis=0), out=hi)
            return
    for i in range(a0, a1):
        dst = view[offs[i]:offs[i + 1]]
        if dst.shape[0] == 0:
            continue
        src = np.asarray(arrs[i])
        fn = fns.get(src.dtype) if fns is not None else None
        if fn is not None and src.ndim == 2 and src.shape == dst.shape and src.flags.c_contiguous:
            rc = fn(src.ctypes.data, dst.shape[0], dst.shape[1], dst.ctypes.data,
                    None if lo is None else lo.ctypes.data, None if hi is None else hi.ctypes.data)
            _lib.check(rc, "mjrl_host_stage")
            continue
        np.copyto(dst, src.reshape(dst.shape), casting="unsafe")
        if lo is not None:
            np.fmin(lo, np.nanmin(dst, axis=0) if dst.shape[0] else lo, out=lo)
            np.fmax(hi, np.nanmax(dst, axis=0) if dst.shape[0] else hi, out=hi)


def host_stage_lo(arrs, view, offs, a0, a1):
    """The low halves float32(x - float32(x)) of arrays a0 .. a1 - 1 (f64 [rows, n])
    into their rows of `view` (float32 [R, n]): mjrl_host_stage_lo_paths_f64."""
    srcs = [np.ascontiguousarray(np.asarray(arrs[i]).reshape(len(arrs[i]), -1), dtype=np.float64)
            for i in range(a0, a1)]
    dst = view[offs[a0]:offs[a1]]
    if not srcs or not dst.shape[0]:
        return
    k = len(srcs)
    ptrs = (C.c_void_p * k)(*[a.ctypes.data for a in srcs])
    rows = (C.c_int64 * k)(*[a.shape[0] for a in srcs])
    _lib.check(_lib.stage_lib().mjrl_host_stage_lo_paths_f64(ptrs, rows, k, view.shape[1], dst.ctypes.data),
               "mjrl_host_stage_lo_paths_f64")


class _PinnedStaging:
    """Host -> HBM staging of sampler paths.

    Per slot (obs, act, rewards, ...) a grow-only pinned host buffer and, for
    reuse=True callers, a grow-only device buffer, reused across batches so a
    training loop pays no multi-GB allocation per train_step.  The rows are cut
    into chunks of paths; a thread pool converts / concatenates each chunk
    straight into the pinned buffer (np.copyto releases the GIL; f64 -> f32 for
    the policy inputs), and each chunk's H2D copy is issued on a copy stream as
    soon as that chunk is done, so the conversion of later chunks overlaps the
    PCIe transfer of earlier ones.  The caller's current stream waits on the copy
    stream.  A pinned slot is rewritten only after its previous copies completed;
    a reused device slot only after the work already queued on the current
    stream (which may still read the previous batch) completed."""

    CHUNK_BYTES = 16 << 20   # tools/staging_probe.py: 1M x 376 f32 obs 31.8 ms at 16 MB vs 39.6 at 64 (fill 26.7 || H2D 26.2)

    def __init__(self):
        self._host = {}
        self._dev = {}
        self._ev = {}
        self._pool = None
        self._copy = {}
        # a list to record per-chunk host fill times and device copy events into
        # (bench.py's e2e timeline), or None
        self.trace = None

    def pool(self):
        if self._pool is None:
            import concurrent.futures as cf
            self._pool = cf.ThreadPoolExecutor(_host_threads(), thread_name_prefix="mjrl_stage")
        return self._pool

    def _copy_stream(self, device):
        st = self._copy.get(device)
        if st is None:
            st = self._copy[device] = torch.cuda.Stream(device=device)
        return st

    def device_slot(self, slot, numel, dtype, device):
        """A reused device buffer of `numel` elements (no host data)."""
        tdt = torch.float64 if dtype == np.float64 else torch.float32
        nbytes = numel * np.dtype(dtype).itemsize
        d = self._dev.get(slot)
        if d is None or d.numel() < max(nbytes, 1) or d.device != torch.device(device):
            d = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
            self._dev[slot] = d
        return d[:nbytes].view(tdt)

    def stage_host(self, slot, src, device, reuse=False):
        """A host array that is already the concatenation, in its final dtype (a
        pool worker's shared-memory view, registered as pinned memory with
        register_host), copied to a device tensor of the same shape in chunks on
        the copy stream: no conversion pass and no pinned staging copy."""
        tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}[src.dtype]
        nbytes = src.nbytes
        if reuse:
            d = self._dev.get(slot)
            if d is None or d.numel() < max(nbytes, 1) or d.device != torch.device(device):
                d = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
                self._dev[slot] = d
            out = d[:nbytes].view(tdt).view(src.shape)
        else:
            out = torch.empty(src.shape, dtype=tdt, device=device)
        if nbytes == 0:
            return out
        cur = torch.cuda.current_stream(device)
        cs = self._copy_stream(device)
        cs.wait_stream(cur)
        hflat = torch.from_numpy(src.reshape(-1).view(np.uint8))
        oflat = out.view(-1).view(torch.uint8)
        with torch.cuda.stream(cs):
            for b0 in range(0, nbytes, self.CHUNK_BYTES):
                b1 = min(nbytes, b0 + self.CHUNK_BYTES)
                oflat[b0:b1].copy_(hflat[b0:b1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cs)
        self._ev["pre:" + slot] = ev   # the host array may be rewritten only after this
        cur.wait_stream(cs)
        return out

    def wait_host(self, slot):
        """Blocks until the last copies out of the host array stage_host(slot)
        was given completed."""
        ev = self._ev.get("pre:" + slot)
        if ev is not None:
            ev.synchronize()

    def stage(self, slot, arrs, ncols, dtype, device, reuse=False, ranges=False, extras=None, low=False):
        """Concatenation of `arrs` (each [rows] or [rows, ncols]) as a device
        tensor [R] / [R, ncols] of `dtype` (np.float32 / np.float64 / np.int64 /
        np.uint8).  ranges=True (float32 [R, ncols] slots): also the per-column
        (min, max) of the staged values, taken in the same conversion pass, as
        self.last_range (two float32 [ncols] arrays).  extras (float32 [R, ncols]
        slots of f64 observations): dict(coeffs=LinearBaseline coefficients or
        None, npred=number of leading arrays to predict) — the same pass also
        computes their fp64 baseline predictions (staged to the device slot
        'base', after the rows) and whether every value was a float32:
        self.last_extras = dict(pred=device f64 [rows of the first npred arrays]
        or None, inexact=bool).  low=True (float32 [R, ncols] of f64 arrays): the
        rows' low halves instead (host_stage_lo), for the device fit's f32 pair."""
        dtype = np.dtype(dtype)
        rows = [int(a.shape[0]) for a in arrs]
        R = sum(rows)
        width = max(ncols, 1)
        nbytes = R * width * dtype.itemsize
        ev = self._ev.get(slot)
        if ev is not None:
            ev.synchronize()
        h = self._host.get(slot)
        if h is None or h.numel() < nbytes:
            h = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
            self._host[slot] = h
        tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
               np.dtype(np.int64): torch.int64, np.dtype(np.uint8): torch.uint8}[dtype]
        shape = (R, ncols) if ncols else (R,)
        if reuse:
            d = self._dev.get(slot)
            if d is None or d.numel() < max(nbytes, 1) or d.device != torch.device(device):
                d = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
                self._dev[slot] = d
            out = d[:nbytes].view(tdt).view(shape)
        else:
            out = torch.empty(shape, dtype=tdt, device=device)
        view = h[:nbytes].numpy().view(dtype).reshape(shape)
        if R == 0:
            if ranges and ncols:
                self.last_range = (np.full(width, np.inf, np.float32), np.full(width, -np.inf, np.float32))
            if extras is not None:
                self.last_extras = dict(pred=None, inexact=False)
            return out
        cur = torch.cuda.current_stream(device)
        cs = self._copy_stream(device)
        cs.wait_stream(cur)   # a reused device slot may still be read by queued work
        # chunks of whole arrays of about CHUNK_BYTES each, and at least two per
        # staging thread (a narrow slot, e.g. the actions, in a few 16 MB chunks
        # left most threads idle: 10.5 ms for 68 MB, tools/stage_convert_probe.py)
        cb = max(1 << 20, min(self.CHUNK_BYTES, nbytes // (2 * _host_threads())))
        bounds, acc, r0 = [0], 0, 0
        for i, r in enumerate(rows):
            acc += r * width * dtype.itemsize
            if acc >= cb:
                bounds.append(i + 1)
                acc = 0
        if bounds[-1] != len(rows):
            bounds.append(len(rows))
        offs = np.concatenate([[0], np.cumsum(rows)])

        ranges = ranges and dtype == np.float32 and bool(ncols)
        nchunk = len(bounds) - 1
        rng = np.empty((nchunk, 2, width), dtype=np.float32) if ranges else None
        if ranges:
            rng[:, 0] = np.inf
            rng[:, 1] = -np.inf

        tr = self.trace
        fill_t = [None] * nchunk
        xs = None
        if extras is not None:
            c = extras.get("coeffs")
            npred = int(extras["npred"])
            Tp = int(offs[npred])
            pv = None
            if c is not None and Tp:
                hp = self._host.get(slot + ":pred")
                if hp is None or hp.numel() < Tp * 8:
                    hp = self._host[slot + ":pred"] = torch.empty(Tp * 8, dtype=torch.uint8, pin_memory=True)
                pv = hp[:Tp * 8].numpy().view(np.float64)
            flags = np.zeros((nchunk, 1), np.int32)
            xs = [dict(coeffs=None if pv is None else np.ascontiguousarray(c, dtype=np.float64), pred=pv,
                       npred=npred, flag=flags[k]) for k in range(nchunk)]

        def fill(k):
            t0 = time.perf_counter() if tr is not None else 0.0
            if low:
                host_stage_lo(arrs, view, offs, bounds[k], bounds[k + 1])
            else:
                host_stage(arrs, view, offs, bounds[k], bounds[k + 1],
                           *((rng[k, 0], rng[k, 1]) if ranges else (None, None)), extras=None if xs is None else xs[k])
            if tr is not None:
                fill_t[k] = (t0, time.perf_counter())

        ex = self.pool()
        futs = [ex.submit(fill, k) for k in range(nchunk)]
        hflat = h[:nbytes]
        oflat = out.view(-1).view(torch.uint8)
        row_bytes = width * dtype.itemsize
        with torch.cuda.stream(cs):
            for k, f in enumerate(futs):
                f.result()
                b0, b1 = offs[bounds[k]] * row_bytes, offs[bounds[k + 1]] * row_bytes
                if b1 > b0:
                    if tr is not None:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(cs)
                    oflat[b0:b1].copy_(hflat[b0:b1], non_blocking=True)
                    if tr is not None:
                        e1.record(cs)
                        tr.append(dict(slot=slot, bytes=int(b1 - b0), fill=fill_t[k], issue=time.perf_counter(),
                                       ev=(e0, e1)))
            if xs is not None:
                pred = None
                if xs[0]["pred"] is not None:
                    pv = xs[0]["pred"]
                    if reuse:
                        pred = self.device_slot("base", pv.shape[0], np.float64, device)
                    else:
                        pred = torch.empty(pv.shape[0], dtype=torch.float64, device=device)
                    pred.copy_(torch.from_numpy(pv), non_blocking=True)
                self.last_extras = dict(pred=pred, inexact=bool(flags.any()))
        ev = torch.cuda.Event()
        ev.record(cs)
        self._ev[slot] = ev
        cur.wait_stream(cs)
        if ranges:
            self.last_range = (rng[:, 0].min(axis=0), rng[:, 1].max(axis=0))
        return out


_STAGING = _PinnedStaging()


def register_host(arr):
    """hipHostRegister of a host array's memory (a pool worker's shared-memory
    segment): H2D copies out of it then run as DMA at full PCIe rate.  Returns
    an unregister callable (None when the runtime refuses: the copies stay
    correct, only staged by the driver)."""
    import ctypes as C
    lib = _hip_runtime()
    ptr = C.c_void_p(arr.ctypes.data)
    if lib.hipHostRegister(ptr, C.c_size_t(arr.nbytes), C.c_uint(0)) != 0:
        return None
    return lambda: lib.hipHostUnregister(ptr)


_HIP = None


def _hip_runtime():
    """The HIP runtime torch loaded (torch/lib/libamdhip64.so)."""
    global _HIP
    if _HIP is None:
        import ctypes as C
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        _HIP = C.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        _HIP.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
        _HIP.hipHostRegister.restype = C.c_int
        _HIP.hipHostUnregister.argtypes = [C.c_void_p]
        _HIP.hipHostUnregister.restype = C.c_int
    return _HIP


class _NoEvent:
    """Stand-in timing event for graph captures that cannot hold event records."""
    def record(self, stream=None):
        pass

    def elapsed_time(self, other):
        return float("nan")


def _on_device(fn):
    """Runs an UpdateEngine method with self.device current, so torch's current
    stream (the one every kernel is launched on, _lib.stream_ptr) belongs to the
    device that holds the workspace, whatever device the caller has current."""
    @functools.wraps(fn)
    def wrapped(self, *args, **kwargs):
        with torch.cuda.device(self.device):
            return fn(self, *args, **kwargs)
    return wrapped


class DeviceBatch:
    """One shard of trajectories in HBM — the hot path's input.

    obs / act: f64 [T_all][n] / [T_all][m], the T RL rows (path order) followed by
    T_demo demonstration rows (DAPG).  rewards, baseline: f64 [T].  path_off:
    i64 [P+1] row offsets; terminated: u8 [P].  advantages (optional, f64 [T]):
    when given, the GAE scan is skipped (train_from_paths semantics)."""

    def __init__(self, obs, act, rewards, baseline, path_off, terminated, advantages=None, T_demo=0, obs_range=None):
        self.obs, self.act = obs, act
        # f32 [2][n] per-column (min, max) of the staged observations, taken by the
        # host staging pass (mjrl_host_stage_*): the split rows' column scales come
        # from it (mjrl_obs_colscale_range) instead of a device pass over obs
        self.obs_range = obs_range
        self.T_global = None   # all-rank row count, cached by a sharded update
        self.rewards, self.baseline = rewards, baseline
        self.path_off, self.terminated = path_off, terminated
        self.advantages = advantages
        # True when obs holds float32 images of values that are not all float32s
        # (set by from_paths; the device LinearBaseline fit then reads obs_lo too)
        self.obs_inexact = False
        self.T_demo = int(T_demo)
        self.T = int(obs.shape[0]) - self.T_demo
        self.P = int(path_off.shape[0]) - 1
        self.lengths = None   # host copy, set by from_paths

    @classmethod
    def from_paths(cls, paths, device, baseline=None, use_advantages=False, demo_paths=None, obs_dtype=np.float32,
                   reuse=False, pre=None):
        """Stages sampler-format paths (mjrl/samplers/base_sampler.py:76-83) into HBM.

        The concatenation (npg_cg.py:87-89) goes straight into pinned host
        buffers, chunk by chunk on a thread pool, each chunk's H2D copy overlapping
        the conversion of the next (_PinnedStaging).  obs_dtype: the staged
        observations / actions — np.float32 (default: the policy's own input
        precision, gaussian_mlp.py:103, half the PCIe bytes) or np.float64 (the
        sampler's values unchanged, as the value baseline sees them on the host).
        A device LinearBaseline predict / fit reads the staged observations.
        reuse: stage into the engine-wide grow-only device buffers (one batch
        alive at a time; stable addresses, so hipGraph replay applies).
        pre: dict(obs=, act=, obs_range=) — the observations / actions of `paths`
        already concatenated in obs_dtype in (registered) host memory, with their
        column ranges: copied as they are (a pool worker's shared segment).
        Baseline predictions of other baselines come from the caller's baseline
        object, per path, as compute_advantages does (process_samples.py:23)."""
        with torch.cuda.device(device):
            return cls._from_paths(paths, device, baseline, use_advantages, demo_paths, np.dtype(obs_dtype), reuse,
                                   pre)

    @classmethod
    def _from_paths(cls, paths, device, baseline, use_advantages, demo_paths, obs_dtype, reuse, pre=None):
        lengths = np.array([len(p["rewards"]) for p in paths], dtype=np.int64)
        T = int(lengths.sum())
        n = paths[0]["observations"].shape[1]
        m = paths[0]["actions"].shape[1]
        dlen = [len(p["observations"]) for p in (demo_paths or [])]
        T_demo = int(sum(dlen))

        def stage(slot, arrs, ncols, dtype=np.float64, ranges=False, extras=None):
            return _STAGING.stage(slot, arrs, ncols, dtype, device, reuse, ranges=ranges, extras=extras)

        # slot after slot: each stage() returns once its copies are issued, so the
        # next slot's conversion overlaps the previous slot's H2D tail (one chunked
        # pipeline for all three slots measured 52 ms against 32.5 ms this way,
        # tools/staging_ab.py, profiles/r03f/staging_ab.txt)
        orange = None
        coeffs = _linear_coeffs(baseline, n) if not use_advantages else False
        hpred, inexact = None, False
        if pre is not None and not demo_paths and pre["obs"].dtype == obs_dtype and pre["obs"].shape == (T, n):
            obs = _STAGING.stage_host("obs", pre["obs"], device, reuse)
            act = _STAGING.stage_host("act", pre["act"], device, reuse)
            if obs_dtype == np.float32 and pre.get("obs_range") is not None:
                orange = stage("orange", [np.stack(pre["obs_range"]).astype(np.float32)], n, np.float32)
            # a pool controller's fill (pool._fill_shard) made the same f64 predictions
            # and exactness check as the extras below
            inexact = bool(pre.get("inexact", False))
            if pre.get("pred") is not None and coeffs is not False and coeffs is not None:
                hpred = stage("base", [pre["pred"]], 0)
        else:
            # f32 rows of f64 sampler observations: the same pass computes the
            # LinearBaseline predictions from the f64 values (a4, fp64 as the
            # reference) and notes whether any value is not a float32 (the fit then
            # stages the low halves, DeviceBatch.obs_lo)
            xt = dict(coeffs=coeffs if coeffs is not False else None, npred=len(paths)) \
                if obs_dtype == np.float32 else None
            obs = stage("obs", [p["observations"] for p in paths] + [p["observations"] for p in demo_paths or []], n,
                        obs_dtype, ranges=obs_dtype == np.float32, extras=xt)
            if xt is not None:
                hpred, inexact = _STAGING.last_extras["pred"], _STAGING.last_extras["inexact"]
            if obs_dtype == np.float32:
                orange = stage("orange", [np.stack(_STAGING.last_range)], n, np.float32)
            act = stage("act", [p["actions"] for p in paths] + [p["actions"] for p in demo_paths or []], m,
                        obs_dtype)
        rew = stage("rew", [p["rewards"] for p in paths], 0)
        off = stage("off", [np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)], 0, np.int64)
        term = stage("term", [np.array([bool(p.get("terminated", False)) for p in paths], dtype=np.uint8)], 0,
                     np.uint8)
        if use_advantages:
            base = None
            adv = stage("adv", [p["advantages"] for p in paths], 0)
        elif coeffs is not False and hpred is not None:
            base = hpred   # the host pass's fp64 predictions (linear_baseline.py:46-49)
            adv = None
        elif coeffs is not False:
            # LinearBaseline.predict on the device (a4), reading the staged obs
            # (f64 staging: the sampler's values; before the first fit: zeros)
            base = _STAGING.device_slot("base", T, np.float64, device) if reuse else \
                torch.empty(T, dtype=torch.float64, device=device)
            base.zero_()
            if coeffs is not None and T > 0:
                c = torch.from_numpy(np.ascontiguousarray(coeffs, dtype=np.float64)).to(device)
                fn = _lib.lib().mjrl_linear_baseline_f32 if obs.dtype == torch.float32 else \
                    _lib.lib().mjrl_linear_baseline
                _lib.check(fn(_lib.ptr(obs), T, n, _lib.ptr(off), len(paths), _lib.ptr(c), _lib.ptr(base),
                              _lib.stream_ptr()), "mjrl_linear_baseline")
            adv = None
        elif hasattr(baseline, "predict_device"):
            # MLPBaseline: one device forward over every staged row
            base = baseline.predict_device(obs, off, lengths)
            adv = None
        else:
            preds = list(_STAGING.pool().map(
                lambda p: baseline.predict(p) if baseline is not None else np.zeros(len(p["rewards"])), paths)) \
                if baseline is not None and _thread_safe_predict(baseline) else \
                [baseline.predict(p) if baseline is not None else np.zeros(len(p["rewards"])) for p in paths]
            base = stage("base", preds, 0)
            adv = None
        b = cls(obs, act, rew, base, off, term, advantages=adv, T_demo=T_demo, obs_range=orange)
        b.lengths = lengths
        b.obs_inexact = inexact
        if pre is not None and pre.get("obs_lo") is not None and inexact:
            b._obs_lo = pre["obs_lo"]   # the controller's low halves, copied on first use
        return b

    def obs_lo(self, paths=None, reuse=True):
        """The low halves float32(x - float32(x)) of the RL rows' observations
        (float32 [T, n] on the device) when they were staged as float32 from
        values that are not all float32s, else None: with obs they give the
        device LinearBaseline fit the sampler's f64 values to 2^-48.  Staged on
        first use from `paths` (the batch's own RL paths) on the staging threads."""
        if not self.obs_inexact or self.obs.dtype != torch.float32:
            return None
        lo = getattr(self, "_obs_lo_dev", None)
        if lo is not None:
            return lo
        src = getattr(self, "_obs_lo", None)
        dev = self.obs.device
        with torch.cuda.device(dev):
            if src is not None:   # host float32 [T, n] (a pool segment)
                lo = _STAGING.stage_host("obs_lo", src, dev, reuse)
            else:
                if paths is None or sum(len(p["rewards"]) for p in paths) != self.T:
                    raise ValueError("DeviceBatch.obs_lo needs the batch's RL paths")
                lo = _STAGING.stage("obs_lo", [p["observations"] for p in paths], self.obs.shape[1], np.float32, dev,
                                    reuse, low=True)
        self._obs_lo_dev = lo
        return lo


# the forward pass assembles the split rows itself where it can (UpdateEngine._fused_pack)
FUSED_PACK = os.environ.get("MJRL_AMD_FUSED_PACK", "1") != "0"
TRPO_DEVICE_TRIALS = int(os.environ.get("MJRL_AMD_TRPO_DEVICE_TRIALS", "4"))   # see UpdateEngine.trpo_device_trials
GRAPH_AUTO_ROWS = 300_000   # UpdateEngine.graphs == "auto": replay graphs up to this many rows (125k-row shard: 2.03 -> 1.97 ms; 1M rows: eager 4 % faster)
HIDDEN_WIDTHS = (32, 64, 128, 256)   # hidden widths the row kernels are built for


def kernel_hidden(n, m, hidden):
    """The (h0, h1) the device kernels run a policy of this shape on.

    MuNet(n, m, (h0, h1)) (mjrl/policies/gaussian_mlp.py:143-158) takes any two
    hidden sizes; the kernels are built for square layers of width 32, 64, 128
    or 256, so a policy is zero-padded to the smallest such square that holds
    both layers: padded units have zero weights and biases, so tanh(0) = 0 flows
    nowhere, their gradients and Fisher rows are exactly zero, and the update of
    the real parameters is unchanged.  Raises ValueError for shapes no kernel
    covers (more than two hidden layers, a layer wider than 256, act_dim > 64)."""
    if m < 1 or m > 64:
        raise ValueError("mjrl_amd kernels support act_dim 1..64, got %d" % m)
    if n < 1:
        raise ValueError("obs_dim must be positive")
    if hidden is None or tuple(hidden) == (0, 0):
        return (0, 0)
    hidden = tuple(int(h) for h in hidden)
    if len(hidden) != 2 or min(hidden) < 1:
        raise ValueError("the Gaussian MLP has two hidden layers (gaussian_mlp.py:143-158), got %r" % (hidden,))
    for w in HIDDEN_WIDTHS:
        if max(hidden) <= w:
            return (w, w)
    raise ValueError("mjrl_amd kernels support hidden sizes up to %d, got %r" % (HIDDEN_WIDTHS[-1], hidden))


def padded_positions(n, m, hidden, kh):
    """Index in the flat parameter vector of the padded (kh) policy of every
    entry of the real flat vector (trainable_params order, gaussian_mlp.py:61-64)."""
    h0, h1 = hidden
    p0, p1 = kh
    o_b0 = p0 * n
    o_w1 = o_b0 + p0
    o_b1 = o_w1 + p1 * p0
    o_w2 = o_b1 + p1
    o_b2 = o_w2 + m * p1
    o_ls = o_b2 + m
    parts = [(np.arange(h0)[:, None] * n + np.arange(n)[None, :]).ravel(),
             o_b0 + np.arange(h0),
             (o_w1 + np.arange(h1)[:, None] * p0 + np.arange(h0)[None, :]).ravel(),
             o_b1 + np.arange(h1),
             (o_w2 + np.arange(m)[:, None] * p1 + np.arange(h1)[None, :]).ravel(),
             o_b2 + np.arange(m),
             o_ls + np.arange(m)]
    return np.concatenate(parts).astype(np.int64)


class UpdateEngine:
    """Owns the HBM workspace for one policy shape and runs updates on it."""

    def __init__(self, n, m, hidden, device=None, comm=None, min_log_std=-3.0, precision=None):
        """precision: 'split' runs the K = obs first layer of the MLP(64,64) passes as
        split-f16 MFMA (hi*hi + hi*lo + lo*hi, f32 accumulate), 'f32'
        on exact-f32 MFMA; default (None / 'auto', or $MJRL_AMD_PRECISION): split
        wherever the kernels support it (mjrl_split_supported), f32 elsewhere."""
        self.lib = _lib.lib()
        real = (0, 0) if hidden is None else (int(hidden[0]), int(hidden[1]))
        kh = kernel_hidden(int(n), int(m), hidden)
        self.shape = _lib.make_shape(int(n), int(m), *kh)
        self.device = torch.device(device if device is not None else "cuda")
        self.hidden = real
        self.pad_idx = None   # real flat index -> padded flat index (None: the kernels run the real shape)
        if kh != real:
            self.pad_idx = torch.from_numpy(padded_positions(int(n), int(m), real, kh)).to(self.device)
            self._pad_bufs = {}
        self.comm = comm or LocalComm()
        self.min_log_std = float(min_log_std)
        self.cap_T = -1
        self.cap_P = -1
        s = self.shape
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.packed_theta = torch.zeros(s.packed, **f32)
        self.packed_new = torch.zeros(s.packed, **f32)
        self.packed_p = torch.zeros(s.packed, **f32)
        self.pvec = {k: torch.zeros(s.d, **f32) for k in ("g", "gsum", "x", "r", "r2", "p", "p2", "z", "theta_new")}
        self.cg = torch.zeros(_lib.CG_STATE, **f32)   # MJRL_CG_STATE
        self.done = torch.zeros(1, dtype=torch.int32, device=dev)
        self.out = torch.zeros(_lib.STEP_OUT, **f32)     # MJRL_STEP_OUT (results + step scratch)
        self.stats = torch.zeros(N_STATS, dtype=torch.float64, device=dev)
        self.mom_part = torch.zeros(4 * 256 + 16, dtype=torch.float64, device=dev)
        self.mom2_part = torch.zeros(_lib.MOM_SCRATCH, dtype=torch.float64, device=dev)   # one-launch moments
        self.transforms = (None, None, None, None)
        self._act_rows = None   # set per update: the batch's f32 actions when the row passes read them in place
        # the device TRPO line search: trials per launch sequence (0: the host loop only),
        # its state (MJRL_LS_STATE floats) and skip flag
        self.trpo_device_trials = TRPO_DEVICE_TRIALS
        self.ls_state = torch.zeros(_lib.LS_STATE, **f32)
        self.ls_skip = torch.zeros(1, dtype=torch.int32, device=dev)
        # sharded schedule (one rank of several, or a one-rank communicator forced
        # onto it): moments through one all-gather + mjrl_moments_combine, an
        # all-reduce between every FVP's gather and its CG step
        self.sharded = bool(getattr(self.comm, "sharded", self.comm.world_size > 1))
        self.gbuf = torch.zeros(max(self.comm.world_size, 1) * 32, dtype=torch.float64, device=dev)
        self.kernel_timing = None   # list -> (start, accumulate done, gather done) events per FVP
        # capture / replay whole updates as hipGraphs (one process): True, False, or
        # "auto" = only for batches of at most GRAPH_AUTO_ROWS rows, where launch
        # gaps matter (measured: 12.5k rows 0.59 vs 0.70 ms eager; 125k rows equal;
        # 1M rows the replay is 4 % slower than eager)
        self.graphs = "auto"
        self._gstate = {}
        self.gae_mode = os.environ.get("MJRL_AMD_GAE", "serial")   # "serial" (exact) or "scan"
        self.fused = bool(self.lib.mjrl_fused_path(C.byref(self.shape)))
        prec = precision or os.environ.get("MJRL_AMD_PRECISION", "auto")
        if prec not in ("auto", "split", "f32"):
            raise ValueError("precision must be 'auto', 'split' or 'f32', got %r" % (prec,))
        can_split = bool(self.lib.mjrl_split_supported(C.byref(self.shape)))
        if prec == "split" and not can_split:
            raise ValueError("split precision is not available for this policy shape")
        self.split = can_split and prec != "f32"
        self.precision = "split" if self.split else "f32"   # the form the policy products compute in

    # ------------------------------------------------------------------
    @property
    def vec(self):
        """The update's flat vectors (g, x, theta_new, ...) in the policy's own
        (real) parameter order; copies when the kernels run a padded shape."""
        if self.pad_idx is None:
            return self.pvec
        return {k: t[self.pad_idx] for k, t in self.pvec.items()}

    @property
    def d(self):
        return self.shape.d if self.pad_idx is None else int(self.pad_idx.numel())

    def _pad(self, t, slot):
        """A real flat vector scattered into a persistent zero-padded buffer."""
        if self.pad_idx is None:
            return t
        b = self._pad_bufs.get(slot)
        if b is None:
            b = self._pad_bufs[slot] = torch.zeros(self.shape.d, dtype=torch.float32, device=self.device)
        b.index_copy_(0, self.pad_idx, t.to(torch.float32))
        return b

    def _unpad(self, t):
        return t if self.pad_idx is None else t[self.pad_idx]

    # ------------------------------------------------------------------
    def set_transformations(self, in_shift=None, in_scale=None, out_shift=None, out_scale=None):
        """MuNet.set_transformations (gaussian_mlp.py:160-174), as f32 device vectors."""
        def dv(v):
            return None if v is None else torch.from_numpy(np.float32(np.asarray(v))).to(self.device)
        ins, isc = dv(in_shift), dv(in_scale)
        if (ins is None) != (isc is None):   # the kernel needs both; defaults are 0 / 1
            ins = ins if ins is not None else torch.zeros(self.shape.n, dtype=torch.float32, device=self.device)
            isc = isc if isc is not None else torch.ones(self.shape.n, dtype=torch.float32, device=self.device)
        new = (ins, isc, dv(out_shift), dv(out_scale))
        # the same device buffers when the set of given vectors is unchanged (the
        # agents re-apply the policy's transformations before every update): stable
        # addresses keep a captured update graph valid
        old = self.transforms
        if all((a is None) == (b is None) and (a is None or a.shape == b.shape) for a, b in zip(old, new)):
            for a, b in zip(old, new):
                if a is not None:
                    a.copy_(b)
            return
        self.transforms = new

    def _ensure(self, T_all, P):
        if T_all <= self.cap_T and P <= self.cap_P:
            return
        s = self.shape
        T_all = max(T_all, 1)
        P = max(P, 1)
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        f64 = dict(dtype=torch.float64, device=dev)
        self.ws = {}
        # workspace generation: part of the update-graph key (an id() of a freed dict
        # can come back for the next workspace)
        self._ws_gen = getattr(self, "_ws_gen", 0) + 1
        if hasattr(self, "_gstate"):
            self._gstate.clear()   # a captured graph reads the old workspace
        w = self.ws
        if self.split:
            # split-f16 rows [hi np | lo np] + power-of-two row and column scales
            # (mjrl_rows.xs / xu / xc)
            w["xs"] = torch.empty((T_all, 2 * s.np), dtype=torch.float16, device=dev)
            w["xu"] = torch.empty(T_all, **f32)
            w["xc"] = torch.empty(s.np, **f32)
        else:
            w["xhat"] = torch.empty((T_all, s.np), **f32)
        w["act32"] = torch.empty((T_all, s.m), **f32)
        w["ret"] = torch.empty(T_all, **f64)
        w["adv64"] = torch.empty(T_all, **f64)
        w["w64"] = torch.empty(T_all, **f64)
        w["path_ret"] = torch.empty(P, **f64)
        w["adv32"] = torch.empty(T_all, **f32)
        w["adv_vpg"] = torch.empty(T_all, **f32)
        h0 = max(s.h0, 1)
        h1 = max(s.h1, 1)
        w["a0"] = torch.empty((T_all, h0), **f32)
        w["a1"] = torch.empty((T_all, h1), **f32)
        w["gu0"] = torch.empty((T_all, h0), **f32)
        w["gu1"] = torch.empty((T_all, h1), **f32)
        w["mu0"] = torch.empty((T_all, s.m), **f32)
        w["ll0"] = torch.empty(T_all, **f32)
        w["gp"] = torch.empty((T_all, s.mp), **f32)
        wf, rd, sl = C.c_int64(), C.c_int64(), C.c_int32()
        _lib.check(self.lib.mjrl_scratch_size(C.byref(s), T_all, C.byref(wf), C.byref(rd), C.byref(sl)),
                   "mjrl_scratch_size")
        w["wpart"] = torch.empty(max(wf.value, 1), **f32)
        w["rpart"] = torch.zeros(max(rd.value, 1), **f64)
        self.scratch_slices = sl.value
        self.cap_T, self.cap_P = T_all, P

    def _scratch(self, T, ws=None):
        """Scratch of a pass over T rows, in ws (default: the main workspace; the
        caller guarantees ws holds mjrl_scratch_size(T)'s wpart / rpart)."""
        ws = self.ws if ws is None else ws
        wf, rd, sl = C.c_int64(), C.c_int64(), C.c_int32()
        self.lib.mjrl_scratch_size(C.byref(self.shape), T, C.byref(wf), C.byref(rd), C.byref(sl))
        sc = _lib.Scratch()
        sc.wpart = ws["wpart"].data_ptr()
        sc.rpart = ws["rpart"].data_ptr()
        sc.slices = sl.value
        return sc

    def _rows(self, T, adv_vpg):
        w = self.ws
        r = _lib.Rows()
        r.T = T
        for k, key in (("act", "act32"), ("adv", "adv32"), ("a0", "a0"), ("a1", "a1"),
                       ("mu0", "mu0"), ("ll0", "ll0"), ("gu0", "gu0"), ("gu1", "gu1"), ("gp", "gp")):
            setattr(r, k, w[key].data_ptr())
        if self._act_rows is not None:   # the batch's own f32 actions (no copy into act32)
            r.act = self._act_rows.data_ptr()
        if self.split:
            r.xs, r.xu, r.xc = w["xs"].data_ptr(), w["xu"].data_ptr(), w["xc"].data_ptr()
        else:
            r.xhat = w["xhat"].data_ptr()
        r.adv_vpg = adv_vpg.data_ptr()
        return r

    def _stat(self, slot, n=3):
        return self.stats[slot:slot + n]

    def _moments(self, x, N, out_slot, center_slot=None, f32=False, reduce=True):
        fn = self.lib.mjrl_moments_f32 if f32 else self.lib.mjrl_moments
        center = None if center_slot is None else C.c_void_p(self.stats[center_slot:].data_ptr())
        _lib.check(fn(_lib.ptr(x), N, center, _lib.ptr(self.mom_part),
                      C.c_void_p(self.stats[out_slot:].data_ptr()), self.st), "mjrl_moments")
        if reduce:
            self.comm.allreduce_sum(self._stat(out_slot))

    def _reduce_stats(self, a, b):
        """SUM all-reduce of the contiguous stats slots [a, b) (sharded only)."""
        if self.sharded:
            self.comm.allreduce_sum(self.stats[a:b])

    def _sharded_moments(self, base, rec, ngroups, st):
        """The local pass-1 / pass-2 records at stats[base:base+rec] of every rank
        all-gathered in ONE collective and folded into the global moments in place
        (mjrl_moments_combine)."""
        W = self.comm.world_size
        g = self.gbuf[:W * rec]
        self.comm.allgather(self.stats[base:base + rec], g)
        _lib.check(self.lib.mjrl_moments_combine(_lib.ptr(g), W, rec, ngroups,
                                                 C.c_void_p(self.stats[base:].data_ptr()), st),
                   "mjrl_moments_combine")

    def _fused_pack(self, batch, T_all, T_vpg):
        """Whether this update's forward pass assembles the split rows itself
        (mjrl_policy_vpg_pack: the pack's read and write of the whole batch saved):
        split rows, f32 observations [T_all][n] 16-byte aligned with n % 4 == 0, the
        identity input normalisation, a forward pass over every staged row.
        MJRL_AMD_FUSED_PACK=0 turns it off (A/B runs)."""
        o = batch.obs
        return (self.split and FUSED_PACK and o.dtype == torch.float32 and batch.act.dtype == torch.float32
                and self.transforms[0] is None and self.shape.n % 4 == 0 and o.is_contiguous()
                and o.data_ptr() % 16 == 0 and T_vpg == T_all and o.dim() == 2 and o.shape[0] >= T_all)

    def _colscale(self, obs, T, st, obs_range=None):
        """The split rows' power-of-two column scales of this batch (w['xc']):
        from the staged per-column ranges (no pass over obs), or a device pass."""
        w = self.ws
        ins, isc, _, _ = self.transforms
        sp = C.byref(self.shape)
        if obs_range is not None:
            _lib.check(self.lib.mjrl_obs_colscale_range(_lib.ptr(obs_range[0]), _lib.ptr(obs_range[1]), sp,
                                                        _lib.ptr(ins), _lib.ptr(isc), _lib.ptr(w["xc"]), st),
                       "mjrl_obs_colscale_range")
        else:
            cs = self.lib.mjrl_obs_colscale_f32 if obs.dtype == torch.float32 else self.lib.mjrl_obs_colscale
            _lib.check(cs(_lib.ptr(obs), T, sp, _lib.ptr(ins), _lib.ptr(isc), _lib.ptr(w["xc"]), st),
                       "mjrl_obs_colscale")

    def _pack(self, obs, act, T, st, obs_range=None):
        """a5 batch assembly: f64 obs / act -> the row format the policy passes read.
        obs_range: the staged batch's per-column (min, max) (DeviceBatch.obs_range),
        from which the split rows' column scales follow without a pass over obs."""
        w = self.ws
        ins, isc, _, _ = self.transforms
        sp = C.byref(self.shape)
        f32 = obs.dtype == torch.float32
        if f32 != (act.dtype == torch.float32):
            raise ValueError("observations and actions must be staged in the same dtype")
        if self.split:
            # column scales of this batch, then the split rows
            self._colscale(obs, T, st, obs_range)
            fn = self.lib.mjrl_pack_batch_split_f32 if f32 else self.lib.mjrl_pack_batch_split
            _lib.check(fn(_lib.ptr(obs), _lib.ptr(act), T, sp, _lib.ptr(ins), _lib.ptr(isc), _lib.ptr(w["xc"]),
                          _lib.ptr(w["xs"]), _lib.ptr(w["xu"]), _lib.ptr(w["act32"]), st), "mjrl_pack_batch_split")
        else:
            fn = self.lib.mjrl_pack_batch_f32 if f32 else self.lib.mjrl_pack_batch
            _lib.check(fn(_lib.ptr(obs), _lib.ptr(act), T, sp, _lib.ptr(ins), _lib.ptr(isc), _lib.ptr(w["xhat"]),
                          _lib.ptr(w["act32"]), st), "mjrl_pack_batch")

    # ------------------------------------------------------------------
    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    @_on_device
    def returns_advantages(self, batch, gamma, gae_lambda, stream=None):
        """process_samples.compute_returns + compute_advantages on device (a1-a3).
        Leaves f64 returns / advantages in ws['ret'] / ws['adv64'].  `stream`: run on
        that HIP stream (update() overlaps the scan with the batch assembly)."""
        st = stream if stream is not None else _lib.stream_ptr()
        if stream is None:
            self.st = st
        self._ensure(batch.T + batch.T_demo, batch.P)
        w = self.ws
        use_gae = not (gae_lambda is None or gae_lambda < 0.0 or gae_lambda > 1.0)
        base = self._baseline_of(batch)
        # "serial": discount_sum's operation order bit for bit (the default); "scan":
        # the wave-parallel scan (regrouped products, ~1e-14 relative)
        fn = self.lib.mjrl_gae_scan if self.gae_mode == "scan" else self.lib.mjrl_gae
        _lib.check(fn(
            _lib.ptr(batch.rewards), _lib.ptr(base), _lib.ptr(batch.path_off), _lib.ptr(batch.terminated),
            batch.P, float(gamma), float(gae_lambda) if use_gae else 0.0, int(use_gae),
            _lib.ptr(w["ret"]), _lib.ptr(w["adv64"]), _lib.ptr(w["path_ret"]), st), "mjrl_gae")
        return w["ret"][:batch.T], w["adv64"][:batch.T]

    @staticmethod
    def _baseline_of(batch):
        """The batch's baseline predictions; a missing one becomes zeros, allocated
        on the current stream and kept on the batch (update() calls this before its
        side stream forks, so the scan never reads the buffer before the fill)."""
        if batch.baseline is None:
            batch.baseline = torch.zeros_like(batch.rewards)
        return batch.baseline

    @_on_device
    def normalize_advantages(self, T):
        """The `normalize` option of compute_advantages (process_samples.py:14-19,30-35)."""
        w = self.ws
        self._moments(w["adv64"], T, S_M1)
        self._moments(w["adv64"], T, S_M2, center_slot=S_M1)
        _lib.check(self.lib.mjrl_whiten(_lib.ptr(w["adv64"]), T, C.c_void_p(self.stats[S_M1:].data_ptr()),
                                        C.c_void_p(self.stats[S_M2:].data_ptr()), 1e-8, None,
                                        _lib.ptr(w["w64"]), self.st), "mjrl_whiten")
        return w["w64"][:T]

    @_on_device
    def update(self, batch, theta, *, algo="npg", gamma=0.995, gae_lambda=0.98, n_step_size=0.01,
               const_lr=None, kl_dist=None, cg_iters=10, damping=1e-4, residual_tol=1e-10,
               demo_coef=None, learn_rate=0.01, T_global=None, trpo_verbose=True, skip_gae=False,
               hvp_sample_frac=None, graph=None):
        """One policy update.  `theta`: f32 device tensor [d] (flat params, reference
        order).  algo in {'npg', 'trpo', 'dapg', 'vpg'}.

        npg:  alpha = sqrt(|delta/(g.x)|), delta = n_step_size (or const_lr)  npg_cg.py:128-141
        trpo: delta = 2 kl_dist + KL backtracking                              trpo.py:98-124
        dapg: g = (T_all/T) vpg(all rows), delta = 2 kl_dist                   dapg.py:62-121
        vpg:  theta + learn_rate * g (BatchREINFORCE)                          batch_reinforce.py:134-145
        hvp_sample_frac < 0.99: each Fisher-vector product runs on its own draw of
        np.random.choice(T_global, int(frac T_global)) rows from numpy's global RNG
        (npg_cg.py:58-62); rank 0 draws, the draw is broadcast, and after the update
        the RNG is left where the reference's early-exiting CG would leave it.
        graph (default self.graphs): replay a captured hipGraph of the update when
        the batch, shape and arguments repeat (npg / vpg / dapg, one process, no
        subsampled Fisher; TRPO's line search continues on the host after the
        replayed graph, which ends at the first evaluation; see _maybe_capture).
        Returns host scalars plus the new device theta (self.vec['theta_new'])."""
        L = self.lib
        s = self.shape
        self.st = st = _lib.stream_ptr()
        theta = self._pad(theta, "theta")
        T, T_demo, P = batch.T, batch.T_demo, batch.P
        T_all = T + T_demo
        # global row count (all ranks): scales every mean; one host round trip per
        # staged batch, cached on it (outside any captured graph)
        if T_global is None and self.comm.world_size > 1:
            T_global = batch.T_global
            if T_global is None:
                tg = torch.tensor([float(T)], dtype=torch.float64, device=self.device)
                self.comm.allreduce_sum(tg)
                T_global = batch.T_global = float(tg.item())
        elif T_global is None:
            T_global = float(T)
        sharded = self.sharded
        sub = None
        if hvp_sample_frac is not None and hvp_sample_frac < 0.99 and algo != "vpg":
            sub = self._hvp_draws(float(hvp_sample_frac), int(round(T_global)), T, int(cg_iters))
        # a subsampled Fisher's rows live in ws_sub (_subsample_rows), so the main
        # workspace keeps its size and the GAE outputs already in it
        self._ensure(T_all, P)
        w = self.ws
        v = self.pvec
        sp = C.byref(s)
        ins, isc, osh, osc = self.transforms
        want = self.graphs if graph is None else graph
        if want == "auto":
            # sharded: always (the graph holds the collectives too, no host launch
            # or collective-call overhead between the latency-bound steps)
            want = T_all <= GRAPH_AUTO_ROWS or sharded
        use_graph = (bool(want) and (self.comm.world_size == 1 or getattr(self.comm, "capturable", False))
                     and sub is None and algo in ("npg", "vpg", "dapg", "trpo"))
        if use_graph:
            key = self._graph_key(batch, T_global, (algo, gamma, gae_lambda, n_step_size, const_lr, kl_dist, cg_iters,
                                                    damping, residual_tol, learn_rate, skip_gae, demo_coef))
            gs = self._gstate
            if gs.get("graph") is not None and gs["key"] == key:
                # replay: the whole update is one graph launch; theta enters through
                # the captured input buffer
                gs["theta_in"].copy_(theta)
                gs["graph"].replay()
                self.last_T, self.last_T_global = T, T_global
                trials = []
                if algo == "trpo":   # the graph ends at the first evaluation; the search stays on the host
                    trials = self._trpo_search(gs["plan"], gs["delta"], kl_dist, trpo_verbose, gs["timing"])
                return self._finish(algo, const_lr, gs["delta"], T_global, None, trials, gs["timing"])

        def launch(theta, ev):
            """Every device launch of the update up to the first evaluation (the
            TRPO line search continues on the host); `ev` makes timing events.
            Under graph capture the current stream is the capture stream."""
            st = _lib.stream_ptr()
            self.st = st
            timing = [ev() for _ in range(4)]

            # a1-a3: returns / advantages.  The scan is a serial fp64 chain per path
            # (latency-bound, few waves): it runs on a side stream beside the HBM-bound
            # batch assembly and joins before the moments.
            main = torch.cuda.current_stream(self.device)
            side = self._side_stream()
            self._baseline_of(batch)
            side.wait_stream(main)
            adv64 = w["adv64"]
            if batch.advantages is not None:
                adv64 = batch.advantages
                # path returns still come from the rewards (npg_cg.py:97)
                self.returns_advantages(batch, gamma, None, stream=C.c_void_p(side.cuda_stream))
            elif not skip_gae:
                self.returns_advantages(batch, gamma, gae_lambda, stream=C.c_void_p(side.cuda_stream))
            # a5: batch assembly (f64 -> f32, input normalisation, bias column); fused
            # into the forward pass below when it can be (_fused_pack): then only the
            # column scales and the f32 actions here
            fused = self._fused_pack(batch, T_all, T_all if (algo == "dapg" and demo_coef is not None) else T)
            self._act_rows = None
            if fused:
                self._colscale(batch.obs, T_all, st, batch.obs_range)
                if batch.act.dtype == torch.float32 and batch.act.is_contiguous() and tuple(batch.act.shape) == (
                        T_all, s.m):
                    # f32 staging: the row passes read the staged actions where they are
                    # (a [T][m] copy into act32 cost ~30 us per 1M-row update)
                    self._act_rows = batch.act
                else:
                    w["act32"][:T_all].copy_(batch.act[:T_all])
            else:
                self._pack(batch.obs, batch.act, T_all, st, batch.obs_range)
            main.wait_stream(side)
            # whitening (npg_cg.py:91) and path-return statistics (npg_cg.py:97-102):
            # two-pass fp64 moments, both quantities in one launch per pass; when
            # sharded, each pass's sums share one all-reduce (plus one MAX for the
            # path-return extrema)
            # (sharded: both passes local — pass 2 about this rank's own mean — then
            # one all-gather of the four records and mjrl_moments_combine)
            sp_ = lambda slot: C.c_void_p(self.stats[slot:].data_ptr())
            mp2 = _lib.ptr(self.mom2_part)
            dapg = algo == "dapg" and demo_coef is not None
            _lib.check(L.mjrl_moments2(_lib.ptr(adv64), T, None, _lib.ptr(w["path_ret"]), P, None, mp2,
                                       sp_(S_M1), sp_(S_PM1), st), "mjrl_moments2")
            _lib.check(L.mjrl_moments2(_lib.ptr(adv64), T, sp_(S_M1), _lib.ptr(w["path_ret"]), P, sp_(S_PM1),
                                       mp2, sp_(S_M2), sp_(S_PM2), st), "mjrl_moments2")
            if sharded:
                self._sharded_moments(S_M1, 32, 2, st)
            # whitening + surr_before = mean(LR * adv) with LR == 1 (npg_cg.py:113) in one
            # launch; the surr_before all-reduce rides with the first post-step evaluation's
            _lib.check(L.mjrl_whiten_moments(_lib.ptr(adv64), T, sp_(S_M1), sp_(S_M2), 1e-6,
                                             _lib.ptr(w["adv32"]), _lib.ptr(w["w64"]) if dapg else None, mp2,
                                             sp_(S_MS), st), "mjrl_whiten_moments")
            ms_pending = [True]
            if dapg:
                _lib.check(L.mjrl_moments2(_lib.ptr(w["w64"]), T, None, None, 0, None, mp2, sp_(S_MW1), None, st),
                           "mjrl_moments2")
                _lib.check(L.mjrl_moments2(_lib.ptr(w["w64"]), T, sp_(S_MW1), None, 0, None, mp2, sp_(S_MW2), None, st),
                           "mjrl_moments2")
                if sharded:
                    self._sharded_moments(S_MW1, 16, 1, st)
                _lib.check(L.mjrl_dapg_adv(_lib.ptr(w["w64"]), T, C.c_void_p(self.stats[S_MW1:].data_ptr()),
                                           C.c_void_p(self.stats[S_MW2:].data_ptr()), T_demo, float(demo_coef),
                                           _lib.ptr(w["adv_vpg"]), st), "mjrl_dapg_adv")
                adv_vpg = w["adv_vpg"]
                T_vpg = T_all
            else:
                adv_vpg = w["adv32"]
                T_vpg = T
            inv_T = 1.0 / T_global
            self.last_T, self.last_T_global = T, T_global

            # a6-a11: forward + VPG (caches a0, a1, mu0, ll0)
            _lib.check(L.mjrl_pack_params(sp, _lib.ptr(theta), _lib.ptr(self.packed_theta), 1, self.min_log_std, st),
                       "mjrl_pack_params")
            sc = self._scratch(T_vpg)
            rows = self._rows(T_vpg, adv_vpg)
            timing[0].record()
            if fused:
                _lib.check(L.mjrl_policy_vpg_pack(sp, C.byref(rows), _lib.ptr(batch.obs), _lib.ptr(self.packed_theta),
                                                  _lib.ptr(osh), _lib.ptr(osc), C.byref(sc), _lib.ptr(v["gsum"]), st),
                           "mjrl_policy_vpg_pack")
            else:
                _lib.check(L.mjrl_policy_vpg(sp, C.byref(rows), _lib.ptr(self.packed_theta), _lib.ptr(osh),
                                             _lib.ptr(osc), C.byref(sc), _lib.ptr(v["gsum"]), st), "mjrl_policy_vpg")
            self.comm.allreduce_sum(v["gsum"])
            if algo == "vpg":
                _lib.check(L.mjrl_scale_vec(_lib.ptr(v["gsum"]), s.d, inv_T, _lib.ptr(v["g"]), st), "mjrl_scale_vec")
            # (otherwise g = gsum / T is formed by the CG initialisation below, in the same launch)
            timing[1].record()

            # a12-a13: conjugate gradient with the device FVP
            rows_fvp = self._rows(T, adv_vpg)
            sc_fvp = self._scratch(T) if T_vpg != T else sc
            if algo == "vpg":
                x = v["g"]
                cg_iters_run = 0
            else:
                _lib.check(L.mjrl_cg_init_scaled(sp, _lib.ptr(v["gsum"]), inv_T, _lib.ptr(v["g"]), _lib.ptr(v["x"]),
                                                 _lib.ptr(v["r"]), _lib.ptr(v["p"]), _lib.ptr(self.packed_p),
                                                 _lib.ptr(self.cg), _lib.ptr(self.done), st), "mjrl_cg_init_scaled")
                prof = self.kernel_timing
                inv_T_fvp = inv_T if sub is None else 1.0 / max(sub["Ts"], 1)
                # gather + CG z fused when no all-reduce sits between them and the CG
                # state holds one p.z partial per 64 parameters
                cg_zx = (s.d + 63) // 64 <= (_lib.CG_STATE - _lib.CG_PZ_PARTS) // 2
                fuse_cg = not sharded and cg_zx
                for k in range(int(cg_iters)):
                    rows_k, sc_k, T_k = rows_fvp, sc_fvp, T
                    if sub is not None:
                        rows_k, sc_k, T_k = self._subsample_rows(sub, k, adv_vpg)
                    if prof is not None:
                        e0, e1, e2 = (ev() for _ in range(3))
                        e0.record()
                    _lib.check(L.mjrl_fvp_accumulate(sp, C.byref(rows_k), T_k, _lib.ptr(self.packed_theta),
                                                     _lib.ptr(self.packed_p), _lib.ptr(osc), _lib.ptr(self.done),
                                                     C.byref(sc_k), st), "mjrl_fvp_accumulate")
                    if prof is not None:
                        e1.record()
                    if fuse_cg:
                        # one process: the slab gather and the z step of the CG iteration in one launch
                        _lib.check(L.mjrl_gather_cg_z(sp, C.byref(rows_k), T_k, C.byref(sc_k), _lib.ptr(self.done),
                                                      _lib.ptr(v["gsum"]), inv_T_fvp, float(damping),
                                                      _lib.ptr(self.packed_theta), _lib.ptr(v["p"]), _lib.ptr(v["z"]),
                                                      _lib.ptr(self.cg), st), "mjrl_gather_cg_z")
                    else:
                        _lib.check(L.mjrl_gather_grads(sp, C.byref(rows_k), T_k, C.byref(sc_k), 0, _lib.ptr(self.done),
                                                       _lib.ptr(v["gsum"]), st), "mjrl_gather_grads")
                    if prof is not None:
                        e2.record()
                        prof.append((e0, e1, e2))
                    if fuse_cg:
                        # the rest of the iteration in one launch; r alternates between two buffers
                        r_in, r_out = (v["r"], v["r2"]) if k % 2 == 0 else (v["r2"], v["r"])
                        _lib.check(L.mjrl_cg_step_xr_p(sp, _lib.ptr(v["x"]), _lib.ptr(r_in), _lib.ptr(r_out),
                                                       _lib.ptr(v["p"]), _lib.ptr(v["z"]), _lib.ptr(self.packed_p),
                                                       _lib.ptr(self.cg), _lib.ptr(self.done), float(residual_tol), st),
                                   "mjrl_cg_step_xr_p")
                        continue
                    self.comm.allreduce_sum(v["gsum"])
                    if cg_zx:
                        # z + p.z partials from the reduced sum, then the one-process iteration tail
                        _lib.check(L.mjrl_cg_z(sp, _lib.ptr(v["gsum"]), inv_T_fvp, float(damping),
                                               _lib.ptr(self.packed_theta), _lib.ptr(v["p"]), _lib.ptr(v["z"]),
                                               _lib.ptr(self.cg), _lib.ptr(self.done), st), "mjrl_cg_z")
                        r_in, r_out = (v["r"], v["r2"]) if k % 2 == 0 else (v["r2"], v["r"])
                        _lib.check(L.mjrl_cg_step_xr_p(sp, _lib.ptr(v["x"]), _lib.ptr(r_in), _lib.ptr(r_out),
                                                       _lib.ptr(v["p"]), _lib.ptr(v["z"]), _lib.ptr(self.packed_p),
                                                       _lib.ptr(self.cg), _lib.ptr(self.done), float(residual_tol),
                                                       st), "mjrl_cg_step_xr_p")
                        continue
                    # the rest of the iteration in one launch; r and p alternate between two buffers each
                    (r_in, r_out), (p_in, p_out) = ((v["r"], v["r2"]), (v["p"], v["p2"])) if k % 2 == 0 else \
                        ((v["r2"], v["r"]), (v["p2"], v["p"]))
                    _lib.check(L.mjrl_cg_step1(sp, _lib.ptr(v["gsum"]), inv_T_fvp, float(damping),
                                               _lib.ptr(self.packed_theta), _lib.ptr(v["x"]), _lib.ptr(r_in),
                                               _lib.ptr(r_out), _lib.ptr(p_in), _lib.ptr(p_out),
                                               _lib.ptr(self.packed_p), _lib.ptr(self.cg), _lib.ptr(self.done),
                                               float(residual_tol), st), "mjrl_cg_step1")
                x = v["x"]
                cg_iters_run = None
            timing[2].record()

            # a14: step size + update; a16 TRPO backtracking.  `plan` holds the
            # buffers the step and the evaluation read (no reference to the engine:
            # a captured graph keeps it for the TRPO search after each replay, and
            # an engine <-> graph cycle would leave the graph's destruction to the
            # cyclic GC, at any later allocation, possibly inside another capture)
            plan = dict(x=x, theta=theta, rows=rows_fvp, sc=sc_fvp, T=T, osh=osh, osc=osc, ms_pending=[True],
                        inv_T=inv_T)
            if algo == "vpg":
                self._step(plan, 1, 0.0, np.float32(learn_rate), 0)
                delta = None
            elif algo == "npg" and const_lr is not None:
                self._step(plan, 1, 0.0, np.float32(const_lr), 1)
                delta = None
            elif algo == "npg":
                delta = n_step_size if kl_dist is None else 2.0 * kl_dist
                self._step(plan, 0, delta, 0.0, 0)
            else:   # trpo / dapg: delta = 2 kl_dist
                delta = 2.0 * kl_dist
                self._step(plan, 0, delta, 0.0, 0)
            self._evaluate(plan)
            if algo == "trpo" and self.trpo_device_trials > 0 and not self.sharded:
                # the first backtracking trials on the device (mjrl_trpo_trial): each
                # tests the last evaluation and, rejected, steps to 0.9 alpha for the
                # next; once one is accepted the rest return at once.  No host round
                # trip per trial, and the whole sequence is part of the captured graph;
                # the host continues past it only when all are rejected (_trpo_search)
                K = int(self.trpo_device_trials)
                for k in range(1, K + 2):
                    _lib.check(L.mjrl_trpo_trial(sp, _lib.ptr(x), _lib.ptr(theta), self.min_log_std,
                                                 _lib.ptr(v["theta_new"]), _lib.ptr(self.packed_new),
                                                 _lib.ptr(self.out), C.c_void_p(self.stats[S_EVAL:].data_ptr()),
                                                 inv_T, float(kl_dist), k, int(k <= K), _lib.ptr(self.ls_state),
                                                 _lib.ptr(self.ls_skip), st), "mjrl_trpo_trial")
                    if k <= K:
                        self._evaluate(plan, skip=self.ls_skip)
                plan["dev_trials"] = K
            if algo != "trpo":
                timing[3].record()
            return plan, delta, timing

        plan, delta, timing = launch(theta, lambda: torch.cuda.Event(enable_timing=True))
        trials = []

        if algo == "trpo":
            trials = self._trpo_search(plan, delta, kl_dist, trpo_verbose, timing)
        result = self._finish(algo, const_lr, delta, T_global, sub, trials, timing)
        if use_graph:
            self._maybe_capture(key, launch, theta, delta, T_global)
        return result

    def _step(self, plan, mode, delta, alpha_in, const):
        """a14: theta_new = theta + alpha x (npg_cg.py:128-141), alpha from the
        step-size rule (mode 0) or given (mode 1), log-std clamp, repack."""
        L = self.lib
        _lib.check(L.mjrl_npg_step(C.byref(self.shape), _lib.ptr(self.pvec["g"]), _lib.ptr(plan["x"]),
                                   _lib.ptr(plan["theta"]), mode, float(delta), float(alpha_in), int(const),
                                   self.min_log_std, _lib.ptr(self.pvec["theta_new"]), _lib.ptr(self.packed_new),
                                   _lib.ptr(self.out), _lib.stream_ptr()), "mjrl_npg_step")

    def _evaluate(self, plan, skip=None):
        """Surrogate and KL at theta_new (npg_cg.py:142-143): one EVAL pass, then
        (sharded) the all-reduce of its sums; the first one carries surr_before's
        moments too.  skip: a device flag that turns the pass into a no-op (the
        device line search's speculative evaluations; one process only)."""
        L = self.lib
        if skip is not None:
            _lib.check(L.mjrl_policy_eval_if(C.byref(self.shape), C.byref(plan["rows"]), plan["T"],
                                             _lib.ptr(self.packed_new), _lib.ptr(self.packed_theta),
                                             _lib.ptr(plan["osh"]), _lib.ptr(plan["osc"]), C.byref(plan["sc"]),
                                             C.c_void_p(self.stats[S_EVAL:].data_ptr()), _lib.ptr(skip),
                                             _lib.stream_ptr()), "mjrl_policy_eval_if")
            return
        _lib.check(L.mjrl_policy_eval(C.byref(self.shape), C.byref(plan["rows"]), plan["T"],
                                      _lib.ptr(self.packed_new), _lib.ptr(self.packed_theta), _lib.ptr(plan["osh"]),
                                      _lib.ptr(plan["osc"]), C.byref(plan["sc"]),
                                      C.c_void_p(self.stats[S_EVAL:].data_ptr()), _lib.stream_ptr()),
                   "mjrl_policy_eval")
        if plan["ms_pending"][0]:
            self._reduce_stats(S_MS, S_EVAL + 2)   # surr_before's moments + the eval sums
            plan["ms_pending"][0] = False
        else:
            self._reduce_stats(S_EVAL, S_EVAL + 2)

    def _trpo_search(self, plan, delta, kl_dist, verbose, timing):
        """TRPO's KL backtracking (trpo.py:98-124) after the first evaluation: alpha
        *= 0.9 while KL >= kl_dist (at most 100 trials), then the final
        re-evaluation at the accepted alpha.  The first trpo_device_trials trials
        ran on the device inside the update's launch sequence (mjrl_trpo_trial): one
        readback of their log here; the host loop takes over only past them (the
        step and the evaluation launch on the current stream, eager, or after a graph
        replay of everything before)."""
        trials = []
        inv_T = plan["inv_T"]
        surr_before = float(self.stats[S_MS].item() / self.stats[S_MS + 2].item())

        def backtrack_msg(kl, surr):
            if verbose:
                print("Step size too high. Backtracking. | kl = %f | surr diff = %f" % (kl, surr - surr_before))

        K = plan.get("dev_trials", 0)
        k0 = 0
        if K:
            ls = self.ls_state.cpu().numpy()
            n, accepted = int(ls[2]), bool(ls[1])
            for t in range(n):
                a, kl, surr = (np.float32(v) for v in ls[_lib.LS_LOG + 3 * t: _lib.LS_LOG + 3 * t + 3])
                trials.append((float(a), float(kl), float(surr)))
                if not (accepted and t == n - 1):
                    backtrack_msg(kl, surr)
            if accepted:
                timing[3].record()
                return trials
            # every device trial rejected: the host steps on from the last one
            alpha = np.float32(0.9 * np.float32(trials[-1][0]))   # trpo.py:114 (python float * np.float32)
            self._step(plan, 1, delta, alpha, 0)
            self._evaluate(plan)
            k0 = n
        else:
            alpha = np.float32(self.out[0].item())
        res = self.stats[S_EVAL:S_EVAL + 2].cpu().numpy()
        for k in range(k0, 100):
            kl = np.float32(res[1] * inv_T)
            surr = np.float32(res[0] * inv_T)
            trials.append((float(alpha), float(kl), float(surr)))
            if kl < kl_dist:
                break
            alpha = np.float32(0.9 * alpha)   # trpo.py:114 (python float * np.float32)
            backtrack_msg(kl, surr)
            if k == 99:
                alpha = np.float32(0.0)
                break
            self._step(plan, 1, delta, alpha, 0)
            self._evaluate(plan)
            res = self.stats[S_EVAL:S_EVAL + 2].cpu().numpy()
        if float(alpha) != trials[-1][0]:   # final re-evaluation (trpo.py:120-123)
            self._step(plan, 1, delta, alpha, 0)
            self._evaluate(plan)
        timing[3].record()
        return trials

    # ------------------------------------------------------------------
    # hipGraph replay of whole updates (one process): the second consecutive
    # update with the same batch buffers, shape and arguments is captured, later
    # ones replay it as ONE graph launch (the ~60 kernel launches of an update
    # then cost no host time and leave no launch gaps).  Theta enters through a
    # captured device buffer; everything else the graph reads is the batch and
    # the engine workspace, whose addresses are part of the key.
    def _graph_key(self, batch, T_global, args):
        ptrs = tuple(0 if t is None else t.data_ptr() for t in (
            batch.obs, batch.act, batch.rewards, batch.baseline, batch.path_off, batch.terminated, batch.advantages,
            batch.obs_range) + tuple(self.transforms))
        return (ptrs, batch.T, batch.T_demo, batch.P, float(T_global), self._ws_gen, self.kernel_timing is not None,
                tuple(args))

    def _maybe_capture(self, key, launch, theta, delta, T_global):
        gs = self._gstate
        if gs.get("seen") != key:          # first sighting: remember, stay eager
            gs.clear()
            gs["seen"] = key
            return
        theta_in = torch.empty_like(theta)
        theta_in.copy_(theta)
        prof_saved = self.kernel_timing
        for ev in (lambda: torch.cuda.Event(enable_timing=True, external=True), _NoEvent):
            if prof_saved is not None:
                self.kernel_timing = []    # the capture's own per-FVP events
            g = torch.cuda.CUDAGraph()
            try:
                with capture(g):
                    out = launch(theta_in, ev)
            except Exception as e:         # timing events inside a capture unsupported: capture without
                err = e
                continue
            finally:
                graph_prof = self.kernel_timing
                self.kernel_timing = prof_saved
            # plan: buffers only (no closure over the engine, see launch())
            gs.update(key=key, graph=g, theta_in=theta_in, timing=out[2], delta=delta, prof=graph_prof, plan=out[0])
            self.st = _lib.stream_ptr()    # launch() cached the capture stream
            return
        import warnings
        warnings.warn("mjrl_amd: hipGraph capture of the update failed (%s); staying eager" % (err,))
        self.graphs = False
        gs.clear()
        self.st = _lib.stream_ptr()

    def graph_kernel_timing(self):
        """(start, accumulate done, gather done) external events of every FVP of the
        captured graph, valid after a replay has completed; None without a graph."""
        return self._gstate.get("prof")

    def _finish(self, algo, const_lr, delta, T_global, sub, trials, timing):
        # single readback: the statistics, the step results and the CG counters in
        # three async copies into one pinned buffer, one synchronisation
        inv_T = 1.0 / T_global
        stats, out, cg = self._readback()
        if sub is not None and sub["rng"] is not None:
            # the reference stops drawing when its CG exits early: replay only the
            # draws of the FVPs that ran, so numpy's global RNG ends in the same state
            np.random.set_state(sub["rng"])
            for _ in range(int(cg[1])):
                np.random.choice(sub["N"], size=sub["Ts"])
        n_p = stats[S_PM1 + 2]
        base_stats = [stats[S_PM1] / n_p, math.sqrt(stats[S_PM2 + 1] / n_p), -stats[S_PM1 + 5], stats[S_PM1 + 4]]
        result = dict(
            alpha=float(out[0]),
            gx=float(out[1]),
            delta=(float(out[2]) if (const_lr is not None and algo == "npg") else delta),
            surr_before=float(np.float32(stats[S_MS] / stats[S_MS + 2])),
            surr_after=float(np.float32(stats[S_EVAL] * inv_T)),
            kl_dist=float(np.float32(stats[S_EVAL + 1] * inv_T)),
            base_stats=base_stats,
            cg_iters=int(cg[1]) if algo != "vpg" else 0,
            trials=trials,
            time_vpg=timing[0].elapsed_time(timing[1]) / 1e3,
            time_npg=timing[1].elapsed_time(timing[2]) / 1e3,
            time_step=timing[2].elapsed_time(timing[3]) / 1e3,
            T_global=T_global,
        )
        if algo == "vpg":
            result["delta"] = None
        return result

    # ------------------------------------------------------------------
    def _readback(self):
        h = getattr(self, "_host_res", None)
        if h is None:
            h = self._host_res = (torch.empty(N_STATS, dtype=torch.float64, pin_memory=True),
                                  torch.empty(8, dtype=torch.float32, pin_memory=True),
                                  torch.empty(8, dtype=torch.float32, pin_memory=True))
        h[0].copy_(self.stats, non_blocking=True)
        h[1].copy_(self.out[:8], non_blocking=True)
        h[2].copy_(self.cg[:8], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return h[0].numpy().copy(), h[1].numpy().copy(), h[2].numpy().copy()

    @_on_device
    def fit_quadratic_baseline(self, batch, baseline, returns=None, return_errors=False, obs_lo=None):
        """QuadraticBaseline.fit (baselines/quadratic_baseline.py:40-65) on the
        batch's rows in HBM: the Gram of its features [o, o_i o_j (i <= j), 1, a ..
        a^4] (o = clip(obs) / 10) with the returns on the device
        (mjrl_quadratic_baseline_gram, n <= 64), then the reference's lstsq retry
        loop; as fit_linear_baseline otherwise."""
        return self.fit_linear_baseline(batch, baseline, returns, return_errors, obs_lo, quadratic=True)

    @_on_device
    def fit_linear_baseline(self, batch, baseline, returns=None, return_errors=False, obs_lo=None, quadratic=False):
        """LinearBaseline.fit (baselines/linear_baseline.py:20-44) on the batch's
        RL rows already in HBM: the Gram products [F y]^T [F y] on the device
        (mjrl_linear_baseline_gram, all-reduced when sharded), then the
        reference's own lstsq retry loop on the k x k system.  `returns`: f64
        device [T] (default: the returns of the last GAE scan).  Sets
        baseline._coeffs; with return_errors, returns (error_before, error_after)
        computed from device residuals as the reference does.  obs_lo: the low
        halves of f32-staged observations (DeviceBatch.obs_lo): the features are
        then formed from hi + lo, the sampler's f64 values to 2^-48."""
        L = self.lib
        st = _lib.stream_ptr()
        n, T, P = int(batch.obs.shape[1]), batch.T, batch.P
        k = n + n * (n + 1) // 2 + 5 if quadratic else n + 4
        y = returns if returns is not None else self.ws["ret"][:T]
        nd = C.c_int64()
        kind = "quadratic" if quadratic else "linear"
        _lib.check(getattr(L, "mjrl_%s_baseline_gram_scratch" % kind)(n, T, C.byref(nd)),
                   "mjrl_%s_baseline_gram_scratch" % kind)
        f64 = dict(dtype=torch.float64, device=self.device)
        scratch = torch.empty(max(nd.value, 1), **f64)
        gram = torch.zeros((k + 1, k + 1), **f64)
        f32 = batch.obs.dtype == torch.float32
        if obs_lo is not None and f32:
            if obs_lo.dtype != torch.float32 or obs_lo.shape[0] < T or obs_lo.shape[1] != n:
                raise ValueError("fit_%s_baseline: obs_lo must be float32 [T, n]" % kind)
        if quadratic and f32:   # one f32 entry, low halves or null
            lo = _lib.ptr(obs_lo) if obs_lo is not None else None
            gram_fn = functools.partial(L.mjrl_quadratic_baseline_gram_f32, _lib.ptr(batch.obs))
            res_fn = functools.partial(L.mjrl_quadratic_baseline_residual_f32, _lib.ptr(batch.obs))
            obs_arg = lo
        elif quadratic:
            gram_fn, res_fn = L.mjrl_quadratic_baseline_gram, L.mjrl_quadratic_baseline_residual
            obs_arg = _lib.ptr(batch.obs)
        elif f32 and obs_lo is not None:
            gram_fn = functools.partial(L.mjrl_linear_baseline_gram_f32x2, _lib.ptr(batch.obs))
            res_fn = functools.partial(L.mjrl_linear_baseline_residual_f32x2, _lib.ptr(batch.obs))
            obs_arg = _lib.ptr(obs_lo)
        else:
            gram_fn = L.mjrl_linear_baseline_gram_f32 if f32 else L.mjrl_linear_baseline_gram
            res_fn = L.mjrl_linear_baseline_residual_f32 if f32 else L.mjrl_linear_baseline_residual
            obs_arg = _lib.ptr(batch.obs)
        _lib.check(gram_fn(obs_arg, _lib.ptr(y), T, n, _lib.ptr(batch.path_off), P,
                           _lib.ptr(scratch), _lib.ptr(gram), st), "mjrl_%s_baseline_gram" % kind)
        self.comm.allreduce_sum(gram)

        def sse(coeffs):
            r = torch.empty(max(T, 1), **f64)
            c = torch.from_numpy(np.ascontiguousarray(coeffs, dtype=np.float64)).to(self.device)
            _lib.check(res_fn(obs_arg, _lib.ptr(y), T, n, _lib.ptr(batch.path_off), P, _lib.ptr(c),
                              _lib.ptr(scratch), _lib.ptr(r), st), "mjrl_%s_baseline_residual" % kind)
            out = torch.zeros(8, **f64)
            part = torch.empty(4 * 256, **f64)
            _lib.check(L.mjrl_moments(_lib.ptr(r), T, None, _lib.ptr(part), _lib.ptr(out), st), "mjrl_moments")
            self.comm.allreduce_sum(out)
            return float(out[1].item())

        G = gram.cpu().numpy()
        FtF, Fty, yy = G[:k, :k], G[:k, k], G[k, k]
        if return_errors:
            err_before = (sse(baseline._coeffs) if baseline._coeffs is not None else yy) / yy
        reg = baseline._reg_coeff
        for _ in range(10):   # linear_baseline.py:31-38, quadratic_baseline.py:51-59
            c = np.linalg.lstsq(FtF + reg * np.identity(k), Fty, rcond=None)[0]
            baseline._coeffs = c
            if not np.any(np.isnan(c)):
                break
            reg *= 10
        if return_errors:
            return err_before, sse(baseline._coeffs) / yy

    def _hvp_draws(self, frac, N, T_local, K):
        """K row draws np.random.choice(N, int(frac N)) (npg_cg.py:58-62) made on
        rank 0, broadcast, and cut to this rank's rows (global index - row offset,
        draw order kept).  One H2D / broadcast for the whole CG solve."""
        Ts = int(frac * N)
        comm = self.comm
        rng = None
        if comm.rank == 0:
            rng = np.random.get_state()
            d = np.stack([np.random.choice(N, size=Ts) for _ in range(K)]) if K else np.zeros((0, Ts))
            idx = torch.from_numpy(np.ascontiguousarray(d, dtype=np.int64)).to(self.device)
        else:
            idx = torch.empty((K, Ts), dtype=torch.int64, device=self.device)
        comm.broadcast(idx)
        if comm.world_size > 1:
            lo = comm.row_offset(T_local, self.device)
            sel = (idx >= lo) & (idx < lo + T_local)
            counts = sel.sum(1).cpu().numpy().astype(np.int64)
            loc = (idx[sel] - lo).contiguous()
        else:
            counts = np.full(K, Ts, dtype=np.int64)
            loc = idx.reshape(-1).contiguous()
        offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        mx = int(counts.max()) if K else 0
        return dict(idx=loc, counts=counts, offs=offs, Ts=Ts, N=N, rng=rng, max=mx)

    def _subsample_rows(self, sub, k, adv_vpg):
        """Compact xhat / a0 / a1 rows of draw k (mjrl_gather_rows) and the Rows /
        Scratch an FVP over them uses."""
        s = self.shape
        n_k = int(sub["counts"][k])
        ip = C.c_void_p(sub["idx"].data_ptr() + 8 * int(sub["offs"][k]))
        w = self.ws
        cap = max(sub["max"], 1)
        f32 = dict(dtype=torch.float32, device=self.device)
        ws = self.__dict__.setdefault("ws_sub", {})
        if "a0s" not in ws or ws["a0s"].shape[0] < cap:
            wf, rd, sl = C.c_int64(), C.c_int64(), C.c_int32()
            _lib.check(self.lib.mjrl_scratch_size(C.byref(s), cap, C.byref(wf), C.byref(rd), C.byref(sl)),
                       "mjrl_scratch_size")
            ws["wpart"] = torch.empty(max(wf.value, 1), **f32)
            ws["rpart"] = torch.zeros(max(rd.value, 1), dtype=torch.float64, device=self.device)
            if self.split:
                ws["xss"] = torch.empty((cap, 2 * s.np), dtype=torch.float16, device=self.device)
                ws["xus"] = torch.empty(cap, **f32)
            else:
                ws["xhs"] = torch.empty((cap, s.np), **f32)
            ws["a0s"] = torch.empty((cap, max(s.h0, 1)), **f32)
            ws["a1s"] = torch.empty((cap, max(s.h1, 1)), **f32)
            # per-row upstream gradients the k_rows FVP writes for k_wgrad
            ws["gu0s"] = torch.empty((cap, max(s.h0, 1)), **f32)
            ws["gu1s"] = torch.empty((cap, max(s.h1, 1)), **f32)
            ws["gps"] = torch.empty((cap, s.mp), **f32)
        pairs = [("xs", "xss", s.np), ("xu", "xus", 1)] if self.split else [("xhat", "xhs", s.np)]
        if s.h0:
            pairs += [("a0", "a0s", s.h0), ("a1", "a1s", s.h1)]
        rows = self._rows(n_k, adv_vpg)
        for src, dst, width in pairs:   # rows of 4 * width bytes (f32, or the f16 hi / lo pair of xs)
            _lib.check(self.lib.mjrl_gather_rows(_lib.ptr(w[src]), 4 * width, ip, n_k, _lib.ptr(ws[dst]), self.st),
                       "mjrl_gather_rows")
            setattr(rows, src, ws[dst].data_ptr())
        rows.gu0, rows.gu1, rows.gp = ws["gu0s"].data_ptr(), ws["gu1s"].data_ptr(), ws["gps"].data_ptr()
        return rows, self._scratch(n_k, ws), n_k

    def accumulate_path(self):
        """Accumulate kernel the dispatcher runs for this shape: 2 = K-split
        persistent (k_ks), 1 = fused persistent (k_fused), 0 = k_rows + k_wgrad."""
        return int(self.lib.mjrl_fused_path(C.byref(self.shape)))

    @_on_device
    def fvp(self, v, damping=1e-4, T=None, idx=None):
        """F v + damping v at the parameters of the last update's forward pass
        (the caches a0/a1/mu0 and packed_theta of that pass) — NPG.HVP
        (npg_cg.py:55-74) as a standalone call, used by parity tests and
        `NPG.HVP`.  `v`: f32 device tensor [d].  `idx` (int64 device tensor):
        the rows of a subsampled Fisher (npg_cg.py:58-62), gathered as in the
        update's CG loop.  Returns a new device tensor."""
        L = self.lib
        s = self.shape
        sp = C.byref(s)
        self.st = st = _lib.stream_ptr()
        T = self.last_T if T is None else T
        vv = self.pvec
        T_global = self.last_T_global
        if idx is not None:
            n = int(idx.numel())
            sub = dict(idx=idx.contiguous(), counts=[n], offs=[0], max=n)
            rows, scratch, T = self._subsample_rows(sub, 0, self.ws["adv32"])
            T_global = float(n)
        else:
            scratch = self._scratch(T)
            rows = self._rows(T, self.ws["adv32"])
        v = self._pad(v, "v")
        _lib.check(L.mjrl_cg_init(sp, _lib.ptr(v), _lib.ptr(vv["x"]), _lib.ptr(vv["r"]), _lib.ptr(vv["p"]),
                                  _lib.ptr(self.packed_p), _lib.ptr(self.cg), _lib.ptr(self.done), st), "mjrl_cg_init")
        _lib.check(L.mjrl_policy_fvp(sp, C.byref(rows), T, _lib.ptr(self.packed_theta), _lib.ptr(self.packed_p),
                                     _lib.ptr(self.transforms[3]), C.byref(scratch), _lib.ptr(self.done),
                                     _lib.ptr(vv["gsum"]), st), "mjrl_policy_fvp")
        self.comm.allreduce_sum(vv["gsum"])
        _lib.check(L.mjrl_cg_step(sp, _lib.ptr(vv["gsum"]), 1.0 / T_global, float(damping),
                                  _lib.ptr(self.packed_theta), _lib.ptr(vv["x"]), _lib.ptr(vv["r"]), _lib.ptr(vv["p"]),
                                  _lib.ptr(vv["z"]), _lib.ptr(self.packed_p), _lib.ptr(self.cg), _lib.ptr(self.done),
                                  0.0, st), "mjrl_cg_step")
        return self._unpad(vv["z"]).clone()

    # ------------------------------------------------------------------
    # standalone passes on explicit arrays (the reference's CPI_surrogate /
    # kl_old_new / flat_vpg / HVP called directly, batch_reinforce.py:37-55,
    # npg_cg.py:55-74); the update above never goes through these.  Local to
    # this process (no collectives).
    @_on_device
    def load_rows(self, obs, act, adv=None):
        """Stages f64 obs / act (and f64 advantages, cast to f32 as
        batch_reinforce.py:38 does) as the current rows."""
        T = int(obs.shape[0])
        self._ensure(T, 1)
        self._act_rows = None   # the rows' actions are act32's from here on
        self.st = st = _lib.stream_ptr()
        dev = self.device
        o = torch.from_numpy(np.ascontiguousarray(obs, dtype=np.float64)).to(dev)
        a = torch.from_numpy(np.ascontiguousarray(act, dtype=np.float64)).to(dev)
        ins, isc, _, _ = self.transforms
        self._pack(o, a, T, st)
        if adv is not None:
            self.ws["adv32"][:T].copy_(torch.from_numpy(np.asarray(adv, dtype=np.float64)).float().to(dev))
        else:
            self.ws["adv32"][:T].zero_()
        return T

    @_on_device
    def forward_pass(self, theta, T):
        """Forward + VPG sums at theta over the loaded rows; fills the caches.
        Returns the flat VPG mean (device) = sum / T."""
        L, s = self.lib, self.shape
        theta = self._pad(theta, "theta")
        sp = C.byref(s)
        self.st = st = _lib.stream_ptr()
        _lib.check(L.mjrl_pack_params(sp, _lib.ptr(theta), _lib.ptr(self.packed_theta), 1, self.min_log_std, st),
                   "mjrl_pack_params")
        rows = self._rows(T, self.ws["adv32"])
        sc = self._scratch(T)
        _, _, osh, osc = self.transforms
        _lib.check(L.mjrl_policy_vpg(sp, C.byref(rows), _lib.ptr(self.packed_theta), _lib.ptr(osh), _lib.ptr(osc),
                                     C.byref(sc), _lib.ptr(self.pvec["gsum"]), st), "mjrl_policy_vpg")
        tg = float(T)
        self.last_T, self.last_T_global = T, tg
        _lib.check(L.mjrl_scale_vec(_lib.ptr(self.pvec["gsum"]), s.d, 1.0 / tg, _lib.ptr(self.pvec["g"]), st),
                   "mjrl_scale_vec")
        return self._unpad(self.pvec["g"])

    @_on_device
    def eval_pass(self, theta_new, T):
        """(surrogate, KL) at theta_new against the caches of the last forward_pass."""
        L, s = self.lib, self.shape
        theta_new = self._pad(theta_new, "theta_new")
        sp = C.byref(s)
        self.st = st = _lib.stream_ptr()
        _lib.check(L.mjrl_pack_params(sp, _lib.ptr(theta_new), _lib.ptr(self.packed_new), 1, self.min_log_std, st),
                   "mjrl_pack_params")
        rows = self._rows(T, self.ws["adv32"])
        sc = self._scratch(T)
        _, _, osh, osc = self.transforms
        _lib.check(L.mjrl_policy_eval(sp, C.byref(rows), T, _lib.ptr(self.packed_new), _lib.ptr(self.packed_theta),
                                      _lib.ptr(osh), _lib.ptr(osc), C.byref(sc),
                                      C.c_void_p(self.stats[S_EVAL:].data_ptr()), st), "mjrl_policy_eval")
        res = self.stats[S_EVAL:S_EVAL + 2].cpu().numpy()
        return np.float32(res[0] / T), np.float32(res[1] / T)


def device_returns_advantages(rewards, baseline, lengths, terminated, gamma, gae_lambda, device=None,
                              normalize=False):
    """compute_returns / compute_advantages (process_samples.py:3-35) on the GPU for
    host arrays; returns f64 numpy (returns, advantages), bit-identical to the
    reference's discount_sum order.  normalize: (adv - mean) / (std + 1e-8) over
    all paths (process_samples.py:14-19, 30-35), two-pass fp64 moments."""
    L = _lib.lib()
    dev = torch.device(device if device is not None else "cuda")
    lengths = np.asarray(lengths, dtype=np.int64)
    T = int(lengths.sum())
    P = len(lengths)
    use_gae = not (gae_lambda is None or gae_lambda < 0.0 or gae_lambda > 1.0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)
    rw = t(rewards, np.float64)
    bl = t(baseline if baseline is not None else np.zeros(T), np.float64)
    off = t(np.concatenate([[0], np.cumsum(lengths)]), np.int64)
    term = t(np.asarray(terminated, dtype=np.uint8), np.uint8)
    ret = torch.empty(max(T, 1), dtype=torch.float64, device=dev)
    adv = torch.empty(max(T, 1), dtype=torch.float64, device=dev)
    pr = torch.empty(max(P, 1), dtype=torch.float64, device=dev)
    _lib.check(L.mjrl_gae(_lib.ptr(rw), _lib.ptr(bl), _lib.ptr(off), _lib.ptr(term), P, float(gamma),
                          float(gae_lambda) if use_gae else 0.0, int(use_gae), _lib.ptr(ret), _lib.ptr(adv),
                          _lib.ptr(pr), _lib.stream_ptr()), "mjrl_gae")
    if normalize and T > 0:
        st = _lib.stream_ptr()
        part = torch.zeros(4 * 256 + 16, dtype=torch.float64, device=dev)
        m = torch.zeros(16, dtype=torch.float64, device=dev)
        out = torch.empty(T, dtype=torch.float64, device=dev)
        _lib.check(L.mjrl_moments(_lib.ptr(adv), T, None, _lib.ptr(part), _lib.ptr(m), st), "mjrl_moments")
        _lib.check(L.mjrl_moments(_lib.ptr(adv), T, _lib.ptr(m), _lib.ptr(part), C.c_void_p(m[8:].data_ptr()), st),
                   "mjrl_moments")
        _lib.check(L.mjrl_whiten(_lib.ptr(adv), T, _lib.ptr(m), C.c_void_p(m[8:].data_ptr()), 1e-8, None,
                                 _lib.ptr(out), st), "mjrl_whiten")
        adv = out
    return ret[:T].cpu().numpy(), adv[:T].cpu().numpy()
