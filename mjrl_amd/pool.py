"""One controller process, N GPU workers: multi-GPU behind an unchanged,
single-process train_agent (SURVEY.md §5, §8 row e).

mjrl's training loop (mjrl/utils/train_agent.py:14-88) is single-process: it
creates the job directories, samples, calls agent.train_step, evaluates and
pickles the policy / baseline / logs.  With `devices` (agent kwarg or
MJRL_AMD_DEVICES="0,1,...,7") the agent keeps ALL of that in the calling process,
which never touches a GPU, and hands each update to N worker processes, one per
GPU, started once:

  controller (train_agent, samplers, pickles)          worker r (cuda:devices[r])
  ---------------------------------------------         --------------------------
  sample N paths (mjrl samplers, host CPUs)
  partition_paths by timestep count; shard r's
  obs / act / rewards / lengths / terminated
  (+ advantages) into shared-memory segment r  --step-->  attach; the agent from its
                                                           pickled state (policy,
                                                           baseline, hyperparameters),
                                                           comm = torch.distributed
                                                           group of the N workers
                                                           (RCCL; gloo in the tests)
                                                           train_from_samples(shard):
                                                           the sharded device update
                                                           with its all-reduces,
                                                           then the baseline fit on
                                                           the union of the shards
  returns / baseline / advantages into the    <--reply--  rank 0: statistics, theta,
  caller's path dicts, policy params, the                  the iteration's log entries,
  iteration's log entries, baseline state,                 baseline state, RNG state;
  numpy RNG state                                          every rank: its shard's
                                                           returns / advantages
                                                           (shared memory)

Every rank ends the update with the same parameters, so rank 0
speaks for all.  The workers are fresh interpreters (`python -m mjrl_amd.pool`,
started with subprocess, not multiprocessing's spawn: a training script without
an `if __name__ == "__main__"` guard is never re-imported) and talk to the
controller over multiprocessing.connection on 127.0.0.1.
"""
import os
import pickle
import secrets
import socket
import subprocess
import sys
import time
import traceback
from multiprocessing import connection, shared_memory

import numpy as np

# agent attributes that stay with the controller / are rebuilt in a worker
_LOCAL = ("env", "logger", "_engine", "_comm", "_last_batch", "_pool", "_devices", "_device", "_backend", "_pre")
# agent attributes a worker's update changes and the controller takes back
_SYNC = ("running_score", "iter_count", "last_update")


def resolve_devices(devices=None):
    """The worker devices of an agent: `devices` (a list of GPU ordinals or a
    count), else MJRL_AMD_DEVICES ("0,1,2,3" or "4"); None for one device (the
    in-process engine)."""
    if devices is None:
        env = os.environ.get("MJRL_AMD_DEVICES", "").strip()
        if not env:
            return None
        devices = [int(d) for d in env.split(",")] if "," in env else int(env)
    if isinstance(devices, int):
        devices = list(range(devices))
    devices = [int(d) for d in devices]
    return devices if len(devices) > 1 else None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Layout:
    """Byte offsets of one shard in its shared-memory segment (64-byte aligned
    fields).  obs / act are in `dtype`: float32 when the agent stages in float32
    (half the bytes; the controller's fill converts them with their column
    ranges, which go in 'orange', so the worker copies the segment to HBM as it
    is), float64 otherwise; the rest float64 / int64."""

    def __init__(self, T, P, n, m, with_adv, dtype=np.float64):
        self.T, self.P, self.n, self.m = T, P, n, m
        self.dtype = dt = np.dtype(dtype)
        f32, f64, i64 = np.dtype(np.float32), np.dtype(np.float64), np.dtype(np.int64)
        off = 0
        self.fields = {}
        x = dt == f32 and not with_adv
        # float32 layouts of sampled paths also carry the controller's f64
        # LinearBaseline predictions ('pred_in'), the low halves of the
        # observations ('obs_lo', written only when some value is not a float32:
        # the untouched pages of a shared segment cost no memory) and two flags
        # ('xflags': [inexact, predictions present])
        for name, count, ft in (("obs", T * n, dt), ("act", T * m, dt), ("orange", 2 * n if dt == f32 else 0, f32),
                                ("pred_in", T if x else 0, f64), ("obs_lo", T * n if x else 0, f32),
                                ("xflags", 2 if x else 0, i64),
                                ("rew", T, f64), ("lengths", P, i64), ("term", P, i64),
                                ("adv_in", T if with_adv else 0, f64), ("ret", T, f64), ("base", T, f64),
                                ("adv", T, f64)):
            self.fields[name] = (off, count, ft)
            off += -(-count * ft.itemsize // 64) * 64
        self.nbytes = max(off, 64)

    def view(self, buf, name):
        off, count, ft = self.fields[name]
        return np.ndarray((count,), dtype=ft, buffer=buf, offset=off)


def _segment_dtype(agent):
    """float32 segments when the agent stages its observations in float32 and
    its baseline predicts and fits from the batch in HBM (the device
    LinearBaseline): nothing in the worker then reads the float64 values.
    Otherwise float64: MLPBaseline builds its features from the path
    observations on the host (clip(o) / 10 in f64, mlp_baseline.py:37-56), which
    float32 views of a segment would round first."""
    f32 = (agent.staging_obs_dtype() if hasattr(agent, "staging_obs_dtype")
           else np.dtype(getattr(agent, "staging_dtype", np.float64))) == np.float32
    dev_fit = type(getattr(agent, "baseline", None)).__name__ == "LinearBaseline"
    return np.float32 if (f32 and dev_fit) else np.float64


def _fill_shard(buf, L, sh, lengths, ex=None, chunk_rows=None, threads=1, coeffs=None):
    """The shard's paths `sh` into its segment.  float32 layouts: the native
    convert-and-range pass (engine.host_stage, the staging path's own) writes
    obs / act and the per-column (min, max) of obs into 'orange'.  ex: a thread
    pool; the paths are then cut into chunks of about chunk_rows timesteps
    (default: two chunks per pool thread, `threads` of them, at least 1024 rows;
    a fixed 64k rows left half of 16 threads idle on a 500k-row shard), converted in parallel
    (ctypes releases the GIL), their ranges folded; the 1-D slots go through the
    same native gather as the staging path's.  Layouts with the 'pred_in' field:
    the same pass makes the f64 LinearBaseline predictions from `coeffs` (None:
    before the first fit) and the exactness check of the staging path
    (engine.host_stage extras), and a second pass the low halves when needed."""
    lengths = np.asarray(lengths, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lengths)])
    if chunk_rows is None:
        chunk_rows = max(1024, int(offs[-1]) // (2 * threads)) if ex is not None and threads > 1 else 1 << 16
    bounds = [0]
    for i in range(len(sh)):
        if offs[i + 1] - offs[bounds[-1]] >= chunk_rows:
            bounds.append(i + 1)
    if bounds[-1] != len(sh):
        bounds.append(len(sh))
    nchunk = len(bounds) - 1
    f32 = L.dtype == np.float32
    rng = np.empty((max(nchunk, 1), 2, L.n), np.float32)
    rng[:, 0], rng[:, 1] = np.inf, -np.inf
    obs_v, act_v = L.view(buf, "obs").reshape(L.T, L.n), L.view(buf, "act").reshape(L.T, L.m)
    if f32:
        from .engine import host_stage, host_stage_lo
    xt = L.fields["pred_in"][1] > 0
    flags = np.zeros((max(nchunk, 1), 1), np.int32)
    pred_v = L.view(buf, "pred_in") if xt else None
    cf = None if coeffs is None else np.ascontiguousarray(coeffs, dtype=np.float64)

    def conv(k):
        a0, a1 = bounds[k], bounds[k + 1]
        if f32:
            host_stage([p["observations"] for p in sh], obs_v, offs, a0, a1, rng[k, 0], rng[k, 1],
                       extras=dict(coeffs=cf, pred=pred_v, npred=len(sh), flag=flags[k]) if xt else None)
            host_stage([p["actions"] for p in sh], act_v, offs, a0, a1)
        else:
            for i in range(a0, a1):
                obs_v[offs[i]:offs[i + 1]] = np.asarray(sh[i]["observations"], np.float64).reshape(-1, L.n)
                act_v[offs[i]:offs[i + 1]] = np.asarray(sh[i]["actions"], np.float64).reshape(-1, L.m)

    if ex is not None and nchunk > 1:
        list(ex.map(conv, range(nchunk)))
    else:
        for k in range(nchunk):
            conv(k)
    if xt:
        inexact = bool(flags.any())
        L.view(buf, "xflags")[:] = (int(inexact), int(cf is not None))
        if inexact:
            lo_v = L.view(buf, "obs_lo").reshape(L.T, L.n)

            def low(k):
                host_stage_lo([p["observations"] for p in sh], lo_v, offs, bounds[k], bounds[k + 1])
            if ex is not None and nchunk > 1:
                list(ex.map(low, range(nchunk)))
            else:
                for k in range(nchunk):
                    low(k)
    if sh:
        from .engine import host_stage
        if f32:
            o = L.view(buf, "orange").reshape(2, L.n)
            o[0], o[1] = rng[:, 0].min(axis=0), rng[:, 1].max(axis=0)
        host_stage([np.asarray(p["rewards"], np.float64) for p in sh], L.view(buf, "rew"), offs, 0, len(sh))
        if L.fields["adv_in"][1]:
            host_stage([np.asarray(p["advantages"], np.float64) for p in sh], L.view(buf, "adv_in"), offs, 0, len(sh))
    L.view(buf, "lengths")[:] = lengths
    L.view(buf, "term")[:] = [int(bool(p.get("terminated", False))) for p in sh]


class DevicePool:
    """N worker processes, one per GPU of `devices`, driven from this process."""

    def __init__(self, devices, backend="nccl", timeout=900.0, connect_timeout=600.0):
        self.devices = list(devices)
        self.world = len(self.devices)
        self.backend = backend
        self.timeout = timeout
        self._shm = [None] * self.world
        self._digests = {}
        self._procs = []
        self._conns = [None] * self.world
        authkey = secrets.token_bytes(16)
        self._listener = connection.Listener(("127.0.0.1", 0), authkey=authkey)
        host, port = self._listener.address
        dist_port = _free_port()
        env = dict(os.environ)
        env["MJRL_AMD_DEVICES"] = ""          # a worker never starts a pool of its own
        # the package's own root first: an import through '' (the caller's cwd)
        # does not survive train_agent's chdir into the job directory
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = os.pathsep.join([root] + [os.path.abspath(p) for p in sys.path if p and os.path.isdir(p)])
        try:
            for r, d in enumerate(self.devices):
                cmd = [sys.executable, "-u", "-m", "mjrl_amd.pool", "--address", "%s:%d" % (host, port),
                       "--authkey", authkey.hex(), "--rank", str(r), "--world", str(self.world), "--device", str(d),
                       "--backend", backend, "--dist-port", str(dist_port)]
                self._procs.append(subprocess.Popen(cmd, env=env))
            self._accept_all(connect_timeout)
            for r in range(self.world):
                msg = self._recv(r)
                if msg[0] != "ready":
                    raise RuntimeError("mjrl_amd pool worker %d failed to start: %s" % (r, msg[1]))
        except BaseException:
            self._abort()
            raise

    def _accept_all(self, connect_timeout):
        """Accepts the workers' connections, polling: a worker that exits before
        it connects ends the wait with a RuntimeError (a blocked accept() is not
        woken by closing its socket from another thread)."""
        import select
        sock = self._listener._listener._socket
        t0 = time.time()
        for _ in range(self.world):
            while not select.select([sock], [], [], 0.25)[0]:
                dead = [r for r, p in enumerate(self._procs) if p.poll() is not None]
                if dead:
                    raise RuntimeError("mjrl_amd pool: worker(s) %s exited before connecting (codes %s)"
                                       % (dead, [self._procs[r].returncode for r in dead]))
                if time.time() - t0 > connect_timeout:
                    raise TimeoutError("mjrl_amd pool: workers did not connect within %.0f s" % connect_timeout)
            c = self._listener.accept()
            rank = c.recv()
            self._conns[rank] = c

    def _abort(self):
        """After any failure: kill every worker (the others may be blocked in a
        collective, or hold a stale reply), unlink the segments, and forget the
        pool, so the next use starts a fresh one."""
        for p in self._procs:
            if p.poll() is None:
                p.kill()
        for p in self._procs:
            try:
                p.wait(timeout=30)
            except Exception:
                pass
        for c in self._conns:
            if c is not None:
                try:
                    c.close()
                except Exception:
                    pass
        self._conns = [None] * self.world
        self._free_segments()
        try:
            self._listener.close()
        except Exception:
            pass
        for k, v in list(_POOLS.items()):
            if v is self:
                del _POOLS[k]

    def _free_segments(self):
        for s in self._shm:
            if s is not None:
                try:
                    s.close()
                    s.unlink()
                except Exception:
                    pass
        self._shm = [None] * self.world

    # ---- plumbing -------------------------------------------------------------
    def _recv(self, r):
        c = self._conns[r]
        t0 = time.time()
        while not c.poll(1.0):
            if self._procs[r].poll() is not None:
                raise RuntimeError("mjrl_amd pool worker %d exited with code %s" % (r, self._procs[r].returncode))
            if time.time() - t0 > self.timeout:
                raise TimeoutError("mjrl_amd pool worker %d did not answer within %.0f s" % (r, self.timeout))
        return c.recv()

    def _recv_all(self):
        """Every worker's reply to a step, in any order: the first error reply or
        dead worker ends the wait at once (the other ranks are then typically
        blocked in a collective with the failed one; the caller aborts them)."""
        replies = [None] * self.world
        pending = set(range(self.world))
        t0 = time.time()
        while pending:
            ready = connection.wait([self._conns[r] for r in pending], timeout=1.0)
            for c in ready:
                r = self._conns.index(c)
                msg = c.recv()
                if msg[0] != "ok":
                    raise RuntimeError("mjrl_amd pool worker %d failed:\n%s" % (r, msg[1]))
                replies[r] = msg
                pending.discard(r)
            for r in pending:
                if self._procs[r].poll() is not None:
                    raise RuntimeError("mjrl_amd pool worker %d exited with code %s" % (r, self._procs[r].returncode))
            if pending and time.time() - t0 > self.timeout:
                raise TimeoutError("mjrl_amd pool workers %s did not answer within %.0f s" % (sorted(pending),
                                                                                            self.timeout))
        return replies

    def _segment(self, r, nbytes):
        s = self._shm[r]
        if s is None or s.size < nbytes:
            if s is not None:
                s.close()
                s.unlink()
            s = self._shm[r] = shared_memory.SharedMemory(create=True, size=nbytes)
        return s

    def close(self):
        for r, c in enumerate(self._conns):
            try:
                c.send(("close",))
            except Exception:
                pass
        for p in self._procs:
            try:
                p.wait(timeout=60)
            except Exception:
                p.kill()
        self._free_segments()
        self._listener.close()
        if getattr(self, "_fillex", None) is not None:
            self._fillex.shutdown(wait=False)
            self._fillex = None

    def _state(self, agent, commit=True):
        """The agent as the workers rebuild it: its __getstate__ (the device
        engine, batch and trainer dropped) minus the controller-local attributes,
        pickled per attribute; only the attributes whose pickle changed since the
        last step travel (DAPG's demo_paths and the hyperparameters once, the
        policy / baseline / running statistics every step).  commit=False: the
        delta without recording it as sent."""
        import hashlib
        d = agent.__getstate__() if hasattr(type(agent), "__getstate__") else dict(agent.__dict__)
        blobs = {k: pickle.dumps(v, protocol=pickle.HIGHEST_PROTOCOL) for k, v in d.items() if k not in _LOCAL}
        digests = {k: hashlib.blake2b(b, digest_size=16).digest() for k, b in blobs.items()}
        changed = {k: b for k, b in blobs.items() if self._digests.get(k) != digests[k]}
        dropped = [k for k in self._digests if k not in blobs]
        if commit:
            self._digests = digests
        return dict(cls=type(agent), changed=changed, dropped=dropped)

    def _fill_pool(self):
        """The controller's conversion threads: 16 per GPU worker, within the CPUs
        this process may use (engine._host_threads)."""
        if getattr(self, "_fillex", None) is None:
            import concurrent.futures as cf
            from .engine import _host_threads
            self._fill_threads = _host_threads(16 * self.world)
            self._fillex = cf.ThreadPoolExecutor(self._fill_threads, thread_name_prefix="mjrl_fill")
        return self._fillex

    # ---- one update -------------------------------------------------------------
    def step(self, agent, paths, mode, gamma=0.995, gae_lambda=0.98, fit=False, return_errors=False):
        """The update of `agent` on `paths` by the workers.  mode 'samples':
        train_from_samples (returns / GAE on the device, written back into the
        paths) and, with fit, the baseline fit on the union; mode 'paths':
        train_from_paths (the paths carry advantages).  Returns rank 0's reply."""
        from .comm import partition_paths
        lengths = np.array([len(p["rewards"]) for p in paths], dtype=np.int64)
        n = int(np.asarray(paths[0]["observations"]).shape[1])
        m = int(np.asarray(paths[0]["actions"]).shape[1])
        parts = partition_paths(lengths, self.world)
        if any(p1 <= p0 for p0, p1 in parts):
            raise ValueError("%d paths over %d GPU workers: every worker needs at least one path"
                             % (len(paths), self.world))
        with_adv = mode == "paths"
        dtype = _segment_dtype(agent)
        from .engine import _linear_coeffs
        c = _linear_coeffs(getattr(agent, "baseline", None), n) if not with_adv else False
        coeffs = None if c is False or c is None else c
        try:
            t0 = time.perf_counter()
            state = self._state(agent)
            t1 = time.perf_counter()
            layouts = []
            rng = np.random.get_state()
            shard_ms = []
            for r in range(self.world):
                tf0 = time.perf_counter()
                # every shard's conversion spread over the controller's thread pool
                # (16 threads per GPU, within the process's CPU share), and the shard
                # handed to its worker as soon as it is filled: worker r stages
                # (H2D) and starts its update while the controller fills shard r + 1
                p0, p1 = parts[r]
                L = _Layout(int(lengths[p0:p1].sum()), p1 - p0, n, m, with_adv, dtype)
                _fill_shard(self._segment(r, L.nbytes).buf, L, paths[p0:p1], lengths[p0:p1], self._fill_pool(),
                            threads=self._fill_threads, coeffs=coeffs)
                layouts.append(L)
                shard_ms.append((time.perf_counter() - tf0) * 1e3)
                self._conns[r].send(("step", dict(state=state, shm=self._shm[r].name, T=L.T, P=L.P, n=n, m=m,
                                                  dtype=L.dtype.str, mode=mode, gamma=gamma, gae_lambda=gae_lambda,
                                                  fit=fit, return_errors=return_errors, rng=rng,
                                                  with_adv=with_adv)))
            t2 = time.perf_counter()
            replies = self._recv_all()
            t3 = time.perf_counter()
        except BaseException:
            self._abort()
            raise
        # shard r is handed to worker r as soon as it is filled, so the workers of the
        # first shards compute while later shards fill: fill_ms is the controller's
        # own conversion time (the sum of the per-shard fills), fill_span_ms the span
        # from the first fill to the last hand-over (worker time overlaps it), and
        # workers_ms the wait after the last hand-over only
        self.last_timing = dict(state_ms=(t1 - t0) * 1e3, fill_ms=float(sum(shard_ms)), fill_shard_ms=shard_ms,
                                fill_span_ms=(t2 - t1) * 1e3, workers_ms=(t3 - t2) * 1e3,
                                worker_train_ms=[msg[1].get("train_ms") for msg in replies])
        if mode == "samples":
            for r in range(self.world):
                p0, p1 = parts[r]
                L, buf = layouts[r], self._shm[r].buf
                ret, base, adv = (L.view(buf, k).copy() for k in ("ret", "base", "adv"))
                o = 0
                for p in paths[p0:p1]:
                    h = len(p["rewards"])
                    p["returns"], p["baseline"], p["advantages"] = ret[o:o + h], base[o:o + h], adv[o:o + h]
                    o += h
        out = replies[0][1]
        np.random.set_state(out["rng"])
        return out


_POOLS = {}


def get_pool(devices, backend=None):
    """The process-wide pool for `devices` (started on first use, closed at
    exit).  backend: MJRL_AMD_POOL_BACKEND, default "nccl" (RCCL); "gloo" runs
    several workers on one GPU (tests)."""
    backend = backend or os.environ.get("MJRL_AMD_POOL_BACKEND", "nccl")
    key = (tuple(devices), backend)
    pool = _POOLS.get(key)
    if pool is None:
        if not _POOLS:
            import atexit
            atexit.register(close_pools)
        pool = _POOLS[key] = DevicePool(devices, backend)
    return pool


def close_pools():
    while _POOLS:
        _, pool = _POOLS.popitem()
        try:
            pool.close()
        except Exception:
            pass


def _worker_paths(L, buf):
    """The shard's paths as dicts of views into the shared segment."""
    obs = L.view(buf, "obs").reshape(L.T, L.n)
    act = L.view(buf, "act").reshape(L.T, L.m)
    rew = L.view(buf, "rew")
    adv = L.view(buf, "adv_in") if L.fields["adv_in"][1] else None
    lengths = L.view(buf, "lengths")
    term = L.view(buf, "term")
    paths, o = [], 0
    for i in range(L.P):
        h = int(lengths[i])
        p = dict(observations=obs[o:o + h], actions=act[o:o + h], rewards=rew[o:o + h], agent_infos={},
                 env_infos={}, terminated=bool(term[i]))
        if adv is not None:
            p["advantages"] = adv[o:o + h]
        paths.append(p)
        o += h
    return paths


def _worker_main(args):
    host, port = args.address.rsplit(":", 1)
    conn = connection.Client((host, int(port)), authkey=bytes.fromhex(args.authkey))
    conn.send(args.rank)
    try:
        import torch
        import torch.distributed as dist
        if args.backend == "nccl":
            torch.cuda.set_device(args.device)
            dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % args.dist_port, rank=args.rank,
                                    world_size=args.world, device_id=torch.device("cuda", args.device))
        else:
            if torch.cuda.is_available():
                torch.cuda.set_device(args.device)
            dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % args.dist_port, rank=args.rank,
                                    world_size=args.world)
        from .comm import DistComm
        from .utils.logger import DataLog
        comm = DistComm()
    except Exception:
        conn.send(("error", traceback.format_exc()))
        return 1
    conn.send(("ready",))
    engines = {}
    blobs = {}          # the agent's attributes as last sent (pickles)
    shm = unreg = None
    while True:
        msg = conn.recv()
        if msg[0] == "close":
            break
        paths = agent = None
        try:
            a = msg[1]
            if shm is None or shm.name != a["shm"]:
                shm, unreg = _attach(shm, unreg, a["shm"])
            L = _Layout(a["T"], a["P"], a["n"], a["m"], a["with_adv"], np.dtype(a["dtype"]))
            paths = _worker_paths(L, shm.buf)
            st = a["state"]
            for k in st["dropped"]:
                blobs.pop(k, None)
            blobs.update(st["changed"])
            agent = st["cls"].__new__(st["cls"])
            # unpickled afresh every step: the update mutates the policy / baseline
            agent.__dict__.update({k: pickle.loads(b) for k, b in blobs.items()})
            agent.env = None
            agent.logger = DataLog()
            agent._comm = comm
            agent._device = None
            agent._devices = None
            if L.dtype == np.float32 and L.T:
                rng = L.view(shm.buf, "orange").reshape(2, L.n)
                # the segment is the staged batch: copied to HBM as it is
                agent._pre = dict(obs=L.view(shm.buf, "obs").reshape(L.T, L.n),
                                  act=L.view(shm.buf, "act").reshape(L.T, L.m), obs_range=(rng[0], rng[1]))
                if L.fields["xflags"][1]:
                    inexact, has_pred = (bool(v) for v in L.view(shm.buf, "xflags"))
                    agent._pre.update(inexact=inexact, pred=L.view(shm.buf, "pred_in") if has_pred else None,
                                      obs_lo=L.view(shm.buf, "obs_lo").reshape(L.T, L.n) if inexact else None)
            key = (agent.policy.n, agent.policy.m, agent.policy.hidden)
            agent._engine = engines.get(key)
            np.random.set_state(a["rng"])
            out = {}
            tw = time.perf_counter()
            if a["mode"] == "samples":
                stats = agent.train_from_samples(paths, a["gamma"], a["gae_lambda"])
                for name, k in (("ret", "returns"), ("base", "baseline"), ("adv", "advantages")):
                    v = L.view(shm.buf, name)
                    if paths:
                        np.concatenate([np.asarray(p[k], np.float64) for p in paths], out=v)
                if a["fit"]:
                    ts = time.time()
                    errs = agent._fit_baseline(paths, return_errors=a["return_errors"])
                    out["time_VF"] = time.time() - ts
                    out["fit_errors"] = errs if a["return_errors"] else None
                    out["baseline"] = pickle.dumps(agent.baseline) if args.rank == 0 else None
            else:
                stats = agent.train_from_paths(paths)
            out["train_ms"] = (time.perf_counter() - tw) * 1e3
            engines[key] = agent._engine
            if args.rank == 0:
                out.update(stats=[float(s) for s in stats], theta=agent.policy.get_param_values(),
                           logs=list(agent.logger.get_current_log().items()) if agent.save_logs else [],
                           sync={k: agent.__dict__[k] for k in _SYNC if k in agent.__dict__},
                           rng=np.random.get_state())
            # the controller rewrites the segment after the reply: the DMA copies
            # out of its registered memory must have completed first
            from .engine import _STAGING
            _STAGING.wait_host("obs")
            _STAGING.wait_host("act")
            _STAGING.wait_host("obs_lo")
            conn.send(("ok", out))
        except Exception:
            conn.send(("error", traceback.format_exc()))
    paths = agent = None
    _attach(shm, unreg, None)
    from .comm import release_comms
    release_comms()
    dist.destroy_process_group()
    return 0


def _attach(shm, unreg, name):
    """Detaches from the current segment (unregistering it as pinned memory) and
    attaches to segment `name`, registered with hipHostRegister when this worker
    has a GPU, so the H2D copies of its batch run as DMA straight out of it."""
    import gc
    import torch
    if shm is not None:
        if unreg is not None:
            torch.cuda.synchronize()
            unreg()
        gc.collect()             # views of the old segment (the last step's paths)
        try:
            shm.close()
        except BufferError:
            pass                 # still viewed: the mapping goes with the process
    if name is None:
        return None, None
    shm = shared_memory.SharedMemory(name=name)
    _untrack(shm)
    unreg = None
    if torch.cuda.is_available():
        from .engine import register_host
        unreg = register_host(np.ndarray((shm.size,), np.uint8, buffer=shm.buf))
    return shm, unreg


def _untrack(shm):
    """The controller owns (and unlinks) the segment: keep this process's
    resource tracker from unlinking it at exit."""
    try:
        from multiprocessing import resource_tracker
        resource_tracker.unregister(shm._name, "shared_memory")
    except Exception:
        pass


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    for k in ("address", "authkey", "backend"):
        ap.add_argument("--" + k, required=True)
    for k in ("rank", "world", "device", "dist-port"):
        ap.add_argument("--" + k, type=int, required=True)
    sys.exit(_worker_main(ap.parse_args()))
