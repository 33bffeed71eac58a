"""Collectives used by the sharded update (one process per GPU).

The update is data-parallel over paths: every rank owns a contiguous range of
paths (balanced by timestep count, `partition_paths`) and all full-batch
quantities are sums over timesteps, so the only exchange is an all-reduce SUM of
  - the whitening moments (2 x 3 doubles) and the path-return moments,
  - the flat VPG sum (d floats) and every Fisher-vector-product sum (d floats),
  - the post-step surrogate / KL sums (2 doubles per line-search trial),
plus one MAX of the path-return extrema.  A subsampled Fisher
(hvp_sample_frac < 1) adds one broadcast of rank 0's row draw per update.
Backend "nccl" is RCCL over xGMI on ROCm; the same code runs on "gloo" for the
CPU tests.
"""
import numpy as np
import torch


class LocalComm:
    """world_size 1: every collective is the identity."""
    rank = 0
    world_size = 1
    sharded = False       # the engine runs its one-process schedule
    capturable = True     # no collective at all: an update graph may be captured

    def allreduce_sum(self, t):
        return t

    def allreduce_max(self, t):
        return t

    def allgather(self, src, dst):
        dst.copy_(src.reshape(-1))
        return dst

    def broadcast(self, t, src=0):
        return t

    def row_offset(self, T, device=None):
        """First global row of this rank's shard (ranks hold contiguous path ranges)."""
        return 0


class DistComm:
    """torch.distributed process group (gloo on CPU for the tests; RCCL on GPU
    when MJRL_AMD_COMM=torch asks for torch's own collectives)."""
    capturable = False    # torch's work objects are not relied on inside a hipGraph capture

    def __init__(self, group=None, force_sharded=False):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.sharded = self.world_size > 1 or bool(force_sharded)

    def allreduce_sum(self, t):
        if self.world_size > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t

    def allreduce_max(self, t):
        if self.world_size > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return t

    def allgather(self, src, dst):
        """dst [world * k] = every rank's src [k], in rank order."""
        src = src.reshape(-1).contiguous()
        if self.world_size > 1:
            parts = list(dst.view(self.world_size, -1).unbind(0))
            self.dist.all_gather(parts, src, group=self.group)
        else:
            dst.copy_(src)
        return dst

    def broadcast(self, t, src=0):
        if self.world_size > 1:
            self.dist.broadcast(t, src=src, group=self.group)
        return t

    def row_offset(self, T, device=None):
        counts = torch.zeros(self.world_size, dtype=torch.float64, device=device)
        counts[self.rank] = float(T)
        self.allreduce_sum(counts)
        return int(counts[:self.rank].sum().item())


# ---------------------------------------------------------------------------
# RCCL driven directly: ncclAllReduce / ncclAllGather / ncclBroadcast issued on the
# caller's current HIP stream from ctypes, on the librccl that torch itself loads.
# Every collective is then an ordinary stream-ordered operation: no torch work
# object, no event fork / join to an internal stream, no host synchronisation —
# so a whole sharded update, all-reduces included, is captured into ONE hipGraph
# and replayed (engine.UpdateEngine._maybe_capture).  RCCL supports stream
# capture and mixes captured and eager collectives on one communicator.
_NCCL_DT = {torch.float32: 7, torch.float64: 8, torch.int64: 4, torch.int32: 2, torch.uint8: 1}
_NCCL_SUM, _NCCL_MAX = 0, 2
_RCCL = None


def _rccl():
    """The librccl of torch's own build (libtorch_hip links it), so the process
    holds one RCCL."""
    global _RCCL
    if _RCCL is None:
        import ctypes as C
        import os
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        lib = C.CDLL(path if os.path.exists(path) else "librccl.so.1")
        vp, sz, i32 = C.c_void_p, C.c_size_t, C.c_int
        lib.ncclGetUniqueId.argtypes = [C.POINTER(_NcclId)]
        lib.ncclCommInitRank.argtypes = [C.POINTER(vp), i32, _NcclId, i32]
        lib.ncclAllReduce.argtypes = [vp, vp, sz, i32, i32, vp, vp]
        lib.ncclAllGather.argtypes = [vp, vp, sz, i32, vp, vp]
        lib.ncclBroadcast.argtypes = [vp, vp, sz, i32, i32, vp, vp]
        lib.ncclCommDestroy.argtypes = [vp]
        lib.ncclGetErrorString.argtypes = [i32]
        lib.ncclGetErrorString.restype = C.c_char_p
        for f in (lib.ncclGetUniqueId, lib.ncclCommInitRank, lib.ncclAllReduce, lib.ncclAllGather,
                  lib.ncclBroadcast, lib.ncclCommDestroy, lib.ncclGroupStart, lib.ncclGroupEnd):
            f.restype = i32
        _RCCL = lib
    return _RCCL


def _nccl_id_type():
    import ctypes as C

    class NcclId(C.Structure):
        _fields_ = [("internal", C.c_char * 128)]
    return NcclId


_NcclId = _nccl_id_type()


class RcclComm:
    """One RCCL communicator over the ranks of a torch.distributed group (one
    process per GPU; the group only carries the unique id and host-side
    barriers / object exchange).  `local(device)` builds a one-rank communicator
    without torch.distributed: the sharded code path, RCCL calls and their
    graph capture then run on a single GPU (tests; pools of one box)."""
    capturable = True

    def __init__(self, device, group=None, rank=None, world_size=None, force_sharded=False):
        import ctypes as C
        lib = _rccl()
        self.device = torch.device(device)
        self.group = group
        if rank is None:
            import torch.distributed as dist
            self.dist = dist
            self.rank, self.world_size = dist.get_rank(group), dist.get_world_size(group)
        else:
            self.dist = None
            self.rank, self.world_size = int(rank), int(world_size)
        uid = _NcclId()
        if self.rank == 0:
            self._check(lib.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        if self.world_size > 1:
            obj = [bytes(uid.internal) if self.rank == 0 else None]
            src = self.dist.get_global_rank(group, 0) if group is not None else 0
            self.dist.broadcast_object_list(obj, src=src, group=group)
            C.memmove(C.addressof(uid), obj[0], 128)
        self._comm = C.c_void_p()
        with torch.cuda.device(self.device):
            self._check(lib.ncclCommInitRank(C.byref(self._comm), self.world_size, uid, self.rank),
                        "ncclCommInitRank")
        self.sharded = self.world_size > 1 or bool(force_sharded)

    @classmethod
    def local(cls, device, force_sharded=True):
        return cls(device, rank=0, world_size=1, force_sharded=force_sharded)

    @staticmethod
    def _check(rc, what):
        if rc != 0:
            msg = _rccl().ncclGetErrorString(rc)
            raise RuntimeError("%s failed: %s (%d)" % (what, msg.decode() if msg else "?", rc))

    def _stream(self, t):
        return torch.cuda.current_stream(t.device).cuda_stream

    def _args(self, t):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm collectives take contiguous device tensors")
        return t.data_ptr(), t.numel(), _NCCL_DT[t.dtype]

    def allreduce_sum(self, t):
        p, n, dt = self._args(t)
        if n:
            self._check(_rccl().ncclAllReduce(p, p, n, dt, _NCCL_SUM, self._comm, self._stream(t)), "ncclAllReduce")
        return t

    def allreduce_max(self, t):
        p, n, dt = self._args(t)
        if n:
            self._check(_rccl().ncclAllReduce(p, p, n, dt, _NCCL_MAX, self._comm, self._stream(t)), "ncclAllReduce")
        return t

    def allgather(self, src, dst):
        ps, n, dt = self._args(src)
        pd, nd, _ = self._args(dst)
        if nd != n * self.world_size:
            raise ValueError("allgather: dst must hold world_size x src elements")
        self._check(_rccl().ncclAllGather(ps, pd, n, dt, self._comm, self._stream(src)), "ncclAllGather")
        return dst

    def broadcast(self, t, src=0):
        p, n, dt = self._args(t)
        if n:
            self._check(_rccl().ncclBroadcast(p, p, n, dt, int(src), self._comm, self._stream(t)), "ncclBroadcast")
        return t

    def row_offset(self, T, device=None):
        counts = torch.zeros(self.world_size, dtype=torch.float64, device=self.device)
        counts[self.rank] = float(T)
        self.allreduce_sum(counts)
        return int(counts[:self.rank].sum().item())

    def close(self):
        if getattr(self, "_comm", None) and self._comm.value:
            _rccl().ncclCommDestroy(self._comm)
            self._comm = None


def default_comm():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return _group_comm()
    return LocalComm()


_RCCL_CACHE = {}


def _group_comm(group=None):
    """The communicator of an initialised torch.distributed group: RCCL driven
    directly (RcclComm) when the group's backend is nccl (= RCCL) and
    MJRL_AMD_COMM is not 'torch'; torch's own collectives (DistComm) otherwise
    (gloo: the CPU tests).  One RcclComm per (group, device) for the life of the
    group: agents built without an explicit comm share it (every new one would
    be another ncclCommInitRank collective, in whatever order each rank builds
    its agents), and it is destroyed at exit (release_comms)."""
    import os
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl" and os.environ.get("MJRL_AMD_COMM", "rccl") != "torch":
        dev = torch.device("cuda", torch.cuda.current_device())
        # the entry holds the group object itself (the default group: the live
        # WORLD object), its rank and size: a group destroyed and created again
        # (even one reusing a freed object's id) gets a new communicator instead
        # of the old world's
        pg = group if group is not None else dist.group.WORLD
        key = (id(pg), dev.index)
        ent = _RCCL_CACHE.get(key)
        live = (dist.get_rank(group), dist.get_world_size(group))
        if ent is not None and (ent[1] is not pg or ent[2] != live or getattr(ent[0], "_comm", None) is None):
            try:
                ent[0].close()
            except Exception:
                pass
            ent = None
        if ent is None:
            if not _RCCL_CACHE:
                import atexit
                atexit.register(release_comms)
            ent = _RCCL_CACHE[key] = (RcclComm(dev, group=group), pg, live)
        return ent[0]
    return DistComm(group)


def release_comms():
    """Destroys the cached RCCL communicators (at exit, or before the process
    group is destroyed)."""
    for c, _, _ in list(_RCCL_CACHE.values()):
        try:
            c.close()
        except Exception:
            pass
    _RCCL_CACHE.clear()


def launched_world():
    """(rank, world_size, local_rank) from a torchrun-style environment, or None
    when the process was not launched as one of several ranks."""
    import os
    try:
        world = int(os.environ.get("WORLD_SIZE", "1"))
    except ValueError:
        return None
    if world <= 1 or "RANK" not in os.environ:
        return None
    return int(os.environ["RANK"]), world, int(os.environ.get("LOCAL_RANK", os.environ["RANK"]))


def auto_comm(backend=None):
    """The communicator an agent uses when the caller passed none.

    - torch.distributed already initialised with world size > 1: that group;
    - launched by torchrun (RANK / WORLD_SIZE / MASTER_ADDR in the environment)
      but not initialised: initialise it here — RCCL ("nccl") on cuda:LOCAL_RANK
      when a GPU is visible, gloo otherwise — so an unchanged training script
      (mjrl/utils/train_agent.py) runs sharded under
      `torchrun --nproc-per-node N script.py`;
    - otherwise LocalComm (one process, the whole batch)."""
    import os
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return _group_comm() if dist.get_world_size() > 1 else LocalComm()
    lw = launched_world()
    if lw is None or not dist.is_available() or "MASTER_ADDR" not in os.environ:
        return LocalComm()
    rank, world, local = lw
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    else:
        dist.init_process_group(backend)
    return _group_comm()


def shard_count(N, world, rank):
    """Paths rank `rank` samples out of N (train_step): ceil(N / world) each, the
    last ranks fewer, as trajectory_sampler.sample_paths_parallel splits N over its
    workers (mjrl/samplers/trajectory_sampler.py:37-45).  Returns (count, first
    global path index) — the first index is also the rank's pegasus seed offset."""
    per = int(np.ceil(N / world))
    first = min(rank * per, N)
    return max(0, min(per, N - first)), first


def partition_paths(lengths, world_size):
    """Contiguous path ranges per rank, balanced by timestep count.

    Returns a list of (p_begin, p_end).  Deterministic; every rank computes the
    same split from the same lengths.  A rank may get an empty range when there
    are fewer paths than ranks."""
    lengths = np.asarray(lengths, dtype=np.int64)
    P = len(lengths)
    if world_size <= 1:
        return [(0, P)]
    cum = np.concatenate([[0], np.cumsum(lengths)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world_size):
        target = total * r / world_size
        # first path boundary at or after the target, never before the previous bound
        b = int(np.searchsorted(cum, target, side="left"))
        b = min(max(b, bounds[-1]), P)
        bounds.append(b)
    bounds.append(P)
    return [(bounds[i], bounds[i + 1]) for i in range(world_size)]
