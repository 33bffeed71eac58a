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

    def allreduce_sum(self, t):
        return t

    def allreduce_max(self, t):
        return t

    def broadcast(self, t, src=0):
        return t

    def row_offset(self, T, device=None):
        """First global row of this rank's shard (ranks hold contiguous path ranges)."""
        return 0


class DistComm:
    """torch.distributed process group (RCCL on GPU, gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)

    def allreduce_sum(self, t):
        if self.world_size > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t

    def allreduce_max(self, t):
        if self.world_size > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return t

    def broadcast(self, t, src=0):
        if self.world_size > 1:
            self.dist.broadcast(t, src=src, group=self.group)
        return t

    def row_offset(self, T, device=None):
        counts = torch.zeros(self.world_size, dtype=torch.float64, device=device)
        counts[self.rank] = float(T)
        self.allreduce_sum(counts)
        return int(counts[:self.rank].sum().item())


def default_comm():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return DistComm()
    return LocalComm()


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
        return DistComm() if dist.get_world_size() > 1 else LocalComm()
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
    return DistComm()


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
