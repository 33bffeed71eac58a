"""world_size-2 / -4 gloo tests of the sharded update's collective schedule (CPU).

Every rank takes its shard of a golden batch (mjrl_amd.comm.partition_paths),
computes the per-shard quantities the device kernels produce (the local moment
records of the advantages and path returns, VPG sum, FVP sums) — here with the
oracle as the stand-in compute, since this container has no GPU — exchanges them
through mjrl_amd.comm.DistComm exactly as mjrl_amd.engine.UpdateEngine.update
does (one all-gather of the moment records folded as mjrl_moments_combine does,
one all-reduce per VPG / FVP sum), and finishes with the replicated CG.  The result must equal the unsharded update.
The same schedule runs over RCCL on the GPU box (tests/test_gpu_dist.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        from mjrl_amd.comm import DistComm, partition_paths
        from oracle import npg_cpu as O
        comm = DistComm()
        c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
        lengths = c["lengths"]
        offs = np.concatenate([[0], np.cumsum(lengths)])
        p0, p1 = partition_paths(lengths, world)[rank]
        r0, r1 = offs[p0], offs[p1]
        adv = c["advantages"][r0:r1]
        T = float(r1 - r0)
        # whitening + path-return stats (engine.update, sharded): each rank's two
        # local passes as moment records, ONE all-gather, the fixed-order fold of
        # mjrl_moments_combine (restated by O.moments_combine)
        pr = np.array([np.sum(c["rewards"][offs[i]:offs[i + 1]]) for i in range(p0, p1)])
        rec = torch.from_numpy(np.concatenate([O.moments_record(adv), O.moments_record(pr)]))
        g = torch.zeros(world * 32, dtype=torch.float64)
        comm.allgather(rec, g)
        g = g.numpy().reshape(world, 32)
        ma = O.moments_combine(g[:, :16])
        mp_ = O.moments_combine(g[:, 16:])
        mean = ma[0] / ma[2]
        w = (adv - mean) / (np.sqrt(ma[9] / ma[2]) + 1e-6)
        pmean = mp_[0] / mp_[2]
        stats = [pmean, np.sqrt(mp_[9] / mp_[2]), -mp_[5], mp_[4]]
        Tg = ma[2]
        # VPG: per-shard sum, all-reduced, divided by the global row count
        pol = O.Policy(int(c["n"]), int(c["m"]), c["hidden_t"], c["theta0"], c["transforms"])
        obs, act = c["obs64"][r0:r1], c["act64"][r0:r1]
        gsum = torch.from_numpy(pol.flat_vpg(obs, act, w).astype(np.float64) * T)
        comm.allreduce_sum(gsum)
        g = (gsum / Tg).numpy().astype(np.float32)
        # CG with the sharded FVP: sum_r T_r (F_r v) / T_global + damping v
        def fvp(v):
            z = torch.from_numpy((pol.fvp(obs, act, v, 0.0).astype(np.float64)) * T)
            comm.allreduce_sum(z)
            return ((z / Tg).numpy() + 1e-4 * v).astype(np.float32)
        x = O.cg_solve(fvp, g, iters=10)
        q.put((rank, w, stats, g, x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("c2_ragged", 2), ("c3_halfcheetah_trpo", 2), ("c2_ragged", 4)])
def test_sharded_schedule_equals_unsharded(name, world):
    from oracle import npg_cpu as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, *vals = q.get(timeout=300)
        out[r] = vals
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
    w = np.concatenate([out[r][0] for r in range(world)])
    np.testing.assert_allclose(w, c["adv_whitened"], rtol=1e-10, atol=1e-12)
    for r in range(world):
        np.testing.assert_allclose(out[r][1], c["base_stats"], rtol=1e-10)
    g0 = out[0][2]
    for r in range(1, world):
        assert np.array_equal(out[r][2], g0)                       # replicated after the all-reduce
    assert np.linalg.norm(g0 - c["vpg_grad"]) / np.linalg.norm(c["vpg_grad"]) < 1e-5
    x0 = out[0][3]
    for r in range(1, world):
        assert np.array_equal(out[r][3], x0)
    tol = max(1e-3, 3 * float(c["spread_x"]))
    assert np.linalg.norm(x0 - c["cg_x"]) / np.linalg.norm(c["cg_x"]) < tol


def _draw_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from types import SimpleNamespace
        from mjrl_amd.comm import DistComm
        from mjrl_amd.engine import UpdateEngine
        T_local = [700, 300][rank]
        np.random.seed(5 if rank == 0 else 77)   # only rank 0's RNG may matter
        fake = SimpleNamespace(comm=DistComm(), device=torch.device("cpu"))
        sub = UpdateEngine._hvp_draws(fake, 0.5, 1000, T_local, 4)
        q.put((rank, sub["idx"].numpy(), sub["counts"], sub["offs"], sub["Ts"], np.random.rand()))
    finally:
        dist.destroy_process_group()


def test_subsampled_fisher_draw_sharding():
    """hvp_sample_frac < 1 on 2 ranks: rank 0's np.random.choice draws
    (npg_cg.py:58-62) are broadcast and each rank keeps its own rows, in draw
    order; together the shards hold exactly the reference's draw."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_draw_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, *vals = q.get(timeout=300)
        out[r] = vals
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.random.seed(5)
    ref = [np.random.choice(1000, size=500) for _ in range(4)]
    assert out[0][3] == out[1][3] == 500
    for k in range(4):
        i0 = out[0][0][out[0][2][k]:out[0][2][k + 1]]
        i1 = out[1][0][out[1][2][k]:out[1][2][k + 1]] + 700
        assert np.array_equal(i0, ref[k][ref[k] < 700])
        assert np.array_equal(i1, ref[k][ref[k] >= 700])
