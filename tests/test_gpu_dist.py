"""Sharded update on the GPU: two ranks on the box's one GPU (gloo carries the
all-reduces of GPU tensors; the driver's 8-GPU runs use the same code over
RCCL).  Each rank stages its path shard and runs UpdateEngine.update with a
DistComm; both ranks must end with identical parameters equal (within the
parity tolerance) to the unsharded reference update."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mjrl_amd.comm import DistComm, partition_paths
        from mjrl_amd.engine import UpdateEngine, DeviceBatch
        from oracle import npg_cpu as O
        c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
        kw = O.case_kwargs(c)
        lengths = c["lengths"]
        offs = np.concatenate([[0], np.cumsum(lengths)])
        p0, p1 = partition_paths(lengths, world)[rank]
        r0, r1 = offs[p0], offs[p1]
        dev = torch.device("cuda:0")
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        obs, act, T_demo = c["obs64"][r0:r1], c["act64"][r0:r1], 0
        if "demo_obs" in c:
            # DAPG: the 200-row demo paths are split over the ranks (BatchREINFORCE._rank_share),
            # so each demo row enters the all-reduced VPG sum once
            nd = c["demo_obs"].shape[0] // 200
            d0, d1 = partition_paths(np.full(nd, 200), world)[rank]
            obs = np.concatenate([obs, c["demo_obs"][200 * d0:200 * d1].astype(np.float64)])
            act = np.concatenate([act, c["demo_act"][200 * d0:200 * d1].astype(np.float64)])
            T_demo = 200 * (d1 - d0)
        b = DeviceBatch(t(obs), t(act), t(c["rewards"][r0:r1]),
                        t(c["baseline"][r0:r1]), t(offs[p0:p1 + 1] - offs[p0]),
                        t(c["terminated"][p0:p1].astype(np.uint8)), T_demo=T_demo)
        eng = UpdateEngine(int(c["n"]), int(c["m"]), c["hidden_t"], device=dev, comm=DistComm())
        if c["transforms"] is not None:
            eng.set_transformations(*c["transforms"])
        args = dict(algo=kw["algo"], gamma=float(c["gamma"]), gae_lambda=float(c["gae_lambda"]), trpo_verbose=False)
        if kw["algo"] == "npg":
            args["n_step_size"] = kw.get("n_step_size", 0.01)
        else:
            args["kl_dist"] = kw["kl_dist"]
        if kw["algo"] == "dapg":
            args["demo_coef"] = kw["demo_coef"]
        if "hvp_sample_frac" in kw:
            # rank 0 draws (and must match the reference's draws); rank 1's RNG is
            # deliberately different to show the broadcast is what it uses
            args["hvp_sample_frac"] = kw["hvp_sample_frac"]
            np.random.seed(kw["np_seed"] if rank == 0 else 99)
        res = eng.update(b, t(c["theta0"].astype(np.float32)), **args)
        q.put((rank, eng.vec["theta_new"].cpu().numpy(), res["base_stats"], res["kl_dist"], res["alpha"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["c2_ragged", "c3_halfcheetah_trpo", "c2_hvp_sub", "c4_humanoid", "c5_door_dapg"])
def test_two_rank_update(name):
    from oracle import npg_cpu as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, *vals = q.get(timeout=600)
        out[r] = vals
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    c = O.load_case(os.path.join(GOLDEN, name + ".npz"))
    th0, th1 = out[0][0], out[1][0]
    assert np.array_equal(th0, th1)                     # replicated parameters
    np.testing.assert_allclose(out[0][1], c["base_stats"], rtol=1e-10)
    tol = max(1e-3, 3 * float(c["spread_theta"]))
    assert np.linalg.norm(th0 - c["theta1"]) / np.linalg.norm(c["theta1"]) < tol
    ktol = max(2e-3, 3 * float(c["spread_kl"]))
    np.testing.assert_allclose(out[0][2], c["log_kl_dist"], rtol=ktol)
