"""The pooled update that train_agent runs with devices= / MJRL_AMD_DEVICES
(mjrl_amd/pool.py), timed end to end at the bench's Humanoid 1M workload: the
controller (this process, no GPU) holds numpy f64 paths, two gloo workers on one
GPU (the one-GPU rehearsal of the N-GPU pool) run train_from_paths; against the
same update in-process (train_from_paths, one GPU).  Prints one JSON line.
    MJRL_AMD_POOL_BACKEND=gloo python tools/pool_bench.py [--paths 1000]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", choices=("pool", "local"), default="pool")
    args = ap.parse_args()
    import bench
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    cfg = dict(bench.CONFIGS["c4"])
    H, n, m = cfg["horizon"], cfg["n"], cfg["m"]
    obs, act, rew = bench.make_paths(0, args.paths, cfg=cfg)
    rs = np.random.RandomState(5)
    paths = [dict(observations=o.astype(np.float64), actions=a.astype(np.float64), rewards=r,
                  advantages=rs.standard_normal(H), terminated=False) for o, a, r in zip(obs, act, rew)]
    del obs, act
    spec = EnvSpec(n, m, H, 1)
    devices = [0, 0] if args.mode == "pool" else None
    agent = NPG(None, MLP(spec, hidden_sizes=cfg["hidden"], seed=0), LinearBaseline(spec), normalized_step_size=0.01,
                save_logs=False, devices=devices)
    t0 = time.perf_counter()
    agent.train_from_paths(paths)                    # pool start + first update
    first = time.perf_counter() - t0
    agent.train_from_paths(paths)                    # warm
    ts, timing = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        agent.train_from_paths(paths)
        ts.append(time.perf_counter() - t0)
        if devices:
            from mjrl_amd import pool
            p = next(iter(pool._POOLS.values()))
            timing.append({k: (round(v, 1) if isinstance(v, float) else [round(x, 1) for x in v])
                           for k, v in p.last_timing.items()})
    T = args.paths * H
    dt = float(np.median(ts))
    print(json.dumps(dict(mode=args.mode, workers=len(devices) if devices else 1,
                          backend=os.environ.get("MJRL_AMD_POOL_BACKEND", "nccl") if devices else None,
                          timesteps=T, ms_per_update=round(dt * 1e3, 1), all_ms=[round(t * 1e3, 1) for t in ts],
                          first_ms=round(first * 1e3, 1), timesteps_per_s=round(T / dt, 1),
                          pool_timing=timing or None)), flush=True)
    if devices:
        from mjrl_amd import pool
        pool.close_pools()


if __name__ == "__main__":
    main()
