"""Benchmark: NPG update throughput (timesteps/s) on the Humanoid 1M-step batch.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Default workload (BASELINE.json configs[3]; --config c4): obs 376,
act 17, MLP(64,64), NPG with 10 CG iterations, damping 1e-4, delta 0.01,
gamma 0.995, lambda 0.97; 1000 paths x 1000 steps = 1,000,000 timesteps per
update, split by paths over the N ranks (strong scaling: the batch is fixed).
Synthetic data: obs / act / rewards ~ N(0,1) from a per-path seeded generator;
LinearBaseline fitted once on 20 paths and frozen.  A step = one full update
from the device-resident batch in the layout train_step stages it (f32
observations / actions, f64 rewards and baseline; --stage-dtype f64 keeps the
sampler's f64): batch assembly, GAE, whitening, forward +
VPG, 10 Fisher-vector products + CG, step, post-step surrogate / KL, host
readback of the statistics.  On one GPU an update of at most
engine.GRAPH_AUTO_ROWS rows is replayed as one captured hipGraph (launch gaps
dominate there; at 1M rows eager launches are faster), and the eager time is
reported beside it (--graph on / off forces either).

--config c2 / c3 / c5 runs the other BASELINE.json GPU shapes (Swimmer NPG,
HalfCheetah TRPO with its line search, door DAPG with demonstrations) with their
own metric names: per-config evidence, not the headline.

Rank 0 prints one JSON line.  `roofline` is measured live with HIP events on the
stream the kernels run on, `cpu_baseline` times the oracle (the CPU restatement
of the reference update, oracle/npg_cpu.py) on a bounded sample on this host.
"""
import argparse
import json
import os
import re
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NPG train_step timesteps/sec, Humanoid 1M-step batch @ 1/2/4/8 MI355X"
GAMMA, LAM, CG_ITERS, DAMPING = 0.995, 0.97, 10, 1e-4
# the reference's own update measured on CPU (8 vCPU Xeon, torch
# CPU, synthetic inputs of the same shapes; BASELINE.json publishes no number), in
# timesteps/s: vs_baseline = value / this, on the config's full batch
REF_CPU = {"c4": (1e6 / 42.08, "BASELINE.md: reference update 42.08 s per 1M timesteps, 8 vCPU Xeon"),
           "c3": (1e5 / 3.084, "BASELINE.md: reference TRPO update 3.084 s per 100k timesteps, 8 vCPU Xeon"),
           "c5": (4e4 / 3.126, "BASELINE.md: reference DAPG update 3.126 s per 40k RL timesteps, 8 vCPU Xeon"),
           "c2": (12500 / 0.180, "BASELINE.md: reference NPG update 0.180 s per 12.5k timesteps, 8 vCPU Xeon")}

CONFIGS = {
    "c4": dict(workload="humanoid_npg_1M", metric=METRIC, n=376, m=17, hidden=(64, 64), paths=1000, horizon=1000,
               algo="npg", step=dict(n_step_size=0.01)),
    "c2": dict(workload="swimmer_npg_12.5k", metric="NPG update timesteps/sec, Swimmer-v2 shape 25 x 500, 1 MI355X",
               n=8, m=2, hidden=(64, 64), paths=25, horizon=500, algo="npg", step=dict(n_step_size=0.01)),
    "c3": dict(workload="halfcheetah_trpo_100k",
               metric="TRPO update timesteps/sec, HalfCheetah-v2 shape 100 x 1000, 1 MI355X",
               n=17, m=6, hidden=(128, 128), paths=100, horizon=1000, algo="trpo", step=dict(kl_dist=0.01)),
    "c5": dict(workload="door_dapg_40k",
               metric="DAPG update timesteps/sec, door-v0 shape 200 x 200 + 25 demos x 200, 1 MI355X",
               n=39, m=28, hidden=(256, 256), paths=200, horizon=200, algo="dapg",
               step=dict(kl_dist=0.005, demo_coef=1.0), demos=25),
}
# the default workload as module constants (used by tests)
N_OBS, N_ACT, HIDDEN = 376, 17, (64, 64)
N_PATHS, HORIZON = 1000, 1000
DELTA = 0.01
PEAK_F32_MFMA = 157.3   # TFLOP/s, MI355X dense fp32 matrix (MI355X_MICROARCH.md)
PEAK_F16_MFMA = 2500.0  # TFLOP/s, dense f16 / bf16 matrix (no sparsity)
PEAK_SPLIT = PEAK_F16_MFMA / 3   # f32-equivalent rate of the split-f16 products (3 f16 MFMAs each)
PEAK_HBM = 8000.0       # GB/s


def flops_per_row(n, m, h0, h1):
    """Algorithmic FLOPs per timestep, split by kernel."""
    jvp = 2 * (n * h0) + 4 * (h0 * h1) + 4 * (h1 * m)
    vjp_act = 2 * (h1 * m) + 2 * (h0 * h1)
    wgrad = 2 * (n * h0) + 2 * (h0 * h1) + 2 * (h1 * m)
    return dict(rows_fvp=jvp + vjp_act, weight_grads=wgrad)


def update_flops_per_row(n, m, h0, h1, K):
    """Algorithmic FLOPs of one whole update per timestep:
    fwd F + VPG (F + 2I) + K FVPs K (2F + 4I) + post-update fwd F, with
    F = 2(n h0 + h0 h1 + h1 m), I = h0 h1 + h1 m (1,563,136 at Humanoid / K = 10)."""
    F = 2 * (n * h0 + h0 * h1 + h1 * m)
    I = h0 * h1 + h1 * m
    return 3 * F + 2 * I + K * (2 * F + 4 * I)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """CPU cores this process may actually use, as the CPU baseline uses them: the
    affinity set, capped by the cgroup CPU quota (a container's affinity can list
    the whole machine while its quota is a fraction of it) and by
    OMP_NUM_THREADS when the environment sets it."""
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
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print("bench: " + msg, file=sys.stderr, flush=True)


def pmc_file():
    """The newest committed PMC summary, profiles/r*/pmc_traffic.json, or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))
    return files[-1] if files else None


def pmc_traffic(kernel_key):
    """HBM bytes per launch of a kernel from the newest committed PMC summary
    (profiles/r*/pmc_traffic.json, written from separate rocprofv3 --pmc passes
    of FETCH_SIZE and WRITE_SIZE with the gfx950 2x FETCH_SIZE correction; the
    correction checks out on k_pack_batch, whose 3.14 GB read is known exactly).
    kernel_key: the demangled instantiation prefix ('k_kx<32, 12, 1, false>'),
    matched after the '::' of the name.  Returns (bytes, source, error): a summary
    that exists but lacks the kernel is an error, not a silent None (tests/
    test_host_logic.py checks the committed file against the default key)."""
    f = pmc_file()
    if f is None:
        return None, None, "no profiles/r*/pmc_traffic.json committed"
    data = json.load(open(f))
    src = os.path.relpath(f, ROOT)
    for name, v in data.items():
        if isinstance(v, dict) and re.search(r"(^|[\s:])" + re.escape(kernel_key), name):
            # the commit the PMC passes measured (recorded when the summary was filed)
            head = data.get("_measured_at_commit")
            return v["hbm_bytes_per_launch"], src + (" @ " + head if head else ""), None
    return None, None, "%s has no entry for %s" % (src, kernel_key)


def _commit():
    """The commit this tree was stamped with before a GPU run (tools/stamp_head.sh), if any."""
    try:
        return open(os.path.join(ROOT, "HEAD_COMMIT")).read().strip() or None
    except OSError:
        return None


def make_paths(p0, p1, seed=123, cfg=None):
    """Paths p0..p1-1 of the synthetic batch, each from its own seeded stream
    (so a rank generates only its shard and N does not change the data)."""
    cfg = cfg or CONFIGS["c4"]
    H, n, m = cfg["horizon"], cfg["n"], cfg["m"]
    obs, act, rew = [], [], []
    for p in range(p0, p1):
        g = np.random.Generator(np.random.PCG64(seed * 100003 + p))
        obs.append(g.standard_normal((H, n), dtype=np.float32))
        act.append(g.standard_normal((H, m), dtype=np.float32))
        rew.append(g.standard_normal(H))
    return obs, act, rew


def baseline_coeffs(cfg=None):
    from mjrl_amd.utils.gym_env import EnvSpec
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    cfg = cfg or CONFIGS["c4"]
    obs, _, rew = make_paths(0, min(20, cfg["paths"]), cfg=cfg)
    paths = []
    for o, r in zip(obs, rew):
        ret = np.zeros_like(r)
        acc = 0.0
        for t in range(len(r) - 1, -1, -1):
            acc = r[t] + GAMMA * acc
            ret[t] = acc
        paths.append(dict(observations=o.astype(np.float64), rewards=r, returns=ret))
    b = LinearBaseline(EnvSpec(cfg["n"], cfg["m"], cfg["horizon"], 1))
    b.fit(paths)
    return b


def param_shapes(cfg):
    h0, h1 = cfg["hidden"]
    n, m = cfg["n"], cfg["m"]
    return [(h0, n), (h0,), (h1, h0), (h1,), (m, h1), (m,), (m,)]


def initial_theta(cfg=None):
    """The update's starting parameters: N(0, 0.05^2) weights from RandomState(0)
    in trainable_params order, log_std 0."""
    cfg = cfg or CONFIGS["c4"]
    rs = np.random.RandomState(0)
    theta = np.concatenate([(rs.randn(int(np.prod(s))) * 0.05).ravel() for s in param_shapes(cfg)]).astype(np.float32)
    theta[-cfg["m"]:] = 0.0
    return theta


def demo_share(cfg, rank, world):
    """This rank's demonstration paths (DAPG): a contiguous share, each demo row
    staged once over all ranks (DAPG._rank_share)."""
    nd = cfg.get("demos", 0)
    if not nd:
        return None
    from mjrl_amd.comm import partition_paths
    d0, d1 = partition_paths(np.full(nd, cfg["horizon"]), world)[rank]
    o, a, _ = make_paths(d0, d1, seed=977, cfg=cfg)
    return o, a


def stage_shard(p0, p1, device, base, cfg=None, demos=None, dtype=np.float32):
    """This rank's paths as a device batch in the layout train_step stages them
    (BatchREINFORCE.staging_dtype: float32 observations / actions by default,
    f64 rewards and baseline predictions)."""
    from mjrl_amd.engine import DeviceBatch
    cfg = cfg or CONFIGS["c4"]
    H, n, m = cfg["horizon"], cfg["n"], cfg["m"]
    obs, act, rew = make_paths(p0, p1, cfg=cfg)
    P = p1 - p0
    T = P * H
    T_demo = 0
    if demos is not None:
        obs, act = obs + demos[0], act + demos[1]
        T_demo = sum(len(o) for o in demos[0])
    tdt = torch.float32 if np.dtype(dtype) == np.float32 else torch.float64
    ho = torch.empty((T + T_demo, n), dtype=tdt, pin_memory=True)
    orange = None
    if tdt == torch.float32:
        # the staging pass (engine.host_stage, as DeviceBatch.from_paths runs it):
        # f32 rows plus each column's range, from which the split rows' column
        # scales follow (DeviceBatch.obs_range)
        from mjrl_amd.engine import host_stage
        lo, hi = np.full(n, np.inf, np.float32), np.full(n, -np.inf, np.float32)
        offs = np.concatenate([[0], np.cumsum([len(o) for o in obs])])
        host_stage(obs, ho.numpy(), offs, 0, len(obs), lo, hi)
        orange = torch.from_numpy(np.stack([lo, hi])).to(device)
    else:
        np.concatenate(obs, out=ho.numpy(), casting="same_kind")
    ha = torch.empty((T + T_demo, m), dtype=tdt, pin_memory=True)
    np.concatenate(act, out=ha.numpy(), casting="same_kind")
    rw = np.concatenate(rew)
    bl = np.concatenate([base.predict(dict(observations=o.astype(np.float64), rewards=r))
                         for o, r in zip(obs[:P], rew)])
    off = (np.arange(P + 1, dtype=np.int64) * H)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    return DeviceBatch(ho.to(device), ha.to(device), t(rw), t(bl), t(off), t(np.zeros(P, np.uint8)), T_demo=T_demo,
                       obs_range=orange)


def update_args(cfg, T_total):
    upd = dict(algo=cfg["algo"], gamma=GAMMA, gae_lambda=LAM, cg_iters=CG_ITERS, damping=DAMPING,
               T_global=float(T_total), trpo_verbose=False)
    upd.update(cfg["step"])
    return upd


def _cpu_list(cpus):
    """'0-15' / '0-7,16-23' form of a CPU id set."""
    cpus = sorted(cpus)
    out, a = [], None
    for i, c in enumerate(cpus):
        if a is None:
            a = c
        if i + 1 == len(cpus) or cpus[i + 1] != c + 1:
            out.append(str(a) if a == c else "%d-%d" % (a, c))
            a = None
    return ",".join(out)


def cpu_baseline(rows, base, reps=3, cfg=None):
    """The oracle (CPU restatement of the reference update) on `rows` timesteps,
    torch on the host cores this process may use, pinned: the process's affinity
    is narrowed to the first host_cores() CPUs of its allowed set for the
    duration (and restored), so the threads do not migrate over a box shared with
    other jobs; the set is recorded.  One warm-up update on a tenth of the sample,
    then the median of `reps` (>= 3 at Humanoid 1M, >= 10 for the
    smaller configs)."""
    from oracle import npg_cpu as O
    cfg = cfg or CONFIGS["c4"]
    H, n, m, hidden = cfg["horizon"], cfg["n"], cfg["m"], cfg["hidden"]
    cores = host_cores()
    saved_aff = None
    try:
        saved_aff = os.sched_getaffinity(0)
        pinned = set(sorted(saved_aff)[:cores])
        os.sched_setaffinity(0, pinned)
    except (AttributeError, OSError):
        pinned = None
    torch.set_num_threads(cores)
    P = max(1, rows // H)
    obs, act, rew = make_paths(0, P, cfg=cfg)
    obs = np.concatenate(obs).astype(np.float64)
    act = np.concatenate(act).astype(np.float64)
    rew = np.concatenate(rew)
    lengths = np.full(P, H)
    bl = np.concatenate([base.predict(dict(observations=o, rewards=r))
                         for o, r in zip(O.split(obs, lengths), O.split(rew, lengths))])
    theta = initial_theta(cfg)
    kw = dict(algo=cfg["algo"], cg_iters=CG_ITERS, damping=DAMPING)
    if cfg["algo"] == "npg":
        kw["n_step_size"] = cfg["step"]["n_step_size"]
    else:
        kw["kl_dist"] = cfg["step"]["kl_dist"]
    if cfg["algo"] == "dapg":
        dmo = demo_share(cfg, 0, 1)
        kw.update(demo_obs=np.concatenate(dmo[0]).astype(np.float64),
                  demo_act=np.concatenate(dmo[1]).astype(np.float64), demo_coef=cfg["step"]["demo_coef"])

    def one(r):
        pol = O.Policy(n, m, hidden, theta.astype(np.float64), None)
        Pr = max(1, r // H)
        r = Pr * H
        t0 = time.perf_counter()
        ret, adv = O.returns_and_advantages(rew[:r], bl[:r], lengths[:Pr], np.zeros(Pr, bool), GAMMA, LAM)
        O.update(pol, obs[:r], act[:r], adv, rew[:r], lengths[:Pr], **kw)
        return time.perf_counter() - t0

    log("cpu baseline: %d timesteps on %d threads" % (P * H, cores))
    try:
        # warm-up at the full sample size: the first update at a new size pays the
        # first touch of its multi-GB temporaries (round 5's first full rep: 50.8 s
        # against 35.7 / 36.1 s after a warm-up on a tenth)
        one(P * H)
        ts = []
        for i in range(reps):
            ts.append(one(P * H))
            log("cpu baseline update %d: %.2f s" % (i + 1, ts[-1]))
    finally:
        if saved_aff is not None:
            os.sched_setaffinity(0, saved_aff)
    ts.sort()
    dt = ts[len(ts) // 2]
    full = P * H >= cfg["paths"] * H
    return dict(value=round(P * H / dt, 1), unit="timesteps/s", cores=cores, kind="port", cpu=cpu_model(),
                affinity=_cpu_list(pinned) if pinned else None, reps=reps, median_s=round(dt, 4),
                spread=round((ts[-1] - ts[0]) / dt, 4),
                sample="%s: %d paths x %d steps (%d timesteps) of the %s workload%s, one update (returns + GAE + "
                       "train_from_paths), oracle/npg_cpu.py on %d torch threads pinned to CPUs %s: median of %d "
                       "updates %.3f s (all: %s)"
                       % ("the full batch" if full else "a bounded sample", P, H, P * H, cfg["workload"],
                          "" if full else " (the rate is the sample's; --cpu-full times the whole batch)",
                          cores, _cpu_list(pinned) if pinned else "(affinity not settable)", reps, dt,
                          ", ".join("%.3f" % t for t in ts)))


def host_threads():
    from mjrl_amd.engine import _host_threads
    return _host_threads()


def e2e_from_host(paths_range, eng, th0, base, upd, device, cfg, reps=3):
    """End-to-end update from numpy sampler paths (what train_agent sees):
    f64 paths -> threaded f32 conversion into reused pinned slabs, chunked H2D
    overlapping it -> device LinearBaseline predict -> update -> readback.
    Reported beside `value` (never as it): SURVEY.md §8 d1."""
    from mjrl_amd.engine import DeviceBatch
    p0, p1 = paths_range
    obs, act, rew = make_paths(p0, p1, cfg=cfg)
    paths = [dict(observations=o.astype(np.float64), actions=a.astype(np.float64), rewards=r, terminated=False)
             for o, a, r in zip(obs, act, rew)]
    del obs, act
    T = sum(len(p["rewards"]) for p in paths)
    th = th0.clone()
    stage_ms = []

    def one():
        nonlocal th
        t0 = time.perf_counter()
        b = DeviceBatch.from_paths(paths, device, baseline=base, reuse=True)
        torch.cuda.synchronize()
        stage_ms.append((time.perf_counter() - t0) * 1e3)
        eng.update(b, th, **upd)
        th = eng.vec["theta_new"].clone()
        torch.cuda.synchronize()

    one()
    one()
    stage_ms.clear()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        one()
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    tl = e2e_timeline(paths, eng, th, base, upd, device)
    return dict(value=round(T / dt, 1), unit="timesteps/s", ms_per_step=round(dt * 1e3, 2),
                staging_ms=round(float(np.median(stage_ms)), 2), timeline=tl,
                note="numpy f64 paths -> f32 into reused pinned slabs on %d host threads, chunked H2D "
                     "overlapping the conversion -> device LinearBaseline.predict -> update -> readback; "
                     "median of %d (staging_ms: the staging alone, synchronised)" % (host_threads(), reps))


def e2e_stream(paths_range, eng, th0, base, upd, device, cfg, nslots=64):
    """train_step's post-sampling critical path with the sampler feeding the
    staging (samplers/stream_staging.StreamSink): the
    vectorised sampler's per-step calls are replayed on the synthetic paths
    (nslots lock-stepped slots, each observation / action row handed over at
    its step, each trajectory copied to HBM when it ends), then from the last
    hand-over: the device batch (gather + 1-D slots) -> update -> readback.
    Reported beside `value` (never as it)."""
    from mjrl_amd.samplers.stream_staging import StreamSink
    p0, p1 = paths_range
    obs, act, rew = make_paths(p0, p1, cfg=cfg)
    paths = [dict(observations=o.astype(np.float64), actions=a.astype(np.float64), rewards=r, terminated=False)
             for o, a, r in zip(obs, act, rew)]
    del obs, act
    N, H = len(paths), cfg["horizon"]
    T = N * H

    def one(th):
        sink = StreamSink(cfg["n"], cfg["m"], H, N, device, baseline=base, nslots=nslots)
        tf = 0.0
        for g0 in range(0, N, nslots):   # lock-stepped rounds of nslots trajectories
            grp = list(range(g0, min(N, g0 + nslots)))
            for j, ep in enumerate(grp):
                sink.begin(j, ep)
            slots = list(range(len(grp)))
            f0 = time.perf_counter()
            for t in range(H):
                ts = [t] * len(grp)
                sink.rows(slots, np.stack([paths[ep]["observations"][t] for ep in grp]), ts)
                sink.actions(slots, np.stack([paths[ep]["actions"][t] for ep in grp]), ts)
                sink.rewards(slots, [paths[ep]["rewards"][t] for ep in grp], ts)
            for j in slots:
                sink.finish(j, H, False)
            tf += time.perf_counter() - f0
        t0 = time.perf_counter()
        b = sink.batch(paths)
        torch.cuda.synchronize()   # the last copies and the 1-D slots (split out for the breakdown)
        t1 = time.perf_counter()
        eng.update(b, th, **upd)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t2 - t0) * 1e3, tf * 1e3, (t1 - t0) * 1e3, (t2 - t1) * 1e3

    one(th0.clone())
    runs = [one(th0.clone()) for _ in range(2)]
    crit = float(np.median([r[0] for r in runs]))
    feed = float(np.median([r[1] for r in runs]))
    return dict(post_sampling_ms=round(crit, 2), feed_ms=round(feed, 1), feed_us_per_row=round(feed * 1e3 / T, 3),
                batch_ms=round(float(np.median([r[2] for r in runs])), 2),
                update_ms=round(float(np.median([r[3] for r in runs])), 2),
                timesteps=T, slots=nslots,
                note="StreamSink fed per lock step as the vectorised sampler feeds it (observation rows through "
                     "mjrl_host_stage_rows_f64x into pinned per-slot slabs, each trajectory copied to HBM in runs "
                     "of StreamSink.FLUSH_ROWS rows as it is sampled and the rest when it ends); batch_ms = the "
                     "last runs' copies and the 1-D slots, update_ms = the update after them; post_sampling_ms = from the last trajectory's hand-over to the update's readback "
                     "(the padded slabs are the batch when every path runs the full horizon, else one device "
                     "gather; offsets / flags; update); feed_ms = the sampler-side cost of the "
                     "hand-overs (spread over sampling, timed without environments); median of 2")


def e2e_timeline(paths, eng, th, base, upd, device):
    """One more end-to-end update with the staging traced (engine._PinnedStaging
    .trace): host conversion spans per chunk, each chunk's H2D copy timed with
    events on the copy stream, and the device update after the staging, all in
    ms from the update's start.  Summarised: conversion span, H2D span and busy
    time, bytes and GB/s, and the update's tail after the last copy."""
    from mjrl_amd import engine as E
    torch.cuda.synchronize()
    E._STAGING.trace = tr = []
    ref = torch.cuda.Event(enable_timing=True)
    ref.record()
    h0 = time.perf_counter()
    try:
        b = E.DeviceBatch.from_paths(paths, device, baseline=base, reuse=True)
    finally:
        E._STAGING.trace = None
    u0 = torch.cuda.Event(enable_timing=True)
    u0.record()
    eng.update(b, th, **upd)
    u1 = torch.cuda.Event(enable_timing=True)
    u1.record()
    torch.cuda.synchronize()
    h1 = time.perf_counter()
    fills = [c["fill"] for c in tr if c["fill"]]
    cp = [(ref.elapsed_time(c["ev"][0]), ref.elapsed_time(c["ev"][1]), c["bytes"], c["slot"]) for c in tr]
    nbytes = sum(c[2] for c in cp)
    busy = sum(c[1] - c[0] for c in cp)
    by_slot = {}
    for c in cp:
        d = by_slot.setdefault(c[3], [0, 0.0])
        d[0] += c[2]
        d[1] += c[1] - c[0]
    return dict(
        chunks=len(cp), h2d_bytes=nbytes,
        convert_ms=[round((min(f[0] for f in fills) - h0) * 1e3, 2), round((max(f[1] for f in fills) - h0) * 1e3, 2)]
        if fills else None,
        h2d_ms=[round(min(c[0] for c in cp), 2), round(max(c[1] for c in cp), 2)] if cp else None,
        h2d_busy_ms=round(busy, 2), h2d_GBps=round(nbytes / busy / 1e6, 1) if busy else None,
        h2d_by_slot={k: dict(bytes=v[0], busy_ms=round(v[1], 3)) for k, v in by_slot.items()},
        update_ms=[round(ref.elapsed_time(u0), 2), round(ref.elapsed_time(u1), 2)],
        wall_ms=round((h1 - h0) * 1e3, 2),
        note="ms from the update's start: host f64 -> f32 conversion span (first chunk start, last chunk end), "
             "device H2D span and summed copy time, the update after the staging (device events)")


def fvp_kernel_key(path, split, mp, np_, h0, h1):
    """(name, demangled rocprof instantiation) of the FVP accumulate kernel: the
    template arguments as kx.h / ks.h instantiate it (k_kx<MP, KG, MODE = 1 (FVP),
    PACK = false>, k_ks<MP, KG, 1, false>)."""
    if path == 0:
        return "k_rows<%d,%d,%d,FVP>+k_wgrad" % (h0, h1, mp), "k_rows<%d, %d, %d, 1>" % (h0, h1, mp)
    if path == 2 and split:
        return "k_kx<%d,%d,FVP>" % (mp, np_ // 32), "k_kx<%d, %d, 1, false>" % (mp, np_ // 32)
    if path == 2:
        return "k_ks<%d,%d,FVP>" % (mp, np_ // 32), "k_ks<%d, %d, 1, false>" % (mp, np_ // 32)
    return "k_fused<%d,%d,%d,FVP>" % (h0, h1, mp), "k_fused<%d, %d, %d, " % (h0, h1, mp)


def kernel_names(eng, cfg):
    """(name, rocprof key, flops/row) of the FVP accumulate step and of the gather."""
    fl = flops_per_row(cfg["n"], cfg["m"], *cfg["hidden"])
    h0, h1 = cfg["hidden"]
    acc = fvp_kernel_key(eng.accumulate_path(), eng.split, eng.shape.mp, eng.shape.np, eng.shape.h0, eng.shape.h1)
    return acc + (fl["rows_fvp"] + fl["weight_grads"], "k_gather", "k_gather", 0)


def main():
    # stdout carries the one JSON line and nothing else: libraries that print to
    # fd 1 (RCCL's version banner at communicator init) are sent to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--paths", type=int, default=None, help="paths per update (default: the config's)")
    ap.add_argument("--cpu-rows", type=int, default=None,
                    help="timesteps of a bounded CPU-baseline sample (default: the config's full batch; about "
                         "40 s per update at Humanoid 1M on 16 cores)")
    ap.add_argument("--cpu-full", action="store_true", help="(the default) CPU baseline on the full batch")
    ap.add_argument("--cpu-reps", type=int, default=None,
                    help="timed CPU-baseline updates (default: 3 at c4, 10 for the smaller configs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end-from-host-paths measurement")
    ap.add_argument("--no-f32", action="store_true", help="skip the exact-f32 companion timing")
    ap.add_argument("--stage-dtype", choices=("f32", "f64"), default="f32",
                    help="observations / actions of the device-resident batch: f32 as train_step stages them "
                         "(BatchREINFORCE.staging_dtype), or the sampler's f64")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse the N > 1 "
                         "path with several ranks on one GPU)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "torch"],
                    help="N > 1 over nccl: RCCL driven directly on the update's stream (comm.RcclComm: the "
                         "sharded update is one captured hipGraph, collectives inside) or torch.distributed's "
                         "own collectives (eager)")
    ap.add_argument("--sharded-path", action="store_true",
                    help="one GPU: run the sharded code path on a one-rank RCCL communicator (all-gathered "
                         "moments, an all-reduce between every FVP and its CG step, RCCL calls inside the "
                         "captured graph) -- the per-rank schedule of an N-GPU run, on this GPU's shard")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="replay each update as one captured hipGraph (one GPU): auto = the engine's "
                         "default, graphs for batches up to engine.GRAPH_AUTO_ROWS rows")
    ap.add_argument("--precision", default=None, choices=["auto", "split", "f32"],
                    help="first-layer MFMA form (UpdateEngine precision; default: split where supported)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.paths:
        cfg["paths"] = args.paths
    n, m, hidden, H = cfg["n"], cfg["m"], cfg["hidden"], cfg["horizon"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    dev_idx = local % ndev if args.backend == "gloo" else local
    torch.cuda.set_device(dev_idx)
    device = torch.device("cuda", dev_idx)
    comm = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        from mjrl_amd.comm import DistComm, RcclComm
        comm = RcclComm(device) if args.backend == "nccl" and args.comm == "rccl" else DistComm()
    elif args.sharded_path:
        from mjrl_amd.comm import RcclComm
        comm = RcclComm.local(device)
    from mjrl_amd.comm import partition_paths
    from mjrl_amd.engine import UpdateEngine

    base = baseline_coeffs(cfg)
    p0, p1 = partition_paths(np.full(cfg["paths"], H), world)[rank]
    batch = stage_shard(p0, p1, device, base, cfg, demo_share(cfg, rank, world),
                        np.float32 if args.stage_dtype == "f32" else np.float64)
    T_total = cfg["paths"] * H

    eng = UpdateEngine(n, m, hidden, device=device, comm=comm, precision=args.precision)
    th0 = torch.from_numpy(initial_theta(cfg)).to(device)
    th = th0.clone()
    upd = update_args(cfg, T_total)
    eng.graphs = {"auto": "auto", "on": True, "off": False}[args.graph]
    # per-FVP (start, accumulate done, gather done) events on eager steps; a captured
    # graph is kept free of them (30 event nodes per update measured +3 % on the
    # replay) and the kernel timings come from eager steps after the timed region
    eng.kernel_timing = None if eng.graphs else []

    def step(graph=None, e=eng):
        nonlocal th
        e.update(batch, th, graph=graph, **upd)
        th = e.vec["theta_new"].clone()

    for _ in range(args.warmup):
        step()
    if eng.kernel_timing is not None:
        eng.kernel_timing.clear()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    log("timed region: %d steps, %.3f ms per step" % (args.steps, elapsed / args.steps * 1e3))
    per_rank = [dict(rank=rank, rows=batch.T, ms_per_step=round(elapsed / args.steps * 1e3, 3))]
    if world > 1:
        # every rank's own rows and time (so the line shows the shards and how far
        # apart the ranks finished), then the max over ranks as the job's time
        t = torch.tensor([float(rank), float(batch.T), elapsed], dtype=torch.float64,
                         device=device if args.backend == "nccl" else "cpu")
        allt = [torch.zeros_like(t) for _ in range(world)]
        torch.distributed.all_gather(allt, t)
        per_rank = [dict(rank=int(a[0]), rows=int(a[1]), ms_per_step=round(float(a[2]) / args.steps * 1e3, 3))
                    for a in (x.cpu().numpy() for x in allt)]
        elapsed = max(float(x[2].item()) for x in allt)

    # dominant-kernel roofline from live HIP events on the launch stream, recorded
    # around every FVP of eager steps: the timed region's when it ran eager, else
    # the same update run eagerly after it (which also gives eager_ms_per_step)
    graphed = bool(eng.graphs) and eng._gstate.get("graph") is not None
    samples = [] if eng.kernel_timing is None else \
        [(a.elapsed_time(b), b.elapsed_time(c)) for a, b, c in eng.kernel_timing]
    eager_ms = None
    if graphed:
        eng.kernel_timing = []
        step(graph=False)
        torch.cuda.synchronize()
        eng.kernel_timing.clear()
        te = time.perf_counter()
        for _ in range(3):   # the same update without the graph
            step(graph=False)
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - te) / 3 * 1e3
        samples = [(a.elapsed_time(b), b.elapsed_time(c)) for a, b, c in eng.kernel_timing]
    if not samples:   # no events available: time the accumulate / gather pair alone
        eng.kernel_timing = []
        step(graph=False)
        samples = [(a.elapsed_time(b), b.elapsed_time(c)) for a, b, c in eng.kernel_timing]
    t_acc = np.mean([a for a, _ in samples]) / 1e3
    t_gat = np.mean([b for _, b in samples]) / 1e3
    acc_name, acc_key, acc_fl, gat_name, gat_key, gat_fl = kernel_names(eng, cfg)
    rows_rank = batch.T
    np_ = eng.shape.np
    h0, h1 = hidden
    # algorithmic HBM bytes per row of one FVP launch: the observation row (f32, or the
    # split-f16 hi / lo pair + row scale) and the cached a0 / a1 activations
    fvp_bytes = 4 * np_ + (4 if eng.split else 0) + 4 * (h0 + h1)
    kern = {acc_name: dict(avg_ms=t_acc * 1e3, tflops=acc_fl * rows_rank / t_acc / 1e12),
            gat_name: dict(avg_ms=t_gat * 1e3, tflops=gat_fl * rows_rank / t_gat / 1e12)}
    dom = max(kern, key=lambda k: kern[k]["avg_ms"])
    traffic, tsrc, terr = pmc_traffic(acc_key if dom == acc_name else gat_key) if args.config == "c4" \
        else (None, None, None)
    if terr is not None:
        log("WARNING: roofline.traffic unavailable: " + terr)
    if traffic is not None and rows_rank != N_PATHS * HORIZON:
        # the committed PMC pass is the default 1-GPU launch (1M rows); scale per row
        traffic = traffic * rows_rank / (N_PATHS * HORIZON)
    # the roofline that binds the dominant kernel: the larger of its ideal MFMA time
    # (algorithmic flops at the matrix peak of the form it computes in) and its ideal
    # HBM time (algorithmic bytes at 8 TB/s)
    t_dom = kern[dom]["avg_ms"] * 1e-3
    peak_mm = PEAK_SPLIT if eng.precision == "split" else PEAK_F32_MFMA
    flops_dom = (acc_fl if dom == acc_name else gat_fl) * rows_rank
    bytes_dom = fvp_bytes * rows_rank if dom == acc_name else None
    t_mm = flops_dom / (peak_mm * 1e12)
    t_hbm = bytes_dom / (PEAK_HBM * 1e9) if bytes_dom else 0.0
    if t_hbm > t_mm:
        roof = dict(bound="hbm", kernel=dom, achieved=round(bytes_dom / t_dom / 1e9, 1), peak=PEAK_HBM, unit="GB/s",
                    frac=round(bytes_dom / t_dom / 1e9 / PEAK_HBM, 4), bytes_per_timestep=fvp_bytes)
    else:
        roof = dict(bound="mfma", kernel=dom, achieved=round(flops_dom / t_dom / 1e12, 3), peak=peak_mm,
                    unit="TFLOP/s", frac=round(flops_dom / t_dom / 1e12 / peak_mm, 4))
    roof.update(traffic=None if traffic is None else round(traffic),
                traffic_unit="bytes/launch (HBM, PMC)", traffic_source=tsrc, traffic_error=terr,
                traffic_GBps=None if traffic is None else round(traffic / t_dom / 1e9, 1),
                flops_per_timestep=acc_fl if dom == acc_name else gat_fl, rows_per_launch=rows_rank,
                mfma_form="split-f16 (3 x v_mfma_f32_16x16x32_f16 per f32 product), peak %.1f TFLOP/s f32-equivalent"
                          % PEAK_SPLIT if eng.precision == "split" else "f32 (v_mfma_f32_16x16x4_f32)",
                ideal_ms=dict(mfma=round(t_mm * 1e3, 4), hbm=round(t_hbm * 1e3, 4)),
                achieved_tflops=round(flops_dom / t_dom / 1e12, 3),
                launches=len(samples), kernels={k: {kk: round(vv, 4) for kk, vv in v.items()}
                                                for k, v in kern.items()})
    # whole-update algorithmic FLOP rate, all kernels and gaps included
    ufl = update_flops_per_row(n, m, h0, h1, CG_ITERS)
    ut = ufl * T_total / (elapsed / args.steps) / 1e12
    # priced against the peak of the form the kernels compute in (split-f16: three
    # f16 MFMAs per f32 product, PEAK_SPLIT), not the exact-f32 matrix peak
    peak_u = PEAK_SPLIT if eng.precision == "split" else PEAK_F32_MFMA
    roof["update"] = dict(flops_per_timestep=ufl, achieved=round(ut, 3), unit="TFLOP/s",
                          peak=round(peak_u * world, 1), frac=round(ut / (peak_u * world), 4),
                          peak_form="split-f16 (f32-equivalent)" if eng.precision == "split" else "exact f32 MFMA",
                          frac_of_exact_f32_peak=round(ut / (PEAK_F32_MFMA * world), 4),
                          note="algorithmic FLOPs of a whole update / wall time per update, vs n_gpus x the "
                               "matrix peak of the form the kernels use (frac); frac_of_exact_f32_peak prices "
                               "the same FLOPs against the exact-f32 MFMA peak, for comparison only")

    # the same update on the exact-f32 MFMA kernels (precision='f32'), for reference
    f32_ms = None
    if world == 1 and eng.precision == "split" and not args.no_f32:
        log("exact-f32 companion timing")
        e32 = UpdateEngine(n, m, hidden, device=device, precision="f32")
        e32.graphs = eng.graphs
        th = th0.clone()
        for _ in range(2):
            step(e=e32)
        torch.cuda.synchronize()
        tf = time.perf_counter()
        for _ in range(3):
            step(e=e32)
        torch.cuda.synchronize()
        f32_ms = (time.perf_counter() - tf) / 3 * 1e3
        del e32
        torch.cuda.empty_cache()

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        out = dict(metric=cfg["metric"], value=round(T_total * args.steps / elapsed, 1), unit="timesteps/s",
                   n_gpus=world, steps=args.steps, warmup=args.warmup, ms_per_step=round(ms, 3),
                   higher_is_better=True, scaling="strong",
                   vs_baseline=round(T_total * args.steps / elapsed / REF_CPU[args.config][0], 1)
                   if args.config in REF_CPU and not args.paths else None,
                   vs_baseline_source=REF_CPU[args.config][1] if args.config in REF_CPU and not args.paths else None,
                   dtype="f32" if eng.precision != "split" else "f32 (split-f16 MFMA, f32 accumulate)",
                   data="synthetic (seeded N(0,1) obs/act/rewards, LinearBaseline fitted on 20 paths)",
                   config=dict(workload=cfg["workload"], obs_dim=n, act_dim=m, hidden=list(hidden),
                               algo=cfg["algo"], timesteps=T_total, paths=cfg["paths"], horizon=H,
                               demo_timesteps=cfg.get("demos", 0) * H, cg_iters=CG_ITERS,
                               parallelism="dp%d" % world,
                               comm=type(eng.comm).__name__ + (" (one rank, sharded code path)"
                                                               if args.sharded_path and world == 1 else "")),
                   commit=_commit(),
                   ranks=per_rank,
                   comm_world_size=int(eng.comm.world_size),
                   comm_backend=(torch.distributed.get_backend() if world > 1 else None),
                   hipgraph=bool(graphed), eager_ms_per_step=None if eager_ms is None else round(eager_ms, 3),
                   f32_ms_per_step=None if f32_ms is None else round(f32_ms, 3),
                   roofline=roof)
        if world == 1 and not args.no_e2e and cfg["algo"] != "dapg":
            th = th0.clone()
            log("end-to-end from host paths")
            out["e2e_from_host"] = e2e_from_host((p0, p1), eng, th, base, upd, device, cfg)
            log("end-to-end with the sampler feeding the staging")
            out["e2e_stream"] = e2e_stream((p0, p1), eng, th0, base, upd, device, cfg)
        if world == 1 and not args.no_cpu_baseline:
            rows = T_total if (args.cpu_full or not args.cpu_rows) else min(args.cpu_rows, T_total)
            reps = args.cpu_reps or (3 if args.config == "c4" else 10)
            out["cpu_baseline"] = cpu_baseline(rows, base, reps=reps, cfg=cfg)
            # BASELINE.md holds no published number (vs_baseline stays null); the
            # ratio to the CPU restatement timed beside it on this host:
            out["vs_cpu_baseline"] = round(out["value"] / out["cpu_baseline"]["value"], 2)
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1:
        from mjrl_amd.comm import release_comms
        release_comms()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
