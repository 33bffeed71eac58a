"""BatchREINFORCE with the API of mjrl/algos/batch_reinforce.py:22-175; the
per-iteration update runs on the gfx950 engine (mjrl_amd.engine).

train_step keeps the reference's flow (batch_reinforce.py:58-103): sample on
host CPUs with the reference's samplers, returns + GAE, the policy update, then
baseline.fit on the paths.  Here the paths are staged into HBM once; the GAE
scan, the whole update and the statistics run on the GPU; returns / baseline /
advantages are written back into the path dicts for baseline.fit.

Several GPUs, two ways:
  - devices=[0, ..., 7] (or MJRL_AMD_DEVICES): this process stays the only one
    running the training loop (an unchanged train_agent: its directories,
    pickles and results.txt are written once) and never touches a GPU; each
    update runs on N worker processes, one per GPU (mjrl_amd/pool.py), over the
    sharded device path below;
  - one process per GPU (e.g. the script under `torchrun --nproc-per-node 8`):
    the communicator comes from comm.auto_comm(); rank r samples its
    ceil(N / world) share of the N paths with the pegasus seed offset of that
    share (the per-worker split of trajectory_sampler.py:37-45).
Either way the update all-reduces its sums over RCCL, every rank ends with the
same parameters, and the baseline is fitted on the union of the shards.
"""
import logging
import os
import time as timer

import multiprocessing as mp

import numpy as np
import torch

from ..comm import LocalComm, auto_comm, partition_paths, shard_count
from ..engine import DeviceBatch, UpdateEngine
from ..utils.logger import DataLog

logging.disable(logging.CRITICAL)   # as the reference's algos do at import

# QuadraticBaseline fits on the device up to this observation width (its Gram has
# n + n(n+1)/2 + 6 columns: 2,150 at 64; mjrl_quadratic_baseline_gram's limit)
QUADRATIC_DEVICE_MAX_N = 64


def _check_policy(policy):
    """Rejects, at agent construction, a policy shape no device kernel covers
    (engine.kernel_hidden: two hidden layers of width <= 256, act_dim <= 64);
    other hidden sizes run zero-padded to the next supported width."""
    from ..engine import kernel_hidden
    try:
        kernel_hidden(int(policy.n), int(policy.m), policy.hidden)
    except ValueError as e:
        raise ValueError("policy shape not supported by the mjrl_amd update engine: %s" % e) from None


def _samplers():
    """The reference's host-CPU samplers (MuJoCo stays on the CPU)."""
    try:
        import mjrl.samplers.trajectory_sampler as trajectory_sampler
        import mjrl.samplers.batch_sampler as batch_sampler
    except ImportError as e:   # pragma: no cover - needs the reference + gym + mujoco-py
        raise ImportError("train_step samples with mjrl's samplers (mjrl.samplers.*, gym, mujoco-py); "
                          "install mjrl alongside mjrl_amd, or stage your own paths and call "
                          "train_from_paths") from e
    return trajectory_sampler, batch_sampler


class BatchREINFORCE:
    algo = "vpg"
    # sampler of train_step's 'trajectories' mode: "reference" (mjrl's process-pool
    # samplers, policy.get_action per observation on the CPU) or "vector"
    # (samplers/vector_sampler.py, SURVEY.md §8f row f3: lock-stepped environments,
    # one device policy forward per step, the same trajectories for the same seeds);
    # default from MJRL_AMD_SAMPLER.  env_factory / num_envs configure "vector"
    # (default factory: mjrl.utils.get_environment(env_name)).
    sampler = None
    env_factory = None
    num_envs = 64
    # with the "vector" sampler: stage each trajectory to HBM while sampling goes on
    # (samplers/stream_staging.py; float32 staging, no demonstration rows)
    stream_staging = True
    # dtype the sampled observations / actions are staged to HBM in: float32 (the
    # policy's own input precision, half the PCIe bytes) or float64; None = auto
    # (staging_obs_dtype): float32, except float64 when the baseline is an
    # MLPBaseline that predicts from the staged rows (its features are
    # float32(clip(x) / 10) of the f64 x, mlp_baseline.py:37-56, which float32
    # rows cannot reproduce bit for bit).  With float32 rows a LinearBaseline still
    # sees the f64 values: the staging pass computes its predictions from them and
    # the device fit reads their low halves (DeviceBatch.obs_lo).
    staging_dtype = None
    # whether MJRL_AMD_DEVICES / devices= may hand the update to the GPU worker pool
    # (an algorithm whose update does not shard, PPO, runs in this process)
    _poolable = True

    def __init__(self, env, policy, baseline, learn_rate=0.01, seed=None, save_logs=False, device=None,
                 comm=None, devices=None):
        self.env = env
        self.policy = policy
        _check_policy(policy)
        self.baseline = baseline
        self.alpha = learn_rate
        self.seed = seed
        self.save_logs = save_logs
        self.running_score = None
        if save_logs:
            self.logger = DataLog()
        self._device = device
        self._comm = comm
        self._engine = None
        self._devices = devices

    # ---- device engine (never pickled: agents stay CPU-picklable) -----------
    def __getstate__(self):
        d = dict(self.__dict__)
        d["_engine"] = None
        d["_last_batch"] = None   # device tensors
        d.pop("_stream", None)    # pinned slabs / device slots of the streaming sink
        d.pop("_pre", None)       # views of a pool worker's shared segment
        if not isinstance(d.get("_comm"), (LocalComm, type(None))):
            d["_comm"] = None     # a process group does not pickle; re-resolved on use
        return d

    def staging_obs_dtype(self):
        """The dtype observations / actions of sampled paths are staged in (see
        staging_dtype)."""
        if self.staging_dtype is not None:
            return np.dtype(self.staging_dtype)
        return np.dtype(np.float64 if hasattr(self.baseline, "predict_device") else np.float32)

    def engine(self):
        if self._engine is None:
            comm = self.comm()
            device = self._device
            if device is None:   # the current device (auto_comm made cuda:LOCAL_RANK current)
                device = torch.device("cuda", torch.cuda.current_device())
            self._engine = UpdateEngine(self.policy.n, self.policy.m, self.policy.hidden, device=device,
                                        comm=comm, min_log_std=self.policy.min_log_std)
        self._engine.set_transformations(*self.policy.transformations())
        return self._engine

    def _sampler_kind(self):
        kind = self.sampler or os.environ.get("MJRL_AMD_SAMPLER", "reference")
        if kind not in ("reference", "vector"):
            raise ValueError("sampler must be 'reference' or 'vector', got %r" % kind)
        return kind

    def _pool(self):
        """The GPU worker pool of this agent (mjrl_amd/pool.py) when it runs on
        several devices from one controller process, else None."""
        from ..comm import launched_world
        from ..pool import resolve_devices, get_pool
        if not self._poolable or self._comm is not None or launched_world() is not None:
            return None
        devices = resolve_devices(getattr(self, "_devices", None))
        return None if devices is None else get_pool(devices)

    def _apply_pool(self, out, paths):
        """Rank 0's reply of a pooled update: parameters, the agent state the
        update changed, the iteration's log entries (then the success rate, as
        _update logs it), the fitted baseline."""
        import pickle
        self.policy.set_param_values(np.asarray(out["theta"], np.float32), set_new=True, set_old=True)
        for k, v in out["sync"].items():
            setattr(self, k, v)
        if self.save_logs:
            for k, v in out["logs"]:
                self.logger.log_kv(k, v)
            self._log_success(paths)
        if out.get("baseline") is not None:
            self.baseline.__dict__.update(pickle.loads(out["baseline"]).__dict__)
        return list(out["stats"])

    def comm(self):
        """The agent's communicator: the one passed in, else comm.auto_comm()
        (torch.distributed's group under torchrun, LocalComm otherwise)."""
        if self._comm is None:
            self._comm = auto_comm()
        return self._comm

    def _theta(self, old=False):
        params = self.policy.old_params if old else self.policy.trainable_params
        flat = np.concatenate([p.data.reshape(-1).numpy() for p in params]).astype(np.float32)
        return torch.from_numpy(flat).to(self.engine().device)

    def _same_old_new(self):
        return all(torch.equal(a.data, b.data) for a, b in zip(self.policy.old_params, self.policy.trainable_params))

    # ---- single passes (batch_reinforce.py:37-55) -----------------------------
    def CPI_surrogate(self, observations, actions, advantages):
        eng = self.engine()
        T = eng.load_rows(observations, actions, advantages)
        eng.forward_pass(self._theta(old=True), T)
        surr, _ = eng.eval_pass(self._theta(), T)
        return torch.tensor(surr)

    def kl_old_new(self, observations, actions):
        eng = self.engine()
        T = eng.load_rows(observations, actions)
        eng.forward_pass(self._theta(old=True), T)
        _, kl = eng.eval_pass(self._theta(), T)
        return torch.tensor(kl)

    def flat_vpg(self, observations, actions, advantages):
        if not self._same_old_new():
            raise ValueError("flat_vpg on the device path is the gradient at old == new parameters "
                             "(likelihood ratio 1), which is every call site of the reference")
        eng = self.engine()
        T = eng.load_rows(observations, actions, advantages)
        return eng.forward_pass(self._theta(), T).cpu().numpy().copy()

    # ---- one iteration (batch_reinforce.py:58-103) ---------------------------
    def train_step(self, N, sample_mode="trajectories", env_name=None, T=1e6, gamma=0.995, gae_lambda=0.98,
                   num_cpu="max"):
        if env_name is None:
            env_name = self.env.env_id
        if sample_mode != "trajectories" and sample_mode != "samples":
            print("sample_mode in NPG must be either 'trajectories' or 'samples'")
            quit()
        pool = self._pool()
        comm = self.comm() if pool is None else LocalComm()
        vector = sample_mode == "trajectories" and comm.world_size == 1 and self._sampler_kind() == "vector"
        trajectory_sampler, batch_sampler = (None, None) if vector else _samplers()
        ts = timer.time()
        if comm.world_size > 1:
            paths = self._sample_shard(trajectory_sampler, batch_sampler, comm, N, sample_mode, env_name, T,
                                       num_cpu)
        elif vector:
            if pool is not None:
                raise ValueError("the vector sampler runs the policy on a GPU; with devices=... the controller "
                                 "process keeps off the GPUs: use the reference samplers there")
            from ..samplers.vector_sampler import sample_paths_vectorized
            sinks = []
            if self.stream_staging and self.staging_obs_dtype() == np.float32 and self._demo_paths() is None:
                from ..samplers.stream_staging import StreamSink

                def sink(n_paths, horizon, nslots):
                    sinks.append(StreamSink(self.policy.n, self.policy.m, horizon, n_paths, self.engine().device,
                                            baseline=self.baseline, nslots=nslots))
                    return sinks[-1]
            else:
                sink = None
            paths = sample_paths_vectorized(N, self.policy, T, env=self.env_factory, env_name=env_name,
                                            pegasus_seed=self.seed, num_envs=self.num_envs,
                                            device=self.engine().device, sink=sink)
            if sinks:
                self._stream = sinks[0]
        elif sample_mode == "trajectories":
            paths = trajectory_sampler.sample_paths_parallel(N, self.policy, T, env_name, self.seed, num_cpu)
        else:
            paths = batch_sampler.sample_paths(N, self.policy, T, env_name=env_name, pegasus_seed=self.seed,
                                               num_cpu=num_cpu)
        if self.save_logs:
            self.logger.log_kv("time_sampling", timer.time() - ts)
        self.seed = self.seed + N if self.seed is not None else self.seed

        if pool is not None:
            # the update and the baseline fit on the GPU workers; this process keeps
            # the paths (returns / baseline / advantages written back), the logs and
            # the policy / baseline objects the caller pickles
            out = pool.step(self, paths, "samples", gamma, gae_lambda, fit=True, return_errors=self.save_logs)
            eval_statistics = self._apply_pool(out, paths)
            eval_statistics.append(N)
            if self.save_logs:
                self.logger.log_kv("time_VF", out["time_VF"])
                self.logger.log_kv("VF_error_before", out["fit_errors"][0])
                self.logger.log_kv("VF_error_after", out["fit_errors"][1])
            return eval_statistics

        eval_statistics = self.train_from_samples(paths, gamma, gae_lambda)
        eval_statistics.append(N)
        if self.save_logs:
            ts = timer.time()
            error_before, error_after = self._fit_baseline(paths, return_errors=True)
            self.logger.log_kv("time_VF", timer.time() - ts)
            self.logger.log_kv("VF_error_before", error_before)
            self.logger.log_kv("VF_error_after", error_after)
        else:
            self._fit_baseline(paths)
        return eval_statistics

    def _sample_shard(self, trajectory_sampler, batch_sampler, comm, N, sample_mode, env_name, T, num_cpu):
        """This rank's share of the sampling.  'trajectories': shard_count(N) paths
        with pegasus seed `seed + first` (the offset trajectory_sampler.py:40-44
        gives worker i).  'samples': n_r = ceil(N / world) timesteps.  On one core
        (batch_sampler.sample_paths_one_core: one seed per path, and a path has at
        least one step, so at most n_r seeds) the rank's seed is `seed + r n_r`,
        rank r's slot of the iteration's N-seed window (the reference itself
        advances the seed by N per iteration, batch_reinforce.py:84; an offset of
        r N would hand rank r - 1 of the next iteration exactly rank r's starting
        seed of this one).  On several cores the reference's loop
        (batch_sampler.py:39-51) advances its seed cumulatively
        (`pegasus_seed += paths_so_far`), far past n_r, so rank slots of any fixed
        width could overlap and two ranks would replay the same env resets in one
        batch: _sample_calls keeps that loop (paths_per_call paths per call until
        more than n_r steps) with the calls of all ranks interleaved instead, call
        k of rank r seeded at `seed + (k world + r) w`, w the seeds one call uses —
        disjoint across ranks and calls within the iteration.  num_cpu='max'
        becomes this rank's share of the host cores."""
        if num_cpu is None or num_cpu == "max":
            num_cpu = max(1, mp.cpu_count() // comm.world_size)
        if sample_mode == "trajectories":
            n_r, first = shard_count(N, comm.world_size, comm.rank)
            if n_r == 0:
                raise ValueError("train_step(N=%d) on %d ranks: every rank needs at least one path"
                                 % (N, comm.world_size))
            seed = self.seed + first if self.seed is not None else None
            return trajectory_sampler.sample_paths_parallel(n_r, self.policy, T, env_name, seed, num_cpu)
        n_r = int(np.ceil(N / comm.world_size))
        if num_cpu != 1:
            return self._sample_calls(trajectory_sampler, comm, n_r, env_name, T, num_cpu)
        seed = self.seed + comm.rank * n_r if self.seed is not None else None
        return batch_sampler.sample_paths(n_r, self.policy, T, env_name=env_name, pegasus_seed=seed,
                                          num_cpu=num_cpu)

    def _sample_calls(self, trajectory_sampler, comm, n_r, env_name, T, num_cpu, paths_per_call=5):
        """batch_sampler.sample_paths' multi-core loop (batch_sampler.py:39-51) for
        rank r of a sharded samples-mode step, seeds interleaved over the ranks
        (see _sample_shard).  One call of trajectory_sampler.sample_paths_parallel
        seeds worker i at base + i ceil(P / c) (trajectory_sampler.py:37-44), so it
        uses w = c ceil(P / c) seeds, c = min(cpu_count, num_cpu)."""
        c = min(mp.cpu_count(), int(num_cpu))
        w = c * int(np.ceil(paths_per_call / c))
        paths, so_far, k = [], 0, 0
        while so_far <= n_r:
            seed = self.seed + (k * comm.world_size + comm.rank) * w if self.seed is not None else None
            new = trajectory_sampler.sample_paths_parallel(paths_per_call, self.policy, T, env_name, seed, num_cpu,
                                                           suppress_print=True, mode="sample")
            paths += new
            so_far += int(np.sum([len(p["rewards"]) for p in new]))
            k += 1
        return paths

    def _fit_baseline(self, paths, return_errors=False):
        """baseline.fit(paths) (batch_reinforce.py:93-101).  A LinearBaseline, and a
        QuadraticBaseline of up to QUADRATIC_DEVICE_MAX_N observation columns, is
        fitted on the device from the batch still in HBM (its Gram products are
        the T x k work); other baselines fit on the host.
        Sharded (world > 1), every rank fits on the union of all ranks' paths:
        the LinearBaseline Gram is all-reduced on device, a baseline with ridge
        normal equations (_features / _reg_coeff: Quadratic) all-reduces its
        host F^T F, F^T y and error sums, a device MLPBaseline all-reduces its
        minibatch gradients, and any other baseline gets the union of the paths
        (all_gather of observations / rewards / returns)."""
        batch = getattr(self, "_last_batch", None)
        self._last_batch = None
        comm = self.comm()
        kind = type(self.baseline).__name__
        if batch is not None and kind in ("LinearBaseline", "QuadraticBaseline") \
                and hasattr(self.baseline, "_reg_coeff") and batch.T == sum(len(p["rewards"]) for p in paths) \
                and (kind == "LinearBaseline" or batch.obs.shape[1] <= QUADRATIC_DEVICE_MAX_N):
            # float32 rows of values that are not float32s: the fit reads their low
            # halves too (staged now from the f64 paths), i.e. the sampler's values
            fit = self.engine().fit_linear_baseline if kind == "LinearBaseline" else \
                self.engine().fit_quadratic_baseline
            return fit(batch, self.baseline, return_errors=return_errors, obs_lo=batch.obs_lo(paths))
        if comm.world_size > 1:
            return _fit_sharded(self.baseline, paths, comm, return_errors)
        return self.baseline.fit(paths, return_errors=return_errors) if return_errors else self.baseline.fit(paths)

    def train_from_samples(self, paths, gamma, gae_lambda):
        """Returns + advantages + update from raw sampled paths with one staging:
        compute_returns / compute_advantages (process_samples.py:3-35) then
        train_from_paths, fused on the device.  Writes returns / baseline /
        advantages into the path dicts like the reference does."""
        eng = self.engine()
        stream = self.__dict__.pop("_stream", None)
        if stream is not None:   # staged while sampling (vector sampler + StreamSink)
            batch = stream.batch(paths)
        else:
            batch = DeviceBatch.from_paths(paths, eng.device, baseline=self.baseline, demo_paths=self._demo_paths(),
                                           obs_dtype=self.staging_obs_dtype(), reuse=True,
                                           pre=self.__dict__.pop("_pre", None))
        ret, adv = eng.returns_advantages(batch, gamma, gae_lambda)
        ret, adv = ret.cpu().numpy(), adv.cpu().numpy()
        base = batch.baseline.cpu().numpy()
        off = np.concatenate([[0], np.cumsum(batch.lengths)])
        for i, p in enumerate(paths):
            p["returns"] = ret[off[i]:off[i + 1]]
            p["baseline"] = base[off[i]:off[i + 1]]
            p["advantages"] = adv[off[i]:off[i + 1]]
        out = self._update(batch, paths, skip_gae=True, gamma=gamma)
        self._last_batch = batch   # obs + returns stay in HBM for the baseline fit
        return out

    def train_from_paths(self, paths):
        pool = self._pool()
        if pool is not None:
            return self._apply_pool(pool.step(self, paths, "paths"), paths)
        eng = self.engine()
        batch = DeviceBatch.from_paths(paths, eng.device, use_advantages=True, demo_paths=self._demo_paths(),
                                       obs_dtype=self.staging_obs_dtype(), reuse=True,
                                       pre=self.__dict__.pop("_pre", None))
        return self._update(batch, paths)

    # ---- hooks for subclasses ---------------------------------------------------
    def _demo_paths(self):
        return None

    def _rank_share(self, paths):
        """This rank's contiguous share of paths every rank holds (DAPG demos):
        partition_paths by length, so the demo rows enter the all-reduced VPG sum
        once, not world-size times (dapg.py:68-70, 97-98)."""
        comm = self.comm()
        if not paths or comm.world_size <= 1:
            return paths
        p0, p1 = partition_paths([len(p["observations"]) for p in paths], comm.world_size)[comm.rank]
        return paths[p0:p1]

    def _update_args(self):
        return dict(algo="vpg", learn_rate=self.alpha)

    def _log_update(self, res):
        self.logger.log_kv("alpha", self.alpha)
        self.logger.log_kv("time_vpg", res["time_vpg"])
        self.logger.log_kv("kl_dist", res["kl_dist"])
        self.logger.log_kv("surr_improvement", res["surr_after"] - res["surr_before"])
        self.logger.log_kv("running_score", self.running_score)

    def _update(self, batch, paths, skip_gae=False, gamma=0.995):
        eng = self.engine()
        args = self._update_args()
        res = eng.update(batch, self._theta(), skip_gae=skip_gae, gamma=gamma, gae_lambda=None, **args)
        self.last_update = res
        base_stats = [float(v) for v in res["base_stats"]]
        mean_return = base_stats[0]
        self.running_score = mean_return if self.running_score is None else \
            0.9 * self.running_score + 0.1 * mean_return
        self.policy.set_param_values(eng.vec["theta_new"].cpu().numpy(), set_new=True, set_old=True)
        if self.save_logs:
            self.logger.log_kv("stoc_pol_mean", base_stats[0])
            self.logger.log_kv("stoc_pol_std", base_stats[1])
            self.logger.log_kv("stoc_pol_max", base_stats[3])
            self.logger.log_kv("stoc_pol_min", base_stats[2])
            self._log_update(res)
            self._log_success(paths)
        return base_stats

    def _log_success(self, paths):
        try:
            self.env.env.env.evaluate_success(paths, self.logger)
        except Exception:
            try:
                success_rate = self.env.env.env.evaluate_success(paths)
                self.logger.log_kv("success_rate", success_rate)
            except Exception:
                pass

    def log_rollout_statistics(self, paths):
        path_returns = [sum(p["rewards"]) for p in paths]
        self.logger.log_kv("stoc_pol_mean", np.mean(path_returns))
        self.logger.log_kv("stoc_pol_std", np.std(path_returns))
        self.logger.log_kv("stoc_pol_max", np.amax(path_returns))
        self.logger.log_kv("stoc_pol_min", np.amin(path_returns))


def _fit_sharded(baseline, paths, comm, return_errors):
    """baseline.fit on the union of every rank's paths (see _fit_baseline)."""
    if hasattr(baseline, "fit_sharded"):
        return baseline.fit_sharded(paths, comm, return_errors=return_errors)
    if hasattr(baseline, "_features") and hasattr(baseline, "_reg_coeff") and hasattr(baseline, "_coeffs"):
        return _fit_normal_equations(baseline, paths, comm, return_errors)
    import torch.distributed as dist
    keep = ("observations", "rewards", "returns", "terminated")
    mine = [{k: p[k] for k in keep if k in p} for p in paths]
    parts = [None] * comm.world_size
    dist.all_gather_object(parts, mine, group=comm.group)
    union = [p for part in parts for p in part]
    return baseline.fit(union, return_errors=return_errors) if return_errors else baseline.fit(union)


def _fit_normal_equations(baseline, paths, comm, return_errors):
    """Ridge normal-equation baselines (linear_baseline.py:20-44,
    quadratic_baseline.py:40-65): F^T F, F^T y, y^T y and the error sums are sums
    over timesteps, all-reduced in fp64; then the reference's lstsq retry loop."""
    feats = baseline._features(paths) if _features_take_paths(baseline) else \
        np.concatenate([baseline._features(p) for p in paths])
    y = np.concatenate([p["returns"] for p in paths])
    k = feats.shape[1]
    dev = _comm_device(comm)
    pre = feats.dot(baseline._coeffs) if (return_errors and baseline._coeffs is not None) else np.zeros_like(y)
    st = np.concatenate([feats.T.dot(feats).ravel(), feats.T.dot(y), [y.dot(y), ((y - pre) ** 2).sum()]])
    t = torch.from_numpy(st).to(dev)
    comm.allreduce_sum(t)
    st = t.cpu().numpy()
    FtF, Fty, yy, sse0 = st[:k * k].reshape(k, k), st[k * k:k * k + k], st[-2], st[-1]
    reg = baseline._reg_coeff
    for _ in range(10):
        c = np.linalg.lstsq(FtF + reg * np.identity(k), Fty, rcond=None)[0]
        baseline._coeffs = c
        if not np.any(np.isnan(c)):
            break
        reg *= 10
    if return_errors:
        t = torch.tensor([((y - feats.dot(baseline._coeffs)) ** 2).sum()], dtype=torch.float64, device=dev)
        comm.allreduce_sum(t)
        return sse0 / yy, float(t.item()) / yy


def _features_take_paths(baseline):
    """Quadratic / MLP baselines take a list of paths, Linear one path."""
    return type(baseline).__name__ != "LinearBaseline"


def _comm_device(comm):
    """Where collective buffers live: the current GPU under RCCL, CPU under gloo."""
    try:
        backend = comm.dist.get_backend(comm.group)
    except Exception:
        backend = "gloo"
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
