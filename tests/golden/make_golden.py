"""Golden-vector generator for the NPG / TRPO / DAPG update path.

Runs the REFERENCE update code (bennevans/mjrl, mounted read-only at
/root/reference) on synthetic, seeded `paths` and stores inputs plus every
intermediate the parity tests check as small .npz fixtures next to this file.

Build-container only: /root/reference does not exist on the GPU box; the GPU box
only ever reads the committed .npz files.  Nothing from the reference is copied:
the fixtures are data (inputs and the outputs the reference produced).

Import recipe: `mjrl.algos.*` imports the samplers, which
import gym; the update path never calls gym, so a stub module is installed
before import.  torch runs single-threaded so a re-run reproduces the files.

Captured per case (reference call sites in brackets):
  returns / baseline / advantages   process_samples.compute_returns/_advantages
                                    (utils/process_samples.py:3-35)
  adv_whitened                      argument of the first CPI_surrogate call
                                    (algos/npg_cg.py:91,113)
  mean0 / ll0                       MLP.mean_LL at the initial params
                                    (policies/gaussian_mlp.py:100-110)
  surr_calls / kl_calls             every CPI_surrogate / kl_old_new result in order
                                    (algos/batch_reinforce.py:37-49)
  vpg_grad                          flat_vpg result (batch_reinforce.py:51-55)
  hvp_v / hvp_out                   NPG.HVP(obs, act, v) for a fixed random v
                                    (algos/npg_cg.py:55-74)
  cg_b / cg_p / cg_z / cg_x         cg_solve trace: rhs, every f_Ax input / output,
                                    the solution (utils/cg_solve.py:3-22)
  theta0 / theta1                   get_param_values before / after the update
  base_stats, log_*                 return value of train_from_paths and DataLog
"""
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
sys.path.insert(0, REF)
sys.modules.setdefault("gym", types.ModuleType("gym"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(1)

from mjrl.utils.gym_env import EnvSpec  # noqa: E402
from mjrl.policies.gaussian_mlp import MLP  # noqa: E402
from mjrl.policies.gaussian_linear import LinearPolicy  # noqa: E402
from mjrl.baselines.linear_baseline import LinearBaseline  # noqa: E402
from mjrl.algos.batch_reinforce import BatchREINFORCE  # noqa: E402
from mjrl.algos.npg_cg import NPG  # noqa: E402
from mjrl.algos.trpo import TRPO  # noqa: E402
from mjrl.algos.dapg import DAPG  # noqa: E402
import mjrl.algos.npg_cg as npg_mod  # noqa: E402
import mjrl.algos.trpo as trpo_mod  # noqa: E402
import mjrl.algos.dapg as dapg_mod  # noqa: E402
import mjrl.utils.process_samples as process_samples  # noqa: E402
from mjrl.utils.cg_solve import cg_solve as ref_cg_solve  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MEAN_ROWS = 2000   # regenerated cases keep the first MEAN_ROWS rows of mean0 / ll0


def make_paths(rs, n, m, lengths, terminated, col_scale=None, spiky=None, act_scale=None):
    """Synthetic paths in the sampler wire format (samplers/base_sampler.py:76-83).
    obs / act are drawn as f32-representable doubles so the fixture can store them
    as float32 losslessly.  col_scale: per-column observation scales; spiky: a
    column mask whose entries are zeroed where the draw is below 1.5 in magnitude
    (contact-force-like columns: mostly zero, occasionally large); act_scale: a
    factor on the actions (the draw order is unchanged by all three, so
    oracle.npg_cpu.regen_inputs replays them)."""
    paths = []
    for H, term in zip(lengths, terminated):
        obs = rs.randn(H, n)
        if spiky is not None:
            obs[:, spiky] *= np.abs(obs[:, spiky]) > 1.5
        if col_scale is not None:
            obs = obs * col_scale
        obs = obs.astype(np.float32).astype(np.float64)
        act = rs.randn(H, m)
        if act_scale is not None:
            act = act * act_scale
        act = act.astype(np.float32).astype(np.float64)
        rew = rs.randn(H)
        paths.append(dict(observations=obs, actions=act, rewards=rew,
                          agent_infos={}, env_infos={}, terminated=bool(term)))
    return paths


class Recorder:
    """Wraps agent methods / cg_solve to record what the reference computes."""

    def __init__(self, agent, modules, exact_ls=False):
        self.agent = agent
        self.surr = []
        self.kl = []
        self.adv_w = None
        self.vpg = []
        self.cg = None
        self._orig = {}
        a = agent
        orig_surr, orig_kl, orig_vpg = a.CPI_surrogate, a.kl_old_new, a.flat_vpg

        def surr(obs, act, adv):
            if self.adv_w is None:
                self.adv_w = np.array(adv, dtype=np.float64, copy=True)
            out = orig_surr(obs, act, adv)
            self.surr.append(float(out.data.numpy().ravel()[0]))
            return out

        def kl(obs, act):
            out = orig_kl(obs, act)
            self.kl.append(float(out.data.numpy().ravel()[0]))
            return out

        def vpg(obs, act, adv):
            g = orig_vpg(obs, act, adv)
            self.vpg.append(np.array(g, copy=True))
            return g

        a.CPI_surrogate, a.kl_old_new, a.flat_vpg = surr, kl, vpg

        def cg(f_Ax, b, x_0=None, cg_iters=10, residual_tol=1e-10):
            trace = dict(b=np.array(b, copy=True), p=[], z=[])

            def f(p):
                z = f_Ax(p)
                if exact_ls:
                    # the log-std block of the reference's double-backprop HVP is the
                    # closed-form curvature c(sigma) plus f32
                    # rounding of its T-row sums (+-5e-7 per element at T = 60k);
                    # this variant puts the exact c(sigma) there, nothing else changes
                    m_ = len(a.policy.log_std_val)
                    s2 = np.exp(2.0 * np.asarray(a.policy.log_std_val, np.float64))
                    cs = np.float32(4 * s2 * (2 * s2 - 1e-8) / (2 * s2 + 1e-8) ** 2)
                    z = np.array(z, copy=True)
                    z[-m_:] = cs * p[-m_:] + np.float32(a.FIM_invert_args["damping"]) * p[-m_:]
                trace["p"].append(np.array(p, copy=True))
                trace["z"].append(np.array(z, copy=True))
                return z

            x = ref_cg_solve(f, b, x_0=x_0, cg_iters=cg_iters, residual_tol=residual_tol)
            trace["x"] = np.array(x, copy=True)
            self.cg = trace
            return x

        for mod in modules:
            self._orig[mod] = mod.cg_solve
            mod.cg_solve = cg

    def restore(self):
        for mod, fn in self._orig.items():
            mod.cg_solve = fn


def concat(paths, key):
    return np.concatenate([p[key] for p in paths])


ONLY = set(sys.argv[1:])   # optional: regenerate only the named cases
SEED_CLAMP = 60           # a seed whose NPG step takes log_std below -3 (checked in run_case)


def run_case(name, reverse_alt=True, **kw):
    """Runs the reference at 1 torch thread (the fixture), again at 8 and at 3
    threads, and again at 1 thread with the path order reversed and with two
    random path permutations (the same batch, every sum over timesteps
    reordered).  The largest difference to the fixture (the reference's own
    reduction-order sensitivity) is stored as spread_* and
    calibrates the end-to-end tolerances of the GPU parity tests."""
    if ONLY and name not in ONLY:
        return None
    alts = []
    for threads in (8, 3):
        torch.set_num_threads(threads)
        alts.append(_run(None, **kw))
    torch.set_num_threads(1)
    if reverse_alt:   # (a subsampled Fisher draws other rows once reordered: no reordering there)
        alts.append(_run(None, reverse=True, **kw))
        for ps in (1, 2):
            alts.append(_run(None, perm_seed=ps, **kw))
    # the reference's own CG on its own FVP, with the exact log-std curvature in place
    # of the f32-rounded one: the fp32 CG amplifies that rounding, so an
    # implementation with an exact log-std block lands this far from the reference
    alts.append(_run(None, exact_ls=True, **kw))
    out = _run(name, alt=alts, **kw)
    _err64(name, out)
    return out


def _err64(name, out):
    """The reference's own error against an fp64 evaluation of the same update
    (the oracle in float64 — oracle/npg_cpu.py, itself pinned to these fixtures):
    err64_* bound how far ANY fp32 implementation may land from the reference."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from oracle import npg_cpu as O
    c = O.load_case(os.path.join(OUT, name + ".npz"))
    pol = O.Policy(int(c["n"]), int(c["m"]), c["hidden_t"], c["theta0"], c["transforms"], dtype=torch.float64)
    kw = O.case_kwargs(c)
    for k in ("demo_obs", "demo_act"):
        if k in kw:
            kw[k] = kw[k].astype(np.float64)
    r = O.update(pol, c["obs64"], c["act64"], c["advantages"], c["rewards"], c["lengths"], **kw)
    rel = lambda a, b: abs(float(a) / float(b) - 1.0) if float(b) != 0 else abs(float(a))
    z = dict(c)
    for k in ("obs64", "act64", "hidden_t", "transforms") + tuple(str(k) for k in c.get("_regen_keys", ())):
        z.pop(k)
    z.pop("_regen_keys", None)
    z["err64_x"] = _nrel(c["cg_x"], r["npg_grad"])
    z["err64_theta"] = _nrel(c["theta1"], r["theta1"])
    z["err64_alpha"] = rel(c["log_alpha"], r["alpha"])
    z["err64_kl"] = rel(c["log_kl_dist"], r["kl_dist"])
    z["err64_surr"] = rel(c["log_surr_improvement"], r["surr_after"] - r["surr_before"])
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **z)
    print("   err64 x %.1e theta %.1e alpha %.1e kl %.1e surr %.1e" % (
        z["err64_x"], z["err64_theta"], z["err64_alpha"], z["err64_kl"], z["err64_surr"]))


def _colrel(a, b, h0, n):
    """Largest per-column error of the W0 block (h0 x n, the first h0 n entries of a
    flat gradient): max over columns k of max_j |a[j,k] - b[j,k]| / max_j |b[j,k]|."""
    a = np.asarray(a, np.float64)[:h0 * n].reshape(h0, n)
    b = np.asarray(b, np.float64)[:h0 * n].reshape(h0, n)
    den = np.abs(b).max(0)
    ok = den > 0
    return float((np.abs(a - b).max(0)[ok] / den[ok]).max())


def _nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _run(name, *, n, m, hidden, lengths, terminated, algo, algo_kwargs,
         gamma=0.995, gae_lambda=0.97, seed=123, policy_seed=0,
         log_std=None, transforms=None, demo=None, linear=False,
         baseline_fit=True, alt=None, reverse=False, np_seed=None, regen=False, perm_seed=None, exact_ls=False,
         col_scale=None, spiky=None, act_scale=None, w0_col_scale=False):
    rs = np.random.RandomState(seed)
    spec = EnvSpec(n, m, max(lengths), 1)
    if linear:
        policy = LinearPolicy(spec, seed=policy_seed)
    else:
        policy = MLP(spec, hidden_sizes=hidden, seed=policy_seed)
    if transforms is not None:
        for mdl in (policy.model, policy.old_model):
            mdl.set_transformations(*transforms)
    if log_std is not None:
        th = policy.get_param_values()
        th[-m:] = log_std
        policy.set_param_values(th, set_new=True, set_old=True)
    if w0_col_scale:
        # a first layer adapted to the feature scales: W0 column k / col_scale[k], so
        # every column contributes O(1) to the pre-activations (none saturate)
        th = policy.get_param_values()
        h0 = hidden[0]
        th[:h0 * n] = (th[:h0 * n].reshape(h0, n) / col_scale[None, :]).ravel()
        policy.set_param_values(th, set_new=True, set_old=True)
    paths = make_paths(rs, n, m, lengths, terminated, col_scale=col_scale, spiky=spiky, act_scale=act_scale)
    demo_paths = None
    if demo is not None:
        demo_paths = make_paths(rs, n, m, demo, [True] * len(demo))

    if reverse:
        paths = paths[::-1]
        demo_paths = demo_paths[::-1] if demo_paths is not None else None
    if perm_seed is not None:
        order = np.random.RandomState(1000 + perm_seed).permutation(len(paths))
        paths = [paths[i] for i in order]
    baseline = LinearBaseline(spec)
    if baseline_fit:
        process_samples.compute_returns(paths, gamma)
        baseline.fit(paths)

    if algo == "npg":
        agent = NPG(None, policy, baseline, save_logs=True, **algo_kwargs)
    elif algo == "trpo":
        agent = TRPO(None, policy, baseline, save_logs=True, **algo_kwargs)
    elif algo == "dapg":
        agent = DAPG(None, policy, baseline, demo_paths=demo_paths, save_logs=True, **algo_kwargs)
    elif algo == "vpg":
        agent = BatchREINFORCE(None, policy, baseline, save_logs=True, **algo_kwargs)
    else:
        raise ValueError(algo)

    theta0 = policy.get_param_values()
    obs = concat(paths, "observations")
    act = concat(paths, "actions")
    mean0, ll0 = policy.mean_LL(obs, act)
    vrs = np.random.RandomState(seed + 7)
    hvp_v = vrs.randn(policy.d).astype(np.float32)
    if np_seed is not None:   # the subsampled HVP draws from numpy's global RNG (npg_cg.py:58-62)
        np.random.seed(np_seed + 1)
    if algo == "vpg":   # BatchREINFORCE has no HVP: the NPG one at the same parameters
        hvp_out = NPG(None, policy, baseline).HVP(obs, act, hvp_v)
    else:
        hvp_out = agent.HVP(obs, act, hvp_v)

    # the update proper (batch_reinforce.py:86-91 minus sampling and fit)
    process_samples.compute_returns(paths, gamma)
    process_samples.compute_advantages(paths, baseline, gamma, gae_lambda)
    rec = Recorder(agent, [npg_mod, trpo_mod, dapg_mod], exact_ls=exact_ls)
    if np_seed is not None:
        np.random.seed(np_seed)
    try:
        base_stats = agent.train_from_paths(paths)
    finally:
        rec.restore()
    theta1 = policy.get_param_values()
    if rec.cg is None:   # BatchREINFORCE: no CG, the step direction is the VPG itself
        rec.cg = dict(b=rec.vpg[0], p=np.zeros((0, policy.d), np.float32), z=np.zeros((0, policy.d), np.float32),
                      x=rec.vpg[0])

    colspread = lambda k, v: (max(_colrel(a[k], v, hidden[0], n) for a in alt)
                              if alt and not linear else 0.0)
    out = dict(
        spread_x=max(_nrel(a["cg_x"], rec.cg["x"]) for a in alt) if alt else 0.0,
        # the reference's own per-W0-column change (threads, path orders) of the VPG
        # and of HVP(v): the per-column tolerance of the split-row parity test
        spread_vpg_col=colspread("vpg_grad", rec.vpg[0]),
        spread_hvp_col=colspread("hvp_out", hvp_out),
        spread_theta=max(_nrel(a["theta1"], theta1) for a in alt) if alt else 0.0,
        spread_kl=max(abs(a["log_kl_dist"] / agent.logger.log["kl_dist"][-1] - 1) for a in alt) if alt else 0.0,
        spread_alpha=max(abs(float(a["log_alpha"]) / agent.logger.log["alpha"][-1] - 1) for a in alt) if alt else 0.0,
        spread_surr=max(abs(a["log_surr_improvement"] / agent.logger.log["surr_improvement"][-1] - 1)
                        for a in alt) if alt else 0.0,
        n=n, m=m, hidden=np.array(hidden if not linear else (0, 0)), linear=int(linear),
        algo=algo, gamma=gamma, gae_lambda=(np.nan if gae_lambda is None else gae_lambda),
        lengths=np.array(lengths, dtype=np.int64),
        terminated=np.array(terminated, dtype=np.uint8),
        obs=obs.astype(np.float32), act=act.astype(np.float32),
        rewards=concat(paths, "rewards"),
        baseline_coeffs=(baseline._coeffs if baseline._coeffs is not None else np.zeros(0)),
        baseline=concat(paths, "baseline"),
        returns=concat(paths, "returns"),
        advantages=concat(paths, "advantages"),
        adv_whitened=rec.adv_w,
        theta0=theta0, theta1=theta1,
        param_sizes=np.array(policy.param_sizes, dtype=np.int64),
        mean0=mean0.data.numpy(), ll0=ll0.data.numpy(),
        hvp_v=hvp_v, hvp_out=hvp_out,
        surr_calls=np.array(rec.surr), kl_calls=np.array(rec.kl),
        vpg_grad=rec.vpg[0],
        # the whole CG trace: every iteration is teacher-forced by the parity tests
        cg_b=rec.cg["b"], cg_p=np.array(rec.cg["p"]), cg_z=np.array(rec.cg["z"]),
        cg_iters_run=len(rec.cg["p"]),
        cg_x=rec.cg["x"],
        base_stats=np.array(base_stats, dtype=np.float64),
        running_score=agent.running_score,
    )
    if col_scale is not None:
        out["col_scale"] = np.asarray(col_scale, np.float64)
    if spiky is not None:
        out["spiky"] = np.asarray(spiky, np.uint8)
    if act_scale is not None:
        out["act_scale"] = np.float64(act_scale)
    if regen:
        # large cases: the inputs are NOT stored.  oracle.npg_cpu.regen_inputs replays
        # make_paths' RandomState stream from gen_seed and load_case checks the
        # result against inputs_sha256; returns / advantages are recomputed by the
        # pinned oracle and checked bit for bit against the reference's hashes
        import hashlib
        sha = lambda *arrs: hashlib.sha256(b"".join(np.ascontiguousarray(a).tobytes() for a in arrs)).hexdigest()
        out["gen_seed"] = np.int64(seed)
        out["inputs_sha256"] = np.array(sha(out["obs"], out["act"], out["rewards"]))
        for k in ("returns", "advantages"):
            out[k + "_sha256"] = np.array(sha(out[k]))
            out[k + "_head"] = out[k][:256]
            del out[k]
        for k in ("obs", "act", "rewards"):
            del out[k]
        out["mean0"] = out["mean0"][:MEAN_ROWS]
        out["ll0"] = out["ll0"][:MEAN_ROWS]
    if np_seed is not None:
        out["np_seed"] = np.int64(np_seed)
        out["hvp_np_seed"] = np.int64(np_seed + 1)
    for k, v in agent.logger.log.items():
        out["log_" + k] = np.array(v[-1], dtype=np.float64)
    for k, v in algo_kwargs.items():
        out["kw_" + k] = np.array(np.nan if v is None else v, dtype=np.float64) \
            if not isinstance(v, dict) else np.array([v["iters"], v["damping"]], dtype=np.float64)
    if transforms is not None:
        for k, v in zip(("in_shift", "in_scale", "out_shift", "out_scale"), transforms):
            out[k] = np.float32(v)
    if demo_paths is not None:
        out["demo_lengths"] = np.array(demo, dtype=np.int64)
        out["demo_obs"] = concat(demo_paths, "observations").astype(np.float32)
        out["demo_act"] = concat(demo_paths, "actions").astype(np.float32)
        out["demo_iter_count"] = agent.iter_count
    if name is None:
        return out
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print("%-22s T=%-6d d=%-6d kl=%s alpha=%.6g spread x %.1e kl %.1e" % (
        name, obs.shape[0], policy.d, rec.kl[-1:], out.get("log_alpha", np.nan), out["spread_x"],
        out["spread_kl"]))
    return out


def main():
    # C1: point_mass shape, linear Gaussian policy (tests/point_mass_test.py, config 1)
    run_case("c1_pointmass_linear", n=6, m=2, hidden=None, linear=True,
             lengths=[25] * 40, terminated=[False] * 40, algo="npg",
             algo_kwargs=dict(normalized_step_size=0.1), gamma=0.95)
    # C1b: the MLP(32,32) that tests/point_mass_test.py:12 actually builds
    run_case("c1_pointmass_mlp32", n=6, m=2, hidden=(32, 32),
             lengths=[25] * 40, terminated=[False] * 40, algo="npg",
             algo_kwargs=dict(normalized_step_size=0.1), gamma=0.95)
    # C2: Swimmer-v2 shape, full size (25 x 500)
    run_case("c2_swimmer", n=8, m=2, hidden=(64, 64),
             lengths=[500] * 25, terminated=[False] * 25, algo="npg",
             algo_kwargs=dict(normalized_step_size=0.1))
    # C2r: ragged lengths, length-1 path, mixed terminated flags
    rs = np.random.RandomState(5)
    lengths = [1, 2, 3, 64, 65, 127] + list(rs.randint(1, 300, size=24))
    term = list(rs.randint(0, 2, size=len(lengths)).astype(bool))
    run_case("c2_ragged", n=8, m=2, hidden=(64, 64), lengths=lengths, terminated=term,
             algo="npg", algo_kwargs=dict(normalized_step_size=0.05), seed=321,
             log_std=np.array([-0.7, 0.3]))
    # C2n: non-GAE mode (gae_lambda=None is train_agent's default)
    run_case("c2_nogae", n=8, m=2, hidden=(64, 64), lengths=[200] * 10,
             terminated=[False] * 9 + [True], algo="npg",
             algo_kwargs=dict(normalized_step_size=0.1), gae_lambda=None, seed=11)
    # C2c: constant learn-rate NPG (npg_cg.py:130-132)
    run_case("c2_constlr", n=8, m=2, hidden=(64, 64), lengths=[100] * 10,
             terminated=[False] * 10, algo="npg",
             algo_kwargs=dict(const_learn_rate=0.05), seed=12)
    # C2s: NPG with a subsampled Fisher (hvp_sample_frac = 0.5, npg_cg.py:58-62)
    run_case("c2_hvp_sub", n=8, m=2, hidden=(64, 64), lengths=[200] * 20,
             terminated=[False] * 20, algo="npg",
             algo_kwargs=dict(normalized_step_size=0.1, hvp_sample_frac=0.5), seed=31, np_seed=2024,
             reverse_alt=False)
    # C2h: non-square hidden sizes MLP(48, 32) (MuNet takes any pair, gaussian_mlp.py:143-158)
    run_case("c2_h48x32", n=8, m=2, hidden=(48, 32), lengths=[200] * 10,
             terminated=[False] * 10, algo="npg", algo_kwargs=dict(normalized_step_size=0.05), seed=43,
             log_std=np.array([-0.5, 0.2]))
    # C2v: BatchREINFORCE (vanilla policy gradient, batch_reinforce.py:106-164)
    run_case("c2_vpg", n=8, m=2, hidden=(64, 64), lengths=[200] * 10,
             terminated=[False] * 10, algo="vpg", algo_kwargs=dict(learn_rate=0.05), seed=41)
    # C3: HalfCheetah shape, TRPO (reduced to 10 x 1000)
    run_case("c3_halfcheetah_trpo", n=17, m=6, hidden=(128, 128),
             lengths=[1000] * 10, terminated=[False] * 10, algo="trpo",
             algo_kwargs=dict(kl_dist=0.01))
    # C3f: the HalfCheetah TRPO config at its full bench size (100 x 1000 rows,
    # BASELINE configs[2]); inputs regenerated from the seed, outputs only
    run_case("c3_halfcheetah_full", n=17, m=6, hidden=(128, 128),
             lengths=[1000] * 100, terminated=[False] * 100, algo="trpo",
             algo_kwargs=dict(kl_dist=0.01), regen=True, seed=131)
    # C3b: TRPO with a step large enough that the line search backtracks
    run_case("c3_trpo_backtrack", n=17, m=6, hidden=(128, 128),
             lengths=[300] * 4, terminated=[False] * 4, algo="trpo",
             algo_kwargs=dict(kl_dist=2.0), seed=77,
             log_std=np.linspace(-1.0, 0.5, 6))
    # C4: Humanoid shape (obs 376, act 17), 60 x 1000 rows: T = 60,000 >= 2 d
    # (d = 29,410), so the Fisher is well conditioned and the reference's own
    # end-to-end spread is small (the 4 x 250 case of round 1 had T < d)
    run_case("c4_humanoid", n=376, m=17, hidden=(64, 64),
             lengths=[1000] * 60, terminated=[False] * 60, algo="npg",
             algo_kwargs=dict(normalized_step_size=0.01), regen=True)
    # C4s: the Humanoid shape with observation columns of very different scales
    # (10^U(-4, 3), every 7th column contact-force-like: mostly zero), a first layer
    # adapted to them (W0 column k / scale k) and 60 x 1000 rows: each row spans
    # ~12 decades, the case a per-row block-floating-point row format gets wrong
    # for its small columns (pins the split rows' column scales)
    crs = np.random.RandomState(404)
    col_scale = 10.0 ** crs.uniform(-4, 3, size=376)
    spiky = np.zeros(376, bool)
    spiky[::7] = True
    run_case("c4_humanoid_scaled", n=376, m=17, hidden=(64, 64),
             lengths=[1000] * 60, terminated=[False] * 60, algo="npg",
             algo_kwargs=dict(normalized_step_size=0.01), regen=True, seed=404,
             col_scale=col_scale, spiky=spiky, w0_col_scale=True)
    # C2l: log_std starting AT min_log_std (-3) with a step that drives part of it
    # below: set_param_values clamps it (gaussian_mlp.py:74-78,86-88), and the
    # post-step surrogate / KL are evaluated at the clamped parameters
    out = run_case("c2_logstd_clamp", n=8, m=2, hidden=(64, 64), lengths=[200] * 10,
                   terminated=[False] * 10, algo="npg", algo_kwargs=dict(normalized_step_size=0.5),
                   seed=SEED_CLAMP, log_std=np.array([-3.0, -3.0]), act_scale=0.05)
    if out is not None:
        step = out["theta0"][-2:] + out["log_alpha"] * out["cg_x"][-2:]
        assert step.min() < -3.0 - 1e-3 and out["theta1"][-2:].min() == -3.0, (step, out["theta1"][-2:])
    # C5: door shape, DAPG with BC-style in/out transformations and demos
    rs = np.random.RandomState(9)
    n, m = 39, 28
    transforms = (rs.randn(n) * 0.5, rs.rand(n) + 0.5, rs.randn(m) * 0.1, rs.rand(m) + 0.5)
    run_case("c5_door_dapg", n=n, m=m, hidden=(256, 256),
             lengths=[200] * 10, terminated=[False] * 10, algo="dapg",
             algo_kwargs=dict(), demo=[200] * 5, transforms=transforms,
             log_std=np.linspace(-1.0, 0.0, m))
    # C5f: the door DAPG config at its full bench size (200 x 200 rows + 25 demos)
    run_case("c5_door_full", n=n, m=m, hidden=(256, 256),
             lengths=[200] * 200, terminated=[False] * 200, algo="dapg",
             algo_kwargs=dict(), demo=[200] * 25, transforms=transforms,
             log_std=np.linspace(-1.0, 0.0, m), regen=True, seed=151)


def baselines_case():
    """Reference LinearBaseline / QuadraticBaseline fit + predict on ragged paths."""
    from mjrl.baselines.quadratic_baseline import QuadraticBaseline
    rs = np.random.RandomState(31)
    n = 5
    lengths = [7, 1, 30, 12]
    paths = make_paths(rs, n, 2, lengths, [False] * 4)
    for p in paths:
        p["observations"] = p["observations"] * 6.0   # exercise the +-10 clip
    process_samples.compute_returns(paths, 0.99)
    spec = EnvSpec(n, 2, 30, 1)
    lin, quad = LinearBaseline(spec), QuadraticBaseline(spec)
    lerr = lin.fit(paths, return_errors=True)
    qerr = quad.fit(paths, return_errors=True)
    np.savez_compressed(os.path.join(OUT, "baselines.npz"),
                        obs=concat(paths, "observations"), rewards=concat(paths, "rewards"),
                        returns=concat(paths, "returns"), lengths=np.array(lengths),
                        lin_coeffs=lin._coeffs, lin_pred=np.concatenate([lin.predict(p) for p in paths]),
                        lin_err=np.array(lerr), quad_coeffs=quad._coeffs,
                        quad_pred=np.concatenate([quad.predict(p) for p in paths]), quad_err=np.array(qerr))


def mlp_baseline_case():
    """Reference MLPBaseline (mlp_baseline.py:15-115, CPU) fit + predict: initial
    weights under torch.manual_seed(7), two fits (the Adam state carries over)
    with np.random.seed(11) / (12) before each, errors and predictions."""
    saved = {k: os.environ.get(k) for k in ("CUDA_VISIBLE_DEVICES", "CUDA_DEVICE_ORDER", "MKL_THREADING_LAYER")}
    from mjrl.baselines.mlp_baseline import MLPBaseline as RefMLP   # sets CUDA_VISIBLE_DEVICES at import
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    rs = np.random.RandomState(53)
    n = 5
    lengths = [300, 200, 250]
    paths = make_paths(rs, n, 2, lengths, [False] * 3)
    for p in paths:
        p["observations"] = p["observations"] * 4.0   # exercise the +-10 clip
    process_samples.compute_returns(paths, 0.99)
    spec = EnvSpec(n, 2, 300, 1)
    torch.manual_seed(7)
    ref = RefMLP(spec, batch_size=64, epochs=2, learn_rate=3e-3)
    init = {k: v.detach().numpy().copy() for k, v in ref.model.state_dict().items()}
    out = dict(obs=concat(paths, "observations"), rewards=concat(paths, "rewards"),
               returns=concat(paths, "returns"), lengths=np.array(lengths))
    for k, v in init.items():
        out["init_" + k.replace(".", "_")] = v
    for it, seed in enumerate((11, 12)):
        np.random.seed(seed)
        err = ref.fit(paths, return_errors=True)
        out["err%d" % it] = np.array(err, dtype=np.float64)
        out["pred%d" % it] = np.concatenate([ref.predict(p) for p in paths])
        out["np_seed%d" % it] = np.int64(seed)
    for k, v in ref.model.state_dict().items():
        out["final_" + k.replace(".", "_")] = v.detach().numpy().copy()
    np.savez_compressed(os.path.join(OUT, "mlp_baseline.npz"), **out)
    print("mlp_baseline errors", out["err0"], out["err1"])


def f64obs_case(name, n, lengths, terminated, seed, col_scale=None, spiky=None, gamma=0.995, gae_lambda=0.97):
    """The baseline / GAE chain on observations that are NOT float32s (MuJoCo's are
    f64): obs = randn(H, n) (spiky columns zeroed where |draw| <= 1.5, times the
    column scales) kept in f64, then rewards randn(H), per path from
    RandomState(seed) (oracle.npg_cpu.regen_f64obs replays it; the inputs are not
    stored, their SHA-256 is).  Reference calls: LinearBaseline.fit on the first
    half of the paths (coeffs0: the previous iteration's baseline,
    linear_baseline.py:20-44), compute_returns + compute_advantages with it on all
    paths (process_samples.py:3-35, predict :23), then fit(return_errors=True) on
    all paths (coeffs1, err); MLPBaseline._features(paths).astype('float32')
    (mlp_baseline.py:37-56, 64), stored as a checksum and its first rows."""
    import hashlib
    saved = {k: os.environ.get(k) for k in ("CUDA_VISIBLE_DEVICES", "CUDA_DEVICE_ORDER", "MKL_THREADING_LAYER")}
    from mjrl.baselines.mlp_baseline import MLPBaseline as RefMLP   # sets CUDA_VISIBLE_DEVICES at import
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    rs = np.random.RandomState(seed)
    paths = []
    for H, term in zip(lengths, terminated):
        obs = rs.randn(H, n)
        if spiky is not None:
            obs[:, spiky] *= np.abs(obs[:, spiky]) > 1.5
        if col_scale is not None:
            obs = obs * col_scale
        paths.append(dict(observations=obs, rewards=rs.randn(H), terminated=bool(term)))
    obs = concat(paths, "observations")
    assert np.mean(obs.astype(np.float32).astype(np.float64) != obs) > 0.5   # genuinely f64
    spec = EnvSpec(n, 1, max(lengths), 1)
    process_samples.compute_returns(paths, gamma)
    lin = LinearBaseline(spec)
    lin.fit(paths[: len(paths) // 2])
    coeffs0 = lin._coeffs.copy()
    process_samples.compute_advantages(paths, lin, gamma, gae_lambda)
    err = lin.fit(paths, return_errors=True)
    # the reference's own sensitivity of that fit to the order its paths arrive in
    # (two path permutations: the normal equations summed in another order); at
    # Humanoid column scales the k x k system is ill-conditioned enough that this,
    # not the 1e-10 of a well-conditioned fit, is the attainable bar
    spread = 0.0
    for ps in (1, 2):
        order = np.random.RandomState(ps).permutation(len(paths))
        alt = LinearBaseline(spec)
        alt.fit([paths[i] for i in order])
        spread = max(spread, float(np.linalg.norm(alt._coeffs - lin._coeffs)))
    feat = RefMLP(spec)._features(paths).astype("float32")
    sha = lambda *arrs: hashlib.sha256(b"".join(np.ascontiguousarray(a).tobytes() for a in arrs)).hexdigest()
    out = dict(n=np.int64(n), lengths=np.array(lengths, np.int64), terminated=np.array(terminated, np.uint8),
               gen_seed=np.int64(seed), gamma=np.float64(gamma), gae_lambda=np.float64(gae_lambda),
               inputs_sha256=np.array(sha(obs, concat(paths, "rewards"))), coeffs0=coeffs0,
               baseline=concat(paths, "baseline"), returns=concat(paths, "returns"),
               advantages=concat(paths, "advantages"), coeffs1=lin._coeffs.copy(), err=np.array(err, np.float64),
               coeffs1_spread=np.float64(spread),
               mlp_feat_sha256=np.array(sha(feat)), mlp_feat_head=feat[:64])
    if col_scale is not None:
        out["col_scale"] = col_scale
    if spiky is not None:
        out["spiky"] = np.asarray(spiky, np.uint8)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print("%-22s T=%-6d n=%-4d inexact %.3f err %s fit spread %.3g" % (
        name, obs.shape[0], n, np.mean(obs.astype(np.float32).astype(np.float64) != obs), err,
        spread / np.linalg.norm(lin._coeffs)))


def f64obs_cases():
    # Swimmer width, ragged lengths with terminated paths, values past the +-10 clip
    rs = np.random.RandomState(606)
    lengths = [500] * 20 + list(rs.randint(1, 500, size=5))
    term = [False] * 20 + [True, False, True, True, False]
    f64obs_case("f64obs_swimmer", 8, lengths, term, seed=607, col_scale=np.array([1, 3, 12, 0.5, 8, 2, 30, 0.1]))
    # Humanoid width with Humanoid-like columns: scales 10^U(-4, 3), every 7th
    # column contact-force-like (mostly zero), so many values sit past the clip
    crs = np.random.RandomState(608)
    col_scale = 10.0 ** crs.uniform(-4, 3, size=376)
    spiky = np.zeros(376, bool)
    spiky[::7] = True
    f64obs_case("f64obs_humanoid", 376, [1000] * 8 + [517, 1, 1000, 250], [False] * 8 + [True, True, False, True],
                seed=609, col_scale=col_scale, spiky=spiky)


def quad_case(name, n, lengths, terminated, seed, col_scale=None, gamma=0.995):
    """QuadraticBaseline.fit (quadratic_baseline.py:10-65) on observations that
    are NOT float32s, inputs replayed from RandomState(seed) as in f64obs_case
    (oracle.npg_cpu.regen_f64obs; stored as their SHA-256): returns
    (process_samples.compute_returns), then fit(return_errors=True) on the first
    half of the paths (coeffs0, err0: no previous coefficients) and again on all
    paths (coeffs1, err1: error_before with coeffs0), the all-path fit's spread
    over two path permutations, and its predict() on the last path."""
    import hashlib
    from mjrl.baselines.quadratic_baseline import QuadraticBaseline as RefQuad
    rs = np.random.RandomState(seed)
    paths = []
    for H, term in zip(lengths, terminated):
        obs = rs.randn(H, n)
        if col_scale is not None:
            obs = obs * col_scale
        paths.append(dict(observations=obs, rewards=rs.randn(H), terminated=bool(term)))
    obs = concat(paths, "observations")
    spec = EnvSpec(n, 1, max(lengths), 1)
    process_samples.compute_returns(paths, gamma)
    q = RefQuad(spec)
    err0 = q.fit(paths[: len(paths) // 2], return_errors=True)
    coeffs0 = q._coeffs.copy()
    err1 = q.fit(paths, return_errors=True)
    spread = 0.0
    for ps in (1, 2):
        order = np.random.RandomState(ps).permutation(len(paths))
        alt = RefQuad(spec)
        alt.fit([paths[i] for i in order])
        spread = max(spread, float(np.linalg.norm(alt._coeffs - q._coeffs)))
    sha = lambda *arrs: hashlib.sha256(b"".join(np.ascontiguousarray(a).tobytes() for a in arrs)).hexdigest()
    out = dict(n=np.int64(n), lengths=np.array(lengths, np.int64), terminated=np.array(terminated, np.uint8),
               gen_seed=np.int64(seed), gamma=np.float64(gamma),
               inputs_sha256=np.array(sha(obs, concat(paths, "rewards"))), returns=concat(paths, "returns"),
               coeffs0=coeffs0, err0=np.array(err0, np.float64), coeffs1=q._coeffs.copy(),
               err1=np.array(err1, np.float64), coeffs1_spread=np.float64(spread),
               predict_last=q.predict(paths[-1]))
    if col_scale is not None:
        out["col_scale"] = col_scale
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print("%-22s T=%-6d n=%-3d k=%-4d inexact %.3f err0 %s err1 %s fit spread %.3g" % (
        name, obs.shape[0], n, len(q._coeffs), np.mean(obs.astype(np.float32).astype(np.float64) != obs), err0, err1,
        spread / np.linalg.norm(q._coeffs)))


def quad_cases():
    # point_mass width (reference tests/point_mass_test.py: 40 trajectories x 25 steps)
    quad_case("quad_point_mass", 4, [25] * 40, [False] * 40, seed=701)
    # Swimmer width, ragged, terminated paths, values past the +-10 clip
    rs = np.random.RandomState(702)
    lengths = [500] * 12 + list(rs.randint(1, 500, size=5))
    quad_case("quad_swimmer", 8, lengths, [False] * 12 + [True, False, True, True, False], seed=703,
              col_scale=np.array([1, 3, 12, 0.5, 8, 2, 30, 0.1]))
    # HalfCheetah width (k = 175 features: three 64-column Gram tiles)
    quad_case("quad_halfcheetah", 17, [1000] * 6 + [333, 1], [False] * 6 + [True, True], seed=704,
              col_scale=10.0 ** np.random.RandomState(705).uniform(-1, 1.3, size=17))


def bc_case():
    """Reference BC (behavior_cloning.py:11-68): MLE of expert actions by minibatch
    Adam, minibatches from np.random.choice after np.random.seed(17); the
    transformations it sets, the per-epoch full-data losses, the final params."""
    from mjrl.algos.behavior_cloning import BC as RefBC
    rs = np.random.RandomState(61)
    n, m = 6, 3
    lengths = [100, 80, 120]
    paths = make_paths(rs, n, m, lengths, [False] * 3)
    for p in paths:
        p["observations"] = p["observations"] * 3.0 + 1.0
        p["actions"] = np.tanh(p["observations"][:, :m]) + 0.1 * p["actions"]
    spec = EnvSpec(n, m, 120, 1)
    policy = MLP(spec, hidden_sizes=(32, 32), seed=5)
    init = policy.get_param_values()
    bc = RefBC(paths, policy, epochs=2, batch_size=32, lr=1e-3)
    np.random.seed(17)
    bc.train()
    t = policy.model.transformations
    np.savez_compressed(os.path.join(OUT, "bc.npz"), obs=concat(paths, "observations"),
                        act=concat(paths, "actions"), lengths=np.array(lengths), init=init,
                        final=policy.get_param_values(), loss=np.array(bc.logger.log["loss"], dtype=np.float64),
                        in_shift=t["in_shift"], in_scale=t["in_scale"], out_shift=t["out_shift"],
                        out_scale=t["out_scale"], np_seed=np.int64(17))
    print("bc losses", bc.logger.log["loss"])


def ppo_case():
    """Reference PPO (ppo_clip.py:23-120) train_from_paths, two iterations (the
    Adam state carries over) after np.random.seed(23) / (24): base_stats, the
    logged kl / surrogate improvement and the params after each."""
    from mjrl.algos.ppo_clip import PPO as RefPPO
    rs = np.random.RandomState(71)
    n, m = 6, 2
    lengths = [150, 90, 200, 160]
    spec = EnvSpec(n, m, 200, 1)
    policy = MLP(spec, hidden_sizes=(32, 32), seed=3, init_log_std=-0.5)
    ppo = RefPPO(None, policy, None, clip_coef=0.2, epochs=2, mb_size=64, learn_rate=3e-3, save_logs=True)
    out = dict(init=policy.get_param_values(), lengths=np.array(lengths))
    for it, seed in enumerate((23, 24)):
        paths = make_paths(rs, n, m, lengths, [False] * 4)
        for p in paths:
            p["advantages"] = rs.randn(len(p["rewards"])) * 2.0 + 0.3
        np.random.seed(seed)
        stats = ppo.train_from_paths(paths)
        out["obs%d" % it] = concat(paths, "observations")
        out["act%d" % it] = concat(paths, "actions")
        out["rew%d" % it] = concat(paths, "rewards")
        out["adv%d" % it] = concat(paths, "advantages")
        out["np_seed%d" % it] = np.int64(seed)
        out["base_stats%d" % it] = np.array(stats, dtype=np.float64)
        out["params%d" % it] = policy.get_param_values()
        for k in ("kl_dist", "surr_improvement", "running_score"):
            out["%s%d" % (k, it)] = np.float64(ppo.logger.log[k][-1])
    np.savez_compressed(os.path.join(OUT, "ppo.npz"), **out)
    print("ppo kl", out["kl_dist0"], out["kl_dist1"], "surr", out["surr_improvement0"], out["surr_improvement1"])


if __name__ == "__main__":
    if not ONLY or "f64obs" in ONLY:
        f64obs_cases()
    if not ONLY or "quad" in ONLY:
        quad_cases()
    if ONLY and ONLY <= {"f64obs", "quad"}:
        sys.exit(0)
    main()
    if not ONLY or "baselines" in ONLY:
        baselines_case()
    if not ONLY or "mlp_baseline" in ONLY:
        mlp_baseline_case()
    if not ONLY or "bc" in ONLY:
        bc_case()
    if not ONLY or "ppo" in ONLY:
        ppo_case()
