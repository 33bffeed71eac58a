"""ORACLE — CPU restatement of the mjrl NPG / TRPO / DAPG update path.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the checker
or as the timed CPU baseline.  The product path (`mjrl_amd`) never imports it and
fails loudly when its HIP library is missing.

What it restates (reference = bennevans/mjrl, file:line under /root/reference):
  discount_sum            mjrl/utils/process_samples.py:37-44
  returns / advantages    mjrl/utils/process_samples.py:3-35 (GAE branch :21-29,
                          plain branch :10-13)
  whitening, path stats   mjrl/algos/npg_cg.py:86-105 (same in trpo.py:57-75,
                          dapg.py:57-85)
  policy forward          mjrl/policies/gaussian_mlp.py:176-182 (MuNet.forward),
                          gaussian_linear.py:171-175 (LinearModel.forward)
  log-likelihood          gaussian_mlp.py:100-110
  likelihood ratio / KL   gaussian_mlp.py:124-140
  CPI surrogate / KL      mjrl/algos/batch_reinforce.py:37-49
  flat VPG                batch_reinforce.py:51-55
  Fisher-vector product   mjrl/algos/npg_cg.py:55-74 (double backprop)
  conjugate gradient      mjrl/utils/cg_solve.py:3-22
  NPG step                npg_cg.py:128-144
  TRPO line search        mjrl/algos/trpo.py:98-124
  DAPG augmented grad     mjrl/algos/dapg.py:62-121
  set_param_values clamp  gaussian_mlp.py:66-88

The restatement keeps the reference's numerics and costs on purpose (it is also
the CPU baseline of bench.py): fp64 numpy for GAE / whitening, fp32 torch
autograd with a fresh f64->f32 conversion on every policy evaluation, a
double-backprop Fisher-vector product, fp32 numpy CG.

Parity pinning: tests/test_oracle_golden.py checks every stage of this module
against fixtures produced by running the reference itself
(tests/golden/make_golden.py).
"""
import numpy as np
import torch

LOG2PI = np.log(2 * np.pi)


# --------------------------------------------------------------------------
# a1-a3: reverse discounted sums, returns, advantages (fp64)
# --------------------------------------------------------------------------
def discount_sum(x, gamma, terminal=0.0):
    """y_t = x_t + gamma * y_{t+1}, y_H = terminal (process_samples.py:37-44).
    Multiply-then-add per step, evaluated back to front."""
    y = np.empty(len(x), dtype=np.float64)
    acc = terminal
    for t in range(len(x) - 1, -1, -1):
        acc = x[t] + gamma * acc
        y[t] = acc
    return y


def split(arr, lengths):
    offs = np.concatenate([[0], np.cumsum(lengths)])
    return [arr[offs[i]:offs[i + 1]] for i in range(len(lengths))]


def returns_and_advantages(rewards, baseline, lengths, terminated, gamma, gae_lambda):
    """Per-path returns and advantages, concatenated (process_samples.py:3-35)."""
    rets, advs = [], []
    use_gae = not (gae_lambda is None or gae_lambda < 0.0 or gae_lambda > 1.0)
    for r, b, term in zip(split(rewards, lengths), split(baseline, lengths), terminated):
        ret = discount_sum(r, gamma)
        rets.append(ret)
        if not use_gae:
            advs.append(ret - b)
            continue
        b1 = np.append(b, 0.0 if term else b[-1])
        td = r + gamma * b1[1:] - b1[:-1]
        advs.append(discount_sum(td, gamma * gae_lambda))
    return np.concatenate(rets), np.concatenate(advs)


def whiten(adv):
    """npg_cg.py:91 — population std, 1e-6 guard."""
    return (adv - np.mean(adv)) / (np.std(adv) + 1e-6)


def path_return_stats(rewards, lengths):
    """npg_cg.py:97-102 — builtin sum per path (sequential), numpy stats."""
    pr = [sum(r) for r in split(rewards, lengths)]
    return [np.mean(pr), np.std(pr), np.amin(pr), np.amax(pr)]


def moments_record(x):
    """One shard's 16-double moment record of the sharded update (the layout
    mjrl_moments_combine folds): pass 1 [sum, sum^2, n, min, max, -min] at 0..5,
    pass 2 about the shard's own mean [sum(x - m_r), sum((x - m_r)^2), n, ...] at
    8..13.  The mean / std of npg_cg.py:91, 97-102 over the union of the shards
    follow from the records alone (moments_combine)."""
    x = np.asarray(x, dtype=np.float64)
    r = np.zeros(16)
    n = float(len(x))
    mn, mx = (x.min(), x.max()) if len(x) else (np.inf, -np.inf)
    r[0:6] = [x.sum(), (x * x).sum(), n, mn, mx, -mn]
    c = x.sum() / n if len(x) else 0.0
    r[8:14] = [(x - c).sum(), ((x - c) ** 2).sum(), n, mn, mx, -mn]
    return r


def moments_combine(records):
    """The fold of every shard's record (rank order): global [S, SS, N, min, max,
    -min] and [sum(x - mean), M2 about the global mean, N, ...], with M2 =
    sum_r [M2_r + 2 (m_r - mean) D_r + n_r (m_r - mean)^2] — exact algebra, so
    mean = out[0] / out[2] and std = sqrt(out[9] / out[2]) are np.mean / np.std of
    the concatenation up to rounding."""
    R = np.asarray(records, dtype=np.float64).reshape(len(records), 16)
    S, SS, N = R[:, 0].sum(), R[:, 1].sum(), R[:, 2].sum()
    mn, mx = R[:, 3].min(), R[:, 4].max()
    mean = S / N
    D = M2 = 0.0
    for r in R:
        if r[2] > 0:
            dm = r[0] / r[2] - mean
            M2 += r[9] + 2.0 * dm * r[8] + r[2] * dm * dm
            D += r[8] + r[2] * dm
    out = np.zeros(16)
    out[0:6] = [S, SS, N, mn, mx, -mn]
    out[8:14] = [D, M2, N, mn, mx, -mn]
    return out


def linear_baseline_features(obs_path):
    """LinearBaseline._features (baselines/linear_baseline.py:10-18)."""
    o = np.clip(obs_path, -10, 10)
    H = o.shape[0]
    al = np.arange(H).reshape(-1, 1) / 1000.0
    return np.concatenate([o, al, al ** 2, al ** 3, np.ones((H, 1))], axis=1)


def linear_baseline_predict(coeffs, obs, lengths):
    """LinearBaseline.predict per path, concatenated (linear_baseline.py:46-49)."""
    if coeffs is None or len(coeffs) == 0:
        return np.zeros(obs.shape[0])
    return np.concatenate([linear_baseline_features(o).dot(coeffs) for o in split(obs, lengths)])


def linear_baseline_fit(obs, returns, lengths, reg_coeff=1e-5):
    """LinearBaseline.fit normal equations (linear_baseline.py:20-44)."""
    F = np.concatenate([linear_baseline_features(o) for o in split(obs, lengths)])
    reg = reg_coeff
    for _ in range(10):
        c = np.linalg.lstsq(F.T.dot(F) + reg * np.identity(F.shape[1]), F.T.dot(returns), rcond=None)[0]
        if not np.any(np.isnan(c)):
            break
        reg *= 10
    return c


# --------------------------------------------------------------------------
# a6-a15: Gaussian MLP / linear policy in torch fp32
# --------------------------------------------------------------------------
def param_shapes(n, m, hidden):
    """trainable_params order: [W0, b0, W1, b1, W2, b2, log_std] (gaussian_mlp.py:33-38;
    nn.Linear weight is [out, in]).  hidden=None/(0,0) -> linear policy [W, b, log_std]."""
    if hidden is None or tuple(hidden) == (0, 0):
        return [(m, n), (m,), (m,)]
    h0, h1 = hidden
    return [(h0, n), (h0,), (h1, h0), (h1,), (m, h1), (m,), (m,)]


class Policy:
    """fp32 torch policy on the flat parameter vector (new + old copies).

    dtype=torch.float64 gives the same computation in double precision: the
    "truth" the parity tests measure the reference's own fp32 error against."""

    def __init__(self, n, m, hidden, theta, transforms=None, min_log_std=-3.0, dtype=torch.float32):
        self.n, self.m = n, m
        self.dtype = dtype
        self.shapes = param_shapes(n, m, hidden)
        self.sizes = [int(np.prod(s)) for s in self.shapes]
        self.d = sum(self.sizes)
        self.min_log_std = min_log_std
        tr = transforms or (None, None, None, None)
        self.in_shift = torch.from_numpy(np.float32(tr[0])) if tr[0] is not None else torch.zeros(n)
        self.in_scale = torch.from_numpy(np.float32(tr[1])) if tr[1] is not None else torch.ones(n)
        self.out_shift = torch.from_numpy(np.float32(tr[2])) if tr[2] is not None else torch.zeros(m)
        self.out_scale = torch.from_numpy(np.float32(tr[3])) if tr[3] is not None else torch.ones(m)
        self.in_shift, self.in_scale, self.out_shift, self.out_scale = (
            t.to(dtype) for t in (self.in_shift, self.in_scale, self.out_shift, self.out_scale))
        self.new = self._tensors(theta, grad=True)
        self.old = self._tensors(theta, grad=False)

    def _tensors(self, theta, grad):
        out, i = [], 0
        for shp, sz in zip(self.shapes, self.sizes):
            t = torch.from_numpy(np.asarray(theta[i:i + sz]).reshape(shp)).to(self.dtype)
            out.append(t)
            i += sz
        out[-1] = torch.clamp(out[-1], self.min_log_std)   # gaussian_mlp.py:74-78
        if grad:
            for t in out:
                t.requires_grad_(True)
        return out

    def set_params(self, theta, set_new=True, set_old=True):
        if set_new:
            self.new = self._tensors(theta, grad=True)
        if set_old:
            self.old = self._tensors(theta, grad=False)

    def get_params(self):
        return np.concatenate([t.detach().reshape(-1).numpy() for t in self.new]).copy()

    def mean(self, params, obs_f64):
        x = torch.from_numpy(obs_f64).to(self.dtype)   # per-call f64->f32 (gaussian_mlp.py:103)
        h = (x - self.in_shift) / (self.in_scale + 1e-8)
        if len(params) == 3:
            pre = torch.addmm(params[1], h, params[0].t())
        else:
            W0, b0, W1, b1, W2, b2 = params[:6]
            h = torch.tanh(torch.addmm(b0, h, W0.t()))
            h = torch.tanh(torch.addmm(b1, h, W1.t()))
            pre = torch.addmm(b2, h, W2.t())
        return pre * self.out_scale + self.out_shift

    def mean_ll(self, params, obs, act):
        mu = self.mean(params, obs)
        a = torch.from_numpy(act).to(self.dtype)
        s = params[-1]
        zs = (a - mu) / torch.exp(s)
        ll = -0.5 * torch.sum(zs ** 2, dim=1) - torch.sum(s) - 0.5 * self.m * LOG2PI
        return mu, ll

    def surrogate(self, obs, act, adv_f64):
        """CPI surrogate mean(exp(LL_new - LL_old) * adv) (batch_reinforce.py:37-43)."""
        adv = torch.from_numpy(adv_f64).to(self.dtype)
        _, ll_old = self.mean_ll(self.old, obs, act)
        _, ll_new = self.mean_ll(self.new, obs, act)
        return torch.mean(torch.exp(ll_new - ll_old) * adv)

    def kl(self, obs, act):
        """mean KL(old || new) in the reference's form (gaussian_mlp.py:130-140)."""
        mu_o, _ = self.mean_ll(self.old, obs, act)
        mu_n, _ = self.mean_ll(self.new, obs, act)
        so, sn = self.old[-1], self.new[-1]
        num = (mu_o - mu_n) ** 2 + torch.exp(so) ** 2 - torch.exp(sn) ** 2
        den = 2 * torch.exp(sn) ** 2 + 1e-8
        return torch.mean(torch.sum(num / den + sn - so, dim=1))

    def flat_vpg(self, obs, act, adv):
        g = torch.autograd.grad(self.surrogate(obs, act, adv), self.new)
        return np.concatenate([t.reshape(-1).numpy() for t in g])

    def fvp(self, obs, act, v, damping):
        """Hessian of mean KL times v by double backprop (npg_cg.py:55-74)."""
        vt = torch.from_numpy(np.asarray(v)).to(self.dtype)
        g1 = torch.autograd.grad(self.kl(obs, act), self.new, create_graph=True)
        h = torch.sum(torch.cat([t.reshape(-1) for t in g1]) * vt)
        g2 = torch.autograd.grad(h, self.new)
        return np.concatenate([t.reshape(-1).numpy() for t in g2]) + damping * v


# --------------------------------------------------------------------------
# a13: conjugate gradient (fp32 numpy; x0 ignored as in the reference)
# --------------------------------------------------------------------------
def cg_solve(f_Ax, b, iters=10, tol=1e-10, trace=None):
    x = np.zeros_like(b)
    r = b.copy()
    p = r.copy()
    rr = r.dot(r)
    for _ in range(iters):
        z = f_Ax(p)
        if trace is not None:
            trace.append((p.copy(), np.array(z, copy=True)))
        step = rr / p.dot(z)
        x += step * p
        r -= step * z
        rr_new = r.dot(r)
        p = r + (rr_new / rr) * p
        rr = rr_new
        if rr < tol:
            break
    return x


# --------------------------------------------------------------------------
# a5-a18: one update (train_from_paths after returns/advantages)
# --------------------------------------------------------------------------
def update(policy, obs, act, adv_raw, rewards, lengths, algo="npg", *,
           n_step_size=0.01, const_lr=None, kl_dist=None, cg_iters=10, damping=1e-4,
           demo_obs=None, demo_act=None, demo_coef=None, trace=None, hvp_sample_frac=None, np_seed=None,
           learn_rate=0.01):
    """Runs the policy update on concatenated arrays and returns a result dict.

    algo: 'npg'  (npg_cg.py:84-165), 'trpo' (trpo.py:54-145), 'dapg' (dapg.py:54-141),
    'vpg' (BatchREINFORCE.train_from_paths, batch_reinforce.py:106-164: theta +
    learn_rate * vpg_grad in f32, then surr_after / kl).
    For 'npg' with kl_dist set, n_step_size = 2*kl_dist (npg_cg.py:47).
    For 'dapg', demo_coef = lam_0 * lam_1**iter_count (dapg.py:65).
    hvp_sample_frac < 0.99: every Fisher-vector product runs on
    np.random.choice(N, int(frac N)) rows (with replacement) drawn from numpy's
    global RNG (npg_cg.py:58-62); np_seed, if given, seeds it first.
    """
    if np_seed is not None:
        np.random.seed(np_seed)
    res = {}
    adv = whiten(adv_raw)
    res["adv_whitened"] = adv
    res["base_stats"] = path_return_stats(rewards, lengths)
    res["surr_before"] = float(policy.surrogate(obs, act, adv).detach().numpy())

    if algo == "dapg" and demo_obs is not None:
        all_obs = np.concatenate([obs, demo_obs])
        all_act = np.concatenate([act, demo_act])
        demo_adv = demo_coef * np.ones(demo_obs.shape[0])
        all_adv = 1e-2 * np.concatenate([adv / (np.std(adv) + 1e-8), demo_adv])
        g = (all_adv.shape[0] / adv.shape[0]) * policy.flat_vpg(all_obs, all_act, all_adv)
    else:
        g = policy.flat_vpg(obs, act, adv)
    res["vpg_grad"] = g
    if algo == "vpg":
        theta = policy.get_params()
        new = theta + learn_rate * g   # f32 numpy (batch_reinforce.py:139-140)
        policy.set_params(new, set_new=True, set_old=False)
        res["surr_after"] = float(policy.surrogate(obs, act, adv).detach().numpy())
        res["kl_dist"] = float(policy.kl(obs, act).detach().numpy())
        policy.set_params(new, set_new=True, set_old=True)
        res.update(npg_grad=g, cg_trace=[], alpha=learn_rate, delta=None, theta1=policy.get_params())
        return res

    cg_trace = [] if trace else None
    def f_Ax(v):
        if hvp_sample_frac is not None and hvp_sample_frac < 0.99:
            idx = np.random.choice(obs.shape[0], size=int(hvp_sample_frac * obs.shape[0]))
            return policy.fvp(obs[idx], act[idx], v, damping)
        return policy.fvp(obs, act, v, damping)

    x = cg_solve(f_Ax, g, iters=cg_iters, trace=cg_trace)
    res["npg_grad"] = x
    res["cg_trace"] = cg_trace
    gx = np.dot(g.T, x)

    theta = policy.get_params()
    if algo == "npg":
        if const_lr is not None:
            alpha = const_lr
            delta = (alpha ** 2) * gx
        else:
            delta = n_step_size if kl_dist is None else 2.0 * kl_dist
            alpha = np.sqrt(np.abs(delta / (gx + 1e-20)))
    else:
        delta = 2.0 * kl_dist
        alpha = np.sqrt(np.abs(delta / (gx + 1e-20)))
    res["delta"] = delta

    if algo == "trpo":
        trials = []
        for k in range(100):
            policy.set_params(theta + alpha * x, set_new=True, set_old=False)
            kl = float(policy.kl(obs, act).detach().numpy())
            surr = float(policy.surrogate(obs, act, adv).detach().numpy())
            trials.append((float(alpha), kl, surr))
            if kl < kl_dist:
                break
            alpha = 0.9 * alpha
            if k == 99:
                alpha = 0.0
        res["trials"] = trials
        policy.set_params(theta + alpha * x, set_new=True, set_old=False)
        res["kl_dist"] = float(policy.kl(obs, act).detach().numpy())
        res["surr_after"] = float(policy.surrogate(obs, act, adv).detach().numpy())
    else:
        policy.set_params(theta + alpha * x, set_new=True, set_old=False)
        res["surr_after"] = float(policy.surrogate(obs, act, adv).detach().numpy())
        res["kl_dist"] = float(policy.kl(obs, act).detach().numpy())
    policy.set_params(theta + alpha * x, set_new=True, set_old=True)
    res["alpha"] = alpha
    res["theta1"] = policy.get_params()
    return res


def hvp_rows(c):
    """Row indices of a fixture's standalone NPG.HVP call: all rows, or — for a
    subsampled Fisher — the draw the reference made after np.random.seed(hvp_np_seed)
    (npg_cg.py:58-62)."""
    N = c["obs"].shape[0]
    frac = float(c["kw_hvp_sample_frac"]) if "kw_hvp_sample_frac" in c else 1.0
    if frac >= 0.99:
        return np.arange(N)
    np.random.seed(int(c["hvp_np_seed"]))
    return np.random.choice(N, size=int(frac * N))


def cg_rows(c):
    """Row indices of each Fisher-vector product in the fixture's CG trace: the
    k-th draw after np.random.seed(np_seed), the reference's only global-RNG use
    in train_from_paths (npg_cg.py:58-62, cg_solve.py:10)."""
    N = c["obs"].shape[0]
    frac = float(c["kw_hvp_sample_frac"]) if "kw_hvp_sample_frac" in c else 1.0
    k = int(c["cg_iters_run"])
    if frac >= 0.99:
        return [np.arange(N)] * k
    np.random.seed(int(c["np_seed"]))
    return [np.random.choice(N, size=int(frac * N)) for _ in range(k)]


def regen_inputs(seed, n, m, lengths, col_scale=None, spiky=None, act_scale=None):
    """The synthetic paths of tests/golden/make_golden.py:make_paths, replayed from
    np.random.RandomState(seed) (legacy stream, stable across numpy versions): per
    path obs randn(H, n) (spiky columns zeroed where |draw| <= 1.5, times the column
    scales) and act randn(H, m) (times act_scale) rounded to f32, then rewards
    randn(H)."""
    rs = np.random.RandomState(int(seed))
    obs, act, rew = [], [], []
    for H in lengths:
        o = rs.randn(int(H), n)
        if spiky is not None:
            o[:, spiky] *= np.abs(o[:, spiky]) > 1.5
        if col_scale is not None:
            o = o * col_scale
        obs.append(o.astype(np.float32))
        a = rs.randn(int(H), m)
        if act_scale is not None:
            a = a * act_scale
        act.append(a.astype(np.float32))
        rew.append(rs.randn(int(H)))
    return np.concatenate(obs), np.concatenate(act), np.concatenate(rew)


def regen_f64obs(seed, n, lengths, col_scale=None, spiky=None):
    """The f64-observation fixtures' inputs (tests/golden/make_golden.py:f64obs_case)
    replayed from np.random.RandomState(seed): per path obs randn(H, n) (spiky
    columns zeroed where |draw| <= 1.5, times the column scales) kept in f64, then
    rewards randn(H).  Returns the per-path lists (obs, rewards)."""
    rs = np.random.RandomState(int(seed))
    obs, rew = [], []
    for H in lengths:
        o = rs.randn(int(H), n)
        if spiky is not None:
            o[:, spiky] *= np.abs(o[:, spiky]) > 1.5
        if col_scale is not None:
            o = o * col_scale
        obs.append(o)
        rew.append(rs.randn(int(H)))
    return obs, rew


def load_f64obs(path):
    """An f64-observation fixture with its inputs regenerated and checked against
    the stored checksum: dict of the .npz arrays plus obs_paths / rew_paths."""
    z = np.load(path, allow_pickle=False)
    c = {k: z[k] for k in z.files}
    obs, rew = regen_f64obs(c["gen_seed"], int(c["n"]), c["lengths"], col_scale=c.get("col_scale"),
                            spiky=c["spiky"].astype(bool) if "spiky" in c else None)
    if _sha(np.concatenate(obs), np.concatenate(rew)) != str(c["inputs_sha256"]):
        raise ValueError("%s: regenerated inputs do not match the fixture's checksum" % path)
    c["obs_paths"], c["rew_paths"] = obs, rew
    return c


def _sha(*arrs):
    import hashlib
    return hashlib.sha256(b"".join(np.ascontiguousarray(a).tobytes() for a in arrs)).hexdigest()


_CASES = {}


def load_case(path):
    """Loads a golden fixture into oracle-ready arrays (cached per path: treat the
    returned arrays as read-only).

    Large fixtures (gen_seed present) do not store their inputs: obs / act /
    rewards are replayed with regen_inputs and checked against the stored
    inputs_sha256; returns / advantages are recomputed by returns_and_advantages
    and checked bit for bit against the hashes of the reference's own arrays."""
    if path in _CASES:
        return _CASES[path]
    z = np.load(path, allow_pickle=False)
    c = {k: z[k] for k in z.files}
    if "gen_seed" in c:
        n, m = int(c["n"]), int(c["m"])
        c["obs"], c["act"], c["rewards"] = regen_inputs(
            c["gen_seed"], n, m, c["lengths"], col_scale=c.get("col_scale"),
            spiky=c["spiky"].astype(bool) if "spiky" in c else None,
            act_scale=float(c["act_scale"]) if "act_scale" in c else None)
        if _sha(c["obs"], c["act"], c["rewards"]) != str(c["inputs_sha256"]):
            raise ValueError("%s: regenerated inputs do not match the fixture's checksum" % path)
        lam = None if np.isnan(c["gae_lambda"]) else float(c["gae_lambda"])
        c["returns"], c["advantages"] = returns_and_advantages(c["rewards"], c["baseline"], c["lengths"],
                                                               c["terminated"].astype(bool), float(c["gamma"]),
                                                               lam)
        for k in ("returns", "advantages"):
            if _sha(c[k]) != str(c[k + "_sha256"]):
                raise ValueError("%s: recomputed %s differ from the reference's" % (path, k))
        c["_regen_keys"] = np.array(["obs", "act", "rewards", "returns", "advantages"])
    c["obs64"] = c["obs"].astype(np.float64)
    c["act64"] = c["act"].astype(np.float64)
    hidden = tuple(int(h) for h in c["hidden"])
    c["hidden_t"] = None if int(c["linear"]) else hidden
    tr = None
    if "in_shift" in c:
        tr = (c["in_shift"], c["in_scale"], c["out_shift"], c["out_scale"])
    c["transforms"] = tr
    _CASES[path] = c
    return c


def case_kwargs(c):
    """Algorithm kwargs of a fixture, in update()'s vocabulary."""
    algo = str(c["algo"])
    kw = dict(algo=algo)
    if "kw_hvp_sample_frac" in c:
        kw["hvp_sample_frac"] = float(c["kw_hvp_sample_frac"])
    if "np_seed" in c:
        kw["np_seed"] = int(c["np_seed"])
    if "kw_FIM_invert_args" in c:
        kw["cg_iters"] = int(c["kw_FIM_invert_args"][0])
        kw["damping"] = float(c["kw_FIM_invert_args"][1])
    if algo == "npg":
        if "kw_const_learn_rate" in c:
            kw["const_lr"] = float(c["kw_const_learn_rate"])
        if "kw_normalized_step_size" in c:
            kw["n_step_size"] = float(c["kw_normalized_step_size"])
        if "kw_kl_dist" in c:
            kw["kl_dist"] = float(c["kw_kl_dist"])
    elif algo == "trpo":
        kw["kl_dist"] = float(c["kw_kl_dist"]) if "kw_kl_dist" in c else 0.01
    elif algo == "vpg":
        kw["learn_rate"] = float(c["kw_learn_rate"]) if "kw_learn_rate" in c else 0.01
    elif algo == "dapg":
        kw["kl_dist"] = float(c["kw_kl_dist"]) if "kw_kl_dist" in c else 0.5 * 0.01
        kw["demo_obs"] = c["demo_obs"].astype(np.float64)
        kw["demo_act"] = c["demo_act"].astype(np.float64)
        kw["demo_coef"] = 1.0 * (0.95 ** (float(c["demo_iter_count"]) - 1.0))
    return kw
