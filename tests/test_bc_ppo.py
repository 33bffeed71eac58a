"""BC and PPO against fixtures of the reference's own
runs (tests/golden/make_golden.py bc_case / ppo_case).  CPU tests here run BC's
minibatch steps on the CPU device (the same math the GPU replays); the GPU
variants are in test_gpu_api.py."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _bc_paths(z):
    offs = np.concatenate([[0], np.cumsum(z["lengths"])])
    return [dict(observations=z["obs"][offs[i]:offs[i + 1]], actions=z["act"][offs[i]:offs[i + 1]])
            for i in range(len(z["lengths"]))]


def run_bc(device):
    from mjrl_amd.algos.behavior_cloning import BC
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    z = np.load(os.path.join(GOLDEN, "bc.npz"))
    policy = MLP(EnvSpec(6, 3, 120, 1), hidden_sizes=(32, 32), seed=5)
    np.testing.assert_array_equal(policy.get_param_values(), z["init"])
    bc = BC(_bc_paths(z), policy, epochs=2, batch_size=32, lr=1e-3, device=device)
    t = policy.model.transformations
    for k in ("in_shift", "in_scale", "out_shift", "out_scale"):
        np.testing.assert_allclose(t[k], z[k], rtol=1e-12)
    np.random.seed(int(z["np_seed"]))
    bc.train()
    return bc, policy, z


def test_bc_matches_reference_cpu_device():
    bc, policy, z = run_bc("cpu")
    # same CPU torch kernels, the functional forward: agreement to f32 rounding
    np.testing.assert_allclose(np.array(bc.logger.log["loss"], dtype=np.float64), z["loss"], rtol=1e-5)
    ref = z["final"]
    assert np.linalg.norm(policy.get_param_values() - ref) <= 1e-5 * np.linalg.norm(ref)
    assert bc.logger.log["epoch"] == [0, 1, 2]


def test_bc_pickles_and_keeps_optimizer_state():
    import pickle
    bc, policy, z = run_bc("cpu")
    st = bc.optimizer.state[policy.trainable_params[0]]
    nmb = int(sum(z["lengths"]) / 32)
    assert float(st["step"]) == 2 * nmb          # the CPU optimizer carries the device steps
    clone = pickle.loads(pickle.dumps(bc))
    assert clone._trainer is None
    np.testing.assert_array_equal(clone.policy.get_param_values(), policy.get_param_values())


def test_ppo_surrogate_gradient_matches_autograd():
    """The minibatch PPO loss of _device_sgd (functional policy, LR != 1) has the
    gradient of the reference's PPO_surrogate on the CPU modules (ppo_clip.py:47-54)."""
    from mjrl_amd.algos._device_sgd import DeviceTrainer
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    rs = np.random.RandomState(0)
    policy = MLP(EnvSpec(5, 2, 10, 1), hidden_sizes=(16, 8), seed=1, init_log_std=-0.3)
    theta = policy.get_param_values()
    policy.set_param_values(theta + 0.05 * rs.randn(theta.size).astype(np.float32), set_new=True, set_old=False)
    obs, act, adv = rs.randn(40, 5), rs.randn(40, 2), rs.randn(40)
    # reference form on the CPU modules
    LLn = policy.new_dist_info(obs, act)[0]
    LLo = policy.old_dist_info(obs, act)[0]
    LR = torch.exp(LLn - LLo)
    a = torch.from_numpy(adv).float()
    surr = torch.mean(torch.min(LR * a, torch.clamp(LR, 0.8, 1.2) * a))
    g_ref = torch.autograd.grad(surr, policy.trainable_params)
    opt = torch.optim.Adam(policy.trainable_params, lr=1e-3)
    tr = DeviceTrainer(policy, opt, "cpu")
    tr.pull()
    O, A = torch.from_numpy(obs).float(), torch.from_numpy(act).float()
    ll_old = tr.log_likelihood(O, A, [p.data for p in policy.old_params])
    LR2 = torch.exp(tr.log_likelihood(O, A) - ll_old)
    s2 = torch.mean(torch.min(LR2 * a, torch.clamp(LR2, 0.8, 1.2) * a))
    g = torch.autograd.grad(s2, tr.params)
    assert abs(float(s2.detach()) - float(surr.detach())) < 1e-6
    for x, y in zip(g, g_ref):
        np.testing.assert_allclose(x.numpy(), y.numpy(), rtol=1e-4, atol=1e-7)


def test_ppo_matches_reference_cpu_device():
    """PPO.train_from_paths twice on the CPU device, the surrogate / KL passes
    taken from the CPU policy (the HIP evaluation passes are GPU-tested):
    parameters, KL and surrogate improvement equal the reference's run —
    including its second iteration, where set_param_values has left the old and
    new mean networks sharing storage (PPO._old_on_device)."""
    from mjrl_amd.algos.ppo_clip import PPO
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    z = np.load(os.path.join(GOLDEN, "ppo.npz"))
    policy = MLP(EnvSpec(6, 2, 200, 1), hidden_sizes=(32, 32), seed=3, init_log_std=-0.5)
    ppo = PPO(None, policy, None, clip_coef=0.2, epochs=2, mb_size=64, learn_rate=3e-3, save_logs=True,
              device="cpu")

    def cpi(o, a, adv):
        LLn, LLo = policy.new_dist_info(o, a)[0], policy.old_dist_info(o, a)[0]
        return torch.mean(torch.exp(LLn - LLo) * torch.from_numpy(adv).float()).detach()

    ppo.CPI_surrogate = cpi
    ppo.kl_old_new = lambda o, a: policy.mean_kl(policy.new_dist_info(o, a), policy.old_dist_info(o, a)).detach()
    ppo.engine = lambda: type("E", (), {"device": torch.device("cpu")})
    offs = np.concatenate([[0], np.cumsum(z["lengths"])])
    for it in range(2):
        sl = lambda k: [z["%s%d" % (k, it)][offs[i]:offs[i + 1]] for i in range(len(z["lengths"]))]
        paths = [dict(observations=o, actions=a, rewards=r, advantages=v)
                 for o, a, r, v in zip(sl("obs"), sl("act"), sl("rew"), sl("adv"))]
        np.random.seed(int(z["np_seed%d" % it]))
        stats = ppo.train_from_paths(paths)
        np.testing.assert_allclose(stats, z["base_stats%d" % it], rtol=1e-12)
        ref = z["params%d" % it]
        assert np.linalg.norm(policy.get_param_values() - ref) <= 1e-6 * np.linalg.norm(ref), it
        np.testing.assert_allclose(ppo.logger.log["kl_dist"][-1], z["kl_dist%d" % it], rtol=1e-4)
        np.testing.assert_allclose(ppo.logger.log["surr_improvement"][-1], z["surr_improvement%d" % it],
                                   rtol=1e-4, atol=1e-7)
