"""Host-side logic of the drop-in API (no GPU): the policy mirror reproduces the
reference's parameters, layout, clamps and pickling; path partitioning; DataLog;
the baselines that feed the GAE scan."""
import copy
import os
import pickle

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import npg_cpu as O


def case(name):
    return O.load_case(os.path.join(GOLDEN, name + ".npz"))


@pytest.mark.parametrize("name,hidden", [("c2_swimmer", (64, 64)), ("c3_halfcheetah_trpo", (128, 128)),
                                         ("c4_humanoid", (64, 64)), ("c1_pointmass_mlp32", (32, 32))])
def test_mlp_init_matches_reference_bitwise(name, hidden):
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    c = case(name)
    pol = MLP(EnvSpec(int(c["n"]), int(c["m"]), 10, 1), hidden_sizes=hidden, seed=0)
    assert pol.d == c["theta0"].size
    assert np.array_equal(pol.get_param_values(), c["theta0"])
    assert pol.param_sizes == list(c["param_sizes"])


def test_linear_policy_init_matches_reference_bitwise():
    from mjrl_amd.policies.gaussian_linear import LinearPolicy
    from mjrl_amd.utils.gym_env import EnvSpec
    c = case("c1_pointmass_linear")
    pol = LinearPolicy(EnvSpec(6, 2, 25, 1), seed=0)
    assert np.array_equal(pol.get_param_values(), c["theta0"])


def test_set_param_values_clamps_log_std_and_keeps_order():
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    pol = MLP(EnvSpec(5, 3, 10, 1), hidden_sizes=(32, 32), seed=1)
    th = np.arange(pol.d, dtype=np.float64) * 1e-3
    th[-3:] = [-5.0, -3.0, 0.25]
    pol.set_param_values(th, set_new=True, set_old=False)
    got = pol.get_param_values()
    assert np.array_equal(got[:-3], th[:-3].astype(np.float32))
    assert np.array_equal(got[-3:], np.float32([-3.0, -3.0, 0.25]))   # min_log_std = -3
    assert np.allclose(pol.log_std_val, [-3.0, -3.0, 0.25])
    old = np.concatenate([p.data.reshape(-1).numpy() for p in pol.old_params])
    assert not np.array_equal(old, got)                                   # set_old=False
    pol.set_param_values(th, set_new=False, set_old=True)
    old = np.concatenate([p.data.reshape(-1).numpy() for p in pol.old_params])
    assert np.array_equal(old, got)
    # W0 is [h0, n] row-major first, then b0, ... (gaussian_mlp.py:38, 61-64)
    assert np.array_equal(pol.model.fc0.weight.data.numpy().ravel(), th[:32 * 5].astype(np.float32))


def test_cpu_mirror_forward_matches_reference_outputs():
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    c = case("c2_swimmer")
    pol = MLP(EnvSpec(8, 2, 10, 1), seed=0)
    mu, ll = pol.mean_LL(c["obs64"], c["act64"])
    np.testing.assert_allclose(mu.detach().numpy(), c["mean0"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(ll.detach().numpy(), c["ll0"], rtol=1e-5)


def test_policy_pickles_and_deepcopies_to_cpu_state():
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    pol = MLP(EnvSpec(4, 2, 10, 1), hidden_sizes=(32, 32), seed=3)
    for clone in (pickle.loads(pickle.dumps(pol)), copy.deepcopy(pol)):
        assert np.array_equal(clone.get_param_values(), pol.get_param_values())
        a, info = clone.get_action(np.ones(4))
        assert a.shape == (2,) and set(info) == {"mean", "log_std", "evaluation"}
        assert all(not p.is_cuda for p in clone.trainable_params)


def test_agent_pickles_without_device_state():
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.baselines.zero_baseline import ZeroBaseline
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    spec = EnvSpec(4, 2, 10, 1)
    agent = NPG(None, MLP(spec, (32, 32), seed=0), ZeroBaseline(spec), normalized_step_size=0.1, save_logs=True)
    agent._engine = lambda: None   # stands in for a live (unpicklable) device engine
    clone = pickle.loads(pickle.dumps(agent))
    assert clone._engine is None
    assert np.array_equal(clone.policy.get_param_values(), agent.policy.get_param_values())


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_partition_paths_balanced_contiguous(world):
    from mjrl_amd.comm import partition_paths
    rs = np.random.RandomState(world)
    lengths = rs.randint(1, 1000, size=57)
    parts = partition_paths(lengths, world)
    assert len(parts) == world
    assert parts[0][0] == 0 and parts[-1][1] == len(lengths)
    for (a, b), (c, d) in zip(parts, parts[1:]):
        assert b == c and a <= b
    loads = [lengths[a:b].sum() for a, b in parts]
    assert max(loads) - min(loads) <= 2 * lengths.max()
    # fewer paths than ranks: empty shards are allowed, coverage still exact
    p2 = partition_paths([5, 5], 4)
    assert sum(b - a for a, b in p2) == 2


def test_datalog_roundtrip(tmp_path):
    from mjrl_amd.utils.logger import DataLog
    log = DataLog()
    for i in range(3):
        log.log_kv("alpha", 0.1 * i)
        log.log_kv("kl_dist", 0.01 * i)
    log.log_kv("alpha", 9.0)
    log.save_log(str(tmp_path))
    assert log.get_current_log() == {"alpha": 9.0, "kl_dist": 0.02}
    other = DataLog()
    other.read_log(str(tmp_path / "log.csv"))
    assert other.log["alpha"] == [0.0, 0.1, 0.2, 9.0]
    assert other.log["kl_dist"] == [0.0, 0.01, 0.02]
    with open(tmp_path / "log.pickle", "rb") as f:   # file written by this test
        assert pickle.load(f)["alpha"][-1] == 9.0


def test_baselines_match_reference():
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.baselines.quadratic_baseline import QuadraticBaseline
    from mjrl_amd.utils.gym_env import EnvSpec
    z = np.load(os.path.join(GOLDEN, "baselines.npz"))
    lengths = z["lengths"]
    offs = np.concatenate([[0], np.cumsum(lengths)])
    paths = [dict(observations=z["obs"][offs[i]:offs[i + 1]], rewards=z["rewards"][offs[i]:offs[i + 1]],
                  returns=z["returns"][offs[i]:offs[i + 1]]) for i in range(len(lengths))]
    spec = EnvSpec(z["obs"].shape[1], 2, 30, 1)
    for cls, key in ((LinearBaseline, "lin"), (QuadraticBaseline, "quad")):
        b = cls(spec)
        assert np.array_equal(b.predict(paths[0]), np.zeros(lengths[0]))
        err = b.fit(paths, return_errors=True)
        np.testing.assert_allclose(b._coeffs, z[key + "_coeffs"], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(np.concatenate([b.predict(p) for p in paths]), z[key + "_pred"], rtol=1e-9,
                                   atol=1e-12)
        np.testing.assert_allclose(err, z[key + "_err"], rtol=1e-9)


def test_linear_baseline_predictions_feed_gae_bitexact():
    """The fixture's baseline column came from the reference LinearBaseline."""
    from mjrl_amd.baselines.linear_baseline import LinearBaseline
    from mjrl_amd.utils.gym_env import EnvSpec
    c = case("c2_ragged")
    b = LinearBaseline(EnvSpec(8, 2, 10, 1))
    b._coeffs = c["baseline_coeffs"]
    offs = np.concatenate([[0], np.cumsum(c["lengths"])])
    pred = np.concatenate([b.predict(dict(observations=c["obs64"][offs[i]:offs[i + 1]],
                                          rewards=c["rewards"][offs[i]:offs[i + 1]]))
                           for i in range(len(c["lengths"]))])
    assert np.array_equal(pred, c["baseline"])


def test_engine_methods_run_on_their_device():
    """Every UpdateEngine entry point that launches kernels makes self.device
    current first (the kernels go to torch's current stream of that device)."""
    from mjrl_amd.engine import UpdateEngine
    for name in ("update", "returns_advantages", "normalize_advantages", "fit_linear_baseline",
                 "fit_quadratic_baseline", "fvp",
                 "load_rows", "forward_pass", "eval_pass"):
        fn = getattr(UpdateEngine, name)
        assert getattr(fn, "__wrapped__", None) is not None, name


def test_unsupported_policy_shape_rejected_at_construction():
    """Hidden sizes the kernels cannot run are rejected when the agent is built,
    not deep inside the first update; others run zero-padded."""
    import pytest
    from mjrl_amd.algos.npg_cg import NPG
    from mjrl_amd.engine import kernel_hidden, padded_positions
    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.utils.gym_env import EnvSpec
    assert kernel_hidden(8, 2, (48, 32)) == (64, 64)
    assert kernel_hidden(8, 2, (100, 50)) == (128, 128)
    assert kernel_hidden(8, 2, None) == (0, 0)
    NPG(None, MLP(EnvSpec(8, 2, 10, 1), hidden_sizes=(100, 50), seed=0), None)   # fine: padded
    with pytest.raises(ValueError, match="hidden sizes up to 256"):
        NPG(None, MLP(EnvSpec(8, 2, 10, 1), hidden_sizes=(300, 64), seed=0), None)
    with pytest.raises(ValueError, match="act_dim"):
        NPG(None, MLP(EnvSpec(8, 70, 10, 1), hidden_sizes=(64, 64), seed=0), None)
    idx = padded_positions(8, 2, (48, 32), (64, 64))
    assert len(idx) == 48 * 8 + 48 + 32 * 48 + 32 + 2 * 32 + 2 + 2 and len(set(idx.tolist())) == len(idx)


def test_mlp_baseline_mirror_matches_reference_init_and_leaves_env_alone():
    """MLPBaseline (mlp_baseline.py:15-35): same modules in the same order, so
    torch.manual_seed gives the reference's initial weights bit for bit; importing
    it changes no environment variable (the reference sets CUDA_VISIBLE_DEVICES)."""
    import importlib
    import os
    import sys
    before = dict(os.environ)
    sys.modules.pop("mjrl_amd.baselines.mlp_baseline", None)
    mod = importlib.import_module("mjrl_amd.baselines.mlp_baseline")
    assert dict(os.environ) == before
    from mjrl_amd.utils.gym_env import EnvSpec
    z = np.load(os.path.join(GOLDEN, "mlp_baseline.npz"))
    torch.manual_seed(7)
    b = mod.MLPBaseline(EnvSpec(5, 2, 300, 1), batch_size=64, epochs=2, learn_rate=3e-3)
    for k, v in b.model.state_dict().items():
        assert np.array_equal(v.numpy(), z["init_" + k.replace(".", "_")]), k
    offs = np.concatenate([[0], np.cumsum(z["lengths"])])
    paths = [dict(observations=z["obs"][offs[i]:offs[i + 1]], rewards=z["rewards"][offs[i]:offs[i + 1]])
             for i in range(len(z["lengths"]))]
    f = b._features(paths)
    t = np.concatenate([np.arange(L) / 1000.0 for L in z["lengths"]])
    np.testing.assert_array_equal(f[:, :5], np.clip(z["obs"], -10, 10) / 10.0)
    np.testing.assert_array_equal(f[:, 5:], np.stack([t, t ** 2, t ** 3, t ** 4], 1))
    clone = pickle.loads(pickle.dumps(b))
    assert all(torch.equal(a, c) for a, c in zip(clone.model.parameters(), b.model.parameters()))


def test_mlp_baseline_device_mirror_tracks_cpu_parameters():
    """MLPBaseline's staleness key changes when the CPU parameters are replaced
    or modified in place, so a forward re-copies them to the device."""
    from mjrl_amd.baselines.mlp_baseline import MLPBaseline
    from mjrl_amd.utils.gym_env import EnvSpec
    b = MLPBaseline(EnvSpec(4, 1, 10, 1))
    k0 = b._cpu_key()
    with torch.no_grad():
        next(b.model.parameters()).add_(1.0)
    k1 = b._cpu_key()
    assert k1 != k0
    p = next(b.model.parameters())
    p.data = p.data.clone()
    assert b._cpu_key() != k1
    assert b._cpu_key() == b._cpu_key()


def test_bench_pmc_key_matches_committed_summary():
    """bench.py's roofline.traffic comes from the newest committed PMC summary:
    the key it builds for the default workload's FVP kernel (k_kx<32, 12, 1,
    false> at Humanoid: MP 32, NP 384) must name an entry of that file (round 5
    printed traffic: null after the kernel gained a template argument)."""
    import bench
    name, key = bench.fvp_kernel_key(2, True, 32, 384, 64, 64)
    assert key == "k_kx<32, 12, 1, false>"
    b, src, err = bench.pmc_traffic(key)
    assert err is None and b > 2.0e9, (src, err)
