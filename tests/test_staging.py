"""Host side of the paths -> HBM staging, on the CPU:
the native convert-and-range pass (mjrl_host_stage_*, engine.host_stage) and the
moment records of the sharded update (oracle.moments_record / moments_combine,
the restatement of mjrl_moments_combine)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib():
    from mjrl_amd import _lib, build
    import os
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    return _lib.load()


def _paths(rs, dtype):
    out = []
    for H in (1, 7, 300, 1000, 0, 64):
        o = rs.standard_normal((H, 37)) * np.logspace(-4, 3, 37)
        if H > 3:
            o[2, 5] = np.nan           # skipped by the range, kept in the data
            o[3, 6] = -1e30            # overflows to -inf in f32
        out.append(o.astype(dtype))
    return out


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_host_stage_converts_and_takes_ranges(lib, dtype):
    from mjrl_amd.engine import host_stage
    rs = np.random.RandomState(3)
    arrs = _paths(rs, dtype)
    arrs.append(np.asfortranarray(rs.standard_normal((50, 37))))   # non-contiguous: numpy fallback
    offs = np.concatenate([[0], np.cumsum([len(a) for a in arrs])])
    view = np.empty((offs[-1], 37), np.float32)
    lo, hi = np.full(37, np.inf, np.float32), np.full(37, -np.inf, np.float32)
    host_stage(arrs, view, offs, 0, len(arrs), lo, hi)
    ref = np.concatenate(arrs).astype(np.float32)     # torch .float(): round to nearest
    assert np.array_equal(view, ref, equal_nan=True)
    np.testing.assert_array_equal(lo, np.nanmin(ref, axis=0))
    np.testing.assert_array_equal(hi, np.nanmax(ref, axis=0))
    # without ranges: the conversion alone
    view2 = np.empty_like(view)
    host_stage(arrs, view2, offs, 0, len(arrs))
    assert np.array_equal(view2, ref, equal_nan=True)


@pytest.mark.parametrize("n", [1, 15, 16, 17, 37, 376, 9000])
def test_host_stage_avx512_equals_portable(lib, n):
    """The AVX-512 path (block buffer + streaming stores, run-time selected) writes
    the same floats and the same ranges as the portable loop, for every column
    count (masked tails), destination alignment (streamed head / body / tail) and
    special value (NaN skipped by the range, -0.0 vs 0.0 ties, f32 overflow);
    n = 9000 is wider than the block buffer (the portable loop takes over)."""
    import ctypes as C
    from mjrl_amd import _lib
    L = _lib.stage_lib()
    if not L.mjrl_host_stage_avx512():
        pytest.skip("no AVX-512 on this CPU")
    rs = np.random.RandomState(n)
    rows = 3 if n == 9000 else 203
    src = rs.standard_normal((rows, n)) * np.logspace(-3, 3, n)
    src[1, 0] = np.nan
    src[2, -1] = -0.0
    src[0, -1] = 0.0
    src[-1, n // 2] = 1e300
    for shift in (0, 1, 5, 15):   # destination misalignment in floats
        outs = []
        for fn in (L.mjrl_host_stage_f64, L.mjrl_host_stage_f64_portable):
            buf = np.zeros(rows * n + 32, np.float32)
            dst = buf[shift:shift + rows * n]
            lo, hi = np.full(n, np.inf, np.float32), np.full(n, -np.inf, np.float32)
            assert fn(src.ctypes.data, rows, n, dst.ctypes.data, lo.ctypes.data, hi.ctypes.data) == 0
            outs.append((buf.copy(), lo, hi))
        (b0, lo0, hi0), (b1, lo1, hi1) = outs
        assert np.array_equal(b0.view(np.uint32), b1.view(np.uint32))     # bit for bit, padding untouched
        assert np.array_equal(lo0.view(np.uint32), lo1.view(np.uint32))
        assert np.array_equal(hi0.view(np.uint32), hi1.view(np.uint32))
        assert np.array_equal(b0[shift:shift + rows * n].reshape(rows, n), src.astype(np.float32), equal_nan=True)


def test_host_stage_under_asan(tmp_path):
    """csrc/stage.cpp built with the host AddressSanitizer and UBSan into the
    driver tests/native/stage_asan.cpp and run over exactly-sized heap buffers:
    masked tails, streamed heads at every misalignment, the next-block prefetch and
    the batched per-chunk entry stay inside their buffers (ASan aborts otherwise)."""
    import os
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    here = os.path.dirname(os.path.abspath(__file__))
    exe = str(tmp_path / "stage_asan")
    subprocess.run([gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=undefined", os.path.join(here, "native", "stage_asan.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=180)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("dtype", [np.float64, np.int64, np.uint8])
def test_host_gather_concatenates_1d_slots(lib, dtype):
    """1-D slots (rewards, offsets, flags) go through mjrl_host_gather: the same
    bytes as np.concatenate, for empty arrays too; a non-contiguous array falls
    back to numpy."""
    from mjrl_amd.engine import host_stage
    rs = np.random.RandomState(5)
    arrs = [(rs.standard_normal(h) * 100).astype(dtype) for h in (1000, 0, 7, 1, 333)]
    arrs.append((rs.standard_normal(40) * 100).astype(dtype)[::2])   # strided
    offs = np.concatenate([[0], np.cumsum([len(a) for a in arrs])])
    view = np.zeros(offs[-1], dtype)
    host_stage(arrs, view, offs, 0, 5)
    host_stage(arrs, view, offs, 5, 6)
    assert np.array_equal(view.view(np.uint8), np.concatenate(arrs).view(np.uint8))
    from mjrl_amd import _lib
    assert _lib.stage_lib().mjrl_host_gather(None, None, -1, None) != 0


def test_staging_chunks_fold_ranges(lib):
    """_PinnedStaging folds the per-chunk ranges of many chunks (device-free part:
    the chunk fills, driven directly)."""
    from mjrl_amd.engine import host_stage
    rs = np.random.RandomState(4)
    arrs = [rs.standard_normal((100, 9)) * (i + 1) for i in range(40)]
    offs = np.concatenate([[0], np.cumsum([len(a) for a in arrs])])
    view = np.empty((offs[-1], 9), np.float32)
    bounds = [0, 7, 19, 33, 40]
    rng = np.empty((4, 2, 9), np.float32)
    rng[:, 0], rng[:, 1] = np.inf, -np.inf
    for k in range(4):
        host_stage(arrs, view, offs, bounds[k], bounds[k + 1], rng[k, 0], rng[k, 1])
    allv = np.concatenate(arrs).astype(np.float32)
    np.testing.assert_array_equal(rng[:, 0].min(0), allv.min(0))
    np.testing.assert_array_equal(rng[:, 1].max(0), allv.max(0))


@pytest.mark.parametrize("sizes", [(500, 700), (1, 999, 0), (250, 250, 250, 250), (1000,)])
def test_moment_records_combine_to_global_moments(sizes):
    """Sharded whitening / path-return statistics (npg_cg.py:91, 97-102): the fold
    of the shards' local two-pass records gives np.mean / np.std of the whole
    batch; with one shard it is that shard's own pass-2 sum bit for bit."""
    from oracle import npg_cpu as O
    rs = np.random.RandomState(sum(sizes))
    x = rs.standard_normal(sum(sizes)) * 3.0 + 1e3
    parts = np.split(x, np.cumsum(sizes)[:-1])
    out = O.moments_combine([O.moments_record(p) for p in parts])
    assert out[2] == len(x)
    np.testing.assert_allclose(out[0] / out[2], np.mean(x), rtol=1e-14)
    np.testing.assert_allclose(np.sqrt(out[9] / out[2]), np.std(x), rtol=1e-12)
    assert out[4] == x.max() and -out[5] == x.min()
    if len(sizes) == 1:
        rec = O.moments_record(x)
        assert out[9] == rec[9] and out[8] == rec[8]


F64OBS = ["f64obs_swimmer", "f64obs_humanoid"]


def _f64obs(name):
    import os
    from oracle import npg_cpu as O
    return O.load_f64obs(os.path.join(os.path.dirname(__file__), "golden", name + ".npz"))


def _pred_bound(coeffs, obs_paths):
    """|f . c| summed termwise: the scale a 1e-12 relative bound on a dot product
    of these features is taken against (a prediction near zero by cancellation
    carries the rounding of its large terms)."""
    from oracle import npg_cpu as O
    return np.concatenate([np.abs(O.linear_baseline_features(o)).dot(np.abs(coeffs)) for o in obs_paths])


@pytest.mark.parametrize("name", F64OBS)
def test_oracle_pinned_on_f64_observations(name):
    """The oracle's returns / GAE and LinearBaseline predict / fit against what the
    reference computed on observations that are not float32s."""
    from oracle import npg_cpu as O
    c = _f64obs(name)
    obs, rew, lengths = np.concatenate(c["obs_paths"]), np.concatenate(c["rew_paths"]), c["lengths"]
    term = c["terminated"].astype(bool)
    pred = O.linear_baseline_predict(c["coeffs0"], obs, lengths)
    assert np.all(np.abs(pred - c["baseline"]) <= 1e-12 * _pred_bound(c["coeffs0"], c["obs_paths"]))
    ret, adv = O.returns_and_advantages(rew, c["baseline"], lengths, term, float(c["gamma"]), float(c["gae_lambda"]))
    assert np.array_equal(ret, c["returns"]) and np.array_equal(adv, c["advantages"])
    coeffs = O.linear_baseline_fit(obs, c["returns"], lengths)
    assert np.linalg.norm(coeffs - c["coeffs1"]) <= fit_bound(c)


def fit_bound(c):
    """Bound on ||coeffs - reference's||: 1e-10 relative, or 3x the reference's
    own spread over path orders where its normal equations are ill-conditioned
    (Humanoid column scales: cond ~1e10, the spread ~5e-7 relative)."""
    return max(1e-10 * np.linalg.norm(c["coeffs1"]), 3.0 * float(c["coeffs1_spread"]))


@pytest.mark.parametrize("name", F64OBS)
def test_host_stage_extras_on_f64_observations(lib, name):
    """The staging pass's LinearBaseline extras (mjrl_host_stage_paths_f64x): the
    fp64 predictions from the sampler's own values within 1e-12 of the
    reference's LinearBaseline.predict, the advantages the GAE makes of them
    within the same bound of the reference's, the inexact flag raised, and the
    low halves carrying every value to 2^-48 (the device fit's f32 pair)."""
    from oracle import npg_cpu as O
    from mjrl_amd.engine import host_stage, host_stage_lo
    c = _f64obs(name)
    arrs, lengths = c["obs_paths"], c["lengths"]
    n = int(c["n"])
    offs = np.concatenate([[0], np.cumsum(lengths)])
    T = int(offs[-1])
    view = np.empty((T, n), np.float32)
    lo, hi = np.full(n, np.inf, np.float32), np.full(n, -np.inf, np.float32)
    pred, flag = np.full(T, np.nan), np.zeros(1, np.int32)
    mid = len(arrs) // 2   # two chunks, as the staging threads cut them
    for a0, a1 in ((0, mid), (mid, len(arrs))):
        host_stage(arrs, view, offs, a0, a1, lo, hi, extras=dict(coeffs=c["coeffs0"], pred=pred, npred=len(arrs),
                                                                 flag=flag))
    obs = np.concatenate(arrs)
    assert np.array_equal(view, obs.astype(np.float32))
    assert flag[0] == 1
    bound = 1e-12 * _pred_bound(c["coeffs0"], arrs)
    assert np.all(np.abs(pred - c["baseline"]) <= bound)
    _, adv = O.returns_and_advantages(np.concatenate(c["rew_paths"]), pred, lengths, c["terminated"].astype(bool),
                                      float(c["gamma"]), float(c["gae_lambda"]))
    np.testing.assert_allclose(adv, c["advantages"], rtol=0, atol=1e-10 * np.abs(c["advantages"]).max())
    low = np.empty_like(view)
    host_stage_lo(arrs, low, offs, 0, len(arrs))
    rec = view.astype(np.float64) + low
    assert np.all(np.abs(rec - obs) <= 2.0 ** -48 * np.abs(obs))
    # the fit from hi + lo (the device Gram's input) matches the reference's fit
    assert np.linalg.norm(O.linear_baseline_fit(rec, c["returns"], lengths) - c["coeffs1"]) <= fit_bound(c)


def test_host_stage_extras_portable_and_specials(lib):
    """The AVX-512 extras equal the portable loop's (NaN propagates through the
    clip as np.clip does, values past the float range, masked column tails), the
    flag stays 0 for float32-representable input, demo arrays (past npred) get no
    prediction, and a value past the float range gets a zero low half."""
    from mjrl_amd import _lib
    from mjrl_amd.engine import host_stage, host_stage_lo
    from oracle import npg_cpu as O
    L = _lib.stage_lib()
    rs = np.random.RandomState(8)
    for n in (1, 7, 8, 9, 37, 376):
        arrs = [rs.standard_normal((H, n)) * 6 for H in (3, 250, 1)]
        arrs[1][5, 0] = np.nan
        arrs[1][6, n - 1] = 1e39
        coeffs = rs.standard_normal(n + 4)
        offs = np.concatenate([[0], np.cumsum([len(a) for a in arrs])])
        view = np.empty((offs[-1], n), np.float32)
        pred, flag = np.full(offs[2], -7.0), np.zeros(1, np.int32)
        host_stage(arrs, view, offs, 0, 3, extras=dict(coeffs=coeffs, pred=pred, npred=2, flag=flag))
        ref = O.linear_baseline_predict(coeffs, np.concatenate(arrs[:2]), [3, 250])
        assert np.array_equal(np.isnan(pred), np.isnan(ref))
        ok = ~np.isnan(ref)
        assert np.all(np.abs(pred[ok] - ref[ok]) <= 1e-12 * _pred_bound(coeffs, arrs[:2])[ok])
        assert flag[0] == 1
        import ctypes as C
        for a, o0 in zip(arrs[:2], offs[:2]):
            pp, fl = np.zeros(len(a)), np.zeros(1, np.int32)
            assert L.mjrl_host_extras_portable(a.ctypes.data, len(a), n, coeffs.ctypes.data, pp.ctypes.data,
                                               fl.ctypes.data) == 0
            got = pred[o0:o0 + len(a)]
            assert np.array_equal(np.isnan(pp), np.isnan(got))
            m = ~np.isnan(pp)
            assert np.all(np.abs(pp[m] - got[m]) <= 1e-13 * (np.abs(got[m]) + 1))
        low = np.empty_like(view)
        host_stage_lo(arrs, low, offs, 0, 3)
        assert low[offs[1] + 6, n - 1] == 0.0 and np.isinf(view[offs[1] + 6, n - 1])
        exact = [a.astype(np.float32).astype(np.float64) for a in arrs[:1]] + [np.zeros((4, n))]
        eoffs = np.concatenate([[0], np.cumsum([len(a) for a in exact])])
        flag[0] = 0
        host_stage(exact, np.empty((eoffs[-1], n), np.float32), eoffs, 0, 2,
                   extras=dict(coeffs=None, pred=None, npred=2, flag=flag))
        assert flag[0] == 0


def test_rows_entry_equals_block_pass(lib):
    """mjrl_host_stage_rows_f64x (one row per environment per step, scattered into
    the trajectories' slabs: the streaming sink's call) writes the same floats,
    predictions (bit for bit: the same per-row arithmetic), ranges and flag as
    the block pass over the finished paths."""
    import ctypes as C
    from mjrl_amd import _lib
    from mjrl_amd.engine import host_stage
    L = _lib.stage_lib()
    rs = np.random.RandomState(12)
    for n in (6, 17, 376):
        lengths = [5, 40, 1, 33]
        arrs = [rs.standard_normal((H, n)) * 7 for H in lengths]
        arrs[1][3, 2] = np.nan
        coeffs = rs.standard_normal(n + 4)
        offs = np.concatenate([[0], np.cumsum(lengths)])
        T = int(offs[-1])
        view = np.empty((T, n), np.float32)
        lo, hi = np.full(n, np.inf, np.float32), np.full(n, -np.inf, np.float32)
        pred, flag = np.zeros(T), np.zeros(1, np.int32)
        host_stage(arrs, view, offs, 0, len(arrs), lo, hi, extras=dict(coeffs=coeffs, pred=pred, npred=len(arrs),
                                                                       flag=flag))
        # the same rows handed over step by step, the live paths of each step at once
        dst = np.full((T, n), -1.0, np.float32)
        lo2, hi2 = np.full(n, np.inf, np.float32), np.full(n, -np.inf, np.float32)
        pred2, flag2 = np.zeros(T), np.zeros(1, np.int32)
        for t in range(max(lengths)):
            live = [i for i, H in enumerate(lengths) if t < H]
            src = np.ascontiguousarray(np.stack([arrs[i][t] for i in live]))
            ptrs = (C.c_void_p * len(live))(*[dst[offs[i] + t:].ctypes.data for i in live])
            tidx = np.full(len(live), t, np.int64)
            pr = np.zeros(len(live))
            assert L.mjrl_host_stage_rows_f64x(src.ctypes.data, len(live), n, ptrs, lo2.ctypes.data, hi2.ctypes.data,
                                               coeffs.ctypes.data, tidx.ctypes.data, pr.ctypes.data,
                                               flag2.ctypes.data) == 0
            for j, i in enumerate(live):
                pred2[offs[i] + t] = pr[j]
        assert np.array_equal(dst, view, equal_nan=True)
        assert np.array_equal(pred2, pred, equal_nan=True)
        assert np.array_equal(lo2, lo) and np.array_equal(hi2, hi) and flag2[0] == flag[0] == 1
