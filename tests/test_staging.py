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
