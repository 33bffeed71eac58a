"""The C-ABI library loads and exports every entry point include/mjrl_amd.h
declares; the host-only entry points (shape / scratch sizing) work without a GPU."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mjrl_amd.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\bint\s+(mjrl_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from mjrl_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    return _lib.load()


def test_every_declared_symbol_is_exported(lib):
    from mjrl_amd import _lib
    names = declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    # and every binding the Python side declares exists in the header
    assert set(_lib.SIGNATURES) <= set(names)
    assert set(names) <= set(_lib.SIGNATURES), set(names) - set(_lib.SIGNATURES)


def test_stage_lib_exports_every_host_entry_point(lib):
    """The host-only lib/libmjrl_stage.so carries every mjrl_host_* entry point the
    header declares (the pool controller loads only it)."""
    from mjrl_amd import _lib
    host = [n for n in declared() if n.startswith("mjrl_host_")]
    assert set(host) == set(_lib.STAGE_FUNCS)
    S = _lib.stage_lib()
    for n in host:
        assert hasattr(S, n), n


@pytest.mark.parametrize("n,m,h,np_,mp,d", [
    (6, 2, (0, 0), 16, 16, 16),            # point_mass, linear policy
    (8, 2, (64, 64), 16, 16, 4868),        # swimmer
    (17, 6, (128, 128), 32, 16, 19596),    # halfcheetah
    (376, 17, (64, 64), 384, 32, 29410),   # humanoid
    (39, 28, (256, 256), 48, 32, 83256),   # door
    (15, 40, (32, 32), 16, 64, 15 * 32 + 32 + 32 * 32 + 32 + 40 * 32 + 40 + 40),
])
def test_shape_padding(lib, n, m, h, np_, mp, d):
    from mjrl_amd import _lib
    s = _lib.make_shape(n, m, h[0], h[1])
    assert (s.np, s.mp, s.d) == (np_, mp, d)
    assert s.np >= n + 1 and s.np % 16 == 0        # bias column always present
    wf, rd, sl = C.c_int64(), C.c_int64(), C.c_int32()
    assert lib.mjrl_scratch_size(C.byref(s), 1000000, C.byref(wf), C.byref(rd), C.byref(sl)) == 0
    assert 1 <= sl.value <= 256 and wf.value > 0 and rd.value > 0


@pytest.mark.parametrize("n,m,h", [(6, 2, (0, 0)), (8, 2, (64, 64)), (17, 6, (128, 128)), (376, 17, (64, 64)),
                                   (39, 28, (256, 256)), (15, 40, (32, 32)), (45, 24, (128, 128))])
def test_scratch_size_is_monotonic(lib, n, m, h):
    """A scratch sized by mjrl_scratch_size for T rows must hold every pass over
    T' <= T rows (the engine sizes it once for the batch, then runs FVPs over the
    RL rows only, subsampled rows, ...): sizes and slice counts never shrink as T
    grows, over the tile-count boundaries of every kernel's grid."""
    from mjrl_amd import _lib
    s = _lib.make_shape(n, m, h[0], h[1])
    prev_w, prev_s = 0, 0
    Ts = sorted(set([1, 15, 16, 17, 31, 32, 33, 63, 64, 65] + [k * 16 + d for k in range(1, 1200, 7) for d in (-1, 0, 1)]
                    + [b * t + d for b in (16, 32, 64) for t in (128, 256) for d in (-1, 0, 1, b, b + 1)]
                    + [8192 * 32 + d for d in (-33, -1, 0, 1, 33)] + [1000000, 1000001]))
    for T in Ts:
        wf, rd, sl = C.c_int64(), C.c_int64(), C.c_int32()
        assert lib.mjrl_scratch_size(C.byref(s), T, C.byref(wf), C.byref(rd), C.byref(sl)) == 0
        assert wf.value >= prev_w and sl.value >= prev_s, T
        prev_w, prev_s = wf.value, sl.value


def test_unsupported_shape_is_rejected(lib):
    from mjrl_amd import _lib
    s = _lib.Shape()
    assert lib.mjrl_shape_init(C.byref(s), 10, 3, 48, 48) == _lib.MJRL_ESHAPE
    assert lib.mjrl_shape_init(C.byref(s), 0, 3, 64, 64) == _lib.MJRL_EINVAL
    with pytest.raises(_lib.MjrlError):
        _lib.make_shape(10, 100, 64, 64)


def test_null_arguments_fail_loudly(lib):
    from mjrl_amd import _lib
    s = _lib.make_shape(8, 2, 64, 64)
    # argument validation happens before any launch: no GPU needed
    assert lib.mjrl_pack_batch(None, None, 10, C.byref(s), None, None, None, None, None) == _lib.MJRL_EINVAL
    assert lib.mjrl_gae(None, None, None, None, 5, 0.99, 0.97, 1, None, None, None, None) == _lib.MJRL_EINVAL
    assert lib.mjrl_policy_fvp(C.byref(s), None, 10, None, None, None, None, None, None, None) == _lib.MJRL_EINVAL
    assert lib.mjrl_gather_rows(None, 16, None, 4, None, None) == _lib.MJRL_EINVAL
    assert lib.mjrl_gather_rows(C.c_void_p(16), 6, C.c_void_p(16), 4, C.c_void_p(16), None) == _lib.MJRL_EINVAL
    assert lib.mjrl_gather_rows(None, 16, None, 0, None, None) == _lib.MJRL_OK


def test_no_gpu_means_no_compute():
    """On a host without a GPU the product path refuses to run (no CPU fallback)."""
    import torch
    from mjrl_amd import _lib
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.MjrlError):
        _lib.lib()
