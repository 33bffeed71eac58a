"""CPU model of the split-f16 row format (mjrl_rows.xs, csrc/common.h), checked on
the reference-generated c4_humanoid_scaled fixture's observations.

The GPU pack is tested against this bound in tests/test_gpu_split.py; here a
numpy emulation of the two row formats (np.float16 conversion rounds to nearest
even, as v_cvt_f16_f32 does; y - hi is exact in f32) shows why the column scales
exist:
  round-2 format: one power-of-two scale per ROW, max |y| in [1/2, 1)
  round-3 format: one power of two per COLUMN (batch max), then one per row with
                  max |y| in [2^14, 2^15)
and measures what each does to gradient-like column sums sum_t g[t, j] x[t, k]
(the W0 block of the VPG and of F v), per observation column.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _pow2_exp(m):
    """E with m 2^-E in [1/2, 1) (frexp), 0 for m == 0."""
    _, e = np.frexp(m)
    return np.where(m > 0, e, 0)


def split_pair(y):
    y = np.asarray(y, np.float32)
    hi = y.astype(np.float16)
    lo = (y - hi.astype(np.float32)).astype(np.float16)
    return hi.astype(np.float64) + lo.astype(np.float64)


def rows_round2(x):
    s = np.ldexp(1.0, -_pow2_exp(np.abs(x).max(1)))[:, None]
    return split_pair(x * s) / s


def rows_round3(x):
    colmax = np.abs(x).max(0)
    xc = np.where(colmax > 0, np.ldexp(1.0, _pow2_exp(colmax)), 1.0)
    y = x / xc[None, :]
    e = _pow2_exp(np.abs(y).max(1))
    s = np.ldexp(1.0, 15 - e)[:, None]
    return split_pair(y * s) / s * xc[None, :], colmax


@pytest.fixture(scope="module")
def scaled_obs():
    from oracle import npg_cpu as O
    c = O.load_case(os.path.join(GOLDEN, "c4_humanoid_scaled.npz"))
    x = c["obs"][:6000].astype(np.float32)
    x = np.concatenate([x, np.ones((x.shape[0], 1), np.float32)], 1)   # the bias column
    return x


def _colsum_err(x, xr, rs):
    g = rs.randn(x.shape[0], 8)
    ref = g.T @ x.astype(np.float64)
    got = g.T @ xr
    den = np.abs(ref).max(0)
    ok = den > 0
    return np.abs(got - ref).max(0)[ok] / den[ok]


def test_fixture_rows_span_many_decades(scaled_obs):
    x = np.abs(scaled_obs[:, :-1].astype(np.float64))
    nz = np.where(x > 0, x, np.inf).min(1)
    assert np.median(x.max(1) / nz) > 1e8   # ~8.6 decades per row


def test_round3_element_bound(scaled_obs):
    x = scaled_obs.astype(np.float64)
    rec, colmax = rows_round3(scaled_obs)
    bound = 2.0 ** -23 * np.abs(x) + 2.0 ** -38 * colmax[None, :]
    assert np.all(np.abs(rec - x) <= bound)


def test_column_sums_round3_vs_round2(scaled_obs):
    """Per-column relative error of sum_t g x[:, k]: round-3 rows stay at f32 level
    (< 2e-7 on every column); the round-2 rows (row block, no column scale) lose
    the small-scale columns entirely."""
    rs = np.random.RandomState(0)
    e3 = _colsum_err(scaled_obs, rows_round3(scaled_obs)[0], rs)
    rs = np.random.RandomState(0)
    e2 = _colsum_err(scaled_obs, rows_round2(scaled_obs), rs)
    assert e3.max() < 2e-7, e3.max()
    assert e2.max() > 1e-2, e2.max()
    print("per-column max rel err: round-3 %.2e, round-2 %.2e (median %.2e)" % (e3.max(), e2.max(), np.median(e2)))
