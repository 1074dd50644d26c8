"""DTW without the cost matrix (checkpoint mode, the default when the caller does not ask for
the matrix): the band kernel keeps every 64th column of C and the path costs are recomputed per
64 x 64 tile the path visits (dtw_path_tile_kernel).  The result must be bit-identical to the
full-store path (want_cost=True), which the oracle tests pin against dtw.go:55-217: same path,
same per-point costs, same distance -- including banded runs, sizes that are and are not
multiples of 64, and non-finite inputs (math.Min's NaN / -Inf rules, border points)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _same(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape
    assert np.array_equal(np.isnan(a), np.isnan(b))
    m = ~np.isnan(a)
    assert np.array_equal(a[m].view(np.uint64), b[m].view(np.uint64))


def _check(ctx, q, r, band=-1):
    ck = ctx.dtw(q, r, band=band)
    full = ctx.dtw(q, r, band=band, want_cost=True)
    assert np.array_equal(ck["path_q"], full["path_q"])
    assert np.array_equal(ck["path_r"], full["path_r"])
    _same(ck["path_cost"], full["path_cost"])
    _same([ck["distance"]], [full["distance"]])
    return ck


@pytest.mark.parametrize("nq,nr,dim,band", [
    (1, 1, 1, -1), (5, 300, 3, -1), (64, 64, 12, -1), (65, 128, 12, -1), (130, 129, 2, -1),
    (200, 320, 12, -1), (777, 1000, 12, 100), (1000, 640, 1, -1), (300, 250, 7, 40), (129, 4000, 12, -1),
    (3000, 2500, 12, -1), (4097, 4031, 12, -1),
])
def test_checkpoint_equals_full_store(ctx, nq, nr, dim, band):
    rng = np.random.default_rng(nq * 7 + nr)
    q = rng.random((nq, dim))
    r = np.concatenate([q, q])[:nr] + 0.05 * rng.random((nr, dim)) if nr <= 2 * nq else rng.random((nr, dim))
    _check(ctx, q, r, band)


@pytest.mark.parametrize("kind", ["nan", "inf", "ninf"])
def test_checkpoint_nonfinite_inputs(ctx, kind):
    rng = np.random.default_rng(3)
    q, r = rng.random((300, 12)), rng.random((280, 12))
    v = {"nan": np.nan, "inf": np.inf, "ninf": -np.inf}[kind]
    q[17, 3] = v
    r[100:103, 0] = v
    r[0, 5] = v                         # a non-finite first column: paths along the border
    _check(ctx, q, r)


def test_checkpoint_matches_oracle(ctx):
    """The checkpoint path against the oracle directly (path, costs, distance)."""
    rng = np.random.default_rng(11)
    q = rng.random((700, 12))
    r = np.roll(q, 5, axis=0)[:650] + 0.01 * rng.random((650, 12))
    got = ctx.dtw(q, r)
    ref = O.dtw(q, r)
    assert np.array_equal(got["path_q"], ref["path_q"])
    assert np.array_equal(got["path_r"], ref["path_r"])
    _same(got["path_cost"], ref["path_cost"])
    _same([got["distance"]], [ref["distance"]])
