"""The DTW backtrack walk's code stream at block edges.  The walk stores its 2-bit moves 16 per
word and 64 words (1,024 moves) per flush; paths whose length ends a 64-word block with a
partly filled last word (P % 1024 in 1009..1023), ends it exactly, or spills one move past it
are compared with the oracle (path, costs, distance bit-exact).  An earlier walk left the whole
last block unstored when P % 16 != 0 and ceil(P / 16) % 64 == 0."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1009, 1015, 1023, 1024, 1025, 2047, 2048, 2049, 3071, 3073])
def test_walk_block_edges_diagonal(ctx, n):
    """Identical sequences: the path is the diagonal, P = n."""
    rng = np.random.default_rng(n)
    q = rng.random((n, 12))
    got = ctx.dtw(q, q.copy())
    assert len(got["path_q"]) == n
    assert np.array_equal(got["path_q"], np.arange(n)) and np.array_equal(got["path_r"], np.arange(n))
    ref = O.dtw(q, q.copy())
    assert got["distance"] == ref["distance"]
    assert np.array_equal(got["path_cost"], ref["path_cost"])


@pytest.mark.parametrize("nq,nr", [(700, 330), (1000, 17), (513, 1530), (2000, 1999)])
def test_walk_block_edges_ragged(ctx, nq, nr):
    rng = np.random.default_rng(nq * 7 + nr)
    q, r = rng.random((nq, 12)), rng.random((nr, 12))
    got, ref = ctx.dtw(q, r), O.dtw(q, r)
    assert got["distance"] == ref["distance"]
    for k in ("path_q", "path_r", "path_cost"):
        assert np.array_equal(np.asarray(got[k]), np.asarray(ref[k])), k


@pytest.mark.parametrize("nq,nr,band", [
    (1, 1, -1), (2, 40, -1), (63, 5, -1), (64, 1, -1), (65, 2, -1), (66, 300, -1), (128, 3000, -1),
    (3000, 7, -1), (1000, 1000, 30), (4033, 2900, -1), (5000, 5100, 200), (130, 5000, -1), (200, 9000, -1),
])
def test_band_walk_equals_serial_walk(ctx, nq, nr, band, monkeypatch):
    """The backtrack by bands (exit map + chain + parallel band walks) writes the same move stream
    as the one-wave serial walk (SONAR_DTW_SERIAL_WALK=1): same path, same costs."""
    rng = np.random.default_rng(nq * 31 + nr)
    q, r = rng.random((nq, 12)), rng.random((nr, 12))
    got = ctx.dtw(q, r, band=band)
    monkeypatch.setenv("SONAR_DTW_SERIAL_WALK", "1")
    ser = ctx.dtw(q, r, band=band)
    for k in ("path_q", "path_r", "path_cost"):
        assert np.array_equal(np.asarray(got[k]), np.asarray(ser[k])), k
    if nq * nr <= 2_000_000:
        ref = O.dtw(q, r, band=band) if band > 0 else O.dtw(q, r)
        assert np.array_equal(np.asarray(got["path_q"]), np.asarray(ref["path_q"]))
        assert np.array_equal(np.asarray(got["path_r"]), np.asarray(ref["path_r"]))


@pytest.mark.parametrize("kind", ["nan", "inf"])
def test_band_walk_nonfinite(ctx, kind, monkeypatch):
    """math.Min's non-finite rules steer the codes; the exit map follows the same codes."""
    rng = np.random.default_rng(5)
    q, r = rng.random((700, 12)), rng.random((650, 12))
    q[[3, 200, 420], 2] = np.nan if kind == "nan" else np.inf
    got = ctx.dtw(q, r)
    monkeypatch.setenv("SONAR_DTW_SERIAL_WALK", "1")
    ser = ctx.dtw(q, r)
    for k in ("path_q", "path_r"):
        assert np.array_equal(np.asarray(got[k]), np.asarray(ser[k])), k
