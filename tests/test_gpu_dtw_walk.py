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
