"""The batched pair path of sonar_align_pairs (one band-kernel launch over a batch's chroma DTWs,
batched walk / path decode, one host sync per batch) against the unbatched path
(SONAR_PAIR_BATCH=0: one sonar_align_pair_device per pair).  Pairs are independent and both paths
run the same arithmetic, so records must be identical (NaN-aware), for pairs of different lengths,
any batch cut, and a pair whose chroma is not finite (the batch redoes it through the exact
math.Min path and flags the record SONAR_PAIR_REDONE_NONFINITE).  Every batched run here also
checks that no band pipeline timed out (the retry would hide it)."""
import numpy as np
import pytest
import torch  # noqa: F401 -- before the library loads HIP (one HIP runtime in the process)

import sonar
from sonar import synth

pytestmark = pytest.mark.gpu


def _same(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return a.shape == b.shape and np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
        np.nan_to_num(a), np.nan_to_num(b))


@pytest.fixture(scope="module")
def mixed_pairs():
    rng = np.random.default_rng(11)
    qs, rs = [], []
    for k, (sq, sr_) in enumerate([(6.0, 7.5), (9.0, 5.0), (3.3, 3.3), (12.0, 10.7), (4.1, 8.9)]):
        q, r = synth.c3_pair(max(sq, sr_), 0.4 + 0.3 * k)[:2]
        qs.append(np.ascontiguousarray(q[: int(sq * 44100)]))
        rs.append(np.ascontiguousarray(r[: int(sr_ * 44100)] + 1e-3 * rng.standard_normal(int(sr_ * 44100))))
    return qs, rs


def _run(ctx, monkeypatch, qs, rs, **env):
    env.setdefault("SONAR_PAIR_RETRY", 0)     # a timed-out pipeline is an error here, never a silent redo
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    try:
        ctx.dtw_counters(reset=True)
        out = ctx.align_pairs(qs, rs, max_lag_seconds=4.0, workers=4)
        assert ctx.dtw_counters(reset=True)["dtw_timeouts"] == 0
        return out
    finally:
        for k in env:
            monkeypatch.delenv(k)


@pytest.mark.parametrize("streams", [1, 2, 3])
def test_batched_equals_unbatched_mixed_lengths(ctx, monkeypatch, mixed_pairs, streams):
    qs, rs = mixed_pairs
    ref = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_BATCH=0)
    got = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=streams)
    assert np.all(ref["status"] == 0) and np.all(got["status"] == 0)
    for f in sonar.PAIR_FIELDS:
        assert _same(got[f], ref[f]), f


def test_batched_memory_budget_cut(ctx, monkeypatch, mixed_pairs):
    """A tiny device budget forces one pair per batch: same records."""
    qs, rs = mixed_pairs
    ref = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_BATCH=0)
    got = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=1, SONAR_PAIR_BATCH_GB=0.001)
    for f in sonar.PAIR_FIELDS:
        assert _same(got[f], ref[f]), f


def test_batched_nonfinite_pair_redone_exactly(ctx, monkeypatch, mixed_pairs):
    qs, rs = [x.copy() for x in mixed_pairs[0]], [x.copy() for x in mixed_pairs[1]]
    qs[1][5000] = np.nan                      # chroma frames around it become NaN
    rs[3][7000] = np.inf
    ref = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_BATCH=0)
    got = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=2)
    assert np.array_equal(got["status"], ref["status"])
    for f in sonar.PAIR_FIELDS:
        assert _same(got[f], ref[f]), f
    flagged = np.nonzero(got["flags"])[0].tolist()
    assert flagged == [1, 3], flagged
    assert np.all(got["flags"][[1, 3]] == sonar.PAIR_REDONE_NONFINITE)


def test_trim_releases_and_reallocates(ctx, monkeypatch, mixed_pairs):
    """sonar_trim frees the cached buffers of the context and its pair workers; the next call
    allocates again and gives the same records."""
    qs, rs = mixed_pairs
    ref = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=2)
    ctx.trim()
    got = _run(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=2)
    for f in sonar.PAIR_FIELDS:
        assert _same(got[f], ref[f]), f


@pytest.fixture(scope="module")
def device_pairs():
    """Device-resident pairs of 5-12 s (chroma frames of 256 samples: the batched feature launches
    take the whole batch), plus the same with one 3.3 s pair (257-sample frames: per-pair path)."""
    rng = np.random.default_rng(12)
    qs, rs = [], []
    for k, (sq, sr_) in enumerate([(6.0, 7.5), (9.0, 5.0), (12.0, 10.7), (5.5, 8.9), (7.0, 7.0), (3.3, 3.3)]):
        q, r = synth.c3_pair(max(sq, sr_), 0.4 + 0.3 * k)[:2]
        qs.append(torch.from_numpy(np.ascontiguousarray(q[: int(sq * 44100)])).cuda())
        rs.append(torch.from_numpy(np.ascontiguousarray(r[: int(sr_ * 44100)] +
                                                        1e-3 * rng.standard_normal(int(sr_ * 44100)))).cuda())
    torch.cuda.synchronize()
    return qs, rs


def _run_dev(ctx, monkeypatch, qs, rs, **env):
    env.setdefault("SONAR_PAIR_RETRY", 0)
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    try:
        ctx.dtw_counters(reset=True)
        out = ctx.align_pairs([q.data_ptr() for q in qs], [r.data_ptr() for r in rs],
                              nq=[q.numel() for q in qs], nr=[r.numel() for r in rs], max_lag_seconds=4.0,
                              workers=8, device_ptrs=True)
        assert ctx.dtw_counters(reset=True)["dtw_timeouts"] == 0
        assert np.all(out["flags"] == 0)
        return out
    finally:
        for k in env:
            monkeypatch.delenv(k)


@pytest.mark.parametrize("with_short", [False, True])
@pytest.mark.parametrize("streams", [1, 2])
def test_batched_features_equal_per_pair(ctx, monkeypatch, device_pairs, streams, with_short):
    """Device-resident pairs: the batch's music features and NCCs in batched launches (default)
    against the per-pair launches inside a batch (SONAR_FEAT_BATCH=0) and the unbatched path
    (SONAR_PAIR_BATCH=0): identical records.  with_short adds a pair whose chroma frames are 257
    samples, so its batch falls back to the per-pair launches."""
    qs, rs = device_pairs
    if not with_short:
        qs, rs = qs[:-1], rs[:-1]
    ref = _run_dev(ctx, monkeypatch, qs, rs, SONAR_PAIR_BATCH=0)
    per = _run_dev(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=streams, SONAR_FEAT_BATCH=0)
    got = _run_dev(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=streams)
    assert np.all(ref["status"] == 0) and np.all(got["status"] == 0) and np.all(per["status"] == 0)
    for f in sonar.PAIR_FIELDS:
        assert _same(got[f], ref[f]), f
        assert _same(per[f], ref[f]), f


@pytest.mark.parametrize("streams", [1, 3])
def test_device_scorer_equals_host_scorer(ctx, monkeypatch, device_pairs, streams):
    """The batch's scorer reductions on the device (pair_score_kernel: path sums, correlation
    peak / noise / sidelobes in Go's order) against the same batch scored on the host from the
    copied-back paths and correlations (SONAR_PAIR_HOST_SCORES=1): identical records, bit for bit."""
    qs, rs = device_pairs
    qs, rs = qs[:-1], rs[:-1]
    host = _run_dev(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=streams, SONAR_PAIR_HOST_SCORES=1)
    dev = _run_dev(ctx, monkeypatch, qs, rs, SONAR_PAIR_STREAMS=streams)
    assert np.all(host["status"] == 0) and np.all(dev["status"] == 0)
    for f in sonar.PAIR_FIELDS:
        assert _same(dev[f], host[f]), f


def test_device_scorer_edge_pairs(ctx, monkeypatch):
    """Device vs host scorer on pairs whose paths and correlations are degenerate: identical
    streams (a pure diagonal, a correlation peak at lag 0), a silent query (an all-zero energy
    correlation: no peak beyond index 0, zero sidelobes), a constant tone against itself shifted,
    and the shortest streams the batch takes (paths of a few points)."""
    rng = np.random.default_rng(21)
    base, _ = synth.c3_pair(6.0, 0.7)[:2]
    tone = (0.3 * np.sin(2 * np.pi * 440.0 * np.arange(int(5.0 * 44100)) / 44100.0)).astype(np.float64)
    short = 0.2 * rng.standard_normal(1024 + 256 * 9)
    qs = [base[: 5 * 44100], np.zeros(5 * 44100), tone, short, base[: 6 * 44100]]
    rs = [base[: 5 * 44100].copy(), base[: 5 * 44100], np.roll(tone, 1234), short[::-1].copy(),
          base[44100: 6 * 44100] + 1e-3 * rng.standard_normal(5 * 44100)]
    qd = [torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda() for x in qs]
    rd = [torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda() for x in rs]
    torch.cuda.synchronize()

    def run(**env):
        env.setdefault("SONAR_PAIR_RETRY", 0)
        for k, v in env.items():
            monkeypatch.setenv(k, str(v))
        try:
            return ctx.align_pairs([q.data_ptr() for q in qd], [r.data_ptr() for r in rd],
                                   nq=[q.numel() for q in qd], nr=[r.numel() for r in rd],
                                   max_lag_seconds=2.0, workers=8, device_ptrs=True)
        finally:
            for k in env:
                monkeypatch.delenv(k)

    host = run(SONAR_PAIR_HOST_SCORES=1, SONAR_PAIR_STREAMS=1)
    dev = run(SONAR_PAIR_STREAMS=1)
    assert np.array_equal(host["status"], dev["status"])
    for f in sonar.PAIR_FIELDS:
        assert _same(dev[f], host[f]), f
