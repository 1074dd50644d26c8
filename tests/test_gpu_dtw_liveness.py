"""Liveness of the DTW band pipeline (the round-2 C5 timeouts): every wait of
the band kernels is bounded in time, the first wave that gives up writes the DTW's diagnostic
record, and the rest of the block and every band below it give up within milliseconds, so a stalled
pipeline is an error that names its cause, not a hang -- and the context stays usable.

The stall is injected (SONAR_DTW_DBG_STALL=<band>: that band's sweep stops after 1,024 steps
without publishing more), in the single-DTW path (sonar_dtw) and in the batched pair path
(sonar_align_pairs), with the retry off (the batch's own diagnosed error) and on (the pair is redone
on the single-pair path, its record flagged SONAR_PAIR_REDONE_TIMEOUT, the timeout counted)."""
import time

import numpy as np
import pytest

import oracle as O
import sonar
from sonar import synth

pytestmark = pytest.mark.gpu


def _seq(n, seed):
    return np.random.default_rng(seed).random((n, 12))


def test_injected_stall_is_a_diagnosed_error(ctx, monkeypatch):
    q, r = _seq(2000, 1), _seq(3000, 2)           # 32 bands of 64 rows
    monkeypatch.setenv("SONAR_DTW_DBG_STALL", "5")
    t0 = time.perf_counter()
    with pytest.raises(sonar.SonarError) as ei:
        ctx.dtw(q, r)
    dt = time.perf_counter() - t0
    msg = str(ei.value)
    assert "dtw band pipeline timed out" in msg and "no progress for" in msg, msg
    assert "first sentinel column" in msg, msg   # the record's E probes ran
    assert dt < 10.0, dt                          # one bound, not one per band below the stall
    assert ctx.dtw_counters(reset=True)["dtw_timeouts"] >= 1
    monkeypatch.delenv("SONAR_DTW_DBG_STALL")
    got, ref = ctx.dtw(q, r), O.dtw(q, r)           # the context is usable afterwards
    assert np.array_equal(got["path_q"], ref["path_q"]) and np.array_equal(got["path_r"], ref["path_r"])
    assert got["distance"] == ref["distance"]


def test_injected_stall_in_pair_batch_names_the_pair(ctx, monkeypatch):
    qs, rs = [], []
    for k in range(3):
        q, r, _ = synth.c5_pair(k, seconds=8.0)    # 1,374 chroma frames: 22 bands
        qs.append(q)
        rs.append(r)
    monkeypatch.setenv("SONAR_DTW_DBG_STALL", "4")
    monkeypatch.setenv("SONAR_PAIR_STREAMS", "1")
    monkeypatch.setenv("SONAR_PAIR_RETRY", "0")   # the batch's own diagnosed error, not the single-pair redo
    t0 = time.perf_counter()
    with pytest.raises(sonar.SonarError) as ei:
        ctx.align_pairs(qs, rs, max_lag_seconds=3.0, workers=8)
    dt = time.perf_counter() - t0
    msg = str(ei.value)
    assert msg.startswith("[-5] pair 0: dtw band pipeline timed out"), msg
    assert "2 more pairs failed" in msg, msg
    assert dt < 15.0, dt
    monkeypatch.delenv("SONAR_DTW_DBG_STALL")
    got = ctx.align_pairs(qs, rs, max_lag_seconds=3.0, workers=8)
    assert np.all(got["status"] == 0)


def test_injected_batch_stall_is_redone_and_flagged(ctx, monkeypatch):
    """Retry on (the default): a pair whose batched band pipeline stalls (injected into the batch
    launch only, "b<band>") is redone on the single-pair path -- status 0, the record equal to the
    unbatched path's, flagged SONAR_PAIR_REDONE_TIMEOUT -- and the timeout is counted."""
    qs, rs = [], []
    for k in range(3):
        q, r, _ = synth.c5_pair(k, seconds=8.0)
        qs.append(q)
        rs.append(r)
    monkeypatch.setenv("SONAR_PAIR_BATCH", "0")
    ref = ctx.align_pairs(qs, rs, max_lag_seconds=3.0, workers=8)
    monkeypatch.delenv("SONAR_PAIR_BATCH")
    ctx.dtw_counters(reset=True)
    monkeypatch.setenv("SONAR_DTW_DBG_STALL", "b4")
    monkeypatch.setenv("SONAR_PAIR_STREAMS", "1")
    got = ctx.align_pairs(qs, rs, max_lag_seconds=3.0, workers=8)
    monkeypatch.delenv("SONAR_DTW_DBG_STALL")
    assert np.all(got["status"] == 0)
    assert np.all(got["flags"] == sonar.PAIR_REDONE_TIMEOUT), got["flags"]
    assert ctx.dtw_counters(reset=True)["dtw_timeouts"] >= 1
    for f in sonar.PAIR_FIELDS:
        a, b = np.asarray(got[f], float), np.asarray(ref[f], float)
        assert np.array_equal(a, b, equal_nan=True), f
