"""BASELINE configs[4] (C5) at its own shape on the product's batched path: sonar_align_pairs with
its defaults -- 128 pairs in flight = 16 worker streams x batches of 8 pairs, one band-major
dtw_band_kernel<12, true, false, true> launch per batch (multi_api.cpp align_batch) -- over 128
pairs of 60 s C5 streams (seed 1000 + k, lag uniform in [0, 20) s), i.e. every
stream busy at once, as in the bench's C5 leg.

Checks (reference: fingerprint/extractors/alignment.go:139-219 -> algorithms/stats/dtw.go:55-188):
  * no band pipeline timed out (sonar_dtw_counters), over three repetitions of the whole call,
    and the three repetitions give identical records;
  * every record equals the unbatched path's (SONAR_PAIR_BATCH=0: one sonar_align_pair_device
    per pair, the single-DTW band kernel);
  * on two pairs, the batched DTW's raw outputs (SONAR_PAIR_DUMP: path, path costs, C[nq][nr])
    equal the oracle's serial DTW (oracle/dtw_oracle.c via O.dtw) of the same chroma features
    bit for bit -- a stale band edge would change C values and show here even when it does not
    stall -- and the whole record equals the oracle composition O.align_features_reference
    (integers exact, floats 1e-12)."""
import numpy as np
import pytest
import torch

import oracle as O
import sonar
from sonar import pairs

pytestmark = pytest.mark.gpu

NPAIRS = 128
SECONDS = 60.0
MAX_LAG = 20.0
SR, W, H = 44100, 1024, 256


def _same(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return a.shape == b.shape and np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
        np.nan_to_num(a), np.nan_to_num(b))


@pytest.fixture(scope="module")
def c5():
    data = [pairs.c5_pair_device(k, SECONDS, device="cuda") for k in range(NPAIRS)]
    torch.cuda.synchronize()
    return data


def _run(ctx, data, monkeypatch, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    try:
        return ctx.align_pairs([q.data_ptr() for q, _, _ in data], [r.data_ptr() for _, r, _ in data],
                               nq=[q.numel() for q, _, _ in data], nr=[r.numel() for _, r, _ in data],
                               max_lag_seconds=MAX_LAG, workers=128, device_ptrs=True)
    finally:
        for k in env:
            monkeypatch.delenv(k)


def _dump(path, k):
    with open(path / f"pair_{k}.bin", "rb") as f:
        b = f.read()
    P = int(np.frombuffer(b[:8], np.int64)[0])
    cnm = float(np.frombuffer(b[8:16], np.float64)[0])
    o = 16
    pc = np.frombuffer(b[o:o + 8 * P], np.float64)
    pq = np.frombuffer(b[o + 8 * P:o + 12 * P], np.int32)
    pr = np.frombuffer(b[o + 12 * P:o + 16 * P], np.int32)
    return P, cnm, pc, pq, pr


def test_c5_default_shape_batched(ctx, c5, monkeypatch, tmp_path):
    ctx.dtw_counters(reset=True)
    runs = [_run(ctx, c5, monkeypatch, SONAR_PAIR_DUMP=tmp_path)]
    runs += [_run(ctx, c5, monkeypatch) for _ in range(2)]
    cnt = ctx.dtw_counters(reset=True)
    assert cnt["dtw_timeouts"] == 0 and cnt["waves_timed_out"] == 0, cnt
    for got in runs:
        assert np.all(got["status"] == 0)
        for f in sonar.PAIR_FIELDS:
            assert _same(got[f], runs[0][f]), f
    ref = _run(ctx, c5, monkeypatch, SONAR_PAIR_BATCH=0)
    assert np.all(ref["status"] == 0)
    for f in sonar.PAIR_FIELDS:
        assert _same(runs[0][f], ref[f]), f
    # the injected lag is recovered by the energy NCC on (almost) every pair (bench's criterion)
    lag_frames = np.array([lag for _, _, lag in c5]) * SR / H
    pl = runs[0]["peak_lag"]
    ok = np.minimum(np.abs(pl - lag_frames), np.abs(pl + lag_frames)) <= 1.5
    assert ok.mean() >= 0.95

    for k in (0, 77):
        q, r, _ = c5[k]
        qh, rh = q.cpu().numpy(), r.cpu().numpy()
        eq, cq = ctx.music_alignment_features(qh, SR, W, H, W, H)
        er, cr = ctx.music_alignment_features(rh, SR, W, H, W, H)
        od = O.dtw(cq, cr)
        P, cnm, pc, pq, pr = _dump(tmp_path, k)
        assert P == len(od["path_q"])
        assert np.array_equal(pq, od["path_q"]) and np.array_equal(pr, od["path_r"])
        assert np.array_equal(pc, od["path_cost"])
        assert cnm / P == od["distance"]
        ref_k = O.align_features_reference(eq, er, cq, cr, len(qh), len(rh), SR, SR, H, MAX_LAG)
        assert runs[0]["peak_lag"][k] == ref_k["peak_lag"]
        assert runs[0]["method"][k] == ref_k["method"]
        assert runs[0]["dtw_distance"][k] == ref_k["dtw_distance"]
        for f in ("temporal_offset", "offset_confidence", "alignment_similarity", "alignment_quality"):
            a, b = runs[0][f][k], ref_k[f]
            assert abs(a - b) <= 1e-12 * max(1.0, abs(b)), (k, f, a, b)
