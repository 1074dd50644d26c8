"""C5 path B on the GPU: MusicFeatureExtractor energy + chroma (sonar_music_alignment_features)
against the oracle composition, and whole-pair alignment (sonar/pairs.py) recovering the
injected lag.  Energy: sequential float64 RMS in Go order -> within 1e-12 of the oracle (the DC
IIR is chunked with a warm-up on the device); chroma 1e-9 (as the chroma kernel's own test)."""
import numpy as np
import pytest
import torch

import oracle as O
import sonar
from sonar import pairs, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seconds,W,H", [(3.0, 1024, 256), (2.3, 2048, 512), (1.0, 1024, 100)])
def test_music_alignment_features_match_oracle(ctx, seconds, W, H):
    x = synth.c3_pair(seconds=seconds, lag_s=0.5)[0]
    e, c = ctx.music_alignment_features(x, 44100, W, H, W, H)
    pre = O.preemphasis(O.dc_removal(x, 0.995), 0.95)
    re_ = O.short_time_energy(pre, W, H)
    F = sonar.stft_frames(len(x), W, H)
    rc = O.chroma_music(x, F, H, 44100)
    assert e.shape == re_.shape and c.shape == rc.shape == (F, 12)
    assert np.max(np.abs(e - re_) / np.maximum(np.abs(re_), 1e-300)) < 1e-12
    assert np.max(np.abs(c - rc)) < 1e-9


def test_music_alignment_features_errors(ctx):
    with pytest.raises(sonar.SonarError, match="invalid input data"):
        ctx.music_alignment_features(np.zeros(0), 44100)
    with pytest.raises(sonar.SonarError, match="signal too short"):
        ctx.music_alignment_features(np.zeros(500), 44100)


def test_pair_alignment_matches_oracle_composition(ctx):
    """One C5 pair (20 s here, lag 3.58 s): the GPU pipeline equals the oracle composition and the
    energy cross-correlation recovers the injected lag within one hop.  max lag 6 s keeps every
    lag's overlap >= 14 s (at near-zero overlap the per-lag normalisation of correlation.go:373-409
    makes edge lags spuriously large -- reference behaviour, reproduced by the oracle as well)."""
    q, r, lag_s = synth.c5_pair(2, seconds=20.0)
    rec, got = pairs.align_pair(ctx, q, r, 44100, max_lag_seconds=6.0, lag_seconds_true=lag_s)
    pq = O.preemphasis(O.dc_removal(q, 0.995), 0.95)
    pr = O.preemphasis(O.dc_removal(r, 0.995), 0.95)
    F = sonar.stft_frames(len(q), 1024, 256)
    ref = O.align_features_reference(O.short_time_energy(pq, 1024, 256), O.short_time_energy(pr, 1024, 256),
                                     O.chroma_music(q, F, 256, 44100), O.chroma_music(r, F, 256, 44100),
                                     len(q), len(r), 44100, 44100, 256, 6.0)
    assert got["peak_lag"] == ref["peak_lag"]
    assert np.array_equal(got["dtw_path_query"], ref["dtw_path_query"])
    assert got["method"] == ref["method"]
    lag_frames = lag_s * 44100 / 256
    assert min(abs(got["peak_lag"] - lag_frames), abs(got["peak_lag"] + lag_frames)) <= 1.5
    assert abs(abs(rec[pairs.RECORD_FIELDS.index("corr_offset_seconds")]) - lag_s) <= 1.5 * 256 / 44100


def test_pair_alignment_device_inputs(ctx):
    """Device-resident pair (the bench's path): same record as the host-array path."""
    q, r, lag_s = pairs.c5_pair_device(9, seconds=12.0, device="cuda")      # lag 1.72 s
    rec_d, res_d = pairs.align_pair(ctx, q, r, 44100, max_lag_seconds=4.0, lag_seconds_true=lag_s)
    rec_h, res_h = pairs.align_pair(ctx, q.cpu().numpy(), r.cpu().numpy(), 44100, max_lag_seconds=4.0,
                                    lag_seconds_true=lag_s)
    assert np.array_equal(rec_d, rec_h, equal_nan=True)
    assert sorted(res_d) == sorted(res_h)                       # sonar_align_pair_device: same result arrays
    for k in res_h:
        assert np.array_equal(res_d[k], res_h[k], equal_nan=True), k
    lag_frames = lag_s * 44100 / 256
    pl = rec_d[pairs.RECORD_FIELDS.index("peak_lag")]
    assert min(abs(pl - lag_frames), abs(pl + lag_frames)) <= 1.5
