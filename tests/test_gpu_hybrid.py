"""Row a16's hybrid half on the GPU: AlignmentAnalyzer.AlignFeatures with
its three methods (algorithms/stats/alignment.go:84-106, alignWithHybrid :308-337 with the F8
result aliasing), AlignmentAnalyzer.AlignAudio (:108-126, extractEnergyFeatures :341-361) and
AlignmentExtractor.AlignAudioFiles (fingerprint/extractors/alignment.go:489-553) against the
oracle composition (oracle.analyzer_align_reference and friends).

Bit-exact: the energy frames (Go's sequential sums), every correlation, the peak lag, the DTW
path (query / reference indices and point costs) and distance.  Scalars: exact or within 1e-12
relative (host scorers in Go's order on both sides).  Both hybrid branches are exercised:
correlation confidence above 0.7 (a lagged C3 pair) and at or below it (unrelated streams),
the latter at the C3 size, 51,676 x 51,676 energy frames (d = 1)."""
import os

import numpy as np
import pytest

import oracle as O
import sonar
from sonar import synth

pytestmark = pytest.mark.gpu

ARRAYS = ("correlations", "dtw_path_query", "dtw_path_reference", "dtw_path_cost")


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _same(got, ref, rtol=1e-12):
    for k, v in ref.items():
        assert k in got, k
        g = np.asarray(got[k], np.float64).reshape(-1)
        r = np.asarray(v, np.float64).reshape(-1)
        assert g.shape == r.shape, (k, g.shape, r.shape)
        if k in ARRAYS or k in ("dtw_distance", "peak_lag", "peak_index", "offset", "dtw_ran", "method"):
            assert np.array_equal(g, r), k                       # bit-exact / integer
        else:
            both_inf = np.isinf(g) & np.isinf(r) & (np.sign(g) == np.sign(r))
            err = np.where(both_inf, 0.0, np.abs(g - r) / np.maximum(np.abs(r), 1e-300))
            ok = (err <= rtol) | (g == r) | (np.isnan(g) & np.isnan(r))
            assert ok.all(), (k, g, r)


def _noise_pair(seconds, seed):
    rng = np.random.default_rng(seed)
    n = int(seconds * 44100)
    return rng.standard_normal(n), rng.standard_normal(n)


def test_align_audio_files_xcorr_branch_c3(ctx):
    """C3 (2 x 5 min, lag 12.34 s): the energy correlation is confident (> 0.7), so the hybrid
    returns the correlation result; the peak lands at +2,126 frames."""
    q, r = synth.c3_pair(seconds=300.0, lag_s=12.34)
    got = ctx.align_audio_files(q, r, 44100, hop=256, window=1024, max_lag_seconds=60.0)
    ref = O.align_audio_files_reference(q, r, 44100, 44100, 256, 1024, 60.0)
    assert ref["dtw_ran"] == 0 and ref["confidence"] > 0.7
    assert int(np.asarray(got["peak_lag"]).reshape(-1)[0]) == 2126 and len(got["correlations"]) == 2 * 10335 + 1
    assert "dtw_path_query" not in got
    _same(got, ref)


def test_align_audio_files_dtw_branch_c3_size(ctx):
    """Two unrelated 5-min streams: the correlation confidence is <= 0.7, so the hybrid runs the
    d = 1 DTW over 51,676 x 51,676 energy frames (2.67e9 cells) and blends with F8 aliasing."""
    q, r = _noise_pair(300.0, 77)
    got = ctx.align_audio_files(q, r, 44100, hop=256, window=1024, max_lag_seconds=60.0)
    ref = O.align_audio_files_reference(q, r, 44100, 44100, 256, 1024, 60.0)
    assert ref["dtw_ran"] == 1 and ref["query_length"] == 51676 and ref["reference_length"] == 51676
    _same(got, ref)
    assert got["dtw_ran"] == 1


@pytest.mark.parametrize("method", [O.ALIGN_DTW, O.ALIGN_XCORR, O.ALIGN_HYBRID])
@pytest.mark.parametrize("dim,shift,max_lag", [(1, 0, 120), (12, 37, 120), (3, 5, 2000)])
def test_analyzer_align_features_methods(ctx, method, dim, shift, max_lag):
    rng = np.random.default_rng(100 + dim)
    n = 1500
    base = np.abs(np.convolve(rng.standard_normal(n + shift + 50), np.ones(7) / 7, mode="same"))[:, None]
    base = base * (1 + rng.random((len(base), dim)))
    q, r = base[shift:shift + n], base[:n - 3]
    got = ctx.analyzer_align_features(q, r, 44100, method=method, max_lag=max_lag, hop=256)
    ref = O.analyzer_align_reference(q, r, 44100, method, max_lag, 256)
    _same(got, ref)


def test_hybrid_both_branches_small(ctx):
    """The same analyzer on a confident pair (correlation result) and on noise (DTW branch)."""
    q, r = synth.c3_pair(seconds=30.0, lag_s=4.0)
    for a, b in ((q, r), _noise_pair(40.0, 3)):
        got = ctx.align_audio(a, b, 44100, method=O.ALIGN_HYBRID, max_lag=1000, hop=256, window=1024)
        ref = O.align_audio_reference(a, b, 44100, O.ALIGN_HYBRID, 1000, 256, 1024)
        _same(got, ref)
    assert ref["dtw_ran"] == 1


def test_align_audio_short_and_panics(ctx):
    rng = np.random.default_rng(9)
    a, b = rng.standard_normal(900), rng.standard_normal(1000)
    # (900 - 1024) / 256 truncates to 0: one frame over the whole short signal (end = len)
    got = ctx.align_audio(a, b, 44100, method=O.ALIGN_HYBRID, max_lag=100, hop=256, window=1024)
    ref = O.align_audio_reference(a, b, 44100, O.ALIGN_HYBRID, 100, 256, 1024)
    _same(got, ref)
    with pytest.raises(sonar.SonarError, match="makeslice: len out of range") as e:
        ctx.align_audio(a[:500], b, 44100, hop=256, window=1024)      # (500 - 1024) / 256 + 1 = -1
    assert e.value.code == sonar.ERR_PANIC
    with pytest.raises(sonar.SonarError, match="integer divide by zero"):
        ctx.align_audio(a, b, 44100, hop=0, window=1024)
    with pytest.raises(sonar.SonarError, match="unsupported alignment method: 2"):
        ctx.align_audio(a, b, 44100, method=O.ALIGN_PHASE, hop=256, window=1024)


def test_align_audio_files_errors(ctx):
    rng = np.random.default_rng(4)
    a = rng.standard_normal(5000)
    with pytest.raises(sonar.SonarError, match="alignment failed: empty feature sequences provided"):
        ctx.align_audio_files(a[:1000], a, 44100, hop=256, window=1024)   # ShortTimeEnergy: len < W -> empty
    with pytest.raises(sonar.SonarError, match="integer divide by zero"):
        ctx.align_audio_files(a, a, 44100, hop=0, window=1024)
    with pytest.raises(sonar.SonarError, match="empty feature sequences provided"):
        ctx.analyzer_align_features(np.zeros((0, 3)), np.ones((10, 3)), 44100)


def test_align_audio_files_device_ptrs_equal_host(ctx):
    import torch
    q, r = synth.c3_pair(seconds=20.0, lag_s=2.5)
    dq = torch.from_numpy(np.ascontiguousarray(q)).cuda()
    dr = torch.from_numpy(np.ascontiguousarray(r)).cuda()
    torch.cuda.synchronize()
    got = ctx.align_audio_files((dq.data_ptr(), len(q)), (dr.data_ptr(), len(r)), 44100, hop=256, window=1024,
                                max_lag_seconds=10.0, device_ptrs=True)
    host = ctx.align_audio_files(q, r, 44100, hop=256, window=1024, max_lag_seconds=10.0)
    assert got.keys() == host.keys()
    for k in got:
        assert np.array_equal(np.asarray(got[k]), np.asarray(host[k]), equal_nan=True), k
