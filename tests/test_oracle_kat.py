"""CPU: the oracle against analytic known answers and numpy.
The Go reference has no tests/fixtures and cannot run here (no Go toolchain), so
these KATs + numpy are what pin the oracle ("parity unpinned" w.r.t. Go)."""
import numpy as np
import pytest

import oracle as O
from sonar import synth


def test_fft_matches_numpy():
    rng = np.random.default_rng(0)
    for n in (8, 256, 1024, 2048, 255, 1000, 441):
        x = rng.standard_normal(n)
        assert np.max(np.abs(O.fft(x) - np.fft.fft(x))) < 1e-10 * n


def test_hann_normalisation_factor():
    w = O.window("hann", 1024)
    raw = 0.5 * (1 - np.cos(2 * np.pi * np.arange(1024) / 1023))
    assert w[512] / raw[512] == pytest.approx(1.6337911062772983, rel=1e-12)
    assert np.mean(w ** 2) == pytest.approx(1.0, rel=1e-12)    # unit power gain (windowing.go:427-437)


def test_stft_kaiser_and_tukey_windows_are_rectangular():
    """F16: ComputeSTFTWithWindow's WindowConfig literal (spectral.go:415-420) sets only Type, Size,
    Normalize and Symmetric, so Beta and Alpha are Go's zero values, not DefaultWindowConfig's 8.6 /
    0.5 (windowing.go:66-73): Kaiser = I0(0 * ...)/I0(0) = 1, Tukey taper int(0 * N / 2) = 0 -- the STFT
    of either equals the rectangular one exactly.  The parameterised windows themselves still follow
    windowing.go:304-340."""
    x = np.random.default_rng(4).standard_normal(1024 * 6)
    rect = O.stft_mag(x, 1024, 256, window_type="rectangular")
    for kind in ("kaiser", "tukey"):
        assert np.array_equal(O.stft_mag(x, 1024, 256, window_type=kind), rect), kind
    assert not np.allclose(O.window("kaiser", 64, beta=8.6), O.window("rectangular", 64))
    assert np.array_equal(O.window("kaiser", 64, beta=0.0), O.window("rectangular", 64))
    assert np.array_equal(O.window("tukey", 64, alpha=0.0), O.window("rectangular", 64))


def test_mel_bin_points_and_nnz():
    fb = O.filterbank(26, 1024, 44100, 0, 22050)
    assert np.count_nonzero(fb) == 933
    assert np.count_nonzero(O.filterbank(40, 1024, 44100, 0, 22050)) == 940
    # integer bin points [0,2,5,8,11,15,19,24,...,392,449,512]: peak (weight 1) positions
    peaks = [int(np.argmax(r)) for r in fb]
    assert peaks[:6] == [2, 5, 8, 11, 15, 19] and peaks[-1] == 449


def test_frame_count_10s():
    assert O.stft_frames(441000, 1024, 256) == 1719
    assert O.stft_frames(158_760_000, 1024, 256) == 620_153
    assert O.stft_frames(13_230_000, 1024, 256) == 51_676
    assert O.stft_frames(28_800_000, 512, 128) == 224_997


def test_sample_rate_zero_mfcc_constant():
    mag = O.stft_mag(synth.sweep(1.0), 1024, 256)
    m = O.mfcc_frames(mag, 0)
    assert np.allclose(m[:, 0], -117.409263, atol=1e-6)
    assert np.abs(m[:, 1:]).max() < 1e-12


def test_bin_centred_sine_energy_concentration():
    k, W = 40, 1024
    x = np.sin(2 * np.pi * k * np.arange(W * 4) / W)
    mag = O.stft_mag(x, W, 256)
    e = mag ** 2
    assert np.all(e[:, k - 1:k + 2].sum(1) / e.sum(1) > 0.99)


def test_ncc_delay_kat():
    rng = np.random.default_rng(1)
    s = np.convolve(rng.standard_normal(3000), np.ones(7), "same")
    d = 25
    corr, met = O.ncc(s[:2000], s[d:2000 + d] if False else np.concatenate([np.zeros(d), s[:2000 - d]]), 100)
    assert met["peak_lag"] == d


def test_dtw_identical_is_diagonal():
    q = np.random.default_rng(2).random((50, 3))
    r = O.dtw(q, q)
    assert r["distance"] == 0.0
    assert np.array_equal(r["path_q"], np.arange(50)) and np.array_equal(r["path_r"], np.arange(50))


def test_chroma_a440_bin9():
    # with a fine frame (fs = 8192 -> 5.4 Hz bins) 440 Hz folds to pitch class 9 (A);
    # the music extractor's own frames are ~hop long (F6), far too coarse for this KAT
    t = np.arange(8192 * 10) / 44100
    x = np.sin(2 * np.pi * 440 * t)
    c = O.chroma_frames(x, 10, 4096, 8192, 44100)
    assert np.all(np.argmax(c[:-2], axis=1) == 9)


def test_yin_finds_220hz():
    sr = 16000
    t = np.arange(1024) / sr
    p, c, tau = O.yin_raw(np.sin(2 * np.pi * 220 * t), sr)
    assert abs(p - 220) < 2 and c > 0.5


def test_autocorr_fft_matches_direct_sums():
    """The oracle's restatement of CrossCorrelation.computeFFT (recursive radix-2, z-scored,
    stats/correlation.go:231-297, 726-774) equals the direct lag sums it stands for."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal(2048) * np.hanning(2048) + 0.3
    z = (x - x.mean()) / x.std()
    got = O.autocorr_fft(x, 1024)
    full = np.correlate(z, z, mode="full")                    # lags -(n-1) .. n-1
    ref = full[2047 - 1024: 2047 + 1025]
    assert got.shape == (2049,)
    assert np.max(np.abs(got - ref)) < 1e-10 * np.max(np.abs(ref))


def test_formant_frame_structure():
    """AnalyzeFormants invariants: <= 4 ascending formants >= 200 Hz apart inside [50, sr/2],
    bandwidth clamp [50, 500], VTL default 17.5, too-short frames rejected (format.go:85-411)."""
    from sonar import synth
    x = synth.c4_speech(seconds=4.0, sr=16000)
    r = O.formant_frames(x, 16000)
    assert len(r["status"]) == (len(x) - 2048 - 1) // 1024 + 1
    for k in range(len(r["status"])):
        n = r["n_formants"][k]
        f = r["frequency"][k][:n]
        assert n <= 4 and np.all(np.diff(f) >= 200.0) and np.all((f >= 50) & (f <= 8000))
        assert np.all((r["bandwidth"][k][:n] >= 50) & (r["bandwidth"][k][:n] <= 500))
        if n == 0 and r["status"][k] == 0:
            assert r["vocal_tract_length"][k] == 17.5 and r["quality"][k] == 0.0
    short = O.formant_frame(x[:2000], 16000)
    assert short["status"][0] == 1
    silent = O.formant_frame(np.zeros(4096), 16000)
    assert silent["status"][0] == 3                               # "zero energy signal"


def test_voice_quality_kat():
    """AnalyzeVoiceQuality (voice_quality.go:56-111): a steady 200 Hz harmonic tone gives
    periods of int(16000 / f0) = 79..80 samples, zero jitter and F0 near 200 Hz; errors for
    < 1 s (:57) and for noise without pitch periods (:67)."""
    sr = 16000
    t = np.arange(2 * sr) / sr
    x = np.sin(2 * np.pi * 200 * t) + 0.3 * np.sin(2 * np.pi * 400 * t)
    vq, st = O.voice_quality(x, sr)
    assert st == 0 and vq["num_periods"] > 100
    assert abs(vq["mean_f0"] - 200) < 1 and vq["jitter"] == 0.0 and vq["f0_stability"] > 0.99
    assert vq["hnr"] > 20 and 0.9 < vq["overall_quality"] <= 1.0
    assert O.voice_quality(x[: sr - 1], sr)[1] == -1
    assert O.voice_quality(np.random.default_rng(0).standard_normal(2 * sr), sr)[1] == -2
    v, st = O.voice_quality(O.preemphasis(synth.voiced(), 0.97), sr)
    assert st == 0 and v["jitter"] > 0 and v["shimmer"] > 0 and abs(v["mean_f0"] - 140) < 5


def test_alignment_consistency_and_truncate_kat():
    """AnalyzeAlignmentConsistency (stats/alignment.go:709-800): the perturbation is deterministic,
    so all trials agree (std 0, range 0, consistency 1) and a 9-frame shift is found by NCC (x hop)
    and by the DTW mean offset; TruncateToAlignmentPCM (extractors/alignment.go:223-297) index rules."""
    rng = np.random.default_rng(4)
    base = np.abs(np.convolve(rng.standard_normal(700), np.ones(9) / 9, mode="same"))[:, None] * \
        (1 + rng.random((700, 3)))
    q, r = base[9:609], base[:600]
    st = O.alignment_consistency_reference(q, r, 44100, O.ALIGN_XCORR, 50, 256, num_trials=4)
    assert st["trials"] == 4 and abs(st["offset"]) == 9 * 256
    assert st["stddev_offset"] == 0.0 and st["offset_range"] == 0.0 and st["consistency"] == 1.0
    assert st["mean_offset"] == st["median_offset"] == st["offset"]
    assert O.alignment_consistency_reference(q, r, 44100, O.ALIGN_XCORR, 50, 256, num_trials=1)["trials"] == 5
    d = O.alignment_consistency_reference(q, r, 44100, O.ALIGN_DTW, 50, 256)
    assert abs(d["offset"]) <= 9
    with pytest.raises(ValueError, match="no successful alignments"):
        O.alignment_consistency_reference(q, r, 44100, O.ALIGN_PHASE, 50, 256)
    assert O.truncate_to_alignment_reference(44100 * 10, 44100 * 10, 44100, 2.0) == (22050, 88200 + 22050,
                                                                                      441000 - 88200 - 44100)
    assert O.truncate_to_alignment_reference(1000, 1000, 44100, 0.0) == (0, 0, 1000)      # no padding room
    with pytest.raises(ValueError, match="offset too large"):
        O.truncate_to_alignment_reference(1000, 1000, 44100, -1.0)


def test_bytes_to_float64_kat():
    """Decoder.bytesToFloat64 (decoder.go:850-871): little-endian IEEE doubles, ragged tail trimmed."""
    import oracle as O
    data = bytes([0, 0, 0, 0, 0, 0, 0xF0, 0x3F,          # 1.0
                  0, 0, 0, 0, 0, 0, 0, 0xC0,             # -2.0
                  0x18, 0x2D, 0x44, 0x54, 0xFB, 0x21, 0x09, 0x40,   # pi
                  1, 2, 3])                              # 3 trailing bytes: dropped
    got = O.bytes_to_float64(data)
    assert got.tolist() == [1.0, -2.0, 3.141592653589793]
    assert O.bytes_to_float64(b"") is None and O.bytes_to_float64(b"\x00" * 7) is None


def test_spectral_contrast_known_answers():
    """SpectralContrast (spectral_contrast.go:26-185): a flat spectrum has 0 dB in every band; a band
    whose top 20 % of power sits 100x above the rest reads 20 dB; sr = 0 puts the six bands on
    bins [0,1), [1,2), ... (Go's int(+Inf) -> MinInt64 -> 0, then the monotonic fix-up)."""
    K = 513
    flat = np.ones((2, K))
    assert np.allclose(O.spectral_contrast(flat, 44100), 0.0, atol=0)
    mag = np.ones((1, K))
    c0 = O.spectral_contrast(mag, 44100)
    # band 5 = bins [234, 512): 278 values, top int(0.2 * 278) = 55 of them at power 100
    mag[0, 512 - 55:512] = 10.0
    c = O.spectral_contrast(mag, 44100)
    assert c[0, 5] == pytest.approx(20.0, abs=1e-12) and np.array_equal(c[0, :5], c0[0, :5])
    z = np.abs(np.random.default_rng(0).standard_normal((3, K))) + 0.1
    cz = O.spectral_contrast(z, 0)
    # bands of one bin each: bottom and top 20 % are that bin -> 0 dB
    assert np.allclose(cz, 0.0, atol=1e-12)
