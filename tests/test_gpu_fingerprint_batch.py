"""sonar_fingerprint_batch -- SpectralAnalyzer.ComputeSTFTBatch (fingerprint/analyzers/spectral.go:234-285):
ComputeSTFTWithWindow over many signals with one configuration.

The f32 MFCC configuration at W = 1024 runs every signal's frame pairs in one mfcc_pair_kernel
launch (a segment table; a wave's pair range crosses signal boundaries), so each signal's rows must
equal what sonar_fingerprint returns for that signal alone -- bit for bit, since every frame runs
the same arithmetic.  Other configurations run the per-signal path.  Errors follow the Go entry:
"no signals provided" for an empty batch, "error processing signal i: <ComputeSTFTWithWindow's
error>" for the first failing signal (spectral.go:235-237, :276-281)."""
import numpy as np
import pytest
import torch  # before the library loads HIP (one HIP runtime in the process, as in test_gpu_ingest)

import oracle as O
import sonar
from parity import assert_mfcc

pytestmark = pytest.mark.gpu


def _cfg(ctx, **kw):
    base = dict(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13,
                precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    base.update(kw)
    return ctx.config(**base)


def _signals(seed, lengths):
    rng = np.random.default_rng(seed)
    out = []
    for n in lengths:
        t = np.arange(n) / 44100.0
        x = 0.4 * np.sin(2 * np.pi * rng.uniform(80, 4000) * t) + 0.05 * rng.standard_normal(n)
        out.append(x.astype(np.float32))
    return out


def _singles(ctx, sigs, cfg):
    return [ctx.fingerprint(x, cfg)["mfcc"] for x in sigs]


# F = 1, 2, 3 (odd: the last pair's second frame is past the signal), 8, then longer ones
EDGE_LENGTHS = [1024, 1280, 1536, 1024 + 7 * 256, 1024 + 7 * 256 + 255, 5000, 44100, 3 * 44100 + 17,
                88200, 1100, 200_003, 1024 + 2 * 256]


def test_batch_equals_single_calls(ctx):
    cfg = _cfg(ctx)
    sigs = _signals(1, EDGE_LENGTHS)
    got = ctx.fingerprint_batch(sigs, cfg)
    assert ctx.last_fp_kernel() == "mfcc_pair_kernel"
    ref = _singles(ctx, sigs, cfg)
    assert len(got) == len(sigs)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g["mfcc"].shape == r.shape, i
        assert np.array_equal(g["mfcc"], r), f"signal {i} (n={len(sigs[i])})"


def test_many_short_signals_cross_wave_boundaries(ctx):
    """300 signals of 1 to ~80 frames: the waves' pair ranges start and end inside signals."""
    rng = np.random.default_rng(7)
    lengths = [int(1024 + 256 * rng.integers(0, 80) + rng.integers(0, 256)) for _ in range(300)]
    cfg = _cfg(ctx)
    sigs = _signals(2, lengths)
    got = ctx.fingerprint_batch(sigs, cfg)
    ref = _singles(ctx, sigs, cfg)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert np.array_equal(g["mfcc"], r), f"signal {i} (n={lengths[i]})"
    again = ctx.fingerprint_batch(sigs, cfg)
    assert all(np.array_equal(a["mfcc"], b["mfcc"]) for a, b in zip(got, again)), "nondeterministic"


def test_batch_against_oracle(ctx):
    cfg = _cfg(ctx)
    sigs = _signals(3, [44100, 1536, 30000])
    got = ctx.fingerprint_batch(sigs, cfg)
    for g, x in zip(got, sigs):
        mag = O.stft_mag(x.astype(np.float64), 1024, 256, nthreads=8)
        assert_mfcc(g["mfcc"].astype(np.float64), O.mfcc_frames(mag, 44100, n_coef=13, n_mels=40), 1e-4)


def test_batch_power_input(ctx):
    """MusicFeatureExtractor's |X|^2 input (F5) through the batched kernel."""
    cfg = _cfg(ctx, mfcc_input_power=1)
    sigs = _signals(4, [1536, 44100, 1024 + 256 * 9])
    got = ctx.fingerprint_batch(sigs, cfg)
    assert ctx.last_fp_kernel() == "mfcc_pair_kernel"
    for g, r in zip(got, _singles(ctx, sigs, cfg)):
        assert np.array_equal(g["mfcc"], r)


def test_batch_other_configurations_per_signal(ctx):
    """Configurations off the one-launch path (f64 output, magnitude, another W) equal per-signal calls."""
    sigs = _signals(5, [2048, 44100, 1536 + 100])
    for kw in [dict(out_dtype=sonar.F64), dict(flags=sonar.FP_MFCC | sonar.FP_MAGNITUDE),
               dict(window_size=512, hop_size=128), dict(precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64)]:
        cfg = _cfg(ctx, **kw)
        got = ctx.fingerprint_batch(sigs, cfg)
        for g, x in zip(got, sigs):
            r = ctx.fingerprint(x, cfg)
            assert g.keys() == r.keys()
            for k in r:
                assert np.array_equal(g[k], r[k]), (kw, k)


def test_batch_device_pointers(ctx):
    cfg = _cfg(ctx)
    sigs = _signals(6, [1536, 44100, 5000, 1024])
    dev = [torch.from_numpy(x).cuda() for x in sigs]
    F = [sonar.stft_frames(len(x), 1024, 256) for x in sigs]
    outs = [torch.zeros((f, 13), dtype=torch.float32, device="cuda") for f in F]
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        ctx.fingerprint_batch_device([t.data_ptr() for t in dev], [len(x) for x in sigs],
                                     [o.data_ptr() for o in outs], cfg)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    host = ctx.fingerprint_batch(sigs, cfg)
    for o, h in zip(outs, host):
        assert np.array_equal(o.cpu().numpy(), h["mfcc"])


def test_batch_errors(ctx):
    cfg = _cfg(ctx)
    with pytest.raises(sonar.SonarError) as e:
        ctx.fingerprint_batch([], cfg)
    assert e.value.code == sonar.ERR_EMPTY and e.value.msg == "no signals provided"
    # signal 3: (700 - 1024) / 256 + 1 = 0 frames (Go truncating division; 1000 samples would give 1)
    sigs = _signals(8, [2048, 4096, 3000, 700, 5000])
    with pytest.raises(sonar.SonarError) as e:
        ctx.fingerprint_batch(sigs, cfg)
    assert e.value.code == sonar.ERR_TOO_SHORT
    assert e.value.msg == "error processing signal 3: signal too short for given window size and hop size"
    sigs[1] = np.zeros(0, np.float32)
    with pytest.raises(sonar.SonarError) as e:
        ctx.fingerprint_batch(sigs, cfg)
    assert e.value.code == sonar.ERR_EMPTY and e.value.msg == "error processing signal 1: empty signal"
    with pytest.raises(sonar.SonarError) as e:
        ctx.fingerprint_batch(_signals(9, [2048]), _cfg(ctx, hop_size=0))
    assert e.value.msg == "error processing signal 0: hop size must be positive"
