"""sonar_ingest_f64le (the decoder's f64le byte stream, transcode/decoder.go:850-871)
against the oracle's bytesToFloat64.  Integer/byte work: bit-exact, f64 kept as-is, f32 = round to
nearest even (Go float32(x), numpy astype) in both conversion modes; NaNs compared by position."""
import numpy as np
import pytest
import torch

import oracle as O
import sonar

pytestmark = pytest.mark.gpu

MODES = [sonar.INGEST_DEVICE_CONVERT, sonar.INGEST_HOST_CONVERT]


def _specials():
    f32 = np.finfo(np.float32)
    return np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 1e-40, -1e-42, 1.4e-45, 7e-46, 1e-300,
                     3.4028235677973366e38, 3.5e38, -1e39, float(f32.max), float(f32.tiny), 0.1, 1 / 3,
                     1.0000000596046448, 1.0000001788139343], np.float64)


def _signal(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n) * 0.3
    sp = _specials()
    x[rng.integers(0, n, size=min(n, 64))] = rng.choice(sp, size=min(n, 64))
    x[: min(n, len(sp))] = sp[: min(n, len(sp))]
    return x


def _ingest(ctx, data, out_dtype, mode, threads=0):
    n = ctx.ingest_f64le(data, None)
    t = torch.empty(n, dtype=torch.float32 if out_dtype == sonar.F32 else torch.float64, device="cuda:0")
    assert ctx.ingest_f64le(data, t.data_ptr(), out_dtype, mode, threads) == n
    ctx.synchronize()
    return t.cpu().numpy()


def _same(got, want):
    assert got.shape == want.shape
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan)
    ui = np.uint32 if got.dtype == np.float32 else np.uint64
    assert np.array_equal(got[~nan].view(ui), want[~nan].view(ui))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("out_dtype", [sonar.F32, sonar.F64])
@pytest.mark.parametrize("n,tail", [(1, 0), (3, 5), (1027, 7), (9_000_003, 3), (21_000_001, 0)])
def test_ingest_matches_bytes_to_float64(ctx, mode, out_dtype, n, tail):
    x = _signal(n, n)
    data = x.astype("<f8").tobytes() + bytes(range(tail))
    want = O.bytes_to_float64(data) if n < 100_000 else np.frombuffer(data[: 8 * n], "<f8")
    if n < 100_000:
        assert np.array_equal(want.view(np.uint64), x.view(np.uint64))
    want = want.astype(np.float32) if out_dtype == sonar.F32 else want
    _same(_ingest(ctx, data, out_dtype, mode), want)


@pytest.mark.parametrize("threads", [1, 5])
def test_ingest_unaligned_source_and_thread_counts(ctx, threads):
    x = _signal(5_000_011, 3)
    raw = bytearray(3) + bytearray(x.astype("<f8").tobytes())
    view = memoryview(raw)[3:]
    for mode in MODES:
        _same(_ingest(ctx, view, sonar.F32, mode, threads), x.astype(np.float32))


@pytest.mark.parametrize("nbytes", [0, 1, 7])
def test_ingest_empty(ctx, nbytes):
    with pytest.raises(sonar.SonarError) as e:
        ctx.ingest_f64le(bytes(nbytes), None)
    assert e.value.code == sonar.ERR_EMPTY and "no audio samples decoded" in e.value.msg
    assert O.bytes_to_float64(bytes(nbytes)) is None


def test_ingest_then_fingerprint(ctx):
    """f64le bytes -> device f32 -> fused MFCC equals the host-f32 entry on the same samples."""
    n = 44100 * 20 + 123
    x = (0.5 * np.sin(np.arange(n) * 0.01) + 0.05 * np.random.default_rng(5).standard_normal(n))
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    want = ctx.fingerprint(x.astype(np.float32), cfg)["mfcc"]
    for mode in MODES:
        pcm = torch.empty(n, dtype=torch.float32, device="cuda:0")
        assert ctx.ingest_f64le(x.astype("<f8").tobytes(), pcm.data_ptr(), sonar.F32, mode) == n
        out = torch.empty(want.shape, dtype=torch.float32, device="cuda:0")
        ctx.fingerprint_device(pcm.data_ptr(), n, cfg, mfcc=out.data_ptr())
        ctx.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("mode", MODES)
def test_fingerprint_f64le_matches_host_entry(ctx, mode):
    """One call from decoder bytes to MFCC + descriptors equals sonar_fingerprint on the f32 samples."""
    n = 44100 * 7 + 77
    x = np.sin(np.arange(n) * 0.003) * 0.4 + 0.05 * np.random.default_rng(11).standard_normal(n)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32,
                     flags=sonar.FP_MFCC | sonar.FP_SPECTRAL | sonar.FP_ZCR | sonar.FP_ENERGY,
                     energy_window=1024, energy_hop=256)
    want = ctx.fingerprint(x.astype(np.float32), cfg)
    got = ctx.fingerprint_f64le(x.astype("<f8").tobytes() + b"\x01\x02", cfg, mode)
    assert set(got) == set(want)
    for k in want:
        assert np.array_equal(got[k], want[k], equal_nan=True), k


@pytest.mark.parametrize("mode", MODES)
def test_fingerprint_f64le_default_cfg_keeps_f64(ctx, mode):
    """The default cfg (pcm_dtype F64, precision F64) stays float64 end to end: the result equals
    sonar_fingerprint on the float64 samples, not on float32-rounded ones (Go's []float64)."""
    n = 44100 * 3 + 5
    x = np.sin(np.arange(n) * 0.0031) * 0.4 + 0.05 * np.random.default_rng(12).standard_normal(n)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100,
                     flags=sonar.FP_MFCC | sonar.FP_SPECTRAL | sonar.FP_ZCR | sonar.FP_ENERGY,
                     energy_window=1024, energy_hop=256)
    want = ctx.fingerprint(x, cfg)
    got = ctx.fingerprint_f64le(x.astype("<f8").tobytes(), cfg, mode)
    assert set(got) == set(want)
    for k in want:
        assert np.array_equal(got[k], want[k], equal_nan=True), k
    rounded = ctx.fingerprint(x.astype(np.float32).astype(np.float64), cfg)
    assert not np.array_equal(got["energy"], rounded["energy"])


def test_fingerprint_f64le_errors(ctx):
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, precision=sonar.F32,
                     pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    for data, code, msg in ((b"\x00" * 5, sonar.ERR_EMPTY, "no audio samples decoded"),
                            (np.zeros(100).tobytes(), sonar._abi.ERR_TOO_SHORT, "signal too short")):
        with pytest.raises(sonar.SonarError) as e:
            ctx.fingerprint_f64le(data, cfg)
        assert e.value.code == code and msg in e.value.msg
