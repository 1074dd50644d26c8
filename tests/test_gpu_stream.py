"""STFTStreamer (SpectralAnalyzer.ComputeSTFTStreaming + ProcessChunk, fingerprint/analyzers/
spectral.go:287-374) through sonar_stft_stream_* against (1) one sonar_fingerprint call over the
whole stream with the per-frame kernel (SONAR_FP_GENERIC): rows bit-identical, whatever the
chunking; (2) a Python model of ProcessChunk's buffer arithmetic for which frames are emitted when;
(3) the oracle's STFT of those frames (magnitude 1e-11 of the frame's peak in float64, the MFCC at
the f32 / f64 tiers of tests/parity.py).  Chunk sizes split frames: 1, H - 1, W + 1, odd sizes and a
mixed random sequence."""
import numpy as np
import pytest

import oracle as O
import sonar
from parity import assert_mfcc

pytestmark = pytest.mark.gpu


def go_stream_frames(chunks, W, H):
    """ProcessChunk (spectral.go:322-366) on lengths only: the absolute start of every frame emitted by
    each push, and the buffered count afterwards."""
    base, buf, out = 0, 0, []
    for n in chunks:
        if n == 0:
            out.append([])
            continue
        buf += n
        starts = []
        while buf >= W:
            starts.append(base)
            if H >= buf:
                base += buf
                buf = 0
            else:
                base += H
                buf -= H
        out.append(starts)
    return out, buf


def _sig(n, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 44100.0
    return 0.5 * np.sin(2 * np.pi * (300 * t + 2000 * t * t)) + 0.1 * rng.standard_normal(n)


def _chunks(kind, W, H, n, seed=1):
    if kind == "mixed":
        rng = np.random.default_rng(seed)
        out = []
        while sum(out) < n:
            out.append(int(rng.choice([0, 1, H - 1, W + 1, 777, 3 * W + 5, int(rng.integers(1, 2 * W))])))
        return out
    size = {"one": 1, "hop-1": H - 1, "w+1": W + 1, "odd": 777}[kind]
    return [size] * (n // size + 1)


def _run(ctx, x, cfg, chunks):
    """Push x in `chunks` (the last one cut at the end of x): (outputs per push, buffered samples
    afterwards, the chunk lengths actually pushed)."""
    st = ctx.stft_stream(cfg)
    outs, used, pos = [], [], 0
    for m in chunks:
        piece = x[pos:pos + m]
        r = st.push(piece)
        pos += len(piece)
        outs.append(r)
        used.append(len(piece))
        if pos >= len(x):
            break
    buffered = st.buffered
    st.close()
    return outs, buffered, used


@pytest.mark.parametrize("kind", ["one", "hop-1", "w+1", "odd", "mixed"])
@pytest.mark.parametrize("prec", [sonar.F64, sonar.F32])
def test_stream_rows_equal_one_shot(ctx, kind, prec):
    W, H = 1024, 256
    n = 44100 if kind != "one" else 6000
    x = _sig(n)
    flags = sonar.FP_MAGNITUDE | sonar.FP_MFCC | sonar.FP_PHASE
    cfg = ctx.config(window_size=W, hop_size=H, sample_rate=44100, n_filters=40, n_mfcc=13, precision=prec,
                     pcm_dtype=sonar.F64, out_dtype=sonar.F64, flags=flags)
    outs, buffered, used = _run(ctx, x, cfg, _chunks(kind, W, H, n))
    starts, buf = go_stream_frames(used, W, H)
    assert buffered == buf
    for r, s in zip(outs, starts):                              # frames emitted by each push
        assert (r["magnitude"].shape[0] if r else 0) == len(s)
    got = {k: np.concatenate([r[k] for r in outs if r]) for k in ("magnitude", "mfcc", "phase")}
    F = len(got["magnitude"])
    assert sum(used) == n and F == sonar.stft_frames(n, W, H)
    one = ctx.fingerprint(x[: (F - 1) * H + W], ctx.config(**{f: getattr(cfg, f) for f, _ in cfg._fields_}
                                                         | {"flags": flags | sonar.FP_GENERIC}))
    assert ctx.last_fp_kernel() == "fp_wave_kernel"
    for k in got:
        assert np.array_equal(got[k], one[k]), k                # bit-identical rows
    ref = O.stft_mag(x[: (F - 1) * H + W], W, H)
    tol = 1e-11 if prec == sonar.F64 else 2e-6
    assert np.max(np.abs(got["magnitude"] - ref) / ref.max(axis=1)[:, None]) < tol
    assert_mfcc(got["mfcc"], O.mfcc_frames(ref, 44100, n_coef=13, n_mels=40), 1e-9 if prec == sonar.F64 else 1e-4)


@pytest.mark.parametrize("W,H,chunks", [(256, 512, [300, 300, 100, 700, 1024, 5, 900]),
                                        (256, 700, [1000, 1, 255, 2000, 260]),
                                        (512, 128, [100, 411, 1, 1, 129, 2048])])
def test_stream_go_buffer_rules(ctx, W, H, chunks):
    """H > W: a frame whose hop reaches past the buffered samples clears the buffer (:355-362), so the
    rest of the skip is dropped and the next frame starts at the next chunk -- frame placement depends
    on the chunking.  Every emitted frame equals the oracle's STFT of the samples Go windows."""
    x = _sig(sum(chunks), seed=3)
    cfg = ctx.config(window_size=W, hop_size=H, precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64,
                     flags=sonar.FP_MAGNITUDE | sonar.FP_COMPLEX)
    st = ctx.stft_stream(cfg)
    starts, buf = go_stream_frames(chunks, W, H)
    pos = 0
    for m, s in zip(chunks, starts):
        assert st.frames(m) == len(s)
        r = st.push(x[pos:pos + m])
        pos += m
        if not s:
            assert not r or r["magnitude"].shape[0] == 0
            continue
        for row, a in enumerate(s):
            ref = O.stft_mag(x[a:a + W], W, W)[0]
            assert np.max(np.abs(r["magnitude"][row] - ref)) < 1e-11 * ref.max()
            re, _ = O.stft_complex(x[a:a + W], W, W)
            cplx = r["complex"][row][:, 0] + 1j * r["complex"][row][:, 1]
            assert np.max(np.abs(cplx - re[0])) < 1e-11 * ref.max()
    assert st.buffered == buf
    st.close()


def test_stream_device_pointers(ctx):
    import torch
    W, H = 1024, 256
    x = _sig(30000, seed=5).astype(np.float32)
    cfg = ctx.config(window_size=W, hop_size=H, sample_rate=44100, n_filters=40, n_mfcc=13, precision=sonar.F32,
                     pcm_dtype=sonar.F32, out_dtype=sonar.F32, flags=sonar.FP_MFCC)
    one = ctx.fingerprint(x, ctx.config(**{f: getattr(cfg, f) for f, _ in cfg._fields_}
                                        | {"flags": sonar.FP_MFCC | sonar.FP_GENERIC}))["mfcc"]
    cfg.device_ptrs = 1
    st = ctx.stft_stream(cfg)
    dx = torch.from_numpy(x).cuda()
    out = torch.zeros((len(one), 13), dtype=torch.float32, device="cuda")
    pos, row = 0, 0
    for m in [5000, 1, 3000, 1023, 20976]:
        F = st.frames(m)
        got = st.push_device(dx.data_ptr() + 4 * pos, m, mfcc=out.data_ptr() + 4 * 13 * row)
        assert got == F
        pos += m
        row += F
    torch.cuda.synchronize()
    assert row == len(one)
    assert np.array_equal(out.cpu().numpy(), one)
    st.close()


def test_stream_errors_and_empty_chunks(ctx):
    with pytest.raises(sonar.SonarError) as e:
        ctx.stft_stream(ctx.config(window_size=0, flags=sonar.FP_MAGNITUDE))
    assert e.value.msg == "failed to generate window: window size must be positive: 0"
    with pytest.raises(sonar.SonarError) as e:
        ctx.stft_stream(ctx.config(window_size=1048577, flags=sonar.FP_MAGNITUDE))
    assert "window size too large: 1048577" in e.value.msg
    with pytest.raises(sonar.SonarError) as e:
        ctx.stft_stream(ctx.config(flags=sonar.FP_MAGNITUDE | sonar.FP_SPECTRAL))
    assert e.value.code == sonar._abi.ERR_UNSUPPORTED
    st = ctx.stft_stream(ctx.config(window_size=256, hop_size=0, flags=sonar.FP_MAGNITUDE, pcm_dtype=sonar.F64))
    assert st.push(np.zeros(0)) == {} and st.push(np.ones(100)) == {}      # no frame due: fine
    assert st.buffered == 100
    with pytest.raises(sonar.SonarError, match="never advances"):
        st.push(np.ones(200))
    st.close()
    st = ctx.stft_stream(ctx.config(window_size=256, hop_size=-3, flags=sonar.FP_MAGNITUDE, pcm_dtype=sonar.F64))
    with pytest.raises(sonar.SonarError) as e:
        st.push(np.ones(300))
    assert e.value.code == sonar.ERR_PANIC and e.value.msg == "runtime error: slice bounds out of range [-3:]"
    st.close()
