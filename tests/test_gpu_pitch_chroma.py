"""YIN core and music chroma on the GPU vs the oracle."""
import numpy as np
import pytest

import oracle as O
import sonar
from sonar import synth

pytestmark = pytest.mark.gpu


def test_yin_raw_bit_exact(ctx):
    sr = 16000
    x = synth.c4_speech(seconds=3.0, sr=sr)
    t = np.arange(len(x)) / sr
    x = x + 0.3 * np.sin(2 * np.pi * 220 * t)
    p, c, tau = ctx.pitch_yin(x, sr)
    F = O.lib().or_pitch_frames(len(x))
    assert len(p) == F
    for i in range(F):
        rp, rc, rt = O.yin_raw(x[i * 512: i * 512 + 1024], sr)
        assert tau[i] == rt
        assert p[i] == rp and c[i] == rc


def test_chroma_matches_oracle(ctx):
    x = synth.sweep(3.0)
    F = O.stft_frames(len(x), 1024, 256)
    got = ctx.chroma_stft(x, F, 256, 44100)
    ref = O.chroma_music(x, F, 256, 44100)
    assert np.max(np.abs(got - ref)) < 1e-9


def test_chroma_a440(ctx):
    t = np.arange(8192 * 10) / 44100
    x = np.sin(2 * np.pi * 440 * t)
    got = ctx.chroma_stft(x, 10, 4096, 44100, preprocess=False)     # fs = n / F = 8192
    assert np.all(np.argmax(got[:-2], axis=1) == 9)
    assert np.max(np.abs(got - O.chroma_frames(x, 10, 4096, 8192, 44100))) < 1e-9
