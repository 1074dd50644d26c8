"""Edge cases of the lane-dense music-feature kernels (misc_kernels.hip, round 4) against the
oracle's serial float64 chains (oracle.dc_removal / preemphasis, dc_removal.go:101-124 +
pre_emphasis.go:135-155; oracle.short_time_energy, energy.go:25-50).

* dc_block_kernel / dc_carry_kernel: 4,096-sample blocks of 16-sample lane chunks whose start
  states come from affine-map scans.  With a ShortTimeEnergy window and hop of ONE sample the
  energy of frame i is |z_i|, so the per-sample output of the scan is compared directly, at
  lengths around the chunk and block sizes (ragged last chunk / block, one block + 1 sample,
  a single chunk).  Bound: 1e-13 of max |z| (the scan reassociates the carries: a few ulp of the
  signal scale, DESIGN.md Kernel 4).
* energy_wave_kernel: one lane per frame over 16-sample LDS rounds -- windows that are not a
  multiple of 16, shorter than a round, hops larger than the window, frame counts that leave
  partial waves and blocks.  The sums are Go's sequential chains on the kernel's z, so against
  the oracle they inherit only z's rounding: 1e-12 relative."""
import numpy as np
import pytest

import oracle as O
from sonar import synth

pytestmark = pytest.mark.gpu

SR = 44100


def _z_ref(x):
    return O.preemphasis(O.dc_removal(x, 0.995), 0.95)


@pytest.mark.parametrize("n", [1024, 1040, 4095, 4096, 4097, 8192 + 17, 65536 + 4096 * 3 + 5, 300_001])
def test_dc_scan_per_sample(ctx, n):
    rng = np.random.default_rng(n)
    x = 0.4 * np.sin(2 * np.pi * 97.0 * np.arange(n) / SR) + 0.05 * rng.standard_normal(n) + 0.2
    e, _ = ctx.music_alignment_features(x, SR, 1024, 256, 1, 1)
    z = _z_ref(x)
    assert e.shape == (n,)
    err = np.max(np.abs(e - np.abs(z)))
    assert err <= 1e-13 * np.max(np.abs(z)), err


@pytest.mark.parametrize("W,H", [(1000, 333), (5, 3), (17, 17), (16, 40), (2048, 7), (1024, 256)])
def test_energy_odd_windows(ctx, W, H):
    n = 44100 + 123
    x = synth.c3_pair(seconds=n / SR, lag_s=0.25)[0][:n]
    e, _ = ctx.music_alignment_features(x, SR, 1024, 256, W, H)
    ref = O.short_time_energy(_z_ref(x), W, H)
    assert e.shape == ref.shape
    assert np.max(np.abs(e - ref) / np.maximum(np.abs(ref), 1e-300)) < 1e-12


def test_energy_single_frame_and_window_equal_signal(ctx):
    x = synth.c3_pair(seconds=0.05, lag_s=0.01)[0][:2000]
    for W, H in [(2000, 256), (1999, 1), (1024, 4096)]:
        e, _ = ctx.music_alignment_features(x, SR, 1024, 256, W, H)
        ref = O.short_time_energy(_z_ref(x), W, H)
        assert e.shape == ref.shape, (W, H)
        assert np.max(np.abs(e - ref) / np.maximum(np.abs(ref), 1e-300)) < 1e-12, (W, H)
