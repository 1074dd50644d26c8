"""Host-side kernel selection of sonar_fingerprint (sonar_fp_kernel_plan: no device needed).

The headline kernel (mfcc_pair_kernel) indexes frames with 32-bit integers; a call with more than
SONAR_PAIR_MAX_FRAMES frames must take the 64-bit general kernel instead of overflowing (ADVICE r04:
at hop 1 that is ~8.6 GB of f32 PCM).  Validation errors come back in ComputeSTFTWithWindow's order
(fingerprint/analyzers/spectral.go:386-412)."""
import sonar
from sonar import Context


def _cfg(**kw):
    base = dict(window_size=1024, hop_size=256, precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32,
                flags=sonar.FP_MFCC)
    base.update(kw)
    return Context.config(**base)


def test_pair_kernel_frame_limit():
    W = 1024
    n_at = lambda F, H: (F - 1) * H + W          # noqa: E731 -- samples giving exactly F frames
    assert sonar.fp_kernel_plan(_cfg(), 44100 * 3600) == sonar.PLAN_PAIR
    lim = sonar.PAIR_MAX_FRAMES
    assert sonar.stft_frames(n_at(lim, 1), W, 1) == lim
    assert sonar.fp_kernel_plan(_cfg(hop_size=1), n_at(lim, 1)) == sonar.PLAN_PAIR
    assert sonar.fp_kernel_plan(_cfg(hop_size=1), n_at(lim + 1, 1)) == sonar.PLAN_WAVE
    assert sonar.fp_kernel_plan(_cfg(hop_size=1), n_at(1 << 33, 1)) == sonar.PLAN_WAVE
    # odd frame counts at the limit: the last pair's second frame index is 2 NP - 1 <= lim
    assert sonar.fp_kernel_plan(_cfg(hop_size=1), n_at(lim - 1, 1)) == sonar.PLAN_PAIR


def test_plan_routes_like_the_call():
    assert sonar.fp_kernel_plan(_cfg(precision=sonar.F64), 10 ** 6) == sonar.PLAN_WAVE     # f32 output
    # float64 arithmetic + output: the pair kernel's double instantiation, PCM of either type
    assert sonar.fp_kernel_plan(_cfg(precision=sonar.F64, out_dtype=sonar.F64), 10 ** 6) == sonar.PLAN_PAIR
    assert sonar.fp_kernel_plan(_cfg(precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64),
                                10 ** 6) == sonar.PLAN_PAIR
    assert sonar.fp_kernel_plan(_cfg(pcm_dtype=sonar.F64), 10 ** 6) == sonar.PLAN_WAVE
    assert sonar.fp_kernel_plan(_cfg(out_dtype=sonar.F64), 10 ** 6) == sonar.PLAN_WAVE
    assert sonar.fp_kernel_plan(_cfg(flags=sonar.FP_MFCC | sonar.FP_SPECTRAL), 10 ** 6) == sonar.PLAN_WAVE
    assert sonar.fp_kernel_plan(_cfg(flags=sonar.FP_MFCC | sonar.FP_GENERIC), 10 ** 6) == sonar.PLAN_WAVE
    assert sonar.fp_kernel_plan(_cfg(window_size=2048), 10 ** 6) == sonar.PLAN_WAVE
    assert sonar.fp_kernel_plan(_cfg(window_size=1000), 10 ** 6) == sonar.PLAN_DFT
    assert sonar.fp_kernel_plan(_cfg(flags=sonar.FP_ZCR), 10 ** 6) == sonar.PLAN_NONE


def test_plan_validation_errors_in_go_order():
    assert sonar.fp_kernel_plan(_cfg(), 0) == sonar.ERR_EMPTY
    assert sonar.fp_kernel_plan(_cfg(window_size=0), 4096) == sonar.ERR_INVALID
    assert sonar.fp_kernel_plan(_cfg(hop_size=0), 4096) == sonar.ERR_INVALID
    assert sonar.fp_kernel_plan(_cfg(), 700) == sonar.ERR_TOO_SHORT
    assert sonar.fp_kernel_plan(_cfg(window_size=1000, flags=sonar.FP_SPECTRAL), 10 ** 5) == sonar.PLAN_DFT
    assert sonar.fp_kernel_plan(_cfg(window_size=9000, flags=sonar.FP_MFCC), 10 ** 5) == sonar._abi.ERR_UNSUPPORTED
