"""SURVEY.md 8(f) rank 4 on the GPU: AlignmentAnalyzer.AnalyzeAlignmentConsistency
(stats/alignment.go:709-800; addNoise perturbation kernel + the NCC / DTW kernels) and
AlignmentExtractor.TruncateToAlignmentPCM (extractors/alignment.go:223-297) against the oracle
composition.  Offsets are integers and the statistics are functions of them: exact."""
import numpy as np
import pytest

import oracle as O
import sonar

pytestmark = pytest.mark.gpu


def _features(seed, n, dim, shift):
    rng = np.random.default_rng(seed)
    base = np.abs(np.convolve(rng.standard_normal(n + shift + 100), np.ones(9) / 9, mode="same"))[:, None]
    base = base * (1 + rng.random((len(base), dim)))
    return base[shift:shift + n], base[:n]


@pytest.mark.parametrize("method", [O.ALIGN_XCORR, O.ALIGN_DTW, O.ALIGN_HYBRID])
@pytest.mark.parametrize("dim,shift,trials", [(1, 0, 5), (12, 37, 3), (3, 5, 1)])
def test_consistency_matches_oracle(ctx, method, dim, shift, trials):
    q, r = _features(11 + dim, 900, dim, shift)
    got = ctx.alignment_consistency(q, r, 44100, method=method, max_lag=120, hop=256, num_trials=trials)
    ref = O.alignment_consistency_reference(q, r, 44100, method, 120, 256, num_trials=trials)
    assert got == ref


def test_consistency_errors(ctx):
    q, r = _features(3, 200, 2, 4)
    with pytest.raises(sonar.SonarError, match="no successful alignments"):
        ctx.alignment_consistency(q, r, 44100, method=O.ALIGN_PHASE)
    with pytest.raises(sonar.SonarError, match="no successful alignments"):
        ctx.alignment_consistency(np.zeros((0, 2)), r, 44100)


def test_truncate_to_alignment(ctx):
    rng = np.random.default_rng(5)
    cases = [(441000, 441000, 44100, 2.0), (441000, 300000, 44100, -3.25), (1000, 1000, 44100, 0.0),
             (44100, 44100, 16000, 0.5), (50000, 80000, 44100, 1e-9)]
    cases += [(int(rng.integers(1, 10 ** 6)), int(rng.integers(1, 10 ** 6)), 44100, float(rng.normal(0, 5)))
              for _ in range(200)]
    for n1, n2, sr, off in cases:
        try:
            want = O.truncate_to_alignment_reference(n1, n2, sr, off)
        except ValueError as e:
            with pytest.raises(sonar.SonarError, match=str(e).split(":")[0]):
                ctx.truncate_to_alignment(n1, n2, sr, off)
            continue
        assert ctx.truncate_to_alignment(n1, n2, sr, off) == want, (n1, n2, sr, off)
