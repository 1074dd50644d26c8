"""FingerprintComparator on the GPU gallery vs the CPU oracle (comparison.go).

Every (query, candidate) pair of seeded synthetic galleries is compared through the C ABI
(sonar_gallery_add -> sonar_compare / sonar_find_best_matches) and by the oracle, which
recomputes the statistics from the full arrays on each call as the Go code does.  float64
throughout; the statistics are reduced in a different order on the device (row chunks),
so scores agree to 1e-12 relative, and integer fields (masks, status, ranks, candidates,
match types) exactly.  Parity to Go is unpinned (see test_compare_cpu.py).
"""
import numpy as np
import pytest

import oracle
from compare_fixtures import gallery, random_fingerprint
from sonar import Context, SonarError
from sonar._abi import FpFeatures
from sonar.compare import (FD_KEYS, Features, Fingerprint, FingerprintComparator, Gallery, make_cfg, marshal)

pytestmark = pytest.mark.gpu

SCORE = ["overall_similarity", "feature_similarity", "confidence", "data_availability", "feature_coverage",
         "temporal_alignment", "noise_level", "dynamic_range_match", "spectral_coherence"]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def _close(x, y, rtol=1e-12):
    return (x != x and y != y) or abs(x - y) <= rtol * max(1.0, abs(x), abs(y))


def _same(g, o, tag):
    for k in SCORE:
        assert _close(getattr(g, k), getattr(o, k)), (tag, k, getattr(g, k), getattr(o, k))
    for n in range(6):
        if o.distance_mask & (1 << n):
            assert _close(g.feature_distances[n], o.feature_distances[n]), (tag, FD_KEYS[n])
    for k in ("distance_mask", "content_type_match", "has_quality", "status"):
        assert getattr(g, k) == getattr(o, k), (tag, k, getattr(g, k), getattr(o, k))


def _structs(fps):
    out, keep = [], []
    for fp in fps:
        f, k = marshal(fp)
        out.append(f)
        keep.append(k)
    return out, keep


@pytest.mark.parametrize("seed,cf", [(1, False), (2, True)])
def test_all_pairs_vs_oracle(ctx, seed, cf):
    fps = gallery(seed, 48)
    g = Gallery(ctx)
    assert g.add(fps, keep_sequences=False) == 0 and len(g) == 48
    cfg = make_cfg({"similarity_threshold": 0.5, "max_candidates": 5, "enable_content_filter": cf})
    out, nc = g.compare(np.arange(48), None, cfg)
    st, keep = _structs(fps)
    for i in range(48):
        for j in range(48):
            _same(out[i * nc + j], oracle.fp_compare(st[i], st[j], cfg), (seed, i, j))
    g.close()


def test_detailed_metrics_vs_oracle(ctx):
    rng = np.random.default_rng(3)
    fps = [random_fingerprint(rng, k, n_frames=int(rng.integers(2, 300)), full=True, equal_len=257)
           for k in range(20)]
    g = Gallery(ctx)
    g.add(fps[:7], keep_sequences=True)
    g.add(fps[7:], keep_sequences=True)                    # two adds: growth + pool offsets
    cfg = make_cfg({"similarity_threshold": 0.0, "max_candidates": 50, "enable_detailed_metrics": True})
    cands = np.array([3, 0, 19, 7, 7, 11])
    out, nc = g.compare(np.arange(20), cands, cfg)
    st, keep = _structs(fps)
    for i in range(20):
        for j, c in enumerate(cands):
            _same(out[i * nc + j], oracle.fp_compare(st[i], st[c], cfg), (i, c))
    g.close()


def test_detailed_metrics_errors(ctx):
    a = Fingerprint("a", "music", 1, Features(spectral={"centroid": np.ones(10), "rolloff": np.ones(10),
                                                        "flux": np.ones(9)}))
    b = Fingerprint("b", "music", 1, Features(spectral={"centroid": np.ones(11), "rolloff": np.ones(11),
                                                        "flux": np.ones(10)}))
    n = Fingerprint("n", "music", 1, None)
    g = Gallery(ctx)
    g.add([a, b, n], keep_sequences=True)
    cfg = make_cfg({"enable_detailed_metrics": True})
    with pytest.raises(SonarError, match="length mismatch"):     # gonum stat.Correlation panics
        g.compare([0], [1], cfg)
    with pytest.raises(SonarError, match="nil"):                 # nil Features dereference
        g.compare([0], [2], cfg)
    out, _ = g.compare([0], [1], make_cfg({}))                   # fine without detailed metrics
    assert out[0].status == 0
    g.close()


def test_long_and_wide_matrices(ctx):
    """Multi-chunk reductions (200k frames) and the > 256-column path."""
    rng = np.random.default_rng(4)
    big = Fingerprint("big", "news", 100.0, Features(
        mfcc=rng.normal(3, 2, (200_003, 13)), chroma=np.abs(rng.normal(0, 1, (200_003, 12))),
        spectral={"centroid": rng.normal(1e3, 10, 200_003), "rolloff": rng.normal(4e3, 5, 200_003),
                  "flux": rng.normal(0, 1, 200_002)}))
    wide = Fingerprint("wide", "news", 3.0, Features(mfcc=rng.normal(0, 1, (700, 300)),
                                                     chroma=np.abs(rng.normal(0, 1, (700, 300)))))
    wide2 = Fingerprint("wide2", "news", 3.0, Features(mfcc=rng.normal(1, 1, (1000, 300)),
                                                       chroma=np.abs(rng.normal(0, 1, (1000, 300)))))
    fps = [big, wide, wide2, big]
    g = Gallery(ctx)
    g.add(fps)
    cfg = make_cfg({})
    out, nc = g.compare(np.arange(4), None, cfg)
    st, keep = _structs(fps)
    for i in range(4):
        for j in range(4):
            _same(out[i * nc + j], oracle.fp_compare(st[i], st[j], cfg), (i, j))
    g.close()


@pytest.mark.parametrize("thr,K", [(0.0, 50), (0.5, 3), (0.9, 10), (0.0, 0)])
def test_find_best_matches_vs_oracle(ctx, thr, K):
    fps = gallery(9, 64)
    g = Gallery(ctx)
    g.add(fps)
    cfg = make_cfg({"similarity_threshold": thr, "max_candidates": K})
    queries = np.array([0, 5, 17, 63])
    res = g.find_best_matches(queries, None, cfg)
    st, keep = _structs(fps)
    arr = (FpFeatures * len(st))(*st)
    for qi, q in enumerate(queries):
        want = oracle.find_best_matches(st[q], arr, cfg)
        got = res[qi]
        assert len(got) == len(want), (q, len(got), len(want))
        for a, b in zip(got, want):
            assert (a.candidate, a.rank, a.match_type) == (b.candidate, b.rank, b.match_type), q
            _same(a.similarity, b.similarity, (q, a.candidate))
    g.close()


def test_comparator_api(ctx):
    """FingerprintComparator mirror: Compare / BatchCompare / FindBestMatches / ValidateConfig."""
    fps = gallery(12, 16, full=True, n_frames=120)
    fc = FingerprintComparator({"similarity_threshold": 0.2, "max_candidates": 4, "method": "auto"}, ctx=ctx)
    fc.validate_config()
    r = fc.compare(fps[0], fps[1])
    fa, ka = marshal(fps[0])
    fb, kb = marshal(fps[1])
    o = oracle.fp_compare(fa, fb, fc.cfg)
    assert _close(r["overall_similarity"], o.overall_similarity)
    batch = fc.batch_compare(fps[0], [None] + fps)            # nil and self are skipped
    assert len(batch) == sum(fp.id != fps[0].id for fp in fps)
    m = fc.find_best_matches(fps[0], fps)
    assert len(m) <= 4 and all(x["fingerprint"] is not fps[0] for x in m)
    assert [x["rank"] for x in m] == list(range(1, len(m) + 1))
    with pytest.raises(SonarError):
        FingerprintComparator({"similarity_threshold": 2.0, "max_candidates": 1}, ctx=ctx).validate_config()


def test_generated_fingerprints(ctx):
    """Fingerprints from sonar_generate_fingerprint (speech extractor output) compared."""
    from sonar.synth import sweep
    fps = []
    for k, (f0, ct) in enumerate([(100.0, "music"), (150.0, "music"), (100.0, "news")]):
        x = sweep(4.0, f0=f0)
        fps.append(FingerprintComparator.fingerprint_from_pcm(ctx, x, 44100, ct, f"g{k}"))
    g = Gallery(ctx)
    g.add(fps)
    cfg = make_cfg(None)
    out, nc = g.compare(np.arange(3), None, cfg)
    st, keep = _structs(fps)
    for i in range(3):
        for j in range(3):
            _same(out[i * nc + j], oracle.fp_compare(st[i], st[j], cfg), (i, j))
    assert out[0 * nc + 1].overall_similarity > 0.5
    g.close()
