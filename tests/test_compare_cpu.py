"""FingerprintComparator oracle checks on CPU (no GPU).

The C oracle (oracle/compare_oracle.c) is checked against a second, independent
pure-Python restatement of comparison.go written directly from the Go text below; the
reference has no tests or golden vectors for the comparator, so
parity to Go is unpinned and this cross-check is what pins the oracle.
"""
import math

import numpy as np
import pytest

import oracle
from compare_fixtures import gallery
from sonar.compare import FD_KEYS, Fingerprint, Features, make_cfg, marshal, get_similarity_statistics


# ---- pure-Python restatement of comparison.go (small cases only) -----------------------
def _mean(v):
    return sum(v) / len(v)


def _var(v):
    mu = _mean(v)
    ss = sum((x - mu) ** 2 for x in v)
    comp = sum(x - mu for x in v)
    n = len(v)
    return (ss - comp * comp / n) / (n - 1) if n > 1 else float("nan")


def _sqrt(x):
    return math.sqrt(x) if x == x else float("nan")


def _cos(a, b):
    if len(a) != len(b) or not a:
        return 0.0
    if any(x != x for x in a + b):
        return float("nan")
    dot = sum(x * y for x, y in zip(a, b))
    n1, n2 = math.sqrt(sum(x * x for x in a)), math.sqrt(sum(x * x for x in b))
    if n1 == 0 or n2 == 0:
        return 0.0
    return dot / (n1 * n2)


def _seq(s1, s2):
    s1, s2 = list(map(float, s1)), list(map(float, s2))
    return _cos([_mean(s1), _sqrt(_var(s1))], [_mean(s2), _sqrt(_var(s2))])


def _scalar(a, b):
    if a == 0 and b == 0:
        return 1.0
    mx = max(abs(a), abs(b))
    return 1.0 if mx == 0 else max(0.0, 1.0 - abs(a - b) / mx)


W = {"news": [.5, .25, .05, .15, .1, .05], "talk": [.5, .25, .05, .15, .1, .05],
     "music": [.3, .2, .25, .1, .05, .15], "sports": [.25, .2, .05, .25, .1, .05]}


def py_compare(a: Fingerprint, b: Fingerprint, detailed=False, content_filter=False):
    r = {"match": a.content_type == b.content_type, "dist": {}, "fs": 0.0}
    if content_filter and not r["match"]:
        r["conf"] = 0.25
        return r
    fa, fb = a.features, b.features
    if fa is not None and fb is not None:
        w = ([a.feature_weights.get(k, 0.0) for k in FD_KEYS] if a.feature_weights is not None
             else W.get(a.content_type, [.35, .25, .1, .2, .1, .1]))
        sims, ws = [], []

        def add(i, s):
            sims.append(s)
            ws.append(w[i])
            r["dist"][FD_KEYS[i]] = 1.0 - s

        if fa.mfcc is not None and fb.mfcc is not None and len(fa.mfcc) and len(fb.mfcc):
            def st(m):
                m = np.asarray(m, dtype=float)
                if m.shape[1] == 0:
                    return []
                return [_mean(list(m[:, c])) for c in range(m.shape[1])] + \
                       [_sqrt(_var(list(m[:, c]))) for c in range(m.shape[1])]
            s1, s2 = st(fa.mfcc), st(fb.mfcc)
            add(0, _cos(s1, s2) if s1 and s2 else 0.0)
        if fa.spectral is not None and fb.spectral is not None:
            v = [_seq(fa.spectral[k], fb.spectral[k]) for k in ("centroid", "rolloff", "flux")
                 if len(fa.spectral[k]) and len(fb.spectral[k])]
            add(1, _mean(v) if v else 0.0)
        if fa.chroma is not None and fb.chroma is not None and len(fa.chroma) and len(fb.chroma):
            m1 = np.asarray(fa.chroma).mean(axis=0).tolist()
            m2 = np.asarray(fb.chroma).mean(axis=0).tolist()
            add(2, _cos(m1, m2))
        if fa.temporal is not None and fb.temporal is not None:
            t1, t2 = fa.temporal, fb.temporal
            v = []
            if t1["dynamic_range"] > 0 and t2["dynamic_range"] > 0:
                v.append(_scalar(t1["dynamic_range"], t2["dynamic_range"]))
            v.append(_scalar(t1["silence_ratio"], t2["silence_ratio"]))
            if t1["onset_density"] > 0 and t2["onset_density"] > 0:
                v.append(_scalar(t1["onset_density"], t2["onset_density"]))
            if len(t1["rms_energy"]) and len(t2["rms_energy"]):
                v.append(_seq(t1["rms_energy"], t2["rms_energy"]))
            add(3, _mean(v))
        if fa.speech is not None and fb.speech is not None:
            s1, s2 = fa.speech, fb.speech
            v = []
            if s1["speech_rate"] > 0 and s2["speech_rate"] > 0:
                v.append(_scalar(s1["speech_rate"], s2["speech_rate"]))
            if s1["vocal_tract_length"] > 0 and s2["vocal_tract_length"] > 0:
                v.append(_scalar(s1["vocal_tract_length"], s2["vocal_tract_length"]))
            if len(s1["voicing_probability"]) and len(s2["voicing_probability"]):
                v.append(_seq(s1["voicing_probability"], s2["voicing_probability"]))
            add(4, _mean(v) if v else 0.0)
        if fa.harmonic is not None and fb.harmonic is not None:
            v = [_seq(fa.harmonic[k], fb.harmonic[k]) for k in ("harmonic_ratio", "pitch_estimate")
                 if len(fa.harmonic[k]) and len(fb.harmonic[k])]
            add(5, _mean(v) if v else 0.0)
        if sims:
            r["fs"] = sum(x * y for x, y in zip(ws, sims)) / sum(ws)
    nd = len(r["dist"])
    conf = 0.5 + (0.3 if r["fs"] > 0.8 else 0.2 if r["fs"] > 0.6 else 0.0)
    conf += 0.1 if r["match"] else 0.0
    conf += nd * 0.05
    r["conf"] = conf if conf != conf else max(0.0, min(1.0, conf))
    return r


def _close(x, y):
    return (x != x and y != y) or abs(x - y) <= 1e-9 * max(1.0, abs(x), abs(y))


def test_oracle_matches_python_restatement():
    fps = gallery(11, 24)
    cfg = make_cfg({"similarity_threshold": 0.0, "max_candidates": 10})
    structs = [marshal(fp) for fp in fps]
    for i, (fa, _) in enumerate(structs):
        for j, (fb, _) in enumerate(structs):
            s = oracle.fp_compare(fa, fb, cfg)
            p = py_compare(fps[i], fps[j])
            assert _close(s.overall_similarity, p["fs"]), (i, j, s.overall_similarity, p["fs"])
            assert _close(s.confidence, p["conf"]), (i, j)
            got = {k: s.feature_distances[n] for n, k in enumerate(FD_KEYS) if s.distance_mask & (1 << n)}
            assert got.keys() == p["dist"].keys(), (i, j)
            for k in got:
                assert _close(got[k], p["dist"][k]), (i, j, k)
            assert bool(s.content_type_match) == p["match"]


def test_oracle_content_filter_and_status():
    a = Fingerprint("a", "music", 10, Features(mfcc=np.ones((4, 13))))
    b = Fingerprint("b", "news", 10, Features(mfcc=np.ones((4, 13))))
    fa, _ = marshal(a)
    fb, _ = marshal(b)
    s = oracle.fp_compare(fa, fb, make_cfg({"enable_content_filter": True}))
    assert s.overall_similarity == 0.0 and s.confidence == 0.25 and s.distance_mask == 0
    s = oracle.fp_compare(fa, fa, make_cfg({}))
    assert s.status == 1                                    # same ID: skipped by BatchCompare
    n = Fingerprint("n", "music", 10, None)
    fn, _ = marshal(n)
    s = oracle.fp_compare(fa, fn, make_cfg({}))
    assert s.status == 2 and s.overall_similarity == 0.0    # "features cannot be nil"
    with pytest.raises(ValueError):                         # detailed metrics deref nil Features
        oracle.fp_compare(fa, fn, make_cfg({"enable_detailed_metrics": True}))


def test_oracle_find_best_matches_semantics():
    fps = gallery(5, 30, full=True, n_frames=50)
    cfg = make_cfg({"similarity_threshold": 0.3, "max_candidates": 7})
    fq, kq = marshal(fps[0])
    arr = (type(fq) * len(fps))()
    keep = []
    for i, fp in enumerate(fps):
        arr[i], k = marshal(fp)
        keep.append(k)
    m = oracle.find_best_matches(fq, arr, cfg)
    assert len(m) <= 7
    sims = [x.similarity.overall_similarity for x in m]
    assert sims == sorted(sims, reverse=True)
    assert all(s >= 0.3 for s in sims)
    assert [x.rank for x in m] == list(range(1, len(m) + 1))
    assert all(x.candidate != 0 for x in m)                 # self (same ID) skipped
    assert oracle.find_best_matches(fq, arr, make_cfg({"similarity_threshold": 0.0, "max_candidates": 0})) == []


def test_ragged_mfcc_rows_pad_with_zero():
    rows = [[1.0, 2.0, 3.0], [4.0], [5.0, 6.0, 7.0, 8.0]]
    f, keep = marshal(Fingerprint("r", features=Features(mfcc=rows)))
    m = keep[0]
    assert f.mfcc_coeffs == 3 and f.mfcc_frames == 3
    assert np.array_equal(m, [[1, 2, 3], [4, 0, 0], [5, 6, 7]])


def test_similarity_statistics():
    res = [{"overall_similarity": x, "feature_similarity": x, "confidence": 0.5} for x in (0.2, 0.9, 0.4, 0.6)]
    st = get_similarity_statistics(res)
    assert st["overall_min"] == 0.2 and st["overall_max"] == 0.9
    assert st["overall_median"] == 0.4                      # Empirical quantile: first with cum >= p n
    assert abs(st["overall_mean"] - 0.525) < 1e-15
    assert st["total_comparisons"] == 4.0
