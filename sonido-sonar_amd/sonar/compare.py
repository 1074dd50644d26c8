"""FingerprintComparator over a device gallery (fingerprint/comparison.go).

Mirror of the reference's comparator API -- ``FingerprintComparator(cfg).compare``,
``batch_compare``, ``find_best_matches``, ``validate_config`` and
``get_similarity_statistics`` -- on the C ABI's gallery (include/sonar_gpu.h,
``sonar_gallery_*``, ``sonar_compare``, ``sonar_find_best_matches``).

Fingerprints are plain Python objects (``Fingerprint`` / ``Features`` below) shaped like
``AudioFingerprint`` / ``ExtractedFeatures`` (fingerprint/fingerprint.go:15-26,
extractors/features.go): ``None`` stands for a nil Go pointer or slice.  Each fingerprint's
statistics are reduced on the GPU once, when it first enters the comparator's gallery;
Compare then reads two records (the reference recomputes them on every call).
No CPU fallback: without the HIP library every call raises.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from ._abi import CompareCfg, FpFeatures, Match, SonarError, Similarity, lib, OK, ERR_INVALID

FEAT_FEATURES, FEAT_MFCC, FEAT_SPECTRAL, FEAT_CHROMA = 1, 2, 4, 8
FEAT_TEMPORAL, FEAT_SPEECH, FEAT_HARMONIC, FEAT_WEIGHTS = 16, 32, 64, 128
FD_KEYS = ["mfcc", "spectral", "chroma", "temporal", "speech", "harmonic"]
MATCH_TYPES = ["exact", "very_similar", "similar", "somewhat_similar", "weak"]
CONTENT_TYPES = {"music": 0, "news": 1, "sports": 2, "talk": 3, "mixed": 4, "unknown": 5}
METHODS = {"auto": 0, "fast": 1, "precise": 2}

_content_codes: Dict[str, int] = dict(CONTENT_TYPES)
_id_codes: Dict[str, int] = {}


def content_code(ct: str) -> int:
    """config.ContentType is a string; distinct strings get distinct codes (match = equality)."""
    if ct not in _content_codes:
        _content_codes[ct] = len(_content_codes) + 1
    return _content_codes[ct]


def id_code(fid: str) -> int:
    if fid not in _id_codes:
        _id_codes[fid] = len(_id_codes)
    return _id_codes[fid]


@dataclass
class Features:
    """extractors.ExtractedFeatures fields the comparator reads (None = nil)."""
    mfcc: Optional[object] = None            # [frames][coeffs] (rows may be ragged)
    chroma: Optional[object] = None          # [frames][bins]
    spectral: Optional[Dict[str, object]] = None   # centroid, rolloff, flux
    temporal: Optional[Dict[str, object]] = None   # dynamic_range, silence_ratio, onset_density, rms_energy
    speech: Optional[Dict[str, object]] = None     # speech_rate, vocal_tract_length, voicing_probability
    harmonic: Optional[Dict[str, object]] = None   # harmonic_ratio, pitch_estimate


@dataclass
class Fingerprint:
    """fingerprint.AudioFingerprint (ID, ContentType, Duration, Features, Metadata weights)."""
    id: str
    content_type: str = "unknown"
    duration: float = 0.0                    # seconds
    features: Optional[Features] = None
    feature_weights: Optional[Dict[str, float]] = None   # Metadata["feature_weights"]


def _mfcc_matrix(m) -> np.ndarray:
    """Rows are len(mfcc[0]) wide; a shorter row contributes 0 (comparison.go:784-789)."""
    if isinstance(m, np.ndarray) and m.ndim == 2:
        return np.ascontiguousarray(m, dtype=np.float64)
    rows = list(m)
    if not rows:
        return np.zeros((0, 0))
    C_ = len(rows[0])
    out = np.zeros((len(rows), C_))
    for t, r in enumerate(rows):
        r = np.asarray(r, dtype=np.float64)[:C_]
        out[t, :len(r)] = r
    return out


def _chroma_matrix(m) -> np.ndarray:
    if isinstance(m, np.ndarray) and m.ndim == 2:
        return np.ascontiguousarray(m, dtype=np.float64)
    rows = list(m)
    if not rows:
        return np.zeros((0, 0))
    widths = {len(r) for r in rows}
    if len(widths) != 1:
        raise SonarError(ERR_INVALID, "ragged chroma rows are not supported")
    return np.ascontiguousarray(np.asarray(rows, dtype=np.float64))


def marshal(fp: Fingerprint):
    """Fingerprint -> (FpFeatures, keep-alive list of the numpy arrays it points into)."""
    f = FpFeatures()
    keep = []
    f.id = id_code(fp.id)
    f.content_type = content_code(fp.content_type)
    f.duration_seconds = float(fp.duration)
    pres = 0

    def arr(x):
        a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
        keep.append(a)
        return C.c_void_p(a.ctypes.data) if a.size else None, a.size

    ft = fp.features
    if ft is not None:
        pres |= FEAT_FEATURES
        if ft.mfcc is not None:
            pres |= FEAT_MFCC
            m = _mfcc_matrix(ft.mfcc)
            keep.append(m)
            f.mfcc = m.ctypes.data if m.size else None
            f.mfcc_frames, f.mfcc_coeffs = m.shape[0], (m.shape[1] if m.shape[0] else 0)
        if ft.chroma is not None:
            pres |= FEAT_CHROMA
            m = _chroma_matrix(ft.chroma)
            keep.append(m)
            f.chroma = m.ctypes.data if m.size else None
            f.chroma_frames, f.chroma_bins = m.shape[0], (m.shape[1] if m.shape[0] else 0)
        if ft.spectral is not None:
            pres |= FEAT_SPECTRAL
            for key, name in (("centroid", "spectral_centroid"), ("rolloff", "spectral_rolloff"),
                              ("flux", "spectral_flux")):
                p, n = arr(ft.spectral.get(key, []))
                setattr(f, name, p)
                setattr(f, "n_" + name, n)
        if ft.temporal is not None:
            pres |= FEAT_TEMPORAL
            t = ft.temporal
            f.dynamic_range = float(t.get("dynamic_range", 0.0))
            f.silence_ratio = float(t.get("silence_ratio", 0.0))
            f.onset_density = float(t.get("onset_density", 0.0))
            f.rms_energy, f.n_rms_energy = arr(t.get("rms_energy", []))
        if ft.speech is not None:
            pres |= FEAT_SPEECH
            sp = ft.speech
            f.speech_rate = float(sp.get("speech_rate", 0.0))
            f.vocal_tract_length = float(sp.get("vocal_tract_length", 0.0))
            f.voicing_probability, f.n_voicing_probability = arr(sp.get("voicing_probability", []))
        if ft.harmonic is not None:
            pres |= FEAT_HARMONIC
            h = ft.harmonic
            f.harmonic_ratio, f.n_harmonic_ratio = arr(h.get("harmonic_ratio", []))
            f.pitch_estimate, f.n_pitch_estimate = arr(h.get("pitch_estimate", []))
    if fp.feature_weights is not None:
        pres |= FEAT_WEIGHTS
        for i, k in enumerate(FD_KEYS):
            f.feature_weights[i] = float(fp.feature_weights.get(k, 0.0))   # missing key -> 0
    f.present = pres
    return f, keep


def make_cfg(cfg: Optional[dict]) -> CompareCfg:
    """config.ComparisonConfig; None -> DefaultComparisonConfig (config/config.go:120-128)."""
    d = {"similarity_threshold": 0.75, "method": "auto", "max_candidates": 50,
         "enable_detailed_metrics": False, "enable_content_filter": False}
    if cfg is not None:
        d = {"similarity_threshold": 0.0, "method": "", "max_candidates": 0,
             "enable_detailed_metrics": False, "enable_content_filter": False, **cfg}
    c = CompareCfg()
    c.similarity_threshold = float(d["similarity_threshold"])
    c.max_candidates = int(d["max_candidates"])
    c.enable_detailed_metrics = int(bool(d["enable_detailed_metrics"]))
    c.enable_content_filter = int(bool(d["enable_content_filter"]))
    c.method = METHODS.get(d["method"], 0)
    c._src = d
    return c


def similarity_dict(s: Similarity) -> dict:
    """SimilarityResult as a dict (JSON names of comparison.go:28-49)."""
    out = {"overall_similarity": s.overall_similarity, "feature_similarity": s.feature_similarity,
           "content_type_match": bool(s.content_type_match), "confidence": s.confidence,
           "feature_distances": {k: s.feature_distances[i] for i, k in enumerate(FD_KEYS)
                                 if s.distance_mask & (1 << i)},
           "quality_metrics": None, "status": s.status, "alignment_applied": False,
           "temporal_offset_seconds": 0.0}
    if s.has_quality:
        out["quality_metrics"] = {k: getattr(s, k) for k in (
            "data_availability", "feature_coverage", "temporal_alignment", "noise_level",
            "dynamic_range_match", "spectral_coherence")}
    return out


class Gallery:
    """sonar_gallery: device-resident records of many fingerprints."""

    def __init__(self, ctx):
        self._ctx = ctx
        self._L = lib()
        h = C.c_void_p()
        ctx._check(self._L.sonar_gallery_create(ctx._h, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.sonar_gallery_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self._L.sonar_gallery_size(self._h))

    def add(self, fps: List[Fingerprint], keep_sequences=True) -> int:
        recs = (FpFeatures * max(1, len(fps)))()
        keep = []
        for i, fp in enumerate(fps):
            f, k = marshal(fp)
            recs[i] = f
            keep.append(k)
        first = C.c_int64()
        self._ctx._check(self._L.sonar_gallery_add(self._h, recs, len(fps), int(keep_sequences), 0,
                                                   C.byref(first)))
        return first.value

    def add_raw(self, recs, count, keep_sequences=False, device_ptrs=False) -> int:
        first = C.c_int64()
        self._ctx._check(self._L.sonar_gallery_add(self._h, recs, count, int(keep_sequences),
                                                   int(device_ptrs), C.byref(first)))
        return first.value

    def compare(self, queries, candidates, cfg: CompareCfg):
        q = np.ascontiguousarray(queries, dtype=np.int64)
        cand = None if candidates is None else np.ascontiguousarray(candidates, dtype=np.int64)
        nc = len(self) if cand is None else len(cand)
        out = (Similarity * max(1, len(q) * nc))()
        self._ctx._check(self._L.sonar_compare(
            self._h, q.ctypes.data_as(C.POINTER(C.c_int64)), len(q),
            None if cand is None else cand.ctypes.data_as(C.POINTER(C.c_int64)), nc, C.byref(cfg),
            C.cast(out, C.c_void_p), 0))
        return out, nc

    def compare_device(self, queries, candidates, cfg: CompareCfg, out_ptr: int):
        """sonar_compare with the results left in device memory at out_ptr (nq x nc records)."""
        q = np.ascontiguousarray(queries, dtype=np.int64)
        cand = None if candidates is None else np.ascontiguousarray(candidates, dtype=np.int64)
        nc = len(self) if cand is None else len(cand)
        self._ctx._check(self._L.sonar_compare(
            self._h, q.ctypes.data_as(C.POINTER(C.c_int64)), len(q),
            None if cand is None else cand.ctypes.data_as(C.POINTER(C.c_int64)), nc, C.byref(cfg),
            C.c_void_p(out_ptr), 1))
        return nc

    def find_best_matches_raw(self, queries, candidates, cfg: CompareCfg):
        """sonar_find_best_matches as the C arrays: (Match array nq x K, counts[nq])."""
        q = np.ascontiguousarray(queries, dtype=np.int64)
        cand = None if candidates is None else np.ascontiguousarray(candidates, dtype=np.int64)
        nc = len(self) if cand is None else len(cand)
        K = max(0, cfg.max_candidates)
        out = (Match * max(1, len(q) * K))()
        nm = np.zeros(max(1, len(q)), dtype=np.int64)
        self._ctx._check(self._L.sonar_find_best_matches(
            self._h, q.ctypes.data_as(C.POINTER(C.c_int64)), len(q),
            None if cand is None else cand.ctypes.data_as(C.POINTER(C.c_int64)), nc, C.byref(cfg), out,
            nm.ctypes.data_as(C.POINTER(C.c_int64))))
        return out, nm[: len(q)]

    def find_best_matches(self, queries, candidates, cfg: CompareCfg):
        q = np.ascontiguousarray(queries, dtype=np.int64)
        cand = None if candidates is None else np.ascontiguousarray(candidates, dtype=np.int64)
        nc = len(self) if cand is None else len(cand)
        K = max(0, cfg.max_candidates)
        out = (Match * max(1, len(q) * K))()
        nm = np.zeros(max(1, len(q)), dtype=np.int64)
        self._ctx._check(self._L.sonar_find_best_matches(
            self._h, q.ctypes.data_as(C.POINTER(C.c_int64)), len(q),
            None if cand is None else cand.ctypes.data_as(C.POINTER(C.c_int64)), nc, C.byref(cfg), out,
            nm.ctypes.data_as(C.POINTER(C.c_int64))))
        return [[out[i * K + k] for k in range(int(nm[i]))] for i in range(len(q))]


def merge_matches(lists, counts, cand_base, nq, max_candidates):
    """sonar_merge_matches: rank-local FindBestMatches lists (ctypes Match arrays of nq x K, with
    counts[r][q] valid rows) -> the single call's result over all ranks' candidates, as Match
    lists per query (candidates numbered from cand_base[r])."""
    L = lib()
    R, K = len(lists), max(0, int(max_candidates))
    lp = (C.c_void_p * max(1, R))(*[C.cast(x, C.c_void_p).value for x in lists])
    cnt = np.ascontiguousarray(np.asarray(counts, dtype=np.int64).reshape(R * nq) if R else np.zeros(1, np.int64))
    base = np.ascontiguousarray(np.asarray(cand_base, dtype=np.int64) if R else np.zeros(1, np.int64))
    out = (Match * max(1, nq * K))()
    nm = np.zeros(max(1, nq), dtype=np.int64)
    rc = L.sonar_merge_matches(lp, cnt.ctypes.data_as(C.POINTER(C.c_int64)), base.ctypes.data_as(C.POINTER(C.c_int64)),
                               R, nq, K, out, nm.ctypes.data_as(C.POINTER(C.c_int64)))
    if rc != OK:
        raise SonarError(rc, "sonar_merge_matches: invalid arguments")
    return [[out[i * K + k] for k in range(int(nm[i]))] for i in range(nq)]


def find_best_matches_distributed(local_lists, nq, max_candidates, n_local_candidates, group=None):
    """FindBestMatches across torch.distributed ranks (comparison.go:197-263):
    every rank passes its own gallery's top lists (Gallery.find_best_matches_raw), the fixed-size
    byte records are all-gathered (RCCL on GPUs, gloo in the CPU tests) with each rank's candidate
    count, and every rank merges them in the single call's order.  Returns the merged lists."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    K = max(0, int(max_candidates))
    matches, counts = local_lists
    raw = C.string_at(C.addressof(matches), nq * K * C.sizeof(Match)) if nq * K else b""
    payload = torch.frombuffer(bytearray(raw + np.asarray(counts, np.int64).tobytes()
                                         + np.int64(n_local_candidates).tobytes()), dtype=torch.uint8)
    parts = [torch.empty_like(payload) for _ in range(world)]
    dist.all_gather(parts, payload, group=group)
    lists, cnts, base, b = [], [], [], 0
    lb = nq * K * C.sizeof(Match)
    for part in parts:
        buf = part.numpy().tobytes()
        arr = (Match * max(1, nq * K)).from_buffer_copy(buf[:lb] + bytes(max(0, C.sizeof(Match) * max(1, nq * K) - lb)))
        lists.append(arr)
        cnts.append(np.frombuffer(buf[lb:lb + 8 * nq], dtype=np.int64))
        base.append(b)
        b += int(np.frombuffer(buf[lb + 8 * nq:lb + 8 * nq + 8], dtype=np.int64)[0])
    return merge_matches(lists, cnts, base, nq, K)


class FingerprintComparator:
    """fingerprint.FingerprintComparator (comparison.go:69-117) on a device gallery."""

    def __init__(self, cfg: Optional[dict] = None, ctx=None):
        from ._abi import Context
        self.ctx = ctx if ctx is not None else Context(0)
        self.cfg = make_cfg(cfg)
        self.config = self.cfg._src
        self.gallery = Gallery(self.ctx)
        self._index: Dict[int, int] = {}
        self._pinned: List[Fingerprint] = []      # keeps id(fp) unique while cached

    def index_of(self, fps: List[Fingerprint]) -> List[int]:
        new, seen = [], set()
        for fp in fps:
            if id(fp) not in self._index and id(fp) not in seen:
                seen.add(id(fp))
                new.append(fp)
        if new:
            first = self.gallery.add(new, keep_sequences=True)
            for i, fp in enumerate(new):
                self._index[id(fp)] = first + i
                self._pinned.append(fp)
        return [self._index[id(fp)] for fp in fps]

    def compare(self, fp1: Fingerprint, fp2: Fingerprint) -> dict:
        """Compare (comparison.go:133-194)."""
        if fp1 is None or fp2 is None:
            raise SonarError(ERR_INVALID, "fingerprints cannot be nil")
        a, b = self.index_of([fp1, fp2])
        out, _ = self.gallery.compare([a], [b], self.cfg)
        return similarity_dict(out[0])

    def batch_compare(self, query: Fingerprint, candidates: List[Optional[Fingerprint]]) -> List[dict]:
        """BatchCompare (:1107-1151): nil and same-ID candidates are skipped."""
        if query is None:
            raise SonarError(ERR_INVALID, "query fingerprint cannot be nil")
        cands = [c for c in candidates if c is not None]
        if not cands:
            return []
        idx = self.index_of([query] + cands)
        out, nc = self.gallery.compare([idx[0]], idx[1:], self.cfg)
        return [similarity_dict(out[i]) for i in range(nc) if out[i].status != 1]

    def find_best_matches(self, query: Fingerprint, candidates: List[Optional[Fingerprint]]) -> List[dict]:
        """FindBestMatches (:197-263)."""
        if query is None:
            raise SonarError(ERR_INVALID, "query fingerprint cannot be nil")
        cands = [c for c in candidates if c is not None]
        if self.cfg.max_candidates < 0:
            raise SonarError(ERR_INVALID, "max candidates must not be negative (Go panics)")
        if not cands:
            return []
        idx = self.index_of([query] + cands)
        res = self.gallery.find_best_matches([idx[0]], idx[1:], self.cfg)[0]
        return [{"fingerprint": cands[m.candidate], "similarity": similarity_dict(m.similarity),
                 "rank": m.rank, "match_type": MATCH_TYPES[m.match_type]} for m in res]

    @staticmethod
    def fingerprint_from_result(res: dict, fid: str, content_type: Optional[str] = None) -> Fingerprint:
        """AudioFingerprint view of a sonar_generate_fingerprint result (the extractor's
        ExtractedFeatures groups are non-nil exactly when their arrays are present)."""
        names = {v: k for k, v in CONTENT_TYPES.items()}
        if content_type is None:
            content_type = names.get(int(res["content_type"].reshape(-1)[0]), "unknown") if "content_type" in res \
                else "unknown"

        def sc(k):
            return float(res[k].reshape(-1)[0]) if k in res else 0.0

        def vec(k):
            return np.asarray(res[k], dtype=np.float64).reshape(-1) if k in res else np.zeros(0)

        feat = Features()
        if "mfcc" in res:
            feat.mfcc = np.asarray(res["mfcc"], dtype=np.float64)
        if "spectral_centroid" in res:
            feat.spectral = {"centroid": vec("spectral_centroid"), "rolloff": vec("spectral_rolloff"),
                             "flux": vec("spectral_flux")}
        if "rms_energy" in res or "dynamic_range" in res:
            feat.temporal = {"dynamic_range": sc("dynamic_range"), "silence_ratio": sc("silence_ratio"),
                             "onset_density": sc("onset_density"), "rms_energy": vec("rms_energy")}
        if "vocal_tract_length" in res or "speech_rate" in res or "voicing_probability" in res:
            feat.speech = {"speech_rate": sc("speech_rate"), "vocal_tract_length": sc("vocal_tract_length"),
                           "voicing_probability": vec("voicing_probability")}
        if "pitch_estimate" in res:
            feat.harmonic = {"harmonic_ratio": vec("harmonic_ratio"), "pitch_estimate": vec("pitch_estimate")}
        return Fingerprint(id=fid, content_type=content_type, duration=sc("duration_seconds"), features=feat)

    @staticmethod
    def fingerprint_from_pcm(ctx, pcm, sample_rate: int, content_type: str, fid: str) -> Fingerprint:
        """GenerateFingerprint (fingerprint.go:137) on the GPU, as a comparator input."""
        res = ctx.generate_fingerprint(pcm, sample_rate, content_type)
        return FingerprintComparator.fingerprint_from_result(res, fid, content_type)

    def validate_config(self):
        """ValidateConfig (:1208-1223)."""
        c = self.config
        if c["similarity_threshold"] < 0 or c["similarity_threshold"] > 1:
            raise SonarError(ERR_INVALID, "similarity threshold must be between 0 and 1: %f"
                             % c["similarity_threshold"])
        if c["max_candidates"] <= 0:
            raise SonarError(ERR_INVALID, "max candidates must be positive: %d" % c["max_candidates"])
        if c["method"] not in METHODS:
            raise SonarError(ERR_INVALID, "invalid method: %s (must be 'auto', 'fast', or 'precise')"
                             % c["method"])


def get_similarity_statistics(results: List[dict]) -> Dict[str, float]:
    """GetSimilarityStatistics (comparison.go:1154-1205); hash similarities are all 0."""
    if not results:
        return {}

    def stats(v):
        v = [float(x) for x in v]
        s = sorted(v)
        n = len(v)
        mean = math.fsum(v) / n if n else float("nan")
        var = float("nan")
        if n > 1:
            d = [x - mean for x in v]
            var = (sum(x * x for x in d) - sum(d) ** 2 / n) / (n - 1)
        cum, med = 0.0, s[-1]
        for x in s:                       # stat.Quantile(0.5, Empirical, sorted, nil)
            cum += 1
            if cum >= 0.5 * n:
                med = x
                break
        return {"mean": mean, "min": s[0], "max": s[-1], "median": med, "std": math.sqrt(var)}

    o = stats([r["overall_similarity"] for r in results])
    h = stats([0.0] * len(results))
    f = stats([r["feature_similarity"] for r in results])
    c = stats([r["confidence"] for r in results])
    return {"overall_mean": o["mean"], "overall_min": o["min"], "overall_max": o["max"],
            "overall_median": o["median"], "overall_std": o["std"], "hash_mean": h["mean"],
            "feature_mean": f["mean"], "confidence_mean": c["mean"], "total_comparisons": float(len(results))}


def device_features(G: int, F: int, device, seed: int = 0, content_types=("news", "music")):
    """Bench inputs: G speech-extractor-shaped fingerprints of F STFT frames generated on the
    device (MFCC F x 13, centroid/rolloff F, flux F-1, RMS F, voicing F, harmonic ratio and
    pitch F/2), as sonar_fp_features with device pointers.  Returns (buffer, structs, bytes
    of feature data per fingerprint)."""
    import torch
    Fp = max(1, F // 2)
    parts = [("mfcc", F * 13), ("spectral_centroid", F), ("spectral_rolloff", F), ("spectral_flux", F - 1),
             ("rms_energy", F), ("voicing_probability", F), ("harmonic_ratio", Fp), ("pitch_estimate", Fp)]
    per = sum(n for _, n in parts)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    buf = torch.randn(G, per, generator=gen, device=device, dtype=torch.float64).abs_()
    structs = (FpFeatures * G)()
    base = buf.data_ptr()
    for i in range(G):
        f = structs[i]
        f.id = i
        f.present = FEAT_FEATURES | FEAT_MFCC | FEAT_SPECTRAL | FEAT_TEMPORAL | FEAT_SPEECH | FEAT_HARMONIC
        f.content_type = content_code(content_types[i % len(content_types)])
        f.duration_seconds = F * 256 / 44100.0
        f.dynamic_range, f.silence_ratio, f.onset_density = 20.0 + i % 7, 0.1, 1.0 + i % 3
        f.speech_rate, f.vocal_tract_length = 3.0, 17.5
        off = base + i * per * 8
        for name, n in parts:
            if name == "mfcc":
                f.mfcc, f.mfcc_frames, f.mfcc_coeffs = off, F, 13
            else:
                setattr(f, name, off)
                setattr(f, "n_" + name, n)
            off += n * 8
    return buf, structs, per * 8
