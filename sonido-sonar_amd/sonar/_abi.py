"""ctypes binding of include/sonar_gpu.h (see package docstring)."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))       # sonido-sonar_amd/
_REPO = os.path.dirname(_PKG)
LIB_PATH = os.environ.get("SONAR_LIB") or os.path.join(_PKG, "lib", "libsonar_gpu.so")   # override: A/B builds
HEADER = os.path.join(_REPO, "include", "sonar_gpu.h")

OK, ERR_INVALID, ERR_TOO_SHORT, ERR_EMPTY, ERR_UNSUPPORTED, ERR_DEVICE, ERR_NOMEM = 0, -1, -2, -3, -4, -5, -6
ERR_PANIC = -7          # SONAR_ERR_PANIC: the Go reference panics on this input (message: its runtime error)
FP_MFCC, FP_MAGNITUDE, FP_SPECTRAL, FP_ZCR, FP_ENERGY, FP_COMPLEX, FP_PHASE = 1, 2, 4, 8, 16, 32, 64
FP_GENERIC = 1 << 30   # force the general fused kernel (A/B checks of the f32 MFCC path)
F32, F64 = 0, 1
INGEST_DEVICE_CONVERT, INGEST_HOST_CONVERT = 0, 1   # sonar_ingest_f64le modes
WINDOWS = {"hann": 0, "hamming": 1, "blackman": 2, "blackman_harris": 3, "kaiser": 4,
           "tukey": 5, "rectangular": 6, "bartlett": 7, "welch": 8}
SPECTRAL_NAMES = ["centroid", "rolloff", "bandwidth", "flatness", "crest", "slope", "flux",
                  "low_ratio", "high_ratio"]
NCC_KEYS = ["peak_correlation", "peak_lag", "peak_index", "p_value", "snr", "sharpness",
            "second_peak", "peak_to_sidelobe", "overlap_length", "num_lags"]


def _exported_symbols():
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(sonar_[a-z0-9_]+)\s*\(", txt)))


EXPORTED_SYMBOLS = _exported_symbols()


class SonarError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.msg = msg


class FpConfig(C.Structure):
    _fields_ = [("window_size", C.c_int32), ("hop_size", C.c_int32), ("window_type", C.c_int32),
                ("sample_rate", C.c_int32), ("n_mfcc", C.c_int32), ("n_filters", C.c_int32),
                ("filterbank", C.c_int32), ("use_lifter", C.c_int32), ("low_freq", C.c_double),
                ("high_freq", C.c_double), ("lifter", C.c_double), ("mfcc_input_power", C.c_int32),
                ("energy_window", C.c_int32), ("energy_hop", C.c_int32), ("preemph_alpha", C.c_double),
                ("flags", C.c_uint32), ("precision", C.c_int32), ("pcm_dtype", C.c_int32),
                ("out_dtype", C.c_int32), ("device_ptrs", C.c_int32)]


class FpOut(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["mfcc", "magnitude", "centroid", "rolloff", "bandwidth", "flatness",
                                          "crest", "slope", "flux", "low_ratio", "high_ratio", "zcr", "energy",
                                          "complex", "phase"]]


class FingerprintConfig(C.Structure):
    _fields_ = [("window_size", C.c_int32), ("hop_size", C.c_int32), ("feature_window_size", C.c_int32),
                ("feature_hop_size", C.c_int32), ("enable_content_detect", C.c_int32),
                ("window_type", C.c_int32), ("precision", C.c_int32),
                ("acoustic_detection", C.c_int32), ("default_content_type", C.c_int32),
                ("auto_detect_threshold", C.c_double), ("genre", C.c_char_p), ("station", C.c_char_p),
                ("url", C.c_char_p)]


class AcousticFeatures(C.Structure):
    """sonar_acoustic_features (content_detector.go:104-115)."""
    _fields_ = [(n, C.c_double) for n in ("zero_crossing_rate", "spectral_centroid", "energy_variance",
                                          "silence_ratio", "harmonic_ratio", "low_freq_energy", "high_freq_energy",
                                          "dynamic_range", "temporal_stability", "classification_confidence")]


CONTENT_NAMES = ["music", "news", "sports", "talk", "mixed", "unknown"]


class FeatureConfig(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ["sample_rate", "window_size", "hop_size", "stft_window_size",
                                         "stft_hop_size", "window_type", "enable_mfcc", "enable_speech_features",
                                         "enable_temporal_features", "mfcc_coefficients", "is_news", "precision"]]


class FormantFrame(C.Structure):
    _fields_ = [("status", C.c_int32), ("n_formants", C.c_int32), ("frequency", C.c_double * 4),
                ("bandwidth", C.c_double * 4), ("amplitude", C.c_double * 4), ("confidence", C.c_double * 4),
                ("vocal_tract_length", C.c_double), ("quality", C.c_double), ("gain", C.c_double),
                ("residual_energy", C.c_double), ("stable", C.c_int32), ("lpc_order", C.c_int32)]


class VoiceQuality(C.Structure):
    """sonar_voice_quality (speech.VoiceQualityResult, voice_quality.go:21-43)."""
    _fields_ = [(n, C.c_double) for n in ("jitter", "shimmer", "hnr", "noise_measure", "f0_stability",
                                          "amplitude_stability", "voicing_strength", "overall_quality")] + \
               [("num_periods", C.c_int64)] + \
               [(n, C.c_double) for n in ("mean_f0", "f0_range", "analysis_quality")]


class AlignmentStats(C.Structure):
    """sonar_alignment_stats (stats.AlignmentStats, alignment.go:700-707) + the offset and trials."""
    _fields_ = [(n, C.c_double) for n in ("mean_offset", "stddev_offset", "median_offset", "offset_range",
                                          "consistency")] + [("offset", C.c_int64), ("trials", C.c_int32)]


ALIGN_DTW, ALIGN_XCORR, ALIGN_PHASE, ALIGN_HYBRID = 0, 1, 2, 3


class FpFeatures(C.Structure):
    """sonar_fp_features (one AudioFingerprint as FingerprintComparator reads it)."""
    _fields_ = [("id", C.c_int64), ("present", C.c_uint32), ("content_type", C.c_int32),
                ("duration_seconds", C.c_double),
                ("mfcc", C.c_void_p), ("mfcc_frames", C.c_int64), ("mfcc_coeffs", C.c_int32),
                ("chroma", C.c_void_p), ("chroma_frames", C.c_int64), ("chroma_bins", C.c_int32),
                ("spectral_centroid", C.c_void_p), ("n_spectral_centroid", C.c_int64),
                ("spectral_rolloff", C.c_void_p), ("n_spectral_rolloff", C.c_int64),
                ("spectral_flux", C.c_void_p), ("n_spectral_flux", C.c_int64),
                ("dynamic_range", C.c_double), ("silence_ratio", C.c_double), ("onset_density", C.c_double),
                ("rms_energy", C.c_void_p), ("n_rms_energy", C.c_int64),
                ("speech_rate", C.c_double), ("vocal_tract_length", C.c_double),
                ("voicing_probability", C.c_void_p), ("n_voicing_probability", C.c_int64),
                ("harmonic_ratio", C.c_void_p), ("n_harmonic_ratio", C.c_int64),
                ("pitch_estimate", C.c_void_p), ("n_pitch_estimate", C.c_int64),
                ("feature_weights", C.c_double * 6)]


class CompareCfg(C.Structure):
    _fields_ = [("similarity_threshold", C.c_double), ("max_candidates", C.c_int32),
                ("enable_detailed_metrics", C.c_int32), ("enable_content_filter", C.c_int32),
                ("method", C.c_int32)]


class Similarity(C.Structure):
    _fields_ = [("overall_similarity", C.c_double), ("feature_similarity", C.c_double),
                ("confidence", C.c_double), ("feature_distances", C.c_double * 6),
                ("data_availability", C.c_double), ("feature_coverage", C.c_double),
                ("temporal_alignment", C.c_double), ("noise_level", C.c_double),
                ("dynamic_range_match", C.c_double), ("spectral_coherence", C.c_double),
                ("distance_mask", C.c_uint32), ("content_type_match", C.c_int32),
                ("has_quality", C.c_int32), ("status", C.c_int32)]


class Match(C.Structure):
    _fields_ = [("candidate", C.c_int64), ("rank", C.c_int32), ("match_type", C.c_int32),
                ("similarity", Similarity)]


class PairRecord(C.Structure):
    """sonar_pair_record: what ExtractAlignmentFeatures leaves per pair (extractors/alignment.go:139-219)."""
    _fields_ = [(n, C.c_double) for n in ("temporal_offset", "offset_confidence", "alignment_similarity",
                                          "alignment_quality", "method", "corr_offset_seconds", "dtw_distance",
                                          "peak_lag")] + [("status", C.c_int32), ("flags", C.c_int32)]


PAIR_FIELDS = [f for f, _ in PairRecord._fields_[:8]]
PAIR_REDONE_TIMEOUT = 1     # sonar_pair_record.flags (include/sonar_gpu.h)
PAIR_REDONE_NONFINITE = 2

_lib = None
_vp, _d, _i32p, _i64p = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_int64)


def build():
    """Compile libsonar_gpu.so in-tree for gfx950 (hipcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-j8", "-C", _PKG], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SonarError(ERR_DEVICE, f"{LIB_PATH} not built: run `make -C sonido-sonar_amd` "
                                     "(there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    L.sonar_create.argtypes = [C.c_int, C.POINTER(_vp)]
    L.sonar_destroy.argtypes = [_vp]
    L.sonar_destroy.restype = None
    L.sonar_last_error.argtypes = [_vp]
    L.sonar_last_error.restype = C.c_char_p
    L.sonar_set_stream.argtypes = [_vp, _vp]
    L.sonar_synchronize.argtypes = [_vp]
    L.sonar_last_kernel_ms.argtypes = [_vp, _d]
    L.sonar_enable_kernel_timing.argtypes = [_vp, C.c_int]
    L.sonar_dtw_last_timing.argtypes = [_vp, C.POINTER(C.c_double)]
    if hasattr(L, "sonar_dtw_counters"):      # (absent from A/B builds of earlier rounds)
        L.sonar_dtw_counters.argtypes = [_vp, C.POINTER(C.c_int64), C.c_int32]
    if hasattr(L, "sonar_trim"):
        L.sonar_trim.argtypes = [_vp]
    L.sonar_last_fp_kernel.argtypes = [_vp]
    L.sonar_last_fp_kernel.restype = C.c_char_p
    for f in ("sonar_stft_frames", "sonar_energy_frames"):
        getattr(L, f).argtypes = [C.c_int64, C.c_int32, C.c_int32]
        getattr(L, f).restype = C.c_int64
    L.sonar_pitch_frames.argtypes = [C.c_int64]
    L.sonar_pitch_frames.restype = C.c_int64
    L.sonar_fp_cfg_default.argtypes = [C.POINTER(FpConfig)]
    L.sonar_fp_cfg_default.restype = None
    L.sonar_stft_stream_create.argtypes = [_vp, C.POINTER(FpConfig), C.POINTER(_vp)]
    L.sonar_stft_stream_frames.argtypes = [_vp, C.c_int64]
    L.sonar_stft_stream_frames.restype = C.c_int64
    L.sonar_stft_stream_buffered.argtypes = [_vp]
    L.sonar_stft_stream_buffered.restype = C.c_int64
    L.sonar_stft_stream_push.argtypes = [_vp, _vp, C.c_int64, C.POINTER(FpOut), C.POINTER(C.c_int64)]
    L.sonar_stft_stream_destroy.argtypes = [_vp]
    L.sonar_stft_stream_destroy.restype = None
    L.sonar_fp_kernel_plan.argtypes = [C.POINTER(FpConfig), C.c_int64]
    L.sonar_fp_kernel_plan.restype = C.c_int32
    L.sonar_fingerprint.argtypes = [_vp, _vp, C.c_int64, C.POINTER(FpConfig), C.POINTER(FpOut)]
    L.sonar_fingerprint_batch.argtypes = [_vp, C.POINTER(_vp), C.POINTER(C.c_int64), C.c_int32,
                                          C.POINTER(FpConfig), C.POINTER(FpOut)]
    L.sonar_pitch_yin.argtypes = [_vp, _vp, C.c_int64, C.c_int32, _vp, _vp, _vp, C.c_int32]
    L.sonar_chroma_stft.argtypes = [_vp, _vp, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _vp, C.c_int32]
    L.sonar_ncc.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int32, _vp, _vp, C.c_int32]
    L.sonar_music_alignment_features.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                                 C.c_int32, _vp, _vp, C.c_int32]
    L.sonar_dtw.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int32, C.c_int32, _d, _vp, _vp, _vp, _i64p,
                            _vp, C.c_int32]
    L.sonar_fingerprint_config_default.argtypes = [C.POINTER(FingerprintConfig)]
    L.sonar_fingerprint_config_default.restype = None
    L.sonar_generate_fingerprint.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.c_char_p,
                                             C.POINTER(FingerprintConfig), C.POINTER(_vp)]
    L.sonar_feature_config_default.argtypes = [C.POINTER(FeatureConfig)]
    L.sonar_feature_config_default.restype = None
    L.sonar_extract_speech_features.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.POINTER(FeatureConfig),
                                                C.POINTER(_vp)]
    if hasattr(L, "sonar_extract_music_features"):
        L.sonar_extract_music_features.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.POINTER(FeatureConfig),
                                                   C.POINTER(_vp)]
    L.sonar_align_features.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, _vp, C.c_int64, _vp, C.c_int64,
                                       C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                       C.c_double, C.POINTER(_vp)]
    L.sonar_formant_frame_count.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32]
    L.sonar_formant_frame_count.restype = C.c_int64
    L.sonar_formants.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp, C.c_int32]
    L.sonar_align_pair_device.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                          C.c_int32, C.c_double, C.POINTER(C.c_void_p)]
    _pairs = [C.c_int64, C.POINTER(C.c_void_p), _i64p, C.POINTER(C.c_void_p), _i64p, C.c_int32, C.c_int32,
              C.c_int32, C.c_int32, C.c_double, C.c_int32]
    L.sonar_align_pairs.argtypes = [_vp] + _pairs + [C.c_int32, C.POINTER(PairRecord)]
    L.sonar_align_pairs_multi.argtypes = [_vp] + _pairs + [C.POINTER(PairRecord)]
    L.sonar_multi_create.argtypes = [_i32p, C.c_int32, C.POINTER(C.c_void_p)]
    L.sonar_multi_destroy.argtypes = [_vp]
    L.sonar_multi_destroy.restype = None
    L.sonar_multi_last_error.argtypes = [_vp]
    L.sonar_multi_last_error.restype = C.c_char_p
    L.sonar_multi_size.argtypes = [_vp]
    L.sonar_multi_ctx.argtypes = [_vp, C.c_int32]
    L.sonar_multi_ctx.restype = _vp
    L.sonar_multi_shard.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _i64p, _i64p, _i64p,
                                    _i64p]
    L.sonar_fingerprint_multi.argtypes = [_vp, _vp, C.c_int64, C.POINTER(FpConfig), C.POINTER(FpOut)]
    L.sonar_fingerprint_multi_gather.argtypes = [_vp, C.POINTER(C.c_void_p), C.c_int64, C.POINTER(FpConfig),
                                                 C.POINTER(C.c_void_p)]
    L.sonar_alignment_consistency.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                              C.c_int32, C.c_int32, C.c_int32, C.POINTER(AlignmentStats)]
    L.sonar_analyzer_align_features.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                                C.c_int32, C.c_int32, C.c_int32, C.POINTER(_vp)]
    L.sonar_align_audio.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                    C.c_int32, C.c_int32, C.POINTER(_vp)]
    L.sonar_align_audio_files.argtypes = [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                          C.c_int32, C.c_double, C.c_int32, C.POINTER(_vp)]
    L.sonar_truncate_to_alignment.argtypes = [_vp, C.c_int64, C.c_int64, C.c_int32, C.c_double,
                                              C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.sonar_voice_quality.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.POINTER(VoiceQuality)]
    L.sonar_fingerprint_f64le.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.POINTER(FpConfig), C.POINTER(FpOut)]
    L.sonar_ingest_f64le.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _vp, _i64p]
    L.sonar_detect_from_audio.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.c_double, _i32p,
                                          C.POINTER(AcousticFeatures)]
    L.sonar_detect_content_type.argtypes = [_vp, _vp, C.c_int64, C.c_int32, C.c_int32, C.c_char_p, C.c_char_p,
                                            C.c_char_p, C.c_char_p, C.c_int32, C.c_int32, C.c_double, _i32p]
    L.sonar_gallery_create.argtypes = [_vp, C.POINTER(_vp)]
    L.sonar_gallery_destroy.argtypes = [_vp]
    L.sonar_gallery_destroy.restype = None
    L.sonar_gallery_size.argtypes = [_vp]
    L.sonar_gallery_size.restype = C.c_int64
    L.sonar_gallery_add.argtypes = [_vp, C.POINTER(FpFeatures), C.c_int32, C.c_int32, C.c_int32, _i64p]
    L.sonar_compare.argtypes = [_vp, _i64p, C.c_int64, _i64p, C.c_int64, C.POINTER(CompareCfg), _vp, C.c_int32]
    L.sonar_find_best_matches.argtypes = [_vp, _i64p, C.c_int64, _i64p, C.c_int64, C.POINTER(CompareCfg),
                                          C.POINTER(Match), _i64p]
    L.sonar_merge_matches.argtypes = [C.POINTER(C.c_void_p), _i64p, _i64p, C.c_int32, C.c_int64, C.c_int32,
                                      C.POINTER(Match), _i64p]
    L.sonar_find_best_matches_multi.argtypes = [_vp, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int64,
                                                C.POINTER(C.c_void_p), _i64p, C.POINTER(CompareCfg),
                                                C.POINTER(Match), _i64p]
    L.sonar_result_get.argtypes = [_vp, C.c_char_p, C.POINTER(_d), _i64p, _i64p]
    L.sonar_result_count.argtypes = [_vp]
    L.sonar_result_name.argtypes = [_vp, C.c_int]
    L.sonar_result_name.restype = C.c_char_p
    L.sonar_result_free.argtypes = [_vp]
    L.sonar_result_free.restype = None
    _lib = L
    return L


def _formant_dict(recs, F):
    a = np.ctypeslib.as_array(recs)[:F] if F else np.zeros(0, dtype=np.dtype(FormantFrame))
    return {k: np.array(a[k]) for k in ("status", "n_formants", "frequency", "bandwidth", "amplitude", "confidence",
                                        "vocal_tract_length", "quality", "gain", "residual_energy", "stable")}


def abi_version():
    return lib().sonar_abi_version()


def stft_frames(n, W, H):
    return int(lib().sonar_stft_frames(n, W, H))


PLAN_NONE, PLAN_PAIR, PLAN_WAVE, PLAN_DFT = 0, 1, 2, 3
PAIR_MAX_FRAMES = 2147483646          # SONAR_PAIR_MAX_FRAMES: mfcc_pair_kernel's 32-bit frame indices


def fp_kernel_plan(cfg, n):
    """sonar_fp_kernel_plan: the transform kernel sonar_fingerprint runs for (cfg, n) (host logic)."""
    return int(lib().sonar_fp_kernel_plan(C.byref(cfg), n))


def energy_frames(n, W, H):
    return int(lib().sonar_energy_frames(n, W, H))


def pitch_frames(n):
    return int(lib().sonar_pitch_frames(n))


def multi_shard(n, W, H, n_shards, shard):
    """sonar_multi_shard: (f0, f1, s0, s1) of frame shard `shard` of `n_shards` (pure arithmetic)."""
    v = [C.c_int64() for _ in range(4)]
    rc = lib().sonar_multi_shard(n, W, H, n_shards, shard, *[C.byref(x) for x in v])
    if rc != OK:
        raise SonarError(rc, "sonar_multi_shard")
    return tuple(x.value for x in v)


def _pair_arrays(qs, rs):
    """ctypes pointer/length arrays of two lists of streams (device int pointers or numpy arrays)."""
    keep = []

    def ptr(x):
        if isinstance(x, (int, np.integer)):
            return int(x)
        a = _f64(x)
        keep.append(a)
        return a.ctypes.data
    n = len(qs)
    qp = (C.c_void_p * n)(*[ptr(x) for x in qs])
    rp = (C.c_void_p * n)(*[ptr(x) for x in rs])
    return qp, rp, keep


def records_dict(recs):
    """sonar_pair_record array -> dict of numpy arrays (PAIR_FIELDS + status)."""
    out = {f: np.array([getattr(r, f) for r in recs]) for f in PAIR_FIELDS}
    out["status"] = np.array([r.status for r in recs], dtype=np.int32)
    out["flags"] = np.array([r.flags for r in recs], dtype=np.int32)
    return out


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class _ResultOwner:
    """Owns a sonar_result handle; freed (sonar_result_free) when no view of it remains."""
    def __init__(self, L, h):
        self._L, self._h = L, h

    def __del__(self):
        if self._h:
            self._L.sonar_result_free(self._h)
            self._h = None


class _ResultView:
    """numpy's array interface over one result array; the array's base keeps the owner alive."""
    def __init__(self, owner, addr, shape):
        self._owner = owner
        self.__array_interface__ = {"shape": shape, "typestr": "<f8", "data": (addr, False), "version": 3}


def _pcm_arg(x, device_ptrs):
    """(pointer, length, owner) of a PCM argument: a host float64 array, or (device pointer, n); the
    caller keeps `owner` alive across the call (a converted copy)."""
    if device_ptrs:
        p, n = x
        return C.c_void_p(int(p)), int(n), None
    a = _f64(x)
    return (_ptr(a) if a.size else None), int(a.size), a


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Context:
    """One sonar_ctx (one HIP stream) on `device`."""

    def __init__(self, device=0):
        L = lib()
        h = C.c_void_p()
        rc = L.sonar_create(device, C.byref(h))
        if rc != OK:
            raise SonarError(rc, "sonar_create failed (no GPU visible?)")
        self._h = h
        self._L = L

    @classmethod
    def wrap(cls, handle, owner=None):
        """A non-owning Context over an existing sonar_ctx (e.g. sonar_multi_ctx); `owner` is kept
        alive with it.  close() does not destroy the handle."""
        self = cls.__new__(cls)
        self._h = handle if isinstance(handle, C.c_void_p) else C.c_void_p(handle)
        self._L = lib()
        self._borrowed = owner if owner is not None else True
        return self

    def close(self):
        if getattr(self, "_h", None):
            if not getattr(self, "_borrowed", None):
                self._L.sonar_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != OK:
            raise SonarError(rc, self._L.sonar_last_error(self._h).decode())

    # -- stream / timing -------------------------------------------------
    def set_stream(self, stream_handle):
        self._check(self._L.sonar_set_stream(self._h, C.c_void_p(stream_handle or 0) if stream_handle else None))

    def synchronize(self):
        self._check(self._L.sonar_synchronize(self._h))

    def enable_kernel_timing(self, on=True):
        self._check(self._L.sonar_enable_kernel_timing(self._h, int(on)))

    def last_kernel_ms(self):
        v = C.c_double()
        self._check(self._L.sonar_last_kernel_ms(self._h, C.byref(v)))
        return v.value

    def dtw_last_timing(self):
        """(band sweep, walk, path decode) kernel ms of the last dtw call (HIP events)."""
        v = (C.c_double * 3)()
        self._check(self._L.sonar_dtw_last_timing(self._h, v))
        return tuple(v)

    def dtw_counters(self, reset=False):
        """Band-pipeline liveness counters since the last reset (sonar_dtw_counters): edge refresh
        fences, fences followed by new edge values, timed-out DTWs, timed-out waves."""
        v = (C.c_int64 * 4)()
        self._check(self._L.sonar_dtw_counters(self._h, v, int(bool(reset))))
        return {"edge_refresh_fences": v[0], "edge_refresh_hits": v[1], "dtw_timeouts": v[2],
                "waves_timed_out": v[3]}

    def trim(self):
        """Free the device / pinned host buffers this context and its pair workers cache
        (sonar_trim); the next call allocates again."""
        self._check(self._L.sonar_trim(self._h))

    def last_fp_kernel(self):
        """Name of the fused kernel the last fingerprint call launched (diagnostics)."""
        return self._L.sonar_last_fp_kernel(self._h).decode()

    # -- path A ------------------------------------------------------------
    @staticmethod
    def config(**kw):
        cfg = FpConfig()
        lib().sonar_fp_cfg_default(C.byref(cfg))
        for k, v in kw.items():
            if k == "window_type" and isinstance(v, str):
                v = WINDOWS[v]
            setattr(cfg, k, v)
        return cfg

    def fingerprint(self, pcm, cfg: FpConfig):
        """Host-buffer form: returns a dict of numpy arrays for the requested flags."""
        pcm = np.ascontiguousarray(pcm, dtype=np.float64 if cfg.pcm_dtype == F64 else np.float32)
        n = len(pcm)
        cfg.device_ptrs = 0
        res, out = self._fp_outputs(n, cfg)
        self._check(self._L.sonar_fingerprint(self._h, _ptr(pcm) if n else None, n, C.byref(cfg), C.byref(out)))
        return res

    def fingerprint_batch(self, signals, cfg: FpConfig):
        """sonar_fingerprint_batch (SpectralAnalyzer.ComputeSTFTBatch, spectral.go:234-285), host
        buffers: one dict of numpy arrays per signal, as fingerprint() returns."""
        dt = np.float64 if cfg.pcm_dtype == F64 else np.float32
        sigs = [np.ascontiguousarray(x, dtype=dt) for x in signals]
        cfg.device_ptrs = 0
        k = len(sigs)
        ptrs = (_vp * max(k, 1))(*[x.ctypes.data if x.size else None for x in sigs])
        ns = (C.c_int64 * max(k, 1))(*[x.size for x in sigs])
        outs = (FpOut * max(k, 1))()
        res = []
        for i, x in enumerate(sigs):
            r, o = self._fp_outputs(x.size, cfg)
            res.append(r)
            outs[i] = o
        self._check(self._L.sonar_fingerprint_batch(self._h, ptrs, ns, k, C.byref(cfg), outs))
        return res

    def fingerprint_batch_device(self, pcm_ptrs, ns, mfcc_ptrs, cfg: FpConfig):
        """Device-pointer form (async on the ctx stream): MFCC outputs only (mfcc_ptrs[i] -> F_i x n_mfcc)."""
        cfg.device_ptrs = 1
        k = len(pcm_ptrs)
        outs = (FpOut * max(k, 1))()
        for i, m in enumerate(mfcc_ptrs):
            outs[i].mfcc = m
        self._check(self._L.sonar_fingerprint_batch(self._h, (_vp * max(k, 1))(*pcm_ptrs),
                                                    (C.c_int64 * max(k, 1))(*ns), k, C.byref(cfg), outs))

    def fingerprint_f64le(self, data, cfg: FpConfig, mode=INGEST_HOST_CONVERT):
        """sonar_fingerprint_f64le: the decoder's f64le bytes (decoder.go:850-871) straight into path A."""
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
            else np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        cfg.device_ptrs = 0
        res, out = self._fp_outputs(buf.size // 8, cfg)
        self._check(self._L.sonar_fingerprint_f64le(self._h, buf.ctypes.data if buf.size else None, buf.size, mode,
                                                    C.byref(cfg), C.byref(out)))
        return res

    def _fp_outputs(self, n, cfg, frames=None):
        if frames is not None:
            F = frames
        else:
            F = stft_frames(n, cfg.window_size, cfg.hop_size) if n > 0 and cfg.window_size > 0 and cfg.hop_size > 0 else 0
        od = np.float64 if cfg.out_dtype == F64 else np.float32
        out, res = FpOut(), {}
        if F > 0:
            K = cfg.window_size // 2 + 1
            nm = cfg.n_mfcc if cfg.n_mfcc > 0 else 13
            if cfg.flags & FP_MFCC:
                res["mfcc"] = np.zeros((F, nm), od)
                out.mfcc = res["mfcc"].ctypes.data
            if cfg.flags & FP_MAGNITUDE:
                res["magnitude"] = np.zeros((F, K), od)
                out.magnitude = res["magnitude"].ctypes.data
            if cfg.flags & FP_COMPLEX:      # (re, im) interleaved: a complex view of an F x K x 2 array
                res["complex"] = np.zeros((F, K, 2), od)
                out.complex = res["complex"].ctypes.data
            if cfg.flags & FP_PHASE:
                res["phase"] = np.zeros((F, K), od)
                out.phase = res["phase"].ctypes.data
            if cfg.flags & FP_SPECTRAL:
                for nme in SPECTRAL_NAMES:
                    res[nme] = np.zeros(max(F - 1, 0) if nme == "flux" else F, od)
                    setattr(out, nme, res[nme].ctypes.data if res[nme].size else None)
            if cfg.flags & FP_ZCR:
                res["zcr"] = np.zeros(F, od)
                out.zcr = res["zcr"].ctypes.data
            if cfg.flags & FP_ENERGY:
                fe = energy_frames(n, cfg.energy_window, cfg.energy_hop)
                res["energy"] = np.zeros(fe, od)
                out.energy = res["energy"].ctypes.data if fe > 0 else None
        return res, out

    def stft_stream(self, cfg: FpConfig):
        """sonar_stft_stream_create: SpectralAnalyzer.ComputeSTFTStreaming (spectral.go:287-312)."""
        h = C.c_void_p()
        self._check(self._L.sonar_stft_stream_create(self._h, C.byref(cfg), C.byref(h)))
        return StftStream(self, h, cfg)

    def fingerprint_device(self, pcm_ptr, n, cfg: FpConfig, **out_ptrs):
        """Device-pointer form (async on the ctx stream): out_ptrs name -> device address."""
        cfg.device_ptrs = 1
        out = FpOut()
        for k, v in out_ptrs.items():
            setattr(out, k, v)
        self._check(self._L.sonar_fingerprint(self._h, C.c_void_p(pcm_ptr), n, C.byref(cfg), C.byref(out)))

    def pitch_yin(self, pcm, sample_rate):
        pcm = _f64(pcm)
        F = pitch_frames(len(pcm))
        p, c, t = np.zeros(F), np.zeros(F), np.zeros(F, np.int32)
        self._check(self._L.sonar_pitch_yin(self._h, _ptr(pcm), len(pcm), sample_rate, _ptr(p), _ptr(c), _ptr(t), 0))
        return p, c, t

    def chroma_stft(self, pcm, n_frames, hop, sample_rate, preprocess=True):
        pcm = _f64(pcm)
        out = np.zeros((n_frames, 12))
        self._check(self._L.sonar_chroma_stft(self._h, _ptr(pcm), len(pcm), n_frames, hop, sample_rate,
                                              int(preprocess), _ptr(out), 0))
        return out

    def music_alignment_features(self, pcm, sample_rate, stft_window=1024, stft_hop=256, feature_window=1024,
                                 feature_hop=256):
        """MusicFeatureExtractor's ShortTimeEnergy + ChromaFeatures (host arrays) -> (energy, chroma)."""
        pcm = _f64(pcm)
        n = len(pcm)
        F = stft_frames(n, stft_window, stft_hop) if n > 0 else 0
        energy = np.zeros(max(energy_frames(n, feature_window, feature_hop), 0))
        chroma = np.zeros((max(F, 0), 12))
        self._check(self._L.sonar_music_alignment_features(
            self._h, _ptr(pcm) if n else None, n, sample_rate, stft_window, stft_hop, feature_window, feature_hop,
            _ptr(energy) if len(energy) else None, _ptr(chroma) if len(chroma) else None, 0))
        return energy, chroma

    def music_alignment_features_device(self, pcm_ptr, n, sample_rate, energy_ptr, chroma_ptr, stft_window=1024,
                                        stft_hop=256, feature_window=1024, feature_hop=256):
        """Device-pointer form (float64 buffers, async on the ctx stream)."""
        self._check(self._L.sonar_music_alignment_features(
            self._h, C.c_void_p(pcm_ptr), n, sample_rate, stft_window, stft_hop, feature_window, feature_hop,
            C.c_void_p(energy_ptr), C.c_void_p(chroma_ptr), 1))

    def align_pair_device(self, q_ptr, nq, r_ptr, nr, sample_rate=44100, stft_window=1024, hop=256,
                          feature_window=1024, max_lag_seconds=60.0):
        """sonar_align_pair_device: music features + ExtractAlignmentFeatures of one pair of
        device-resident float64 streams; returns the align_features result dict."""
        h = C.c_void_p()
        self._check(self._L.sonar_align_pair_device(self._h, C.c_void_p(q_ptr), nq, C.c_void_p(r_ptr), nr, sample_rate,
                                                    stft_window, hop, feature_window, max_lag_seconds, C.byref(h)))
        return self._result(h)

    def align_pairs(self, qs, rs, nq=None, nr=None, sample_rate=44100, stft_window=1024, hop=256,
                    feature_window=1024, max_lag_seconds=20.0, workers=128, device_ptrs=False):
        """sonar_align_pairs: records of many pairs (workers = pairs in flight).  qs / rs: lists of host arrays, or of device
        pointers (ints) with device_ptrs=True and the lengths in nq / nr."""
        n = len(qs)
        qp, rp, keep = _pair_arrays(qs, rs)
        nqa = (C.c_int64 * n)(*(nq if nq is not None else [len(x) for x in qs]))
        nra = (C.c_int64 * n)(*(nr if nr is not None else [len(x) for x in rs]))
        recs = (PairRecord * max(n, 1))()
        self._check(self._L.sonar_align_pairs(self._h, n, qp, nqa, rp, nra, sample_rate, stft_window, hop,
                                              feature_window, max_lag_seconds, workers, int(bool(device_ptrs)),
                                              recs))
        del keep
        return records_dict(recs[:n])

    # -- path B ------------------------------------------------------------
    def ncc(self, a, b, max_lag):
        a, b = _f64(a), _f64(b)
        L = max(0, min(max_lag, len(a) - 1, len(b) - 1)) if len(a) and len(b) else 0
        corr = np.zeros(2 * L + 1)
        met = np.zeros(10)
        self._check(self._L.sonar_ncc(self._h, _ptr(a) if len(a) else None, len(a), _ptr(b) if len(b) else None,
                                      len(b), max_lag, _ptr(corr), _ptr(met), 0))
        return corr, dict(zip(NCC_KEYS, met.tolist()))

    def formants(self, pcm, sample_rate, frame_size=0, hop_size=0, want_lpc=False):
        """FormantAnalyzer.AnalyzeMultipleFrames; every attempted frame, `status` != 0 where Go skips."""
        pcm = _f64(pcm)
        L = lib()
        F = int(L.sonar_formant_frame_count(len(pcm), sample_rate, frame_size, hop_size))
        recs = (FormantFrame * max(F, 1))()
        p = 12 + sample_rate // 1000
        co = np.zeros((F, p + 1)) if want_lpc else None
        rf = np.zeros((F, p)) if want_lpc else None
        self._check(L.sonar_formants(self._h, _ptr(pcm), len(pcm), sample_rate, frame_size, hop_size, recs,
                                     _ptr(co) if want_lpc else None, _ptr(rf) if want_lpc else None, 0))
        out = _formant_dict(recs, F)
        if want_lpc:
            out["lpc_coeffs"], out["reflection"] = co, rf
        return out

    def alignment_consistency(self, query, reference, sample_rate, method=ALIGN_XCORR, max_lag=100, hop=256,
                              num_trials=5):
        """AlignmentAnalyzer.AnalyzeAlignmentConsistency -> dict of AlignmentStats (+ offset, trials)."""
        q, r = _f64(query), _f64(reference)
        if q.ndim == 1:
            q = q[:, None]
        if r.ndim == 1:
            r = r[:, None]
        st = AlignmentStats()
        self._check(self._L.sonar_alignment_consistency(
            self._h, _ptr(q) if q.size else None, len(q), _ptr(r) if r.size else None, len(r),
            q.shape[1] if q.size else 1, method, max_lag, hop, sample_rate, num_trials, C.byref(st)))
        return {k: getattr(st, k) for k, _ in AlignmentStats._fields_}

    def analyzer_align_features(self, query, reference, sample_rate, method=ALIGN_HYBRID, max_lag=100, hop=256):
        """AlignmentAnalyzer.AlignFeatures (stats/alignment.go:84-106) for DTW / CrossCorrelation /
        Hybrid -> the AlignmentResult fields (+ "correlations", NCC metrics, "dtw_path_*")."""
        q, r = _f64(query), _f64(reference)
        if q.ndim == 1:
            q = q[:, None]
        if r.ndim == 1:
            r = r[:, None]
        h = C.c_void_p()
        self._check(self._L.sonar_analyzer_align_features(
            self._h, _ptr(q) if q.size else None, len(q) if q.size else 0, _ptr(r) if r.size else None,
            len(r) if r.size else 0, q.shape[1] if q.size else 1, method, max_lag, hop, sample_rate, 0, C.byref(h)))
        return self._result(h)

    def align_audio(self, q_pcm, r_pcm, sample_rate, method=ALIGN_HYBRID, max_lag=100, hop=256, window=1024,
                    device_ptrs=False):
        """AlignmentAnalyzer.AlignAudio (stats/alignment.go:108-126): RMS energy frames of both signals
        (extractEnergyFeatures :341-361), then AlignFeatures.  q_pcm / r_pcm: float64 arrays, or device
        pointers (ints) with lengths as (ptr, n) tuples when device_ptrs."""
        (qp, nq, qa), (rp, nr, ra) = _pcm_arg(q_pcm, device_ptrs), _pcm_arg(r_pcm, device_ptrs)
        h = C.c_void_p()
        self._check(self._L.sonar_align_audio(self._h, qp, nq, rp, nr, method, max_lag, hop, window, sample_rate,
                                              int(device_ptrs), C.byref(h)))
        del qa, ra
        return self._result(h)

    def align_audio_files(self, q_pcm, r_pcm, sample_rate, feature_sample_rate=None, hop=256, window=1024,
                          max_lag_seconds=60.0, device_ptrs=False):
        """AlignmentExtractor.AlignAudioFiles (extractors/alignment.go:489-553): ShortTimeEnergy of
        both PCM streams, then the extractor's Hybrid AlignFeatures."""
        (qp, nq, qa), (rp, nr, ra) = _pcm_arg(q_pcm, device_ptrs), _pcm_arg(r_pcm, device_ptrs)
        fsr = sample_rate if feature_sample_rate is None else feature_sample_rate
        h = C.c_void_p()
        self._check(self._L.sonar_align_audio_files(self._h, qp, nq, rp, nr, sample_rate, fsr, hop, window,
                                                    float(max_lag_seconds), int(device_ptrs), C.byref(h)))
        del qa, ra
        return self._result(h)

    def truncate_to_alignment(self, n1, n2, sample_rate, temporal_offset):
        """AlignmentExtractor.TruncateToAlignmentPCM -> (start1, start2, length)."""
        a, b, n = C.c_int64(), C.c_int64(), C.c_int64()
        self._check(self._L.sonar_truncate_to_alignment(self._h, n1, n2, sample_rate, temporal_offset, C.byref(a),
                                                        C.byref(b), C.byref(n)))
        return a.value, b.value, n.value

    def ingest_f64le(self, data, d_out=None, out_dtype=F32, mode=INGEST_DEVICE_CONVERT, host_threads=0):
        """Decoder.bytesToFloat64 (decoder.go:850-871) into device memory: `data` is the ffmpeg f64le
        byte stream (bytes / bytearray / uint8 or float64 array), `d_out` a device pointer of
        n * (4 if out_dtype == F32 else 8) bytes (None: only count).  Returns the sample count."""
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
            else np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        n = C.c_int64()
        self._check(self._L.sonar_ingest_f64le(self._h, buf.ctypes.data if buf.size else None, buf.size, out_dtype,
                                               mode, host_threads, d_out, C.byref(n)))
        return n.value

    def voice_quality(self, signal, sample_rate):
        """VoiceQualityAnalyzer.AnalyzeVoiceQuality -> dict of VoiceQualityResult fields."""
        x = _f64(signal)
        q = VoiceQuality()
        self._check(self._L.sonar_voice_quality(self._h, _ptr(x) if len(x) else None, len(x), sample_rate,
                                                C.byref(q)))
        return {k: getattr(q, k) for k, _ in VoiceQuality._fields_}

    def dtw(self, q, r, band=-1, want_cost=False):
        q, r = _f64(q), _f64(r)
        if q.ndim == 1:
            q = q[:, None]
        if r.ndim == 1:
            r = r[:, None]
        nq, d = q.shape if q.size else (0, 1)
        nr = r.shape[0] if r.size else 0
        cap = nq + nr + 1
        pq, pr, pc = np.zeros(cap, np.int32), np.zeros(cap, np.int32), np.zeros(cap)
        plen, dist = C.c_int64(), C.c_double()
        cost = np.zeros((nq, nr + 1)) if want_cost else None
        self._check(self._L.sonar_dtw(self._h, _ptr(q) if nq else None, nq, _ptr(r) if nr else None, nr, d, band,
                                      C.byref(dist), _ptr(pq), _ptr(pr), _ptr(pc), C.byref(plen),
                                      _ptr(cost) if want_cost else None, 0))
        P = plen.value
        return {"distance": dist.value, "path_q": pq[:P], "path_r": pr[:P], "path_cost": pc[:P], "cost": cost}

    # -- Go API mirror -----------------------------------------------------
    def _result(self, h):
        """The result's arrays as numpy views of its memory (no copy; large arrays live in pinned
        host memory the device copied into); the handle is freed when the last view goes."""
        L = self._L
        owner = _ResultOwner(L, h)
        out = {}
        for i in range(L.sonar_result_count(h)):
            name = L.sonar_result_name(h, i).decode()
            data, rows, cols = _d(), C.c_int64(), C.c_int64()
            L.sonar_result_get(h, name.encode(), C.byref(data), C.byref(rows), C.byref(cols))
            n = rows.value * cols.value
            shape = (rows.value, cols.value) if cols.value > 1 else (n,)
            addr = C.cast(data, C.c_void_p).value
            out[name] = np.asarray(_ResultView(owner, addr, shape)) if n else np.zeros(0)
        return out

    @staticmethod
    def fingerprint_config(**kw):
        cfg = FingerprintConfig()
        lib().sonar_fingerprint_config_default(C.byref(cfg))
        for k, v in kw.items():
            setattr(cfg, k, v)
        return cfg

    def generate_fingerprint(self, pcm, sample_rate, content_type, cfg: FingerprintConfig = None):
        pcm = _f64(pcm)
        cfg = cfg or self.fingerprint_config()
        h = C.c_void_p()
        self._check(self._L.sonar_generate_fingerprint(self._h, _ptr(pcm) if len(pcm) else None, len(pcm),
                                                       sample_rate, content_type.encode(), C.byref(cfg),
                                                       C.byref(h)))
        return self._result(h)

    def detect_from_audio(self, pcm, sample_rate, auto_detect_threshold=2.0):
        """ContentDetector.DetectFromAudio -> (content type name, AcousticFeatures dict)."""
        pcm = _f64(pcm)
        ct = C.c_int32()
        f = AcousticFeatures()
        self._check(self._L.sonar_detect_from_audio(self._h, _ptr(pcm) if len(pcm) else None, len(pcm), sample_rate,
                                                    auto_detect_threshold, C.byref(ct), C.byref(f)))
        return CONTENT_NAMES[ct.value], {k: getattr(f, k) for k, _ in AcousticFeatures._fields_}

    def detect_content_type(self, pcm, sample_rate, metadata=None, acoustic_detection=True,
                            default_content_type="unknown", auto_detect_threshold=2.0):
        """ContentDetector.DetectContentType; metadata = dict(content_type, genre, station, url) or None."""
        pcm = _f64(pcm)
        ct = C.c_int32()
        md = metadata or {}
        enc = lambda k: md.get(k, "").encode() if md.get(k) else None  # noqa: E731
        self._check(self._L.sonar_detect_content_type(
            self._h, _ptr(pcm) if len(pcm) else None, len(pcm), sample_rate, int(metadata is not None),
            enc("content_type"), enc("genre"), enc("station"), enc("url"), int(acoustic_detection),
            CONTENT_NAMES.index(default_content_type), auto_detect_threshold, C.byref(ct)))
        return CONTENT_NAMES[ct.value]

    @staticmethod
    def feature_config(**kw):
        cfg = FeatureConfig()
        lib().sonar_feature_config_default(C.byref(cfg))
        for k, v in kw.items():
            setattr(cfg, k, v)
        return cfg

    def extract_speech_features(self, pcm, sample_rate, cfg: FeatureConfig = None):
        pcm = _f64(pcm)
        cfg = cfg or self.feature_config()
        h = C.c_void_p()
        self._check(self._L.sonar_extract_speech_features(self._h, _ptr(pcm) if len(pcm) else None, len(pcm),
                                                          sample_rate, C.byref(cfg), C.byref(h)))
        return self._result(h)

    def extract_music_features(self, pcm, sample_rate, cfg: FeatureConfig = None):
        """sonar_extract_music_features: MusicFeatureExtractor.ExtractFeatures as a dict of arrays.
        Where the Go reference panics (SONAR_ERR_PANIC) this raises SonarError whose .partial holds
        the arrays computed before the panic."""
        pcm = _f64(pcm)
        cfg = cfg or self.feature_config()
        h = C.c_void_p()
        rc = self._L.sonar_extract_music_features(self._h, _ptr(pcm) if len(pcm) else None, len(pcm), sample_rate,
                                                  C.byref(cfg), C.byref(h))
        partial = self._result(h) if h.value else None
        if rc != OK:
            err = SonarError(rc, self._L.sonar_last_error(self._h).decode())
            err.partial = partial
            raise err
        return partial

    def align_features(self, q_energy, r_energy, q_chroma=None, r_chroma=None, q_pcm_len=0, r_pcm_len=0,
                       sample_rate=44100, feature_sample_rate=44100, hop_size=256, window_size=1024,
                       max_lag_seconds=60.0):
        qe, re_ = _f64(q_energy), _f64(r_energy)
        qc = _f64(q_chroma) if q_chroma is not None else np.zeros((0, 12))
        rc = _f64(r_chroma) if r_chroma is not None else np.zeros((0, 12))
        h = C.c_void_p()
        self._check(self._L.sonar_align_features(
            self._h, _ptr(qe) if len(qe) else None, len(qe), _ptr(re_) if len(re_) else None, len(re_),
            _ptr(qc) if len(qc) else None, len(qc), _ptr(rc) if len(rc) else None, len(rc),
            q_pcm_len, r_pcm_len, sample_rate, feature_sample_rate, hop_size, window_size, max_lag_seconds,
            C.byref(h)))
        return self._result(h)


class StftStream:
    """STFTStreamer (fingerprint/analyzers/spectral.go:314-366) over sonar_stft_stream_*: push(chunk)
    is ProcessChunk and returns the emitted frames as a dict of arrays (the cfg's outputs, rows =
    frames; empty arrays when no frame is complete).  Host buffers (cfg.device_ptrs = 0) unless
    push_device is used."""

    def __init__(self, ctx, h, cfg):
        self._ctx, self._h, self.cfg = ctx, h, cfg

    def frames(self, n):
        return int(self._ctx._L.sonar_stft_stream_frames(self._h, n))

    @property
    def buffered(self):
        return int(self._ctx._L.sonar_stft_stream_buffered(self._h))

    def push(self, chunk):
        cfg = self.cfg
        x = np.ascontiguousarray(chunk, dtype=np.float64 if cfg.pcm_dtype == F64 else np.float32)
        n = len(x)
        F = self.frames(n)
        res, out = self._ctx._fp_outputs(n, cfg, frames=max(F, 0))
        got = C.c_int64()
        self._ctx._check(self._ctx._L.sonar_stft_stream_push(self._h, _ptr(x) if n else None, n, C.byref(out),
                                                             C.byref(got)))
        assert got.value == max(F, 0), (got.value, F)
        return res

    def push_device(self, ptr, n, **out_ptrs):
        """Device chunk and outputs (cfg.device_ptrs must be 1): async on the ctx stream; returns the
        number of frames written."""
        out = FpOut()
        for k, v in out_ptrs.items():
            setattr(out, k, v)
        got = C.c_int64()
        self._ctx._check(self._ctx._L.sonar_stft_stream_push(self._h, C.c_void_p(ptr), n, C.byref(out), C.byref(got)))
        return got.value

    def close(self):
        if getattr(self, "_h", None):
            self._ctx._L.sonar_stft_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """sonar_multi: one context per device + an RCCL communicator over them (one process)."""

    def __init__(self, devices):
        L = lib()
        devs = (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        rc = L.sonar_multi_create(devs, len(devices), C.byref(h))
        if rc != OK:
            raise SonarError(rc, "sonar_multi_create failed (GPUs / RCCL)")
        self._h, self._L, self.devices = h, L, list(devices)

    def close(self):
        if getattr(self, "_h", None):
            self._L.sonar_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != OK:
            raise SonarError(rc, self._L.sonar_multi_last_error(self._h).decode())

    def size(self):
        return int(self._L.sonar_multi_size(self._h))

    def ctx(self, rank):
        """Rank `rank`'s context (sonar_multi_ctx) as a non-owning Context."""
        return Context.wrap(self._L.sonar_multi_ctx(self._h, rank), owner=self)

    def find_best_matches(self, galleries, queries, candidates, cfg):
        """sonar_find_best_matches_multi: galleries[g] on rank g (sonar.compare.Gallery built on
        Context wrappers of sonar_multi_ctx), queries[g] the queries' indices in galleries[g],
        candidates[g] rank g's candidates (None: the whole gallery).  Returns per query the merged
        Match list (candidates numbered globally, rank g's after ranks 0..g-1)."""
        G = len(galleries)
        nq = len(queries[0])
        qs = [np.ascontiguousarray(q, dtype=np.int64) for q in queries]
        cs = None if candidates is None else [np.ascontiguousarray(c, dtype=np.int64) for c in candidates]
        nc = np.array([len(g) if cs is None else len(cs[i]) for i, g in enumerate(galleries)], dtype=np.int64)
        gp = (C.c_void_p * G)(*[g._h.value for g in galleries])
        qp = (C.c_void_p * G)(*[q.ctypes.data for q in qs])
        cp = None if cs is None else (C.c_void_p * G)(*[c.ctypes.data if len(c) else None for c in cs])
        K = max(0, cfg.max_candidates)
        out = (Match * max(1, nq * K))()
        nm = np.zeros(max(1, nq), dtype=np.int64)
        self._check(self._L.sonar_find_best_matches_multi(self._h, gp, qp, nq, cp, nc.ctypes.data_as(_i64p),
                                                          C.byref(cfg), out, nm.ctypes.data_as(_i64p)))
        return [[out[i * K + k] for k in range(int(nm[i]))] for i in range(nq)]

    def fingerprint(self, pcm, cfg: FpConfig):
        """sonar_fingerprint_multi (host PCM, host outputs): MFCC / magnitude / descriptors."""
        F = stft_frames(len(pcm), cfg.window_size, cfg.hop_size)
        if F <= 0:
            raise SonarError(-2, "signal too short for given window size and hop size")
        pdt = np.float32 if cfg.pcm_dtype == F32 else np.float64
        odt = np.float32 if cfg.out_dtype == F32 else np.float64
        x = np.ascontiguousarray(pcm, dtype=pdt)
        res, o = {}, FpOut()
        if cfg.flags & FP_MFCC:
            res["mfcc"] = np.zeros((F, cfg.n_mfcc if cfg.n_mfcc > 0 else 13), odt)
            o.mfcc = res["mfcc"].ctypes.data
        if cfg.flags & FP_MAGNITUDE:
            res["magnitude"] = np.zeros((F, cfg.window_size // 2 + 1), odt)
            o.magnitude = res["magnitude"].ctypes.data
        if cfg.flags & FP_COMPLEX:
            res["complex"] = np.zeros((F, cfg.window_size // 2 + 1, 2), odt)
            o.complex = res["complex"].ctypes.data
        if cfg.flags & FP_PHASE:
            res["phase"] = np.zeros((F, cfg.window_size // 2 + 1), odt)
            o.phase = res["phase"].ctypes.data
        if cfg.flags & FP_SPECTRAL:
            for k in ("centroid", "rolloff", "bandwidth", "flatness", "crest", "slope", "low_ratio", "high_ratio"):
                res[k] = np.zeros(F, odt)
                setattr(o, k, res[k].ctypes.data)
        self._check(self._L.sonar_fingerprint_multi(self._h, x.ctypes.data, len(x), C.byref(cfg), C.byref(o)))
        return res

    def fingerprint_gather(self, pcm_ptrs, n, cfg: FpConfig, mfcc_ptrs):
        """sonar_fingerprint_multi_gather: device slices in, the MFCC timeline on every device."""
        G = len(pcm_ptrs)
        pp = (C.c_void_p * G)(*pcm_ptrs)
        mp = (C.c_void_p * G)(*mfcc_ptrs)
        self._check(self._L.sonar_fingerprint_multi_gather(self._h, pp, n, C.byref(cfg), mp))

    def align_pairs(self, qs, rs, sample_rate=44100, stft_window=1024, hop=256, feature_window=1024,
                    max_lag_seconds=20.0, workers=128):
        """sonar_align_pairs_multi: host streams, pair ranges per device, records all-gathered over RCCL."""
        n = len(qs)
        qp, rp, keep = _pair_arrays(qs, rs)
        nqa = (C.c_int64 * n)(*[len(x) for x in qs])
        nra = (C.c_int64 * n)(*[len(x) for x in rs])
        recs = (PairRecord * max(n, 1))()
        self._check(self._L.sonar_align_pairs_multi(self._h, n, qp, nqa, rp, nra, sample_rate, stft_window, hop,
                                                    feature_window, max_lag_seconds, workers, recs))
        del keep
        return records_dict(recs[:n])
