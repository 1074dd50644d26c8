"""sonar -- Python view of the MI355X sonido-sonar hot path.

Thin ctypes binding over the C ABI in include/sonar_gpu.h (library
sonido-sonar_amd/lib/libsonar_gpu.so).  Names and argument meaning follow the
Go reference (RyanBlaney/sonido-sonar) so that tests read like the reference's
API:  ``Context.fingerprint`` ~ ComputeSTFTWithWindow + MFCC.ComputeFrames,
``Context.ncc`` ~ CrossCorrelation.Compute, ``Context.dtw`` ~ DTWAlignment.Align,
``Context.generate_fingerprint`` ~ FingerprintGenerator.GenerateFingerprint,
``Context.align_features`` ~ AlignmentExtractor.ExtractAlignmentFeatures.

There is no CPU fallback: if the shared library is missing or no GPU is
visible, calls raise.
"""
from ._abi import (  # noqa: F401
    LIB_PATH,
    SonarError,
    Context,
    Multi,
    FpConfig,
    PairRecord,
    PAIR_FIELDS,
    PAIR_REDONE_NONFINITE,
    PAIR_REDONE_TIMEOUT,
    multi_shard,
    WINDOWS,
    abi_version,
    build,
    lib,
    stft_frames,
    energy_frames,
    pitch_frames,
    fp_kernel_plan,
    PLAN_NONE,
    PLAN_PAIR,
    PLAN_WAVE,
    PLAN_DFT,
    PAIR_MAX_FRAMES,
    FP_MFCC,
    FP_MAGNITUDE,
    FP_SPECTRAL,
    FP_ZCR,
    FP_ENERGY,
    FP_COMPLEX,
    FP_PHASE,
    FP_GENERIC,
    F32,
    F64,
    INGEST_DEVICE_CONVERT,
    INGEST_HOST_CONVERT,
    ERR_INVALID,
    ERR_EMPTY,
    ERR_TOO_SHORT,
    ERR_PANIC,
    EXPORTED_SYMBOLS,
)
