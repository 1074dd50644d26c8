"""CPU: the C-ABI library loads and exports every symbol include/sonar_gpu.h
declares; size helpers follow Go's integer rules.  No compute call needs a GPU."""
import ctypes

import pytest

import sonar


def test_library_exports_header_symbols():
    L = ctypes.CDLL(sonar.LIB_PATH)
    missing = [s for s in sonar.EXPORTED_SYMBOLS if not hasattr(L, s)]
    assert not missing, missing
    assert len(sonar.EXPORTED_SYMBOLS) >= 20


def test_abi_version_and_sizes():
    assert sonar.abi_version() == 4
    assert sonar.stft_frames(441000, 1024, 256) == 1719
    assert sonar.stft_frames(1000, 1024, 256) == 1        # Go truncating division
    assert sonar.stft_frames(0, 1024, 256) < 0
    assert sonar.energy_frames(1000, 1024, 256) == 0
    assert sonar.energy_frames(441000, 1024, 256) == 1719
    assert sonar.pitch_frames(28_800_000) == 56_249
    assert sonar.pitch_frames(600) == 1 and sonar.pitch_frames(400) == 0


def test_context_creation_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(sonar.SonarError):
        sonar.Context(0)


# ---- the header as C sees it (cgo compiles the sonar_gpu.h preamble as C) --------------------
import os  # noqa: E402
import subprocess  # noqa: E402

from sonar import _abi  # noqa: E402

CABI = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_abi")
MIRRORS = {"sonar_fp_cfg": _abi.FpConfig, "sonar_fp_out": _abi.FpOut, "sonar_formant_frame": _abi.FormantFrame,
           "sonar_voice_quality_result": _abi.VoiceQuality, "sonar_fingerprint_config": _abi.FingerprintConfig,
           "sonar_feature_config": _abi.FeatureConfig, "sonar_alignment_stats": _abi.AlignmentStats,
           "sonar_acoustic_features": _abi.AcousticFeatures, "sonar_fp_features": _abi.FpFeatures,
           "sonar_compare_cfg": _abi.CompareCfg, "sonar_similarity": _abi.Similarity, "sonar_match": _abi.Match,
           "sonar_pair_record": _abi.PairRecord}


def _c_layout():
    subprocess.run(["make", "-s", "-C", CABI, "build/layout"], check=True)
    out = subprocess.run([os.path.join(CABI, "build", "layout")], check=True, capture_output=True, text=True).stdout
    sizes, offs = {}, {}
    for line in out.splitlines():
        kind, name, val = line.split()
        if kind == "struct":
            sizes[name] = int(val)
        else:
            s, m = name.split(".")
            offs.setdefault(s, []).append((m, int(val)))
    return sizes, offs


def test_header_compiles_as_c99_pedantic():
    """gcc -std=c99 -Wall -Wextra -Werror -pedantic accepts the header (layout.c pins every size)."""
    sizes, _ = _c_layout()
    assert set(sizes) == set(MIRRORS)


def test_ctypes_mirrors_match_c_layout():
    sizes, offs = _c_layout()
    for cname, cls in MIRRORS.items():
        assert ctypes.sizeof(cls) == sizes[cname], (cname, ctypes.sizeof(cls), sizes[cname])
        names = [f[0] for f in cls._fields_]
        assert names == [m for m, _ in offs[cname]], (cname, names)
        for m, off in offs[cname]:
            assert getattr(cls, m).offset == off, (cname, m, getattr(cls, m).offset, off)


def test_exported_symbols_are_the_header_declarations():
    import re
    with open(os.path.join(os.path.dirname(CABI), "..", "include", "sonar_gpu.h")) as f:
        text = f.read()
    decl = set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(sonar_[a-z_0-9]+)\s*\(", text, re.M))
    assert decl == set(sonar.EXPORTED_SYMBOLS), decl ^ set(sonar.EXPORTED_SYMBOLS)
