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
    assert sonar.abi_version() == 2
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
