"""The library driven from C99 (tests/c_abi/demo.c, built by __graft_entry__.build() /
make -C tests/c_abi): sonar_create, sonar_fingerprint (path A), sonar_dtw (path B), Go's error
texts through sonar_last_error, sonar_destroy -- what a cgo caller does, with no Python between."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
CABI = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_abi")


def test_c99_consumer_runs():
    exe = os.path.join(CABI, "build", "demo")
    # a no-op when the binary is newer than demo.c, the header and the library
    subprocess.run(["make", "-s", "-C", CABI, "build/demo"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("demo ok"), r.stdout
