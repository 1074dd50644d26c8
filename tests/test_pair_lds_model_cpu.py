"""The LDS bank-conflict model behind mfcc_pair_kernel's float64 layout (tools/pair_lds_model.py,
DESIGN.md Kernel 1a "LDS re-laid for 16-byte accesses"), and the layout constants the kernel and
the host tables share (csrc/kernels.h).  Layout-only phases need no filterbank, so the synthetic
chunk table below keeps this test fast; the measured counterparts are profiles/r06ap_* / r06aq_*."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pair_lds_model as M  # noqa: E402


def _table():
    ks = [min(512, 8 * l) for l in range(64)]
    src = [[2 * (m + k) for k in range(4)] for m in range(40)]
    return dict(J=12, JS=13, ks=ks, src=src, nf=40, NMP=40, MS=4)


def test_bank_model_primitives():
    # 16 lanes of one ds_read_b128 group on 16 distinct 16-B slots of a 256-B row: conflict-free
    g0 = M.B128_GROUPS[0]
    addr = [None] * 64
    for j, l in enumerate(g0):
        addr[l] = 16 * j
    assert M.extra("read_b128", addr) == 0
    # the same 16 lanes 256 B apart: one bank quad, 16 distinct dwords -> 15 extra cycles
    for j, l in enumerate(g0):
        addr[l] = 256 * j
    assert M.extra("read_b128", addr) == 15
    # identical addresses broadcast
    assert M.extra("read_b64", [0] * 64) == 0
    # ds_write_b128: 8 contiguous lanes, mod-32 banking: a 32-B lane stride wraps twice
    assert M.extra("write_b128", [32 * l for l in range(64)]) == 8


def test_float64_layout_phases():
    t = _table()
    old = M.model(t, True, tw2_row=8, dct_pad=4, pad=2, planes=False)
    new = M.model(t, True, tw2_row=9, dct_pad=2, pad=1, planes=True)
    # the stage-2 twiddle rows (ds_read2_b64, mod 32): 8-way at rows of 8 complex, none at 9
    assert old["tw2"] == 392 and new["tw2"] == 0
    assert old["dct_coef"] == 40 and new["dct_coef"] == 0
    assert old["partial_store"] == 16 and new["partial_store"] == 0
    assert old["power_store"] == 72 and new["power_store"] == 8
    assert new["t2_store"] == 0 and new["t2_load"] == 0


def test_float32_layout_unchanged():
    ph = M.model(_table(), False)
    assert ph["t2_store"] == 0 and ph["t2_load"] == 0 and ph["dct_coef"] == 0 and ph["partial_store"] == 0


def test_kernel_constants_match_the_model():
    src = open(os.path.join(ROOT, "sonido-sonar_amd", "csrc", "kernels.h")).read()
    assert re.search(r"mfcc_pair_pad_rows\(int f64\) \{ return f64 \? 1 : 2; \}", src)
    assert re.search(r"mfcc_pair_dct_pad\(int f64\) \{ return f64 \? 2 : 4; \}", src)
    assert re.search(r"kPairTw2Row = 9;", src)
