#!/usr/bin/env python3
"""LDS bank-conflict model of one mfcc_pair_kernel pair (csrc/mfcc_pair.hip), per phase and per instance.

Replays the byte addresses every LDS instruction of one pair issues (the instruction kinds are the
ones the compiler emits: hipcc -S of mfcc_pair.hip, tools/isa_count.py) and counts the extra LDS
cycles the lane groups of each kind cost, with the banking table of MI355X_MICROARCH.md §LDS:
  read_b64   2 x 32 lanes, bank = dword mod 64        read_b128 4 x 16 (the table's groups), mod 64
  read2_b64  two accesses, each 4 x 16 contiguous, mod 32
  write_b32  2 x 32, mod 32   write_b64 4 x 16 contiguous, mod 32   write_b128 8 x 8 contiguous, mod 32
Extra cycles of a group = (most distinct dwords on one bank) - 1, summed over groups -- the
quantity SQ_LDS_BANK_CONFLICT counts.  The chunk tables (lane order, sources) are rebuilt here as
build_pair_tables (csrc/sonar_api.cpp) builds them, from the oracle's filterbank.

Usage: python tools/pair_lds_model.py [sample_rate n_filters]   (default 44100 40, the headline bank)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def _oracle():
    """the oracle's filterbank (test/tool infrastructure only); imported on use"""
    try:
        from oracle import oracle as o
    except ImportError:          # tests put oracle/ itself on sys.path
        import oracle as o
    return o

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]


def groups(kind):
    if kind in ("read_b64", "write_b32", "read_b32"):
        return [list(range(0, 32)), list(range(32, 64))]
    if kind == "read_b128":
        return B128_GROUPS
    if kind in ("write_b64", "read2_b64"):
        return [list(range(16 * i, 16 * i + 16)) for i in range(4)]
    if kind == "write_b128":
        return [list(range(8 * i, 8 * i + 8)) for i in range(8)]
    raise ValueError(kind)


MOD = {"read_b64": 64, "read_b128": 64, "read2_b64": 32, "write_b32": 32, "read_b32": 32, "write_b64": 32,
       "write_b128": 32}
WIDTH = {"read_b64": 2, "read_b128": 4, "read2_b64": 2, "write_b32": 1, "read_b32": 1, "write_b64": 2,
         "write_b128": 4}


def extra(kind, addr):
    """addr: 64 byte addresses (None = lane inactive) -> extra LDS cycles of one wave-instruction"""
    if kind == "read2_b64":   # two accesses, the second 8 bytes on
        return extra("_r2", addr) + extra("_r2", [None if a is None else a + 8 for a in addr])
    k = "read2_b64" if kind == "_r2" else kind
    tot = 0
    for g in groups(k):
        banks = {}
        for l in g:
            if addr[l] is None:
                continue
            d0 = addr[l] // 4
            for d in range(d0, d0 + WIDTH[k]):
                banks.setdefault(d % MOD[k], set()).add(d)
        if banks:
            tot += max(len(s) for s in banks.values()) - 1
    return tot


PAD = {False: 2, True: 2}     # pad rows per 16 power rows, per instance (float64: True)


def prow(k, pad=2):
    return k + pad * (k >> 4)


def tables(sr, nf, W=1024, order_kind="b64", pad=2):
    K = W // 2 + 1
    fb = _oracle().filterbank(nf, W, sr, 0.0, sr / 2.0)
    lo, hi = [], []
    for m in range(nf):
        nz = np.nonzero(fb[m])[0]
        lo.append(int(nz[0]) if len(nz) else 0)
        hi.append(int(nz[-1]) + 1 if len(nz) else 0)
    segs = []
    for k in range(K):
        act = [m for m in range(nf) if lo[m] <= k < hi[m]]
        if not act:
            continue
        if segs and segs[-1][1] == k:
            g = segs[-1]
            u = [g[2]] + ([g[3]] if g[3] >= 0 else [])
            fits = len(act) >= len(u)
            for a in act:
                if fits and a not in u:
                    if len(u) == 2:
                        fits = False
                    else:
                        u.append(a)
            if fits:
                g[1] = k + 1
                if len(u) == 2:
                    g[2], g[3] = min(u), max(u)
                continue
        segs.append([k, k + 1, act[0], act[1] if len(act) > 1 else -1])
    J = 1
    while sum((g[1] - g[0] + J - 1) // J for g in segs) > 64:
        J += 1
    chunks = [(k0, gi) for gi, g in enumerate(segs) for k0 in range(g[0], g[1], J)]
    chunks += [(0, -1)] * (64 - len(chunks))
    order = list(range(64))

    def fb_cost(o):
        if order_kind == "b64":
            tot = 0
            for i in range(J):
                a = [None] * 64
                for l in range(64):
                    k = chunks[o[l]][0]
                    a[l] = 8 * prow(k) + 8 * i + (16 if i >= 16 - (k & 15) else 0)
                tot += extra("read_b64", a)
            return tot
        tot = 0
        for i in range(J):
            a = [None] * 64
            for l in range(64):
                k = chunks[o[l]][0]
                a[l] = 16 * prow(k, pad) + 16 * i + (16 * pad if i >= 16 - (k & 15) else 0)
            tot += extra("read_b128", a)
        return tot

    best, improved = fb_cost(order), True
    pairs = ([(a, b) for a in range(32) for b in range(32, 64)] if order_kind == "b64"
             else [(a, b) for a in range(64) for b in range(a + 1, 64)])
    while improved:
        improved = False
        for a, b in pairs:
            order[a], order[b] = order[b], order[a]
            c = fb_cost(order)
            if c < best:
                best, improved = c, True
            else:
                order[a], order[b] = order[b], order[a]
    lane_of = [0] * 64
    for l in range(64):
        lane_of[order[l]] = l
    ks = [0] * 64
    src = [[] for _ in range(nf)]
    for ci, (k0, gi) in enumerate(chunks):
        if gi < 0:
            continue
        lane = lane_of[ci]
        ks[lane] = k0
        src[segs[gi][2]].append(2 * lane)
        if segs[gi][3] >= 0:
            src[segs[gi][3]].append(2 * lane + 1)
    return dict(J=J, JS=J | 1, ks=ks, src=src, nf=nf, NMP=(nf + 7) // 8 * 8,
                MS=max(len(s) for s in src))


T2_IRREG = [[63 * 136, 60 * 136, 61 * 136, 62 * 136, 63 * 136 + 64, 62 * 136 + 64, 61 * 136 + 64, 60 * 136 + 64],
            [56 * 136, 57 * 136, 58 * 136, 59 * 136, 59 * 136 + 64, 58 * 136 + 64, 57 * 136 + 64, 56 * 136 + 64]]


def model(t, f64, tw2_row=8, dct_pad=4, pad=2, planes=False):
    ES = 8 if f64 else 4
    CB, T2S, PB = 2 * ES, 34 * ES, 2 * ES
    PartOff, R128 = 600 * PB, 8 * (16 + pad) * PB

    def prow(k):
        return k + pad * (k >> 4)
    LogOff = PartOff + 256 * ES
    J, JS, NMP, nf = t["J"], t["JS"], t["NMP"], t["nf"]
    rd2 = "read_b128" if f64 else "read_b64"
    wr2 = "write_b128" if f64 else "write_b64"
    ph = {}

    def add(name, kind, addr):
        ph[name] = ph.get(name, 0) + extra(kind, addr)

    # T2 transpose: regular lanes (kl != 0) and the irregular lanes 0-7 as two instruction streams
    for c in range(8):
        for h in range(2):
            a = [None] * 64
            b = [None] * 64
            for l in range(64):
                b0, kl = l & 7, l >> 3
                if kl:
                    a[l] = ((kl - 1) * 8 * T2S + CB * b0 + T2S * c) if h == 0 else \
                        ((7 - kl) * 8 * T2S + 8 * CB + CB * b0 + T2S * (7 - c))
                else:
                    b[l] = CB * b0 + T2_IRREG[h][c] * (CB // 8)
            add("t2_store", wr2, a)
            add("t2_store", wr2, b)
    for j in range(16):
        add("t2_load", rd2, [l * T2S + CB * j for l in range(64)])
    # power rows
    rA = []
    for l in range(64):
        rA.append((l >> 3) + 1 + 16 * (l & 7) if l < 56 else 8 + 16 * (l - 56) if l < 60 else
                  16 * (l - 59) if l < 63 else 0)
    rB = [64 if l == 63 else 128 - rA[l] for l in range(64)]
    pA = [prow(r) * PB for r in rA]
    pB = [prow(r) * PB for r in rB]
    for c in range(4):
        add("power_store", wr2, [pA[l] + R128 * c for l in range(64)])
    for c in range(4, 8):
        add("power_store", wr2, [pB[l] + R128 * (7 - c) for l in range(64)])
    if pad == 2:
        add("power_store", wr2, [PB * (prow(512) if l == 63 else 18 * (l & 31) + 16 + (l >> 5)) for l in range(64)])
    # (pad 1: only lane 63 stores bin 512)
    # filterbank: power rows and weights
    for i in range(J):
        add("fb_power", rd2, [PB * prow(k) + PB * i + (pad * PB if i >= 16 - (k & 15) else 0) for k in t["ks"]])
        add("fb_weight", rd2, [(l * JS + i) * CB for l in range(64)])
    if f64 and planes:
        add("partial_store", "write_b128", [PartOff + 16 * l for l in range(64)])
        add("partial_store", "write_b128", [PartOff + 1024 + 16 * l for l in range(64)])
    elif f64:
        add("partial_store", "write_b128", [PartOff + 32 * l for l in range(64)])
        add("partial_store", "write_b128", [PartOff + 32 * l + 16 for l in range(64)])
    else:
        add("partial_store", "write_b128", [PartOff + 16 * l for l in range(64)])
    # ln: lane = filter, its sources
    for i in range(t["MS"]):
        a = [None] * 64
        for m in range(nf):
            s = t["src"][m]
            if i >= len(s):
                a[m] = 64 * T2S
            elif planes:
                a[m] = PartOff + 16 * (s[i] >> 1) + 1024 * (s[i] & 1)
            else:
                a[m] = PartOff + 2 * ES * s[i]
        for m in range(nf, NMP):
            a[m] = 64 * T2S
        add("ln_load", rd2, a)
    wl = "write_b64" if f64 else "write_b32"
    add("logmel_store", wl, [LogOff + ES * l if l < NMP else None for l in range(64)])
    add("logmel_store", wl, [LogOff + ES * (NMP + l) if l < NMP else None for l in range(64)])
    # DCT
    half = NMP // 2
    dct0 = 1 << 20   # a separate table: only its relative addresses matter
    for m in range(0, half, 4):
        for sub in ((0, 2) if f64 else (0,)):
            add("dct_logmel", "read_b128",
                [LogOff + ES * (((l >> 4) & 1) * NMP + (l >> 5) * half + m + sub) for l in range(64)])
            add("dct_coef", "read_b128",
                [dct0 + ES * ((l & 15) * (NMP + dct_pad) + (l >> 5) * half + m + sub) for l in range(64)])
    if f64:
        for c in range(1, 8):
            add("tw2", "read2_b64", [((l & 7) * tw2_row + c) * 16 for l in range(64)])
    return ph


def main():
    sr, nf = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (44100, 40)
    t32 = tables(sr, nf, order_kind="b64")
    print(f"bank {sr} Hz x {nf}: J {t32['J']}  NMP {t32['NMP']}  max sources {t32['MS']}")
    rows = [("float32", model(t32, False)), ("float64 (as built)", model(t32, True))]
    rows.append(("float64, tw2 rows of 9 + DCT pad 2", model(t32, True, tw2_row=9, dct_pad=2)))
    rows.append(("  + 1 pad row + partial planes", model(t32, True, tw2_row=9, dct_pad=2, pad=1, planes=True)))
    t64 = tables(sr, nf, order_kind="b128", pad=1)
    rows.append(("  + b128 lane order", model(t64, True, tw2_row=9, dct_pad=2, pad=1, planes=True)))
    t64b = tables(sr, nf, order_kind="b128", pad=2)
    rows.append(("  (2 pad rows, b128 lane order, planes)", model(t64b, True, tw2_row=9, dct_pad=2, pad=2, planes=True)))
    for name, ph in rows:
        print(f"{name:55s} total {sum(ph.values()):4d}  " + "  ".join(f"{k} {v}" for k, v in ph.items()))


if __name__ == "__main__":
    main()
