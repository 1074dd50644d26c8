"""LDS bank-conflict model of mfcc_pair_kernel's per-pair LDS accesses (CPU only).  Lane
addresses from the kernel's index formulas and the headline tables (40 mels at 44.1 kHz, W 1024,
the host's chunk builder restated); bank rules from MI355X_MICROARCH.md's LDS table.  Prints the
extra cycles per access kind per pair (what SQ_LDS_BANK_CONFLICT counts)."""
import sys, os
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "oracle")]
import oracle as O

K = 513
fb = np.asarray(O.filterbank(40, 1024, 44100, 0.0, 22050.0, "mel"))
lo = [int(np.flatnonzero(r)[0]) if r.any() else 0 for r in fb]
hi = [int(np.flatnonzero(r)[-1]) + 1 if r.any() else 0 for r in fb]
# the host's runs of bins whose nonzero filters fit one pair (sonar_api.cpp build_pair_tables)
segs = []
for k in range(K):
    act = [m for m in range(40) if lo[m] <= k < hi[m]]
    if not act:
        continue
    if segs and segs[-1][1] == k:
        g = segs[-1]
        u = [g[2]] + ([g[3]] if g[3] >= 0 else [])
        fits = len(act) >= len(u)
        for a in act:
            if a not in u:
                if len(u) == 2:
                    fits = False
                    break
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
ks = []
for g in segs:
    for k0 in range(g[0], g[1], J):
        ks.append(k0)
ks += [0] * (64 - len(ks))
print("J", J, "chunks", len(segs), "ks", ks)


def prow(k):
    return k + 2 * (k >> 4)


def conflicts(addrs, groups, bankmod, width_dw):
    """extra LDS cycles of one wave-instruction: per group, max over banks of distinct addresses - 1"""
    extra = 0
    for grp in groups:
        banks = {}
        for l in grp:
            a = addrs[l]
            if a is None:
                continue
            for d in range(width_dw):
                b = (a // 4 + d) % bankmod
                banks.setdefault(b, set()).add(a // 4 + d)
        extra += max((len(v) for v in banks.values()), default=1) - 1
    return extra


R64 = [list(range(32)), list(range(32, 64))]
W64 = [list(range(g, g + 16)) for g in (0, 16, 32, 48)]
R128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27], [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
R128 += [[x + 32 for x in g] for g in R128]
tot = {}
# filterbank reads: pr + 8 i + (i >= ib ? 16 : 0), pr = prow(ks) * 8
for i in range(J):
    addrs = []
    for l in range(64):
        ib = 16 - (ks[l] & 15)
        addrs.append(prow(ks[l]) * 8 + 8 * i + (16 if i >= ib else 0))
    tot["filterbank power reads (b64)"] = tot.get("filterbank power reads (b64)", 0) + conflicts(addrs, R64, 64, 2)
for k, v in tot.items():
    print(f"{k:40s} {v} extra cycles / pair")


def fb_cost(order):
    """filterbank read conflicts for lane -> chunk order"""
    c = 0
    for i in range(J):
        addrs = []
        for l in range(64):
            k = ks[order[l]]
            ib = 16 - (k & 15)
            addrs.append(prow(k) * 8 + 8 * i + (16 if i >= ib else 0))
        c += conflicts(addrs, R64, 64, 2)
    return c


order = list(range(64))
best = fb_cost(order)
improved = True
while improved:
    improved = False
    for a in range(32):
        for b in range(32, 64):
            o2 = order[:]
            o2[a], o2[b] = o2[b], o2[a]
            c = fb_cost(o2)
            if c < best:
                best, order, improved = c, o2, True
print("after swapping chunks between the two 32-lane groups:", best, "extra cycles / pair")
print("group 0 chunks:", sorted(order[:32]))

# ---- the other per-pair accesses (same formulas as mfcc_pair.hip) ----
kT2 = 136
irreg = [[63 * 136, 60 * 136, 61 * 136, 62 * 136, 63 * 136 + 64, 62 * 136 + 64, 61 * 136 + 64, 60 * 136 + 64],
         [56 * 136, 57 * 136, 58 * 136, 59 * 136, 59 * 136 + 64, 58 * 136 + 64, 57 * 136 + 64, 56 * 136 + 64]]
other = {}
def add(k, v):
    other[k] = other.get(k, 0) + v
for c in range(8):
    for h in range(2):
        addrs = []
        for l in range(64):
            b0, kl = l & 7, l >> 3
            if kl != 0:
                addrs.append(((kl - 1) * 8 * kT2 + 8 * b0 + kT2 * c) if h == 0 else ((7 - kl) * 8 * kT2 + 64 + 8 * b0 + kT2 * (7 - c)))
            else:
                addrs.append(8 * b0 + irreg[h][c])
        add("T2 writes (b64)", conflicts(addrs, W64, 32, 2))
for j in range(16):
    add("T2 reads (b64)", conflicts([l * kT2 + 8 * j for l in range(64)], R64, 64, 2))
rA = []
for l in range(64):
    if l < 56: rA.append((l >> 3) + 1 + 16 * (l & 7))
    elif l < 60: rA.append(8 + 16 * (l - 56))
    elif l < 63: rA.append(16 * (l - 59))
    else: rA.append(0)
rB = [64 if l == 63 else 128 - rA[l] for l in range(64)]
for c in range(4):
    add("power writes (b64)", conflicts([prow(rA[l]) * 8 + 1152 * c for l in range(64)], W64, 32, 2))
add("power writes (b64)", conflicts([prow(rB[l]) * 8 + 3456 for l in range(64)], W64, 32, 2))
for c in range(5, 8):
    add("power writes (b64)", conflicts([prow(rB[l]) * 8 + 1152 * (7 - c) for l in range(64)], W64, 32, 2))
add("power writes (b64)", conflicts([8 * (prow(512) if l == 63 else 18 * (l & 31) + 16 + (l >> 5)) for l in range(64)], W64, 32, 2))
for k, v in other.items():
    print(f"{k:40s} {v} extra cycles / pair")

# the host's search (sonar_api.cpp build_pair_tables): first-improvement swaps, kept in place
order = list(range(64))
best = fb_cost(order)
improved = True
while improved:
    improved = False
    for a in range(32):
        for b in range(32, 64):
            order[a], order[b] = order[b], order[a]
            c = fb_cost(order)
            if c < best:
                best, improved = c, True
            else:
                order[a], order[b] = order[b], order[a]
print("host search:", best, "extra cycles / pair (filterbank reads)")
