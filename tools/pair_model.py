"""Lane-level numpy model of mfcc_pair.hip's FFT data flow (index algebra check).

Emulates 64 lanes x 16 complex registers through pass 1, T1 (permlane32/16 swaps,
row_ror:8 exchange), pass 2, T2 (LDS combo layout), pass 3 and the pair split, and
checks the per-bin power of both frames against numpy.fft.rfft."""
import numpy as np

L = np.arange(64)


def dft(x, axis):  # forward DFT along axis
    return np.fft.fft(x, axis=axis)


def model(x0, x1):
    z = x0 + 1j * x1                       # windowing omitted (linear)
    v = np.empty((64, 16), complex)        # v[lane, reg]
    for a in range(16):
        v[:, a] = z[64 * a + L]
    v = dft(v, 1)                          # pass 1: DFT16 over a -> k1
    v *= np.exp(-2j * np.pi * np.outer(L, np.arange(16)) / 1024)
    # T1: reg bit2 <-> lane bit5 (permlane32_swap on (j, j+4))
    for j in range(16):
        if j & 4 == 0:
            a, b = v[:, j].copy(), v[:, j + 4].copy()
            v[:32, j], v[32:, j] = a[:32], b[:32]
            v[:32, j + 4], v[32:, j + 4] = a[32:], b[32:]
    for j in range(16):                    # reg bit1 <-> lane bit4 (permlane16_swap)
        if j & 2 == 0:
            a, b = v[:, j].copy(), v[:, j + 2].copy()
            na, nb = a.copy(), b.copy()
            for r in range(4):
                s = slice(16 * r, 16 * r + 16)
                if r % 2 == 0:
                    na[s] = a[s]; nb[s] = a[16 * (r + 1):16 * (r + 2)]
                else:
                    na[s] = b[16 * (r - 1):16 * r]; nb[s] = b[s]
            v[:, j], v[:, j + 2] = na, nb
    hi3 = (L & 8) != 0
    for j in range(0, 16, 2):              # reg bit0 <-> lane bit3 (row_ror:8 = lane ^ 8)
        a, b = v[:, j].copy(), v[:, j + 1].copy()
        v[:, j] = np.where(hi3, b[L ^ 8], a)
        v[:, j + 1] = np.where(hi3, b, a[L ^ 8])
    b0 = L & 7
    for h in range(2):                     # pass 2: DFT8 over b1 -> c0, twiddle w64^{b0 c0}
        v[:, 8 * h:8 * h + 8] = dft(v[:, 8 * h:8 * h + 8], 1)
        v[:, 8 * h:8 * h + 8] *= np.exp(-2j * np.pi * np.outer(b0, np.arange(8)) / 64)
    # T2 through a flat LDS image (float2 units, stride 17 per lane row)
    lds = np.full(64 * 17, np.nan, complex)
    irr = [[63 * 17, 60 * 17, 61 * 17, 62 * 17, 63 * 17 + 8, 62 * 17 + 8, 61 * 17 + 8, 60 * 17 + 8],
           [56 * 17, 57 * 17, 58 * 17, 59 * 17, 59 * 17 + 8, 58 * 17 + 8, 57 * 17 + 8, 56 * 17 + 8]]
    kl = L >> 3
    for lane in range(64):
        for c in range(8):
            if kl[lane] != 0:
                lds[(kl[lane] - 1) * 8 * 17 + b0[lane] + 17 * c] = v[lane, c]
                lds[(7 - kl[lane]) * 8 * 17 + 8 + b0[lane] + 17 * (7 - c)] = v[lane, 8 + c]
            else:
                lds[b0[lane] + irr[0][c]] = v[lane, c]
                lds[b0[lane] + irr[1][c]] = v[lane, 8 + c]
    assert not np.isnan(lds.reshape(64, 17)[:, :16]).any()
    v = np.stack([lds[lane * 17:lane * 17 + 16] for lane in range(64)])
    v[:, :8] = dft(v[:, :8], 1)           # pass 3
    v[:, 8:] = dft(v[:, 8:], 1)
    rA = np.where(L < 56, (L >> 3) + 1 + 16 * (L & 7), np.where(L < 60, 8 + 16 * (L - 56), np.where(L < 63, 16 * (L - 59), 0)))
    rB = np.where(L == 63, 64, 128 - rA)
    P0 = np.full(513, np.nan); P1 = np.full(513, np.nan)

    def pw(a, b, k):
        s = a + np.conj(b); d = a - np.conj(b)
        assert np.isnan(P0[k]), k
        P0[k] = abs(s) ** 2 / 4; P1[k] = abs(d) ** 2 / 4

    for lane in range(64):
        self = lane == 63
        A, B = v[lane, :8], v[lane, 8:]
        for c in range(4):
            pw(A[c], A[(8 - c) & 7] if self else B[7 - c], rA[lane] + 128 * c)
        pw(B[4] if self else A[4], B[3], rB[lane] + 384)
        for c in range(5, 8):
            pw(B[c] if self else A[c], B[7 - c], rB[lane] + 128 * (7 - c))
        if self:
            pw(A[4], A[4], 512)
    return P0, P1


rng = np.random.default_rng(0)
x0, x1 = rng.standard_normal(1024), rng.standard_normal(1024)
P0, P1 = model(x0, x1)
R0, R1 = abs(np.fft.rfft(x0)) ** 2, abs(np.fft.rfft(x1)) ** 2
print("max rel err frame t  :", np.max(abs(P0 - R0) / R0.max()))
print("max rel err frame t+1:", np.max(abs(P1 - R1) / R1.max()))
assert np.allclose(P0, R0, rtol=1e-9, atol=1e-9 * R0.max()) and np.allclose(P1, R1, rtol=1e-9, atol=1e-9 * R1.max())
print("pair model OK")
