"""CPU model of the DTW backtrack by bands (align_kernels.hip: dtw_exit_map_kernel,
dtw_walk_chain_kernel, dtw_walk_band_kernel) against the serial backtrack (dtw.go:165-188, the
one-wave dtw_walk_kernel) on arbitrary direction-code matrices.

The band form rests on one recurrence: X(l, j), the column at which the path from cell
(64b+1+l, j) reaches row 64b, is X(l-1, j) for an up code, X(l, j-1) for left and X(l-1, j-1) for
diagonal, with X(-1, j) = j and X(l, 0) = 0.  The GPU evaluates it per 1,024-column segment with
the left edge as symbols; this model does the same (small segments, so symbols cross several
segments) and checks that chain + per-band walks reproduce the serial move stream exactly."""
import numpy as np
import pytest

UP, LEFT, DIAG = 0, 1, 2


def serial_walk(codes, nq, nr):
    """Moves of the serial backtrack from (nq, nr); codes[i, j] for 1 <= i <= nq, 1 <= j <= nr."""
    i, j, moves = nq, nr, []
    while i > 0 and j > 0:
        c = codes[i, j]
        moves.append(c)
        if c == UP:
            i -= 1
        elif c == LEFT:
            j -= 1
        else:
            i -= 1
            j -= 1
    while i > 0 or j > 0:                       # findPreviousStep on the borders
        moves.append(LEFT if i == 0 else UP)
        if i == 0:
            j -= 1
        else:
            i -= 1
    return moves


def exit_map(codes, nq, nr, b, seg):
    """Row lv's X over all columns for band b, segment by segment with left-edge symbols -(l+1),
    plus each segment's right-edge column (the kernel's Xm and Xr)."""
    lo = 64 * b
    lv = min(63, nq - 1 - lo)
    xm = np.zeros(nr + 1, dtype=np.int64)
    xr = []
    for k, J0 in enumerate(range(1, nr + 1, seg)):
        J1 = min(J0 + seg, nr + 1)
        left = [0 if k == 0 else -(l + 1) for l in range(lv + 1)]   # X(l, J0-1)
        for j in range(J0, J1):
            prev_row = j                                               # X(-1, j)
            prev_row_diag = j - 1                                      # X(-1, j-1)
            for l in range(lv + 1):
                c = codes[lo + 1 + l, j]
                x = prev_row if c == UP else (left[l] if c == LEFT else prev_row_diag)
                prev_row_diag = left[l]                                # X(l, j-1) for row l+1
                prev_row = x
                left[l] = x
            xm[j] = left[lv]
        xr.append(list(left))
    return xm, xr


def band_walk(codes, nq, nr, seg):
    nb = (nq + 63) // 64
    maps = [exit_map(codes, nq, nr, b, seg) for b in range(nb)]
    ent = [0] * nb
    e = nr
    ent[nb - 1] = e
    for b in range(nb - 1, 0, -1):                                     # the chain
        if e > 0:
            xm, xr = maps[b]
            v, k = int(xm[e]), (e - 1) // seg
            while v < 0:                                               # a segment's left edge
                k -= 1
                v = xr[k][-v - 1]
            e = v
        ent[b - 1] = e
    moves = []
    for b in range(nb - 1, -1, -1):                                    # walk order: last band first
        lo = 64 * b
        i, j = lo + min(63, nq - 1 - lo) + 1, ent[b]
        while i > lo and j > 0:
            c = codes[i, j]
            moves.append(c)
            if c == UP:
                i -= 1
            elif c == LEFT:
                j -= 1
            else:
                i -= 1
                j -= 1
        if b == 0:
            while i > 0 or j > 0:
                moves.append(LEFT if i == 0 else UP)
                if i == 0:
                    j -= 1
                else:
                    i -= 1
        else:
            while i > lo:                                              # column 0: up to the band top
                moves.append(UP)
                i -= 1
    return moves


@pytest.mark.parametrize("nq,nr,seg,p_left", [
    (1, 1, 4, 0.3), (63, 5, 4, 0.3), (64, 64, 16, 0.2), (65, 40, 8, 0.3), (130, 300, 32, 0.6),
    (200, 90, 16, 0.1), (257, 257, 64, 0.33), (129, 700, 16, 0.9),
])
def test_band_walk_model_equals_serial(nq, nr, seg, p_left):
    rng = np.random.default_rng(nq * 1000 + nr)
    p = [(1 - p_left) / 2, p_left, (1 - p_left) / 2]
    codes = rng.choice(3, size=(nq + 1, nr + 1), p=p)
    assert band_walk(codes, nq, nr, seg) == serial_walk(codes, nq, nr)
