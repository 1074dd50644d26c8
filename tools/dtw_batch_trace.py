#!/usr/bin/env python3
"""Summarise a batched-DTW band trace (SONAR_DTW_TRACE=<file> with sonar_align_pairs, e.g. under
tools/c5_stress.py): records {pair, band, t_start, t_first, t_end, sweep spins | xcc | hw_id,
sweep spins on its distance waves, sweep spins on the band above's edge, distance-wave-0 waits,
code-wave waits} (10 u64 each, s_memrealtime ticks of 10 ns; see dtw_band_kernel's trace words).

    python3 tools/dtw_batch_trace.py <trace file> [steps_per_band]

Prints per-band time split (waiting for the first edge, sweeping, the sweep's spins inside the
sweep), ns per sweep step, and the band slots' occupancy over the traced span (band-time summed /
(slots x span))."""
import sys

import numpy as np


def main():
    if len(sys.argv) < 2:
        sys.exit(__doc__)
    r = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 10).astype(np.int64)
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
    pair, band, t0, t1, t2 = r[:, 0], r[:, 1], r[:, 2], r[:, 3], r[:, 4]
    spins = r[:, 5] & 0xFFFFFF
    ok = (t2 > t1) & (t1 >= t0) & (t0 > 0)
    r, pair, band, t0, t1, t2, spins = r[ok], pair[ok], band[ok], t0[ok], t1[ok], t2[ok], spins[ok]
    tick_ns = 10.0
    wait_first = (t1 - t0) * tick_ns / 1e3          # us
    sweep = (t2 - t1) * tick_ns / 1e3               # us
    spin = spins * tick_ns / 1e3                    # us (low 24 bits of the sweep's wait ticks)
    span = (t2.max() - t0.min()) * tick_ns / 1e6    # ms
    busy = (t2 - t0).sum() * tick_ns / 1e6          # band-ms
    print(f"bands {len(r)}  pairs {len(np.unique(pair))}  traced span {span:.1f} ms")
    print(f"band-time {busy:.1f} band-ms -> mean resident bands {busy / span:.1f} (slots: 512 at 2 blocks/CU)")
    sd, se = r[:, 6] * tick_ns / 1e3, r[:, 7] * tick_ns / 1e3
    dw, cw = r[:, 8] * tick_ns / 1e3, r[:, 9] * tick_ns / 1e3
    for name, v in [("first-edge wait us", wait_first), ("sweep us", sweep), ("sweep spins us", spin),
                    ("  on distances us", sd), ("  on edge above us", se), ("  on code wave us", spin - sd - se),
                    ("dist wave 0 waits us", dw), ("code wave waits us", cw)]:
        print(f"{name:20s} median {np.median(v):9.1f}  p10 {np.percentile(v, 10):9.1f}  p90 {np.percentile(v, 90):9.1f}"
              f"  sum {v.sum() / 1e3:9.1f} ms")
    if steps:
        ns = sweep * 1e3 / steps
        busy_ns = (sweep - spin) * 1e3 / steps
        print(f"ns/step (sweep incl. waits) median {np.median(ns):.1f}  p10 {np.percentile(ns, 10):.1f}  "
              f"p90 {np.percentile(ns, 90):.1f};  excluding the sweep's spins median {np.median(busy_ns):.1f}")
    # chain pacing: within a pair, band b's sweep time against band b-1's
    by = {}
    for p, b, s in zip(pair, band, sweep):
        by.setdefault(int(p), {})[int(b)] = s
    ratios = [d[b] / d[b - 1] for d in by.values() for b in d if b - 1 in d and d[b - 1] > 0]
    if ratios:
        print(f"sweep(b) / sweep(b-1) median {np.median(ratios):.3f}  p90 {np.percentile(ratios, 90):.3f}")


if __name__ == "__main__":
    main()
