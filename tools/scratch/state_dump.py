#!/usr/bin/env python3
"""Decode SONAR_DTW_STATE dumps (state_pair<k>.bin): per band-kernel block, how each wave ended.
Waves: 0 sweep, 1-4 distance, 5 feeder, 6 code, 7 edge.  how: 0 never wrote (still running or
never started), 1 finished, 2 saw the block's abort word, 3 timed out, 4 saw the DTW's error word."""
import glob, sys
import numpy as np
HOW = {0: "-", 1: "done", 2: "abort", 3: "STALL", 4: "cascade"}
for fn in sorted(glob.glob(sys.argv[1] + "/state_pair*.bin")):
    w = np.fromfile(fn, np.uint64).reshape(-1, 8)
    print(fn)
    for B, row in enumerate(w):
        hows = [(int(x) >> 60) for x in row]
        if all(h == 1 for h in hows):
            continue
        desc = []
        for wv, x in enumerate(row):
            x = int(x)
            desc.append(f"{HOW[x >> 60]}@{(x >> 32) & 0xFFFFFFF}/p{(x >> 16) & 0xFFFF}/e{x & 0xFFFF}")
        print(f"  B{B:4d}: " + " ".join(desc))
