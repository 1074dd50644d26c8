#!/usr/bin/env python3
"""Band-slot supply against demand over a batched-DTW band trace (SONAR_DTW_TRACE records, see
tools/dtw_batch_trace.py): per time bin, the resident bands (started, not ended) and the PENDING
bands -- bands of a pair whose first band has started (its batch's band kernel is executing) but
which have not started themselves.  Idle slots while bands are pending mean blocks that could run
are not being placed (CU resources held by other kernels, dispatcher order); idle slots with
nothing pending mean the worker streams have no band work ready (features / walks / host).

    python3 tools/c5_pending.py <trace file> [bin_ms] [slots]

A trace holding several calls (warm-up + timed) is split where no band is resident for > 2 ms;
pair ids repeat across calls, so launch times are taken per call."""
import json
import sys

import numpy as np


def main():
    if len(sys.argv) < 2:
        sys.exit(__doc__)
    r = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 10).astype(np.int64)
    bin_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    slots = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    pair, t0, t2 = r[:, 0], r[:, 2], r[:, 4]
    xcd = (r[:, 5] >> 24) & 0xF                       # XCC_ID of the block that ran the band
    cu = xcd * 256 + ((r[:, 5] >> 40) & 0xFF)         # + HW_ID CU/SH/SE bits: one id per CU
    ok = (t2 > t0) & (t0 > 0)
    pair, t0, t2, xcd, cu = pair[ok], t0[ok], t2[ok], xcd[ok], cu[ok]
    tick_ns = 10.0
    # split into calls at gaps with nothing resident
    o = np.argsort(t0)
    pair, t0, t2, xcd, cu = pair[o], t0[o], t2[o], xcd[o], cu[o]
    run_end = np.maximum.accumulate(t2)
    gap = np.where(t0[1:] - run_end[:-1] > 2e6 / tick_ns)[0]
    cuts = [0, *(gap + 1).tolist(), len(t0)]
    out = {"bin_ms": bin_ms, "slots": slots, "calls": []}
    for c in range(len(cuts) - 1):
        a, b = cuts[c], cuts[c + 1]
        p, s, e, x, u = pair[a:b], t0[a:b], t2[a:b], xcd[a:b], cu[a:b]
        base = s.min()
        s, e = (s - base) * tick_ns / 1e6, (e - base) * tick_ns / 1e6   # ms
        first = {}
        for pi, si in zip(p.tolist(), s.tolist()):
            if pi not in first:
                first[pi] = si                                           # sorted by start
        launch = np.array([first[pi] for pi in p.tolist()])
        nb = int(np.ceil(e.max() / bin_ms))
        edges = np.arange(nb + 1) * bin_ms
        mid = edges[:-1] + bin_ms / 2
        # sampled at bin midpoints (exact counts, not averages)
        res = np.array([np.count_nonzero((s <= t) & (e > t)) for t in mid])
        pend = np.array([np.count_nonzero((launch <= t) & (s > t)) for t in mid])
        idle = slots - res
        # per XCD (slots / 8 each): idle slots on an XCD with none of its own bands pending, while
        # another XCD still has some -- the static workgroup -> XCD round robin leaving work behind
        nx = 8
        xs = slots // nx
        res_x = np.array([[np.count_nonzero((x == k) & (s <= t) & (e > t)) for k in range(nx)] for t in mid])
        pend_x = np.array([[np.count_nonzero((x == k) & (launch <= t) & (s > t)) for k in range(nx)] for t in mid])
        idle_x = np.maximum(xs - res_x, 0)
        idle_dry = (idle_x * (pend_x == 0)).sum(axis=1)            # idle slots on XCDs with nothing pending
        idle_wet = (np.minimum(idle_x, pend_x) * (pend_x > 0)).sum(axis=1)
        # per CU: how many CUs hold 0 / 1 / 2+ band blocks at each sampled instant (averaged over the
        # bins where some XCD has idle slots AND pending bands)
        cus = np.unique(u)
        cidx = np.searchsorted(cus, u)
        hist = np.zeros((len(mid), 3))
        for i, t in enumerate(mid):
            live = (s <= t) & (e > t)
            cnt = np.bincount(cidx[live], minlength=len(cus))
            hist[i] = [np.count_nonzero(cnt == 0), np.count_nonzero(cnt == 1), np.count_nonzero(cnt >= 2)]
        wet = idle_wet > 0.05 * slots
        starved = (idle > 0.05 * slots) & (pend == 0)
        blocked = (idle > 0.05 * slots) & (pend > 0)
        out["calls"].append({
            "span_ms": round(float(e.max()), 2), "bands": int(b - a),
            "mean_resident": round(float(res.mean()), 1),
            "bins_idle_gt5pct": int(np.count_nonzero(idle > 0.05 * slots)),
            "bins_idle_nothing_pending": int(np.count_nonzero(starved)),
            "bins_idle_with_pending": int(np.count_nonzero(blocked)),
            "idle_slot_ms_nothing_pending": round(float((idle * starved).sum() * bin_ms), 1),
            "idle_slot_ms_with_pending": round(float((np.minimum(idle, pend) * blocked).sum() * bin_ms), 1),
            "idle_slot_ms_total": round(float(np.maximum(idle, 0).sum() * bin_ms), 1),
            "xcd_idle_slot_ms_own_nothing_pending": round(float(idle_dry.sum() * bin_ms), 1),
            "xcd_idle_slot_ms_own_pending": round(float(idle_wet.sum() * bin_ms), 1),
            "xcd_band_share": [round(float(np.count_nonzero(x == k)) / len(x), 4) for k in range(nx)],
            "xcd_mean_resident": [round(float(v), 1) for v in res_x.mean(axis=0)],
            "cus_seen": int(len(cus)),
            "cus_with_0_1_2_bands_when_idle_with_pending": [round(float(v), 1) for v in hist[wet].mean(axis=0)] if wet.any() else None,
            "cus_with_0_1_2_bands_other_bins": [round(float(v), 1) for v in hist[~wet].mean(axis=0)] if (~wet).any() else None,
            "resident": res.tolist(), "pending": pend.tolist()})
    summary = {k: v for k, v in out.items() if k != "calls"}
    for c in out["calls"]:
        print(json.dumps({**summary, **{k: v for k, v in c.items() if k not in ("resident", "pending")}}))
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
