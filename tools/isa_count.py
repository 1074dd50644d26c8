#!/usr/bin/env python3
"""Instruction mix of one kernel's hottest loop in a hipcc --save-temps .s file.

The loop is taken as the innermost-depth loop block range that contains the most VALU: from its
header label (comment '=>This Loop Header') to the last branch back to it.  Prints VALU / LDS /
VMEM / SALU / s_nop / s_waitcnt counts.  Usage: python tools/isa_count.py file.s kernel_symbol"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if ln.startswith(sym + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end + 1]
    # loops: every "Loop Header" label, spanning to the last branch back to it
    best = None
    for i, ln in enumerate(body):
        m = re.match(r"^\.(LBB\w+):", ln)
        if not m or "Loop Header" not in ln:
            continue
        lab = m.group(1)
        brs = [j for j, x in enumerate(body) if re.search(r"s_(cbranch\w*|branch)\s+\." + lab + r"\b", x)]
        if not brs:
            continue
        seg = body[i:max(brs) + 1]
        nv = sum(1 for x in seg if re.match(r"^\s+v_", x))
        if best is None or nv > best[0]:
            best = (nv, lab, seg)
    nv, lab, seg = best
    cnt = lambda pat: sum(1 for ln in seg if re.match(pat, ln))  # noqa: E731
    pats = {"dpp": r"^\s+v_\w+_dpp", "permlane": r"^\s+v_permlane", "vmov": r"^\s+v_mov", "lds": r"^\s+ds_",
            "lds_read": r"^\s+ds_read", "lds_write": r"^\s+ds_write", "vmem": r"^\s+(global|buffer|flat)_",
            "salu": r"^\s+s_(?!nop|waitcnt|cbranch|branch)", "s_nop": r"^\s+s_nop", "s_waitcnt": r"^\s+s_waitcnt",
            "scratch": r"^\s+scratch_"}
    c = {k: cnt(v) for k, v in pats.items()}
    print(f"{sym}: loop {lab}, {len(seg)} lines")
    print("  VALU %d (dpp %d, permlane %d, mov %d)  LDS %d (read %d, write %d)  VMEM %d  SALU %d  s_nop %d  "
          "s_waitcnt %d  scratch %d" % (nv, c["dpp"], c["permlane"], c["vmov"], c["lds"], c["lds_read"],
                                         c["lds_write"], c["vmem"], c["salu"], c["s_nop"], c["s_waitcnt"], c["scratch"]))

if __name__ == "__main__":
    main()
