#!/usr/bin/env python3
"""Static SGPR-spill report for a kernel in a hipcc -S listing: per loop (innermost
header, depth) the instruction / VALU counts and the v_readlane reloads and
v_writelane stores that go through the spill VGPRs.

usage: tools/spill_loops.py <file.s> [kernel-symbol-prefix]
"""
import collections
import re
import sys

src = sys.argv[1]
sym = sys.argv[2] if len(sys.argv) > 2 else "_ZN3sgk12align_kernelILi128ELb0E"
s = open(src).read().split("\n")
start = [i for i, l in enumerate(s) if l.startswith(sym) and l.split(":")[0].endswith("E") or l.startswith(sym + "EvNS_5KArgsE:")][0]
end = [i for i in range(start, len(s)) if s[i].strip().startswith(".Lfunc_end")][0]
body = s[start:end]
spillv = collections.Counter()
for l in body:
    m = re.match(r"v_writelane_b32 (v\d+), s\d+, \d+", l.strip())
    if m:
        spillv[m.group(1)] += 1
sv = set(spillv)
cur = None
stats = collections.defaultdict(lambda: [0, 0, 0, 0])
for l in body:
    m = re.search(r"in Loop: Header=(BB\d+_\d+) Depth=(\d+)", l)
    m2 = re.search(r"=>\s*This (?:Inner )?Loop Header: Depth=(\d+)", l)
    if l.startswith(".LBB"):
        cur = (l.split(":")[0][1:], int(m2.group(1))) if m2 else ((m.group(1), int(m.group(2))) if m else None)
    elif l.startswith("; %bb"):
        cur = (m.group(1), int(m.group(2))) if m else None
    t = l.strip()
    if not l.startswith("\t") or t.startswith((".", ";")):
        continue
    st = stats[cur or ("top", 0)]
    st[0] += 1
    st[1] += t.startswith("v_")
    mm = re.match(r"v_readlane_b32 s\d+, (v\d+), \d+$", t)
    st[2] += bool(mm and mm.group(1) in sv)
    mw = re.match(r"v_writelane_b32 (v\d+), s\d+, \d+", t)
    st[3] += bool(mw and mw.group(1) in sv)
print("spill VGPRs:", dict(spillv))
print("loop-header depth [instrs, valu, reloads, spills]")
for (h, d), v in sorted(stats.items(), key=lambda x: (-x[0][1], -x[1][2])):
    if v[2] or v[3]:
        print(h, d, v)
