#!/usr/bin/env python3
"""Per-phase cycles per CMux step of a TAE_X4_PROF build (br512x4.hpp): averages the last launch's lines
`x4prof wave W: dec .. passA .. ...` over the 677 steps; prints one row per wave, sorted by wave."""
import re
import sys

KEYS = ["dec", "passA", "passB", "barF", "mac", "barM", "store", "invB", "invA", "end"]
rows = {}
for ln in open(sys.argv[1]):
    m = re.match(r"x4prof wave\s+(\d+): (.*)", ln)
    if m:
        vals = dict(zip(m.group(2).split()[0::2], map(int, m.group(2).split()[1::2])))
        rows[int(m.group(1))] = vals  # the last launch wins
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 677
print("wave " + " ".join(f"{k:>6}" for k in KEYS) + "   total")
for w in sorted(rows):
    v = [rows[w][k] / steps for k in KEYS]
    print(f"{w:4d} " + " ".join(f"{x:6.0f}" for x in v) + f"  {sum(v):6.0f}")
