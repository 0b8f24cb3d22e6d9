#!/usr/bin/env python3
"""ISA statistics of one kernel in a gfx950 `.s` file (hipcc --cuda-device-only -S):
register use, spills, and instruction classes of the whole kernel and of its largest loop body
(the blocks between a loop header label and the backward branch to it).

usage: isa_stats.py FILE.s NAME_SUBSTRING [NAME_SUBSTRING ...]
"""
import re
import sys
from collections import Counter

CLASSES = [
    ("f64", re.compile(r"^v_(fma|fmac|add|mul|mad|min|max|ldexp|cvt_f64|fract|trig|div)\w*_f64")),
    ("cvt", re.compile(r"^v_cvt_")),
    ("permlane", re.compile(r"^v_permlane")),
    ("cndmask_vcc", re.compile(r"^v_cndmask_b32_e32")),
    ("cndmask_sgpr", re.compile(r"^v_cndmask_b32_e64")),
    ("valu_other", re.compile(r"^v_")),
    ("ds_read", re.compile(r"^ds_read")),
    ("ds_write", re.compile(r"^ds_write")),
    ("vmem", re.compile(r"^(buffer|global|flat)_")),
    ("smem", re.compile(r"^s_(load|buffer_load|memtime|memrealtime)")),
    ("waitcnt", re.compile(r"^s_waitcnt")),
    ("nop", re.compile(r"^s_nop")),
    ("setprio", re.compile(r"^s_setprio")),
    ("barrier", re.compile(r"^s_barrier")),
    ("branch", re.compile(r"^s_(cbranch|branch)")),
    ("salu", re.compile(r"^s_")),
]


def classify(op):
    for name, rx in CLASSES:
        if rx.match(op):
            return name
    return "other"


def kernel_body(text, sub):
    for m in re.finditer(r"^(_Z\S+):\s*;", text, re.M):
        if sub in m.group(1):
            end = text.find(".Lfunc_end", m.end())
            return m.group(1), text[m.end():end], text[end:end + 4000]
    raise SystemExit(f"no kernel matching {sub}")


def stats(lines):
    c = Counter()
    for ln in lines:
        op = ln.split()[0]
        c[classify(op)] += 1
    c["total"] = len(lines)
    return c


def main():
    text = open(sys.argv[1]).read()
    for sub in sys.argv[2:]:
        name, body, tail = kernel_body(text, sub)
        raw = body.split("\n")
        instr = [(i, ln.strip()) for i, ln in enumerate(raw) if ln.startswith("\t") and not ln.startswith("\t.")
                 and not ln.strip().startswith(";") and ln.strip()]
        labels = {ln.split(":")[0]: i for i, ln in enumerate(raw) if re.match(r"^\.LBB\w+:", ln)}
        # loops: a branch at line j to a label at line i < j
        loops = []
        for j, ln in instr:
            m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", ln)
            if m and m.group(1) in labels and labels[m.group(1)] < j:
                loops.append((labels[m.group(1)], j))
        regs = {k: re.search(k + r":\s+(\d+)", tail) for k in ("NumVgprs", "NumAgprs", "NumSgprs", "ScratchSize", "Occupancy")}
        print(name)
        print("  " + "  ".join(f"{k}={v.group(1)}" for k, v in regs.items() if v))
        print("  kernel:", dict(stats([ln for _, ln in instr]).most_common()))
        if loops:
            a, b = max(loops, key=lambda x: x[1] - x[0])
            body_lines = [ln for i, ln in instr if a <= i <= b]
            print(f"  largest loop ({len(body_lines)} instrs):", dict(stats(body_lines).most_common()))


if __name__ == "__main__":
    main()
