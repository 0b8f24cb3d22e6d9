#!/usr/bin/env python3
"""Summarise a rocprofv3 run (kernel trace + separate --pmc passes) per (kernel, grid size): the 8-bit
model launches one blind-rotation kernel at two shapes (the CBS PBS over every bit, the extract_bits
chain over one ciphertext per byte), which the per-kernel --stats table averages together.

usage: prof_split_summary.py <dir with kt/ pmc_fetch/ pmc_write/ pmc_sq/> <out.json>
Traffic = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes; MI355X_MICROARCH.md): L2-miss bytes, Infinity-Cache
hits included."""
import csv
import glob
import json
import sys
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()


def main():
    d, dst = sys.argv[1], sys.argv[2]
    res = defaultdict(lambda: {"durations_ms": []})
    for f in glob.glob(d + "/kt/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
            res[k]["durations_ms"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    pmc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq"):
        for f in glob.glob(d + "/" + sub + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
                pmc[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {}
    for k, v in sorted(res.items(), key=lambda kv: -sum(kv[1]["durations_ms"])):
        ds = v["durations_ms"]
        e = {"kernel": k[0], "grid_threads": k[1], "calls": len(ds), "avg_ms": sum(ds) / len(ds), "total_ms": sum(ds)}
        cs = {c: sum(x.values()) / len(x) for c, x in pmc.get(k, {}).items()}
        if cs:
            e["pmc_avg_per_dispatch"] = cs
            if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                e["traffic_bytes_per_launch"] = 2 * cs["FETCH_SIZE"] * 1024 + cs["WRITE_SIZE"] * 1024
            if cs.get("SQ_WAVE_CYCLES"):
                e["wait_any_share"] = cs.get("SQ_WAIT_ANY", 0) / cs["SQ_WAVE_CYCLES"]
                e["valu_active_share_per_wave"] = cs.get("SQ_ACTIVE_INST_VALU", 0) / cs["SQ_WAVE_CYCLES"]
            if cs.get("SQ_ACTIVE_INST_LDS"):
                e["lds_bank_conflict_per_lds_active"] = cs.get("SQ_LDS_BANK_CONFLICT", 0) / cs["SQ_ACTIVE_INST_LDS"]
        out["%s @%d" % k] = e
    json.dump(out, open(dst, "w"), indent=1)
    for k, e in list(out.items())[:8]:
        print("%-60s calls=%-4d avg=%9.3f ms total=%9.1f ms traffic=%s" % (
            k[:60], e["calls"], e["avg_ms"], e["total_ms"], e.get("traffic_bytes_per_launch")))


if __name__ == "__main__":
    main()
