#!/usr/bin/env python3
"""Summarise the rocprofv3 CSV outputs of scripts/bench_profile.sh.

Writes into <out>/summary/: kernel_stats.csv (copy of the --stats table) and pmc.json with the
per-kernel average of every collected counter per dispatch, plus the HBM traffic per launch of
each kernel: 2 x FETCH_SIZE (gfx950 reports half the bytes of wide coalesced reads,
MI355X_MICROARCH.md HBM section) + WRITE_SIZE, in bytes (the counters are in KB).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def find(out, sub, pattern):
    hits = sorted(glob.glob(os.path.join(out, sub, "**", pattern), recursive=True))
    return hits[0] if hits else None


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()


def counters(path):
    """{kernel: {counter: [value per dispatch]}}"""
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    with open(path) as fh:
        for row in csv.DictReader(fh):
            k = short(row["Kernel_Name"])
            per[(k, row.get("Dispatch_Id") or row.get("Correlation_Id"))][row["Counter_Name"]] += float(row["Counter_Value"])
    res = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            res[k][c].append(v)
    return res


def main():
    out = sys.argv[1]
    dst = os.path.join(out, "summary")
    os.makedirs(dst, exist_ok=True)
    stats = find(out, "prof", "*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
        with open(stats) as fh:
            rows = list(csv.DictReader(fh))
        print("kernel stats (%s):" % os.path.basename(stats))
        for r in rows[:12]:
            name = r.get("Name") or r.get("KernelName") or ""
            avg = float(r.get("AverageNs") or r.get("Average") or 0)
            print("  %-44s calls=%-5s avg=%.3f ms  %5.1f%%" % (short(name)[:44], r.get("Calls"), avg / 1e6,
                                                               float(r.get("Percentage") or 0)))
    pmc = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_dram", "pmc_mfma"):
        path = find(out, sub, "*counter_collection.csv")
        if not path:
            continue
        for k, cs in counters(path).items():
            for c, vals in cs.items():
                pmc.setdefault(k, {})[c] = {"avg_per_dispatch": sum(vals) / len(vals), "dispatches": len(vals)}
    for k, cs in pmc.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            fetch = 2 * cs["FETCH_SIZE"]["avg_per_dispatch"] * 1024
            write = cs["WRITE_SIZE"]["avg_per_dispatch"] * 1024
            cs["hbm_bytes_per_launch"] = fetch + write
            cs["hbm_read_bytes_per_launch_corrected"] = fetch
            cs["hbm_write_bytes_per_launch"] = write
            # L2 misses (FETCH_SIZE) include Infinity-Cache hits (MI355X_MICROARCH.md HBM section).
            # TCC_EA0_RDREQ_DRAM reads equal TCC_EA0_RDREQ for every large kernel here, so it does not
            # separate Infinity-Cache hits either: no DRAM-only figure is derived from it.
    with open(os.path.join(dst, "pmc.json"), "w") as fh:
        json.dump(pmc, fh, indent=1, sort_keys=True)
    blocks = int(sys.argv[2]) if len(sys.argv) > 2 else None
    latest = {"blocks_per_gpu": blocks,
              "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of bench.py --steps 1 "
                        "--key-schedule plain (scripts/bench_profile.sh); bytes = 2 x FETCH_SIZE + WRITE_SIZE "
                        "(L2 misses incl. Infinity-Cache hits; no counter separates the bytes that reached HBM)",
              "kernels": {k: {c: (v["avg_per_dispatch"] if isinstance(v, dict) else v) for c, v in cs.items()}
                          for k, cs in pmc.items()}}
    with open(os.path.join(dst, "pmc_latest.json"), "w") as fh:
        json.dump(latest, fh, indent=1, sort_keys=True)
    for k, cs in pmc.items():
        print("pmc %-40s %s" % (k[:40], {c: (round(v["avg_per_dispatch"]) if isinstance(v, dict) else round(v))
                                          for c, v in cs.items()}))


if __name__ == "__main__":
    main()
