#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory into one JSON (committed under profiles/).

HBM traffic per launch follows MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and WRITE_SIZE
come from separate --pmc passes, are in KiB, and on gfx950 FETCH_SIZE reports half the bytes of a
wide streaming read, so traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

usage: tools/summarize_prof.py <profile dir> <kernel substring> <algorithmic bytes per launch> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, kname, alg, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                            "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                            "pct": float(r["Percentage"])}
    hot = [k for k in stats if kname in k]
    counters = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                counters[r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    per_launch = {}
    for c, vals in counters.items():
        by = collections.defaultdict(float)
        for disp, v in vals:
            by[disp] += v
        per_launch[c] = sum(by.values()) / len(by)
    res = {"kernel": hot[0] if hot else None, "kernel_stats": stats[hot[0]] if hot else None,
           "all_kernels": stats, "pmc_per_launch": per_launch,
           "algorithmic_bytes_per_launch": alg}
    if "FETCH_SIZE" in per_launch and "WRITE_SIZE" in per_launch:
        rd = 2 * per_launch["FETCH_SIZE"] * 1024
        wr = per_launch["WRITE_SIZE"] * 1024
        res["hbm_traffic_bytes_per_launch"] = rd + wr
        res["hbm_read_bytes_per_launch"] = rd
        res["hbm_write_bytes_per_launch"] = wr
        res["traffic_over_algorithmic"] = (rd + wr) / alg
    if hot:
        res["achieved_GBps_from_trace"] = alg / (stats[hot[0]]["avg_ns"] * 1e-9) / 1e9
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "all_kernels"}, indent=1))


if __name__ == "__main__":
    main()
