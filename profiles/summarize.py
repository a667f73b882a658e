#!/usr/bin/env python3
"""Summarise a rocprofv3 profile directory (profiles/run_profile.sh output) into one JSON:
per-kernel average duration (kernel trace --stats) and per-launch PMC values, with the gfx950
HBM correction of MI355X_MICROARCH.md sec. HBM: FETCH_SIZE reports 1/2 of wide streaming reads
(doubled here), WRITE_SIZE is exact for 16-B/lane streaming stores.  Units: FETCH/WRITE_SIZE KB."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import source_hash  # noqa: E402


def kname(name: str) -> str:
    """Kernel key: the demangled name without arguments, return type or template arguments
    ("void pe::fit_mask_lds_kernel<2, 1, 1, 2>(...)" -> "pe::fit_mask_lds_kernel")."""
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n.split("<")[0].strip()


def main(d):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {"source_hash": source_hash(root), "kernels": {}, "pmc": collections.defaultdict(dict)}
    for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):   # the full bench
        for r in csv.DictReader(open(f)):
            out["kernels"][kname(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                                       "total_ns": float(r["TotalDurationNs"])}
    # the greedy walk passes (warm / cold) and the aggregation pass: their kernel stats apart
    for sub, key in (("walk_warm", ("greedy", "warm")), ("walk_cold", ("greedy", "cold")), ("agg", ("aggregation", None))):
        for f in glob.glob(os.path.join(d, sub, "*kernel_stats.csv")):
            stats = {kname(r["Name"]): {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                        "total_ns": float(r["TotalDurationNs"])} for r in csv.DictReader(open(f))}
            if key[1]:
                out.setdefault(key[0], {})[key[1]] = stats
            else:
                out[key[0]] = stats
    # PMC passes: the fit passes into "pmc", the greedy passes (walk_fetch / walk_write) into
    # greedy.pmc -- per-launch averages of each kernel
    gpmc = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        dest = gpmc if os.path.basename(os.path.dirname(f)).startswith("walk_") else out["pmc"]
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            acc[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            dest[k][c] = sum(v) / len(v)
            dest[k][c + "_launches"] = len(v)
    for pm in (out["pmc"], gpmc):
        for k, p in pm.items():
            if "FETCH_SIZE" in p:
                p["hbm_read_bytes_corrected"] = p["FETCH_SIZE"] * 1024 * 2
            if "WRITE_SIZE" in p:
                p["hbm_write_bytes"] = p["WRITE_SIZE"] * 1024
            if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
                p["hbm_traffic_bytes"] = p["hbm_read_bytes_corrected"] + p["hbm_write_bytes"]
    if gpmc:
        out.setdefault("greedy", {})["pmc"] = gpmc
    # the workload the passes ran (bench.py's JSON line under the kernel trace)
    for f in glob.glob(os.path.join(d, "bench_trace.json")):
        lines = [ln for ln in open(f) if ln.startswith("{")]
        if lines:
            b = json.loads(lines[-1])
            out["workload"] = {"nodes": b["config"]["nodes"], "jobs": b["config"]["jobs"],
                               "fit_path": b["roofline"].get("fit_path"), "bench_value": b["value"],
                               "bench_kernel_ms": b["roofline"].get("kernel_ms")}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
