#!/usr/bin/env python3
"""Copy the judged part of a run_profile.sh output (gpurun_out/prof_<tag>) into profiles/<name>:
the rocprofv3 --stats kernel summary, the bench line printed under the trace, the PMC rows of the
step kernels (fit mask, encode, walk, apply; the full counter CSVs hold every launch of the run)
and summary.json.  --latest: LATEST names this profile alone; --latest-add: appended to LATEST (another
box's profile of the same sources -- bench.py takes the one whose fit step is closest to its run's).
    python3 profiles/collect.py gpurun_out/prof_r8a r8a_head [--latest | --latest-add]"""
import csv
import os
import shutil
import sys

KEEP = ("fit_mask", "encode_", "walk_kernel", "apply_kernel", "node_ranks", "pg_agg_seg")


def main(src, name, latest):
    root = os.path.dirname(os.path.abspath(__file__))
    dst = os.path.join(root, name)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench_trace.json"), os.path.join(dst, "bench_trace.json"))
    shutil.copy(os.path.join(src, "summary.json"), os.path.join(dst, "summary.json"))
    # the greedy walk passes (warm / cold, PE_WALK_FLUSH) and the aggregation pass: kernel stats + bench lines
    for sub, stem in (("walk_warm", "walk"), ("walk_cold", "walk"), ("agg", "agg")):
        f = os.path.join(src, sub, f"{stem}_kernel_stats.csv")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(dst, f"kernel_stats_{sub}.csv"))
    for f in ("bench_walk_warm.json", "bench_walk_cold.json", "agg.out"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    for pas in ("fetch", "write", "sq", "sq2", "walk_fetch", "walk_write"):
        f = os.path.join(src, pas, f"{pas}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = list(csv.DictReader(open(f)))
        with open(os.path.join(dst, f"pmc_{pas}.csv"), "w", newline="") as o:
            w = csv.DictWriter(o, fieldnames=list(rows[0].keys()) if rows else ["empty"])
            w.writeheader()
            seen = {}
            for r in rows:   # at most 4 launches per (kernel, counter)
                k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
                if any(s in k[0] for s in KEEP) and seen.get(k, 0) < 4:
                    seen[k] = seen.get(k, 0) + 1
                    w.writerow(r)
    if latest == "add":
        path = os.path.join(root, "LATEST")
        tags = open(path).read().split() if os.path.exists(path) else []
        if name not in tags:
            tags.append(name)
        with open(path, "w") as f:
            f.write("".join(t + "\n" for t in tags))
    elif latest:
        with open(os.path.join(root, "LATEST"), "w") as f:
            f.write(name + "\n")
    print("profiles/" + name)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "add" if "--latest-add" in sys.argv[3:] else "--latest" in sys.argv[3:])
