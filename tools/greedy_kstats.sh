#!/bin/bash
# Kernel-time stats (rocprofv3 --kernel-trace --stats) of the bench's greedy line alone, per library
# (PE_LIBRARY, "" = the in-tree one): average duration of walk / apply per launch.
#   tools/greedy_kstats.sh lib1.so lib2.so ...
set -e
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  d=gpurun_out/gks_$i
  rm -rf $d
  PE_LIBRARY=${lib:+$PWD/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o k --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-configs --no-cpu-baseline --no-walk-passes --greedy-steps 3 > $d.json 2> $d.err
  python3 - "$lib" $d <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    n = r["Name"]
    for k in ("walk_kernel", "apply_kernel", "walk_build_kernel"):
        if "pe::" + k + "(" in n:
            out.append(f'{k} {float(r["AverageNs"]) / 1e3:.1f} us x {r["Calls"]}')
print(sys.argv[1] or "in-tree", " | ".join(out), flush=True)
PY
  i=$((i+1))
done
