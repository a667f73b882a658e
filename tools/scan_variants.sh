#!/bin/bash
# Kernel-trace A/B of libplacement builds on the greedy bench (PE_LIBRARY selects the build).
#   tools/scan_variants.sh lib_a.so lib_b.so ...   (paths under build_variants/)
set -e
export TMPDIR=/tmp
for lib in "$@"; do
  out=gpurun_out/scanvar_$(basename $lib .so)
  rm -rf $out
  PE_LIBRARY=$PWD/build_variants/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out -o t --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --greedy-steps 2 $SCANVAR_ARGS > $out.json 2> $out.err
  python3 - "$lib" "$out" <<'PY'
import csv, glob, json, sys
lib, out = sys.argv[1], sys.argv[2]
rows = {r["Name"].split("(")[0]: r for f in glob.glob(out + "/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(f))}
b = json.loads(open(out + ".json").read().strip().splitlines()[-1])
g = b["greedy"]
ks = " ".join(f'{k.split("::")[-1]}={float(rows[k]["AverageNs"])/1e3:.1f}us' for k in rows if "scan" in k or "merge" in k or "prep" in k)
print(f'{lib:<14} greedy {g["ms_per_batch"]:.1f} ms ({g["gang_placements_per_s"]:.0f}/s)  {ks}', flush=True)
PY
done
