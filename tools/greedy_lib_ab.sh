#!/bin/bash
# Greedy A/B of libplacement builds (PE_LIBRARY, build_variants/), interleaved, cfg3 on 1M nodes.
#   GLV="lib_a lib_b" tools/greedy_lib_ab.sh [bench args]
set -e
for i in 1 2 3; do for v in ${GLV:-lib_base}; do
  PE_LIBRARY=$PWD/build_variants/$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 \
    --warmup 1 --greedy-steps 3 "$@" > gpurun_out/glab.json 2> gpurun_out/glab.err
  python3 - "$v" <<'PY'
import json, sys
g = json.loads(open("gpurun_out/glab.json").read().strip().splitlines()[-1])["greedy"]
print(f'{sys.argv[1]:<12} {g["ms_per_batch"]:6.1f} ms  {g["gang_placements_per_s"]:8.0f}/s  wait {g["device_wait_ms_per_batch"]:.1f}  host {g["host_resolve_ms_per_batch"]:.1f}', flush=True)
PY
done; done
