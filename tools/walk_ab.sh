#!/bin/bash
# Walk-kernel A/B of libplacement builds (build_variants/<v>.so), interleaved: cfg3 mix on the 1M-node
# inventory; per run the batch time, the device wait, the host resolve and the walk kernel time per
# batch (hipEvents around every walk launch, bench.py's greedy roofline pass).
#   WAV="wbase wc2k" tools/walk_ab.sh [reps]
set -e
for i in $(seq ${1:-3}); do for v in ${WAV:-wbase}; do
  PE_LIBRARY=$PWD/build_variants/$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 \
    --warmup 1 --greedy-steps 3 > gpurun_out/wab.json 2> gpurun_out/wab.err
  python3 - "$v" <<'PY'
import json, sys
g = json.loads(open("gpurun_out/wab.json").read().strip().splitlines()[-1])["greedy"]
r = g["roofline"]
print(f'{sys.argv[1]:<8} {g["ms_per_batch"]:6.2f} ms  wait {g["device_wait_ms_per_batch"]:.2f}  host {g["host_resolve_ms_per_batch"]:.2f}'
      f'  walk {r["walk_ms_per_batch"]:.2f} ms / {r["walk_launches"]} launches', flush=True)
PY
done; done
