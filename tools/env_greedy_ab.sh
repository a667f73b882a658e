#!/bin/bash
# Greedy A/B of environment settings on one library build, interleaved: cfg3 mix on the 1M-node
# inventory; per run the batch time, device wait, host resolve (bench.py greedy line).
#   tools/env_greedy_ab.sh reps "NAME=VAR=VAL ..." "NAME2=" ...     e.g. "sync=PE_NO_GROUP_SIGNAL=1" "signal="
set -e
reps=$1; shift
for i in $(seq $reps); do for spec in "$@"; do
  name=${spec%%=*}; env=${spec#*=}
  env $env timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 --warmup 1 --greedy-steps 3 \
    > gpurun_out/eab.json 2> gpurun_out/eab.err
  python3 - "$name" <<'PY'
import json, sys
g = json.loads(open("gpurun_out/eab.json").read().strip().splitlines()[-1])["greedy"]
print(f'{sys.argv[1]:<8} {g["ms_per_batch"]:6.2f} ms  {g["gang_placements_per_s"]:8.0f}/s  wait {g["device_wait_ms_per_batch"]:.2f}'
      f'  host {g["host_resolve_ms_per_batch"]:.2f}  walk {g["roofline"].get("warm", {}).get("walk_ms_per_batch", float("nan")):.2f}', flush=True)
PY
done; done
