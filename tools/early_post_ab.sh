#!/bin/bash
# Early-post A/B (PE_EARLY_POST=0: the helper gets apply(i) + scan(i + 2) after the first group of window
# i + 1 was seen; default: as soon as window i landed), interleaved on one box over window sizes: cfg3
# batch on the 1M-node inventory, bench.py's greedy pass.
#   tools/early_post_ab.sh [reps] [window sizes...]
set -e
reps=${1:-2}; shift || true
for i in $(seq $reps); do for wg in ${*:-80 96 112}; do for ep in 0 1; do
  PE_EARLY_POST=$ep timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 --warmup 1 --greedy-steps 3 \
    --window-groups $wg > gpurun_out/ep.json 2> gpurun_out/ep.err
  python3 - "$wg" "$ep" <<'PY'
import json, sys
g = json.loads(open("gpurun_out/ep.json").read().strip().splitlines()[-1])["greedy"]
print(f'wg {sys.argv[1]:<4} early {sys.argv[2]}  {g["ms_per_batch"]:6.2f} ms  wait {g["device_wait_ms_per_batch"]:.2f}  '
      f'host {g["host_resolve_ms_per_batch"]:.2f}  windows {g["windows_per_batch"]}', flush=True)
PY
done; done; done
