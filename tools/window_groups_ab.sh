#!/bin/bash
set -e
for i in 1 2 3; do for wg in 80 96 112 128; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 --warmup 1 --greedy-steps 3 --window-groups $wg > gpurun_out/wg.json 2> gpurun_out/wg.err
  python3 - "$wg" <<'PY'
import json, sys
g = json.loads(open("gpurun_out/wg.json").read().strip().splitlines()[-1])["greedy"]
print(f'wg {sys.argv[1]:<4} {g["ms_per_batch"]:6.2f} ms  wait {g["device_wait_ms_per_batch"]:.2f}  host {g["host_resolve_ms_per_batch"]:.2f} windows {g["windows_per_batch"]}', flush=True)
PY
done; done
