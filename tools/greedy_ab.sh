#!/bin/bash
# Greedy A/B on the bench workload (cfg3 mix, 1M nodes): one bench process per argument set.
#   tools/greedy_ab.sh "--greedy-flags 0" "--greedy-flags 2" ...
set -e
export TMPDIR=/tmp
i=0
for a in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 --warmup 1 --greedy-steps 3 $a \
    > gpurun_out/gab_$i.json 2> gpurun_out/gab_$i.err
  python3 - "$a" gpurun_out/gab_$i.json <<'PY'
import json, sys
g = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["greedy"]
print(f'{sys.argv[1]:<40} {g["ms_per_batch"]:6.1f} ms  {g["gang_placements_per_s"]:8.0f}/s  windows {g["windows_per_batch"]:.0f}'
      f'  rescans {g["rescans_per_batch"]:.0f}  wait {g["device_wait_ms_per_batch"]:.1f}  host {g["host_resolve_ms_per_batch"]:.1f}', flush=True)
PY
  i=$((i+1))
done
