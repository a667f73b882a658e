#!/bin/bash
# Window size x walk-index rebuild threshold on the bench's greedy batch (cfg3 mix, 1M nodes), one box:
# batch time, host resolve, device wait, walk kernel time per batch (hipEvents pass), overlay per group.
set -e
mkdir -p gpurun_out/sw4
for wg in ${WGS:-64 96 128}; do for rn in ${RNS:-8192 12288 20480}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 --warmup 1 --greedy-steps 3 \
    --window-groups $wg --resort-nodes $rn > gpurun_out/sw4/g_${wg}_${rn}.json 2> gpurun_out/sw4/g_${wg}_${rn}.err
  python3 - $wg $rn <<'PY'
import json, sys
wg, rn = sys.argv[1], sys.argv[2]
g = json.loads(open(f"gpurun_out/sw4/g_{wg}_{rn}.json").read().strip().splitlines()[-1])["greedy"]
r = g.get("roofline", {})
w = r.get("warm", {})
print(f'wg {wg:>3} resort {rn:>6}: {g["ms_per_batch"]:6.2f} ms/batch host {g["host_resolve_ms_per_batch"]:.2f} wait '
      f'{g["device_wait_ms_per_batch"]:.2f} windows {g["windows_per_batch"]:.0f} rescans {g["rescans_per_batch"]:.0f} '
      f'walk {w.get("events_walk_ms_per_batch", 0):.2f} ms ({w.get("events_walk_ms_per_batch", 0) * 1e3 / max(1, g["windows_per_batch"]):.1f} us/launch) '
      f'ovl/grp {r.get("overlay_per_group", 0):.0f} rounds/grp {r.get("rounds_per_group", 0):.2f}', flush=True)
PY
done; done
