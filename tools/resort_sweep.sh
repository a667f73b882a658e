set -e
mkdir -p gpurun_out/r2i
for rn in 4096 8192 16384 32768 2048; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 1 --warmup 1 --greedy-steps 3 --resort-nodes $rn > gpurun_out/r2i/g_$rn.json 2> gpurun_out/r2i/g_$rn.err
  python3 - $rn <<'PY'
import json, sys
g = json.loads(open(f"gpurun_out/r2i/g_{sys.argv[1]}.json").read().strip().splitlines()[-1])["greedy"]
r = g.get("roofline", {})
print(f'resort {sys.argv[1]:>6} {g["ms_per_batch"]:6.1f} ms {g["gang_placements_per_s"]:8.0f}/s wait {g["device_wait_ms_per_batch"]:.1f} host {g["host_resolve_ms_per_batch"]:.1f} walk {r.get("walk_ms_per_batch",0):.1f} ms ovl/grp {r.get("overlay_per_group",0):.0f} rounds/grp {r.get("rounds_per_group",0):.2f}', flush=True)
PY
done
