#!/bin/bash
# Planes fit-mask kernels on the cfg5 bench workload (1M nodes x 100k jobs), one bench process
# each: the block-major stream kernel (fit_path_mask bit5) against the row-major sweep (default).
# Kernel experiments from the r5 study are in profiles/r5_write_patterns.txt.
#   tools/fit_variants.sh > gpurun_out/fit_variants.txt
set -e
run() {
  local tag="$1"; shift
  local line
  line=$(timeout -k 10 120 python bench.py --no-greedy --no-cpu-baseline --steps 10 --warmup 3 "$@")
  python - "$tag" "$line" <<'EOF'
import json, sys
d = json.loads(sys.argv[2])
r = d["roofline"]
print(f'{sys.argv[1]:<24} {r["kernel"]:<34} kernel {r["kernel_ms"]:.3f} ms  step {d["ms_per_step"]:.3f} ms  '
      f'frac {r["frac"]:.3f}  feasible {d["config"]["feasible_pairs"]}', flush=True)
EOF
}
run "planes block-major" --fit-path-mask 48
run "planes row-major" --fit-path-mask 16
run "default" --fit-path-mask 0
