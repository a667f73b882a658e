#!/bin/bash
# Planes fit-mask kernel variants on the cfg5 bench workload (1M nodes x 100k jobs), one bench
# process per variant; the env knobs are read by pe_create (pe_engine.cpp).
#   tools/fit_variants.sh > gpurun_out/fit_variants.txt
set -e
run() {
  local tag="$1"; shift
  local line
  line=$(env "$@" timeout -k 10 120 python bench.py --no-greedy --no-cpu-baseline --steps 10 --warmup 3)
  python - "$tag" "$line" <<'EOF'
import json, sys
d = json.loads(sys.argv[2])
r = d["roofline"]
print(f'{sys.argv[1]:<40} kernel {r["kernel_ms"]:.3f} ms  step {d["ms_per_step"]:.3f} ms  frac {r["frac"]:.3f}  '
      f'feasible {d["config"]["feasible_pairs"]}', flush=True)
EOF
}
run "blockmajor (r4)" PE_FIT_ROWS=0
for pol in ${POLS:-0 1 2}; do
  for R in ${RS:-0 16}; do
    for lds in ${LDSS:-0}; do
      for pad in ${PADS:-1}; do
        run "rows pol=$pol R=$R lds=$lds pad=$pad" PE_FIT_ROWS=1 PE_FIT_POL=$pol PE_FIT_R=$R PE_FIT_LDS=$lds PE_FIT_PAD=$pad
      done
    done
  done
done
