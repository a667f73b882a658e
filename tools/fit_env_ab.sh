#!/bin/bash
# Fit-kernel A/B of environment settings (one bench process per setting, interleaved, kernel ms).
#   tools/fit_env_ab.sh "PE_PL_WAVES=1024" "PE_PL_WAVES=1968" ...
set -e
for i in $(seq ${REPS:-3}); do for e in "$@"; do
  line=$(env $e timeout -k 10 120 python bench.py --no-greedy --no-configs --no-cpu-baseline --steps 10 --warmup 3)
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['roofline']['kernel_ms'],3), d['config']['feasible_pairs'])" "$e" "$line"
done; done
