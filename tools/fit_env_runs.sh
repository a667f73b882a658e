#!/bin/bash
# Fit-step A/B of environment settings, one bench process per run (each run its own mask
# allocation), interleaved: headline fit kernel ms.
#   tools/fit_env_runs.sh reps "NAME=VAR=VAL" ...
set -e
reps=$1; shift
for i in $(seq $reps); do for spec in "$@"; do
  name=${spec%%=*}; env=${spec#*=}
  env $env timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --no-greedy --steps 10 --warmup 3 \
    > gpurun_out/fer.json 2> gpurun_out/fer.err
  python3 - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/fer.json").read().strip().splitlines()[-1])
print(f'{sys.argv[1]:<8} kernel {d["roofline"]["kernel_ms"]:.4f} ms  step {d["ms_per_step"]:.4f} ms', flush=True)
PY
done; done
