#!/bin/bash
# Greedy A/B of environment settings over every bench greedy line (cfg3 mix on 1M nodes + cfg2,
# cfg3, cfg4, cfg4_gang8 at their own sizes), interleaved: gang placements/s, ms, windows, rescans.
#   tools/env_configs_ab.sh reps "NAME=VAR=VAL ..." ...
set -e
reps=$1; shift
for i in $(seq $reps); do for spec in "$@"; do
  name=${spec%%=*}; env=${spec#*=}
  env $env timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --greedy-steps 2 \
    > gpurun_out/ecab.json 2> gpurun_out/ecab.err
  python3 - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ecab.json").read().strip().splitlines()[-1])
g = d["greedy"]
row = [f'1M {g["ms_per_batch"]:.2f} ms']
for k, v in d["configs"].items():
    row.append(f'{k} {v["ms_per_batch"]:.2f} ms {v["windows_per_batch"]:.0f}w {v["rescans_per_batch"]:.0f}r')
print(f'{sys.argv[1]:<7}', " | ".join(row), flush=True)
PY
done; done
