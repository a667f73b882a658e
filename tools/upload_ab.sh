#!/bin/bash
# pe_jobs_upload / end-to-end fit batch A/B of environment settings, interleaved (bench.py's
# fit_end_to_end line: upload = host planning + H2D of the 100k-job batch).
#   tools/upload_ab.sh reps "NAME=VAR=VAL" ...
set -e
reps=$1; shift
for i in $(seq $reps); do for spec in "$@"; do
  name=${spec%%=*}; env=${spec#*=}
  env $env timeout -k 10 300 python bench.py --no-cpu-baseline --no-greedy --steps 3 --warmup 1 --agg-jobs 1000 \
    > gpurun_out/uab.json 2> gpurun_out/uab.err
  python3 - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/uab.json").read().strip().splitlines()[-1])
e = d["fit_end_to_end"]
print(f'{sys.argv[1]:<8} upload {e["upload_ms"]:.3f} ms  end-to-end {e["ms_per_batch"]:.3f} ms', flush=True)
PY
done; done
