#!/bin/bash
# Strong-scaling rehearsal on one GPU: the per-rank fit step of the 1M x 100k cfg5 batch at N ranks is
# one context over a 1M/N-node inventory and the whole batch (no collective on the data path).
set -e
mkdir -p gpurun_out/strong
for n in 1000000 500000 250000 125000; do
  timeout -k 10 200 python bench.py --nodes $n --no-greedy --no-configs --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/strong/s_$n.json 2> gpurun_out/strong/s_$n.err
  python3 - $n <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/strong/s_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(f'nodes {int(sys.argv[1]):>8}  ms/step {d["ms_per_step"]:.3f}  kernel {d["roofline"]["kernel_ms"]:.3f}  frac {d["roofline"]["frac"]:.3f}  ideal-from-1M {2.2 * int(sys.argv[1]) / 1e6:.3f}', flush=True)
PY
done
