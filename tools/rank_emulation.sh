#!/bin/bash
# Per-rank fit workload of the weak-scaling bench at N = 1/2/4/8 emulated on one GPU: a rank holds
# 1M/N nodes and 100k x N jobs (the shard is a fresh synthetic inventory of that size).
set -e
for cfg in "1000000 100000" "500000 200000" "250000 400000" "125000 800000"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --nodes $1 --fit-jobs $2 --no-greedy --no-configs --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/emu_$1.json
  python -c "
import json;d=json.load(open('gpurun_out/emu_$1.json'));r=d['roofline'];print('$1', d['config']['jobs'], round(r['kernel_ms'],3), round(d['ms_per_step'],3), round(r['frac'],3), '%.3e'%d['value'])"
done
