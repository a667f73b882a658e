#!/bin/bash
# The 8-rank exchange study of verdict r5 item 3, on the GPU box (one GPU, 8 shard contexts in a process):
#   1. the host merge microbenchmark on the box's CPU (tools/bench_merge.cc)
#   2. the zero-copy exchange at 8 ranks, 1 merge thread vs 4 (tools/xchg_w8.py)
#   3. the copying all-gather + merge_shards_kernel at 8 ranks under rocprofv3 (kernel time per launch)
# Output: gpurun_out/$TAG_*.  Every GPU step is bounded; the script stops at the first failure.
set -e
TAG=${1:-r21}
OUT=gpurun_out
mkdir -p $OUT
g++ -O3 -std=c++17 -march=x86-64-v3 -Wno-psabi -Itraining-operator_amd/csrc tools/bench_merge.cc -o $OUT/bench_merge
timeout -k 10 120 $OUT/bench_merge 2 4 8 16 > $OUT/${TAG}_merge_bench.txt
lscpu | grep -E "Model name|^CPU\(s\)" >> $OUT/${TAG}_merge_bench.txt
timeout -k 10 400 python -u tools/xchg_w8.py --world 8 --threads 1,4 --reps 2 --out $OUT/${TAG}_xchg_w8.json > $OUT/${TAG}_xchg_w8.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_merge_dev -o run -- python3 tools/xchg_w8.py --world 8 --copy --reps 1 --out $OUT/${TAG}_xchg_w8_copy.json > $OUT/${TAG}_merge_dev.log 2>&1
echo done
