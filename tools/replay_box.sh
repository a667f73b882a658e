#!/bin/bash
# Host-resolver replay A/B on the GPU box's CPU (the EPYC the bench's host half runs on): builds
# tools/replay_resolver.cc against each resolver source given (default: the tree's), replays the
# recorded window dump (tools/dumps/*.xz, from tools/greedy_dump.py) interleaved, min / median ms.
#   tools/replay_box.sh dump.bin.xz [src.cpp[:DEFS] ...]   (a src beside its own pe_resolver.h uses that header)
set -e
dump=$1; shift
mkdir -p /tmp/rb && xz -dc "$dump" > /tmp/rb/d.bin
srcs=("$@"); [ ${#srcs[@]} -eq 0 ] && srcs=(training-operator_amd/csrc/pe_resolver.cpp)
i=0
for s in "${srcs[@]}"; do
  f=${s%%:*}; defs=""; [[ "$s" == *:* ]] && defs=${s#*:}
  g++ -O3 -march=x86-64-v3 -std=c++17 $defs -I"$(dirname "$f")" -Itraining-operator_amd/csrc -Iinclude tools/replay_resolver.cc "$f" -o /tmp/rb/r$i -lpthread
  i=$((i+1))
done
for rep in 1 2 3; do
  for j in $(seq 0 $((i-1))); do
    taskset -c 2,3 /tmp/rb/r$j /tmp/rb/d.bin 7 | python3 -c "
import sys,re
L=list(sys.stdin); v=sorted(float(re.search(r'([0-9.]+) ms in resolve',l).group(1)) for l in L if 'in resolve' in l)
print('${srcs[$j]}', 'min %.2f med %.2f'%(v[0],v[len(v)//2]), L[1].split('result')[-1].strip(), flush=True)"
  done
done
