#!/bin/bash
# Interleaved A/B of resolver SOURCES / build flags on the GPU box's CPU: records the bench batch's
# windows on the GPU (tools/greedy_dump.py; env GREEDY_DUMP_ARGS passes engine options), builds
# tools/replay_resolver.cc against each variant (the tree's pe_resolver.h unless the source sits
# beside its own), replays them in turn; result checksums must agree.
#   tools/replay_src_ab.sh reps A.cpp B.cpp[:-DFLAG=1] ...
set -e
reps=$1; shift
mkdir -p /tmp/rsa
timeout -k 10 300 python tools/greedy_dump.py /tmp/rsa/d.bin > /dev/null
i=0
for v in "$@"; do
  s=${v%%:*}; defs=""; [[ "$v" == *:* ]] && defs=${v#*:}
  g++ -O3 -march=x86-64-v3 -std=c++17 $defs -I"$(dirname "$s")" -Itraining-operator_amd/csrc -Iinclude \
    tools/replay_resolver.cc "$s" -o /tmp/rsa/r$i -lpthread
  i=$((i+1))
done
for rep in $(seq $reps); do
  j=0
  for v in "$@"; do
    echo "$v $(taskset -c 2,3 /tmp/rsa/r$j /tmp/rsa/d.bin 5 | awk '/^rep/ {r=r" "$6; h=$NF} END {print r, h}')"
    j=$((j+1))
  done
done
