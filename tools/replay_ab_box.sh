#!/bin/bash
# Interleaved A/B of two resolver sources on the GPU box's CPU (no GPU use): replays the recorded
# window dump (tools/greedy_dump.py) with each, result checksums printed (must agree).
#   tools/replay_ab_box.sh dump.bin.xz A.cpp A_include_dir B.cpp B_include_dir [rounds]
set -e
mkdir -p /tmp/rpab && xz -dc "$1" > /tmp/rpab/d.bin
g++ -O3 -march=x86-64-v3 -std=c++17 -I"$3" -Itraining-operator_amd/csrc -Iinclude tools/replay_resolver.cc "$2" -o /tmp/rpab/a -lpthread
g++ -O3 -march=x86-64-v3 -std=c++17 -I"$5" -Itraining-operator_amd/csrc -Iinclude tools/replay_resolver.cc "$4" -o /tmp/rpab/b -lpthread
for i in $(seq 1 ${6:-4}); do
  for v in a b; do
    echo "$v $(taskset -c 2,3 /tmp/rpab/$v /tmp/rpab/d.bin 5 | awk '/^rep/ {r=r" "$6; h=$NF} /^best/ {b=$2} END {print "best", b, "resolve", r, h}')"
  done
done
