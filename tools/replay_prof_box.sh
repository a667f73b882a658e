#!/bin/bash
# Section cycle profile (-DPE_RES_PROF) of the host resolver on the GPU box's CPU: replays the recorded
# window dump (tools/greedy_dump.py) with the tree's resolver, 3 reps on 2 pinned CPUs.
#   tools/replay_prof_box.sh dump.bin.xz [src.cpp]
set -e
mkdir -p /tmp/rp && xz -dc "$1" > /tmp/rp/d.bin
src=${2:-training-operator_amd/csrc/pe_resolver.cpp}
g++ -O3 -march=x86-64-v3 -std=c++17 -DPE_RES_PROF -I"$(dirname "$src")" -Itraining-operator_amd/csrc -Iinclude \
  tools/replay_resolver.cc "$src" -o /tmp/rp/rp -lpthread
g++ -O3 -march=x86-64-v3 -std=c++17 -I"$(dirname "$src")" -Itraining-operator_amd/csrc -Iinclude \
  tools/replay_resolver.cc "$src" -o /tmp/rp/r -lpthread
taskset -c 2,3 /tmp/rp/r /tmp/rp/d.bin 5 2>&1 | grep -v "^rep"
taskset -c 2,3 /tmp/rp/rp /tmp/rp/d.bin 3 2>&1 | grep -v "^rep"
