#!/bin/bash
# Section cycle profile (-DPE_RES_PROF) of the host resolver on the GPU box's CPU, on a dump recorded
# there first (tools/greedy_dump.py: the bench batch's windows), plus the unprofiled replay time.
#   tools/replay_prof_gen.sh [src.cpp ...]
set -e
mkdir -p /tmp/rpg
timeout -k 10 300 python tools/greedy_dump.py /tmp/rpg/d.bin > /dev/null
srcs=("$@"); [ ${#srcs[@]} -eq 0 ] && srcs=(training-operator_amd/csrc/pe_resolver.cpp)
for s in "${srcs[@]}"; do
  g++ -O3 -march=x86-64-v3 -std=c++17 -DPE_RES_PROF -I"$(dirname "$s")" -Itraining-operator_amd/csrc -Iinclude \
    tools/replay_resolver.cc "$s" -o /tmp/rpg/rp -lpthread
  g++ -O3 -march=x86-64-v3 -std=c++17 -I"$(dirname "$s")" -Itraining-operator_amd/csrc -Iinclude \
    tools/replay_resolver.cc "$s" -o /tmp/rpg/r -lpthread
  echo "== $s"
  taskset -c 2,3 /tmp/rpg/r /tmp/rpg/d.bin 5 2>&1 | grep -v "^rep [1-4]"
  taskset -c 2,3 /tmp/rpg/rp /tmp/rpg/d.bin 3 2>&1 | grep -v "^rep"
done
