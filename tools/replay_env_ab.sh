#!/bin/bash
# Host-resolver replay A/B of ENVIRONMENT settings on the GPU box's CPU: records the bench batch's
# windows on the GPU (tools/greedy_dump.py), then replays them interleaved with each setting, e.g.
#   tools/replay_env_ab.sh 4 "huge=" "nohuge=PE_NO_HUGE=1"
set -e
reps=$1; shift
mkdir -p /tmp/rea
timeout -k 10 300 python tools/greedy_dump.py /tmp/rea/d.bin > /dev/null
g++ -O3 -march=x86-64-v3 -std=c++17 -Itraining-operator_amd/csrc -Iinclude tools/replay_resolver.cc \
  training-operator_amd/csrc/pe_resolver.cpp -o /tmp/rea/r -lpthread
for i in $(seq $reps); do for spec in "$@"; do
  name=${spec%%=*}; env=${spec#*=}
  echo "$name $(env $env taskset -c 2,3 /tmp/rea/r /tmp/rea/d.bin 5 | awk '/^rep/ {r=r" "$6; h=$NF} END {print "resolve", r, h}')"
done; done
