#!/bin/bash
# Greedy host-resolve time vs host thread placement on the GPU box: interleaved runs with the
# resolver bound to the GPU's NUMA node (default) and left to the OS (PE_NUMA_BIND=0); prints the
# per-window resolve summary (PE_GREEDY_TRACE) and the CPUs the two threads ran on.
set -e
lscpu | grep -E "Model name|NUMA node"
for i in 1 2 3 4; do   # PE_NUMA_BIND was an experimental build switch (see profiles/r6_greedy_ab.txt)
  for b in 1 0; do
    PE_NUMA_BIND=$b PE_GREEDY_TRACE=1 timeout -k 10 120 python bench.py --no-configs --no-cpu-baseline --steps 1 \
      --warmup 1 --greedy-steps 1 > gpurun_out/hm.json 2> gpurun_out/hm.err
    echo "bind=$b $(grep -E 'resolve' gpurun_out/hm.err | tail -1 | cut -c1-60) | $(grep cpus gpurun_out/hm.err | tail -1)"
  done
done
