#!/bin/bash
# Fit-kernel A/B of libplacement builds (PE_LIBRARY): bench --no-greedy per build, twice, kernel ms.
#   FXV="lib_a lib_b" tools/fit_lib_ab.sh      (builds under build_variants/)
# r5 findings: dropping the per-job count work (popcount + batched column sums + atomics) made
# the kernel SLOWER (2.16/2.23 -> 2.44 ms: the VALU work paces the 1-KiB stores), and an
# s_sleep after each store was slower too (2.33 -> 2.37 ms); 8 / 16 / 32 extra dependent VALU per
# job cost +3 / +6 / +17 % (2.21 -> 2.28 / 2.34 / 2.61 ms): per-job VALU issue is on the critical
# path, so the "no count" slowdown is the compiler's different schedule, not pacing.
set -e
for i in 1 2; do for v in ${FXV:-lib_base}; do
  line=$(PE_LIBRARY=$PWD/build_variants/$v.so timeout -k 10 120 python bench.py --no-greedy --no-configs --no-cpu-baseline --steps 10 --warmup 3)
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['roofline']['kernel_ms'],3))" $v "$line"
done; done
