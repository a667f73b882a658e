#!/bin/bash
# Kernel trace + HBM PMC passes (separate runs) of the high-cardinality fit batches: the LDS digit-plane
# kernel's traffic against its algorithmic bytes.  Output: gpurun_out/prof_fitcases/<case>_*.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_fitcases
mkdir -p $OUT
for c in many worst adversarial; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${c}_trace -o trace --output-format csv -- \
    python3 tools/fit_case.py $c 3 > $OUT/${c}.json 2> $OUT/${c}_trace.err
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${c}_fetch -o fetch --output-format csv -- \
    python3 tools/fit_case.py $c 2 > /dev/null 2> $OUT/${c}_fetch.err
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${c}_write -o write --output-format csv -- \
    python3 tools/fit_case.py $c 2 > /dev/null 2> $OUT/${c}_write.err
  echo "$c done"
done
