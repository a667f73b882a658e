#!/bin/bash
# SQ counter passes (one rocprofv3 run each, separate from the kernel trace) of one LDS fit case:
# LDS issue / wait / conflicts and VALU / SALU activity of fit_mask_lds_kernel.
#   tools/profile_lds_sq.sh <case> <tag>     -> gpurun_out/prof_lds_<tag>/
set -e
export TMPDIR=/tmp
c=${1:-adversarial}; OUT=gpurun_out/prof_lds_${2:-x}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- \
  python3 tools/fit_case.py $c 3 > $OUT/${c}.json 2> $OUT/trace.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU \
  -d $OUT/sqa -o sqa --output-format csv -- python3 tools/fit_case.py $c 2 > /dev/null 2> $OUT/sqa.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL \
  -d $OUT/sqb -o sqb --output-format csv -- python3 tools/fit_case.py $c 2 > /dev/null 2> $OUT/sqb.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- \
  python3 tools/fit_case.py $c 2 > /dev/null 2> $OUT/write.err
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/*/*/*counter_collection.csv") + glob.glob(out + "/*/*counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "fit_mask_lds" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f.split("/")[-3], k, "%.4g per launch (%d launches)" % (sum(v) / len(v), len(v)))
PY
