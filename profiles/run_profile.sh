#!/bin/bash
# Profiles the bench workload on the GPU box (run via gpurun from the repo root).
#   1) kernel trace + stats of the full bench (fit mask + greedy)        -> gpurun_out/prof_<tag>
#   2) separate PMC passes (never combined with sys/runtime traces):
#      FETCH_SIZE, WRITE_SIZE (HBM traffic; gfx950 FETCH_SIZE reads 1/2 of wide streaming reads),
#      SQ instruction mix of the fit-mask kernel
# Usage: profiles/run_profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r1}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
BENCH_SMALL="--steps 2 --warmup 1 --no-greedy --no-configs --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- \
  python3 bench.py $BENCH_SMALL "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- \
  python3 bench.py $BENCH_SMALL "$@" > $OUT/bench_write.json 2> $OUT/write.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  -d $OUT/sq -o sq --output-format csv -- python3 bench.py $BENCH_SMALL "$@" > $OUT/bench_sq.json 2> $OUT/sq.err
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 \
  -d $OUT/sq2 -o sq2 --output-format csv -- python3 bench.py $BENCH_SMALL "$@" > $OUT/bench_sq2.json 2> $OUT/sq2.err
# greedy walk kernel without the bench's hipEvent passes: warm (as the bench runs) and cold (a 512 MiB
# buffer rewritten before every walk launch, PE_WALK_FLUSH)
GREEDY_ONLY="--steps 2 --warmup 1 --no-configs --no-cpu-baseline --no-walk-passes"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/walk_warm -o walk --output-format csv -- \
  python3 bench.py $GREEDY_ONLY "$@" > $OUT/bench_walk_warm.json 2> $OUT/walk_warm.err
PE_WALK_FLUSH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/walk_cold -o walk --output-format csv -- \
  python3 bench.py $GREEDY_ONLY "$@" > $OUT/bench_walk_cold.json 2> $OUT/walk_cold.err
# HBM-side traffic of the greedy passes (FETCH_SIZE / WRITE_SIZE per walk launch, separate passes)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/walk_fetch -o walk_fetch --output-format csv -- \
  python3 bench.py $GREEDY_ONLY "$@" > $OUT/bench_walk_fetch.json 2> $OUT/walk_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/walk_write -o walk_write --output-format csv -- \
  python3 bench.py $GREEDY_ONLY "$@" > $OUT/bench_walk_write.json 2> $OUT/walk_write.err
# aggregation: the 1M-job call alone
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/agg -o agg --output-format csv -- \
  python3 tools/agg_calls.py > $OUT/agg.out 2> $OUT/agg.err
python3 profiles/summarize.py $OUT > $OUT/summary.json
echo "profile $TAG done"
