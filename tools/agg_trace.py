#!/usr/bin/env python3
"""Phase times of pe_pg_min_resources calls (PE_AGG_TRACE=1: planning, packing, launch, flag wait,
unpack) at the crossover's batch sizes, the bench's v1 batch; the engine prints one line per call.
    python tools/agg_trace.py [J ...] 2> trace.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "training-operator_amd")]
import bench  # noqa: E402
from placement import Engine, synth  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [1, 256, 1024, 2048, 4096, 8192]
eng = Engine(0)
agg = synth.make_pg_batch(max(sizes), synth.SEED["cfg3"])
for J in sizes:
    call, _ = bench.agg_raw_call(eng.lib.pe_pg_min_resources, (eng.h,), 1, bench.pg_slice(agg, 0, J))
    for _ in range(30):
        call()
    os.environ["PE_AGG_TRACE"] = "1"
    for _ in range(5):
        call()
    del os.environ["PE_AGG_TRACE"]
    print(f"J {J}: median {bench.time_calls(call, 100)[0]:.1f} us", flush=True)
eng.close()
