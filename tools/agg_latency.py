#!/usr/bin/env python3
"""pe_pg_min_resources per-call latency across batch sizes and call-path knobs (A/B on one box):
median of N calls through the C ABI (ctypes pointers built once), the bench's v1 batch.
    AGG_AB_CONFIGS='[{}, {"PE_AGG_SEG_JOBS": "256"}]' python tools/agg_latency.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "training-operator_amd")]
import bench  # noqa: E402
from placement import Engine, synth  # noqa: E402

configs = json.loads(os.environ.get("AGG_AB_CONFIGS", "[{}]"))
sizes = [int(x) for x in os.environ.get("AGG_AB_SIZES", "1,16,64,256,1024,8192,100000,1000000").split(",")]
eng = Engine(0)
agg = synth.make_pg_batch(max(sizes), synth.SEED["cfg3"])
for rep in range(2):
    for cfg in configs:
        for k in ("PE_AGG_SEG_JOBS", "PE_AGG_DEVICE"):
            os.environ.pop(k, None)
        os.environ.update(cfg)
        row = []
        for J in sizes:
            sub = bench.pg_slice(agg, 0, J)
            call, _ = bench.agg_raw_call(eng.lib.pe_pg_min_resources, (eng.h,), 1, sub)
            n = 400 if J <= 1024 else (50 if J <= 100000 else 7)
            med, _ = bench.time_calls(call, n, warm=3 if J > 100000 else 20)
            row.append(f"{J}:{med:.1f}")
        print(f"rep {rep} {str(cfg):<36} us " + " ".join(row), flush=True)
eng.close()
