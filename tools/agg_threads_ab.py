#!/usr/bin/env python3
"""1M-job aggregation call (the bench's v1 batch) under planning-thread / chunk settings, each in a
child process (the engine reads PE_AGG_THREADS / PE_AGG_CHUNKS once): median of 9 calls after 3
warm-ups, interleaved over 2 reps.
    python tools/agg_threads_ab.py "8,8" "16,8" "16,16" ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, statistics
sys.path[:0] = [%r, os.path.join(%r, "training-operator_amd")]
from placement import Engine, synth
eng = Engine(0)
agg = synth.make_pg_batch(1_000_000, synth.SEED["cfg3"])
for _ in range(3): eng.pg_min_resources(1, *agg)
t = []
for _ in range(9):
    t0 = time.perf_counter(); eng.pg_min_resources(1, *agg); t.append((time.perf_counter() - t0) * 1e3)
print("%%.3f %%.3f" %% (statistics.median(t), min(t)))
''' % (ROOT, ROOT)
for rep in range(2):
    for cfg in sys.argv[1:]:
        th, ch = cfg.split(",")
        env = dict(os.environ, PE_AGG_THREADS=th, PE_AGG_CHUNKS=ch)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
        print(f"threads {th:>2} chunks {ch:>2}: median/min ms {out.stdout.strip()} {out.stderr.strip()[-200:]}", flush=True)
