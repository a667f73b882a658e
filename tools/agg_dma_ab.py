#!/usr/bin/env python3
"""The 1M-job aggregation call (bench.py's v1 batch, the C ABI on caller-owned arrays as the bench times
it) under call-path settings, each in a child process (the engine reads PE_AGG_CHUNKS once):
median of 9 calls after 3 warm-ups, interleaved over 2 reps, beside the box's PCIe rates and the
batch's bound (max(in / h2d, out / d2h)) and the round-2 path (PE_AGG_DEVICE=1).
    python tools/agg_dma_ab.py "dma,8" "dma,16" "zc,8" "dma,8,PE_AGG_ONE_PLAN=1" ...
(a third field: environment settings of that child, K=V joined by +)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, statistics, json
sys.path[:0] = [%r, os.path.join(%r, "training-operator_amd")]
import bench
from placement import Engine, synth
eng = Engine(0)
agg = synth.make_pg_batch(1_000_000, synth.SEED["cfg3"])
call, outs = bench.agg_raw_call(eng.lib.pe_pg_min_resources, (eng.h,), 1, agg)
for _ in range(3): call()
t = []
for _ in range(9):
    t0 = time.perf_counter(); call(); t.append((time.perf_counter() - t0) * 1e3)
ref = eng.pg_min_resources(1, *agg)
same = all((a == b).all() for a, b in zip(outs, ref))
print(json.dumps({"median_ms": statistics.median(t), "min_ms": min(t), "same_as_wrapper": bool(same)}))
''' % (ROOT, ROOT)

sys.path[:0] = [ROOT, os.path.join(ROOT, "training-operator_amd")]
res = {}
for rep in range(2):
    for cfg in sys.argv[1:] + ["r2,8"]:
        mode, ch, *extra = cfg.split(",")
        env = dict(os.environ, PE_AGG_CHUNKS=ch)
        for kv in (extra[0].split("+") if extra else []):   # "dma,8,PE_AGG_ONE_PLAN=1+PE_POOL_SPIN_US=0"
            k, v = kv.split("=")
            env[k] = v
        env.pop("PE_AGG_ZEROCOPY", None)
        env.pop("PE_AGG_DEVICE", None)
        if mode == "zc":
            env["PE_AGG_ZEROCOPY"] = "1"
        if mode == "r2":
            env["PE_AGG_DEVICE"] = "1"
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=180)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        r = json.loads(line[0]) if line else {"error": out.stderr[-500:]}
        res.setdefault(cfg, []).append(r)
        print(cfg, r, flush=True)
import bench  # noqa: E402
from placement import synth  # noqa: E402
agg = synth.make_pg_batch(1_000_000, synth.SEED["cfg3"])
mb = bench.agg_bytes(agg[0], agg[3])
pcie = bench.pcie_rates()
inb, outb = mb - 38 * 1_000_000, 38 * 1_000_000
summary = {"runs": res, "pcie": pcie, "alg_bytes": mb,
           "pcie_bound_ms": mb / pcie["h2d_gbs"] / 1e6 if pcie else None,
           "pcie_bound_duplex_ms": max(inb / pcie["h2d_gbs"], outb / pcie["d2h_gbs"]) / 1e6 if pcie else None}
print(json.dumps(summary))
