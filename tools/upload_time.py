"""Median host time of pe_jobs_upload (planning + H2D) for the cfg5 batches (headline, 400 cpu values,
worst case), one engine; library from PE_LIBRARY like the bench."""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "training-operator_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402

from fit_case import batch  # noqa: E402
from placement import Engine, synth  # noqa: E402

inv = synth.make_inventory(1_000_000, synth.SEED["cfg5"], gpu_frac=0.2)
eng = Engine(0, max_nodes=1_000_000)
eng.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
out = []
for case in ("headline", "many", "worst"):
    req, need = batch(case, 100_000)
    ts = []
    for _ in range(7):
        eng.synchronize()
        t0 = time.perf_counter()
        eng.jobs_upload(req, need)
        ts.append(time.perf_counter() - t0)
    out.append(f"{case} {np.median(ts) * 1e3:.3f} ms")
print(os.path.basename(os.environ.get("PE_LIBRARY", "tree")), " | ".join(out))
eng.close()
