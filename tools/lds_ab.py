"""LDS digit-plane fit path: step time per batch shape and configuration (1M nodes x 100k jobs).
HIP events on the engine stream, median of 5 steps.  Configurations come from the environment the
engine reads at upload (PE_LDS_W = block size 2048 W, PE_LDS_MAXL = digit levels cap).
    python tools/lds_ab.py [shape ...]            shapes: many worst adversarial cfg5
"""
import os
import statistics
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "training-operator_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
from bench import HipEvents  # noqa: E402
from placement import Engine, synth  # noqa: E402

N, J = 1_000_000, 100_000


def batch(shape):
    req, need = synth.make_fit_jobs(J, synth.SEED["cfg5"])
    if shape == "many":
        req[:, 0] = 250 * (1 + np.arange(J) % 400)
    elif shape == "worst":
        req, need = synth.make_fit_jobs_worst(J, synth.SEED["cfg5"], (1,))
    elif shape == "adversarial":
        req, need = synth.make_fit_jobs_worst(J, synth.SEED["cfg5"], (0, 1, 3))
    return req, need


def main():
    shapes = sys.argv[1:] or ["many", "worst", "adversarial", "cfg5"]
    configs = [dict(), dict(PE_LDS_W="4"), dict(PE_LDS_W="2"), dict(PE_LDS_W="1"), dict(PE_LDS_MAXL="2"),
               dict(PE_LDS_MAXL="3", PE_LDS_W="2")]
    if os.environ.get("LDS_AB_CONFIGS"):   # JSON list of environment dicts
        import json
        configs = json.loads(os.environ["LDS_AB_CONFIGS"])
    inv = synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2)
    ev = HipEvents()
    a, b = ev.create(), ev.create()
    os.environ["PE_LDS_DEBUG"] = "1"
    for shape in shapes:
        req, need = batch(shape)
        ref = None
        for cfg in configs:
            for k in ("PE_LDS_W", "PE_LDS_MAXL", "PE_LDS_NOSORT", "PE_LDS_R", "PE_LDS_SORTED"):
                os.environ.pop(k, None)
            os.environ.update(cfg)
            e = Engine(0, max_nodes=N, fit_path_mask=64 if shape != "cfg5" else 0)
            e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
            e.jobs_upload(req, need)
            e.fit_mask_run()
            e.synchronize()
            t = []
            for _ in range(5):
                ev.record(a, e.stream())
                e.fit_mask_run()
                ev.record(b, e.stream())
                e.synchronize()
                t.append(ev.elapsed_ms(a, b))
            s = e.stats()
            cnt = e.fit_counts()
            ref = cnt if ref is None else ref
            path = "lds" if s["fit_runs_lds"] else ("planes" if s["fit_runs_planes"] else "other")
            lib = os.path.basename(os.environ.get("PE_LIBRARY", "libplacement.so"))
            print(f"{lib:<16} {shape:<12} {str(cfg):<40} {statistics.median(t):7.3f} ms  path {path}  "
                  f"same {bool(np.array_equal(cnt, ref))}", flush=True)
            e.close()


if __name__ == "__main__":
    main()
