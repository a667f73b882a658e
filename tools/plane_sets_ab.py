"""Fit-mask time for cfg5-sized batches with many distinct request values (1M nodes x 100k jobs):
plane sets (default) against the paths that held such batches before (fit_path_mask 7: int64 /
int32 compare and the dictionary-coded kernel).  HIP events on the engine stream, median of 5.
  python tools/plane_sets_ab.py
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


def shapes():
    rng = np.random.default_rng(7)
    req, need = synth.make_fit_jobs(J, synth.SEED["cfg5"])
    yield "cfg5 (25 pairs, one set)", req.copy(), need.copy()
    r = req.copy()
    r[:, 0] = rng.integers(1, 64, J) * 250                       # 63 cpu values
    yield "cpu x63", r, need.copy()
    r = req.copy()
    r[:, 0] = rng.integers(1, 120, J) * 250                      # 119 cpu, 59 mem, 29 eph values
    r[:, 1] = rng.integers(1, 60, J) * (1 << 28)
    r[:, 3] = rng.integers(0, 30, J) * (1 << 30)
    yield "cpu x119 mem x59 eph x30 (random)", r, need.copy()
    r = req.copy()
    r[:, 0] = 250 * (1 + np.arange(J) % 400)                    # 400 cpu values
    yield "cpu x400", r, need.copy()


def main():
    inv = synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2)
    ev = HipEvents()
    a, b = ev.create(), ev.create()
    for name, req, need in shapes():
        pairs = sum(len(np.unique(req[:, d])) for d in range(4)) + len(np.unique(need))
        res = {}
        for label, mask in (("planes/sets", 0), ("no planes", 7)):
            e = Engine(0, max_nodes=N, fit_path_mask=mask)
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
            path = [k for k in ("fit_runs_planes", "fit_runs_coded", "fit_runs_i32", "fit_runs_i64") if s[k]][0]
            res[label] = (statistics.median(t), path, int(e.fit_counts().sum()))
            e.close()
        line = "  ".join(f"{k}: {v[0]:.3f} ms ({v[1][9:]})" for k, v in res.items())
        same = res["planes/sets"][2] == res["no planes"][2]
        print(f"{name:<28} pairs {pairs:4d}  {line}  feasible equal {same}", flush=True)


if __name__ == "__main__":
    main()
