"""Run one cfg5-sized fit batch on the GPU a few times (for rocprofv3 kernel-trace / PMC passes on a
single fit path): the headline batch, the 400-cpu-value batch, the worst case (memory unique per
job) or the adversarial one (cpu, memory and ephemeral unique per job) -- the same batches as
bench.py's fit lines.  Prints the path, hipEvent-free wall ms per step and the algorithmic bytes.
    python tools/fit_case.py worst [steps]"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "training-operator_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from placement import Engine, synth  # noqa: E402


def batch(case, J):
    req, need = synth.make_fit_jobs(J, synth.SEED["cfg5"])
    if case == "many":
        req = req.copy()
        req[:, 0] = 250 * (1 + np.arange(J) % 400)
    elif case == "worst":
        req, need = synth.make_fit_jobs_worst(J, synth.SEED["cfg5"], (1,))
    elif case == "adversarial":
        req, need = synth.make_fit_jobs_worst(J, synth.SEED["cfg5"], (0, 1, 3))
    return req, need


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "worst"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    N, J = 1_000_000, 100_000
    inv = synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2)
    eng = Engine(0, max_nodes=N)
    eng.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    req, need = batch(case, J)
    st0 = eng.stats()
    eng.jobs_upload(req, need)
    eng.fit_mask_run()
    eng.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.fit_mask_run()
    eng.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    path = bench.fit_path_of(eng.stats(), st0, False)
    print(json.dumps({"case": case, "fit_path": path, "kernel": bench.STEP_KERNELS[path][0], "ms_per_step": ms,
                      "alg_bytes": bench.fit_bytes(N, J), "feasible_pairs": int(eng.fit_counts().sum())}))
    eng.close()


if __name__ == "__main__":
    main()
