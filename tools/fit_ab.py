"""In-process A/B of fit-mask variants on the cfg5 workload (1M nodes x 100k jobs): separate
bench processes drift by a few % (box clocks, order), so the variants here share one process and
their timed runs are interleaved round-robin.  A variant = env settings read by the engine at
upload time (row layout) or at launch time (launch parameters); one Engine per variant.
  python tools/fit_ab.py "PE_NOPAD=1" "" "PE_ROWS_LDS=98304" ...   ("" = default)
"""
import os
import statistics
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "training-operator_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
from bench import HipEvents  # noqa: E402
from placement import Engine, synth  # noqa: E402

N, J, ROUNDS, REPS = 1_000_000, 100_000, 8, 4


def env_of(spec):
    return dict(kv.split("=", 1) for kv in spec.split(",") if kv)


def main():
    specs = sys.argv[1:] or [""]
    keys = {k for s in specs for k in env_of(s)}
    inv = synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2)
    req, need = synth.make_fit_jobs(J, synth.SEED["cfg5"])
    ev = HipEvents()

    def apply(spec):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env_of(spec))

    engs = []
    for s in specs:
        apply(s)
        e = Engine(0, max_nodes=N)
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        e.jobs_upload(req, need)
        e.fit_mask_run()
        e.synchronize()
        engs.append(e)
    times = [[] for _ in specs]
    a, b = ev.create(), ev.create()
    for _ in range(ROUNDS):
        for i, (s, e) in enumerate(zip(specs, engs)):
            apply(s)
            ev.record(a, e.stream())
            for _ in range(REPS):
                e.fit_mask_run()
            ev.record(b, e.stream())
            times[i].append(ev.elapsed_ms(a, b) / REPS)
    for i, (s, e) in enumerate(zip(specs, engs)):
        t = times[i]
        print(f"{i} {s or 'default':<34} median {statistics.median(t):.3f} ms  min {min(t):.3f}  max {max(t):.3f}  "
              f"pitch {e.fit_mask_row_pitch()}  feasible {int(e.fit_counts().sum())}", flush=True)
        e.close()


if __name__ == "__main__":
    main()
