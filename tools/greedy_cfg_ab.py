"""Interleaved greedy A/B in ONE process: several engine configurations (pe_config window / K /
resort settings) over the same 1M-node inventory and cfg3-mix batch, run round-robin so the shared
host's speed drift hits every configuration alike; median ms per batch (+ host / wait) per config.
    python tools/greedy_cfg_ab.py "wg=64" "wg=128" "wg=128,k=320" ... [--reps 5]"""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "training-operator_amd")]
from placement import Engine, synth  # noqa: E402

KEYS = {"wg": "window_groups", "wp": "window_pods", "k": "topk", "rs": "resort_nodes", "gf": "greedy_flags"}
ENVS = {"d": "PE_PIPE_DEPTH", "ar": "PE_ASYNC_RESORT"}   # environment settings read per pe_place_greedy call


def parse(spec):
    kw, env = {}, {}
    for part in spec.split(","):
        k, v = part.split("=")
        if k in ENVS:
            env[ENVS[k]] = v
        else:
            kw[KEYS[k]] = int(v)
    return kw, env


def with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = 5
    if "--reps" in sys.argv:
        reps = int(sys.argv[sys.argv.index("--reps") + 1])
        args = [a for a in args if a != str(reps)]
    inv = synth.make_inventory(1_000_000, synth.SEED["cfg5"], gpu_frac=0.2)
    batch = synth.make_jobs(10_000, synth.SEED["cfg3"], "mixed")
    engines = []
    for spec in args:
        kw, env = parse(spec)
        e = Engine(0, max_nodes=1_000_000, **kw)
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        with_env(env, lambda: e.place_batch(batch))   # warm-up
        engines.append((spec, e, [], env))
    ref = None
    for _ in range(reps):
        for spec, e, rec, env in engines:
            e.reset_residuals()
            e.reset_stats()
            e.synchronize()
            pods, st = with_env(env, lambda: e.place_batch(batch))
            s = e.stats()
            rec.append((s["last_greedy_ms"], s["greedy_host_ms"], s["greedy_wait_ms"], s["windows"], s["rescans"]))
            if ref is None:
                ref = (pods, st)
            assert np.array_equal(ref[0], pods) and np.array_equal(ref[1], st), spec
    for spec, e, rec, _ in engines:
        a = np.array(rec)
        m = np.median(a, axis=0)
        print(f"{spec:<28} {m[0]:6.2f} ms ({a[:, 0].min():.2f}-{a[:, 0].max():.2f})  {10_000 / m[0] * 1e3:8.0f}/s  "
              f"host {m[1]:5.2f}  wait {m[2]:5.2f}  windows {m[3]:.0f}  rescans {m[4]:.0f}", flush=True)
        e.close()


if __name__ == "__main__":
    main()
