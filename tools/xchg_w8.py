"""Exchange cost of the sharded greedy at W ranks, rehearsed on one GPU (verdict r5 item 3): the bench's
10k-job cfg3 batch on the 1M-node inventory through W shard contexts in one process over the native
shared-memory exchange, per rank: the exchange thread's merge and wait per window against the resolve
per window (pe_stats xchg_merge_ms / xchg_wait_ms / greedy_host_ms over windows).

    python tools/xchg_w8.py [--world 8] [--threads 1,4] [--copy] [--reps 2] [--out file.json]

--threads: PE_XCHG_THREADS values to compare (zero-copy host merge); --copy: the copying all-gather +
merge_shards_kernel at W ranks instead (run it under rocprofv3 --kernel-trace for the kernel's time).
Every rank's placements are checked against one unsharded context's."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "training-operator_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

from placement import Engine, HostExchange, synth  # noqa: E402


def run_world(inv, batch, W, reps, ref):
    name = f"/pe_xw_{os.getpid()}_{time.monotonic_ns() % 100000}"
    hxs = [HostExchange(name, r, W, 128 * (16 + 8 * 256)) for r in range(W)]
    engines = [Engine(0, rank=r, world_size=W, exchange=hxs[r], max_nodes=inv.n) for r in range(W)]
    for e in engines:
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    per = []
    for rep in range(reps):
        for e in engines:
            e.reset_residuals()
            e.reset_stats()
        out, errs = [None] * W, []

        def go(r):
            try:
                out[r] = engines[r].place_batch(batch)
            except Exception as ex:   # noqa: BLE001
                errs.append((r, repr(ex)))
        th = [threading.Thread(target=go, args=(r,)) for r in range(W)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join(300)
        wall = (time.perf_counter() - t0) * 1e3
        assert not errs, errs
        for r in range(W):
            assert np.array_equal(out[r][0], ref[0]) and np.array_equal(out[r][1], ref[1]), f"rank {r} differs"
        st = [e.stats() for e in engines]
        win = max(1, st[0]["windows"])
        per.append({"batch_ms": wall, "windows": st[0]["windows"], "rescans": st[0]["rescans"],
                    "zc_windows": st[0]["xchg_zc_windows"],
                    "merge_us_per_window": [s["xchg_merge_ms"] * 1e3 / win for s in st],
                    "wait_us_per_window": [s["xchg_wait_ms"] * 1e3 / win for s in st],
                    "resolve_us_per_window": [s["greedy_host_ms"] * 1e3 / win for s in st]})
    for e in engines:
        e.close()
    for x in hxs:
        x.close()
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--threads", default="1,4")
    ap.add_argument("--copy", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--jobs", type=int, default=10_000)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    inv = synth.make_inventory(a.nodes, synth.SEED["cfg5"], 0.2)
    batch = synth.make_jobs(a.jobs, synth.SEED["cfg3"], "mixed")
    e = Engine(0, max_nodes=a.nodes)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    ref = e.place_batch(batch)
    e.reset_stats()
    e.reset_residuals()
    t0 = time.perf_counter()
    e.place_batch(batch)
    s1 = e.stats()
    one = {"batch_ms": (time.perf_counter() - t0) * 1e3, "windows": s1["windows"],
           "resolve_us_per_window": s1["greedy_host_ms"] * 1e3 / max(1, s1["windows"])}
    e.close()
    res = {"world": a.world, "nodes": a.nodes, "jobs": a.jobs, "one_rank": one, "runs": {}}
    if a.copy:
        os.environ["PE_NO_ZC_EXCHANGE"] = "1"
        res["runs"]["copy+merge_shards_kernel"] = run_world(inv, batch, a.world, a.reps, ref)
    else:
        for t in [int(x) for x in a.threads.split(",")]:
            os.environ["PE_XCHG_THREADS"] = str(t)
            res["runs"][f"zc host merge, {t} thread(s)"] = run_world(inv, batch, a.world, a.reps, ref)
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
