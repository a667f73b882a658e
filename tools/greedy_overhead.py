"""Where a greedy batch's time goes outside the host resolve and the device wait: the bench's batch
(cfg3 mix, 10k jobs, 1M nodes), per repetition the Python-level wall time of place_batch, the engine's
own wall time (pe_stats.last_greedy_ms), its host resolve and device wait; the rest is set-up (walk
index rebuild, resolver construction, threads) and tail (final sync, outputs).
    python tools/greedy_overhead.py [reps]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "training-operator_amd")]
from placement import Engine, synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
inv = synth.make_inventory(1_000_000, synth.SEED["cfg5"], gpu_frac=0.2)
batch = synth.make_jobs(10_000, synth.SEED["cfg3"], "mixed")
e = Engine(0, max_nodes=1_000_000)
e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
e.place_batch(batch)
for r in range(reps):
    e.reset_residuals()
    e.synchronize()
    e.reset_stats()
    t0 = time.perf_counter()
    e.place_batch(batch)
    wall = (time.perf_counter() - t0) * 1e3
    s = e.stats()
    eng, host, wait = s["last_greedy_ms"], s["greedy_host_ms"], s["greedy_wait_ms"]
    print(f"wall {wall:.2f} ms  engine {eng:.2f}  host {host:.2f}  wait {wait:.2f}  rest {eng - host - wait:.2f}  "
          f"python {wall - eng:.2f}  windows {s['windows']}", flush=True)
