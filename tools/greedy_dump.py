"""Record the host resolver's input of one cfg3-mix batch on the 1M-node inventory (the bench's
greedy line) for tools/replay_resolver.cc: PE_DUMP_WINDOWS=<file> on the second, warm pass.
    python tools/greedy_dump.py out.bin [max_windows]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "training-operator_amd")]
from placement import Engine, synth  # noqa: E402

out = sys.argv[1]
inv = synth.make_inventory(1_000_000, synth.SEED["cfg5"], gpu_frac=0.2)
batch = synth.make_jobs(10_000, synth.SEED["cfg3"], "mixed")
e = Engine(0, max_nodes=1_000_000)
e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
e.place_batch(batch)
e.reset_residuals()
os.environ["PE_DUMP_WINDOWS"] = out
if len(sys.argv) > 2:
    os.environ["PE_DUMP_MAX_WINDOWS"] = sys.argv[2]
e.place_batch(batch)
print(e.stats()["windows"])
