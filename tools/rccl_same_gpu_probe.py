"""Can two RCCL ranks share this box's one GPU?  Two processes, each an engine context with a 1-of-2
RCCL communicator on device 0 (comm id from rank 0 through a file), place a small batch and compare
with the oracle.  Prints the outcome per rank (a set-up error is an answer too).
    python tools/rccl_same_gpu_probe.py"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, time
sys.path[:0] = [{root!r}, os.path.join({root!r}, "training-operator_amd")]
import numpy as np
import oracle
from placement import Engine, PlacementError, comm_id, synth
rank, path = int(sys.argv[1]), sys.argv[2]
if rank == 0:
    open(path + ".tmp", "wb").write(comm_id()); os.rename(path + ".tmp", path)
while not os.path.exists(path): time.sleep(0.05)
cid = open(path, "rb").read()
t0 = time.time()
try:
    e = Engine(0, rank=rank, world_size=2, comm=cid, topk=16, window_groups=16)
except PlacementError as ex:
    print("RANK", rank, "SETUP-ERR", ex.code, str(ex)[:200], round(time.time() - t0, 1), flush=True); os._exit(0)
print("RANK", rank, "comm ranks", e.comm_ranks(), flush=True)
inv = synth.make_inventory(4000, 7, 0.25); b = synth.make_jobs(200, 9, "mixed")
e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
try:
    pods, st = e.place_batch(b)
    w = oracle.place_greedy(inv.residual(), inv.labels, b.job_group_off, b.priority, b.group_count, b.group_req, b.group_need)
    print("RANK", rank, "PLACED", "exact" if (np.array_equal(pods, w[0]) and np.array_equal(st, w[1])) else "MISMATCH",
          e.stats()["windows"], flush=True)
except PlacementError as ex:
    print("RANK", rank, "PLACE-ERR", ex.code, str(ex)[:200], flush=True)
e.close()
os._exit(0)
"""
with tempfile.TemporaryDirectory() as d:
    path = os.path.join(d, "cid")
    env = dict(os.environ, PE_RCCL_INIT_TIMEOUT_S="30", PE_RCCL_TIMEOUT_S="20")
    ps = [subprocess.Popen([sys.executable, "-c", CHILD.format(root=ROOT), str(r), path], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    for p in ps:
        try:
            out, _ = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        print("\n".join(ln for ln in out.splitlines() if "RANK" in ln or "rror" in ln)[-2000:], flush=True)
