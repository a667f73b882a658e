#!/usr/bin/env python3
"""Where does a 2-rank RCCL set-up with one rank missing end?  pe_create(world 2, rank 0) with
PE_RCCL_INIT_TIMEOUT_S=5, in a child process per comm id (a real unique id: rank 0 is the root and
waits for rank 1; a garbage id), timestamps on every step and at process exit; each child under
its own time limit."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, time
t0 = time.time()
def say(*a): print("[%6.2fs]" % (time.time() - t0), *a, flush=True)
sys.path[:0] = [{root!r}, os.path.join({root!r}, "training-operator_amd")]
from placement import Engine, PlacementError, comm_id
cid = {cid}
say("create")
try:
    e = Engine(0, rank=0, world_size=2, comm=cid)
    say("CREATED")
except PlacementError as ex:
    say("RC", ex.code)
say("exit")
if os.environ.get("PROBE_HARD_EXIT"):
    os._exit(0)
"""
for hard in ("0", "1"):
    for cid in ("comm_id()", "bytes(range(128))"):
        env = dict(os.environ, PE_RCCL_INIT_TIMEOUT_S="5")
        if hard == "1":
            env["PROBE_HARD_EXIT"] = "1"
        t0 = time.time()
        print(f"--- cid={cid} hard_exit={hard}", flush=True)
        try:
            p = subprocess.run([sys.executable, "-u", "-c", CHILD.format(root=ROOT, cid=cid)], env=env, timeout=40,
                               capture_output=True, text=True)
            print(p.stdout[-2000:], p.stderr[-600:], "rc", p.returncode, f"process ended after {time.time() - t0:.1f}s",
                  flush=True)
        except subprocess.TimeoutExpired as ex:
            print("TIMEOUT", (ex.stdout or b"")[-2000:], (ex.stderr or b"")[-1500:], flush=True)
