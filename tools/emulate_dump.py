"""Inputs of tools/emulate_dump.cc: the bench's greedy workload (cfg3 10k-job mix on the 1M-node
cfg5-seed inventory), or another (nodes, seed, jobs, mix), as one raw file.
    python tools/emulate_dump.py inputs.bin [n_nodes inv_seed n_jobs job_seed mix gpu_frac]"""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "training-operator_amd")]
from placement import synth  # noqa: E402

a = sys.argv[2:]
N = int(a[0]) if a else 1_000_000
inv = synth.make_inventory(N, int(a[1]) if a else synth.SEED["cfg5"], float(a[5]) if len(a) > 5 else 0.2)
b = synth.make_jobs(int(a[2]) if a else 10_000, int(a[3]) if a else synth.SEED["cfg3"], a[4] if a else "mixed")
with open(sys.argv[1], "wb") as f:
    np.array([N, b.n_jobs], dtype=np.int64).tofile(f)
    np.ascontiguousarray(inv.residual(), dtype=np.int64).tofile(f)
    np.ascontiguousarray(inv.labels, dtype=np.uint32).tofile(f)
    np.ascontiguousarray(b.job_group_off, dtype=np.int32).tofile(f)
    np.ascontiguousarray(b.priority, dtype=np.int32).tofile(f)
    np.ascontiguousarray(b.group_count, dtype=np.int32).tofile(f)
    np.ascontiguousarray(b.group_req, dtype=np.int64).tofile(f)
    np.ascontiguousarray(b.group_need, dtype=np.uint32).tofile(f)
