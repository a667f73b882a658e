"""N>1 path on CPU: world_size-2 torch.distributed (gloo), one process per inventory shard.

Each rank owns a contiguous node shard, produces its per-group candidate blob (test-side scan
emulation of the device kernels), the ranks all-gather the blobs over gloo -- the role RCCL plays
on the GPU -- and every rank runs the product's host resolver (pe_resolver_*).  All ranks must
make identical decisions, apply only their own residual updates, and match the unsharded oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, mix, K, out_dir):
    import sys
    for p in (ROOT, os.path.join(ROOT, "training-operator_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    from placement import Resolver, synth
    from scan_emulator import shard_blob
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inv = synth.make_inventory(900, 77, 0.3)
    batch = synth.make_jobs(80, 79, mix)
    N = inv.n
    b, e = N * rank // world, N * (rank + 1) // world
    res = inv.residual()[:, b:e].copy()                  # this rank's shard only
    labels = inv.labels[b:e]
    R = Resolver(batch.job_group_off, batch.priority, batch.group_count, batch.group_req, batch.group_need)
    windows = 0
    while not R.done():
        groups = R.next_window(8, 64)
        mine = shard_blob(res, labels, b, batch.group_req[groups], batch.group_need[groups], K)
        parts = [None] * world
        dist.all_gather_object(parts, mine)              # the exchange RCCL does on the device
        upd, _ = R.resolve(groups, b"".join(parts), world, K)
        for row in upd:
            gid = int(row[0])
            if b <= gid < e:
                res[:, gid - b] = row[1:]
        windows += 1
    pods, st = R.results()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), pods=pods, st=st, res=res, b=b, e=e, windows=windows)
    dist.destroy_process_group()


@pytest.mark.parametrize("mix,K", [("mixed", 4), ("gang8", 2)])
def test_two_rank_gloo_matches_oracle(tmp_path, mix, K):
    import oracle
    from placement import synth
    world = 2
    mp.start_processes(worker, args=(world, free_port(), mix, K, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    inv = synth.make_inventory(900, 77, 0.3)
    batch = synth.make_jobs(80, 79, mix)
    w_pods, w_st, w_res = oracle.place_greedy(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                              batch.group_count, batch.group_req, batch.group_need)
    full = np.zeros_like(w_res)
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        np.testing.assert_array_equal(d["st"], w_st)
        np.testing.assert_array_equal(d["pods"], w_pods)
        full[:, int(d["b"]):int(d["e"])] = d["res"]
    np.testing.assert_array_equal(full, w_res)
