"""One rank of tests/test_gpu_multiproc.py: a separate process holding one inventory shard context of
the engine on device 0, exchanging the per-window candidate blobs with the other ranks over gloo
(the pe_config.exchange hook -- RCCL's role on a multi-GPU node).  Writes its results to out_dir.

    python tests/mp_shard_worker.py <rank> <world> <port> <mix> <n_nodes> <n_jobs> <out_dir> [gloo|shm]

Transport "shm": the native shared-memory exchange (pe_host_exchange) instead of the Python gloo
callback -- its zero-copy windows unless PE_NO_ZC_EXCHANGE=1; gloo then only broadcasts the segment
name.  Transport "shm-grow": the zero-copy exchange with lists of 8 keys (rescans) and segment slots
that hold the grown stride, so the ranks' lists grow to 16 after the first rescan.  Transport "shm-stall": both ranks place a small batch, then rank 0 places the test batch while
the other ranks sleep and exit -- rank 0 must fail with PE_ERCCL within the device timeout (no hang).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "training-operator_amd")):
    sys.path.insert(0, p)


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    mix, n_nodes, n_jobs, out_dir = sys.argv[4], int(sys.argv[5]), int(sys.argv[6]), sys.argv[7]
    transport = sys.argv[8] if len(sys.argv) > 8 else "gloo"
    import numpy as np
    import torch.distributed as dist

    from placement import Engine, HostExchange, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(blob: bytes) -> bytes:
        parts = [None] * world
        dist.all_gather_object(parts, blob)
        return b"".join(parts)

    if transport.startswith("shm"):
        names = [f"/pe_mp_{port}_{os.getpid()}" if rank == 0 else None]
        dist.broadcast_object_list(names, src=0)
        exchange = HostExchange(names[0], rank, world, 128 * (16 + 8 * (16 if transport == "shm-grow" else 256)))
        dist.barrier()
    topk = 8 if transport == "shm-grow" else 0

    inv = synth.make_inventory(n_nodes, 3, 0.2 if mix != "gang8" else 1.0)
    batch = synth.make_jobs(n_jobs, 3, mix)
    e = Engine(0, rank=rank, world_size=world, exchange=exchange, max_nodes=n_nodes, topk=topk)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    b, en = e.shard_range()
    if transport == "shm-stall":
        import time

        from placement import PlacementError
        e.place_batch(synth.make_jobs(20, 5, mix))   # (every rank: the zero-copy agreement, a few windows)
        zc0 = e.stats()["xchg_zc_windows"]
        if rank != 0:
            time.sleep(8)
            e.close()
            return
        t0 = time.monotonic()
        try:
            e.place_batch(batch)
            err = "no error"
        except PlacementError as ex:
            err = f"{ex.code}:{ex}"
        np.savez(os.path.join(out_dir, "stall.npz"), err=err, secs=time.monotonic() - t0, zc0=zc0)
        e.close()
        return
    pods, st = e.place_batch(batch)
    res = e.read_residuals()
    # a second batch on the updated inventory: every rank's device shard and host mirror stay in step
    batch2 = synth.make_jobs(n_jobs // 2, 4, mix)
    pods2, st2 = e.place_batch(batch2)
    res2 = e.read_residuals()
    s = e.stats()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), pods=pods, st=st, res=res, pods2=pods2, st2=st2, res2=res2,
             b=b, e=en, windows=s["windows"], zc=s["xchg_zc_windows"], rescans=s["rescans"],
             xmerge_ms=s["xchg_merge_ms"], xwait_ms=s["xchg_wait_ms"], host_ms=s["greedy_host_ms"])
    e.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
