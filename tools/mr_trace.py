"""Multi-rank greedy on one GPU, traced (diagnostics for the host-exchange path).

    python tools/mr_trace.py [world] [cfg] [topk]      # cfg3 (default) or cfg4; topk 0 = the engine default

The parent never touches the GPU: it starts `world` rank processes (this file with a rank argument),
each holding one node shard of the bench's cfg inventory on device 0 and exchanging through the
native shared-memory exchange (zero-copy windows unless PE_NO_ZC_EXCHANGE=1).  Each rank prints its
median batch time and the engine's wait / resolve split; PE_GREEDY_TRACE=1 adds per-window times.
Run it under `rocprofv3 --kernel-trace --stats -- python tools/mr_trace.py` for the kernel timeline.
"""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = {"cfg3": ("mixed", 100_000, 10_000, 0.2), "cfg4": ("island8", 100_000, 10_000, 1.0)}


def rank_main(rank, world, port, cfg, topk):
    for p in (ROOT, os.path.join(ROOT, "training-operator_amd")):
        sys.path.insert(0, p)
    import numpy as np
    import torch.distributed as dist

    from placement import Engine, HostExchange, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    names = [f"/pe_mrt_{port}" if rank == 0 else None]
    dist.broadcast_object_list(names, src=0)
    hx = HostExchange(names[0], rank, world, 128 * (16 + 8 * 256))
    dist.barrier()
    mix, n_nodes, n_jobs, frac = CFG[cfg]
    inv = synth.make_inventory(n_nodes, synth.SEED[cfg], frac)
    batch = synth.make_jobs(n_jobs, synth.SEED[cfg], mix)
    e = Engine(0, rank=rank, world_size=world, exchange=hx if world > 1 else None, max_nodes=n_nodes,
               topk=topk)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    e.place_batch(batch)
    e.reset_stats()
    ts = []
    for _ in range(5):
        e.reset_residuals()
        e.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        e.place_batch(batch)
        ts.append(time.perf_counter() - t0)
    s = e.stats()
    n = len(ts)
    print(f"rank {rank}/{world} {cfg} topk {topk or 'default'}: median {np.median(ts) * 1e3:.2f} ms (min {min(ts) * 1e3:.2f}) | per batch: "
          f"wait {s['greedy_wait_ms'] / n:.2f} ms, resolve {s['greedy_host_ms'] / n:.2f} ms, windows "
          f"{s['windows'] / n:.0f}, zero-copy {s['xchg_zc_windows'] / n:.0f}", flush=True)
    e.close()
    hx.close()
    dist.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cfg = sys.argv[2] if len(sys.argv) > 2 else "cfg3"
    topk = sys.argv[3] if len(sys.argv) > 3 else "0"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), str(world), str(port), cfg, topk])
             for r in range(world)]
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            rc = 1
    sys.exit(rc)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--rank":
        rank_main(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], int(sys.argv[6]))
    else:
        main()
