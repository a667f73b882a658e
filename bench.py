#!/usr/bin/env python3
"""Benchmark of the gang-placement hot path (BASELINE.json metric).

A "step" = one fit-mask pass (config 5): every job of the batch evaluated against every node of
the 1M-node inventory, mask + per-job counts written to HBM, inputs already resident.  The
inventory is node-sharded over the ranks (north_star); scaling is weak: the batch holds
100k x n_gpus jobs, so every rank evaluates 100k jobs x 1M nodes worth of pairs (its 1M/N-node
shard x the whole batch) per step with no collective on the data path.
`value` = job x node fit evaluations per second for the whole job (all ranks).  The second half
of the metric, gang placements/s, is measured on the same 1M-node inventory with a 10k-job
mixed PyTorch/MPI/JAX batch (config 3 mix) and reported in the "greedy" object.

    python bench.py [--gpus N --steps K --warmup W]          (N>1: one rank per GPU, torchrun)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "training-operator_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

from placement import Engine, comm_id, synth  # noqa: E402

METRIC = "job×node fit evals/sec + gang placements/sec, 1M-node inventory, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# chip-wide integer VALU issue ceiling, wave-instructions/s: profiles/r1_ubench_valu.txt
# (v_add_u32 / v_addc_co at 8 waves per SIMD: 4.24 cycles per wave-instruction per SIMD, 256 CUs x 4 SIMDs)
VALU_ISSUE_CEILING = 5.79e11
KERNEL_OF_PATH = {"planes": "pe::fit_mask_planes_rows_kernel", "planes-blocks": "pe::fit_mask_planes_kernel", "coded-therm": "pe::fit_mask_coded_kernel", "coded-swar": "pe::fit_mask_coded_kernel",
                  "i32": "pe::fit_mask_kernel", "i64": "pe::fit_mask_kernel"}
PROFILES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")


class HipEvents:
    """hipEvent timing on the engine's own stream (torch events only see torch's stream)."""

    def __init__(self):
        self.lib = ctypes.CDLL("libamdhip64.so")
        self.lib.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.lib.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        self.lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        self.lib.hipEventDestroy.argtypes = [ctypes.c_void_p]

    def create(self):
        ev = ctypes.c_void_p()
        assert self.lib.hipEventCreate(ctypes.byref(ev)) == 0
        return ev

    def record(self, ev, stream):
        assert self.lib.hipEventRecord(ev, ctypes.c_void_p(stream)) == 0

    def elapsed_ms(self, a, b):
        assert self.lib.hipEventSynchronize(b) == 0
        ms = ctypes.c_float()
        assert self.lib.hipEventElapsedTime(ctypes.byref(ms), a, b) == 0
        return float(ms.value)


def fit_bytes(n_nodes: int, n_jobs: int) -> int:
    """Algorithmic HBM bytes of one fit-mask launch over n_nodes:
    node residuals 4x8 B + labels 4 B read once, job request 4x8 B + need 4 B read once,
    mask J*ceil(N/64)*8 B written once, per-job counts 8 B written."""
    return n_nodes * 36 + n_jobs * 36 + n_jobs * ((n_nodes + 63) // 64) * 8 + n_jobs * 8


def profiled_counter(kernel: str, n_nodes: int, n_jobs: int, counter: str):
    """One PMC counter per launch of `kernel` from the committed profile (profiles/LATEST), if it was
    taken on this same workload; else None."""
    try:
        tag = open(os.path.join(PROFILES, "LATEST")).read().strip()
        summ = json.load(open(os.path.join(PROFILES, tag, "summary.json")))
    except (OSError, ValueError):
        return None
    wl = summ.get("workload", {})
    if wl.get("nodes") != n_nodes or wl.get("jobs") != n_jobs:
        return None
    for k, p in summ.get("pmc", {}).items():
        if k.startswith(kernel) and counter in p:
            return p[counter]
    return None


def profiled_traffic(kernel: str, n_nodes: int, n_jobs: int):
    """HBM bytes per launch of `kernel` from the committed PMC passes (profiles/LATEST names the
    directory; FETCH_SIZE doubled per MI355X_MICROARCH.md, + WRITE_SIZE), if they were taken on this
    same workload.  None when no matching profile exists."""
    try:
        tag = open(os.path.join(PROFILES, "LATEST")).read().strip()
        summ = json.load(open(os.path.join(PROFILES, tag, "summary.json")))
    except (OSError, ValueError):
        return None, None
    wl = summ.get("workload", {})
    if wl.get("nodes") != n_nodes or wl.get("jobs") != n_jobs:
        return None, None
    for k, p in summ.get("pmc", {}).items():
        if k.startswith(kernel) and "hbm_traffic_bytes" in p:
            return p["hbm_traffic_bytes"], f"profiles/{tag}/summary.json (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE)"
    return None, None


def _count(n: int) -> str:
    return f"{n // 1_000_000}M" if n % 1_000_000 == 0 else (f"{n // 1000}k" if n % 1000 == 0 else str(n))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--fit-jobs", type=int, default=100_000)
    ap.add_argument("--greedy-jobs", type=int, default=10_000)
    ap.add_argument("--greedy-steps", type=int, default=2)
    ap.add_argument("--topk", type=int, default=0)
    ap.add_argument("--window-groups", type=int, default=0)
    ap.add_argument("--window-pods", type=int, default=0)
    ap.add_argument("--no-greedy", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the cfg2-4 greedy lines")
    ap.add_argument("--cpu-sample-jobs", type=int, default=20000)
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: batch = fit-jobs x n_gpus (fixed per-rank work); strong: batch = fit-jobs")
    ap.add_argument("--fit-path-mask", type=int, default=0, help="pe_config.fit_path_mask (0 = every kernel)")
    ap.add_argument("--greedy-flags", type=int, default=0,
                    help="pe_config.greedy_flags (bit0: sequential windows, bit1: full scan instead of the sorted walk)")
    ap.add_argument("--resort-nodes", type=int, default=0, help="pe_config.resort_nodes (0 = default)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    cid, exchange, device = None, None, local
    host_exchange = os.environ.get("PE_BENCH_EXCHANGE", "rccl") == "host"
    if world > 1:
        import torch
        import torch.distributed as dist
        if host_exchange:
            # rehearsal mode for a 1-GPU box: every rank on one device, candidate blobs exchanged
            # over gloo instead of RCCL (the driver's multi-GPU runs use the RCCL default)
            dist.init_process_group("gloo")
            device = int(os.environ.get("PE_BENCH_DEVICE", "0"))
            tdev = "cpu"

            def exchange(blob: bytes) -> bytes:
                parts = [None] * world
                dist.all_gather_object(parts, blob)
                return b"".join(parts)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            tdev = "cuda"

        def new_comm():
            """A fresh RCCL unique id per engine (an id bootstraps exactly one communicator)."""
            if host_exchange:
                return None
            ids = [comm_id() if rank == 0 else None]
            dist.broadcast_object_list(ids, src=0)
            return ids[0]

        cid = new_comm()

        def barrier():
            dist.barrier()

        def allmax(x: float) -> float:
            t = torch.tensor([x], dtype=torch.float64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())

        def allsum(x: int) -> int:
            t = torch.tensor([x], dtype=torch.int64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            return int(t.item())
    else:
        def new_comm():
            return None

        def barrier():
            pass

        def allmax(x):
            return x

        def allsum(x):
            return x

    N = args.nodes
    J = args.fit_jobs * (world if args.scaling == "weak" else 1)
    inv = synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2)
    eng = Engine(device, rank=rank, world_size=world, comm=cid, exchange=exchange, max_nodes=N, topk=args.topk,
                 window_groups=args.window_groups, window_pods=args.window_pods, fit_path_mask=args.fit_path_mask,
                 greedy_flags=args.greedy_flags, resort_nodes=args.resort_nodes)
    eng.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    b, e = eng.shard_range()
    Ns = e - b
    req, need = synth.make_fit_jobs(J, synth.SEED["cfg5"])
    eng.jobs_upload(req, need)
    stream = eng.stream()
    ev = HipEvents()

    for _ in range(args.warmup):
        eng.fit_mask_run()
    eng.synchronize()
    feasible = allsum(int(eng.fit_counts().sum()))

    e0, e1 = ev.create(), ev.create()
    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    ev.record(e0, stream)
    for _ in range(args.steps):
        eng.fit_mask_run()
    ev.record(e1, stream)
    eng.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = allmax(t1 - t0)
    kern_ms = ev.elapsed_ms(e0, e1) / args.steps
    value = float(N) * J * args.steps / elapsed
    st0 = eng.stats()
    fit_path = (("planes-blocks" if args.fit_path_mask & 32 else "planes") if st0["fit_runs_planes"] else
                (("coded-therm" if st0["fit_runs_therm"] else "coded-swar") if st0["fit_runs_coded"] else
                 ("i32" if st0["fit_runs_i32"] else "i64")))
    alg = fit_bytes(Ns, J)
    achieved = alg / (kern_ms * 1e-3) / 1e9
    kname = KERNEL_OF_PATH[fit_path]
    traffic, tsrc = profiled_traffic(kname, Ns, J)
    valu_frac = None
    if fit_path == "coded-therm":   # 3 VALU per (job, 64 nodes): or, add_co, addc
        valu_frac = 3.0 * (-(-J // 64) * 64) * (Ns / 64.0) / (kern_ms * 1e-3) / VALU_ISSUE_CEILING
    else:                           # PMC SQ_INSTS_VALU per launch (committed profile, same workload)
        insts = profiled_counter(kname, Ns, J, "SQ_INSTS_VALU")
        if insts is not None:
            valu_frac = insts / (kern_ms * 1e-3) / VALU_ISSUE_CEILING

    out = {
        "metric": METRIC, "value": value, "unit": "job*node fit evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": "int64", "data": "synthetic (splitmix64, SURVEY.md 8d)",
        "config": {"workload": f"cfg5: fit bitmask, {_count(N)}-node inventory x {_count(args.fit_jobs)} jobs"
                               f"{' per GPU' if args.scaling == 'weak' else ''} ({J} jobs in all), device-resident",
                   "nodes": N, "jobs": J, "jobs_per_gpu": J // world if args.scaling == "weak" else J,
                   "shard_nodes": Ns,
                   "parallelism": f"node-shard x{world}" + (" (host exchange rehearsal)" if host_exchange and world > 1 else ""), "feasible_pairs": feasible},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": tsrc, "kernel_ms": kern_ms, "alg_bytes_per_launch": alg,
                     "fit_path": fit_path, "valu_issue_frac": valu_frac,
                     "note": "kernel_ms = hipEvent time on the engine stream / fit_mask_run (one count memset, "
                             "the node encode and the fit kernel) on this rank's shard; achieved = algorithmic "
                             "bytes (shard nodes x 36 + jobs x 44 + jobs x ceil(shard/64) x 8) / kernel_ms; the "
                             "fit kernel is bound by its mask stores (HBM write)"},
    }

    if not args.no_configs:
        # the same step on a batch with 400 distinct cpu requests (more than one plane set holds):
        # plane sets, all swept in one launch; informational, not the headline value
        mreq = req.copy()
        mreq[:, 0] = 250 * (1 + np.arange(J) % 400)
        eng.jobs_upload(mreq, need)
        eng.fit_mask_run()
        eng.synchronize()
        m0, m1 = ev.create(), ev.create()
        ev.record(m0, stream)
        for _ in range(args.steps):
            eng.fit_mask_run()
        ev.record(m1, stream)
        eng.synchronize()
        mms = ev.elapsed_ms(m0, m1) / args.steps
        out["fit_many_values"] = {"workload": "cfg5 batch with 400 distinct cpu requests (plane sets)",
                                  "kernel_ms": mms, "evals_per_s_this_rank": float(Ns) * J / (mms * 1e-3),
                                  "fit_path": "planes" if eng.stats()["fit_runs_planes"] > st0["fit_runs_planes"]
                                  else "fallback"}
        eng.jobs_upload(req, need)                  # back to the headline batch (counts for the CPU check)
        eng.fit_mask_run()
        eng.synchronize()

    if not args.no_greedy:
        batch = synth.make_jobs(args.greedy_jobs, synth.SEED["cfg3"], "mixed")
        eng.reset_residuals()
        eng.place_batch(batch)                      # warm-up pass (allocations, code paths)
        times = []
        placed = 0
        for _ in range(args.greedy_steps):
            eng.reset_residuals()
            eng.synchronize()
            barrier()
            g0 = time.perf_counter()
            pods, st = eng.place_batch(batch)
            barrier()
            times.append(allmax(time.perf_counter() - g0))
            placed = int((st == 0).sum())
        s = eng.stats()
        gt = float(np.median(times))
        out["greedy"] = {"workload": "cfg3 mix on the 1M-node inventory: 10k jobs (50% PyTorch, 25% MPI, 25% JAX)",
                         "jobs": args.greedy_jobs, "pods": batch.n_pods, "jobs_placed": placed,
                         "gang_placements_per_s": args.greedy_jobs / gt, "ms_per_batch": gt * 1e3,
                         "windows_per_batch": s["windows"] / (args.greedy_steps + 1),
                         "rescans_per_batch": s["rescans"] / (args.greedy_steps + 1),
                         "scan_evals_per_s": s["scan_evals"] / (args.greedy_steps + 1) * world / gt,
                         "device_wait_ms_per_batch": s["greedy_wait_ms"] / (args.greedy_steps + 1),
                         "host_resolve_ms_per_batch": s["greedy_host_ms"] / (args.greedy_steps + 1),
                         "naive_pod_x_node_evals_per_s": batch.n_pods * float(N) / gt}

    if not args.no_configs:
        # BASELINE.json configs 2-4 at their own sizes (greedy best-fit, all-or-nothing); every rank
        # holds its shard of each inventory and makes the same calls
        out["configs"] = {}
        for cfg, mix, n_nodes, n_jobs, gpu_frac, what in (
                ("cfg2", "pytorch", 10_000, 1_000, 0.2, "10k nodes x 1k PyTorchJobs (Master 1 + Worker 0-15)"),
                ("cfg3", "mixed", 100_000, 10_000, 0.2, "100k nodes x 10k jobs, 50% PyTorch / 25% MPI / 25% JAX"),
                ("cfg4", "gang8", 100_000, 10_000, 1.0,
                 "100k 8-GPU nodes x 10k gangs of 1-16 pods x 8 GPUs, label-constrained, all-or-nothing")):
            cinv = synth.make_inventory(n_nodes, synth.SEED[cfg], gpu_frac)
            cb = synth.make_jobs(n_jobs, synth.SEED[cfg], mix)
            ce = Engine(device, rank=rank, world_size=world, comm=new_comm(), exchange=exchange, max_nodes=n_nodes,
                        topk=args.topk, window_groups=args.window_groups, window_pods=args.window_pods,
                        greedy_flags=args.greedy_flags, resort_nodes=args.resort_nodes)
            ce.load_nodes(cinv.cap, cinv.used, cinv.labels, cinv.island)
            ce.place_batch(cb)                       # warm-up
            ts = []
            for _ in range(3):
                ce.reset_residuals()
                ce.synchronize()
                barrier()
                g0 = time.perf_counter()
                _, cst = ce.place_batch(cb)
                barrier()
                ts.append(allmax(time.perf_counter() - g0))
            ct = float(np.median(ts))
            cs = ce.stats()
            out["configs"][cfg] = {"workload": what, "nodes": n_nodes, "jobs": n_jobs, "pods": cb.n_pods,
                                   "jobs_placed": int((cst == 0).sum()), "gang_placements_per_s": n_jobs / ct,
                                   "ms_per_batch": ct * 1e3, "windows_per_batch": cs["windows"] / 4.0,
                                   "rescans_per_batch": cs["rescans"] / 4.0}
            ce.close()

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        nthreads = max(1, min(16, os.cpu_count() or 1))
        js = min(args.cpu_sample_jobs, J)
        res = inv.residual()
        oracle.fit_mask(res, inv.labels, req[:16], need[:16], want_mask=False, nthreads=nthreads)  # warm-up
        reps = []
        for _ in range(3):
            c0 = time.perf_counter()
            _, ocounts = oracle.fit_mask(res, inv.labels, req[:js], need[:js], want_mask=True, nthreads=nthreads)
            reps.append(time.perf_counter() - c0)
        ct = float(np.median(reps))
        gpu_counts = eng.fit_counts()[:js] if world == 1 else None
        out["cpu_baseline"] = {"value": js * float(N) / ct, "unit": "job*node fit evals/s", "cores": nthreads,
                               "kind": "port", "sample": f"C oracle (oracle/oracle.c, OpenMP x{nthreads}, "
                               f"{cpu_model()}) on the first {js} jobs x all {N} nodes, median of 3; "
                               "the Go reference cannot be timed (no Go toolchain, SURVEY.md 0.3)",
                               "counts_match_gpu": bool(np.array_equal(ocounts, gpu_counts))}
        if "greedy" in out:
            gb = synth.make_jobs(40, synth.SEED["cfg3"], "mixed")
            c0 = time.perf_counter()
            oracle.place_greedy(res, inv.labels, gb.job_group_off, gb.priority, gb.group_count, gb.group_req,
                                gb.group_need, nthreads=nthreads)
            ct = time.perf_counter() - c0
            out["cpu_baseline"]["greedy"] = {"gang_placements_per_s": 40 / ct, "cores": nthreads,
                                             "sample": "naive per-pod argmin oracle, first 40 jobs of the batch"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
