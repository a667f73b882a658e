#!/usr/bin/env python3
"""Benchmark of the gang-placement hot path (BASELINE.json metric).

A "step" = one fit-mask pass (config 5): every job of the 100k-job batch evaluated against every
node of the 1M-node inventory, mask + per-job counts written to HBM, inputs already resident.  The
inventory is node-sharded over the ranks (north_star) and the batch is FIXED (strong scaling, the
BASELINE cfg5 "1M nodes x 100k jobs at 1/2/4/8 GPUs"): every rank evaluates the whole batch against
its 1M/N-node shard with no collective on the data path.  `value` = job x node fit evaluations per
second for the whole job (all ranks).  A weak-scaling line (batch 100k x N) is reported beside it
at N > 1.  The second half of the metric, gang placements/s, is measured on the same 1M-node
inventory with a 10k-job mixed PyTorch/MPI/JAX batch (config 3 mix) and reported in "greedy".

    python bench.py [--gpus N --steps K --warmup W]

With --gpus N > 1 and no WORLD_SIZE in the environment this process starts the N ranks itself
(torch.distributed.run, 127.0.0.1) and exits with their status; it never loads the engine or
touches a GPU.  Under torchrun (WORLD_SIZE set) --gpus must equal WORLD_SIZE.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PROFILES = os.path.join(ROOT, "profiles")

METRIC = "job×node fit evals/sec + gang placements/sec, 1M-node inventory, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# chip-wide integer VALU issue ceiling, wave-instructions/s: profiles/r1_ubench_valu.txt
# (v_add_u32 / v_addc_co at 8 waves per SIMD: 4.24 cycles per wave-instruction per SIMD, 256 CUs x 4 SIMDs)
VALU_ISSUE_CEILING = 5.79e11
# a committed profile's step time may differ from this run's by this fraction and still count as the
# same kernel (identical sources and workload are checked separately).  Kept tight on purpose: boxes
# and mask allocations move the fit step by up to ~9 % (2.16-2.36 ms, profiles/r8_fit_waves.txt), and
# a run outside 5 % reports traffic null rather than borrow counters from a different-speed run; the
# delta is printed beside the borrowed counters (profile_step_delta)
PROFILE_TOL = 0.05
# per fit path: the kernels of one fit step (the first is the dominant one, the roofline's kernel)
STEP_KERNELS = {
    "planes": ("pe::fit_mask_planes_rows_kernel", "pe::encode_planes_kernel"),
    "planes-sets": ("pe::fit_mask_planes_sets_kernel", "pe::encode_planes_sets_kernel"),
    "planes-blocks": ("pe::fit_mask_planes_kernel", "pe::encode_planes_kernel"),
    "lds": ("pe::fit_mask_lds_kernel", "pe::node_ranks_kernel"),
    "coded-therm": ("pe::fit_mask_coded_kernel", "pe::encode_nodes_kernel"),
    "coded-swar": ("pe::fit_mask_coded_kernel", "pe::encode_nodes_kernel"),
    "i32": ("pe::fit_mask_kernel", "pe::compress_res_kernel"),
    "i64": ("pe::fit_mask_kernel",),
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--fit-jobs", type=int, default=100_000)
    ap.add_argument("--greedy-jobs", type=int, default=10_000)
    ap.add_argument("--greedy-steps", type=int, default=5)
    ap.add_argument("--topk", type=int, default=0)
    ap.add_argument("--window-groups", type=int, default=0)
    ap.add_argument("--window-pods", type=int, default=0)
    ap.add_argument("--no-greedy", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the cfg2-4 greedy lines and the extra fit lines")
    ap.add_argument("--cpu-sample-jobs", type=int, default=20000)
    ap.add_argument("--cpu-greedy-jobs", type=int, default=1000)
    ap.add_argument("--agg-jobs", type=int, default=1_000_000)
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="strong (default): the 100k-job batch is fixed, the nodes are sharded; "
                         "weak: batch = fit-jobs x n_gpus (fixed per-rank work)")
    ap.add_argument("--fit-path-mask", type=int, default=0, help="pe_config.fit_path_mask (0 = every kernel)")
    ap.add_argument("--greedy-flags", type=int, default=0,
                    help="pe_config.greedy_flags (bit0: sequential windows, bit1: full scan instead of the sorted walk)")
    ap.add_argument("--resort-nodes", type=int, default=0, help="pe_config.resort_nodes (0 = default)")
    ap.add_argument("--no-walk-passes", action="store_true",
                    help="skip the greedy roofline's hipEvent passes (warm and cold); used by the profile passes")
    return ap.parse_args(argv)


def progress(msg: str):
    """One line on stderr per bench stage (a long GPU run stays visibly alive)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(args, argv):
    """The torchrun command line of the N-rank run (one rank per GPU, 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)


def maybe_launch(args, argv, run=subprocess.call):
    """Parent side of `--gpus N` without torchrun: start the N ranks as a child process and return
    its exit status; None when this process is a rank itself (or N == 1).  Imports nothing that
    loads the engine or initialises a GPU."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    return run(launch_cmd(args, argv))


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


def agg_bytes(job_group_off, group_cont_off) -> int:
    """SURVEY.md 8(d) aggregation bytes: per job G*(4 + 32 + 1) + 32 + 4 + 1 + 1, with the
    container records (32 + 1 B each) counted as they are read.  Of these, 38 B per job are outputs
    (res 32 + members 4 + present 1 + overflow 1), the rest inputs."""
    J = len(job_group_off) - 1
    G = int(job_group_off[-1])
    C = int(group_cont_off[-1])
    return G * (4 + 4) + C * (32 + 1) + J * (4 + 4 + 32 + 1 + 4 + 1)


def pg_slice(agg, a: int, b: int):
    """Jobs [a, b) of a pe_pg_min_resources CSR batch (job_group_off, min_member, group_replicas,
    group_cont_off, cont_req, cont_flags), offsets rebased."""
    jgo, mm, rep, gco, cont, flags = agg
    g0, g1 = int(jgo[a]), int(jgo[b])
    c0, c1 = int(gco[g0]), int(gco[g1])
    return (jgo[a:b + 1] - g0, mm[a:b], rep[g0:g1], gco[g0:g1 + 1] - c0, cont[c0:c1], flags[c0:c1])


AGG_LATENCY_JOBS = (1, 16, 256)
AGG_CROSSOVER_JOBS = (1, 16, 256, 512, 1024, 1536, 2048, 3072, 4096, 6144, 8192, 16384)


def agg_raw_call(fn, head, mode, sub):
    """A zero-argument closure calling a pe_pg_min_resources-shaped C function on the CSR batch `sub`
    (pg_slice output) with the ctypes pointers built once: what is timed per call is the C call
    (plus the ctypes dispatch, reported separately as ctypes_call_us), not numpy conversions.
    Returns (call, outputs)."""
    import numpy as np
    jgo, mm, rep, gco, cont, flags = [np.ascontiguousarray(a) for a in sub]
    J = len(jgo) - 1
    outs = (np.zeros((J, 4), np.int64), np.zeros(J, np.uint8), np.zeros(J, np.int32), np.zeros(J, np.uint8))
    keep = (jgo, mm, rep, gco, cont, flags) + outs
    ptrs = [a.ctypes.data_as(ctypes.c_void_p) for a in keep]
    args = tuple(head) + (mode, J, *ptrs)

    def call():
        return fn(*args)
    call.keep = keep
    return call, outs


def pcie_rates():
    """Pinned H2D / D2H rates of 128 MB copies on this box (torch pinned tensors), GB/s."""
    try:
        import torch
        if not torch.cuda.is_available():
            return None
        h = torch.empty(128 << 20, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(128 << 20, dtype=torch.uint8, device="cuda")
        rates = {}
        for name, dst, src in (("h2d_gbs", d, h), ("d2h_gbs", h, d)):
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                dst.copy_(src, non_blocking=True)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            rates[name] = (128 << 20) / sorted(ts)[2] / 1e9
        del h, d
        return rates
    except Exception:   # noqa: BLE001 -- a reported figure, never a reason to fail the bench
        return None


def time_calls(call, reps: int, warm: int = 20):
    """Median and p90 wall time of one call, microseconds."""
    for _ in range(warm):
        call()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter_ns()
        call()
        ts.append(time.perf_counter_ns() - t0)
    ts.sort()
    return ts[len(ts) // 2] / 1e3, ts[int(len(ts) * 0.9)] / 1e3


def profile_summaries():
    """The committed profiles profiles/LATEST names, one tag per line -- [(tag, summary.json)].  Several
    tags are profiles of the same sources taken on different boxes (their HBM rates differ by up to
    ~10 %): the fit check below takes the one whose step time is closest to this run's."""
    out = []
    try:
        tags = [t.strip() for t in open(os.path.join(PROFILES, "LATEST")).read().split() if t.strip()]
    except OSError:
        return out
    for tag in tags:
        try:
            out.append((tag, json.load(open(os.path.join(PROFILES, tag, "summary.json")))))
        except (OSError, ValueError):
            pass
    return out


def profile_summary(src_hash: str | None = None):
    """The first committed profile (of these sources, when src_hash is given), or (None, None)."""
    for tag, summ in profile_summaries():
        if src_hash is None or summ.get("source_hash") == src_hash:
            return tag, summ
    return None, None


def profile_check(path: str, n_nodes: int, n_jobs: int, kern_ms: float, src_hash: str):
    """Compare the committed profile with this run: same engine sources, same workload, and a fit
    step (sum of the step kernels' average durations) within PROFILE_TOL of this run's hipEvent time
    (the same kernel measures 2.16-2.36 ms across boxes and mask allocations, profiles/r8_fit_waves.txt;
    the traffic is a property of the code and the workload, which the hash and workload checks pin).
    Returns the roofline fields taken from it (traffic and counters are null unless all hold).  Among
    several committed profiles of these sources (LATEST), the one whose step is closest to this run's."""
    names = STEP_KERNELS[path]

    def step_ms(summ):
        k = summ.get("kernels", {})
        return sum(k[n]["avg_ns"] for n in names if n in k) / 1e6 if names[0] in k else None

    cands = profile_summaries()
    same_src = [(t, sm) for t, sm in cands if sm.get("source_hash") == src_hash and step_ms(sm) is not None]
    pool = same_src or cands[:1]
    tag, summ = min(pool, key=lambda c: abs((step_ms(c[1]) or 0.0) - kern_ms)) if pool else (None, None)
    out = {"profile": None, "profile_kernel_ms": None, "profile_step_ms": None, "profile_matches": False,
           "traffic": None, "traffic_source": None, "pmc": {}}
    if summ is None:
        return out
    out["profile"] = f"profiles/{tag}/summary.json"
    # every candidate of these sources with its step, so a reader sees which one matched and the spread
    # the choice was made from (advice r5: the best of N is an easier match than one profile)
    out["profile_candidates"] = [{"profile": f"profiles/{t}/summary.json", "step_ms": step_ms(sm)} for t, sm in pool]
    steps = [c["step_ms"] for c in out["profile_candidates"] if c["step_ms"]]
    out["profile_candidates_spread"] = (max(steps) / min(steps) - 1.0) if len(steps) > 1 else 0.0
    kernels = summ.get("kernels", {})
    if names[0] not in kernels:
        return out
    out["profile_kernel_ms"] = kernels[names[0]]["avg_ns"] / 1e6
    out["profile_step_ms"] = sum(kernels[k]["avg_ns"] for k in names if k in kernels) / 1e6
    out["profile_step_delta"] = out["profile_step_ms"] / kern_ms - 1.0
    wl = summ.get("workload", {})
    same = (summ.get("source_hash") == src_hash and wl.get("nodes") == n_nodes and wl.get("jobs") == n_jobs
            and abs(out["profile_step_ms"] - kern_ms) <= PROFILE_TOL * kern_ms)
    out["profile_matches"] = bool(same)
    if same:
        p = summ.get("pmc", {}).get(names[0], {})
        out["pmc"] = p
        if "hbm_traffic_bytes" in p:
            out["traffic"] = p["hbm_traffic_bytes"]
            out["traffic_source"] = (f"profiles/{tag}/summary.json (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE, "
                                     f"per launch of {names[0]})")
    return out


AGG_PROFILE_CALLS = 7   # tools/agg_calls.py: 1M-job calls in the profile's aggregation pass


def agg_profile_ms(src_hash: str):
    """Kernel time of one 1M-job pe_pg_min_resources call (the sum of its chunk launches of
    pg_agg_seg_kernel) in the committed profile's aggregation pass (tools/agg_calls.py), when taken
    on the same engine sources; else None."""
    _, summ = profile_summary(src_hash)
    if summ is None:
        return None
    k = summ.get("aggregation", {}).get("pe::pg_agg_seg_kernel")
    return k["total_ns"] / AGG_PROFILE_CALLS / 1e6 if k else None


def agg_roofline(in_bytes: int, out_bytes: int, call_ms: float, events_ms: float, profile_ms, pcie, wire_bytes=None):
    """Roofline of the 1M-job aggregation call.  The batch crosses PCIe: the packed input host to device
    (a DMA per chunk, pe_engine.cpp) while the kernels write the outputs into pinned memory device to
    host -- the two directions of a full-duplex link, each at the box's measured pinned rate.  The bound
    is the slower direction's time, max(in / h2d, out / d2h) (the input, 3x the output); frac = that
    bound / the whole call's wall time (planning, packing, DMA, kernels, copy-out: what the caller
    waits for).  full_duplex_frac prices (in + out) against h2d + d2h together -- out of reach by
    construction (<= 0.65 here: the output direction idles 3/4 of the time).  wire_bytes: the packed
    segments that actually crossed (requests narrowed to 32 bits above a per-key shift where that is
    exact), priced as wire_frac = (wire_bytes / h2d) / call_ms -- the link's busy share; the bound and
    frac above stay priced on the caller's arrays, so frac can pass 1 when the wire carries less."""
    bound = max(in_bytes / pcie["h2d_gbs"], out_bytes / pcie["d2h_gbs"]) / 1e6 if pcie else None
    ach = in_bytes / (call_ms * 1e-3) / 1e9
    return {"bound": "pcie (host to device: the packed batch)", "kernel": "pe::pg_agg_seg_kernel",
            "call_ms": call_ms, "bound_ms": bound, "events_call_ms": events_ms, "profile_kernel_ms": profile_ms,
            "in_bytes": in_bytes, "out_bytes": out_bytes, "achieved": ach, "unit": "GB/s",
            "peak": pcie["h2d_gbs"] if pcie else None, "frac": bound / call_ms if bound else None,
            "full_duplex_frac": (in_bytes + out_bytes) / (call_ms * 1e-3) / 1e9 / (pcie["h2d_gbs"] + pcie["d2h_gbs"])
            if pcie else None,
            "hbm_frac": (in_bytes + out_bytes) / (call_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "wire_bytes": wire_bytes,
            "wire_frac": wire_bytes / pcie["h2d_gbs"] / 1e6 / call_ms if pcie and wire_bytes else None}


def greedy_profile(src_hash: str):
    """Average walk_kernel durations (ns) of the committed profile's greedy passes (warm; cold =
    PE_WALK_FLUSH), only when taken on the same engine sources; {} otherwise."""
    tag, summ = profile_summary(src_hash)
    if summ is None or "greedy" not in summ:
        return {}
    g = summ["greedy"]
    out = {"profile": f"profiles/{tag}/summary.json"}
    for mode in ("warm", "cold"):
        k = g.get(mode, {}).get("pe::walk_kernel")
        if k:
            out[mode] = k["avg_ns"]
    p = g.get("pmc", {}).get("pe::walk_kernel", {})
    if "hbm_traffic_bytes" in p:   # per walk launch (FETCH_SIZE x 2 per the gfx950 note + WRITE_SIZE)
        out["traffic_per_launch"] = p["hbm_traffic_bytes"]
        out["read_per_launch"] = p["hbm_read_bytes_corrected"]
        out["write_per_launch"] = p["hbm_write_bytes"]
    return out


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


def cpu_share() -> int:
    """Host threads this process may use: the box's stated CPU share (OMP_NUM_THREADS, 16 per GPU
    on the GPU pool), else the affinity mask.  os.cpu_count() shows the whole machine there."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def fit_path_of(stats: dict, before: dict, blocks: bool) -> str:
    d = {k: stats[k] - before.get(k, 0) for k in stats if isinstance(stats[k], int)}
    if d.get("fit_runs_lds", 0):
        return "lds"
    if d.get("fit_runs_planes", 0):
        return "planes-blocks" if blocks else ("planes-sets" if d.get("fit_runs_sets", 0) else "planes")
    if d.get("fit_runs_coded", 0):
        return "coded-therm" if d.get("fit_runs_therm", 0) else "coded-swar"
    return "i32" if d.get("fit_runs_i32", 0) else "i64"


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    rc = maybe_launch(args, argv)
    if rc is not None:
        sys.exit(rc)

    sys.path[:0] = [p for p in (ROOT, os.path.join(ROOT, "training-operator_amd"), PROFILES) if p not in sys.path]
    import numpy as np

    from placement import Engine, HostExchange, PlacementError, comm_id, synth
    from provenance import source_hash

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    dist = None
    cid, exchange, device = None, None, local
    # PE_BENCH_EXCHANGE: "rccl" (default), "host" (rehearsal on one node, e.g. a 1-GPU box: the native
    # shared-memory all-gather pe_host_exchange), "gloo" (rehearsal through a Python gloo callback)
    xmode = os.environ.get("PE_BENCH_EXCHANGE", "rccl")
    host_exchange = xmode in ("host", "gloo")
    if world > 1:
        import torch
        import torch.distributed as dist
        if host_exchange:
            # rehearsal mode for a 1-GPU box: every rank on one device (RCCL cannot put two ranks on
            # one GPU), candidate blobs exchanged through host memory instead of RCCL (the driver's
            # multi-GPU runs use the RCCL default)
            dist.init_process_group("gloo")
            device = int(os.environ.get("PE_BENCH_DEVICE", "0"))
            tdev = "cpu"

            if xmode == "gloo":
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

        # a gloo group beside the RCCL one: the fallback exchange and the fallback vote must not
        # depend on the transport whose set-up failed
        gloo = dist.new_group(backend="gloo")

        hx = []

        def shm_exchange():
            """One pe_host_exchange per process (the ranks of this node; shared by every engine of the
            bench, which all make their calls in the same order on every rank)."""
            if not hx:
                names = [f"/pe_bench_{os.getpid()}_{time.time_ns() & 0xFFFFFFFF:x}" if rank == 0 else None]
                dist.broadcast_object_list(names, src=0, group=gloo)
                wg = args.window_groups or 112
                k = args.topk or 256
                k = max(k, min(2 * k, 1023))   # slots for the lists grown after a rescan (pe_engine.cpp)
                hx.append(HostExchange(names[0], rank, world, wg * (16 + 8 * k)))
                dist.barrier(group=gloo)
            return hx[0]

        hb = []

        def tight_barrier():
            """A barrier whose ranks leave within microseconds: a one-byte all-gather over a shared-memory
            segment of its own (pe_host_exchange spins; gloo's barrier lets ranks leave up to ~0.5 ms
            apart, which a 1-2 ms greedy batch would time as exchange waits)."""
            if not hb:
                names = [f"/pe_bench_b{os.getpid()}_{time.time_ns() & 0xFFFFFFFF:x}" if rank == 0 else None]
                dist.broadcast_object_list(names, src=0, group=gloo)
                hb.append(HostExchange(names[0], rank, world, 8))
                dist.barrier(group=gloo)
            hb[0].allgather(b"\0")

        def first_error(err):
            """Every rank's set-up error (None = fine) -> the first one, on every rank."""
            errs = [None] * world
            dist.all_gather_object(errs, err, group=gloo)
            return next((e for e in errs if e is not None), None)

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

        def allgather(x):
            parts = [None] * world
            dist.all_gather_object(parts, x)
            return parts
    else:
        def new_comm():
            return None

        def shm_exchange():
            return None

        def barrier():
            pass

        def first_error(err):
            return err

        def tight_barrier():
            pass

        def allmax(x):
            return x

        def allsum(x):
            return x

        def allgather(x):
            return [x]

    fallbacks = []
    if world > 1 and xmode == "host":
        exchange = shm_exchange()

    def make_engine(**kw):
        """An engine on this rank's GPU with a fresh RCCL communicator (world > 1).  If the RCCL set-up
        fails on any rank (pe_create returns PE_ERCCL within PE_RCCL_INIT_TIMEOUT_S), every rank builds
        its engine with the node's shared-memory all-gather instead (pe_host_exchange: the same
        sharded, pipelined and per-group signalled greedy with another transport); the JSON line says
        so at its top level ("degraded") and in config.greedy_exchange."""
        err = None
        try:
            if world > 1 and rank == world - 1 and os.environ.get("PE_BENCH_SIMULATE_RCCL_FAIL"):   # (test hook)
                new_comm()
                raise RuntimeError("simulated RCCL set-up failure (PE_BENCH_SIMULATE_RCCL_FAIL)")
            e = Engine(device, rank=rank, world_size=world, comm=new_comm(), exchange=exchange, **kw)
        except Exception as ex:   # noqa: BLE001 -- any set-up failure takes the fallback
            e, err = None, f"rank {rank}: {type(ex).__name__}: {ex}"
        err = first_error(err)
        if err is None:
            return e
        if e is not None:
            e.close()
        fallbacks.append(err)
        return Engine(device, rank=rank, world_size=world, comm=None, exchange=shm_exchange(), **kw)

    PE_ERCCL = -5

    def exchange_cost(st):
        """The host exchange's cost per greedy window (engine counters, this rank): waiting for the
        ranks' lists and merging them on the host -- null on one GPU and on the RCCL transport."""
        if world == 1 or st["windows"] == 0 or st["xchg_wait_ms"] + st["xchg_merge_ms"] == 0:
            return None
        return {"wait": st["xchg_wait_ms"] / st["windows"] * 1e3, "merge": st["xchg_merge_ms"] / st["windows"] * 1e3}

    def place_timed(holder, batch, kw, node_inv):
        """One timed greedy batch (barrier + wall clock, max over ranks) on holder[0].  A window whose
        RCCL all-gather does not complete within PE_RCCL_TIMEOUT_S makes pe_place_greedy abort the
        communicator and return PE_ERCCL (its peers' windows time out the same way); the ranks then
        agree through gloo, rebuild the engine on the node's shared-memory exchange, reload the
        inventory and place the batch again -- flagged "degraded" like a failed set-up."""
        for attempt in range(2):
            barrier()
            tight_barrier()
            g0 = time.perf_counter()
            err, r = None, None
            try:
                r = holder[0].place_batch(batch)
            except PlacementError as ex:
                if world == 1 or ex.code != PE_ERCCL or attempt:
                    raise
                err = f"rank {rank}: PlacementError: {ex}"
            t = time.perf_counter() - g0
            err = first_error(err) if world > 1 else err
            if err is None:
                barrier()
                return r, allmax(t)
            holder[0].close()
            fallbacks.append(f"mid-batch: {err}")
            holder[0] = Engine(device, rank=rank, world_size=world, comm=None, exchange=shm_exchange(), **kw)
            holder[0].load_nodes(node_inv.cap, node_inv.used, node_inv.labels, node_inv.island)
        raise AssertionError("unreachable")

    # PE_BENCH_INTERLEAVE_ONE=1 (multi-rank rehearsals, tests/test_gpu_multirank.py): after every timed
    # sharded greedy batch, rank 0 places the same batch alone on an unsharded context of the whole
    # inventory while the other ranks wait at a barrier -- a 1-rank reference timed on the same box in
    # the same minutes (interleaved), so a 2-rank / 1-rank bound does not compare two bench launches
    interleave = world > 1 and os.environ.get("PE_BENCH_INTERLEAVE_ONE") == "1"

    def solo_engine(kw, node_inv, batch):
        if not interleave or rank != 0:
            return None
        se = Engine(device, **kw)
        se.load_nodes(node_inv.cap, node_inv.used, node_inv.labels, node_inv.island)
        se.place_batch(batch)   # warm-up
        return se

    def solo_timed(se, batch):
        """rank 0 alone on its unsharded context (the other ranks at the barrier): seconds, or None"""
        if not interleave:
            return None
        barrier()
        t = None
        if se is not None:
            se.reset_residuals()
            se.synchronize()
            g0 = time.perf_counter()
            se.place_batch(batch)
            t = time.perf_counter() - g0
        barrier()
        return t

    N = args.nodes
    J = args.fit_jobs * (world if args.scaling == "weak" else 1)
    inv = synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2)
    eng_kw = dict(max_nodes=N, topk=args.topk, window_groups=args.window_groups, window_pods=args.window_pods,
                  fit_path_mask=args.fit_path_mask, greedy_flags=args.greedy_flags, resort_nodes=args.resort_nodes)
    eng = make_engine(**eng_kw)
    eng.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    b, e = eng.shard_range()
    Ns = e - b
    req, need = synth.make_fit_jobs(J, synth.SEED["cfg5"])
    stream = eng.stream()
    ev = HipEvents()
    blocks = bool(args.fit_path_mask & 32)

    def time_fit(rq, nd, steps, warmup, label):
        """Upload a batch, warm up, time `steps` fit steps (barrier + sync on both sides, max over
        ranks).  Returns (wall seconds, hipEvent ms per step on this rank, fit path, feasible pairs)."""
        st0 = eng.stats()
        eng.jobs_upload(rq, nd)
        for _ in range(warmup):
            eng.fit_mask_run()
        eng.synchronize()
        feas = allsum(int(eng.fit_counts().sum()))
        e0, e1 = ev.create(), ev.create()
        barrier()
        eng.synchronize()
        t0 = time.perf_counter()
        ev.record(e0, stream)
        for _ in range(steps):
            eng.fit_mask_run()
        ev.record(e1, stream)
        eng.synchronize()
        t1 = time.perf_counter()      # this rank's K steps are done (the closing barrier is not timed)
        barrier()
        wall = allmax(t1 - t0)        # from the common start to the last rank's finish
        return wall, ev.elapsed_ms(e0, e1) / steps, fit_path_of(eng.stats(), st0, blocks), feas

    progress("fit headline")
    elapsed, kern_ms, fit_path, feasible = time_fit(req, need, args.steps, args.warmup, "headline")
    value = float(N) * J * args.steps / elapsed
    alg = fit_bytes(Ns, J)
    achieved = alg / (kern_ms * 1e-3) / 1e9
    kname = STEP_KERNELS[fit_path][0]
    src_hash = source_hash(ROOT)
    prof = profile_check(fit_path, Ns, J, kern_ms, src_hash)
    valu_frac = None
    if "SQ_INSTS_VALU" in prof["pmc"]:   # PMC SQ_INSTS_VALU per launch (committed profile, same build)
        valu_frac = prof["pmc"]["SQ_INSTS_VALU"] / (kern_ms * 1e-3) / VALU_ISSUE_CEILING
    shards = allgather(Ns)
    rccl = eng.comm_ranks()

    out = {
        "metric": METRIC, "value": value, "unit": "job*node fit evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": "int64", "data": "synthetic (splitmix64, SURVEY.md 8d)",
        "config": {"workload": f"cfg5: fit bitmask, {_count(N)}-node inventory x {_count(args.fit_jobs)} jobs"
                               f"{' per GPU' if args.scaling == 'weak' else ''} ({J} jobs in all), device-resident",
                   "nodes": N, "jobs": J, "jobs_per_gpu": J // world if args.scaling == "weak" else J,
                   "shard_nodes": Ns, "shard_nodes_per_rank": shards, "rccl_ranks": rccl,
                   "parallelism": f"node-shard x{world}" + (" (host exchange rehearsal)" if host_exchange and world > 1
                                                            else ""),
                   "feasible_pairs": feasible,
                   "greedy_exchange": ("none (one GPU)" if world == 1
                                       else f"host shared-memory exchange (zero-copy windows): RCCL set-up failed ({fallbacks[0]})"
                                       if fallbacks
                                       else "gloo host exchange (rehearsal)" if xmode == "gloo"
                                       else "host shared-memory exchange, zero-copy windows (rehearsal)" if host_exchange
                                       else "RCCL all-gather + device merge")},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": prof["traffic"],
                     "traffic_source": prof["traffic_source"], "kernel_ms": kern_ms,
                     "profile_kernel_ms": prof["profile_kernel_ms"], "profile_step_ms": prof["profile_step_ms"],
                     "profile": prof["profile"], "profile_matches": prof["profile_matches"],
                     "profile_step_delta": prof.get("profile_step_delta"),
                     "source_hash": src_hash, "alg_bytes_per_launch": alg, "fit_path": fit_path,
                     "valu_issue_frac": valu_frac,
                     "note": "kernel_ms = hipEvent time on the engine stream / fit step (count memset, node encode, fit "
                             "kernel) on this rank's shard; achieved = algorithmic bytes (shard nodes x 36 + jobs x 44 + "
                             "jobs x ceil(shard/64) x 8) / kernel_ms; traffic / valu_issue_frac come from the committed "
                             "profile only when it was taken on the same engine sources and workload and its step time "
                             f"agrees with kernel_ms within {PROFILE_TOL:.0%} (profile_matches; profile_step_delta = "
                             "profile step / this run's step - 1): those counters are the profile's, not this run's"},
    }

    if world > 1:
        # weak scaling beside the strong headline: batch 100k x N, every rank the whole batch
        Jw = args.fit_jobs * world
        wreq, wneed = synth.make_fit_jobs(Jw, synth.SEED["cfg5"])
        wt, wms, wpath, _ = time_fit(wreq, wneed, args.steps, 1, "weak")
        out["fit_weak_scaling"] = {"workload": f"cfg5 batch of {Jw} jobs (100k per GPU) x {_count(N)} nodes",
                                   "jobs": Jw, "value": float(N) * Jw * args.steps / wt,
                                   "ms_per_step": wt / args.steps * 1e3, "kernel_ms": wms, "fit_path": wpath}

    if not args.no_configs:
        # end-to-end fit batch: host planning + H2D (pe_jobs_upload) + fit step + counts D2H
        reps = []
        for _ in range(3):
            eng.synchronize()
            barrier()
            t0 = time.perf_counter()
            eng.jobs_upload(req, need)
            eng.fit_mask_run()
            eng.fit_counts()
            barrier()
            reps.append(allmax(time.perf_counter() - t0))
        t_up = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.jobs_upload(req, need)
            t_up.append(time.perf_counter() - t0)
        e2e = float(np.median(reps))
        out["fit_end_to_end"] = {"workload": "headline batch incl. pe_jobs_upload (host planning + H2D), the fit step "
                                             "and the per-job counts D2H", "ms_per_batch": e2e * 1e3,
                                 "upload_ms": float(np.median(t_up)) * 1e3,
                                 "evals_per_s": float(N) * J / e2e}
        # high-cardinality batches (not the headline): 400 distinct cpu values; unique memory per job
        # with 1000 cpu and 100 ephemeral values; unique cpu, memory and ephemeral per job
        mreq = req.copy()
        mreq[:, 0] = 250 * (1 + np.arange(J) % 400)
        cases = [("fit_many_values", "cfg5 batch with 400 distinct cpu requests", mreq, need)]
        wreq, wneed = synth.make_fit_jobs_worst(J, synth.SEED["cfg5"], (1,))
        cases.append(("fit_worst_case", "cfg5 batch, memory unique per job, cpu over 1000 and ephemeral over 100 "
                                        "values", wreq, wneed))
        areq, aneed = synth.make_fit_jobs_worst(J, synth.SEED["cfg5"], (0, 1, 3))
        cases.append(("fit_adversarial", "cfg5 batch, cpu, memory and ephemeral each unique per job", areq, aneed))
        for key, what, rq, nd in cases:
            progress(key)
            wt, wms, wpath, wfeas = time_fit(rq, nd, max(2, args.steps // 2), 1, key)
            pairs = {f"distinct_{n}": int(len(np.unique(rq[:, d]))) for d, n in enumerate(("cpu", "mem", "gpu", "eph"))}
            out[key] = {"workload": what, **pairs, "kernel_ms": wms, "ms_per_step": wt / max(2, args.steps // 2) * 1e3,
                        "vs_headline_step": wms / kern_ms, "fit_path": wpath, "kernel": STEP_KERNELS[wpath][0],
                        "frac": fit_bytes(Ns, J) / (wms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "evals_per_s": float(N) * J / wt * max(2, args.steps // 2), "feasible_pairs": wfeas}
        eng.jobs_upload(req, need)                  # back to the headline batch (counts for the CPU check)
        eng.fit_mask_run()
        eng.synchronize()

        # PodGroup MinResources aggregation (v1 CalcPGMinResources).  The operator calls it once per job
        # per reconcile (job.go:275-277,455-457; coscheduling.go:103-118), so the per-call latency at
        # J = 1 / 16 / 256 is the figure that decides whether the drop-in beats the code it replaces;
        # the 1M-job batch is the throughput line.  Jobs are independent: at N > 1 every rank
        # aggregates its contiguous slice of the batch.
        progress("aggregation")
        agg = synth.make_pg_batch(args.agg_jobs, synth.SEED["cfg3"])
        lat = {}
        call0 = eng.lib.pe_abi_version
        ctypes_us = time_calls(call0, 2000)[0]
        for Jn in AGG_LATENCY_JOBS:
            sub = pg_slice(agg, 0, Jn)
            call, outs = agg_raw_call(eng.lib.pe_pg_min_resources, (eng.h,), 1, sub)
            assert call() in (0, -2)
            med, p90 = time_calls(call, 400)
            os.environ["PE_AGG_DEVICE"] = "1"     # the r2 call path (six H2D + four D2H copies), same box
            try:
                dmed, _ = time_calls(call, 200)
            finally:
                del os.environ["PE_AGG_DEVICE"]
            lat[str(Jn)] = {"median_us": med, "p90_us": p90, "r2_path_median_us": dmed,
                            "alg_bytes": agg_bytes(sub[0], sub[3])}
        lo_j, hi_j = rank * args.agg_jobs // world, (rank + 1) * args.agg_jobs // world
        mine = pg_slice(agg, lo_j, hi_j)
        # the C call with caller-owned outputs allocated once (the ABI's contract, like the latency
        # lines); the Python wrapper, which allocates fresh zeroed outputs per call (38 B per job of
        # first-touch page faults), is timed beside it as wrapper_ms_per_call
        mcall, _ = agg_raw_call(eng.lib.pe_pg_min_resources, (eng.h,), 1, mine)
        assert mcall() in (0, -2)
        e0, e1 = ev.create(), ev.create()
        ts, ks = [], []
        st0 = eng.stats()
        for _ in range(5):
            barrier()
            t0 = time.perf_counter()
            ev.record(e0, stream)
            mcall()
            ev.record(e1, stream)
            ts.append(allmax(time.perf_counter() - t0))
            ks.append(ev.elapsed_ms(e0, e1))
        st1 = eng.stats()
        # the packed segments that crossed per call (requests narrowed where exact: pe_kernels.h agg_seg_layout)
        wire = {k: (st1[k] - st0[k]) / 5 for k in ("agg_wire_bytes", "agg_segments", "agg_narrow_segments")}
        at = float(np.median(ts))
        kms = float(np.median(ks))
        wts = []
        for _ in range(3):
            barrier()
            t0 = time.perf_counter()
            eng.pg_min_resources(1, *mine)
            wts.append(allmax(time.perf_counter() - t0))
        os.environ["PE_AGG_DEVICE"] = "1"
        try:
            dts = []
            for _ in range(3):
                barrier()
                t0 = time.perf_counter()
                mcall()
                dts.append(allmax(time.perf_counter() - t0))
        finally:
            del os.environ["PE_AGG_DEVICE"]
        ab = agg_bytes(agg[0], agg[3])
        mb = agg_bytes(mine[0], mine[3])
        pcie = pcie_rates()
        out["aggregation"] = {
            "workload": f"{args.agg_jobs} v1 PyTorchJob-like jobs (Master 1 + Worker 0-63, 1-2 containers), "
                        "CalcPGMinResources on the GPU, host arrays in and out (the C ABI's contract)"
                        + (f", split over {world} ranks ({hi_j - lo_j} jobs on rank {rank})" if world > 1 else ""),
            "jobs_per_s": args.agg_jobs / at, "ms_per_call": at * 1e3, "alg_bytes": ab,
            "achieved_gbs": ab / at / 1e9, "r2_path_ms_per_call": float(np.median(dts)) * 1e3,
            "wrapper_ms_per_call": float(np.median(wts)) * 1e3,
            "pcie": pcie,
            "pcie_bound_ms": (mb / pcie["h2d_gbs"] / 1e6) if pcie else None,
            "latency_us": lat, "ctypes_call_us": ctypes_us,
            "pcie_bound_duplex_ms": (max((mb - 38 * (hi_j - lo_j)) / pcie["h2d_gbs"], 38 * (hi_j - lo_j) / pcie["d2h_gbs"])
                                     / 1e6) if pcie else None,
            "roofline": agg_roofline(mb - 38 * (hi_j - lo_j), 38 * (hi_j - lo_j), at * 1e3, kms,
                                     agg_profile_ms(source_hash(ROOT)), pcie, wire["agg_wire_bytes"]),
            "wire_bytes_per_call": wire["agg_wire_bytes"], "segments_per_call": wire["agg_segments"],
            "narrowed_segments_per_call": wire["agg_narrow_segments"],
            "note": "latency_us: one pe_pg_min_resources call on the first J jobs (median / p90 of 400, ctypes pointers "
                    "built once; ctypes_call_us = the dispatch cost of an empty ABI call, included); r2_path = the "
                    "round-2 call path (PE_AGG_DEVICE=1: six H2D + four D2H copies + stream sync) on the same box; "
                    "ms_per_call = the C call on caller-owned input and output arrays (allocated once), max over ranks; "
                    "wrapper_ms_per_call = the Python wrapper, which allocates fresh zeroed outputs every call"}

    if not args.no_greedy:
        progress("greedy")
        batch = synth.make_jobs(args.greedy_jobs, synth.SEED["cfg3"], "mixed")
        holder = [eng]
        eng.reset_residuals()
        place_timed(holder, batch, eng_kw, inv)     # warm-up pass (allocations, code paths)
        eng = holder[0]
        solo = solo_engine(eng_kw, inv, batch)
        eng.reset_stats()
        times, solo_t = [], []
        placed = 0
        for _ in range(args.greedy_steps):
            eng.reset_residuals()
            eng.synchronize()
            (pods, st), t = place_timed(holder, batch, eng_kw, inv)
            if holder[0] is not eng:                # rebuilt mid-run: its stats start here
                eng = holder[0]
                times = []
            times.append(t)
            placed = int((st == 0).sum())
            t1 = solo_timed(solo, batch)
            if t1 is not None:
                solo_t.append(t1)
        if solo is not None:
            solo.close()
        s = eng.stats()
        gt = float(np.median(times))
        gs = args.greedy_steps
        out["greedy"] = {"workload": "cfg3 mix on the 1M-node inventory: 10k jobs (50% PyTorch, 25% MPI, 25% JAX)",
                         "jobs": args.greedy_jobs, "pods": batch.n_pods, "jobs_placed": placed,
                         "gang_placements_per_s": args.greedy_jobs / gt, "ms_per_batch": gt * 1e3,
                         "windows_per_batch": s["windows"] / gs, "rescans_per_batch": s["rescans"] / gs,
                         "device_wait_ms_per_batch": s["greedy_wait_ms"] / gs,
                         "host_resolve_ms_per_batch": s["greedy_host_ms"] / gs,
                         "zero_copy_exchange_windows_per_batch": s["xchg_zc_windows"] / gs,
                         "exchange_us_per_window": exchange_cost(s),
                         "naive_pod_x_node_evals_per_s": batch.n_pods * float(N) / gt}
        if solo_t:
            out["greedy"]["interleaved_one_rank_ms_per_batch"] = float(np.median(solo_t)) * 1e3
        if s["walk_groups"] > 0:
            # greedy roofline of the walk kernel.  Bytes it reads per batch (engine counters of the timed
            # batches): per group the round summaries (first key 8 B, max residual 32 B, label OR 4 B per
            # round), the overlay entries (state 32 + 4 B, id 4 B) and the visited sorted entries (key 8 B,
            # residuals 32 B, labels 4 B).  Time per batch = walk launches x the walk kernel's average
            # duration: from the committed rocprof profile of the same sources when there is one (warm
            # and cold passes, profiles/run_profile.sh), else from a live pass with hipEvents around every
            # launch (the events add host gaps and inflate it).  WARM = the batch as the bench runs it: the
            # ~50 MB walk index stays in the 256 MiB Infinity Cache; COLD = a 512 MiB buffer rewritten
            # before every walk launch (PE_WALK_FLUSH), so the walk reads come from HBM.
            walked = (s["walk_prepass"] * 44 + s["walk_overlay"] * 40 + s["walk_rounds"] * 1024 * 44) / gs
            launches = s["windows"] / gs
            ev_ms = {}
            if not args.no_walk_passes:
                for mode, env in (("warm", {"PE_WALK_EVENTS": "1"}), ("cold", {"PE_WALK_EVENTS": "1", "PE_WALK_FLUSH": "1"})):
                    eng.reset_residuals()
                    eng.reset_stats()
                    os.environ.update(env)
                    try:
                        eng.place_batch(batch)
                    finally:
                        for k in env:
                            del os.environ[k]
                    ev_ms[mode] = eng.stats()["walk_ms"]
            gprof = greedy_profile(source_hash(ROOT))
            roof = {"kernel": "pe::walk_kernel", "bytes_per_batch": walked, "walk_launches_per_batch": launches,
                    "rounds_per_group": s["walk_rounds"] / max(1, s["walk_groups"]),
                    "overlay_per_group": s["walk_overlay"] / max(1, s["walk_groups"]), "unit": "GB/s",
                    "profile": gprof.get("profile")}
            # The walk is LATENCY-bound (one block per group walks a few dependent rounds; the launch lasts
            # as long as its slowest block), not bandwidth-bound: "bound" says so, "achieved" is the
            # algorithmic read rate it reaches anyway, hbm_frac that rate against the HBM spec (no Infinity
            # Cache peak is claimed).  Per launch and per walked round: launch time / mean rounds per group
            # (the slow blocks that set a launch walk ~2x the mean; profiles/r17_walk_prof.txt has the
            # per-phase block times).
            for mode in ("warm", "cold"):
                avg_ns = gprof.get(mode)
                if avg_ns:
                    ms, src = avg_ns * launches / 1e6, f"rocprof average walk_kernel duration ({gprof['profile']}) x launches"
                elif mode in ev_ms:
                    ms, src = ev_ms[mode], "hipEvents around every walk launch (live pass; events inflate it)"
                else:
                    continue
                us_launch = ms * 1e3 / max(1.0, launches)
                roof[mode] = {"bound": "latency", "walk_ms_per_batch": ms, "time_source": src,
                              "us_per_launch": us_launch,
                              "us_per_launch_per_mean_round": us_launch / max(1e-9, roof["rounds_per_group"]),
                              "achieved": walked / (ms * 1e-3) / 1e9, "peak": None,
                              "hbm_frac": walked / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                              "cache": "L2 + Infinity Cache resident index" if mode == "warm"
                                       else "index evicted before every launch (PE_WALK_FLUSH): reads from HBM"}
                if mode in ev_ms:
                    roof[mode]["events_walk_ms_per_batch"] = ev_ms[mode]
            if "traffic_per_launch" in gprof:
                # counted HBM-side traffic (L2 misses + writes) of the walk, per batch = per launch x launches,
                # from the profile's greedy PMC passes; traffic_ratio = counted / algorithmic bytes
                roof["traffic"] = gprof["traffic_per_launch"] * launches
                roof["traffic_read"] = gprof["read_per_launch"] * launches
                roof["traffic_write"] = gprof["write_per_launch"] * launches
                roof["traffic_ratio"] = roof["traffic"] / walked if walked else None
                # share of the walk's algorithmic reads served by the caches (L2 / Infinity Cache): 1 - the
                # HBM-side reads (FETCH_SIZE, gfx950-corrected) over the algorithmic read bytes
                roof["cache_hit_share"] = 1.0 - roof["traffic_read"] / walked if walked else None
                roof["traffic_source"] = f"{gprof['profile']} greedy PMC passes (FETCH_SIZE x2 + WRITE_SIZE per walk launch)"
            else:
                roof["traffic"] = None
            roof["note"] = ("latency-bound, not bandwidth-bound: one 1024-thread block per group walks a few rounds of "
                            "1024 sorted nodes (dependent steps: loads, key, append, barrier, stop test) and the launch "
                            "lasts as long as its slowest group; cache_hit_share = the reads the caches served")
            out["greedy"]["roofline"] = roof

    if not args.no_configs:
        # BASELINE.json configs 2-4 at their own sizes (greedy best-fit, all-or-nothing); every rank
        # holds its shard of each inventory and makes the same calls
        out["configs"] = {}
        for cfg, mix, n_nodes, n_jobs, gpu_frac, what in (
                ("cfg2", "pytorch", 10_000, 1_000, 0.2, "10k nodes x 1k PyTorchJobs (Master 1 + Worker 0-15)"),
                ("cfg3", "mixed", 100_000, 10_000, 0.2, "100k nodes x 10k jobs, 50% PyTorch / 25% MPI / 25% JAX"),
                ("cfg4", "island8", 100_000, 10_000, 1.0,
                 "100k 8-GPU nodes x 10k 8-GPU gang jobs on single-node xGMI islands (island groups of 1-8 pods "
                 "x 8/M GPUs co-located on one node; 1/4 multi-node gangs of 2-4 whole-node pods), all-or-nothing"),
                ("cfg4_gang8", "gang8", 100_000, 10_000, 1.0,
                 "100k 8-GPU nodes x 10k gangs of 1-16 whole-node pods x 8 GPUs, label-constrained, all-or-nothing")):
            progress(cfg)
            cinv = synth.make_inventory(n_nodes, synth.SEED[cfg[:4]], gpu_frac)
            cb = synth.make_jobs(n_jobs, synth.SEED[cfg[:4]], mix)
            ckw = dict(max_nodes=n_nodes, topk=args.topk, window_groups=args.window_groups,
                       window_pods=args.window_pods, greedy_flags=args.greedy_flags, resort_nodes=args.resort_nodes)
            ch = [make_engine(**ckw)]
            ch[0].load_nodes(cinv.cap, cinv.used, cinv.labels, cinv.island)
            place_timed(ch, cb, ckw, cinv)           # warm-up
            solo = solo_engine(ckw, cinv, cb)
            ce = ch[0]
            ce.reset_stats()
            ts, solo_t = [], []
            for _ in range(3):
                ce.reset_residuals()
                ce.synchronize()
                (_, cst), t = place_timed(ch, cb, ckw, cinv)
                if ch[0] is not ce:                  # rebuilt mid-run: its stats start here
                    ce = ch[0]
                    ts = []
                ts.append(t)
                t1 = solo_timed(solo, cb)
                if t1 is not None:
                    solo_t.append(t1)
            if solo is not None:
                solo.close()
            ct = float(np.median(ts))
            cs = ce.stats()
            out["configs"][cfg] = {"workload": what, "nodes": n_nodes, "jobs": n_jobs, "pods": cb.n_pods,
                                   "jobs_placed": int((cst == 0).sum()), "gang_placements_per_s": n_jobs / ct,
                                   "ms_per_batch": ct * 1e3, "windows_per_batch": cs["windows"] / 3.0,
                                   "rescans_per_batch": cs["rescans"] / 3.0,
                                   "host_resolve_ms_per_batch": cs["greedy_host_ms"] / 3.0,
                                   "device_wait_ms_per_batch": cs["greedy_wait_ms"] / 3.0,
                                   "zero_copy_exchange_windows_per_batch": cs["xchg_zc_windows"] / 3.0,
                                   "exchange_us_per_window": exchange_cost(cs)}
            if solo_t:
                out["configs"][cfg]["interleaved_one_rank_ms_per_batch"] = float(np.median(solo_t)) * 1e3
            ce.close()

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        import oracle
        from placement import Resolver
        nthreads = cpu_share()
        js = min(args.cpu_sample_jobs, J)
        res = inv.residual()
        oracle.fit_mask(res, inv.labels, req[:16], need[:16], want_mask=False, nthreads=nthreads)  # warm-up
        reps = []
        for _ in range(3):
            c0 = time.perf_counter()
            _, ocounts = oracle.fit_mask(res, inv.labels, req[:js], need[:js], want_mask=True, nthreads=nthreads)
            reps.append(time.perf_counter() - c0)
        ct = float(np.median(reps))
        c0 = time.perf_counter()
        oracle.fit_mask(res, inv.labels, req[:200], need[:200], want_mask=True, nthreads=1)
        c1 = time.perf_counter() - c0
        gpu_counts = eng.fit_counts()[:js]
        out["cpu_baseline"] = {"value": js * float(N) / ct, "unit": "job*node fit evals/s", "cores": nthreads,
                               "kind": "port", "sample": f"C oracle (oracle/oracle.c, OpenMP x{nthreads}, "
                               f"{cpu_model()}) on the first {js} jobs x all {N} nodes, mask written, median of 3; "
                               "the Go reference cannot be timed (no Go toolchain, SURVEY.md 0.3)",
                               "single_thread_value": 200 * float(N) / c1, "nproc": os.cpu_count(),
                               "affinity_cpus": len(os.sched_getaffinity(0)),
                               "threads_note": "threads = this box's CPU share (OMP_NUM_THREADS, else the affinity "
                                               "mask); nproc counts the whole machine, shared with other GPUs' jobs",
                               "counts_match_gpu": bool(np.array_equal(ocounts, gpu_counts))}
        if "aggregation" in out:
            # the same aggregation rule on the CPU (oracle.c orc_pg_min_resources, one thread, the same CSR
            # arrays), per call at the operator's sizes and on the whole batch; outputs checked equal to the GPU's
            ol = oracle.lib()
            clat = {}
            same = True
            for Jn in AGG_LATENCY_JOBS:
                sub = pg_slice(agg, 0, Jn)
                ccall, couts = agg_raw_call(ol.orc_pg_min_resources, (), 1, sub)
                gcall, gouts = agg_raw_call(eng.lib.pe_pg_min_resources, (eng.h,), 1, sub)
                ccall()
                gcall()
                same &= all(np.array_equal(a, b) for a, b in zip(couts, gouts))
                clat[str(Jn)] = {"median_us": time_calls(ccall, 400)[0]}
            ccall, couts = agg_raw_call(ol.orc_pg_min_resources, (), 1, agg)
            reps = []
            for _ in range(3):
                c0 = time.perf_counter()
                ccall()
                reps.append(time.perf_counter() - c0)
            gout = eng.pg_min_resources(1, *agg)
            same &= all(np.array_equal(a, b) for a, b in zip(couts, gout))
            # the crossover: the smallest batch (jobs per call) where one engine call beats the same
            # arithmetic on one CPU core, both timed here on the same CSR prefixes (outputs checked equal)
            sweep, crossover = [], None
            for Jn in AGG_CROSSOVER_JOBS:
                sub = pg_slice(agg, 0, Jn)
                ccall, couts = agg_raw_call(ol.orc_pg_min_resources, (), 1, sub)
                gcall, gouts = agg_raw_call(eng.lib.pe_pg_min_resources, (eng.h,), 1, sub)
                ccall()
                gcall()
                same &= all(np.array_equal(a, b) for a, b in zip(couts, gouts))
                n = 200 if Jn <= 2048 else 60
                g_us, c_us = time_calls(gcall, n)[0], time_calls(ccall, n)[0]
                sweep.append({"jobs": Jn, "gpu_us": g_us, "cpu_us": c_us})
                if crossover is None and g_us < c_us:
                    crossover = Jn
            if "aggregation" in out:
                out["aggregation"]["crossover_jobs"] = crossover
                out["aggregation"]["crossover_sweep"] = sweep
                out["aggregation"]["crossover_note"] = (
                    "smallest jobs-per-call of the sweep where pe_pg_min_resources (median of the C call) beats "
                    "cpu_baseline.aggregation's rule (oracle.c, one core) on the same jobs; below it the operator's "
                    "per-reconcile call (J = 1) is cheaper on its own CPU")
            out["cpu_baseline"]["aggregation"] = {
                "jobs_per_s": args.agg_jobs / float(np.median(reps)), "ms_per_call": float(np.median(reps)) * 1e3,
                "cores": 1, "kind": "port", "latency_us": clat, "outputs_match_gpu": bool(same),
                "sample": f"C oracle orc_pg_min_resources (oracle/oracle.c, single thread, {cpu_model()}) on the same "
                          f"CSR arrays: the first 1 / 16 / 256 jobs per call (median of 400) and all {args.agg_jobs} "
                          "jobs (median of 3); the Go reference (map + resource.Quantity per pod) cannot be timed here"}
        if "greedy" in out:
            # the same algorithm on the CPU: windowed protocol (K = 256, 128 groups / 1024 pods per window, the engine defaults),
            # each window's candidate lists built by the C oracle over all 1M nodes (OpenMP over groups),
            # resolved by the product's host resolver -- on the first jobs of the same batch
            gj = args.cpu_greedy_jobs
            full = synth.make_jobs(args.greedy_jobs, synth.SEED["cfg3"], "mixed")
            gb = synth.make_jobs(gj, synth.SEED["cfg3"], "mixed")
            c0 = time.perf_counter()
            _, gst, _, gw = oracle.place_greedy_windowed(Resolver, res, inv.labels, gb, K=256, nthreads=nthreads)
            ct = time.perf_counter() - c0
            c0 = time.perf_counter()
            oracle.place_greedy(res, inv.labels, gb.job_group_off[:41], gb.priority[:40], gb.group_count,
                                gb.group_req, gb.group_need, nthreads=nthreads)
            cn = time.perf_counter() - c0
            out["cpu_baseline"]["greedy"] = {
                "gang_placements_per_s": gj / ct, "cores": nthreads, "windows": gw,
                "sample": f"windowed protocol on the CPU (oracle window scan x{nthreads} threads + the host resolver), "
                          f"first {gj} jobs of the cfg3-mix batch ({full.n_jobs} in the GPU line) on the 1M-node "
                          "inventory", "jobs_placed": int((gst == 0).sum()),
                "naive_gang_placements_per_s": 40 / cn,
                "naive_sample": "naive per-pod argmin over all nodes (oracle.c orc_place_greedy), first 40 jobs"}
    if world > 1:
        # an RCCL set-up failure on any rank moved every engine to the host exchange: same results,
        # another transport -- said at the top level, not only in config.greedy_exchange
        out["degraded"] = bool(fallbacks)
        if fallbacks:
            out["degraded_reason"] = f"{len(fallbacks)} engine(s) without RCCL: {fallbacks[0]}"
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
