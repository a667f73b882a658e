"""Multi-rank readiness on one GPU (the 8-GPU scaling run must not be the first time the
multi-rank bench runs).

1. `bench.py --gpus 2` end to end: the bench parent (which never touches the GPU) starts two ranks
   through torch.distributed.run; both ranks share this box's one GPU and exchange the greedy
   windows' candidate lists over gloo (PE_BENCH_EXCHANGE=host).  Its results must equal the
   one-rank run of the same workload: feasible pairs of the fit mask, placed jobs of every greedy
   line, and the node shards must partition the inventory.  The last rank's engine set-up is made to
   fail (PE_BENCH_SIMULATE_RCCL_FAIL): the ranks vote over gloo and all rebuild their engines with the
   node's shared-memory exchange (pe_host_exchange), which the JSON line reports at its top level
   ("degraded") and in config.greedy_exchange.  That fallback runs the production loop (pipelined
   windows, device merge signalled per group), so the 2-rank cfg3 batch must stay within 2x of the
   1-rank one (round 3's synchronous gloo fallback was 20x).
2. A communicator whose peers never arrive returns PE_ERCCL after PE_RCCL_INIT_TIMEOUT_S instead of
   blocking in ncclCommInitRank (non-blocking RCCL set-up, pe_engine.cpp nccl_settle)."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--nodes", "100000", "--fit-jobs", "5000", "--greedy-jobs", "1000", "--agg-jobs", "20000", "--steps", "3",
        "--warmup", "1", "--greedy-steps", "2", "--no-cpu-baseline"]


def _bench(gpus, extra_env):
    """Run bench.py as a child; its stderr goes to gpurun_out/ (a heartbeat line every 20 s there
    too) so a long run is visibly alive on the GPU box."""
    env = dict(os.environ, **extra_env)
    env.setdefault("OMP_NUM_THREADS", "8")
    logdir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    log = os.path.join(logdir, f"test_multirank_bench_n{gpus}.log")
    outp = os.path.join(logdir, f"test_multirank_bench_n{gpus}.json")
    with open(log, "w") as err, open(outp, "w") as so:
        # its own process group: a hung run is killed with its rank processes, not just the launcher
        p = subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)] + ARGS,
                             stdout=so, stderr=err, text=True, env=env, cwd=ROOT, start_new_session=True)
        t0 = time.time()
        while p.poll() is None:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                err.write(f"[test heartbeat] {time.time() - t0:.0f} s\n")
                err.flush()
                if time.time() - t0 > 300:
                    os.killpg(p.pid, signal.SIGKILL)
                    p.wait()
                    raise
    out = open(outp).read()
    assert p.returncode == 0, out[-3000:] + open(log).read()[-5000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_bench_two_ranks_matches_one():
    one = _bench(1, {})
    # the last rank's engine set-up fails (simulated): every rank falls back to the gloo exchange
    two = _bench(2, {"PE_BENCH_EXCHANGE": "host", "PE_BENCH_SIMULATE_RCCL_FAIL": "1", "PE_BENCH_INTERLEAVE_ONE": "1"})
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["config"]["greedy_exchange"] == "none (one GPU)"
    assert "RCCL set-up failed" in two["config"]["greedy_exchange"] and "simulated" in two["config"]["greedy_exchange"]
    assert "shared-memory" in two["config"]["greedy_exchange"]
    # the exchange's zero-copy windows ran (walk into the registered segment, merge waits on the device)
    assert two["configs"]["cfg3"]["zero_copy_exchange_windows_per_batch"] > 0
    assert one["configs"]["cfg3"]["zero_copy_exchange_windows_per_batch"] == 0
    assert two["degraded"] is True and "simulated" in two["degraded_reason"] and "degraded" not in one
    cfg1, cfg2 = one["config"], two["config"]
    assert sum(cfg2["shard_nodes_per_rank"]) == cfg2["nodes"] == 100000 and len(cfg2["shard_nodes_per_rank"]) == 2
    assert cfg2["feasible_pairs"] == cfg1["feasible_pairs"] > 0
    assert two["greedy"]["jobs_placed"] == one["greedy"]["jobs_placed"] > 0
    for k in one["configs"]:
        assert two["configs"][k]["jobs_placed"] == one["configs"][k]["jobs_placed"], k
    for k in ("fit_many_values", "fit_worst_case", "fit_adversarial"):
        assert two[k]["feasible_pairs"] == one[k]["feasible_pairs"], k
    assert two["value"] > 0 and two["fit_weak_scaling"]["value"] > 0
    # no throughput cliff on the fallback transport (both ranks share this box's one GPU): every greedy
    # line within 2x of one rank, and the exchange's per-window cost reported for the 8-GPU runs.  The
    # 1-rank reference is the 2-rank run's own: rank 0 alone on an unsharded context, its batches
    # interleaved with the 2-rank ones (PE_BENCH_INTERLEAVE_ONE, medians of each) -- the same box in the
    # same minutes, not a separate bench launch (verdict r5 item 7: box drift made the bound flaky).
    # cfg2 (1k jobs, ~1 ms, 18 windows) is bounded per window instead: there the exchange's fixed cost
    # per window on one shared GPU (~40-90 us measured) is of the order of the
    # whole window
    for k in one["configs"]:
        o_ms, t_ms = two["configs"][k]["interleaved_one_rank_ms_per_batch"], two["configs"][k]["ms_per_batch"]
        assert o_ms > 0
        if k == "cfg2":
            per_window_us = (t_ms - o_ms) / two["configs"][k]["windows_per_batch"] * 1e3
            assert per_window_us <= 120.0, (k, per_window_us, two["configs"][k])
        else:
            assert t_ms <= 2.0 * o_ms, (k, two["configs"][k])
        assert one["configs"][k]["exchange_us_per_window"] is None
        assert "interleaved_one_rank_ms_per_batch" not in one["configs"][k]
        x = two["configs"][k]["exchange_us_per_window"]
        assert x is not None and x["merge"] > 0 and x["wait"] >= 0, (k, x)
    g1 = two["greedy"]["interleaved_one_rank_ms_per_batch"]
    assert two["greedy"]["ms_per_batch"] <= 2.0 * g1, two["greedy"]
    assert two["greedy"]["exchange_us_per_window"]["merge"] > 0


_INIT = r"""
import os, sys, time
sys.path[:0] = [{root!r}, os.path.join({root!r}, "training-operator_amd")]
from placement import Engine, PlacementError, comm_id, _abi
cid = {cid}
t0 = time.time()
try:
    Engine(0, rank=0, world_size=2, comm=cid)
    print("CREATED", flush=True)
except PlacementError as e:
    print("RC", e.code, round(time.time() - t0, 1), flush=True)
# the abandoned set-up's thread is still inside RCCL's bootstrap: leave without static teardown
os._exit(0)
"""


@pytest.mark.timeout(300)
@pytest.mark.parametrize("cid", ["comm_id()", "bytes(range(128))"])
def test_rccl_init_without_peers_times_out(cid):
    """Rank 0 of 2 with nobody else: a real unique id (rank 0 is the root, rank 1 never comes) or a
    garbage id.  Either way pe_create returns PE_ERCCL (-5) within the bound."""
    env = dict(os.environ, PE_RCCL_INIT_TIMEOUT_S="5")
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", _INIT.format(root=ROOT, cid=cid)], capture_output=True, text=True,
                       timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "CREATED" not in p.stdout, p.stdout
    rc = [ln.split() for ln in p.stdout.splitlines() if ln.startswith("RC ")]   # (RCCL prints its banner too)
    assert len(rc) == 1 and int(rc[0][1]) == -5, p.stdout + p.stderr[-2000:]
    assert float(rc[0][2]) < 60 and time.time() - t0 < 200
