"""The benchmarked workloads, compared with the C oracle IN FULL (verdict r3, item 1).

bench.py's two headline lines are checked here output for output, not by sampled rows or
invariants:
- `greedy`: the cfg3 10k-job mix on the bench's 1M-node inventory (SEED cfg5, 20 % GPU nodes),
  every pod, job status and residual bit-exact vs `oracle.place_greedy` (the naive sequential
  Appendix-B rule, ~12 s on 16 threads), unsharded and through 2 node shards;
- the cfg5 fit mask: all 100k x 1M mask rows (in chunks of 4096 jobs) and all 100k counts vs
  `oracle.fit_mask`.
The oracle is the checker only; the engine results come from libplacement.so on the GPU."""
import os
import threading

import numpy as np
import pytest

import oracle
from placement import Engine, HostExchange, synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N_NODES = 1_000_000


@pytest.fixture(scope="module")
def bench_inv():
    # bench.py: inv = synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2), shared by every line
    return synth.make_inventory(N_NODES, synth.SEED["cfg5"], 0.2)


@pytest.fixture(scope="module")
def greedy_batch():
    # bench.py greedy line: synth.make_jobs(args.greedy_jobs = 10000, synth.SEED["cfg3"], "mixed")
    return synth.make_jobs(10_000, synth.SEED["cfg3"], "mixed")


@pytest.fixture(scope="module")
def greedy_oracle(bench_inv, greedy_batch):
    inv, b = bench_inv, greedy_batch
    return oracle.place_greedy(inv.residual(), inv.labels, b.job_group_off, b.priority, b.group_count,
                               b.group_req, b.group_need)


def _assert_same(pods, st, res, want):
    w_pods, w_st, w_res = want
    np.testing.assert_array_equal(st, w_st)
    np.testing.assert_array_equal(pods, w_pods)
    np.testing.assert_array_equal(res, w_res)


def test_bench_greedy_batch_vs_oracle(bench_inv, greedy_batch, greedy_oracle):
    inv, b = bench_inv, greedy_batch
    e = Engine(0, max_nodes=N_NODES)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    pods, st = e.place_batch(b)
    _assert_same(pods, st, e.read_residuals(), greedy_oracle)
    assert int((st == 0).sum()) > 0 and int((pods >= 0).sum()) > 0   # (every job fits the 1M-node inventory)
    # the bench times repeated batches after pe_reset_residuals: the second one too
    e.reset_residuals()
    pods, st = e.place_batch(b)
    _assert_same(pods, st, e.read_residuals(), greedy_oracle)
    e.close()


def test_bench_greedy_batch_two_shards_vs_oracle(bench_inv, greedy_batch, greedy_oracle):
    """Two node shards (host exchange, one thread per rank) against the ORACLE, not against the
    unsharded engine; each rank's device shard holds its slice of the oracle's final residuals."""
    inv, b = bench_inv, greedy_batch
    W = 2
    slots = [None] * W
    bar = threading.Barrier(W)

    def ex_for(r):
        def ex(blob):
            slots[r] = blob
            bar.wait(timeout=300)
            out = b"".join(slots)
            bar.wait(timeout=300)
            return out
        return ex

    engines = [Engine(0, rank=r, world_size=W, exchange=ex_for(r), max_nodes=N_NODES) for r in range(W)]
    for en in engines:
        en.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    out = [None] * W
    errs = []

    def run(r):
        try:
            out[r] = engines[r].place_batch(b)
        except Exception as ex:   # noqa: BLE001 -- reported below
            errs.append(ex)
            bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not errs, errs
    w_pods, w_st, w_res = greedy_oracle
    for r in range(W):
        np.testing.assert_array_equal(out[r][1], w_st)
        np.testing.assert_array_equal(out[r][0], w_pods)
        lo, hi = engines[r].shard_range()
        np.testing.assert_array_equal(engines[r].read_residuals(), w_res[:, lo:hi])
    for en in engines:
        en.close()


def _run_ranks(engines, batch, timeout=600):
    out = [None] * len(engines)
    errs = []

    def run(r):
        try:
            out[r] = engines[r].place_batch(batch)
        except Exception as ex:   # noqa: BLE001 -- reported below
            errs.append((r, ex))

    th = [threading.Thread(target=run, args=(r,)) for r in range(len(engines))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=timeout)
    assert not any(t.is_alive() for t in th), "a rank never returned"
    assert not errs, errs
    return out


def test_bench_greedy_batch_eight_shards_vs_oracle(bench_inv, greedy_batch, greedy_oracle):
    """The bench's greedy batch split EIGHT ways, as BASELINE cfg3 shards it over the 8 GPUs of a
    node (verdict r4, item 2a): 8 shard contexts of 125k nodes in one process on the one GPU, over the
    production transport of one node's ranks -- the native shared-memory exchange with zero-copy
    windows (every walk writes its rank's lists into the registered segment, each rank's exchange
    thread merges every group on the host as all 8 ranks signalled it).  Every rank's pods and job
    statuses against the ORACLE, each device shard against its slice of the oracle's residuals, and
    a second batch after pe_reset_residuals (the bench's repeated batches)."""
    inv, b = bench_inv, greedy_batch
    W = 8
    name = f"/pe_fo8_{os.getpid()}"
    hxs = [HostExchange(name, r, W, 128 * (16 + 8 * 256)) for r in range(W)]
    engines = [Engine(0, rank=r, world_size=W, exchange=hxs[r], max_nodes=N_NODES) for r in range(W)]
    for en in engines:
        en.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    w_pods, w_st, w_res = greedy_oracle
    covered = 0
    for rep in range(2):
        if rep:
            for en in engines:
                en.reset_residuals()
        out = _run_ranks(engines, b)
        for r in range(W):
            np.testing.assert_array_equal(out[r][1], w_st)
            np.testing.assert_array_equal(out[r][0], w_pods)
            lo, hi = engines[r].shard_range()
            np.testing.assert_array_equal(engines[r].read_residuals(), w_res[:, lo:hi])
            if not rep:
                covered += hi - lo
    assert covered == N_NODES
    for en in engines:
        s = en.stats()
        assert s["xchg_zc_windows"] > 0 and s["xchg_zc_windows"] == s["windows"], s   # every window zero-copy
    for en in engines:
        en.close()
    for x in hxs:
        x.close()


def test_cfg5_fit_mask_every_row_vs_oracle(bench_inv):
    """All 100k rows of the cfg5 mask (12.5 GB) and all counts, chunk by chunk."""
    inv = bench_inv
    req, need = synth.make_fit_jobs(100_000, synth.SEED["cfg5"])
    e = Engine(0, max_nodes=N_NODES)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    e.jobs_upload(req, need)
    e.fit_mask_run()
    counts = e.fit_counts()
    res = inv.residual()
    C = 4096
    for j0 in range(0, 100_000, C):
        j1 = min(100_000, j0 + C)
        o_mask, o_counts = oracle.fit_mask(res, inv.labels, req[j0:j1], need[j0:j1])
        g_mask = e.fit_mask_rows(j0, j1 - j0)
        if not np.array_equal(g_mask, o_mask):
            bad = np.nonzero((g_mask != o_mask).any(axis=1))[0]
            pytest.fail(f"mask rows differ from the oracle: {len(bad)} rows of [{j0}, {j1}), first job {j0 + bad[0]}")
        np.testing.assert_array_equal(counts[j0:j1], o_counts)
        del o_mask, g_mask
    e.close()
