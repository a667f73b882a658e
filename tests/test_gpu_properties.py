"""Full-size GPU checks at BASELINE.json's configurations.

Where the oracle finishes in seconds the comparison is bit-exact (cfg3, cfg4 greedy); at the 1M-node
sizes the checks are size-independent properties: counts == popcount(mask), sampled mask rows ==
oracle rows, shard sums == unsharded, capacity conservation, all-or-nothing, determinism, and exact
agreement of the first decisions with the oracle's argmin."""
import threading

import numpy as np
import pytest

import oracle
from placement import Engine, synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def popcount_rows(mask):
    return np.unpackbits(mask.view(np.uint8), axis=1).sum(axis=1)


@pytest.fixture(scope="module")
def cfg5():
    inv = synth.make_inventory(1_000_000, synth.SEED["cfg5"], 0.2)
    req, need = synth.make_fit_jobs(100_000, synth.SEED["cfg5"])
    return inv, req, need


def test_cfg5_fit_mask_full(cfg5):
    inv, req, need = cfg5
    e = Engine(0)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    e.jobs_upload(req, need)
    e.fit_mask_run()
    counts = e.fit_counts()
    rng = np.random.default_rng(1)
    rows = np.sort(rng.choice(100_000, 48, replace=False))
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req[rows], need[rows])
    for i, r in enumerate(rows):
        m = e.fit_mask_rows(int(r), 1)
        np.testing.assert_array_equal(m[0], o_mask[i])
        assert popcount_rows(m)[0] == counts[r] == o_counts[i]
    last = e.fit_mask_rows(99_999, 1)                      # ragged last tile band
    assert popcount_rows(last)[0] == counts[99_999]
    # determinism: a second pass gives the same counts
    e.fit_mask_run()
    np.testing.assert_array_equal(e.fit_counts(), counts)
    e.close()
    # 4 shards: per-shard counts sum to the unsharded counts
    total = np.zeros_like(counts)
    for r in range(4):
        s = Engine(0, rank=r, world_size=4, exchange=lambda b: b * 4)
        s.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        s.jobs_upload(req, need)
        s.fit_mask_run()
        total += s.fit_counts()
        s.close()
    np.testing.assert_array_equal(total, counts)


@pytest.mark.parametrize("cfg,mix,n_nodes,n_jobs,gpu_frac", [("cfg3", "mixed", 100_000, 10_000, 0.2),
                                                            ("cfg4", "gang8", 100_000, 10_000, 1.0),
                                                            ("cfg4", "island8", 100_000, 10_000, 1.0)])
def test_greedy_full_size_bit_exact(cfg, mix, n_nodes, n_jobs, gpu_frac):
    inv = synth.make_inventory(n_nodes, synth.SEED[cfg], gpu_frac)
    batch = synth.make_jobs(n_jobs, synth.SEED[cfg], mix)
    e = Engine(0)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    pods, st = e.place_batch(batch)
    w_pods, w_st, w_res = oracle.place_greedy(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                              batch.group_count, batch.group_req, batch.group_need)
    np.testing.assert_array_equal(st, w_st)
    np.testing.assert_array_equal(pods, w_pods)
    np.testing.assert_array_equal(e.read_residuals(), w_res)
    e.close()


def check_invariants(inv, batch, pods, st, res_after):
    """capacity conservation, fit, all-or-nothing."""
    res0 = inv.residual()
    pod_group = np.repeat(np.arange(len(batch.group_count)), batch.group_count)
    job_of_group = np.repeat(np.arange(batch.n_jobs), np.diff(batch.job_group_off))
    pod_job = job_of_group[pod_group]
    placed = pods >= 0
    # all-or-nothing: a job is placed iff every one of its pods is
    per_job_missing = np.bincount(pod_job[~placed], minlength=batch.n_jobs)
    assert np.all((st == 0) == (per_job_missing == 0))
    # conservation: residual_after = residual_before - sum of requests of pods placed there
    used = np.zeros_like(res0)
    for d in range(4):
        np.add.at(used[d], pods[placed], batch.group_req[pod_group[placed], d])
    np.testing.assert_array_equal(res_after, res0 - used)
    # nothing over-committed that was not already
    assert np.all((res_after >= 0) | (res0 < 0))
    # label constraints of placed pods
    need = batch.group_need[pod_group[placed]]
    assert np.all((inv.labels[pods[placed]] & need) == need)


def test_greedy_1m_nodes_properties():
    inv = synth.make_inventory(1_000_000, synth.SEED["cfg3"], 0.2)
    batch = synth.make_jobs(10_000, synth.SEED["cfg3"], "mixed")
    e = Engine(0)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    pods, st = e.place_batch(batch)
    check_invariants(inv, batch, pods, st, e.read_residuals())
    e.reset_residuals()
    pods2, st2 = e.place_batch(batch)                       # determinism
    np.testing.assert_array_equal(pods2, pods)
    np.testing.assert_array_equal(st2, st)
    # the first 3 jobs in priority order decide exactly as the sequential oracle
    order = np.argsort(-batch.priority, kind="stable")[:3]
    sub_off = [0]
    cnt, req, nd, pri = [], [], [], []
    for j in order:
        g0, g1 = batch.job_group_off[j], batch.job_group_off[j + 1]
        cnt += list(batch.group_count[g0:g1])
        req += list(batch.group_req[g0:g1])
        nd += list(batch.group_need[g0:g1])
        pri.append(batch.priority[j])
        sub_off.append(sub_off[-1] + (g1 - g0))
    w_pods, w_st, _ = oracle.place_greedy(inv.residual(), inv.labels, np.array(sub_off), np.array(pri),
                                          np.array(cnt), np.array(req), np.array(nd))
    got = np.concatenate([pods[int(np.sum(batch.group_count[:batch.job_group_off[j]])):
                               int(np.sum(batch.group_count[:batch.job_group_off[j + 1]]))] for j in order])
    np.testing.assert_array_equal(got, w_pods)
    e.close()


def test_greedy_1m_nodes_sharded_equals_unsharded():
    inv = synth.make_inventory(1_000_000, synth.SEED["cfg3"], 0.2)
    batch = synth.make_jobs(2_000, synth.SEED["cfg3"] + 100, "mixed")
    ref = Engine(0)
    ref.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    r_pods, r_st = ref.place_batch(batch)
    ref.close()
    W = 2
    slots = [None] * W
    bar = threading.Barrier(W)

    def ex_for(r):
        def ex(blob):
            slots[r] = blob
            bar.wait(timeout=120)
            out = b"".join(slots)
            bar.wait(timeout=120)
            return out
        return ex

    engines = [Engine(0, rank=r, world_size=W, exchange=ex_for(r)) for r in range(W)]
    for en in engines:
        en.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    out = [None] * W
    th = [threading.Thread(target=lambda r=r: out.__setitem__(r, engines[r].place_batch(batch))) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    for r in range(W):
        np.testing.assert_array_equal(out[r][0], r_pods)
        np.testing.assert_array_equal(out[r][1], r_st)
    for en in engines:
        en.close()
