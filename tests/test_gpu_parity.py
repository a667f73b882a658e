"""GPU parity: every kernel through the C ABI vs the CPU oracle, bit-exact (integer work).

Runs on the MI355X box (`pytest -m gpu`).  Sizes are ones the oracle finishes in seconds;
full-size cases are covered by size-independent properties in test_gpu_properties.py."""
import json
import os
import threading

import numpy as np
import pytest

import oracle
from oracle import flatten as F
from oracle import semantics as S
from placement import Engine, V1, V2, synth

pytestmark = pytest.mark.gpu
GPU = "nvidia.com/gpu"


@pytest.fixture(scope="module")
def eng():
    e = Engine(0, gpu_resource_name=GPU)
    yield e
    e.close()


def load(golden_dir, name):
    with open(os.path.join(golden_dir, name + ".json")) as f:
        return json.load(f)


# ------------------------------------------------------------------ aggregation

def _pc_get(case):
    pri = case.get("priorities", {})
    return lambda name: pri.get(name)


def test_pg_min_resources_v1_golden(eng, golden_dir):
    g = load(golden_dir, "v1_podgroup")
    flat, expect = F.Flat(), []
    for case in g["cases"]:
        if (case["scheduling_policy"] or {}).get("minResources") is not None:
            continue
        mm = S.v1_pg_spec(case["replicas"], case["scheduling_policy"], _pc_get(case))[0]
        F.add_v1_job(flat, mm, case["replicas"], GPU, _pc_get(case))
        expect.append(case)
    arrs = flat.arrays()
    out, pres, mem, ovf = eng.pg_min_resources(V1, *arrs)
    o_out, o_pres, o_mem, o_ovf = oracle.pg_min_resources(oracle.V1, *arrs)
    np.testing.assert_array_equal(out, o_out)
    np.testing.assert_array_equal(pres, o_pres)
    np.testing.assert_array_equal(mem, o_mem)
    for j, case in enumerate(expect):
        want = F.canonical_list({k: S.parse_quantity(v) for k, v in case["want"].items()}, GPU)
        assert F.unflatten(out[j], pres[j], GPU) == want, case["name"]


def test_pg_min_resources_v2_golden(eng, golden_dir):
    g = load(golden_dir, "v2_podgroup")
    flat, expect = F.Flat(), []
    for case in g["cases"]:
        if case["want"] is None:
            continue
        info = S.new_info([(n, 1, pod) for n, pod in case["replicated_jobs"]])
        S.enforce_ml_policy(info, case["ml_policy"], case["trainjob_num_nodes"])
        pods = dict(case["replicated_jobs"])
        for name in sorted(info["TotalRequests"]):
            F.add_v2_pod_group(flat, info["TotalRequests"][name]["Replicas"], pods[name], GPU)
        flat.end_job(0)
        expect.append(case)
    out, pres, mem, ovf = eng.pg_min_resources(V2, *flat.arrays())
    for j, case in enumerate(expect):
        want = F.canonical_list({k: S.parse_quantity(v) for k, v in case["want"]["minResources"].items()}, GPU)
        assert F.unflatten(out[j], pres[j], GPU) == want, case["name"]
        assert mem[j] == case["want"]["minMember"]
        assert ovf[j] == 0


def random_csr(J, seed, big=False):
    rng = np.random.default_rng(seed)
    ng = rng.integers(0, 5, J)
    jgo = np.concatenate([[0], np.cumsum(ng)]).astype(np.int32)
    G = int(jgo[-1])
    rep = rng.integers(-1, 40, G).astype(np.int32)
    rep[rng.random(G) < 0.05] = 2**31 - 1
    nc = rng.integers(0, 5, G)
    gco = np.concatenate([[0], np.cumsum(nc)]).astype(np.int32)
    C = int(gco[-1])
    hi = 2**62 if big else 2**40
    req = rng.integers(0, hi, (C, 4), dtype=np.int64)
    req[rng.random((C, 4)) < 0.3] = 0
    fl = (rng.integers(0, 16, C) | (rng.integers(0, 4, C) << 4)).astype(np.uint8)
    mm = rng.integers(-2, 60, J).astype(np.int32)
    return jgo, mm, rep, gco, req, fl


@pytest.mark.parametrize("mode", [V1, V2])
@pytest.mark.parametrize("big", [False, True])
def test_pg_min_resources_random_vs_oracle(eng, mode, big):
    arrs = random_csr(20000, 7 + mode + 10 * big, big)
    got = eng.pg_min_resources(mode, *arrs)
    want = oracle.pg_min_resources(mode, *arrs)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    if big:
        assert want[3].sum() > 0      # overflow path exercised and flagged identically


@pytest.mark.parametrize("C,bad", [(1000, 777), (400_000, 1_234_567), (400_000, 4 * 400_000 - 1), (400_000, None)])
def test_pg_min_resources_input_validation(eng, C, bad):
    """Input checks (negative requests, non-monotonic offsets) report the FIRST offending index,
    on small arrays and on ones large enough to be scanned by the planning pool's threads."""
    from placement import PlacementError
    jgo = np.arange(C + 1, dtype=np.int32)
    rep = np.ones(C, np.int32)
    mm = np.ones(C, np.int32)
    req = np.ones((C, 4), np.int64)
    fl = np.full(C, 15, np.uint8)
    if bad is None:
        out = eng.pg_min_resources(V1, jgo, mm, rep, jgo.copy(), req, fl)
        assert (out[0] == 1).all()
        gco = jgo.copy()
        gco[C // 2 + 1] = gco[C // 2] - 1                  # non-monotonic group offsets
        with pytest.raises(PlacementError, match="not monotonic"):
            eng.pg_min_resources(V1, jgo, mm, rep, gco, req, fl)
        return
    req.flat[bad] = -1
    req.flat[min(bad + 5, req.size - 1)] = -7              # a later one must not be the one reported
    with pytest.raises(PlacementError, match=f"negative request at index {bad}$"):
        eng.pg_min_resources(V1, jgo, mm, rep, jgo.copy(), req, fl)


def test_pg_min_resources_empty(eng):
    z = np.zeros(1, np.int32)
    out = eng.pg_min_resources(V2, z, None, np.zeros(0, np.int32), z, np.zeros((0, 4), np.int64), np.zeros(0, np.uint8))
    assert out[0].shape == (0, 4)


# ------------------------------------------------------------------ fit mask

@pytest.mark.parametrize("N,J", [(1, 1), (63, 5), (64, 256), (257, 3), (1000, 300), (4097, 513), (20000, 1000)])
def test_fit_mask_vs_oracle(eng, N, J):
    inv = synth.make_inventory(N, 17 + N)
    req, need = synth.make_fit_jobs(J, 19 + J)
    eng.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    counts = eng.fit_mask(req, need)
    mask = eng.fit_mask_rows(0, J)
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    np.testing.assert_array_equal(mask, o_mask)
    np.testing.assert_array_equal(counts, o_counts)
    assert 0 < counts.sum() < N * J or N * J < 10


def test_fit_mask_edge_values(eng):
    # zero requests fit everything incl. exhausted nodes; requests equal to residual fit; negative
    # residual (over-committed node) fits nothing; INT64_MAX capacity
    N = 130
    cap = np.full((4, N), 100, np.int64)
    used = np.zeros_like(cap)
    used[:, 5] = 100                      # exhausted
    cap[:, 7] = np.iinfo(np.int64).max
    used[0, 9] = 150                      # over-committed cpu -> negative residual
    labels = np.arange(N, dtype=np.uint32) % 4
    eng.load_nodes(cap, used, labels)
    req = np.array([[0, 0, 0, 0], [100, 100, 100, 100], [101, 0, 0, 0], [0, 0, 0, 0], [2**62, 0, 0, 0]], np.int64)
    need = np.array([0, 0, 0, 3, 0], np.uint32)
    counts = eng.fit_mask(req, need)
    o_mask, o_counts = oracle.fit_mask(cap - used, labels, req, need)
    np.testing.assert_array_equal(eng.fit_mask_rows(0, 5), o_mask)
    np.testing.assert_array_equal(counts, o_counts)
    assert counts[0] == N - 1 and counts[4] == 1


PATHS = {"planes": (0, "fit_runs_planes", 3), "planes_blocks": (16 | 32, "fit_runs_planes", 2),
         "therm": (5, "fit_runs_therm", 1), "swar": (13, "fit_runs_coded", 1),
         "i32": (3, "fit_runs_i32", 0), "i64": (1, "fit_runs_i64", 0)}


@pytest.mark.parametrize("path", ["planes", "planes_blocks", "therm", "swar", "i32", "i64"])
@pytest.mark.parametrize("N,J", [(5000, 300), (777, 65), (64, 1), (600_000, 2085)])
def test_fit_mask_paths(path, N, J):
    """Every exact fit path on the same data (residuals span the int32 saturation point after
    scaling: nodes with 2^50 B of memory; over-committed nodes with negative residuals)."""
    mask_bits, stat, layout = PATHS[path]
    e = Engine(0, fit_path_mask=mask_bits)
    inv = synth.make_inventory(N, 71 + N, 0.5)
    inv.cap[1, ::7] = 1 << 50
    inv.used[0, 3::11] = inv.cap[0, 3::11] + 1000
    req, need = synth.make_fit_jobs(J, 73 + J)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    counts = e.fit_mask(req, need)
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    np.testing.assert_array_equal(e.fit_mask_rows(0, J), o_mask)
    np.testing.assert_array_equal(counts, o_counts)
    s = e.stats()
    assert s[stat] == 1 and s["fit_runs_planes"] + s["fit_runs_coded"] + s["fit_runs_i32"] + s["fit_runs_i64"] == 1
    assert s["fit_runs_therm"] == (path == "therm")
    assert e.fit_mask_layout() == layout
    e.close()


@pytest.mark.parametrize("N,J,pitch_blocks", [(62 * 8192 - 100, 300, 62), (123 * 8192 - 5000, 64, 123),
                                              (100 * 8192, 70, 100), (5000, 8, 1)])
def test_fit_mask_rows_pitch(N, J, pitch_blocks):
    """Row-major planes mask: the reported row pitch, zero padding bits past the last node (counts
    would include them otherwise), rows handed back exact (first and last rows)."""
    e = Engine(0)
    inv = synth.make_inventory(N, 17 + N % 97, 0.4)
    req, need = synth.make_fit_jobs(J, 19 + J)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    counts = e.fit_mask(req, need)
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    assert e.fit_mask_layout() == 3 and e.fit_mask_row_pitch() == pitch_blocks * 128
    np.testing.assert_array_equal(counts, o_counts)
    np.testing.assert_array_equal(e.fit_mask_rows(0, J), o_mask)
    np.testing.assert_array_equal(e.fit_mask_rows(J - 3, 3), o_mask[J - 3:])
    e.close()


@pytest.mark.parametrize("case", ["many_values", "odd_bytes", "label_antichain", "many_planes", "plane_sets",
                                  "lds", "extreme_values"])
def test_fit_mask_path_fallbacks(eng, case):
    """Each batch shape lands on the path that can hold it (one plane set > LDS digit planes > plane
    sets > coded > int32 > int64), exact.  The compare/coded cases run with the plane paths disabled:
    the LDS digit planes hold them otherwise."""
    N, J = 3000, 400
    inv = synth.make_inventory(N, 91, 0.3)
    req, need = synth.make_fit_jobs(J, 93)
    if case == "many_values":
        req[:, 0] = 500 + np.arange(J) * 7          # 400 distinct cpu requests: no 32-bit code word
        want = "fit_runs_i32"
    elif case == "odd_bytes":
        req[:, 1] = req[:, 1] + np.arange(J) % 3     # odd byte counts, 3 extra values -> still coded
        req[:, 0] = 500 + np.arange(J) * 7
        req[5, 1] += 1                               # and no common power of two -> int64 compare
        want = "fit_runs_i64"
    elif case == "label_antichain":
        inv.labels[:] = np.arange(N, dtype=np.uint32) % 8
        need[:] = np.where(np.arange(J) % 2 == 0, 1, 2)   # {1} and {2}: no chain, but 2 planes
        want = "fit_runs_planes"
    elif case == "many_planes":
        req[:, 0] = 500 + (np.arange(J) % 40) * 7    # 40 distinct cpu values: > 32 planes, SWAR-coded
        want = "fit_runs_coded"
    elif case == "plane_sets":
        req[:, 0] = 500 + (np.arange(J) % 40) * 7    # the same batch with planes but not LDS: plane sets
        want = "fit_runs_planes"
    elif case == "lds":
        req[:, 0] = 500 + (np.arange(J) % 40) * 7    # the same batch with every path: LDS digit planes
        want = "fit_runs_lds"
    else:
        req[0] = [np.iinfo(np.int64).max, 0, 0, 0]   # int64 extremes are just two more planes
        req[1] = [0, np.iinfo(np.int64).max, 0, np.iinfo(np.int64).max]
        inv.used[0, :7] = inv.cap[0, :7] + 5         # over-committed nodes: no request fits them
        want = "fit_runs_planes"
    if case == "plane_sets":
        e = Engine(0, fit_path_mask=16)                   # bit planes (sets), no LDS digit planes
    elif want in ("fit_runs_planes", "fit_runs_lds"):
        e = eng
    else:
        e = Engine(0, fit_path_mask=1 | 2 | 4)            # no planes
    e.reset_stats()
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    counts = e.fit_mask(req, need)
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    np.testing.assert_array_equal(e.fit_mask_rows(0, J), o_mask)
    np.testing.assert_array_equal(counts, o_counts)
    assert e.stats()[want] == 1
    if e is not eng:
        e.close()


@pytest.mark.parametrize("N,J,shape", [(3000, 400, "cpu400"), (20000, 5000, "wide"), (123 * 8192 - 7, 700, "wide"),
                                       (9000, 2000, "unique_mem"), (70000, 64, "wide"), (3000, 1, "wide"),
                                       (3 * 8192 + 777, 1200, "needs_sets")])
def test_fit_mask_plane_sets(N, J, shape):
    """Batches with more than 32 distinct (dimension, value) pairs split into plane sets, each
    encoded and swept by the indexed-row kernel: mask rows and counts exact vs the oracle; the
    same mask as the compare path."""
    rng = np.random.default_rng(N + J)
    inv = synth.make_inventory(N, 31 + N % 89, 0.4)
    req, need = synth.make_fit_jobs(J, 37 + J)
    if shape == "cpu400":
        req[:, 0] = 500 + np.arange(J) * 7                              # 400 distinct cpu values
    elif shape == "wide":                                               # every dimension many-valued
        req[:, 0] = rng.integers(1, 120, J) * 250
        req[:, 1] = rng.integers(1, 60, J) * (1 << 28)
        req[:, 3] = rng.integers(0, 30, J) * (1 << 30)
        need[:] = rng.integers(0, 4, J).astype(np.uint32) << 1
    elif shape == "needs_sets":
        # label-need planes (kind 4) in every set, at least 3 sets, and a last 512-node encode
        # segment that is partial: the per-set offsets and the valid-node masking of the encode meet
        req[:, 0] = 100 * (1 + np.arange(J) % 90)
        need[:] = (np.arange(J) % 6).astype(np.uint32) << 1
        inv.labels[:] |= (np.arange(N, dtype=np.uint32) % 7).astype(np.uint32) << 1
    else:                                                               # unique memory per job
        req[:, 1] = (1 << 30) + np.arange(J) * 4096
    e = Engine(0, fit_path_mask=16)                       # bit planes (+ the int64 fallback), no LDS
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    counts = e.fit_mask(req, need)
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    np.testing.assert_array_equal(counts, o_counts)
    np.testing.assert_array_equal(e.fit_mask_rows(0, J), o_mask)
    s = e.stats()
    pairs = sum(len(np.unique(req[:, d])) for d in range(4)) + len(np.unique(need))
    # planes when the sets fit (<= 256: 400 cpu values make ~31 sets; independent random values in
    # every dimension need hundreds), else a fallback path; exact either way
    assert s["fit_runs_planes"] + s["fit_runs_coded"] + s["fit_runs_i32"] + s["fit_runs_i64"] == 1
    if shape in ("cpu400", "needs_sets") or pairs <= 32:
        assert s["fit_runs_planes"] == 1 and e.fit_mask_layout() == 3
    if shape == "needs_sets":
        assert s["fit_runs_sets"] == 1 and pairs > 3 * 32      # more pairs than 3 sets hold
    # a second run over the same upload is identical (counts re-zeroed, every set re-encoded)
    np.testing.assert_array_equal(e.fit_mask(req, need), o_counts)
    e.close()


def test_fit_mask_plane_sets_sharded():
    """Plane sets on two shard contexts of one inventory: the column blocks concatenate to the
    unsharded oracle mask, per-job counts sum."""
    N, J = 30001, 900
    rng = np.random.default_rng(5)
    inv = synth.make_inventory(N, 41)
    req, need = synth.make_fit_jobs(J, 43)
    req[:, 0] = rng.integers(1, 200, J) * 125
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    total = np.zeros(J, np.int64)
    for rank in range(2):
        e = Engine(0, rank=rank, world_size=2, exchange=lambda b: b + b, fit_path_mask=16)
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        b, en = e.shard_range()
        total += e.fit_mask(req, need)
        assert e.stats()["fit_runs_planes"] == 1
        want, _ = oracle.fit_mask(inv.residual()[:, b:en], inv.labels[b:en], req, need)
        np.testing.assert_array_equal(e.fit_mask_rows(0, J), want)
        e.close()
    np.testing.assert_array_equal(total, o_counts)


def test_fit_mask_sharded_columns(eng):
    """Two shards (ranks) of one inventory: column blocks concatenate to the unsharded mask."""
    N, J = 3001, 130
    inv = synth.make_inventory(N, 23)
    req, need = synth.make_fit_jobs(J, 29)
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    total = np.zeros(J, np.int64)
    for r in range(2):
        e = Engine(0, rank=r, world_size=2, exchange=lambda b: b + b)
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        b, en = e.shard_range()
        total += e.fit_mask(req, need)
        m = e.fit_mask_rows(0, J)
        sub_res = inv.residual()[:, b:en]
        want, _ = oracle.fit_mask(sub_res, inv.labels[b:en], req, need)
        np.testing.assert_array_equal(m, want)
        e.close()
    np.testing.assert_array_equal(total, o_counts)


# ------------------------------------------------------------------ greedy placement

def check_greedy(e, inv, batch):
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    pods, st = e.place_batch(batch)
    w_pods, w_st, w_res = oracle.place_greedy(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                              batch.group_count, batch.group_req, batch.group_need)
    np.testing.assert_array_equal(st, w_st)
    np.testing.assert_array_equal(pods, w_pods)
    b, en = e.shard_range()
    np.testing.assert_array_equal(e.read_residuals(), w_res[:, b:en])
    return st


@pytest.mark.parametrize("mix,N,J,gpu_frac", [("pytorch", 2000, 200, 0.2), ("mixed", 3000, 300, 0.3),
                                               ("gang8", 600, 120, 1.0), ("island8", 800, 300, 0.8)])
def test_greedy_vs_oracle(eng, mix, N, J, gpu_frac):
    inv = synth.make_inventory(N, 31 + N, gpu_frac)
    batch = synth.make_jobs(J, 37 + J, mix)
    st = check_greedy(eng, inv, batch)
    assert (st == 0).any()


@pytest.mark.parametrize("mix,topk", [("gang8", 8), ("island8", 16), ("gang8", 600)])
def test_greedy_list_growth(monkeypatch, mix, topk):
    """Whole-node gangs exhaust short candidate lists (rescans); after the first rescan the engine walks
    lists of 2 x topk (capped at 1023) for the rest of the batch (pe_engine.cpp, one GPU).  Both ways
    bit-exact vs the oracle; growth never rescans more than the fixed length."""
    inv = synth.make_inventory(3000, 71, 1.0)
    batch = synth.make_jobs(400, 73, mix)
    rescans = {}
    for growth in (False, True):
        if growth:
            monkeypatch.delenv("PE_NO_LIST_GROWTH", raising=False)
        else:
            monkeypatch.setenv("PE_NO_LIST_GROWTH", "1")
        e = Engine(0, topk=topk, window_groups=32)
        check_greedy(e, inv, batch)
        rescans[growth] = e.stats()["rescans"]
        e.close()
    assert rescans[True] <= rescans[False]
    if topk < 100:
        assert rescans[False] > 0          # the case does exhaust its lists
        assert rescans[True] < rescans[False]


@pytest.mark.parametrize("topk,wg,wp", [(1, 1, 1), (2, 8, 32), (8, 64, 1024), (256, 16, 4096), (1023, 64, 1024)])
def test_greedy_window_configs(topk, wg, wp):
    e = Engine(0, topk=topk, window_groups=wg, window_pods=wp)
    inv = synth.make_inventory(1500, 41, 0.3)
    batch = synth.make_jobs(150, 43, "mixed")
    check_greedy(e, inv, batch)
    s = e.stats()
    assert s["windows"] > 0
    e.close()


def test_greedy_cfg2_full_size(eng):
    """Config 2 as BASELINE.json names it: 10k nodes x 1k PyTorchJobs, bit-exact."""
    inv = synth.make_inventory(10_000, synth.SEED["cfg2"], 0.2)
    batch = synth.make_jobs(1000, synth.SEED["cfg2"], "pytorch")
    st = check_greedy(eng, inv, batch)
    assert 0 < (st == 0).sum() < 1000


def test_greedy_sharded_exchange():
    """2 shards on one GPU (two contexts, host all-gather between threads) == unsharded oracle."""
    inv = synth.make_inventory(2500, 47, 0.25)
    batch = synth.make_jobs(200, 53, "mixed")
    W = 2
    slots = [None] * W
    bar = threading.Barrier(W)

    def exchange_for(r):
        def ex(blob):
            slots[r] = blob
            bar.wait(timeout=60)
            out = b"".join(slots)
            bar.wait(timeout=60)
            return out
        return ex

    engines = [Engine(0, rank=r, world_size=W, exchange=exchange_for(r), topk=4, window_groups=8) for r in range(W)]
    for e in engines:
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    results = [None] * W

    def run(r):
        results[r] = engines[r].place_batch(batch)

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    w_pods, w_st, w_res = oracle.place_greedy(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                              batch.group_count, batch.group_req, batch.group_need)
    for r in range(W):
        pods, st = results[r]
        np.testing.assert_array_equal(st, w_st)
        np.testing.assert_array_equal(pods, w_pods)
        b, en = engines[r].shard_range()
        np.testing.assert_array_equal(engines[r].read_residuals(), w_res[:, b:en])
    for e in engines:
        e.close()


@pytest.mark.parametrize("host_merge,flags", [(False, 0), (False, 1), (True, 0), (False, 2)])
def test_greedy_rccl_single_rank(host_merge, flags):
    """The RCCL window path (ncclAllGather of the candidate blobs) on a 1-rank communicator: the
    gathered lists merged on the device and signalled per group (default), the same synced
    (greedy_flags bit0: sequential windows) or from the full scan (bit1), or merged on the host
    (PE_HOST_MERGE=1)."""
    from placement import comm_id
    if host_merge:
        os.environ["PE_HOST_MERGE"] = "1"
    try:
        e = Engine(0, world_size=1, comm=comm_id(), topk=8, window_groups=16, greedy_flags=flags)
        inv = synth.make_inventory(3000, 83, 0.25)
        batch = synth.make_jobs(250, 89, "mixed")
        check_greedy(e, inv, batch)
        e.close()
    finally:
        os.environ.pop("PE_HOST_MERGE", None)


@pytest.mark.parametrize("mix,topk", [("gang8", 8), ("island8", 16)])
def test_greedy_rccl_list_growth(mix, topk):
    """Verdict r5 item 3: the RCCL transport grows its lists after a rescan like one GPU does (its
    windows are written, all-gathered and merged at the window's own list length).  A 1-rank RCCL
    context rescans exactly as often as the unsharded context on the same batch, both bit-exact."""
    from placement import comm_id
    inv = synth.make_inventory(3000, 71, 1.0)
    batch = synth.make_jobs(400, 73, mix)
    rescans = {}
    for rccl in (False, True):
        e = Engine(0, world_size=1, comm=comm_id(), topk=topk, window_groups=32) if rccl else \
            Engine(0, topk=topk, window_groups=32)
        check_greedy(e, inv, batch)
        rescans[rccl] = e.stats()["rescans"]
        if rccl:
            assert e.comm_ranks() == 1
        e.close()
    assert rescans[True] == rescans[False] > 0, rescans


def test_greedy_rccl_window_timeout_aborts():
    """A window whose all-gather never completes (verdict r4, item 3): a test kernel holds the stream
    for 8 s right before window 3's ncclAllGather (PE_TEST_STALL_*), so the window's merged lists
    cannot arrive while the stream stays busy -- the case the idle test cannot tell from a slow walk.
    With PE_RCCL_TIMEOUT_S = 2 the call returns PE_ERCCL within the bound, the communicator is aborted,
    and every later call fails fast with PE_ERCCL (the caller rebuilds the context)."""
    import time

    from placement import PlacementError, comm_id
    env = {"PE_TEST_STALL_WINDOW": "3", "PE_TEST_STALL_MS": "8000", "PE_RCCL_TIMEOUT_S": "2"}
    os.environ.update(env)
    try:
        e = Engine(0, world_size=1, comm=comm_id(), topk=8, window_groups=16)
        assert e.comm_ranks() == 1
        inv = synth.make_inventory(3000, 83, 0.25)
        batch = synth.make_jobs(250, 89, "mixed")
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        t0 = time.monotonic()
        with pytest.raises(PlacementError) as ei:
            e.place_batch(batch)
        dt = time.monotonic() - t0
        assert ei.value.code == -5, ei.value                     # PE_ERCCL
        assert "PE_RCCL_TIMEOUT_S" in str(ei.value), str(ei.value)
        assert 1.5 < dt < 6.0, dt                                # the bound, not the 8 s stall
        assert e.comm_ranks() == 0                               # the communicator is gone
        t1 = time.monotonic()
        with pytest.raises(PlacementError) as ei2:
            e.place_batch(batch)
        assert ei2.value.code == -5 and "aborted" in str(ei2.value), ei2.value
        assert time.monotonic() - t1 < 1.0
        e.close()                                                # (joins the abort; the stall has drained)
    finally:
        for k in env:
            os.environ.pop(k, None)
    # the device is fine afterwards: a fresh context places the batch bit-exact
    e2 = Engine(0, world_size=1, comm=comm_id(), topk=8, window_groups=16)
    check_greedy(e2, inv, batch)
    e2.close()


@pytest.mark.parametrize("W", [17, 20])
def test_greedy_wide_host_exchange(W):
    """More ranks than the device merge and the zero-copy windows take (world > 16: several ranks per
    GPU): W shard contexts in one process over the native shared-memory exchange fall back to the
    copying all-gather and the host merge -- still the unsharded oracle's answer on every rank."""
    from placement import HostExchange
    inv = synth.make_inventory(4000, 97, 0.25)
    batch = synth.make_jobs(160, 101, "mixed")
    name = f"/pe_wide_{os.getpid()}_{W}"
    hxs = [HostExchange(name, r, W, 32 * (16 + 8 * 16)) for r in range(W)]
    engines = [Engine(0, rank=r, world_size=W, exchange=hxs[r], topk=16, window_groups=32) for r in range(W)]
    for e in engines:
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    results, errs = [None] * W, []

    def run(r):
        try:
            results[r] = engines[r].place_batch(batch)
        except Exception as ex:   # noqa: BLE001 -- reported below
            errs.append((r, ex))

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th) and not errs, errs
    w_pods, w_st, w_res = oracle.place_greedy(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                              batch.group_count, batch.group_req, batch.group_need)
    covered = 0
    for r in range(W):
        pods, st = results[r]
        np.testing.assert_array_equal(st, w_st)
        np.testing.assert_array_equal(pods, w_pods)
        b, en = engines[r].shard_range()
        covered += en - b
        np.testing.assert_array_equal(engines[r].read_residuals(), w_res[:, b:en])
        assert engines[r].stats()["xchg_zc_windows"] == 0
    assert covered == 4000
    for e in engines:
        e.close()
    for x in hxs:
        x.close()


def test_greedy_reset_residuals(eng):
    inv = synth.make_inventory(800, 59)
    batch = synth.make_jobs(60, 61)
    eng.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    a = eng.place_batch(batch)
    eng.reset_residuals()
    np.testing.assert_array_equal(eng.read_residuals(), inv.residual())
    b = eng.place_batch(batch)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_v2_total_requests_edge_cases(eng):
    """kueue pod formula corners (sidecar order, overhead, key union, zero keys) on the GPU, one
    batch, against hand-derived answers (tests/kueue_cases.py); replicas 3 scales every key."""
    from kueue_cases import CASES
    flat = F.Flat()
    for _, pod, _ in CASES:
        F.add_v2_pod_group(flat, 3, pod, GPU)
        flat.end_job(0)
    out, pres, mem, ovf = eng.pg_min_resources(V2, *flat.arrays())
    for j, (name, _, want) in enumerate(CASES):
        assert F.unflatten(out[j], pres[j], GPU) == {k: 3 * v for k, v in want.items()}, name
        assert mem[j] == 3 and ovf[j] == 0


@pytest.mark.parametrize("case", ["saturating", "over_committed", "low_bits"])
def test_greedy_score_corner_nodes(eng, case):
    """The scan's node-only score terms (K(n) = S(n) << 24 | gid, exact when no term saturates)
    against the oracle's direct Appendix-B key: nodes whose terms saturate take the full formula
    (huge cpu / memory / accelerator counts), over-committed nodes fit nothing, and requests whose
    low memory / ephemeral bits exceed the node's exercise the borrow terms."""
    N, J = 2500, 200
    inv = synth.make_inventory(N, 53, 0.3)
    batch = synth.make_jobs(J, 59, "mixed")
    if case == "saturating":
        inv.cap[0, ::97] = 1 << 41                     # left_cpu > SCORE_MAX
        inv.cap[2, 5::89] = 1 << 21                    # left_gpu << 20 would exceed 2^40
        inv.cap[1, 7::83] = 1 << 61                    # left_mem >> 20 > SCORE_MAX
        inv.cap[0, 9::79] = (1 << 40) - 2              # S(n) reaches SCORE_MAX
    elif case == "over_committed":
        inv.used[0, ::7] = inv.cap[0, ::7] + 1         # negative cpu residual
        inv.used[3, 3::11] = inv.cap[3, 3::11] + 5
    else:
        inv.cap[1] += np.arange(N, dtype=np.int64) * 4099        # odd memory bytes on every node
        inv.cap[3] += np.arange(N, dtype=np.int64) * 65537
        batch.group_req[:, 1] += (np.arange(len(batch.group_count)) % 7) * 131071
        batch.group_req[:, 3] += (np.arange(len(batch.group_count)) % 5) * 9_999_991
    check_greedy(eng, inv, batch)


@pytest.mark.parametrize("mix,N,J,topk,wg", [("mixed", 3000, 400, 64, 64), ("mixed", 1500, 300, 2, 8),
                                             ("gang8", 500, 150, 4, 16), ("pytorch", 2000, 300, 1, 1),
                                             ("island8", 600, 250, 2, 8)])
def test_greedy_pipelined_vs_sequential(mix, N, J, topk, wg):
    """The pipelined window loop (next window scanned while the host resolves the current one,
    the current window's changes seeded as dirty) against the sequential loop and the oracle --
    small K / windows force many discarded speculations (rescans) and cross-window rollbacks."""
    inv = synth.make_inventory(N, 61 + N, 0.4)
    batch = synth.make_jobs(J, 67 + J, mix)
    res = {}
    for flags in (1, 0):     # bit0: sequential windows (default: pipelined)
        e = Engine(0, topk=topk, window_groups=wg, greedy_flags=flags)
        res[flags] = check_greedy(e, inv, batch)
        e.close()
    np.testing.assert_array_equal(res[0], res[1])


@pytest.mark.parametrize("mix,N,J,topk,wg", [("mixed", 4000, 600, 64, 64), ("mixed", 2000, 400, 2, 8),
                                             ("island8", 800, 300, 4, 16), ("pytorch", 3000, 500, 1, 2)])
def test_greedy_signalled_windows(mix, N, J, topk, wg):
    """Pipelined walk windows are taken group by group as the device signals them (the resolver
    starts before the slowest block is done; PE_NO_GROUP_SIGNAL=1 waits for the whole launch):
    both equal the oracle, including small K / windows that discard speculative windows."""
    inv = synth.make_inventory(N, 97 + N, 0.35)
    batch = synth.make_jobs(J, 101 + J, mix)
    res = {}
    for sync in ("1", None):
        if sync:
            os.environ["PE_NO_GROUP_SIGNAL"] = sync
        try:
            e = Engine(0, topk=topk, window_groups=wg)
            res[sync] = check_greedy(e, inv, batch)
            e.place_batch(batch)   # a second batch on the same context: generations keep counting
            e.close()
        finally:
            os.environ.pop("PE_NO_GROUP_SIGNAL", None)
    np.testing.assert_array_equal(res["1"], res[None])


@pytest.mark.parametrize("mix,N,J,topk,wg,resort", [("mixed", 4000, 600, 64, 64, 0), ("mixed", 2000, 400, 2, 8, 0),
                                                    ("island8", 800, 300, 4, 16, 64), ("pytorch", 3000, 500, 1, 2, 16)])
def test_greedy_early_post(mix, N, J, topk, wg, resort):
    """The next window's apply + walk handed to the launch helper as soon as the current window landed
    (default) or after the next window's first group was seen (PE_EARLY_POST=0): both exact vs the
    oracle, identical -- small K / windows drop speculations and restart often, which rewinds the two
    update staging slots the early post rotates."""
    inv = synth.make_inventory(N, 131 + N, 0.35)
    batch = synth.make_jobs(J, 137 + J, mix)
    res = {}
    for ep in ("0", None):
        if ep:
            os.environ["PE_EARLY_POST"] = ep
        try:
            e = Engine(0, topk=topk, window_groups=wg, **({"resort_nodes": resort} if resort else {}))
            res[ep] = check_greedy(e, inv, batch)
            e.place_batch(batch)   # a second batch on the same context
            e.close()
        finally:
            os.environ.pop("PE_EARLY_POST", None)
    np.testing.assert_array_equal(res["0"], res[None])


@pytest.mark.parametrize("flags,resort", [(2, 0), (0, 1), (0, 64), (1, 16), (3, 0)])
@pytest.mark.parametrize("mix,N,J,gpu_frac,topk,wg", [("mixed", 3000, 300, 0.3, 64, 64), ("pytorch", 2500, 300, 0.2, 2, 8),
                                                       ("gang8", 700, 150, 1.0, 4, 16), ("mixed", 5000, 200, 0.5, 1, 1),
                                                       ("island8", 900, 300, 0.7, 4, 16)])
def test_greedy_walk_and_full_scan(flags, resort, mix, N, J, gpu_frac, topk, wg):
    """Both window paths against the oracle: the sorted walk (default; resort_nodes 1 rebuilds the
    sorted index after every applied window, 64 / 16 let the overlay grow across many windows) and
    the full scan + merge (greedy_flags bit1), pipelined (default) and sequential (bit0)."""
    e = Engine(0, topk=topk, window_groups=wg, greedy_flags=flags, resort_nodes=resort)
    inv = synth.make_inventory(N, 71 + N, gpu_frac)
    batch = synth.make_jobs(J, 73 + J, mix)
    check_greedy(e, inv, batch)
    s = e.stats()
    assert (s["resorts"] > 0) == (not flags & 2)
    assert (s["scan_evals"] > 0) == bool(flags & 2)
    if resort == 1 and not flags & 2:
        assert s["resorts"] > 1          # rebuilt during the batch, not only at its start
    e.close()


@pytest.mark.parametrize("resort", [1, 16, 64])
@pytest.mark.parametrize("mix,N,J,gpu_frac", [("mixed", 6000, 600, 0.3), ("island8", 1500, 400, 0.7)])
def test_greedy_walk_rebuild_in_line_and_side_stream(resort, mix, N, J, gpu_frac):
    """The walk index rebuilt in line (PE_ASYNC_RESORT=0) and on the side stream while the walks go on
    (default; and with the takeover held back 3 windows, PE_WALK_SWITCH_DELAY=3, so that updates are
    applied while a rebuild is pending -- the dual overlay writes and the switch's drop of the changed
    nodes' sorted entries): all exact vs the oracle, identical placements, the side-stream rebuilds
    taken over during the batch (resorts > 1), and with the delay, updates applied while pending."""
    inv = synth.make_inventory(N, 91 + N, gpu_frac)
    batch = synth.make_jobs(J, 93 + J, mix)
    out = {}
    for mode, delay in (("0", None), ("1", None), ("1", "3")):
        os.environ["PE_ASYNC_RESORT"] = mode
        if delay:
            os.environ["PE_WALK_SWITCH_DELAY"] = delay
        try:
            e = Engine(0, topk=16, window_groups=16, resort_nodes=resort)
            out[(mode, delay)] = check_greedy(e, inv, batch)
            s = e.stats()
            assert s["resorts"] > 1
            if delay:
                assert s["walk_pend_updates"] > 0, s
            e.close()
        finally:
            os.environ.pop("PE_ASYNC_RESORT", None)
            os.environ.pop("PE_WALK_SWITCH_DELAY", None)
    np.testing.assert_array_equal(out[("0", None)], out[("1", None)])
    np.testing.assert_array_equal(out[("0", None)], out[("1", "3")])


def test_greedy_walk_overlay_compaction():
    """Overlay larger than the LDS candidate buffer (every node updated, resort never triggers):
    the walk's in-loop compaction to the K + 1 smallest keeps the lists exact."""
    N = 20_000
    e = Engine(0, topk=64, resort_nodes=1 << 30)
    inv = synth.make_inventory(N, 83, 0.3)
    batch = synth.make_jobs(4000, 89, "mixed")
    check_greedy(e, inv, batch)
    s = e.stats()
    assert s["resorts"] == 1
    e.close()


def test_greedy_walk_long_walk_then_large_overlay():
    """A walk that collects > 8192 keys followed by an overlay with > 2048 fitting entries (advice r5):
    a homogeneous inventory makes every walk visit all of its rounds (equal node-only keys never fall
    below the stop bound), and 7000 nodes changed by phase 1 (one 1-GPU pod each, cpu 1 + i so the
    LATER-changed nodes are the tighter ones) are all in the overlay and all fit phase 2's cpu-only
    pods.  The overlay step's compaction must run before its appends, or the walk's 14000 keys + up
    to 8192 overlay keys overrun the 16384-key LDS buffer and drop some of the best keys."""
    from placement.synth import Inventory, JobBatch
    N, J1, J2 = 21_000, 7000, 300
    cap = np.zeros((4, N), np.int64)
    cap[0], cap[1], cap[2] = 100_000, 64 << 30, 1
    inv = Inventory(cap, np.zeros_like(cap), np.zeros(N, np.uint32), np.full(N, -1, np.int32))
    J = J1 + J2
    req = np.zeros((J, 4), np.int64)
    req[:J1, 0] = 1 + np.arange(J1)
    req[:J1, 2] = 1
    req[J1:, 0] = 1 + np.arange(J2) % 3
    batch = JobBatch(np.arange(J + 1, dtype=np.int32), np.r_[np.full(J1, 2), np.ones(J2)].astype(np.int32),
                     np.ones(J, np.int32), req, np.zeros(J, np.uint32), np.zeros(J, np.int8))
    e = Engine(0, resort_nodes=1 << 30)
    st = check_greedy(e, inv, batch)
    assert (st == 0).all()
    s = e.stats()
    assert s["resorts"] == 1                    # one index for the whole batch: the changed nodes stay overlaid
    e.close()


def test_greedy_unfittable_and_empty_lists():
    """Requests no node can hold (16 GPUs, more memory than any node, an unknown label) next to
    normal ones: their walks visit every candidate round and return empty lists with limit
    NO_KEY, the jobs fail all-or-nothing and roll back, exact vs the oracle."""
    inv = synth.make_inventory(6000, 101, 0.3)
    batch = synth.make_jobs(400, 103, "mixed")
    req = batch.group_req.copy()
    need = batch.group_need.copy()
    req[::7, 2] = 16                        # more GPUs than any node has
    req[3::11, 1] = 1 << 45                 # more memory than any node has
    need[5::13] |= 1 << 20                  # a label no node carries
    batch.group_req, batch.group_need = req, need
    e = Engine(0)
    st = check_greedy(e, inv, batch)
    assert (st == 1).sum() > 50 and (st == 0).sum() > 50
    e.close()


def test_greedy_topk_beyond_walk_uses_full_scan():
    """K + 1 > 1024 does not fit the walk's block: the windows take the full scan + merge."""
    e = Engine(0, topk=2000, window_groups=16)
    inv = synth.make_inventory(4000, 107, 0.3)
    batch = synth.make_jobs(200, 109, "mixed")
    check_greedy(e, inv, batch)
    s = e.stats()
    assert s["scan_evals"] > 0 and s["resorts"] == 0
    e.close()


def test_greedy_island_groups(eng):
    """Island groups (need bit 31): every pod of the group on one node that has an xGMI island,
    chosen for count x request; island-less nodes (CPU nodes, island -1) never take them even when
    they would fit; a summed request that overflows int64 fails the job; mixed with ordinary
    groups and multi-node gangs in one batch, bit-exact vs the oracle and the independent Python
    restatement."""
    from oracle import semantics as S
    inv = synth.make_inventory(400, 83, 0.5)
    batch = synth.make_jobs(160, 89, "island8")
    # a cpu-only island group (fits CPU nodes too, but only island nodes may take it) and an overflow
    g0 = int(batch.job_group_off[3])
    batch.group_req[g0] = [1000, 1 << 30, 0, 0]
    batch.group_count[g0] = 3
    batch.group_need[g0] = np.uint32(1 << 31)
    g1 = int(batch.job_group_off[5])
    batch.group_req[g1] = [1, 1 << 61, 0, 0]
    batch.group_count[g1] = 8
    batch.group_need[g1] = np.uint32(1 << 31)
    st = check_greedy(eng, inv, batch)
    py_pods, py_st, _ = S.place_greedy_appendix_b(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                                  batch.group_count, batch.group_req, batch.group_need)
    np.testing.assert_array_equal(st, py_st)
    assert st[5] == 1                                   # the overflowing island group fits nowhere
    eng.reset_residuals()
    got_pods, got_st = eng.place_batch(batch)
    np.testing.assert_array_equal(got_pods, py_pods)
    off = np.concatenate([[0], np.cumsum(batch.group_count)])
    for g in np.nonzero(batch.group_need >> 31)[0]:
        nodes = got_pods[off[g]:off[g + 1]]
        if len(nodes) and nodes[0] >= 0:
            assert (nodes == nodes[0]).all() and inv.island[nodes[0]] >= 0   # one island node
