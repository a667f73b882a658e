"""GPU parity of the LDS digit-plane fit path (pe_lds.hip) against the C oracle, bit-exact.

The path takes every batch that one register plane set cannot hold (more than 32 distinct
(dimension, value) pairs): per dimension a digit field of 1-3 levels, single-valued dimensions
folded into the need planes, one plane per distinct need (or per need and crossed single-level
field values).  Cases cover every block size W (2048,
4096, 8192 nodes per workgroup), every level count (four only at W >= 2), ragged last blocks, job counts around the
16-job batch and the phase interleave, int64 extremes, negative residuals, many needs, and shards."""
import os

import numpy as np
import pytest

import oracle
from placement import Engine, synth

pytestmark = pytest.mark.gpu
LDS_ONLY = 64          # pe_config.fit_path_mask: LDS digit planes (int64 compare stays as the fallback)


def batch(shape, J, seed):
    rng = np.random.default_rng(seed)
    req, need = synth.make_fit_jobs(J, seed)
    if shape == "cpu400":
        req[:, 0] = 500 + (np.arange(J) % 400) * 7
    elif shape == "unique_mem":
        req[:, 1] = (1 << 30) + rng.permutation(J) * 4096 + 1              # odd byte counts too
    elif shape == "wide":                                                 # every dimension many-valued
        req[:, 0] = rng.integers(1, 1000, J) * 100
        req[:, 1] = rng.integers(1, 5000, J) * (1 << 24)
        req[:, 2] = rng.integers(0, 9, J)
        req[:, 3] = rng.integers(0, 300, J) * (1 << 30)
        need[:] = (rng.integers(0, 16, J).astype(np.uint32) << 1) | (req[:, 2] > 0)
    elif shape == "adversarial":                                          # cpu, mem, eph unique per job
        req[:, 0] = 1 + rng.permutation(J)
        req[:, 1] = (1 << 20) * (1 + rng.permutation(J))
        req[:, 3] = 7 * rng.permutation(J)
    elif shape == "single":                                               # one value per dimension
        req[:] = [2000, 8 << 30, 0, 10 << 30]
        need[:] = 0
    elif shape == "needs":                                                # 40 distinct label needs
        req[:, 0] = 100 * (1 + np.arange(J) % 50)
        need[:] = (np.arange(J) % 40).astype(np.uint32) << 1
    elif shape == "extremes":
        req[:, 0] = 100 * (1 + np.arange(J) % 60)
        req[0] = [np.iinfo(np.int64).max, 0, 0, 0]
        req[1] = [0, np.iinfo(np.int64).max, 0, np.iinfo(np.int64).max]
        req[2] = [0, 0, 0, 0]
    return req, need


def inventory(N, seed, gpu_frac=0.4):
    inv = synth.make_inventory(N, seed, gpu_frac)
    inv.labels |= (np.arange(N, dtype=np.uint32) * 2654435761 % 31).astype(np.uint32) << 1   # varied label sets
    inv.cap[1, ::7] = 1 << 50
    inv.used[0, 3::11] = inv.cap[0, 3::11] + 1000                                      # negative residuals
    return inv


def run(inv, req, need, W=None, maxl=None, fit_path_mask=LDS_ONLY, rank=0, world=1, env=None):
    env = dict(env or {})
    if W is not None:
        env["PE_LDS_W"] = str(W)
    if maxl is not None:
        env["PE_LDS_MAXL"] = str(maxl)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e = Engine(0, fit_path_mask=fit_path_mask, rank=rank, world_size=world,
                   exchange=(lambda b: b * world) if world > 1 else None)
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        counts = e.fit_mask(req, need)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return e, counts


def check(e, counts, inv, req, need):
    b, en = e.shard_range()
    o_mask, o_counts = oracle.fit_mask(inv.residual()[:, b:en], inv.labels[b:en], req, need)
    J = len(req)
    np.testing.assert_array_equal(counts, o_counts)
    np.testing.assert_array_equal(e.fit_mask_rows(0, J), o_mask)
    s = e.stats()
    assert s["fit_runs_lds"] == 1, s
    assert e.fit_mask_layout() == 3
    assert e.fit_mask_row_pitch() * 64 >= en - b
    return o_counts


@pytest.mark.parametrize("W", [1, 2, 4])
@pytest.mark.parametrize("shape", ["cpu400", "unique_mem", "wide", "adversarial", "needs", "extremes"])
def test_lds_shapes_vs_oracle(shape, W):
    N, J = 20011, 1500
    inv = inventory(N, 5 + W)
    req, need = batch(shape, J, 11 + W)
    e, counts = run(inv, req, need, W=W)
    check(e, counts, inv, req, need)
    assert 0 < counts.sum() < N * J
    e.close()


@pytest.mark.parametrize("maxl", [1, 2, 3, 4])
def test_lds_level_counts(maxl):
    """The same batch through single-level, two-level and three-level digit fields (150 cpu, 150
    memory, 100 ephemeral values: ~410 planes at one level, which only the 2048-node blocks hold)."""
    N, J = 9000, 700
    inv = inventory(N, 21)
    rng = np.random.default_rng(23)
    req, need = synth.make_fit_jobs(J, 23)
    req[:, 0] = rng.integers(1, 151, J) * 100
    req[:, 1] = rng.integers(1, 151, J) * (1 << 26)
    req[:, 3] = rng.integers(0, 100, J) * (1 << 30)
    need[:] = (rng.integers(0, 8, J).astype(np.uint32) << 1) | (req[:, 2] > 0)
    e, counts = run(inv, req, need, maxl=maxl)
    check(e, counts, inv, req, need)
    e.close()


@pytest.mark.parametrize("W,dims", [(2, (0, 1, 3)), (4, (0, 1))])
def test_lds_four_level_fields(W, dims, capfd):
    """Fields that only four digit levels fit into LDS: 60k values unique per job in each of `dims`
    (three fields at 4096-node blocks, two at 8192; at three levels they need ~120 planes each, more
    than the block's budget) -- the four-level kernels, bit-exact, on a ragged last block."""
    N, J = 6001, 60000
    inv = inventory(N, 71 + W)
    rng = np.random.default_rng(73 + W)
    req, need = synth.make_fit_jobs(J, 73 + W)
    scale = {0: 1, 1: 1 << 20, 3: 7}
    for d in dims:
        req[:, d] = scale[d] * (1 + rng.permutation(J))
    os.environ["PE_LDS_DEBUG"] = "1"
    try:
        e, counts = run(inv, req, need, W=W)
    finally:
        os.environ.pop("PE_LDS_DEBUG", None)
    check(e, counts, inv, req, need)
    plan = capfd.readouterr().err            # the engine's PE_LDS_DEBUG line: "lds: W w ... L l B b" per field
    assert f"lds: W {W} " in plan and " L 4 " in plan, plan
    assert 0 < counts.sum() < N * J
    e.close()


@pytest.mark.parametrize("cross", ["1", "0"])
@pytest.mark.parametrize("case", ["gpu_eph", "three", "many_needs", "all_crossed"])
def test_lds_crossed_fields(case, cross, capfd):
    """Single-level fields crossed into the need planes (one plane per need and crossed values, so a
    job reads one plane for its labels and those fields) -- and the same batch with nothing crossed
    (PE_LDS_CROSS=0): both bit-exact, and the plan says how many fields were crossed."""
    N, J = 12289, 2000
    inv = inventory(N, 81)
    rng = np.random.default_rng(83)
    req, need = synth.make_fit_jobs(J, 83)
    req[:, 0] = 500 + (np.arange(J) % 300) * 11                  # a digit field
    req[:, 2] = rng.choice([0, 1, 2, 4, 8], J)                    # 5 values
    req[:, 3] = rng.choice([0, 10, 50, 100], J) * (1 << 30)       # 4 values
    need[:] = (rng.integers(0, 3, J).astype(np.uint32) << 1) | (req[:, 2] > 0)
    if case == "three":                                           # memory too: 3 values
        req[:, 1] = rng.choice([1, 8, 64], J) * (1 << 30)
    elif case == "many_needs":                                    # 24 needs x the crossed values
        need[:] = (rng.integers(0, 12, J).astype(np.uint32) << 1) | (req[:, 2] > 0)
    elif case == "all_crossed":                                   # no digit field left (shape 0,0,0,0)
        req[:, 0] = 1500
        req[:, 1] = 4 << 30
    e, counts = run(inv, req, need, env={"PE_LDS_CROSS": cross, "PE_LDS_DEBUG": "1"})
    check(e, counts, inv, req, need)
    plan = capfd.readouterr().err
    ncross = int(plan.split(" cross ")[1].split()[0])
    if cross == "0":
        assert ncross == 0, plan
    elif case != "many_needs":    # (24 needs: crossing would cost the second workgroup per CU -> planner's call)
        assert ncross >= 1, plan
    assert 0 < counts.sum() < N * J
    e.close()


@pytest.mark.parametrize("N,J", [(1, 1), (63, 17), (2048, 16), (2049, 15), (8191, 33), (8193, 257),
                                 (40961, 4097), (70000, 64)])
def test_lds_ragged_sizes(N, J):
    """Ragged last node blocks (padding bits 0), job counts around the 16-job batch and the phases."""
    inv = inventory(N, 31 + N % 97)
    req, need = batch("cpu400", J, 37 + J)
    e, counts = run(inv, req, need)
    check(e, counts, inv, req, need)
    np.testing.assert_array_equal(e.fit_mask_rows(J - 1, 1), e.fit_mask_rows(0, J)[J - 1:])
    e.close()


def test_lds_single_valued_dims_fold():
    """Every dimension single-valued (nothing but folded conditions and one need plane): still exact,
    including nodes whose residual is negative in a folded dimension."""
    N, J = 5000, 300
    inv = inventory(N, 41)
    req, need = batch("single", J, 43)
    need[::3] = 1
    e, counts = run(inv, req, need)
    check(e, counts, inv, req, need)
    e.close()


def test_lds_is_default_for_many_values_and_reruns():
    """With every path allowed a many-valued batch lands on the LDS path; a second run over the same
    upload (counts re-zeroed, planes rebuilt) gives the same result, and a run after an inventory
    update sees the new residuals."""
    N, J = 30000, 2000
    inv = inventory(N, 51)
    req, need = batch("unique_mem", J, 53)
    e, counts = run(inv, req, need, fit_path_mask=0)
    want = check(e, counts, inv, req, need)
    e.fit_mask_run()
    np.testing.assert_array_equal(e.fit_counts(), want)
    slots = np.arange(0, N, 97, dtype=np.int64)
    cap = inv.cap[:, slots].T.copy()
    used = cap // 2
    e.update_nodes(slots, np.zeros(len(slots), np.uint8), cap, used, inv.labels[slots], inv.island[slots])
    inv.used[:, slots] = used.T
    e.fit_mask_run()
    _, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    np.testing.assert_array_equal(e.fit_counts(), o_counts)
    e.close()


def test_lds_sharded_columns():
    """Three shard contexts of one inventory: their column blocks are the unsharded oracle mask's."""
    N, J = 50001, 900
    inv = inventory(N, 61)
    req, need = batch("wide", J, 63)
    _, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req, need)
    total = np.zeros(J, np.int64)
    for rank in range(3):
        e, counts = run(inv, req, need, rank=rank, world=3)
        check(e, counts, inv, req, need)
        total += counts
        e.close()
    np.testing.assert_array_equal(total, o_counts)


@pytest.mark.parametrize("unique", [(1,), (0, 1, 3)])
def test_lds_full_size_worst_case(unique):
    """cfg5 at full size (1M nodes x 100k jobs) with memory unique per job (the bench's worst batch) or
    cpu, memory and ephemeral-storage unique per job (its adversarial batch: four-level fields and a
    crossed gpu field): sampled rows exact vs the oracle, counts == popcount(rows), the whole count
    vector equal to the int64 compare path's."""
    inv = synth.make_inventory(1_000_000, synth.SEED["cfg5"], 0.2)
    req, need = synth.make_fit_jobs_worst(100_000, synth.SEED["cfg5"], unique)
    e, counts = run(inv, req, need, fit_path_mask=0)
    assert e.stats()["fit_runs_lds"] == 1
    rng = np.random.default_rng(3)
    rows = np.sort(rng.choice(100_000, 24, replace=False))
    o_mask, o_counts = oracle.fit_mask(inv.residual(), inv.labels, req[rows], need[rows])
    for i, r in enumerate(rows):
        m = e.fit_mask_rows(int(r), 1)
        np.testing.assert_array_equal(m[0], o_mask[i])
        assert np.unpackbits(m.view(np.uint8)).sum() == counts[r] == o_counts[i]
    e.close()
    ref, ref_counts = run(inv, req, need, fit_path_mask=1)            # int64 compare kernel
    assert ref.stats()["fit_runs_i64"] == 1
    np.testing.assert_array_equal(ref_counts, counts)
    ref.close()
