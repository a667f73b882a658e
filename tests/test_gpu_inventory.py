"""pe_update_nodes: Node informer deltas scattered into the device
inventory.  The expected inventory is computed here with numpy from the ABI's documented
semantics (last entry per slot wins; SET: residual = cap - used, labels/island replaced, also the
reset snapshot; REMOVE: the slot never fits), then fit mask and greedy are compared with the oracle
on that inventory."""
import numpy as np
import pytest

import oracle
from placement import PE_NODE_REMOVE, PE_NODE_SET, Engine, PlacementError, synth

pytestmark = pytest.mark.gpu

NEVER = np.iinfo(np.int64).min


def make_deltas(n_nodes, n_upd, seed):
    """Random SET/REMOVE batch with repeated slots (SET -> REMOVE -> SET chains)."""
    rng = np.random.default_rng(seed)
    donor = synth.make_inventory(n_upd, seed + 1, 0.5)
    slots = rng.integers(0, n_nodes, n_upd)
    slots[n_upd // 2:n_upd // 2 + 20] = slots[:20]          # repeats: later entries must win
    op = np.where(rng.random(n_upd) < 0.2, PE_NODE_REMOVE, PE_NODE_SET).astype(np.uint8)
    cap = np.ascontiguousarray(donor.cap.T)
    used = np.ascontiguousarray(donor.used.T)
    labels = donor.labels.copy()
    island = rng.integers(-1, 50, n_upd).astype(np.int32)
    return slots, op, cap, used, labels, island


def apply_host(res, labels, island, deltas):
    slots, op, cap, used, lab, isl = deltas
    res, labels, island = res.copy(), labels.copy(), island.copy()
    for i in range(len(slots)):
        s = slots[i]
        if op[i] == PE_NODE_SET:
            res[:, s] = cap[i] - used[i]
            labels[s] = lab[i]
            island[s] = isl[i]
        else:
            res[:, s] = NEVER
            labels[s] = 0
            island[s] = -1
    return res, labels, island


def test_update_nodes_fit_greedy_and_snapshot():
    N = 5000
    inv = synth.make_inventory(N, 41, 0.3)
    deltas = make_deltas(N, 700, 43)
    w_res, w_lab, _ = apply_host(inv.residual(), inv.labels, inv.island, deltas)
    e = Engine(0)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    e.update_nodes(*deltas)
    np.testing.assert_array_equal(e.read_residuals(), w_res)
    req, need = synth.make_fit_jobs(300, 47)
    counts = e.fit_mask(req, need)
    o_mask, o_counts = oracle.fit_mask(w_res, w_lab, req, need)
    np.testing.assert_array_equal(e.fit_mask_rows(0, 300), o_mask)
    np.testing.assert_array_equal(counts, o_counts)
    batch = synth.make_jobs(200, 49, "mixed")
    pods, st = e.place_batch(batch)
    w_pods, w_st, w_after = oracle.place_greedy(w_res, w_lab, batch.job_group_off, batch.priority, batch.group_count,
                                                batch.group_req, batch.group_need)
    np.testing.assert_array_equal(pods, w_pods)
    np.testing.assert_array_equal(st, w_st)
    np.testing.assert_array_equal(e.read_residuals(), w_after)
    last_op = {int(s): int(o) for s, o in zip(deltas[0], deltas[1])}
    removed = [s for s, o in last_op.items() if o == PE_NODE_REMOVE]
    assert removed and not np.any(np.isin(pods, removed))   # nothing lands on an emptied slot
    e.reset_residuals()                                      # snapshot = the updated inventory
    np.testing.assert_array_equal(e.read_residuals(), w_res)
    e.close()


def test_update_after_placement_overrides_placed_residual():
    N = 2000
    inv = synth.make_inventory(N, 51, 0.2)
    e = Engine(0)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    batch = synth.make_jobs(100, 53, "mixed")
    pods, _ = e.place_batch(batch)
    after = e.read_residuals()
    touched = np.unique(pods[pods >= 0])[:10]
    cap = np.full((len(touched), 4), 1000, np.int64)
    used = np.zeros_like(cap)
    e.update_nodes(touched, np.zeros(len(touched), np.uint8), cap, used)
    got = e.read_residuals()
    np.testing.assert_array_equal(got[:, touched], 1000)
    keep = np.setdiff1d(np.arange(N), touched)
    np.testing.assert_array_equal(got[:, keep], after[:, keep])   # placements elsewhere are untouched
    e.close()


def test_update_nodes_sharded_owner_applies():
    N = 3001
    inv = synth.make_inventory(N, 61, 0.3)
    deltas = make_deltas(N, 400, 63)
    w_res, _, _ = apply_host(inv.residual(), inv.labels, inv.island, deltas)
    for r in range(2):
        e = Engine(0, rank=r, world_size=2, exchange=lambda b: b + b)
        e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
        e.update_nodes(*deltas)
        b, en = e.shard_range()
        np.testing.assert_array_equal(e.read_residuals(), w_res[:, b:en])
        e.close()


@pytest.mark.parametrize("bad", ["slot", "op", "negative"])
def test_update_nodes_rejects_whole_batch(bad):
    N = 1000
    inv = synth.make_inventory(N, 71)
    e = Engine(0)
    e.load_nodes(inv.cap, inv.used, inv.labels, inv.island)
    slots, op, cap, used, labels, island = make_deltas(N, 50, 73)
    if bad == "slot":
        slots[-1] = N
    elif bad == "op":
        op[-1] = 7
    else:
        op[-1] = PE_NODE_SET
        cap[-1, 2] = -1
    before = e.read_residuals()
    with pytest.raises(PlacementError, match="PE_EINVAL"):
        e.update_nodes(slots, op, cap, used, labels, island)
    np.testing.assert_array_equal(e.read_residuals(), before)   # nothing applied
    e.close()
