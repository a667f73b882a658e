"""Two independent restatements of the build-defined placement rule agree:
the plain-Python sequential greedy in oracle/semantics.py and the C oracle (oracle.c) that the GPU
parity tests use -- keys, chosen nodes, all-or-nothing rollback and residuals, bit for bit."""
import numpy as np
import pytest

import oracle
from oracle import semantics as S
from placement import synth


def corner_inventory(N, seed):
    inv = synth.make_inventory(N, seed, 0.4)
    rng = np.random.default_rng(seed)
    inv.cap[0, ::9] = (1 << 41) + rng.integers(0, 1 << 20, len(inv.cap[0, ::9]))   # saturating cpu term
    inv.cap[1, 1::11] = (1 << 62)                                                  # huge memory
    inv.cap[2, 2::13] = (1 << 21)                                                  # gpu term saturates
    inv.used[0, 3::7] = inv.cap[0, 3::7] + 5                                       # over-committed
    inv.cap[1, 4::5] += rng.integers(0, 1 << 20, len(inv.cap[1, 4::5]))            # odd low bits
    return inv


@pytest.mark.parametrize("mix,gpu_frac", [("pytorch", 0.2), ("mixed", 0.3), ("gang8", 1.0), ("island8", 0.7)])
@pytest.mark.parametrize("seed", [1, 2])
def test_python_greedy_matches_c_oracle(mix, gpu_frac, seed):
    N, J = 120, 30
    inv = synth.make_inventory(N, 40 + seed, gpu_frac)
    batch = synth.make_jobs(J, 50 + seed, mix)
    want = oracle.place_greedy(inv.residual(), inv.labels, batch.job_group_off, batch.priority, batch.group_count,
                               batch.group_req, batch.group_need)
    pods, st, res = S.place_greedy_appendix_b(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                              batch.group_count, batch.group_req, batch.group_need)
    np.testing.assert_array_equal(np.array(st), want[1])
    np.testing.assert_array_equal(np.array(pods), want[0])
    np.testing.assert_array_equal(np.array(res, dtype=np.int64), want[2])
    assert 0 < sum(1 for s in st if s == 0) <= J


def test_python_greedy_corner_nodes():
    N, J = 90, 25
    inv = corner_inventory(N, 7)
    batch = synth.make_jobs(J, 8, "mixed")
    want = oracle.place_greedy(inv.residual(), inv.labels, batch.job_group_off, batch.priority, batch.group_count,
                               batch.group_req, batch.group_need)
    got = S.place_greedy_appendix_b(inv.residual(), inv.labels, batch.job_group_off, batch.priority,
                                    batch.group_count, batch.group_req, batch.group_need)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(np.array(a, dtype=np.int64), np.asarray(b, dtype=np.int64))


def test_keys_agree_on_corner_values():
    inv = corner_inventory(200, 3)
    res = inv.residual()
    req, need = synth.pod_requests(9, 700, 40)
    req[0] = [0, 0, 0, 0]
    req[1] = [1, 1 << 20, 1, 1 << 24]
    for j in range(len(req)):
        for n in range(0, 200, 3):
            k = S.appendix_b_key(res[:, n], int(inv.labels[n]), req[j], int(need[j]), n)
            o = oracle.key(res[:, n], inv.labels[n], req[j], need[j], n)
            assert (0xFFFFFFFFFFFFFFFF if k is None else k) == o, (j, n)


def test_total_replicas_wraps_like_go_int32():
    assert S.get_total_replicas({"Master": {"replicas": 2**31 - 1}, "Worker": {}}) == -2**31
    assert S.get_total_replicas({"A": {"replicas": 3}, "B": {"replicas": None}}) == 4
