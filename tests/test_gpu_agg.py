"""pe_pg_min_resources call path (round 3): the batch is packed into <= 256-job segments in pinned
host memory and each block stages its segment in LDS over PCIe (pe_kernels.h AggSegHdr); a one-segment
call waits on a flag in pinned memory instead of a stream sync.  Parity vs the C oracle
(oracle/oracle.c orc_pg_min_resources, a restatement of util.go:108-145 / coscheduling.go:108-118)
across segment boundaries, oversized segments read in place, the flag path and the r2 device path."""

import numpy as np
import pytest

import oracle
from placement import V1, V2, Engine
from test_gpu_parity import random_csr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = Engine(0, gpu_resource_name="nvidia.com/gpu")
    yield e
    e.close()


def _check(eng, mode, arrs):
    got = eng.pg_min_resources(mode, *arrs)
    want = oracle.pg_min_resources(mode, *arrs)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("mode", [V1, V2])
@pytest.mark.parametrize("J", [1, 2, 17, 32, 33, 255, 256, 257, 511, 1000, 8192, 8193, 33000, 70001])
def test_agg_segment_sizes(eng, mode, J):
    """Up to 8192 jobs: 32-job segments in one launch whose last block stores the flag (one block up to
    32 jobs); above: 256-job segments, chunked, stream sync; 33k+ jobs take the multi-range planner."""
    _check(eng, mode, random_csr(J, 100 + J + mode, big=(J % 2 == 1)))


@pytest.mark.parametrize("seg_jobs", ["1", "7", "64", "256"])
def test_agg_segment_jobs_override(eng, monkeypatch, seg_jobs):
    """PE_AGG_SEG_JOBS (A/B knob): any segment size gives the same answers, on both call paths."""
    monkeypatch.setenv("PE_AGG_SEG_JOBS", seg_jobs)
    for J in (1, 300, 9000, 40000):   # (40000: the chunked multi-thread path, staging sized from a bound)
        _check(eng, V1, random_csr(J, 700 + J))


def _one_job_csr(n_groups, n_cont_per_group, seed):
    rng = np.random.default_rng(seed)
    jgo = np.array([0, n_groups], np.int32)
    rep = rng.integers(-1, 5, n_groups).astype(np.int32)
    gco = (np.arange(n_groups + 1) * n_cont_per_group).astype(np.int32)
    C = int(gco[-1])
    req = rng.integers(0, 2**30, (C, 4), dtype=np.int64)
    fl = (rng.integers(0, 16, C) | (rng.integers(0, 4, C) << 4)).astype(np.uint8)
    mm = np.array([int(rep.clip(0).sum()) // 2 + 1], np.int32)
    return jgo, mm, rep, gco, req, fl


def _concat(parts):
    """CSR batches back to back."""
    jgo, mm, rep, gco, req, fl = [np.zeros(1, np.int32)], [], [], [np.zeros(1, np.int32)], [], []
    g_off = c_off = 0
    for p in parts:
        jgo.append(p[0][1:] + g_off)
        mm.append(p[1])
        rep.append(p[2])
        gco.append(p[3][1:] + c_off)
        req.append(p[4].reshape(-1, 4))
        fl.append(p[5])
        g_off += int(p[0][-1])
        c_off += int(p[3][-1])
    return (np.concatenate(jgo).astype(np.int32), np.concatenate(mm).astype(np.int32),
            np.concatenate(rep).astype(np.int32), np.concatenate(gco).astype(np.int32),
            np.concatenate(req).astype(np.int64), np.concatenate(fl).astype(np.uint8))


@pytest.mark.parametrize("mode", [V1, V2])
def test_agg_oversized_segments(eng, mode):
    """A job whose groups and containers exceed one segment's LDS budget (48 KB) is read in place,
    alone or between ordinary jobs; also a job with thousands of groups."""
    big_c = _one_job_csr(4, 600, 1)            # 2400 containers x 33 B > 48 KB
    big_g = _one_job_csr(9000, 0, 2)           # 9000 groups, no containers
    for arrs in (big_c, big_g, _concat([random_csr(300, 3), big_c, random_csr(10, 4), big_g, random_csr(600, 5)])):
        _check(eng, mode, arrs)


@pytest.mark.parametrize("mode", [V1, V2])
def test_agg_chunked_batch_with_oversized_jobs(eng, mode):
    """Batches above 32k jobs are planned, packed and DMA'd chunk by chunk (the staging sized from a
    bound before the first chunk is planned): oversized jobs inside and between chunks, and a batch
    of mostly oversized jobs (the most segments per byte the bound allows for)."""
    big_c = _one_job_csr(4, 600, 11)
    big_g = _one_job_csr(9000, 0, 12)
    _check(eng, mode, _concat([random_csr(40000, 13), big_c, random_csr(20000, 14), big_g, big_c,
                               random_csr(30000, 15, big=True)]))
    _check(eng, mode, _concat([big_c] * 40 + [random_csr(33000, 16)] + [big_c] * 40))


def test_agg_alternating_calls(eng):
    """Small (flag) and large (stream sync) calls interleaved: buffers grow and are reused, flag
    generations advance."""
    for i in range(30):
        J = [1, 5000, 3, 256, 100000][i % 5]
        _check(eng, V1 if i % 2 else V2, random_csr(J, 500 + i))


def test_agg_device_path_ab(eng, monkeypatch):
    """PE_AGG_DEVICE=1 (the r2 call path, kept for A/B) still agrees with the oracle."""
    monkeypatch.setenv("PE_AGG_DEVICE", "1")
    for J in (1, 300, 20000):
        _check(eng, V1, random_csr(J, 900 + J))
        _check(eng, V2, random_csr(J, 901 + J, big=True))


@pytest.mark.parametrize("no_karg", ["", "1"])
def test_agg_small_calls_both_paths(eng, monkeypatch, no_karg):
    """A one-segment call of <= 512 B travels in the kernel arguments (pg_agg_karg_kernel); with
    PE_AGG_NO_KARG=1 it is staged from pinned memory.  Both agree with the oracle, including a
    segment just under and just over the argument limit (one job of 12 / 13 containers)."""
    if no_karg:
        monkeypatch.setenv("PE_AGG_NO_KARG", "1")
    for J in (1, 2, 5, 13, 20, 32):
        for mode in (V1, V2):
            _check(eng, mode, random_csr(J, 300 + J + mode))
    for n_cont in (1, 10, 12, 13, 60):   # one job, n_cont containers x 33 B around the limit
        _check(eng, V1, _one_job_csr(1, n_cont, n_cont))


@pytest.mark.parametrize("mode", [V1, V2])
def test_agg_resync_batch_equals_per_object_calls(eng, mode):
    """The adapters' batch entry points (Go PGMinResourcesBatch / EngineCoScheduling.BuildBatch, C++
    kf::CalcPGMinResourcesBatch / CoScheduling::BuildBatch): one-object CSRs appended back to back
    (hip.CSR.AppendJobs; _concat here) and aggregated in ONE call give, job for job, what the
    per-object calls (J = 1, the reconcile path) and the oracle give.  3000 objects: above the
    crossover (bench aggregation.crossover_jobs)."""
    parts = [random_csr(1, 5000 + i + 17 * mode, big=(i % 7 == 0)) for i in range(3000)]
    batch = _concat(parts)
    got = eng.pg_min_resources(mode, *batch)
    want = oracle.pg_min_resources(mode, *batch)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    for i in range(0, 3000, 97):   # the per-object calls agree job for job
        one = eng.pg_min_resources(mode, *parts[i])
        for a, b in zip(one, got):
            np.testing.assert_array_equal(a[0], b[i])


# ------------------------------------------------------------------ key tables (ABI 7)

def random_keys_csr(J, n_keys, seed, big=False):
    """random_csr's structure with n_keys values per container and u32 flags (presence bits of the
    n_keys keys | kind << 16)."""
    jgo, mm, rep, gco, _, fl8 = random_csr(J, seed, big)
    rng = np.random.default_rng(seed + 1)
    C = int(gco[-1])
    hi = 2**62 if big else 2**40
    req = rng.integers(0, hi, (C, n_keys), dtype=np.int64)
    req[rng.random((C, n_keys)) < 0.3] = 0
    pres = rng.integers(0, 1 << n_keys, C, dtype=np.int64).astype(np.uint32)
    fl = pres | ((fl8.astype(np.uint32) >> 4) << 16)
    return jgo, mm, rep, gco, req, fl


def _check_keys(eng, mode, arrs):
    got = eng.pg_min_resources_keys(mode, *arrs)
    want = oracle.pg_min_resources_keys(mode, *arrs)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    return got


@pytest.mark.parametrize("n_keys", [1, 3, 4, 5, 8, 9, 13, 16])
@pytest.mark.parametrize("J", [1, 20, 300, 9000, 40000])
def test_agg_keys_random_vs_oracle(eng, n_keys, J):
    """pe_pg_min_resources_keys for every kernel width (4 / 8 / 16 keys, narrower tables padded) on
    every call path (kernel arguments, one latency launch, chunked batches, the multi-range planner),
    random values incl. int64 overflow, bit-exact vs orc_pg_min_resources_keys."""
    for mode in (V1, V2):
        _check_keys(eng, mode, random_keys_csr(J, n_keys, 40 + J + n_keys + mode, big=(J % 2 == 0)))


def test_agg_keys_equal_fixed_dims(eng):
    """A 4-key table with the fixed dimensions' values gives exactly pe_pg_min_resources' answers."""
    for mode in (V1, V2):
        jgo, mm, rep, gco, req, fl8 = random_csr(5000, 77 + mode, big=True)
        fl = (fl8.astype(np.uint32) & 15) | ((fl8.astype(np.uint32) >> 4) << 16)
        a = eng.pg_min_resources(mode, jgo, mm, rep, gco, req, fl8)
        b = eng.pg_min_resources_keys(mode, jgo, mm, rep, gco, req, fl)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


def test_agg_keys_rejects_bad_flags(eng):
    from placement import PlacementError
    jgo, mm, rep, gco, req, fl = random_keys_csr(50, 5, 3)
    fl = fl.copy()
    fl[7] |= 1 << 5                 # a presence bit past n_keys
    with pytest.raises(PlacementError) as ei:
        eng.pg_min_resources_keys(V1, jgo, mm, rep, gco, req, fl)
    assert ei.value.code == -1 and "cont_flags[7]" in str(ei.value)
    with pytest.raises(PlacementError):
        eng.pg_min_resources_keys(V1, jgo, mm, rep, gco, np.zeros((len(fl), 17), np.int64), fl & 0xFFFF0000)


def test_agg_keys_wide_golden(eng, golden_dir):
    """wide_keys.json on the GPU (verdict r5 item 2): hugepages-2Mi / -1Gi, rdma/hca, nvidia.com/gpu +
    amd.com/gpu, cpu in micro-cores, 21 keys over two 16-key slices, and the overflow case -- every
    answer exact (per-key scales), only the overflow case flagged, bit-exact vs the C oracle."""
    import json
    import os

    import wide_keys as W
    with open(os.path.join(golden_dir, "wide_keys.json")) as f:
        g = json.load(f)
    for mode, cases, flat in ((W.V1, g["v1"], W.v1_flat(g["v1"])), (W.V2, g["v2"], W.v2_flat(g["v2"]))):
        res, members, ovf, raw = W.run(eng.pg_min_resources_keys, mode, flat)
        for arrs, out in raw:
            for a, b in zip(out, oracle.pg_min_resources_keys(mode, *arrs)):
                np.testing.assert_array_equal(a, b)
        for j, case in enumerate(cases):
            want = case["want"] if mode == W.V1 else case["want"]["minResources"]
            assert ovf[j] == int(case.get("overflow", False)), case["name"]
            if not ovf[j]:
                assert W.same(res[j], W.want_list(want)), (case["name"], res[j])


def narrow_values(rng, shape, span_bits, p_zero=0.3):
    """Request values as canonical quantities come: per key a common power-of-two factor (2^0..2^30) times
    an integer below 2^span_bits -- a segment's key narrows to 32 bits exactly when its values span <= 32
    bits above their common trailing zeros."""
    sh = rng.integers(0, 31, shape[1])
    v = rng.integers(0, 2**span_bits, shape, dtype=np.int64) << sh
    v[rng.random(shape) < p_zero] = 0
    return v


@pytest.mark.parametrize("mode", [V1, V2])
@pytest.mark.parametrize("J", [1, 300, 9000, 40000])
def test_agg_narrowed_requests(eng, mode, J):
    """The packed segments carry their requests narrowed (value >> per-key shift in 32 bits) when every
    key of the segment allows it: values spanning exactly 32 bits, keys that are zero throughout, and
    segments one 33-bit value keeps wide, on every call path, bit-exact vs the oracle; the chunked path
    reports narrowed segments in pe_stats."""
    rng = np.random.default_rng(900 + J + mode)
    jgo, mm, rep, gco, _, fl = random_csr(J, 910 + J + mode)
    C = int(gco[-1])
    req = narrow_values(rng, (C, 4), 32)
    req[:, 3] = 0                                        # a key absent from every container
    if C > 0:
        req[:: max(1, C // 7), 1] = (2**32) << 5         # 33 bits above the shift: that segment stays wide
        req[0, 0] = (2**32 - 1) << 29                    # exactly 32 bits
    eng.reset_stats()
    _check(eng, mode, (jgo, mm, rep, gco, req, fl))
    st = eng.stats()
    if J > 8192:
        assert st["agg_narrow_segments"] > 0 and st["agg_narrow_segments"] < st["agg_segments"], st
        assert 0 < st["agg_wire_bytes"]


@pytest.mark.parametrize("n_keys", [1, 4, 5, 9, 16])
def test_agg_keys_narrowed(eng, n_keys):
    """Key tables (4 / 8 / 16-wide kernels) with narrowable values, and with a span of 33 bits."""
    for span, J in ((32, 40000), (33, 9000), (20, 300)):
        arrs = list(random_keys_csr(J, n_keys, 60 + n_keys + span))
        rng = np.random.default_rng(70 + n_keys + span)
        arrs[4] = narrow_values(rng, arrs[4].shape, span)
        for mode in (V1, V2):
            _check_keys(eng, mode, tuple(arrs))


def test_agg_realistic_batch_narrowed(eng):
    """bench.py's batch (synth.make_pg_batch: milli-cpu, memory in MiB multiples, gpu counts): every
    segment narrowed, the packed batch over a quarter smaller than the caller's arrays."""
    from placement import synth
    agg = synth.make_pg_batch(100_000, synth.SEED["cfg3"])
    eng.reset_stats()
    _check(eng, V1, agg)
    st = eng.stats()
    assert st["agg_narrow_segments"] == st["agg_segments"] > 0, st
    caller = sum(a.nbytes for a in agg)
    assert st["agg_wire_bytes"] < 0.75 * caller, (st["agg_wire_bytes"], caller)
