"""Pin the oracle before trusting it: object-level restatement and C restatement vs the
reference's own test answers (tests/golden, transcribed with file:line by make_golden.py)."""
import json
import os
from fractions import Fraction

import numpy as np
import pytest

import oracle
from oracle import flatten as F
from oracle import semantics as S

GPU = "nvidia.com/gpu"


def load(golden_dir, name):
    with open(os.path.join(golden_dir, name + ".json")) as f:
        return json.load(f)


def rlist(d):
    return {k: S.parse_quantity(v) for k, v in d.items()}


# ----------------------------------------------------------------- Quantity parsing

@pytest.mark.parametrize("s,v", [("1", 1), ("500m", Fraction(1, 2)), ("0.8", Fraction(4, 5)), ("4Gi", 4 << 30),
                                 ("404Gi", 404 << 30), ("1600m", Fraction(8, 5)), ("1e3", 1000), ("2k", 2000),
                                 ("1.5Ki", 1536), ("+3", 3), ("-2", -2), ("100M", 10**8), (".5", Fraction(1, 2))])
def test_parse_quantity(s, v):
    assert S.parse_quantity(s) == v


@pytest.mark.parametrize("bad", ["", "abc", "1.2.3", "4Gb", "1ii", "e3"])
def test_parse_quantity_rejects(bad):
    with pytest.raises(ValueError):
        S.parse_quantity(bad)


def test_canonical_units():
    assert S.canonical("cpu", S.parse_quantity("0.8")) == 800
    assert S.canonical("memory", S.parse_quantity("4Gi")) == 4 << 30
    with pytest.raises(ValueError):
        S.canonical("cpu", S.parse_quantity("0.0001"))     # scale < -3: not exact in milli
    with pytest.raises(ValueError):
        S.canonical("memory", S.parse_quantity("1500m"))   # fractional bytes
    with pytest.raises(ValueError):
        S.canonical("cpu", S.parse_quantity("-1"))


# ----------------------------------------------------------------- v2 (pinned by reference tests)

def test_v2_total_requests(golden_dir):
    g = load(golden_dir, "v2_total_requests")
    for case in g["cases"]:
        info = S.new_info([(n, r, pod) for n, r, pod in case["pod_spec_replicas"]])
        got = info["TotalRequests"]
        assert set(got) == set(case["want"]), case["name"]
        for name, want in case["want"].items():
            assert got[name]["Replicas"] == want["Replicas"]
            assert S.same_resource_list(got[name]["PodRequests"], rlist(want["PodRequests"])), case["name"]


def test_v2_enforce_ml_policy(golden_dir):
    g = load(golden_dir, "v2_enforce_ml_policy")
    for case in g["cases"]:
        info = {"TotalRequests": {n: {"Replicas": r, "PodRequests": {}} for n, r in case["replicas"].items()}}
        S.enforce_ml_policy(info, case["ml_policy"], case["trainjob_num_nodes"])
        assert {n: v["Replicas"] for n, v in info["TotalRequests"].items()} == case["want_replicas"], case["name"]


def _v2_pipeline(case):
    info = S.new_info([(n, 1, pod) for n, pod in case["replicated_jobs"]])   # trainingruntime.go:109-112
    S.enforce_ml_policy(info, case["ml_policy"], case["trainjob_num_nodes"])
    return info, S.build_podgroup(info, case["coscheduling"])


def test_v2_podgroup_semantics(golden_dir):
    g = load(golden_dir, "v2_podgroup")
    assert any(c["pinned"] for c in g["cases"])
    for case in g["cases"]:
        _, pg = _v2_pipeline(case)
        if case["want"] is None:
            assert pg is None
            continue
        assert pg["minMember"] == case["want"]["minMember"], case["name"]
        assert S.same_resource_list(pg["minResources"], rlist(case["want"]["minResources"])), case["name"]
        assert pg["scheduleTimeoutSeconds"] == case["want"]["scheduleTimeoutSeconds"]


def test_v2_build_from_info_semantics(golden_dir):
    g = load(golden_dir, "v2_build_from_info")
    for case in g["cases"]:
        info = {"TotalRequests": {n: {"Replicas": v["Replicas"], "PodRequests": rlist(v["PodRequests"])}
                                  for n, v in case["total_requests"].items()}}
        S.enforce_ml_policy(info, case["ml_policy"], case["trainjob_num_nodes"])
        assert {n: v["Replicas"] for n, v in info["TotalRequests"].items()} == case["want_replicas"]
        pg = S.build_podgroup(info, case["coscheduling"])
        assert pg["minMember"] == case["want"]["minMember"]
        assert S.same_resource_list(pg["minResources"], rlist(case["want"]["minResources"])), case["name"]


# ----------------------------------------------------------------- v1 (hand-derived, parity unpinned)

def _pc_get(case):
    pri = case.get("priorities", {})
    return lambda name: pri.get(name)


def test_v1_semantics(golden_dir):
    g = load(golden_dir, "v1_podgroup")
    for case in g["cases"]:
        mm, res = S.v1_pg_spec(case["replicas"], case["scheduling_policy"], _pc_get(case))
        assert mm == case["want_min_member"], case["name"]
        assert S.same_resource_list(res, rlist(case["want"])), case["name"]
        if "want_any_of" in case:
            outs = S.calc_pg_min_resources_all_orders(mm, case["replicas"], _pc_get(case))
            wants = [rlist(w) for w in case["want_any_of"]]
            assert all(any(S.same_resource_list(o, w) for w in wants) for o in outs)
            assert len(outs) == len(wants)


# ----------------------------------------------------------------- C oracle vs golden

def test_c_oracle_v1_matches_golden(golden_dir):
    g = load(golden_dir, "v1_podgroup")
    flat, expect = F.Flat(), []
    for case in g["cases"]:
        if (case["scheduling_policy"] or {}).get("minResources") is not None:
            continue  # verbatim path: no aggregation (job.go:267-269)
        mm = S.v1_pg_spec(case["replicas"], case["scheduling_policy"], _pc_get(case))[0]
        F.add_v1_job(flat, mm, case["replicas"], GPU, _pc_get(case))
        expect.append(case)
    out, pres, members, ovf = oracle.pg_min_resources(oracle.V1, *flat.arrays())
    for j, case in enumerate(expect):
        got = F.unflatten(out[j], pres[j], GPU)
        assert got == F.canonical_list(rlist(case["want"]), GPU), case["name"]
        assert ovf[j] == 0


def test_c_oracle_v2_matches_golden(golden_dir):
    g = load(golden_dir, "v2_podgroup")
    flat, expect = F.Flat(), []
    for case in g["cases"]:
        if case["want"] is None:
            continue
        info, _ = _v2_pipeline(case)
        pods = dict(case["replicated_jobs"])
        for name in sorted(info["TotalRequests"]):
            F.add_v2_pod_group(flat, info["TotalRequests"][name]["Replicas"], pods[name], GPU)
        flat.end_job(0)
        expect.append(case)
    gb = load(golden_dir, "v2_build_from_info")
    for case in gb["cases"]:
        tr = {n: dict(v) for n, v in case["total_requests"].items()}
        for n, r in case["want_replicas"].items():
            tr[n]["Replicas"] = r
        F.add_v2_info_job(flat, tr, GPU)
        expect.append(case)
    out, pres, members, ovf = oracle.pg_min_resources(oracle.V2, *flat.arrays())
    for j, case in enumerate(expect):
        assert F.unflatten(out[j], pres[j], GPU) == F.canonical_list(rlist(case["want"]["minResources"]), GPU), case["name"]
        assert members[j] == case["want"]["minMember"]
        assert ovf[j] == 0


def test_c_oracle_v2_kueue_pins(golden_dir):
    """runtime_test.go:37-104: per-pod TotalRequests 15 and 40 through the C restatement."""
    g = load(golden_dir, "v2_total_requests")
    case = g["cases"][0]
    for name, r, pod in case["pod_spec_replicas"]:
        flat = F.Flat()
        F.add_v2_pod_group(flat, 1, pod, GPU)
        flat.end_job(0)
        out, pres, _, _ = oracle.pg_min_resources(oracle.V2, *flat.arrays())
        want = F.canonical_list(rlist(case["want"][name]["PodRequests"]), GPU)
        assert F.unflatten(out[0], pres[0], GPU) == want


def test_c_oracle_overflow_and_wrap():
    flat = F.Flat()
    flat.add_container({"memory": Fraction(2**62)}, F.K_CONTAINER, GPU)
    flat.end_group(4)                   # 4 * 2^62 overflows int64 -> flagged (Go: inf.Dec fallback)
    flat.end_job(0)
    flat.add_container({"cpu": Fraction(1)}, F.K_CONTAINER, GPU)
    flat.end_group(2**31 - 1)
    flat.add_container({"cpu": Fraction(1)}, F.K_CONTAINER, GPU)
    flat.end_group(2)                   # int32 members wrap like Go's int32 +=
    flat.end_job(0)
    out, pres, members, ovf = oracle.pg_min_resources(oracle.V2, *flat.arrays())
    assert ovf[0] == 1 and ovf[1] == 0
    assert members[1] == -(2**31) + 1
    assert out[1, 0] == (2**31 + 1) * 1000


# ----------------------------------------------------------------- kueue TotalRequests edge cases

from kueue_cases import CASES as KUEUE_CASES  # noqa: E402


@pytest.mark.parametrize("name,pod,want", KUEUE_CASES, ids=[c[0] for c in KUEUE_CASES])
def test_total_requests_edge_cases(name, pod, want):
    """Python restatement and C restatement against hand-derived answers (kueue_cases.py)."""
    assert F.canonical_list(S.total_requests(pod), GPU) == want
    flat = F.Flat()
    F.add_v2_pod_group(flat, 1, pod, GPU)
    flat.end_job(0)
    out, pres, mem, ovf = oracle.pg_min_resources(2, *flat.arrays())
    assert F.unflatten(out[0], pres[0], GPU) == want and mem[0] == 1 and ovf[0] == 0


# ----------------------------------------------------------------- keys beyond the four dimensions

def test_wide_keys_semantics(golden_dir):
    """The object-level restatement gives the hand-derived answers of wide_keys.json (hugepages, rdma,
    two accelerator names, cpu in micro-cores, 21 keys, an int64 overflow)."""
    g = load(golden_dir, "wide_keys")
    for case in g["v1"]:
        mm, res = S.v1_pg_spec(case["replicas"], case["scheduling_policy"], _pc_get(case))
        assert mm == case["want_min_member"], case["name"]
        assert S.same_resource_list(res, rlist(case["want"])), case["name"]
    for case in g["v2"]:
        _, pg = _v2_pipeline(dict(case, coscheduling={}))
        assert pg["minMember"] == case["want"]["minMember"], case["name"]
        assert S.same_resource_list(pg["minResources"], rlist(case["want"]["minResources"])), case["name"]


def test_wide_keys_c_oracle(golden_dir):
    """The C restatement over the key table (orc_pg_min_resources_keys), 16-key slices, per-key
    scales: every answer exact, and only the overflow case flagged (the adapters' reference case)."""
    import wide_keys as W
    g = load(golden_dir, "wide_keys")
    for mode, cases, flat in ((W.V1, g["v1"], W.v1_flat(g["v1"])), (W.V2, g["v2"], W.v2_flat(g["v2"]))):
        res, members, ovf, _ = W.run(oracle.pg_min_resources_keys, mode, flat)
        for j, case in enumerate(cases):
            want = case["want"] if mode == W.V1 else case["want"]["minResources"]
            assert ovf[j] == int(case.get("overflow", False)), case["name"]
            if not ovf[j]:
                assert W.same(res[j], W.want_list(want)), (case["name"], res[j])
            if mode == W.V2:
                assert members[j] == case["want"]["minMember"]
    assert len(W.v2_flat(g["v2"]).keys) > 16                 # the slicing is exercised


def test_key_scales():
    flat = F.KeyFlat()
    flat.add_container({"cpu": S.parse_quantity("1500u"), "memory": S.parse_quantity("1Gi"),
                        "x/y": S.parse_quantity("3k")}, F.K_CONTAINER)
    flat.add_container({"cpu": S.parse_quantity("2"), "x/y": S.parse_quantity("5000")}, F.K_CONTAINER)
    flat.end_group(1)
    flat.end_job(1)
    assert flat.keys == ["cpu", "memory", "x/y"]
    assert flat.scales() == [-4, 0, 3]
    arrs, host_ovf = flat.arrays()
    assert arrs[4].tolist() == [[15, 1 << 30, 3], [20000, 0, 5]] and host_ovf.tolist() == [0]
    assert arrs[5].tolist() == [7, 5]
