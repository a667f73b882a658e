"""Key-table aggregation driver shared by the CPU (oracle) and GPU (engine) tests of
tests/golden/wide_keys.json: flatten the cases over a per-call key table (oracle/flatten.py KeyFlat),
run one call per slice of <= 16 keys through `agg` (oracle.pg_min_resources_keys or
Engine.pg_min_resources_keys), and read each job's result back as exact values."""
from __future__ import annotations

from fractions import Fraction

import numpy as np

from oracle import flatten as F
from oracle import semantics as S

V1, V2 = 1, 2


def _pc_get(case):
    pri = case.get("priorities", {})
    return lambda name: pri.get(name)


def v1_flat(cases):
    kf = F.KeyFlat()
    for case in cases:
        mm = S.v1_pg_spec(case["replicas"], case["scheduling_policy"], _pc_get(case))[0]
        F.add_v1_job_keys(kf, mm, case["replicas"], _pc_get(case))
    return kf


def v2_flat(cases):
    kf = F.KeyFlat()
    for case in cases:
        info = S.new_info([(n, 1, pod) for n, pod in case["replicated_jobs"]])
        S.enforce_ml_policy(info, case["ml_policy"], case["trainjob_num_nodes"])
        pods = dict(case["replicated_jobs"])
        for name in sorted(info["TotalRequests"]):
            F.add_v2_pod_group_keys(kf, info["TotalRequests"][name]["Replicas"], pods[name])
        kf.end_job(0)
    return kf


def run(agg, mode, kf: F.KeyFlat):
    """-> (per job {key: Fraction}, members [J], overflow [J]) over every 16-key slice; also the raw
    per-slice outputs for array comparisons."""
    J = len(kf.min_member)
    res = [dict() for _ in range(J)]
    ovf = np.zeros(J, np.uint8)
    members = None
    raw = []
    nk = max(len(kf.keys), 1)
    for lo in range(0, nk, F.MAX_KEYS):
        hi = min(lo + F.MAX_KEYS, len(kf.keys))
        arrs, host_ovf = kf.arrays(lo, hi)
        out = agg(mode, *arrs)
        raw.append((arrs, out))
        vals, pres, mem, o = out
        members = mem if members is None else members
        assert np.array_equal(mem, members)
        ovf |= o | host_ovf
        for j in range(J):
            if hi > lo:
                res[j].update(kf.unflatten(vals[j], int(pres[j]), lo, hi))
    return res, members, ovf, raw


def want_list(d):
    return {k: S.parse_quantity(v) for k, v in d.items()}


def same(got, want):
    return set(got) == set(want) and all(Fraction(got[k]) == Fraction(want[k]) for k in got)
