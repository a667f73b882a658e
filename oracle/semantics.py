"""Object-level CPU restatement of the reference's PodGroup min-resource semantics.

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; never by the product (include/placement.h + HIP library).

Restates (reference = /root/reference, Go; cannot be compiled here):
  * k8s.io/apimachinery v0.30.7 resource.Quantity parsing/arithmetic [3P, not vendored]:
    exact decimal values; we use fractions.Fraction (never wraps, never rounds).
  * pkg/controller.v1/common/util.go:29-48      ReplicasPriority (priority DESC, sort.Sort)
  * pkg/controller.v1/common/util.go:79-104     AddResourceList (Limits only if Requests is nil)
  * pkg/controller.v1/common/util.go:106-145    CalcPGMinResources
  * pkg/util/k8sutil/k8sutil.go:126-137          GetTotalReplicas (nil replicas count as 1)
  * pkg/controller.v1/common/job.go:250-277      minMember / MinResources selection
  * pkg/runtime.v2/runtime.go:115-145            NewInfo -> kueue v0.6.3 TotalRequests [3P]
  * pkg/runtime.v2/framework/plugins/plainml/plainml.go:45-76, torch/torch.go:52-62,118-132,
    mpi/mpi.go:50-56                             MLPolicy replica rewrite
  * pkg/runtime.v2/framework/plugins/coscheduling/coscheduling.go:103-153  Build + needsCreateOrUpdate

Tie policy (util.go:124 sort.Sort is unstable; equal priorities keep Go map-iteration order,
which is random): this restatement orders equal priorities by replica-type name ascending and
`calc_pg_min_resources_all_orders` returns the result set over every tie permutation so tests
can assert the engine's answer is one the reference could have produced.
"""
from __future__ import annotations

import itertools
import re
from fractions import Fraction
from typing import Callable, Dict, List, Optional, Tuple

# --------------------------------------------------------------------------- Quantity

_BINARY = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DECIMAL = {"n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000), "": Fraction(1),
            "k": Fraction(10**3), "M": Fraction(10**6), "G": Fraction(10**9), "T": Fraction(10**12),
            "P": Fraction(10**15), "E": Fraction(10**18)}
_QRE = re.compile(r"^([+-]?)(\d*)(?:\.(\d*))?(.*)$")


def parse_quantity(s) -> Fraction:
    """resource.ParseQuantity grammar: <signedNumber><suffix>, suffix binarySI | decimalSI |
    decimalExponent. Returns the exact value."""
    if isinstance(s, (int, Fraction)):
        return Fraction(s)
    s = str(s).strip()
    m = _QRE.match(s)
    if not m or (m.group(2) == "" and not m.group(3)):
        raise ValueError(f"quantities must match the regular expression: {s!r}")
    sign, whole, frac, suf = m.group(1), m.group(2) or "0", m.group(3) or "", m.group(4)
    num = Fraction(int(whole + frac), 10 ** len(frac))
    if suf in _BINARY:
        num *= _BINARY[suf]
    elif suf in _DECIMAL:
        num *= _DECIMAL[suf]
    elif suf[:1] in ("e", "E") and re.fullmatch(r"[eE][+-]?\d+", suf):
        num *= Fraction(10) ** int(suf[1:])
    else:
        raise ValueError(f"unable to parse quantity's suffix: {s!r}")
    return -num if sign == "-" else num


ResourceList = Dict[str, Fraction]

CPU, MEMORY, EPHEMERAL = "cpu", "memory", "ephemeral-storage"


def dims(gpu_name: str) -> List[str]:
    """Engine dimension order: 0 cpu (milli), 1 memory (B), 2 <gpu_name> (count), 3 eph (B)."""
    return [CPU, MEMORY, gpu_name, EPHEMERAL]


def canonical(name: str, q: Fraction) -> int:
    """Canonical int64 unit used on the device: cpu -> milli, everything else -> base unit.
    Refuses values that are not exactly representable."""
    v = q * 1000 if name == CPU else q
    if v.denominator != 1:
        raise ValueError(f"{name}={q} is not an exact integer in canonical units")
    if v < 0:
        raise ValueError(f"{name}={q} is negative")
    if v >= 2**63:
        raise OverflowError(f"{name}={q} does not fit int64")
    return int(v)


def rl(d: Optional[dict]) -> Optional[ResourceList]:
    """Parse a {name: "quantity"} map; None stays None (nil map semantics matter in v1)."""
    if d is None:
        return None
    return {k: parse_quantity(v) for k, v in d.items()}


# --------------------------------------------------------------------------- v1

def add_resource_list(lst: ResourceList, req: Optional[ResourceList], limit: Optional[ResourceList]) -> None:
    """util.go:79-104. Requests keys always added (zero values too); Limits only when the
    Requests map is nil -- an empty non-nil map does NOT fall back."""
    for k, q in (req or {}).items():
        lst[k] = lst.get(k, Fraction(0)) + q
    if req is not None:
        return
    for k, q in (limit or {}).items():
        lst[k] = lst.get(k, Fraction(0)) + q


def get_total_replicas(replicas: Dict[str, dict]) -> int:
    """k8sutil.go:126-137: nil Replicas counts as 1; the int32 sum wraps like Go's."""
    return _wrap_int32(sum(1 if r.get("replicas") is None else int(r["replicas"]) for r in replicas.values()))


def _v1_order(replicas: Dict[str, dict], pc_get: Callable[[str], Optional[int]]) -> List[Tuple[int, str]]:
    out = []
    for t, spec in replicas.items():
        pri = pc_get(spec.get("template", {}).get("priorityClassName", ""))
        out.append((0 if pri is None else int(pri), t))  # util.go:114-119: error/nil -> 0
    return out


def _v1_accumulate(order: List[str], min_member: int, replicas: Dict[str, dict]) -> ResourceList:
    res: ResourceList = {}
    pod_cnt = 0
    for t in order:
        spec = replicas[t]
        if spec.get("replicas") is None:  # util.go:129
            continue
        for _ in range(int(spec["replicas"])):
            if pod_cnt >= min_member:
                break
            pod_cnt += 1
            for c in spec.get("template", {}).get("containers", []):
                add_resource_list(res, rl(c.get("requests")), rl(c.get("limits")))
    return res


def calc_pg_min_resources(min_member: int, replicas: Dict[str, dict],
                          pc_get: Callable[[str], Optional[int]] = lambda name: None) -> ResourceList:
    """util.go:108-145 with the deterministic tie policy (priority desc, type name asc)."""
    pri = _v1_order(replicas, pc_get)
    order = [t for _, t in sorted(pri, key=lambda x: (-x[0], x[1]))]
    return _v1_accumulate(order, min_member, replicas)


def calc_pg_min_resources_all_orders(min_member: int, replicas: Dict[str, dict],
                                     pc_get: Callable[[str], Optional[int]] = lambda name: None) -> List[ResourceList]:
    """Every result the reference can return: all permutations of equal-priority types."""
    pri = _v1_order(replicas, pc_get)
    levels = sorted({p for p, _ in pri}, reverse=True)
    groups = [[t for p, t in pri if p == lv] for lv in levels]
    outs = []
    for combo in itertools.product(*[list(itertools.permutations(g)) for g in groups]):
        order = [t for grp in combo for t in grp]
        r = _v1_accumulate(order, min_member, replicas)
        if r not in outs:
            outs.append(r)
    return outs


def v1_pg_spec(replicas: Dict[str, dict], scheduling_policy: Optional[dict],
               pc_get: Callable[[str], Optional[int]] = lambda name: None) -> Tuple[int, ResourceList]:
    """job.go:250-277: minMember = MinAvailable ?? totalReplicas; MinResources verbatim if set."""
    sp = scheduling_policy or {}
    min_member = get_total_replicas(replicas)
    if sp.get("minAvailable") is not None:
        min_member = int(sp["minAvailable"])
    if sp.get("minResources") is not None:
        return min_member, rl(sp["minResources"])
    return min_member, calc_pg_min_resources(min_member, replicas, pc_get)


# --------------------------------------------------------------------------- v2

def _merge_sum(a: ResourceList, b: Optional[ResourceList]) -> ResourceList:
    out = dict(a)
    for k, q in (b or {}).items():
        out[k] = out.get(k, Fraction(0)) + q
    return out


def _merge_max(a: ResourceList, b: ResourceList) -> ResourceList:
    out = dict(a)
    for k, q in b.items():
        out[k] = max(out[k], q) if k in out else q
    return out


def total_requests(pod: dict) -> ResourceList:
    """kueue v0.6.3 pkg/util/limitrange.TotalRequests (called at runtime.go:134), requests only:
    total = max(sum(sidecars) + sum(containers), max_i(init_i + sidecars declared before i)) + overhead.
    Pinned by runtime_test.go:45-101 (5+10 -> 15, 15+25 -> 40) and trainingruntime_test.go:88-94."""
    sidecars: ResourceList = {}
    init_max: ResourceList = {}
    for c in pod.get("initContainers", []):
        req = rl(c.get("requests")) or {}
        if c.get("restartPolicy") == "Always":
            sidecars = _merge_sum(sidecars, req)
        else:
            init_max = _merge_max(init_max, _merge_sum(sidecars, req))
    main: ResourceList = {}
    for c in pod.get("containers", []):
        main = _merge_sum(main, rl(c.get("requests")))
    total = _merge_max(_merge_sum(sidecars, main), init_max)
    return _merge_sum(total, rl(pod.get("overhead")))


JOB_TRAINER_NODE = "trainer-node"   # pkg/constants/constants.go:18
JOB_INITIALIZER = "initializer"     # pkg/constants/constants.go:27


def new_info(pod_spec_replicas: List[Tuple[str, int, dict]]) -> dict:
    """runtime.go:115-145 NewInfo (TotalRequests part)."""
    return {"TotalRequests": {name: {"Replicas": int(r), "PodRequests": total_requests(pod)}
                              for name, r, pod in pod_spec_replicas}}


def enforce_ml_policy(info: dict, ml_policy: Optional[dict], trainjob_num_nodes: Optional[int]) -> None:
    """plainml.go:45-76 / torch.go:52-62,118-132 / mpi.go:50-56: TotalRequests["trainer-node"].Replicas =
    TrainJob.Trainer.NumNodes ?? MLPolicy.NumNodes ?? 1 (DefaultJobReplicas); MPI is a no-op."""
    if ml_policy is None or ml_policy.get("source") == "mpi":
        return
    num_nodes = ml_policy.get("numNodes")
    if trainjob_num_nodes is not None:
        num_nodes = trainjob_num_nodes
    if JOB_TRAINER_NODE in info["TotalRequests"]:
        info["TotalRequests"][JOB_TRAINER_NODE]["Replicas"] = 1 if num_nodes is None else int(num_nodes)


def _wrap_int32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - 2**32 if v >= 2**31 else v


def build_podgroup(info: Optional[dict], coscheduling: Optional[dict]) -> Optional[dict]:
    """coscheduling.go:103-133: MinMember = sum Replicas (Go int32 wrap), MinResources[k] =
    sum Replicas*PodRequests[k] (keys present even for Replicas == 0)."""
    if info is None or coscheduling is None:
        return None
    members = 0
    total: ResourceList = {}
    for trr in info["TotalRequests"].values():
        members = _wrap_int32(members + trr["Replicas"])
        for k, q in trr["PodRequests"].items():
            total[k] = total.get(k, Fraction(0)) + q * trr["Replicas"]
    return {"minMember": members, "minResources": total,
            "scheduleTimeoutSeconds": coscheduling.get("scheduleTimeoutSeconds")}


def needs_create_or_update(old: Optional[dict], new: dict, suspended: bool) -> bool:
    """coscheduling.go:150-153."""
    return old is None or (suspended and (old["spec"] != new["spec"] or old.get("labels") != new.get("labels")
                                          or old.get("annotations") != new.get("annotations")))


def same_resource_list(a: ResourceList, b: ResourceList) -> bool:
    """Reference equality: same key set, each value equal under Quantity.Cmp."""
    return set(a) == set(b) and all(Fraction(a[k]) == Fraction(b[k]) for k in a)


# --------------------------------------------------------------------------- placement (Appendix B)

SCORE_MAX = (1 << 40) - 1
INT64_MAX = (1 << 63) - 1
NEED_ISLAND = 1 << 31   # placement.h PE_NEED_ISLAND: the group's pods as one unit on one island node


def appendix_b_key(res4, labels: int, q4, need: int, node: int) -> Optional[int]:
    """SURVEY.md Appendix B, restated independently of oracle.c: None when the node does not fit,
    else (score << 24) | node with score = sat40(sat40(l0) + sat40(l1 >> 20) + sat40(l2 << 20) +
    sat40(l3 >> 24)), l = residual - request (all non-negative for a fitting node)."""
    if (labels & need) != need:
        return None
    left = [int(r) - int(q) for r, q in zip(res4, q4)]
    if any(v < 0 for v in left):
        return None
    terms = [left[0], left[1] >> 20, left[2] << 20, left[3] >> 24]
    score = min(SCORE_MAX, sum(min(SCORE_MAX, t) for t in terms))
    return (score << 24) | node


def place_greedy_appendix_b(res, labels, job_group_off, priority, group_count, group_req, group_need):
    """The sequential greedy rule in plain Python (small inputs only): jobs by (priority desc, index
    asc), groups in order, each pod on the argmin-key node (an island group, need bit 31: all its pods
    on the one node with the smallest key for count x request), all-or-nothing per job with rollback.
    Returns (pod_node list, job_status list, residual [4][N] as lists of ints)."""
    R = [[int(x) for x in row] for row in res]
    N = len(R[0]) if R else 0
    J = len(priority)
    pod_off = [0]
    for c in group_count:
        pod_off.append(pod_off[-1] + max(0, int(c)))
    pods = [-1] * pod_off[-1]
    status = [0] * J
    order = sorted(range(J), key=lambda j: (-int(priority[j]), j))
    for j in order:
        placed = []
        ok = True
        for g in range(int(job_group_off[j]), int(job_group_off[j + 1])):
            q = [int(x) for x in group_req[g]]
            if int(group_need[g]) & NEED_ISLAND and int(group_count[g]) > 0:
                # island group: every pod on one node, chosen for the summed request
                c = int(group_count[g])
                qe = [x * c for x in q]
                best = None
                if all(v <= INT64_MAX for v in qe):
                    for n in range(N):
                        k = appendix_b_key([R[d][n] for d in range(4)], int(labels[n]), qe, int(group_need[g]), n)
                        if k is not None and (best is None or k < best):
                            best = k
                if best is None:
                    ok = False
                    break
                n = best & 0xFFFFFF
                for p in range(c):
                    for d in range(4):
                        R[d][n] -= q[d]
                    pods[pod_off[g] + p] = n
                    placed.append((g, p, n))
                continue
            for p in range(int(group_count[g])):
                best = None
                for n in range(N):
                    k = appendix_b_key([R[d][n] for d in range(4)], int(labels[n]), q, int(group_need[g]), n)
                    if k is not None and (best is None or k < best):
                        best = k
                if best is None:
                    ok = False
                    break
                n = best & 0xFFFFFF
                for d in range(4):
                    R[d][n] -= q[d]
                pods[pod_off[g] + p] = n
                placed.append((g, p, n))
            if not ok:
                break
        if not ok:
            for g, p, n in placed:
                for d in range(4):
                    R[d][n] += int(group_req[g][d])
                pods[pod_off[g] + p] = -1
            status[j] = 1
    return pods, status, R
