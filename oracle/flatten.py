"""Test-side flattener: object-level job specs -> the CSR arrays of pe_pg_min_resources.

TEST INFRASTRUCTURE ONLY (feeds oracle.c and cross-checks the product's C++ flattener,
training-operator_amd/host).  Layout (include/placement.h):
  job_group_off[J+1], min_member[J] (v1), group_replicas[G] (-1 = nil), group_cont_off[G+1],
  cont_req[C][4] int64 canonical, cont_flags[C] = presence bits 0-3 | kind << 4
  kind: 0 container, 1 init container, 2 sidecar (init, restartPolicy Always), 3 pod overhead
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from . import semantics as S

K_CONTAINER, K_INIT, K_SIDECAR, K_OVERHEAD = 0, 1, 2, 3


class Flat:
    def __init__(self):
        self.job_group_off = [0]
        self.min_member: List[int] = []
        self.group_replicas: List[int] = []
        self.group_cont_off = [0]
        self.cont_req: List[List[int]] = []
        self.cont_flags: List[int] = []

    def add_container(self, res: Optional[S.ResourceList], kind: int, gpu_name: str) -> None:
        names = S.dims(gpu_name)
        vec, pres = [0, 0, 0, 0], 0
        for k, q in (res or {}).items():
            if k not in names:
                raise KeyError(f"resource {k!r} is not an engine dimension")
            d = names.index(k)
            vec[d] = S.canonical(k, q)
            pres |= 1 << d
        self.cont_req.append(vec)
        self.cont_flags.append(pres | (kind << 4))

    def end_group(self, replicas: int) -> None:
        self.group_replicas.append(int(replicas))
        self.group_cont_off.append(len(self.cont_req))

    def end_job(self, min_member: int = 0) -> None:
        self.min_member.append(int(min_member))
        self.job_group_off.append(len(self.group_replicas))

    def arrays(self):
        return (np.array(self.job_group_off, np.int32), np.array(self.min_member, np.int32),
                np.array(self.group_replicas, np.int32), np.array(self.group_cont_off, np.int32),
                np.array(self.cont_req, np.int64).reshape(-1, 4), np.array(self.cont_flags, np.uint8))


def add_v1_job(flat: Flat, min_member: int, replicas: Dict[str, dict], gpu_name: str,
               pc_get: Callable[[str], Optional[int]] = lambda n: None) -> None:
    pri = []
    for t, spec in replicas.items():
        p = pc_get(spec.get("template", {}).get("priorityClassName", ""))
        pri.append((0 if p is None else p, t))
    for _, t in sorted(pri, key=lambda x: (-x[0], x[1])):
        spec = replicas[t]
        for c in spec.get("template", {}).get("containers", []):
            req = S.rl(c.get("requests"))
            flat.add_container(req if req is not None else S.rl(c.get("limits")), K_CONTAINER, gpu_name)
        r = spec.get("replicas")
        flat.end_group(-1 if r is None else r)
    flat.end_job(min_member)


def add_v2_pod_group(flat: Flat, replicas: int, pod: dict, gpu_name: str) -> None:
    for c in pod.get("initContainers", []):
        kind = K_SIDECAR if c.get("restartPolicy") == "Always" else K_INIT
        flat.add_container(S.rl(c.get("requests")) or {}, kind, gpu_name)
    for c in pod.get("containers", []):
        flat.add_container(S.rl(c.get("requests")) or {}, K_CONTAINER, gpu_name)
    if pod.get("overhead"):
        flat.add_container(S.rl(pod["overhead"]), K_OVERHEAD, gpu_name)
    flat.end_group(replicas)


def add_v2_info_job(flat: Flat, total_requests: Dict[str, dict], gpu_name: str) -> None:
    """TotalRequests already computed (runtime.Info): one K_CONTAINER record per entry."""
    for name in sorted(total_requests):
        trr = total_requests[name]
        pr = trr["PodRequests"]
        flat.add_container({k: S.parse_quantity(v) for k, v in pr.items()}, K_CONTAINER, gpu_name)
        flat.end_group(trr["Replicas"])
    flat.end_job(0)


def unflatten(vec, present: int, gpu_name: str) -> Dict[str, int]:
    names = S.dims(gpu_name)
    return {names[d]: int(vec[d]) for d in range(4) if present & (1 << d)}


def canonical_list(rlist: S.ResourceList, gpu_name: str) -> Dict[str, int]:
    return {k: S.canonical(k, q) for k, q in rlist.items()}
