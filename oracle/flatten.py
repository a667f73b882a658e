"""Test-side flattener: object-level job specs -> the CSR arrays of pe_pg_min_resources.

TEST INFRASTRUCTURE ONLY (feeds oracle.c and cross-checks the product's C++ flattener,
training-operator_amd/host).  Layout (include/placement.h):
  job_group_off[J+1], min_member[J] (v1), group_replicas[G] (-1 = nil), group_cont_off[G+1],
  cont_req[C][4] int64 canonical, cont_flags[C] = presence bits 0-3 | kind << 4
  kind: 0 container, 1 init container, 2 sidecar (init, restartPolicy Always), 3 pod overhead
"""
from __future__ import annotations

from fractions import Fraction
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


# --------------------------------------------------------------------------- key tables (ABI 7)

KEYS_KIND_SHIFT = 16   # placement.h PE_KEYS_KIND_SHIFT
MAX_KEYS = 16          # placement.h PE_MAX_KEYS


def exp10(q: Fraction) -> int:
    """The exponent e of q = m * 10^e with m an integer not divisible by 10 (q != 0).  Quantities are
    decimal (or binary-integer) values, so q's denominator divides a power of ten."""
    q = Fraction(q)
    e = 0
    while q.denominator != 1:
        q *= 10
        e -= 1
        if e < -60:
            raise ValueError(f"{q} is not a decimal value")
    n = q.numerator
    while n != 0 and n % 10 == 0:
        n //= 10
        e += 1
    return e


class KeyFlat:
    """Flattener over a per-call KEY TABLE (pe_pg_min_resources_keys): any ResourceName, numbered in
    first-seen order; each key's scale s_k is the finest decimal exponent its quantities in the call
    need, so every value is an exact integer count of 10^s_k.  A value with no int64 at its key's
    scale marks its job host-overflowed (the reference holds such sums in inf.Dec), as the product
    adapters do (go/pkg/placement/hip/flatten.go, training-operator_amd/host/kf.cc)."""

    def __init__(self):
        self.job_group_off = [0]
        self.min_member: List[int] = []
        self.group_replicas: List[int] = []
        self.group_cont_off = [0]
        self.entries: List[Dict[str, Fraction]] = []
        self.kinds: List[int] = []
        self.keys: List[str] = []

    def add_container(self, res: Optional[S.ResourceList], kind: int) -> None:
        ent = {k: Fraction(q) for k, q in (res or {}).items()}
        for k, q in ent.items():
            if q < 0:
                raise ValueError(f"{k}={q} is negative")
            if k not in self.keys:
                self.keys.append(k)
        self.entries.append(ent)
        self.kinds.append(kind)

    def end_group(self, replicas: int) -> None:
        self.group_replicas.append(int(replicas))
        self.group_cont_off.append(len(self.entries))

    def end_job(self, min_member: int = 0) -> None:
        self.min_member.append(int(min_member))
        self.job_group_off.append(len(self.group_replicas))

    def scales(self) -> List[int]:
        out = []
        for k in self.keys:
            es = [exp10(e[k]) for e in self.entries if k in e and e[k] != 0]
            out.append(min(es) if es else 0)
        return out

    def job_of_container(self) -> np.ndarray:
        g_of_c = np.repeat(np.arange(len(self.group_replicas)), np.diff(self.group_cont_off))
        j_of_g = np.repeat(np.arange(len(self.min_member)), np.diff(self.job_group_off))
        return j_of_g[g_of_c] if len(g_of_c) else np.zeros(0, np.int64)

    def arrays(self, key_lo: int = 0, key_hi: Optional[int] = None):
        """CSR arrays for keys [key_lo, key_hi) (<= MAX_KEYS of them) -> (jgo, mm, rep, gco, req [C][nk],
        flags u32 [C]) and host_overflow [J] (values with no int64 at their scale)."""
        key_hi = len(self.keys) if key_hi is None else key_hi
        keys = self.keys[key_lo:key_hi] or ["<none>"]
        sc = (self.scales()[key_lo:key_hi]) or [0]
        assert len(keys) <= MAX_KEYS
        C, J = len(self.entries), len(self.min_member)
        req = np.zeros((C, len(keys)), np.int64)
        flags = np.zeros(C, np.uint32)
        host_ovf = np.zeros(J, np.uint8)
        jc = self.job_of_container()
        for c, ent in enumerate(self.entries):
            f = self.kinds[c] << KEYS_KIND_SHIFT
            for i, k in enumerate(keys):
                if k not in ent:
                    continue
                f |= 1 << i
                v = ent[k] / Fraction(10) ** sc[i]
                assert v.denominator == 1
                if v >= 2**63:
                    host_ovf[jc[c]] = 1
                else:
                    req[c, i] = int(v)
            flags[c] = f
        return (np.array(self.job_group_off, np.int32), np.array(self.min_member, np.int32),
                np.array(self.group_replicas, np.int32), np.array(self.group_cont_off, np.int32), req, flags), host_ovf

    def unflatten(self, vec, present: int, key_lo: int = 0, key_hi: Optional[int] = None) -> Dict[str, Fraction]:
        key_hi = len(self.keys) if key_hi is None else key_hi
        sc = self.scales()
        return {self.keys[key_lo + i]: Fraction(int(vec[i])) * Fraction(10) ** sc[key_lo + i]
                for i in range(key_hi - key_lo) if int(present) >> i & 1}


def add_v1_job_keys(flat: KeyFlat, min_member: int, replicas: Dict[str, dict],
                    pc_get: Callable[[str], Optional[int]] = lambda n: None) -> None:
    """add_v1_job over a key table (util.go:79-104 AddResourceList: any key)."""
    pri = []
    for t, spec in replicas.items():
        p = pc_get(spec.get("template", {}).get("priorityClassName", ""))
        pri.append((0 if p is None else p, t))
    for _, t in sorted(pri, key=lambda x: (-x[0], x[1])):
        spec = replicas[t]
        for c in spec.get("template", {}).get("containers", []):
            req = S.rl(c.get("requests"))
            flat.add_container(req if req is not None else S.rl(c.get("limits")), K_CONTAINER)
        r = spec.get("replicas")
        flat.end_group(-1 if r is None else r)
    flat.end_job(min_member)


def add_v2_pod_group_keys(flat: KeyFlat, replicas: int, pod: dict) -> None:
    for c in pod.get("initContainers", []):
        kind = K_SIDECAR if c.get("restartPolicy") == "Always" else K_INIT
        flat.add_container(S.rl(c.get("requests")) or {}, kind)
    for c in pod.get("containers", []):
        flat.add_container(S.rl(c.get("requests")) or {}, K_CONTAINER)
    if pod.get("overhead"):
        flat.add_container(S.rl(pod["overhead"]), K_OVERHEAD)
    flat.end_group(replicas)
