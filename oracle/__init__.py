"""CPU oracle -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
(and, for bench.py, as the timed CPU baseline).  The product path never imports this package.

  oracle/oracle.c      C restatement (fit mask, score/key, greedy placement, aggregation)
  oracle/semantics.py  object-level restatement of CalcPGMinResources / kueue TotalRequests /
                       CoScheduling.Build, pinned by tests/golden (the reference's own test answers)
Parity status: aggregation pinned (v2 by reference tests; v1 hand-derived, "parity unpinned");
fit/score/greedy are build-defined -> "parity unpinned" against the
reference, which has no placement code at all.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
V1, V2 = 1, 2

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i64, i32 = ctypes.c_int64, ctypes.c_int32
        L.orc_pg_min_resources.argtypes = [i32, i64, P, P, P, P, P, P, P, P, P, P]
        L.orc_pg_min_resources.restype = ctypes.c_int
        L.orc_pg_min_resources_keys.argtypes = [i32, i64, i32, P, P, P, P, P, P, P, P, P, P]
        L.orc_pg_min_resources_keys.restype = ctypes.c_int
        L.orc_fit_mask.argtypes = [i64, P, P, i64, P, P, P, P, ctypes.c_int]
        L.orc_fit_mask.restype = ctypes.c_int
        L.orc_place_greedy.argtypes = [i64, P, P, i64, P, P, P, P, P, P, P, ctypes.c_int]
        L.orc_place_greedy.restype = i64
        L.orc_key.argtypes = [P, ctypes.c_uint32, P, ctypes.c_uint32, ctypes.c_uint64]
        L.orc_key.restype = ctypes.c_uint64
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_window_cands.argtypes = [i64, P, P, i32, P, P, i32, P, ctypes.c_int]
        L.orc_window_cands.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def pg_min_resources(mode, job_group_off, min_member, group_replicas, group_cont_off, cont_req, cont_flags):
    J = len(job_group_off) - 1
    jgo = _c(job_group_off, np.int32)
    mm = _c(min_member if min_member is not None else np.zeros(J), np.int32)
    gr = _c(group_replicas, np.int32)
    gco = _c(group_cont_off, np.int32)
    cr = _c(cont_req, np.int64).reshape(-1, 4)
    cf = _c(cont_flags, np.uint8)
    out = np.zeros((J, 4), dtype=np.int64)
    pres = np.zeros(J, dtype=np.uint8)
    mem = np.zeros(J, dtype=np.int32)
    ovf = np.zeros(J, dtype=np.uint8)
    rc = lib().orc_pg_min_resources(mode, J, _p(jgo), _p(mm), _p(gr), _p(gco), _p(cr), _p(cf),
                                    _p(out), _p(pres), _p(mem), _p(ovf))
    assert rc == 0
    return out, pres, mem, ovf


def pg_min_resources_keys(mode, job_group_off, min_member, group_replicas, group_cont_off, cont_req, cont_flags):
    """Key-table form: cont_req [C][n_keys], cont_flags u32 (presence bits 0..n_keys-1 | kind << 16)."""
    J = len(job_group_off) - 1
    jgo = _c(job_group_off, np.int32)
    mm = _c(min_member if min_member is not None else np.zeros(J), np.int32)
    gr = _c(group_replicas, np.int32)
    gco = _c(group_cont_off, np.int32)
    cr = np.ascontiguousarray(cont_req, dtype=np.int64)
    nk = cr.shape[1]
    cf = _c(cont_flags, np.uint32)
    out = np.zeros((J, nk), dtype=np.int64)
    pres = np.zeros(J, dtype=np.uint16)
    mem = np.zeros(J, dtype=np.int32)
    ovf = np.zeros(J, dtype=np.uint8)
    rc = lib().orc_pg_min_resources_keys(mode, J, nk, _p(jgo), _p(mm), _p(gr), _p(gco), _p(cr), _p(cf),
                                         _p(out), _p(pres), _p(mem), _p(ovf))
    assert rc == 0
    return out, pres, mem, ovf


def fit_mask(res, labels, req, need, want_mask=True, nthreads=0):
    res = _c(res, np.int64)
    N = res.shape[1]
    req = _c(req, np.int64).reshape(-1, 4)
    J = req.shape[0]
    W = (N + 63) // 64
    mask = np.zeros((J, W), dtype=np.uint64) if want_mask else None
    counts = np.zeros(J, dtype=np.int64)
    lib().orc_fit_mask(N, _p(res), _p(_c(labels, np.uint32)), J, _p(req), _p(_c(need, np.uint32)),
                       _p(mask), _p(counts), int(nthreads))
    return mask, counts


def place_greedy(res, labels, job_group_off, priority, group_count, group_req, group_need, nthreads=0):
    """Returns (pod_node[P] int32, job_status[J] int32, residual_after[4][N])."""
    res = np.array(res, dtype=np.int64, copy=True, order="C")
    N = res.shape[1]
    jgo = _c(job_group_off, np.int32)
    J = len(jgo) - 1
    cnt = _c(group_count, np.int32)
    P = int(np.clip(cnt, 0, None).sum())
    pod = np.full(max(P, 1), -1, dtype=np.int32)
    st = np.zeros(max(J, 1), dtype=np.int32)
    lib().orc_place_greedy(N, _p(res), _p(_c(labels, np.uint32)), J, _p(jgo), _p(_c(priority, np.int32)),
                           _p(cnt), _p(_c(group_req, np.int64).reshape(-1, 4)), _p(_c(group_need, np.uint32)),
                           _p(pod), _p(st), int(nthreads))
    return pod[:P], st[:J], res


def key(res4, labels, req4, need, gid):
    r = _c(res4, np.int64)
    q = _c(req4, np.int64)
    return int(lib().orc_key(_p(r), int(labels), _p(q), int(need), int(gid)))


def window_cands(res, labels, group_req, group_need, K: int, nthreads=0) -> bytes:
    """One scan window on the CPU: per group the K best keys + limit, pe_resolver_* blob layout."""
    res = _c(res, np.int64)
    req = _c(group_req, np.int64).reshape(-1, 4)
    G = req.shape[0]
    blob = np.zeros(G * (16 + 48 * K), dtype=np.uint8)
    rc = lib().orc_window_cands(res.shape[1], _p(res), _p(_c(labels, np.uint32)), G, _p(req),
                                _p(_c(group_need, np.uint32)), int(K), _p(blob), int(nthreads))
    assert rc == 0
    return blob.tobytes()


def place_greedy_windowed(Resolver, res, labels, batch, K=256, max_groups=128, max_pods=1024, nthreads=0):
    """The engine's windowed greedy protocol with the scan done by window_cands on the CPU and the
    resolution by the product's host resolver (pe_resolver_*): the same algorithm as
    pe_place_greedy, no device.  Returns (pods, status, residual_after, windows)."""
    res = np.array(res, dtype=np.int64, copy=True)
    R = Resolver(batch.job_group_off, batch.priority, batch.group_count, batch.group_req, batch.group_need)
    # island groups (need bit 31) are scanned for count x request (placement.h PE_NEED_ISLAND)
    isl = (np.asarray(batch.group_need, dtype=np.uint32) >> 31) != 0
    scan_req = np.array(batch.group_req, dtype=np.int64, copy=True)
    for g in np.nonzero(isl)[0]:
        c = max(int(batch.group_count[g]), 0)
        scan_req[g] = [min(int(v) * c, (1 << 63) - 1) for v in batch.group_req[g]]
    windows = 0
    while not R.done():
        groups = R.next_window(max_groups, max_pods)
        blob = window_cands(res, labels, scan_req[groups], batch.group_need[groups], K, nthreads)
        upd, _ = R.resolve(groups, blob, 1, K)
        for row in upd:
            res[:, int(row[0])] = row[1:]
        windows += 1
    pods, st = R.results()
    return pods, st, res, windows


def num_threads() -> int:
    return int(lib().orc_num_threads())
