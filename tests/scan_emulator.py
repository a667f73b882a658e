"""Test-side emulation of the device scan+merge (numpy, vectorised Appendix-B keys).

TEST INFRASTRUCTURE: produces per-shard candidate blobs in the merge kernel's layout so the host
resolver (pe_resolver_*) can be exercised on CPU, sharded over several "ranks", and checked
against the naive oracle.  `weak=True` truncates lists at random exact prefixes (valid limits
that are as tight as the protocol allows) to force the rescan path.
"""
from __future__ import annotations

import struct

import numpy as np

from placement import synth

NO_KEY = np.uint64(0xFFFFFFFFFFFFFFFF)
SMAX = np.uint64((1 << 40) - 1)


def keys(res: np.ndarray, labels: np.ndarray, q, need: int, gid0: int) -> np.ndarray:
    res = np.asarray(res, dtype=np.int64)
    n = res.shape[1]
    q = np.asarray(q, dtype=np.int64)
    fit = (labels.astype(np.uint32) & np.uint32(need)) == np.uint32(need)
    for d in range(4):
        fit &= q[d] <= res[d]
    with np.errstate(over="ignore"):
        left = (res.astype(np.uint64) - q.astype(np.uint64)[:, None])
        a = left[0]
        b = left[1] >> np.uint64(20)
        c = left[2]
        d = left[3] >> np.uint64(24)
        big = (a > SMAX) | (b > SMAX) | (c >= np.uint64(1 << 20)) | (d > SMAX)
        s = a + b + (c << np.uint64(20)) + d
    score = np.where(big | (s > SMAX), SMAX, s)
    gid = np.arange(gid0, gid0 + n, dtype=np.uint64)
    return np.where(fit, (score << np.uint64(24)) | gid, NO_KEY)


def shard_blob(res, labels, gid0, groups_req, groups_need, K, rng=None, weak=False) -> bytes:
    out = bytearray()
    for q, need in zip(groups_req, groups_need):
        k = keys(res, labels, q, int(need), gid0)
        feas = np.sort(k[k != NO_KEY])
        if len(feas) > K:
            lst, limit = feas[:K], int(feas[K])
        else:
            lst, limit = feas, int(NO_KEY)
        if weak and rng is not None and len(lst) > 0:
            cut = int(rng.integers(1, len(lst) + 1))
            if cut < len(lst):
                limit = int(lst[cut])
                lst = lst[:cut]
        out += struct.pack("<iiQ", len(lst), 0, limit)
        for key in lst:
            i = int(key & np.uint64(0xFFFFFF)) - gid0
            out += struct.pack("<Q4qQ", int(key), *[int(res[d, i]) for d in range(4)], int(labels[i]))
        out += b"\0" * (48 * (K - len(lst)))
    return bytes(out)


def run_resolver(Resolver, inv_res, labels, batch, K=8, shards=1, max_groups=16, max_pods=64, weak=False, seed=0):
    """Drive pe_resolver_* over `shards` contiguous node shards; returns (pods, status, residual)."""
    res = np.array(inv_res, dtype=np.int64, copy=True)
    N = res.shape[1]
    bounds = [(N * r // shards, N * (r + 1) // shards) for r in range(shards)]
    R = Resolver(batch.job_group_off, batch.priority, batch.group_count, batch.group_req, batch.group_need)
    scan_req = synth.scan_requests(batch)   # island groups are scanned for count x request
    rng = np.random.default_rng(seed)
    windows = 0
    while not R.done():
        groups = R.next_window(max_groups, max_pods)
        assert len(groups) > 0
        blob = b"".join(shard_blob(res[:, b:e], labels[b:e], b, scan_req[groups], batch.group_need[groups], K,
                                   rng, weak) for b, e in bounds)
        upd, _ = R.resolve(groups, blob, shards, K)
        for row in upd:
            res[:, int(row[0])] = row[1:]
        windows += 1
        assert windows < 10 * (batch.n_pods + batch.n_jobs) + 10
    pods, st = R.results()
    return pods, st, res
