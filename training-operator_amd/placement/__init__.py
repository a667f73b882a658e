"""MI355X gang-placement engine -- Python handle over the libplacement C ABI.

    eng = Engine(device_id=0)                      # one context per process / GPU / shard
    eng.load_nodes(cap, used, labels, island)      # [4][N] int64 SoA of the global inventory
    res, present, members, ovf = eng.pg_min_resources(V1, *csr)   # CalcPGMinResources batch
    counts = eng.fit_mask(req, need)               # J x N feasibility bitmask (device-resident)
    pod_node, status = eng.place_greedy(batch)     # greedy best-fit all-or-nothing gangs

Every call runs on the GPU through include/placement.h; nothing here computes a result itself.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _abi
from ._abi import (PE_JOB_PLACED, PE_JOB_UNSCHEDULABLE, PE_KIND_CONTAINER, PE_KIND_INIT, PE_KIND_OVERHEAD,
                   PE_KIND_SHIFT, PE_KIND_SIDECAR, PE_MODE_V1, PE_MODE_V2, PE_NODE_REMOVE, PE_NODE_SET)

V1, V2 = PE_MODE_V1, PE_MODE_V2

__all__ = ["Engine", "HostExchange", "Resolver", "PlacementError", "V1", "V2", "PE_JOB_PLACED", "PE_JOB_UNSCHEDULABLE",
           "PE_KIND_CONTAINER", "PE_KIND_INIT", "PE_KIND_SIDECAR", "PE_KIND_OVERHEAD", "PE_KIND_SHIFT", "comm_id",
           "PE_NODE_SET", "PE_NODE_REMOVE"]


class PlacementError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_abi.ERR_NAMES.get(code, code)}: {msg}")
        self.code = code


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=dt)


def comm_id() -> bytes:
    buf = (ctypes.c_uint8 * _abi.PE_COMM_ID_BYTES)()
    rc = _abi.load().pe_comm_id(buf)
    if rc != 0:
        raise PlacementError(rc, "pe_comm_id failed")
    return bytes(buf)


class HostExchange:
    """pe_host_exchange: the native shared-memory all-gather of one node's ranks (the sharded greedy's
    transport when RCCL cannot be set up).  Every rank opens the same `name` ("/..."); rank 0 creates
    the segment.  Pass it as Engine(..., exchange=hx): the engine calls the C function directly (no
    Python on the window path)."""

    def __init__(self, name: str, rank: int, world: int, max_bytes: int):
        self.lib = _abi.load()
        h = ctypes.c_void_p()
        rc = self.lib.pe_host_exchange_open(name.encode(), rank, world, max_bytes, ctypes.byref(h))
        if rc != 0:
            raise PlacementError(rc, f"pe_host_exchange_open({name!r}, rank {rank} of {world})")
        self.h = h
        self.rank, self.world = rank, world
        self.fn = ctypes.cast(self.lib.pe_host_exchange_allgather, _abi.ALLGATHER_FN)

    def allgather(self, blob: bytes) -> bytes:
        out = ctypes.create_string_buffer(len(blob) * self.world)
        rc = self.lib.pe_host_exchange_allgather(self.h, blob, out, len(blob))
        if rc != 0:
            raise PlacementError(rc, "pe_host_exchange_allgather")
        return out.raw

    def close(self):
        if getattr(self, "h", None):
            self.lib.pe_host_exchange_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class Engine:
    """One pe_ctx: a GPU, a node-inventory shard, a stream."""

    def __init__(self, device_id: int = 0, rank: int = 0, world_size: int = 1, comm: Optional[bytes] = None,
                 exchange=None, max_nodes: int = 0, gpu_resource_name: str = "amd.com/gpu", topk: int = 0,
                 window_groups: int = 0, window_pods: int = 0, fit_path_mask: int = 0, greedy_flags: int = 0,
                 resort_nodes: int = 0):
        self.lib = _abi.load()
        self._keep = []
        cfg = _abi.PeConfig()
        cfg.device_id = device_id
        cfg.rank = rank
        cfg.world_size = world_size
        if comm is not None:
            cbuf = ctypes.create_string_buffer(bytes(comm), _abi.PE_COMM_ID_BYTES)
            self._keep.append(cbuf)
            cfg.comm_id = ctypes.cast(cbuf, ctypes.c_void_p)
        if isinstance(exchange, HostExchange):   # the native transport: C function + handle
            self._keep.append(exchange)
            cfg.exchange = exchange.fn
            cfg.exchange_user = exchange.h
        elif exchange is not None:
            # exchange(send: bytes) -> bytes (all ranks' blocks concatenated)
            def _cb(user, send, recv, nbytes):
                try:
                    out = exchange(ctypes.string_at(send, nbytes))
                    ctypes.memmove(recv, out, len(out))
                    return 0
                except Exception:  # noqa: BLE001 - reported to the C side as a failure code
                    return 1
            fn = _abi.ALLGATHER_FN(_cb)
            self._keep.append(fn)
            cfg.exchange = fn
        cfg.max_nodes = max_nodes
        self._gname = gpu_resource_name.encode()
        cfg.gpu_resource_name = self._gname
        cfg.topk = topk
        cfg.window_groups = window_groups
        cfg.window_pods = window_pods
        cfg.fit_path_mask = fit_path_mask
        cfg.greedy_flags = greedy_flags
        cfg.resort_nodes = resort_nodes
        self._cfg = cfg
        h = ctypes.c_void_p()
        rc = self.lib.pe_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise PlacementError(rc, "pe_create failed (no GPU? the engine has no CPU fallback)")
        self.h = h
        self.rank, self.world_size = rank, world_size
        self.n_nodes = 0

    def close(self):
        if getattr(self, "h", None):
            self.lib.pe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def _chk(self, rc: int, what: str, ok=(0,)):
        if rc not in ok:
            raise PlacementError(rc, f"{what}: {self.lib.pe_last_error(self.h).decode(errors='replace')}")
        return rc

    # ------------------------------------------------------------ inventory
    def load_nodes(self, cap, used, labels=None, island=None):
        cap = _c(cap, np.int64)
        used = _c(used, np.int64)
        n = cap.shape[1]
        lab = None if labels is None else _c(labels, np.uint32)
        isl = None if island is None else _c(island, np.int32)
        self._chk(self.lib.pe_load_nodes(self.h, n, _p(cap), _p(used), _p(lab), _p(isl)), "pe_load_nodes")
        self.n_nodes = n

    def update_nodes(self, slots, op, cap=None, used=None, labels=None, island=None):
        """pe_update_nodes: per entry op 0 (NODE_SET: cap[i][4], used[i][4], labels, island replace
        the slot) or 1 (NODE_REMOVE).  cap/used are row-major [n][4]."""
        slots = _c(slots, np.int64)
        op = _c(op, np.uint8)
        n = slots.shape[0]
        cap = None if cap is None else _c(cap, np.int64)
        used = None if used is None else _c(used, np.int64)
        lab = None if labels is None else _c(labels, np.uint32)
        isl = None if island is None else _c(island, np.int32)
        self._chk(self.lib.pe_update_nodes(self.h, n, _p(slots), _p(op), _p(cap), _p(used), _p(lab), _p(isl)),
                  "pe_update_nodes")

    def reset_residuals(self):
        self._chk(self.lib.pe_reset_residuals(self.h), "pe_reset_residuals")

    def shard_range(self):
        b, e = ctypes.c_int64(), ctypes.c_int64()
        self._chk(self.lib.pe_shard_range(self.h, ctypes.byref(b), ctypes.byref(e)), "pe_shard_range")
        return b.value, e.value

    def comm_ranks(self) -> int:
        """ncclCommCount of the context's RCCL communicator (0 = host exchange / none)."""
        v = ctypes.c_int32()
        self._chk(self.lib.pe_comm_ranks(self.h, ctypes.byref(v)), "pe_comm_ranks")
        return v.value

    def read_residuals(self) -> np.ndarray:
        b, e = self.shard_range()
        out = np.zeros((4, e - b), dtype=np.int64)
        self._chk(self.lib.pe_read_residuals(self.h, _p(out)), "pe_read_residuals")
        return out

    # ------------------------------------------------------------ aggregation
    def pg_min_resources(self, mode, job_group_off, min_member, group_replicas, group_cont_off, cont_req,
                         cont_flags, allow_overflow=True):
        jgo = _c(job_group_off, np.int32)
        J = len(jgo) - 1
        mm = None if min_member is None else _c(min_member, np.int32)
        rep = _c(group_replicas, np.int32)
        gco = _c(group_cont_off, np.int32)
        req = _c(cont_req, np.int64).reshape(-1, 4)
        fl = _c(cont_flags, np.uint8)
        out = np.zeros((J, 4), dtype=np.int64)
        pres = np.zeros(J, dtype=np.uint8)
        mem = np.zeros(J, dtype=np.int32)
        ovf = np.zeros(J, dtype=np.uint8)
        rc = self.lib.pe_pg_min_resources(self.h, mode, J, _p(jgo), _p(mm), _p(rep), _p(gco), _p(req), _p(fl),
                                          _p(out), _p(pres), _p(mem), _p(ovf))
        self._chk(rc, "pe_pg_min_resources", ok=(0, _abi.PE_EOVERFLOW) if allow_overflow else (0,))
        return out, pres, mem, ovf

    def pg_min_resources_keys(self, mode, job_group_off, min_member, group_replicas, group_cont_off, cont_req,
                              cont_flags, allow_overflow=True):
        """pe_pg_min_resources_keys: cont_req [C][n_keys] int64 (each key at the caller's decimal scale),
        cont_flags [C] u32 = presence bits 0..n_keys-1 | kind << PE_KEYS_KIND_SHIFT.  Returns
        (min_res [J][n_keys], present [J] u16, members, overflow)."""
        jgo = _c(job_group_off, np.int32)
        J = len(jgo) - 1
        mm = None if min_member is None else _c(min_member, np.int32)
        rep = _c(group_replicas, np.int32)
        gco = _c(group_cont_off, np.int32)
        req = np.ascontiguousarray(cont_req, dtype=np.int64)
        if req.ndim != 2:
            raise ValueError("cont_req must be [C][n_keys]")
        nk = req.shape[1]
        fl = _c(cont_flags, np.uint32)
        out = np.zeros((J, nk), dtype=np.int64)
        pres = np.zeros(J, dtype=np.uint16)
        mem = np.zeros(J, dtype=np.int32)
        ovf = np.zeros(J, dtype=np.uint8)
        rc = self.lib.pe_pg_min_resources_keys(self.h, mode, J, nk, _p(jgo), _p(mm), _p(rep), _p(gco), _p(req), _p(fl),
                                               _p(out), _p(pres), _p(mem), _p(ovf))
        self._chk(rc, "pe_pg_min_resources_keys", ok=(0, _abi.PE_EOVERFLOW) if allow_overflow else (0,))
        return out, pres, mem, ovf

    # ------------------------------------------------------------ fit mask
    def jobs_upload(self, req, need=None):
        req = _c(req, np.int64).reshape(-1, 4)
        nd = None if need is None else _c(need, np.uint32)
        self.fit_jobs = req.shape[0]
        self._chk(self.lib.pe_jobs_upload(self.h, req.shape[0], _p(req), _p(nd)), "pe_jobs_upload")

    def fit_mask_run(self):
        self._chk(self.lib.pe_fit_mask_run(self.h), "pe_fit_mask_run")

    def fit_counts(self) -> np.ndarray:
        out = np.zeros(self.fit_jobs, dtype=np.int64)
        self._chk(self.lib.pe_fit_counts(self.h, _p(out)), "pe_fit_counts")
        return out

    def fit_mask(self, req, need=None) -> np.ndarray:
        req = _c(req, np.int64).reshape(-1, 4)
        nd = None if need is None else _c(need, np.uint32)
        counts = np.zeros(req.shape[0], dtype=np.int64)
        dptr, wpr = ctypes.c_void_p(), ctypes.c_int64()
        self._chk(self.lib.pe_fit_mask(self.h, req.shape[0], _p(req), _p(nd), _p(counts), ctypes.byref(dptr),
                                       ctypes.byref(wpr)), "pe_fit_mask")
        self.fit_jobs = req.shape[0]
        self.words_per_row = wpr.value
        return counts

    def fit_mask_layout(self) -> int:
        v = ctypes.c_int32()
        self._chk(self.lib.pe_fit_mask_layout(self.h, ctypes.byref(v)), "pe_fit_mask_layout")
        return v.value

    def fit_mask_row_pitch(self) -> int:
        v = ctypes.c_int64()
        self._chk(self.lib.pe_fit_mask_row_pitch(self.h, ctypes.byref(v)), "pe_fit_mask_row_pitch")
        return v.value

    def fit_mask_rows(self, row0: int, n_rows: int) -> np.ndarray:
        b, e = self.shard_range()
        w = (e - b + 63) // 64
        out = np.zeros((n_rows, w), dtype=np.uint64)
        self._chk(self.lib.pe_fit_mask_rows(self.h, row0, n_rows, _p(out)), "pe_fit_mask_rows")
        return out

    # ------------------------------------------------------------ greedy
    def place_greedy(self, job_group_off, priority, group_count, group_req, group_need=None):
        jgo = _c(job_group_off, np.int32)
        J = len(jgo) - 1
        cnt = _c(group_count, np.int32)
        req = _c(group_req, np.int64).reshape(-1, 4)
        nd = None if group_need is None else _c(group_need, np.uint32)
        P = int(cnt.sum())
        pod = np.full(max(P, 1), -1, dtype=np.int32)
        st = np.zeros(max(J, 1), dtype=np.int32)
        self._chk(self.lib.pe_place_greedy(self.h, J, _p(jgo), _p(_c(priority, np.int32)), _p(cnt), _p(req), _p(nd),
                                           _p(pod), _p(st)), "pe_place_greedy")
        return pod[:P], st[:J]

    def place_batch(self, batch):
        return self.place_greedy(batch.job_group_off, batch.priority, batch.group_count, batch.group_req,
                                 batch.group_need)

    # ------------------------------------------------------------ misc
    def synchronize(self):
        self._chk(self.lib.pe_synchronize(self.h), "pe_synchronize")

    def stream(self) -> int:
        return int(self.lib.pe_stream(self.h) or 0)

    def stats(self) -> dict:
        s = _abi.PeStats()
        self._chk(self.lib.pe_get_stats(self.h, ctypes.byref(s)), "pe_get_stats")
        return s.as_dict()

    def reset_stats(self):
        self._chk(self.lib.pe_reset_stats(self.h), "pe_reset_stats")


class Resolver:
    """pe_resolver_*: the host half of the windowed greedy, driven with externally supplied
    candidate blobs (one block per shard, device merge-kernel layout)."""

    def __init__(self, job_group_off, priority, group_count, group_req, group_need=None):
        self.lib = _abi.load()
        self._jgo = _c(job_group_off, np.int32)
        self.J = len(self._jgo) - 1
        self._cnt = _c(group_count, np.int32)
        self._req = _c(group_req, np.int64).reshape(-1, 4)
        self._need = None if group_need is None else _c(group_need, np.uint32)
        self.P = int(self._cnt.sum())
        h = ctypes.c_void_p()
        rc = self.lib.pe_resolver_create(self.J, _p(self._jgo), _p(_c(priority, np.int32)), _p(self._cnt),
                                         _p(self._req), _p(self._need), ctypes.byref(h))
        if rc != 0:
            raise PlacementError(rc, "pe_resolver_create")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.pe_resolver_destroy(self.h)
            self.h = None

    def set_nodes(self, n_nodes: int):
        """pe_resolver_set_nodes: listed / seeded node ids must lie below n_nodes (PE_EINVAL otherwise)."""
        rc = self.lib.pe_resolver_set_nodes(self.h, int(n_nodes))
        if rc != 0:
            raise PlacementError(rc, "pe_resolver_set_nodes")

    def done(self) -> bool:
        return bool(self.lib.pe_resolver_done(self.h))

    def next_window(self, max_groups: int, max_pods: int) -> np.ndarray:
        out = np.zeros(max_groups, dtype=np.int32)
        n = ctypes.c_int32()
        rc = self.lib.pe_resolver_next_window(self.h, max_groups, max_pods, _p(out), ctypes.byref(n))
        if rc != 0:
            raise PlacementError(rc, "pe_resolver_next_window")
        return out[:n.value].copy()

    def resolve(self, groups: np.ndarray, blob: bytes, n_shards: int, topk: int, seeds=None):
        """seeds: [n][6] int64 {node id, res[0..3], labels} -- nodes changed since the snapshot the
        blob was scanned on, current state (pipelined form, pe_resolver_resolve_seeded)."""
        g = _c(groups, np.int32)
        buf = np.frombuffer(blob, dtype=np.uint8)
        cap = max(64, 2 * self.P + 64)
        upd = np.zeros((cap, 5), dtype=np.int64)
        nu, cons = ctypes.c_int64(), ctypes.c_int32()
        if seeds is not None and len(seeds):
            sd = _c(seeds, np.int64).reshape(-1, 6)
            rc = self.lib.pe_resolver_resolve_seeded(self.h, len(g), _p(g), _p(buf), n_shards, topk, sd.shape[0],
                                                     _p(sd), _p(upd), cap, ctypes.byref(nu), ctypes.byref(cons))
        else:
            rc = self.lib.pe_resolver_resolve(self.h, len(g), _p(g), _p(buf), n_shards, topk, _p(upd), cap,
                                              ctypes.byref(nu), ctypes.byref(cons))
        if rc != 0:
            raise PlacementError(rc, "pe_resolver_resolve")
        return upd[:nu.value].copy(), bool(cons.value)

    def results(self):
        pod = np.full(max(self.P, 1), -1, dtype=np.int32)
        st = np.zeros(max(self.J, 1), dtype=np.int32)
        self.lib.pe_resolver_results(self.h, _p(pod), _p(st))
        return pod[:self.P], st[:self.J]
