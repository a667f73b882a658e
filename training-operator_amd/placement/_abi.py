"""ctypes mirror of include/placement.h -- the Python twin of the cgo stub in INTEGRATION.md.

Loads the in-tree libplacement.so (built by `make -C training-operator_amd/csrc`).  There is no
fallback: a missing library or a machine without a GPU raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("PE_LIBRARY") or os.path.join(PKG_ROOT, "libplacement.so")   # PE_LIBRARY: A/B builds
HEADER = os.path.join(REPO_ROOT, "include", "placement.h")

PE_OK, PE_EINVAL, PE_EOVERFLOW, PE_ENOMEM, PE_EHIP, PE_ERCCL, PE_ESTATE, PE_ENODEV = 0, -1, -2, -3, -4, -5, -6, -7
PE_MODE_V1, PE_MODE_V2 = 1, 2
PE_NODE_SET, PE_NODE_REMOVE = 0, 1
PE_JOB_PLACED, PE_JOB_UNSCHEDULABLE = 0, 1
PE_KIND_CONTAINER, PE_KIND_INIT, PE_KIND_SIDECAR, PE_KIND_OVERHEAD = 0, 1, 2, 3
PE_KIND_SHIFT = 4
PE_MAX_KEYS = 16
PE_KEYS_KIND_SHIFT = 16
PE_COMM_ID_BYTES = 128
PE_DIMS = 4

ERR_NAMES = {PE_EINVAL: "PE_EINVAL", PE_EOVERFLOW: "PE_EOVERFLOW", PE_ENOMEM: "PE_ENOMEM", PE_EHIP: "PE_EHIP",
             PE_ERCCL: "PE_ERCCL", PE_ESTATE: "PE_ESTATE", PE_ENODEV: "PE_ENODEV"}

ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


class PeConfig(ctypes.Structure):
    _fields_ = [("device_id", ctypes.c_int32), ("rank", ctypes.c_int32), ("world_size", ctypes.c_int32),
                ("comm_id", ctypes.c_void_p), ("exchange", ALLGATHER_FN), ("exchange_user", ctypes.c_void_p),
                ("max_nodes", ctypes.c_int64), ("gpu_resource_name", ctypes.c_char_p), ("topk", ctypes.c_int32),
                ("window_groups", ctypes.c_int32), ("window_pods", ctypes.c_int64), ("fit_path_mask", ctypes.c_int32),
                ("greedy_flags", ctypes.c_int32), ("resort_nodes", ctypes.c_int32)]


class PeStats(ctypes.Structure):
    _fields_ = [("fit_evals", ctypes.c_int64), ("scan_evals", ctypes.c_int64), ("windows", ctypes.c_int64),
                ("rescans", ctypes.c_int64), ("groups_scanned", ctypes.c_int64), ("pods_placed", ctypes.c_int64),
                ("jobs_placed", ctypes.c_int64), ("jobs_failed", ctypes.c_int64), ("last_greedy_ms", ctypes.c_double),
                ("greedy_wait_ms", ctypes.c_double), ("greedy_host_ms", ctypes.c_double),
                ("fit_runs_i32", ctypes.c_int64), ("fit_runs_i64", ctypes.c_int64), ("fit_runs_coded", ctypes.c_int64),
                ("fit_runs_therm", ctypes.c_int64), ("fit_runs_planes", ctypes.c_int64), ("resorts", ctypes.c_int64),
                ("fit_runs_lds", ctypes.c_int64), ("fit_runs_sets", ctypes.c_int64), ("walk_rounds", ctypes.c_int64),
                ("walk_overlay", ctypes.c_int64), ("walk_groups", ctypes.c_int64), ("walk_prepass", ctypes.c_int64),
                ("walk_ms", ctypes.c_double), ("walk_pend_updates", ctypes.c_int64),
                ("xchg_zc_windows", ctypes.c_int64), ("xchg_wait_ms", ctypes.c_double),
                ("xchg_merge_ms", ctypes.c_double),
                ("agg_segments", ctypes.c_int64), ("agg_narrow_segments", ctypes.c_int64),
                ("agg_wire_bytes", ctypes.c_int64)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


P = ctypes.c_void_p
i32, i64 = ctypes.c_int32, ctypes.c_int64

# name -> (restype, argtypes); every symbol include/placement.h declares
SIGNATURES = {
    "pe_abi_version": (ctypes.c_int, []),
    "pe_comm_id": (ctypes.c_int, [P]),
    "pe_create": (ctypes.c_int, [ctypes.POINTER(PeConfig), ctypes.POINTER(P)]),
    "pe_destroy": (None, [P]),
    "pe_last_error": (ctypes.c_char_p, [P]),
    "pe_load_nodes": (ctypes.c_int, [P, i64, P, P, P, P]),
    "pe_reset_residuals": (ctypes.c_int, [P]),
    "pe_update_nodes": (ctypes.c_int, [P, i64, P, P, P, P, P, P]),
    "pe_shard_range": (ctypes.c_int, [P, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
    "pe_comm_ranks": (ctypes.c_int, [P, ctypes.POINTER(i32)]),
    "pe_read_residuals": (ctypes.c_int, [P, P]),
    "pe_pg_min_resources": (ctypes.c_int, [P, i32, i64, P, P, P, P, P, P, P, P, P, P]),
    "pe_pg_min_resources_keys": (ctypes.c_int, [P, i32, i64, i32, P, P, P, P, P, P, P, P, P, P]),
    "pe_fit_mask": (ctypes.c_int, [P, i64, P, P, P, ctypes.POINTER(P), ctypes.POINTER(i64)]),
    "pe_jobs_upload": (ctypes.c_int, [P, i64, P, P]),
    "pe_fit_mask_run": (ctypes.c_int, [P]),
    "pe_fit_counts": (ctypes.c_int, [P, P]),
    "pe_fit_mask_rows": (ctypes.c_int, [P, i64, i64, P]),
    "pe_fit_mask_layout": (ctypes.c_int, [P, ctypes.POINTER(i32)]),
    "pe_fit_mask_row_pitch": (ctypes.c_int, [P, ctypes.POINTER(i64)]),
    "pe_place_greedy": (ctypes.c_int, [P, i64, P, P, P, P, P, P, P]),
    "pe_resolver_create": (ctypes.c_int, [i64, P, P, P, P, P, ctypes.POINTER(P)]),
    "pe_resolver_destroy": (None, [P]),
    "pe_resolver_set_nodes": (ctypes.c_int, [P, i64]),
    "pe_resolver_done": (ctypes.c_int, [P]),
    "pe_resolver_next_window": (ctypes.c_int, [P, i32, i64, P, ctypes.POINTER(i32)]),
    "pe_resolver_resolve": (ctypes.c_int, [P, i32, P, P, i32, i32, P, i64, ctypes.POINTER(i64),
                                           ctypes.POINTER(i32)]),
    "pe_resolver_resolve_seeded": (ctypes.c_int, [P, i32, P, P, i32, i32, i64, P, P, i64, ctypes.POINTER(i64),
                                                  ctypes.POINTER(i32)]),
    "pe_resolver_results": (ctypes.c_int, [P, P, P]),
    "pe_synchronize": (ctypes.c_int, [P]),
    "pe_stream": (P, [P]),
    "pe_get_stats": (ctypes.c_int, [P, ctypes.POINTER(PeStats)]),
    "pe_reset_stats": (ctypes.c_int, [P]),
    "pe_host_exchange_open": (ctypes.c_int, [ctypes.c_char_p, i32, i32, ctypes.c_size_t, ctypes.POINTER(P)]),
    "pe_host_exchange_allgather": (ctypes.c_int, [P, P, P, ctypes.c_size_t]),
    "pe_host_exchange_close": (None, [P]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load libplacement.so; raises (never falls back) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"libplacement.so not built at {path}: run `make -C training-operator_amd/csrc` "
                          "(the engine has no CPU fallback)")
    lib = ctypes.CDLL(path)
    # an A/B build named by PE_LIBRARY may predate entry points added since (its callers do not use
    # them); the in-tree library must export every one
    lenient = path != os.path.join(PKG_ROOT, "libplacement.so")
    for name, (res, args) in SIGNATURES.items():
        if lenient and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
