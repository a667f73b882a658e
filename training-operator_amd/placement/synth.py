"""Synthetic cluster inventories and job batches, integer-only and
deterministic: counter-based splitmix64, identical wherever it is evaluated.

Every quantity is drawn from a discrete set so it is an exact canonical int64
(cpu milli, memory bytes, gpu count, ephemeral-storage bytes).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
GiB = 1 << 30
TiB = 1 << 40

# cfg seeds
SEED = {"cfg2": 2, "cfg3": 3, "cfg4": 4, "cfg5": 5}


def mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def stream(seed: int, sid: int, n: int) -> np.ndarray:
    """splitmix64 sequence #sid of `seed`: x_i = mix64(base + (i+1)*GOLD), base = mix64(seed*GOLD + sid)."""
    with np.errstate(over="ignore"):
        base = mix64(np.uint64(seed) * GOLD + np.uint64(sid))
        i = np.arange(1, n + 1, dtype=np.uint64)
        return mix64(base + i * GOLD)


def pick(table, r: np.ndarray) -> np.ndarray:
    t = np.asarray(table, dtype=np.int64)
    return t[(r % np.uint64(len(t))).astype(np.int64)]


@dataclass
class Inventory:
    cap: np.ndarray      # [4][N] int64
    used: np.ndarray     # [4][N] int64
    labels: np.ndarray   # [N] uint32  bit0 = gpu product (mi355x), bits1-3 = zone one-hot
    island: np.ndarray   # [N] int32   xGMI island id (= node id on GPU nodes, -1 otherwise)

    @property
    def n(self) -> int:
        return int(self.cap.shape[1])

    def residual(self) -> np.ndarray:
        return self.cap - self.used


def make_inventory(n: int, seed: int, gpu_frac: float = 0.2) -> Inventory:
    is_gpu = (stream(seed, 1, n) % np.uint64(1000)) < np.uint64(int(round(gpu_frac * 1000)))
    cap = np.empty((4, n), dtype=np.int64)
    cap[0] = np.where(is_gpu, pick([128_000, 192_000], stream(seed, 2, n)),
                      pick([32_000, 64_000, 96_000, 128_000], stream(seed, 3, n)))
    cap[1] = np.where(is_gpu, pick([1 * TiB, 2 * TiB], stream(seed, 4, n)),
                      pick([128 * GiB, 256 * GiB, 512 * GiB], stream(seed, 5, n)))
    cap[2] = np.where(is_gpu, 8, 0)
    cap[3] = np.where(is_gpu, pick([2 * TiB, 4 * TiB], stream(seed, 6, n)),
                      pick([512 * GiB, 1 * TiB], stream(seed, 7, n)))
    used = np.empty_like(cap)
    for d in range(4):
        u = (stream(seed, 10 + d, n) % np.uint64(12)).astype(np.int64)
        used[d] = cap[d] * u // 16
    zone = (stream(seed, 14, n) % np.uint64(3)).astype(np.uint32)
    labels = (is_gpu.astype(np.uint32) | (np.uint32(1) << (np.uint32(1) + zone))).astype(np.uint32)
    island = np.where(is_gpu, np.arange(n, dtype=np.int32), -1).astype(np.int32)
    labels = island_labels(labels, island)
    return Inventory(cap, used, labels, island)


CPU_REQ = [500, 1000, 2000, 4000, 8000, 16000]
MEM_REQ = [g * GiB for g in (1, 2, 4, 8, 16, 32, 64, 128)]
GPU_REQ = [0, 0, 0, 0, 1, 2, 4, 8]
EPH_REQ = [0, 10 * GiB, 50 * GiB, 100 * GiB]


LABEL_ISLAND = np.uint32(1 << 31)   # placement.h PE_LABEL_ISLAND / PE_NEED_ISLAND


def island_labels(labels, island):
    """Node labels as the engine keeps them: bit 31 = the node has an xGMI island (island >= 0)."""
    lab = np.asarray(labels, dtype=np.uint32) & ~LABEL_ISLAND
    return np.where(np.asarray(island) >= 0, lab | LABEL_ISLAND, lab).astype(np.uint32)


def scan_requests(batch: "JobBatch") -> np.ndarray:
    """[G][4] the request each group's candidate lists are scanned for (the resolver's scan_req):
    the pod request, or count x request for an island group (saturated at INT64_MAX on overflow,
    which fits nowhere)."""
    req = np.array(batch.group_req, dtype=np.int64, copy=True)
    isl = (np.asarray(batch.group_need, dtype=np.uint32) & LABEL_ISLAND) != 0
    for g in np.nonzero(isl)[0]:
        c = max(int(batch.group_count[g]), 0)
        req[g] = [min(int(v) * c, (1 << 63) - 1) for v in batch.group_req[g]]
    return req


def pod_requests(seed: int, sid: int, n: int):
    """n pod request vectors [n][4] + label need (bit0 when a GPU is requested)."""
    req = np.empty((n, 4), dtype=np.int64)
    req[:, 0] = pick(CPU_REQ, stream(seed, sid, n))
    req[:, 1] = pick(MEM_REQ, stream(seed, sid + 1, n))
    req[:, 2] = pick(GPU_REQ, stream(seed, sid + 2, n))
    req[:, 3] = pick(EPH_REQ, stream(seed, sid + 3, n))
    need = (req[:, 2] > 0).astype(np.uint32)
    return req, need


@dataclass
class JobBatch:
    """Flattened gang batch: groups of identical pods, CSR over jobs (group order = v1 order)."""
    job_group_off: np.ndarray  # [J+1] int32
    priority: np.ndarray       # [J]   int32
    group_count: np.ndarray    # [G]   int32 pods to place
    group_req: np.ndarray      # [G][4] int64
    group_need: np.ndarray     # [G]   uint32
    kind: np.ndarray           # [J]   int8  0 pytorch, 1 mpi, 2 jax, 3 gpu-gang

    @property
    def n_jobs(self) -> int:
        return int(self.priority.shape[0])

    @property
    def n_pods(self) -> int:
        return int(self.group_count.sum())


def make_jobs(n_jobs: int, seed: int, mix: str = "pytorch") -> JobBatch:
    """mix: 'pytorch' (cfg2: Master 1 + Worker W in [0,15]),
            'mixed'   (cfg3: 50% PyTorch, 25% MPI {Launcher 1 (1 cpu, 2Gi), Worker W}, 25% JAX {Worker W+1}),
            'gang8'   (cfg4: one group of M in {1,2,4,8,16} pods x 8 GPUs, requires label bit0),
            'island8' (cfg4: 8-GPU gang jobs on single-node xGMI islands: one island group of M in
                       {1,2,4,8} pods x 8/M GPUs, all on one island node; with probability 1/4 a
                       multi-node gang of M in {2,4} whole-node pods instead)."""
    J = n_jobs
    pri = (stream(seed, 100, J) % np.uint64(1000)).astype(np.int32)
    w = (stream(seed, 101, J) % np.uint64(16)).astype(np.int32)
    if mix == "pytorch":
        kind = np.zeros(J, dtype=np.int8)
    elif mix == "mixed":
        k = (stream(seed, 102, J) % np.uint64(4)).astype(np.int64)
        kind = np.select([k < 2, k == 2], [0, 1], 2).astype(np.int8)
    elif mix in ("gang8", "island8"):
        kind = np.full(J, 3, dtype=np.int8)
    else:
        raise ValueError(mix)
    ngroups = np.where(kind <= 1, 2, 1).astype(np.int32)
    off = np.zeros(J + 1, dtype=np.int32)
    np.cumsum(ngroups, out=off[1:])
    G = int(off[-1])
    a_req, a_need = pod_requests(seed, 200, J)   # leader group (Master / Launcher)
    b_req, b_need = pod_requests(seed, 300, J)   # worker group
    count = np.empty(G, dtype=np.int32)
    req = np.empty((G, 4), dtype=np.int64)
    need = np.empty(G, dtype=np.uint32)
    first = off[:-1]
    two = ngroups == 2
    # two-group jobs: [leader, worker]
    count[first[two]] = 1
    req[first[two]] = a_req[two]
    need[first[two]] = a_need[two]
    mpi = two & (kind == 1)
    req[first[mpi]] = np.array([1000, 2 * GiB, 0, 0], dtype=np.int64)
    need[first[mpi]] = 0
    count[first[two] + 1] = w[two]
    req[first[two] + 1] = b_req[two]
    need[first[two] + 1] = b_need[two]
    one = ~two
    if mix == "gang8":
        m = pick([1, 2, 4, 8, 16], stream(seed, 103, J)).astype(np.int32)
        count[first] = m
        req[first, 0] = pick([32_000, 64_000, 96_000], stream(seed, 104, J))
        req[first, 1] = pick([256 * GiB, 512 * GiB], stream(seed, 105, J))
        req[first, 2] = 8
        req[first, 3] = 100 * GiB
        need[first] = 1
    elif mix == "island8":
        m = pick([1, 2, 4, 8], stream(seed, 103, J)).astype(np.int64)
        multi = (stream(seed, 106, J) % np.uint64(4)) == 0
        count[first] = np.where(multi, pick([2, 4], stream(seed, 107, J)), m)
        # an island job's totals are a gang8 pod's (8 GPUs, 32-96 cores, 256/512 GiB, 100 GiB eph)
        # split evenly over its M pods; a multi-node gang's pods each take a whole node's GPUs
        cpu = pick([32_000, 64_000, 96_000], stream(seed, 104, J))
        mem = pick([256 * GiB, 512 * GiB], stream(seed, 105, J))
        req[first, 0] = np.where(multi, cpu, cpu // m)
        req[first, 1] = np.where(multi, mem, mem // m)
        req[first, 2] = np.where(multi, 8, 8 // m)
        req[first, 3] = np.where(multi, 100 * GiB, 100 * GiB // m)
        need[first] = np.where(multi, 1, 1 | (1 << 31)).astype(np.uint32)
    else:
        count[first[one]] = w[one] + 1      # JAX Worker W+1
        req[first[one]] = b_req[one]
        need[first[one]] = b_need[one]
    return JobBatch(off, pri, count, req, need, kind)


def make_fit_jobs(n_jobs: int, seed: int):
    """cfg5: one request vector (the trainer pod) per job."""
    return pod_requests(seed, 500, n_jobs)


MiB = 1 << 20


def make_fit_jobs_worst(n_jobs: int, seed: int, unique_dims=(1,)):
    """cfg5-sized batch with high-cardinality requests (the fit mask's hard case): every dimension in
    `unique_dims` gets a value unique to each job (memory: distinct MiB counts in [0.5, 256) GiB;
    cpu: distinct milli counts; ephemeral: distinct MiB counts), cpu and ephemeral-storage that are
    not unique are uniform over 1000 / 100 values (100m steps up to 100 cores, 1 GiB steps), gpu and
    the label need as in cfg5."""
    req, need = pod_requests(seed, 500, n_jobs)
    J = n_jobs
    perm = (stream(seed, 520, J) % np.uint64(1 << 62)).argsort(kind="stable").astype(np.int64)  # a permutation
    req[:, 0] = 100 * (1 + (stream(seed, 521, J) % np.uint64(1000)).astype(np.int64))
    req[:, 3] = GiB * (stream(seed, 523, J) % np.uint64(100)).astype(np.int64)
    if 0 in unique_dims:
        req[:, 0] = 100 + perm                               # J distinct milli values
    if 1 in unique_dims:
        req[:, 1] = (512 + perm * ((256 * 1024 - 512) // max(J, 1))) * MiB
    if 3 in unique_dims:
        req[:, 3] = perm * 7 * MiB
    return req, need


def make_pg_batch(n_jobs: int, seed: int):
    """Aggregation batch (pe_pg_min_resources CSR, v1): PyTorchJob-like jobs, Master 1 + Worker W
    (W in [0, 63]), one or two containers per pod (a trainer + an optional sidecar-style helper),
    cpu/memory always present, gpu on GPU jobs, minMember = total replicas or a random smaller
    MinAvailable.  Returns (job_group_off, min_member, group_replicas, group_cont_off, cont_req,
    cont_flags)."""
    J = n_jobs
    w = (stream(seed, 600, J) % np.uint64(64)).astype(np.int32)
    two_ctr = (stream(seed, 601, J) % np.uint64(2)).astype(bool)
    req, _ = pod_requests(seed, 610, J)
    total = 1 + w
    mm = np.where(stream(seed, 602, J) % np.uint64(4) == 0,
                  1 + (stream(seed, 603, J) % total.astype(np.uint64)).astype(np.int32), total).astype(np.int32)
    jgo = (2 * np.arange(J + 1)).astype(np.int32)
    rep = np.empty(2 * J, np.int32)
    rep[0::2] = 1
    rep[1::2] = w
    nct = np.where(two_ctr, 2, 1).astype(np.int32)
    per_group = np.repeat(nct, 2)
    gco = np.zeros(2 * J + 1, np.int32)
    np.cumsum(per_group, out=gco[1:])
    C = int(gco[-1])
    cont = np.zeros((C, 4), np.int64)
    flags = np.zeros(C, np.uint8)
    first = gco[:-1]
    g_req = np.repeat(req, 2, axis=0)
    cont[first] = g_req
    gpu = g_req[:, 2] > 0
    flags[first] = np.where(gpu, 0b1111, 0b1011)
    helper = first[per_group == 2] + 1
    cont[helper] = [250, 256 * MiB, 0, 0]
    flags[helper] = 0b0011
    return jgo, mm, rep, gco, cont, flags
