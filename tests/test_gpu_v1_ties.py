"""v1 CalcPGMinResources on the GPU when replica types tie on priority.

The reference orders equal-priority types by Go map iteration, i.e. randomly (util.go:110,124), so
with minMember below the total replicas it can return any of several MinResources.  The engine
breaks ties by type name; for random multi-type jobs its answer must be one of the results the
reference can produce (oracle/semantics.py calc_pg_min_resources_all_orders, every tie permutation),
and exactly the name-ordered one."""
import numpy as np
import pytest

from oracle import flatten as F
from oracle import semantics as S
from placement import V1, Engine

pytestmark = pytest.mark.gpu
GPU = "amd.com/gpu"
TYPES = ["Master", "Worker", "Launcher", "Chief"]
CPU = ["250m", "500m", "1", "2", "1500m", "0"]
MEM = ["512Mi", "1Gi", "2Gi", "3G", "0"]


def random_job(rng):
    types = list(rng.choice(TYPES, size=int(rng.integers(2, 5)), replace=False))
    replicas = {}
    for t in types:
        containers = []
        for _ in range(int(rng.integers(1, 3))):
            kind = int(rng.integers(0, 4))
            res = {"cpu": str(rng.choice(CPU)), "memory": str(rng.choice(MEM))}
            if rng.random() < 0.3:
                res[GPU] = str(int(rng.integers(0, 3)))
            if kind == 0:
                containers.append({"requests": res})
            elif kind == 1:
                containers.append({"limits": res})                    # requests nil -> limits
            elif kind == 2:
                containers.append({"requests": {}, "limits": res})    # empty non-nil: no fallback
            else:
                containers.append({"requests": {"cpu": res["cpu"]}, "limits": res})
        spec = {"template": {"containers": containers, "priorityClassName": str(rng.choice(["", "hi", "lo"]))}}
        if rng.random() < 0.85:
            spec["replicas"] = int(rng.integers(0, 6))
        replicas[t] = spec
    total = S.get_total_replicas(replicas)
    min_member = int(rng.integers(0, total + 2))
    return min_member, replicas


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_v1_equal_priorities_in_reference_result_set(seed):
    rng = np.random.default_rng(seed)
    pri = {"hi": 10, "lo": 10} if seed != 3 else {"hi": 10, "lo": 5}   # seed 3: partial ties
    pc_get = lambda name: pri.get(name)                                # "" -> lookup fails -> 0
    jobs = [random_job(rng) for _ in range(400)]
    flat = F.Flat()
    for mm, replicas in jobs:
        F.add_v1_job(flat, mm, replicas, GPU, pc_get)
    e = Engine(0, gpu_resource_name=GPU)
    out, pres, members, ovf = e.pg_min_resources(V1, *flat.arrays())
    e.close()
    ambiguous = 0
    for j, (mm, replicas) in enumerate(jobs):
        got = F.unflatten(out[j], pres[j], GPU)
        outs = [F.canonical_list(o, GPU) for o in S.calc_pg_min_resources_all_orders(mm, replicas, pc_get)]
        assert got in outs, (j, mm, replicas, got, outs)
        assert got == F.canonical_list(S.calc_pg_min_resources(mm, replicas, pc_get), GPU)
        assert ovf[j] == 0
        ambiguous += len(outs) > 1
    assert ambiguous >= 20          # the ties actually change the answer for a good share of jobs
