"""Edge cases of the kueue v0.6.3 TotalRequests pod formula, with
answers derived by hand from the formula the reference calls at pkg/runtime.v2/runtime.go:134:

    sidecars = sum of init containers with restartPolicy Always
    initMax  = max over the other init containers i of (init_i + sidecars declared BEFORE i)
    total    = max(sidecars + sum(containers), initMax) + overhead          (per key, union of keys)

kueue is not in the container; the reference's own tests pin only the 15 / 40 / 31 cases
(tests/golden).  These cases pin the ordering, overhead, key-union and zero-key behaviour the
restatement (oracle/semantics.py total_requests) and the kernel must share; each `want` is written
out, not computed.  TEST INFRASTRUCTURE only."""

SIDE = "Always"

CASES = [
    # sidecar ordering: B only sees S1+S2, A only S1 -> initMax = max(8 + 2, 1 + 5) = 10;
    # sidecars + containers = 5 + 4 = 9 -> 10 (ignoring the order would give 13)
    ("sidecar_order", {"initContainers": [{"requests": {"cpu": "2"}, "restartPolicy": SIDE},
                                          {"requests": {"cpu": "8"}},
                                          {"requests": {"cpu": "3"}, "restartPolicy": SIDE},
                                          {"requests": {"cpu": "1"}}],
                       "containers": [{"requests": {"cpu": "4"}}]},
     {"cpu": 10_000}),
    # a sidecar declared after every init container counts only in the main sum: max(8, 3 + 6) = 9
    ("sidecar_last", {"initContainers": [{"requests": {"cpu": "8"}},
                                         {"requests": {"cpu": "3"}, "restartPolicy": SIDE}],
                      "containers": [{"requests": {"cpu": "6"}}]},
     {"cpu": 9_000}),
    # overhead is added after the max, to every key it names
    ("overhead", {"containers": [{"requests": {"cpu": "1", "memory": "1Gi"}}],
                  "overhead": {"cpu": "250m", "memory": "64Mi"}},
     {"cpu": 1_250, "memory": (1 << 30) + (64 << 20)}),
    # overhead-only key, and overhead on top of an init maximum
    ("overhead_over_init", {"initContainers": [{"requests": {"cpu": "7"}}],
                            "containers": [{"requests": {"cpu": "2"}}],
                            "overhead": {"cpu": "500m", "ephemeral-storage": "1Gi"}},
     {"cpu": 7_500, "ephemeral-storage": 1 << 30}),
    # keys are a union; a zero-valued key stays present
    ("key_union_zero", {"initContainers": [{"requests": {"memory": "2Gi"}}],
                        "containers": [{"requests": {"cpu": "0"}}]},
     {"cpu": 0, "memory": 2 << 30}),
    # the max is per key: cpu from the init container, memory from the main containers
    ("per_key_max", {"initContainers": [{"requests": {"cpu": "8", "memory": "1Gi"}}],
                     "containers": [{"requests": {"cpu": "2", "memory": "4Gi"}}]},
     {"cpu": 8_000, "memory": 4 << 30}),
    # accelerators: init A (1) before sidecar S (1): max(1 + 0, 1 + 2) = 3
    ("gpu_sidecar", {"initContainers": [{"requests": {"nvidia.com/gpu": "1"}},
                                        {"requests": {"nvidia.com/gpu": "1"}, "restartPolicy": SIDE}],
                     "containers": [{"requests": {"nvidia.com/gpu": "2"}}]},
     {"nvidia.com/gpu": 3}),
    # containers without requests contribute no keys; limits are ignored by kueue's requests-only sum
    ("nil_requests", {"initContainers": [{"limits": {"cpu": "9"}}],
                      "containers": [{"limits": {"cpu": "4"}}, {"requests": {"memory": "1Gi"}}]},
     {"memory": 1 << 30}),
    # several sidecars accumulate for later init containers and for the main sum
    ("sidecar_chain", {"initContainers": [{"requests": {"cpu": "1"}, "restartPolicy": SIDE},
                                          {"requests": {"cpu": "1"}, "restartPolicy": SIDE},
                                          {"requests": {"cpu": "5"}},
                                          {"requests": {"cpu": "1"}, "restartPolicy": SIDE}],
                       "containers": [{"requests": {"cpu": "1"}}]},
     {"cpu": 7_000}),
    # empty pod
    ("empty", {}, {}),
]
