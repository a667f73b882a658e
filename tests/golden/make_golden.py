#!/usr/bin/env python3
"""Generates the golden PodGroup fixtures in tests/golden/*.json.

The reference is Go and cannot be compiled or run here (no Go toolchain, dependencies not
vendored -- SURVEY.md sec. 0.3), so these fixtures are TRANSCRIPTIONS: the inputs built by the
reference's own test wrappers and the answers its tests assert, written down as data with the
file:line they come from.  Cases marked "pinned": false have no reference assertion; their
expected values are derived by hand from the cited source and are listed so
the edge cases are covered, not as parity evidence.

Quantities are kept as the strings the reference wrote (resource.MustParse inputs); the tests
parse them exactly (fractions) and compare by value, as go-cmp does through Quantity.Equal.
Run:  python tests/golden/make_golden.py   (rewrites the JSON files next to this script)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

CPU1 = {"cpu": "1"}
CPU1_MEM4 = {"cpu": "1", "memory": "4Gi"}


def initializer_pod(init_req):
    # pkg/util.v2/testing/wrapper.go:495-528 (MakeTrainingRuntimeWrapper) + :741-756
    # (InitContainerDatasetModelInitializer sets Requests on BOTH init containers);
    # busybox container has no resources (plugins/jobset/constants.go:20-23).
    return {"initContainers": [{"name": "dataset-initializer", "requests": init_req},
                               {"name": "model-initializer", "requests": init_req}],
            "containers": [{"name": "busybox"}]}


def trainer_pod(req):
    # wrapper.go:529-551 + :706-720 (ContainerTrainer sets Requests of the trainer container)
    return {"containers": [{"name": "trainer", "requests": req}]}


V2_TOTAL_REQUESTS = {
    "source": "pkg/runtime.v2/runtime_test.go:31-121 TestNewInfo (pinned)",
    "cases": [
        {"name": "all arguments are specified", "ref": "pkg/runtime.v2/runtime_test.go:37-104", "pinned": True,
         "pod_spec_replicas": [
             ["initializer", 1, {"initContainers": [{"requests": {"cpu": "5"}, "restartPolicy": "Always"}],
                                 "containers": [{"requests": {"cpu": "10"}}]}],
             ["trainer-node", 10, {"initContainers": [{"requests": {"cpu": "15"}, "restartPolicy": "Always"}],
                                   "containers": [{"requests": {"cpu": "25"}}]}]],
         "want": {"initializer": {"Replicas": 1, "PodRequests": {"cpu": "15"}},
                  "trainer-node": {"Replicas": 10, "PodRequests": {"cpu": "40"}}}},
        {"name": "all arguments are not specified", "ref": "pkg/runtime.v2/runtime_test.go:105-107", "pinned": True,
         "pod_spec_replicas": [], "want": {}},
    ],
}

V2_ENFORCE_ML_POLICY = {
    "source": "pkg/runtime.v2/framework/core/framework_test.go:154-253 TestRunEnforceMLPolicyPlugins (pinned)",
    "cases": [
        {"name": "plainml MLPolicy is applied to runtime.Info, TrainJob doesn't have numNodes",
         "ref": "framework_test.go:161-191", "pinned": True,
         "ml_policy": {"numNodes": 100, "source": "plainml"}, "trainjob_num_nodes": None,
         "replicas": {"initializer": 1, "trainer-node": 10},
         "want_replicas": {"initializer": 1, "trainer-node": 100}},
        {"name": "plainml MLPolicy is applied to runtime.Info, TrainJob has numNodes",
         "ref": "framework_test.go:192-226", "pinned": True,
         "ml_policy": {"numNodes": 100, "source": "plainml"}, "trainjob_num_nodes": 30,
         "replicas": {"initializer": 1, "trainer-node": 10},
         "want_replicas": {"initializer": 1, "trainer-node": 30}},
        {"name": "registry is empty", "ref": "framework_test.go:227-245", "pinned": True,
         "ml_policy": None, "trainjob_num_nodes": None,
         "replicas": {"initializer": 1, "trainer-node": 10},
         "want_replicas": {"initializer": 1, "trainer-node": 10}},
        {"name": "mpi MLPolicy leaves replicas untouched", "ref": "plugins/mpi/mpi.go:50-56", "pinned": False,
         "ml_policy": {"numNodes": 4, "source": "mpi"}, "trainjob_num_nodes": 8,
         "replicas": {"initializer": 1, "trainer-node": 1},
         "want_replicas": {"initializer": 1, "trainer-node": 1}},
        {"name": "torch MLPolicy without numNodes defaults to 1", "ref": "plugins/torch/torch.go:118-132",
         "pinned": False, "ml_policy": {"numNodes": None, "source": "torch"}, "trainjob_num_nodes": None,
         "replicas": {"initializer": 1, "trainer-node": 7},
         "want_replicas": {"initializer": 1, "trainer-node": 1}},
    ],
}

# End-to-end v2: runtime template -> NewInfo -> EnforceMLPolicy -> CoScheduling.Build
V2_PODGROUP = {
    "source": "reference v2 tests asserting a scheduler-plugins PodGroup (pinned)",
    "cases": [
        {"name": "TrainingRuntime NumNodes 100, TrainJob NumNodes 30",
         "ref": "pkg/runtime.v2/core/trainingruntime_test.go:51-98", "pinned": True,
         "replicated_jobs": [["initializer", initializer_pod(CPU1)], ["trainer-node", trainer_pod(CPU1)]],
         "ml_policy": {"numNodes": 100, "source": "plainml"}, "trainjob_num_nodes": 30,
         "coscheduling": {"scheduleTimeoutSeconds": 120},
         "want": {"minMember": 31, "minResources": {"cpu": "31"}, "scheduleTimeoutSeconds": 120}},
        {"name": "ClusterTrainingRuntime NumNodes 100, TrainJob without NumNodes",
         "ref": "pkg/runtime.v2/core/clustertrainingruntime_test.go:47-83", "pinned": True,
         "replicated_jobs": [["initializer", initializer_pod(CPU1)], ["trainer-node", trainer_pod(CPU1)]],
         "ml_policy": {"numNodes": 100, "source": "plainml"}, "trainjob_num_nodes": None,
         "coscheduling": {"scheduleTimeoutSeconds": 120},
         "want": {"minMember": 101, "minResources": {"cpu": "101"}, "scheduleTimeoutSeconds": 120}},
        {"name": "integration: TrainJob with TrainingRuntime (1 CPU, 4Gi per replica)",
         "ref": "test/integration/controller.v2/trainjob_controller_test.go:106-157", "pinned": True,
         "replicated_jobs": [["initializer", initializer_pod(CPU1_MEM4)], ["trainer-node", trainer_pod(CPU1_MEM4)]],
         "ml_policy": {"numNodes": 100, "source": "plainml"}, "trainjob_num_nodes": None,
         "coscheduling": {"scheduleTimeoutSeconds": 100},
         "want": {"minMember": 101, "minResources": {"cpu": "101", "memory": "404Gi"},
                  "scheduleTimeoutSeconds": 100}},
        {"name": "no coscheduling policy -> nothing to build",
         "ref": "coscheduling.go:104-106", "pinned": False,
         "replicated_jobs": [["trainer-node", trainer_pod(CPU1)]],
         "ml_policy": {"numNodes": 3, "source": "plainml"}, "trainjob_num_nodes": None,
         "coscheduling": None, "want": None},
    ],
}

# Build() directly on a runtime.Info (framework_test.go feeds Info, not a template)
V2_BUILD_FROM_INFO = {
    "source": "pkg/runtime.v2/framework/core/framework_test.go:398-486 (pinned)",
    "cases": [
        {"name": "succeeded to build PodGroup and JobSet with NumNodes from TrainJob",
         "ref": "framework_test.go:398-486", "pinned": True,
         "total_requests": {"initializer": {"Replicas": 1, "PodRequests": CPU1_MEM4},
                            "trainer-node": {"Replicas": 1, "PodRequests": CPU1_MEM4}},
         "ml_policy": {"numNodes": 10, "source": "plainml"}, "trainjob_num_nodes": 100,
         "coscheduling": {"scheduleTimeoutSeconds": 300},
         "want_replicas": {"initializer": 1, "trainer-node": 100},
         "want": {"minMember": 101, "minResources": {"cpu": "101", "memory": "404Gi"},
                  "scheduleTimeoutSeconds": 300}},
        {"name": "replicas zero keeps keys (value 0)", "ref": "coscheduling.go:110-117", "pinned": False,
         "total_requests": {"initializer": {"Replicas": 0, "PodRequests": {"cpu": "2", "memory": "1Gi"}},
                            "trainer-node": {"Replicas": 3, "PodRequests": {"cpu": "500m"}}},
         "ml_policy": None, "trainjob_num_nodes": None, "coscheduling": {"scheduleTimeoutSeconds": None},
         "want_replicas": {"initializer": 0, "trainer-node": 3},
         "want": {"minMember": 3, "minResources": {"cpu": "1500m", "memory": "0"},
                  "scheduleTimeoutSeconds": None}},
    ],
}


def mnist_replicas(n_workers):
    # examples/pytorch/mnist/v1/pytorch_job_mnist_nccl.yaml:7-30: Master 1 + Worker, containers with
    # resources.limits {nvidia.com/gpu: 1} and NO requests (nil map -> limits fallback, util.go:90-92).
    ctr = {"name": "pytorch", "limits": {"nvidia.com/gpu": "1"}}
    return {"Master": {"replicas": 1, "template": {"containers": [ctr]}},
            "Worker": {"replicas": n_workers, "template": {"containers": [ctr]}}}


def sdk_gang_replicas():
    # sdk/python/test/e2e/test_e2e_pytorchjob.py:54-75,342-348: Master 1 + Worker 1, container limits
    # {memory: 2Gi, cpu: 0.8}, no requests.
    ctr = {"name": "pytorch", "limits": {"memory": "2Gi", "cpu": "0.8"}}
    return {"Master": {"replicas": 1, "template": {"containers": [ctr]}},
            "Worker": {"replicas": 1, "template": {"containers": [ctr]}}}


V1_PODGROUP = {
    "source": ("v1 CalcPGMinResources has NO reference test (util_test.go covers only GenGeneralName/MaxInt; "
               "every v1 envtest suite disables gang scheduling). Expected values below are derived by hand "
               "from pkg/controller.v1/common/util.go:79-145 and job.go:250-277 -- parity unpinned."),
    "gpu_resource_name": "nvidia.com/gpu",
    "cases": [
        {"name": "mnist nccl Master 1 + Worker 1 (limits only)", "ref": "examples/pytorch/mnist/v1/pytorch_job_mnist_nccl.yaml:7-30",
         "pinned": False, "replicas": mnist_replicas(1), "scheduling_policy": None,
         "want_min_member": 2, "want": {"nvidia.com/gpu": "2"}},
        {"name": "mnist Master 1 + Worker 3", "ref": "examples/pytorch/mnist/v1/pytorch_job_mnist_nccl.yaml", "pinned": False,
         "replicas": mnist_replicas(3), "scheduling_policy": None, "want_min_member": 4, "want": {"nvidia.com/gpu": "4"}},
        {"name": "mnist Master 1 + Worker 7", "ref": "examples/pytorch/mnist/v1/pytorch_job_mnist_nccl.yaml", "pinned": False,
         "replicas": mnist_replicas(7), "scheduling_policy": None, "want_min_member": 8, "want": {"nvidia.com/gpu": "8"}},
        {"name": "mnist Master 1 + Worker 15", "ref": "examples/pytorch/mnist/v1/pytorch_job_mnist_nccl.yaml", "pinned": False,
         "replicas": mnist_replicas(15), "scheduling_policy": None, "want_min_member": 16, "want": {"nvidia.com/gpu": "16"}},
        {"name": "sdk e2e gang spec, min_available 10 (loop caps at the 2 real pods)",
         "ref": "sdk/python/test/e2e/test_e2e_pytorchjob.py:82-88,342-348", "pinned": False,
         "replicas": sdk_gang_replicas(), "scheduling_policy": {"minAvailable": 10},
         "want_min_member": 10, "want": {"cpu": "1600m", "memory": "4Gi"}},
        {"name": "sdk e2e gang spec, min_available 2", "ref": "sdk/python/test/e2e/test_e2e_pytorchjob.py:89-95",
         "pinned": False, "replicas": sdk_gang_replicas(), "scheduling_policy": {"minAvailable": 2},
         "want_min_member": 2, "want": {"cpu": "1600m", "memory": "4Gi"}},
        {"name": "minAvailable 1 counts only the first type in order (name asc on a tie)", "ref": "util.go:124-141",
         "pinned": False, "replicas": {"Master": {"replicas": 1, "template": {"containers": [{"requests": {"cpu": "2"}}]}},
                                       "Worker": {"replicas": 4, "template": {"containers": [{"requests": {"cpu": "1"}}]}}},
         "scheduling_policy": {"minAvailable": 1}, "want_min_member": 1, "want": {"cpu": "2"},
         "want_any_of": [{"cpu": "2"}, {"cpu": "1"}]},
        {"name": "empty non-nil requests do not fall back to limits", "ref": "util.go:90-92", "pinned": False,
         "replicas": {"Worker": {"replicas": 2, "template": {"containers": [{"requests": {}, "limits": {"cpu": "4"}}]}}},
         "scheduling_policy": None, "want_min_member": 2, "want": {}},
        {"name": "nil replicas type is skipped by the pod loop but counted in minMember", "ref": "util.go:129-131; k8sutil.go:126-137",
         "pinned": False, "replicas": {"Master": {"replicas": None, "template": {"containers": [{"requests": {"cpu": "8"}}]}},
                                       "Worker": {"replicas": 2, "template": {"containers": [{"requests": {"cpu": "1", "memory": "0"}}]}}},
         "scheduling_policy": None, "want_min_member": 3, "want": {"cpu": "2", "memory": "0"}},
        {"name": "explicit MinResources is used verbatim", "ref": "job.go:267-269", "pinned": False,
         "replicas": mnist_replicas(1), "scheduling_policy": {"minResources": {"cpu": "7"}},
         "want_min_member": 2, "want": {"cpu": "7"}},
        {"name": "two containers per pod, requests and limits mixed", "ref": "util.go:79-104,133-140", "pinned": False,
         "replicas": {"Launcher": {"replicas": 1, "template": {"containers": [{"requests": {"cpu": "1", "memory": "2Gi"}}]}},
                      "Worker": {"replicas": 3, "template": {"containers": [
                          {"requests": {"cpu": "500m"}, "limits": {"cpu": "1", "nvidia.com/gpu": "1"}},
                          {"limits": {"nvidia.com/gpu": "2", "ephemeral-storage": "10Gi"}}]}}},
         "scheduling_policy": None, "want_min_member": 4,
         "want": {"cpu": "2500m", "memory": "2Gi", "nvidia.com/gpu": "6", "ephemeral-storage": "30Gi"}},
        {"name": "priority class orders types before the cap", "ref": "util.go:112-124", "pinned": False,
         "priorities": {"high": 1000},
         "replicas": {"Worker": {"replicas": 3, "template": {"containers": [{"requests": {"cpu": "1"}}]}},
                      "Master": {"replicas": 1, "template": {"priorityClassName": "high",
                                                             "containers": [{"requests": {"cpu": "16"}}]}}},
         "scheduling_policy": {"minAvailable": 2}, "want_min_member": 2, "want": {"cpu": "17"}},
    ],
}


# Keys outside the four engine dimensions (verdict r5 item 2): the reference sums ANY ResourceName
# (util.go:80-103 AddResourceList, coscheduling.go:112-116), so the engine's key-table path
# (placement.h pe_pg_min_resources_keys) must too.  No reference test uses such keys: the answers are
# derived by hand from the cited code ("pinned": false), and tests/test_oracle_golden.py checks them
# against the object-level restatement (oracle/semantics.py) as well.  "overflow": true marks a case
# whose int64 sum overflows -- the one case the adapters hand to the reference (inf.Dec).
FAT_POD = {"cpu": "2", "memory": "8Gi", "hugepages-2Mi": "1Gi", "rdma/hca": "1", "nvidia.com/gpu": "1"}
MANY_KEYS = dict({f"example.com/r{i:02d}": "1" for i in range(20)}, cpu="1")
WIDE_KEYS = {
    "source": "hand-derived: keys beyond cpu/memory/one accelerator/ephemeral-storage (parity unpinned)",
    "v1": [
        {"name": "hugepages + rdma + gpu, Master 1 + Worker 3", "ref": "util.go:79-104,126-141", "pinned": False,
         "replicas": {"Master": {"replicas": 1, "template": {"containers": [{"requests": FAT_POD}]}},
                      "Worker": {"replicas": 3, "template": {"containers": [
                          {"requests": dict(FAT_POD, **{"hugepages-2Mi": "512Mi"})}]}}},
         "scheduling_policy": None, "want_min_member": 4,
         "want": {"cpu": "8", "memory": "32Gi", "hugepages-2Mi": "2560Mi", "rdma/hca": "4", "nvidia.com/gpu": "4"}},
        {"name": "two accelerator names and cpu in micro-cores", "ref": "util.go:79-104", "pinned": False,
         "replicas": {"Master": {"replicas": 1, "template": {"containers": [
                          {"requests": {"nvidia.com/gpu": "1", "cpu": "1"}}]}},
                      "Worker": {"replicas": 2, "template": {"containers": [
                          {"requests": {"amd.com/gpu": "8", "cpu": "1500u"}}]}}},
         "scheduling_policy": None, "want_min_member": 3,
         "want": {"nvidia.com/gpu": "1", "amd.com/gpu": "16", "cpu": "1003m"}},
        {"name": "cpu finer than 1m under minAvailable", "ref": "job.go:258-260; util.go:126-141", "pinned": False,
         "replicas": {"Worker": {"replicas": 4, "template": {"containers": [
                          {"requests": {"cpu": "250u", "memory": "100Mi"}}]}}},
         "scheduling_policy": {"minAvailable": 2}, "want_min_member": 2,
         "want": {"cpu": "500u", "memory": "200Mi"}},
        {"name": "limits of extended resources when Requests is nil", "ref": "util.go:90-101", "pinned": False,
         "replicas": {"Worker": {"replicas": 2, "template": {"containers": [
                          {"limits": {"rdma/hca": "2", "hugepages-1Gi": "3Gi"}}]}}},
         "scheduling_policy": None, "want_min_member": 2, "want": {"rdma/hca": "4", "hugepages-1Gi": "6Gi"}},
    ],
    "v2": [
        {"name": "hugepages / rdma in init and main containers, 3 trainer nodes",
         "ref": "runtime.go:134 (kueue TotalRequests); coscheduling.go:108-118", "pinned": False,
         "replicated_jobs": [
             ["initializer", {"initContainers": [{"requests": {"cpu": "1", "hugepages-1Gi": "2Gi"}}],
                              "containers": [{"requests": {"cpu": "500m", "rdma/hca": "1"}}]}],
             ["trainer-node", trainer_pod({"cpu": "4", "amd.com/gpu": "8", "rdma/hca": "2", "hugepages-1Gi": "4Gi"})]],
         "ml_policy": {"numNodes": 3, "source": "plainml"}, "trainjob_num_nodes": None,
         "want": {"minMember": 4, "minResources": {"cpu": "13", "hugepages-1Gi": "14Gi", "rdma/hca": "7",
                                                   "amd.com/gpu": "24"}}},
        {"name": "sidecar in micro-cores, an extended key, pod overhead",
         "ref": "runtime.go:134 (kueue TotalRequests); coscheduling.go:108-118", "pinned": False,
         "replicated_jobs": [
             ["trainer-node", {"initContainers": [{"requests": {"cpu": "1500u", "example.com/fpga": "1"},
                                                   "restartPolicy": "Always"}],
                               "containers": [{"requests": {"cpu": "2", "memory": "1Gi"}}],
                               "overhead": {"cpu": "100m"}}]],
         "ml_policy": {"numNodes": 2, "source": "plainml"}, "trainjob_num_nodes": None,
         "want": {"minMember": 2, "minResources": {"cpu": "4203m", "example.com/fpga": "2", "memory": "2Gi"}}},
        {"name": "21 keys: more than one 16-key slice", "ref": "coscheduling.go:112-116", "pinned": False,
         "replicated_jobs": [["trainer-node", trainer_pod(MANY_KEYS)]],
         "ml_policy": {"numNodes": 5, "source": "plainml"}, "trainjob_num_nodes": None,
         "want": {"minMember": 5, "minResources": {k: "5" for k in MANY_KEYS}}},
        {"name": "an int64 overflow is the reference's (inf.Dec) case", "ref": "coscheduling.go:112-116", "pinned": False,
         "replicated_jobs": [["trainer-node", {"containers": [{"requests": {"example.com/huge": "5e18"}},
                                                              {"requests": {"example.com/huge": "1"}}]}]],
         "ml_policy": {"numNodes": 2, "source": "plainml"}, "trainjob_num_nodes": None, "overflow": True,
         "want": {"minMember": 2, "minResources": {"example.com/huge": "10000000000000000002"}}},
    ],
}


def main():
    for name, obj in [("v2_total_requests", V2_TOTAL_REQUESTS), ("v2_enforce_ml_policy", V2_ENFORCE_ML_POLICY),
                      ("v2_podgroup", V2_PODGROUP), ("v2_build_from_info", V2_BUILD_FROM_INFO),
                      ("v1_podgroup", V1_PODGROUP), ("wide_keys", WIDE_KEYS)]:
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(obj, f, indent=1, sort_keys=False)
            f.write("\n")


if __name__ == "__main__":
    main()
