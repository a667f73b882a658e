// Table-driven tests of the C++ host mirror (training-operator_amd/host), written after the
// reference's Go tests.  `--cpu` runs host-logic cases only (no device); `--gpu` runs the cases
// that aggregate on the MI355X through libplacement.
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "kf.h"

using namespace kf;

static int g_fail = 0, g_run = 0;
#define CHECK(cond)                                                                   \
  do {                                                                                \
    if (!(cond)) {                                                                    \
      std::fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);          \
      ++g_fail;                                                                       \
    }                                                                                 \
  } while (0)

struct Case {
  const char* name;
  bool gpu;
  std::function<void()> fn;
};
static std::vector<Case>& cases() {
  static std::vector<Case> c;
  return c;
}
struct Reg {
  Reg(const char* n, bool gpu, std::function<void()> f) { cases().push_back({n, gpu, std::move(f)}); }
};
#define TEST_CPU(name) static void name(); static Reg reg_##name(#name, false, name); static void name()
#define TEST_GPU(name) static void name(); static Reg reg_##name(#name, true, name); static void name()

static ResourceList RL(std::initializer_list<std::pair<const char*, const char*>> kv) {
  ResourceList r;
  for (auto& p : kv) r[p.first] = Quantity::MustParse(p.second);
  return r;
}
static Container Ctr(std::optional<ResourceList> req, std::optional<ResourceList> lim = std::nullopt,
                     std::optional<std::string> restart = std::nullopt) {
  Container c;
  c.requests = std::move(req);
  c.limits = std::move(lim);
  c.restart_policy = std::move(restart);
  return c;
}
static Engine& eng() {
  static Engine e(0, "nvidia.com/gpu");
  return e;
}
static const PriorityClassGetFunc kNoPC = [](const std::string&) { return std::optional<PriorityClass>(); };

// ------------------------------------------------------------------ CPU: Quantity

TEST_CPU(TestQuantityParse) {
  struct {
    const char *s, *res;
    int64_t want;
  } tcs[] = {{"1", "cpu", 1000},         {"500m", "cpu", 500},          {"0.8", "cpu", 800},
             {"4Gi", "memory", 4LL << 30}, {"404Gi", "memory", 404LL << 30}, {"1e3", "memory", 1000},
             {"2k", "memory", 2000},     {"1.5Ki", "memory", 1536},     {"16", "nvidia.com/gpu", 16}};
  for (auto& tc : tcs) CHECK(Quantity::Parse(tc.s).Canonical(tc.res) == tc.want);
  bool threw = false;
  try {
    Quantity::Parse("4Gb");
  } catch (const QuantityError&) {
    threw = true;
  }
  CHECK(threw);
  threw = false;
  try {
    Quantity::Parse("0.0001").Canonical("cpu");   // scale < -3: no exact milli value
  } catch (const QuantityError&) {
    threw = true;
  }
  CHECK(threw);
  CHECK(Quantity::Parse("1").Equal(Quantity::Parse("1000m")));
  CHECK(Quantity::Parse("1Gi").Equal(Quantity::Parse("1073741824")));
  CHECK(!Quantity::Parse("1G").Equal(Quantity::Parse("1Gi")));
  CHECK(Quantity::FromCanonical("cpu", 1600).Equal(Quantity::Parse("1.6")));
  CHECK(Quantity::FromCanonical("memory", 404LL << 30).String() == "404Gi");
}


// apimachinery quantity.go String() (CanonicalizeBytes): canonical print forms
TEST_CPU(TestQuantityString) {
  struct {
    const char *in, *want;
  } tcs[] = {{"0", "0"},           {"1", "1"},          {"1000m", "1"},        {"100m", "100m"},
             {"0.5", "500m"},      {"1.5", "1500m"},    {"0.1", "100m"},       {"10m", "10m"},
             {"1n", "1n"},         {"5u", "5u"},        {"1000", "1k"},        {"1000M", "1G"},
             {"12345", "12345"},   {"12.345", "12345m"}, {"1e3", "1e3"},       {"129e6", "129e6"},
             {"1.5e3", "1500"},    {"1Gi", "1Gi"},      {"1024Mi", "1Gi"},     {"1.5Gi", "1536Mi"},
             {"1536Ki", "1536Ki"}, {"2000Mi", "2000Mi"}, {"0.5Ki", "512"},     {"1Ki", "1Ki"},
             {"100Ki", "100Ki"},   {"1E", "1E"},        {"2k", "2k"},          {"8Gi", "8Gi"}};
  for (auto& tc : tcs) {
    const std::string got = Quantity::Parse(tc.in).String();
    if (got != tc.want) std::fprintf(stderr, "  %s -> %s (want %s)\n", tc.in, got.c_str(), tc.want);
    CHECK(got == tc.want);
  }
  CHECK(Quantity::Parse("4Gi").format() == Format::kBinarySI);
  CHECK(Quantity::Parse("1e3").format() == Format::kDecimalExponent);
  CHECK(Quantity::Parse("1E").format() == Format::kDecimalSI);
  CHECK(Quantity::FromCanonical("memory", 404LL << 30, Format::kBinarySI).String() == "404Gi");
  CHECK(Quantity::FromCanonical("cpu", 101000, Format::kDecimalSI).String() == "101");
  CHECK(Quantity::FromCanonical("cpu", 1600).String() == "1600m");
  // DecimalSI memory that is not a multiple of 1000: plain digits
  CHECK(Quantity::FromCanonical("memory", 1000000000LL + (1LL << 30), Format::kDecimalSI).String() == "2073741824");
}

// util.go:79-104 AddResourceList + quantity.go Add: the first nonzero contribution's format wins
TEST_CPU(TestMinResourcesFormatsV1) {
  ReplicaSpec m, w;
  m.replicas = 1;
  m.template_spec.containers = {Ctr(RL({{"memory", "0"}, {"cpu", "500m"}}))};
  w.replicas = 3;
  w.template_spec.containers = {Ctr(RL({{"memory", "2Gi"}, {"cpu", "1"}}))};
  auto f = MinResourcesFormatsV1(4, {{"Master", m}, {"Worker", w}}, kNoPC);
  CHECK(f.at("memory") == Format::kBinarySI);   // Master's 0 (DecimalSI) adopts Worker's BinarySI
  CHECK(f.at("cpu") == Format::kDecimalSI);
  // a type that counts no pod contributes no format
  ReplicaSpec e;
  e.replicas = 2;
  e.template_spec.containers = {Ctr(RL({{"memory", "1e9"}}))};
  auto g = MinResourcesFormatsV1(1, {{"A", w}, {"B", e}}, kNoPC);
  CHECK(g.at("memory") == Format::kBinarySI && g.size() == 2);
  auto h = MinResourcesFormatsV1(4, {{"A", w}, {"B", e}}, kNoPC);   // A's 3 pods, then one B pod
  CHECK(h.at("memory") == Format::kBinarySI);
}

// Go JSON of the objects the operator sends (field order of the Go types, omitempty, sorted maps)
TEST_CPU(TestPodGroupJSON) {
  PodGroup pg;
  pg.name = "mnist";
  pg.ns = "kubeflow";
  pg.min_member = 2;
  pg.min_resources = {{"nvidia.com/gpu", Quantity::FromCanonical("nvidia.com/gpu", 2, Format::kDecimalSI)}};
  pg.owner_api_version = "kubeflow.org/v1";
  pg.owner_kind = "PyTorchJob";
  pg.owner_name = "mnist";
  pg.owner_uid = "u-1";
  pg.annotations = {{"b", "x<y"}, {"a", "q\"r"}};
  const std::string want_sp =
      "{\"kind\":\"PodGroup\",\"apiVersion\":\"scheduling.x-k8s.io/v1alpha1\",\"metadata\":{\"name\":\"mnist\","
      "\"namespace\":\"kubeflow\",\"creationTimestamp\":null,\"annotations\":{\"a\":\"q\\\"r\",\"b\":\"x\\u003cy\"},"
      "\"ownerReferences\":[{\"apiVersion\":\"kubeflow.org/v1\",\"kind\":\"PyTorchJob\",\"name\":\"mnist\",\"uid\":\"u-1\","
      "\"controller\":true,\"blockOwnerDeletion\":true}]},\"spec\":{\"minMember\":2,\"minResources\":{\"nvidia.com/gpu\":\"2\"}},"
      "\"status\":{\"scheduleStartTime\":null}}";
  CHECK(PodGroupJSON(pg) == want_sp);
  pg.flavour = GangScheduler::kVolcano;
  pg.queue = "default";
  pg.annotations.clear();
  pg.min_resources.clear();
  const std::string want_v =
      "{\"kind\":\"PodGroup\",\"apiVersion\":\"scheduling.volcano.sh/v1beta1\",\"metadata\":{\"name\":\"mnist\","
      "\"namespace\":\"kubeflow\",\"creationTimestamp\":null,\"ownerReferences\":[{\"apiVersion\":\"kubeflow.org/v1\","
      "\"kind\":\"PyTorchJob\",\"name\":\"mnist\",\"uid\":\"u-1\",\"controller\":true,\"blockOwnerDeletion\":true}]},"
      "\"spec\":{\"minMember\":2,\"queue\":\"default\",\"minResources\":{}},\"status\":{}}";
  CHECK(PodGroupJSON(pg) == want_v);
}

// ------------------------------------------------------------------ CPU: flattening (host logic)

static std::map<ReplicaType, ReplicaSpec> mnist(int workers) {
  // examples/pytorch/mnist/v1/pytorch_job_mnist_nccl.yaml:7-30 (limits only, requests nil)
  ReplicaSpec m, w;
  m.replicas = 1;
  m.template_spec.containers = {Ctr(std::nullopt, RL({{"nvidia.com/gpu", "1"}}))};
  w.replicas = workers;
  w.template_spec.containers = {Ctr(std::nullopt, RL({{"nvidia.com/gpu", "1"}}))};
  return {{"Master", m}, {"Worker", w}};
}

TEST_CPU(TestFlattenV1Mnist) {
  Flat f;
  FlattenV1Job(2, mnist(1), kNoPC, &f);
  CHECK((f.job_group_off == std::vector<int32_t>{0, 2}));
  CHECK((f.group_replicas == std::vector<int32_t>{1, 1}));
  CHECK((f.group_cont_off == std::vector<int32_t>{0, 1, 2}));
  CHECK((f.keys == std::vector<std::string>{"nvidia.com/gpu"}));   // limits -> the gpu key present
  CHECK((f.ent_off == std::vector<int32_t>{0, 1, 2}));
  CHECK(f.ent_q[0].Equal(Quantity::Parse("1")) && f.ent_q[1].Equal(Quantity::Parse("1")));
}

TEST_CPU(TestFlattenV1EmptyRequestsDoNotFallBack) {
  // util.go:90-92: an empty non-nil Requests map does not fall back to Limits
  ReplicaSpec w;
  w.replicas = 2;
  w.template_spec.containers = {Ctr(ResourceList{}, RL({{"cpu", "4"}}))};
  Flat f;
  FlattenV1Job(2, {{"Worker", w}}, kNoPC, &f);
  CHECK(f.ent_off.size() == 2 && f.ent_off[1] == 0 && f.keys.empty());
}

TEST_CPU(TestFlattenV1PriorityOrder) {
  ReplicaSpec w, m;
  w.replicas = 3;
  w.template_spec.containers = {Ctr(RL({{"cpu", "1"}}))};
  m.replicas = 1;
  m.template_spec.priority_class_name = "high";
  m.template_spec.containers = {Ctr(RL({{"cpu", "16"}}))};
  PriorityClassGetFunc pc = [](const std::string& n) {
    return n == "high" ? std::optional<PriorityClass>(PriorityClass{1000}) : std::nullopt;
  };
  Flat f;
  FlattenV1Job(2, {{"Worker", w}, {"Master", m}}, pc, &f);
  CHECK(f.ent_q[0].Equal(Quantity::Parse("16")));   // the high-priority Master is counted first
  CHECK((f.group_replicas == std::vector<int32_t>{1, 3}));
}

// Key tables (verdict r5 item 2): any ResourceName flattens -- hugepages, rdma, a second accelerator,
// cpu finer than 1m -- each key at the finest decimal scale its quantities need; only a negative
// quantity is refused (all-or-nothing append).
TEST_CPU(TestFlattenAnyResourceKeyAndScales) {
  ReplicaSpec w;
  w.replicas = 1;
  w.template_spec.containers = {Ctr(RL({{"hugepages-2Mi", "1Gi"}, {"rdma/hca", "1"}, {"cpu", "1500u"}})),
                                Ctr(RL({{"cpu", "2"}, {"amd.com/gpu", "8"}, {"nvidia.com/gpu", "1"}}))};
  Flat f;
  FlattenV1Job(1, {{"Worker", w}}, kNoPC, &f);
  CHECK(f.keys.size() == 5 && f.key_id.count("hugepages-2Mi") && f.key_id.count("amd.com/gpu"));
  const std::vector<int> sc = f.Scales();
  CHECK(sc[f.key_id.at("cpu")] == -4 && sc[f.key_id.at("hugepages-2Mi")] == 0 && sc[f.key_id.at("rdma/hca")] == 0);
  CHECK(Quantity::Parse("1500u").Scaled(-4) == 15 && Quantity::Parse("2").Scaled(-4) == 20000);
  CHECK(Quantity::Parse("1Gi").Scaled(0) == (1LL << 30) && !Quantity::Parse("1500u").Scaled(-3));
  CHECK(Quantity::Parse("5e18").Scaled(0) == 5000000000000000000LL && !Quantity::Parse("1e19").Scaled(0));
  CHECK(Quantity::Parse("1e19").Scaled(19) == 1 && Quantity::Parse("3k").Exp10() == 3 && Quantity::Parse("1.5Ki").Exp10() == 0);
  CHECK(Quantity::FromScaled(1003, -3, Format::kDecimalSI).String() == "1003m");
  CHECK(Quantity::FromScaled(2560LL << 20, 0, Format::kBinarySI).String() == "2560Mi");
  ReplicaSpec bad;
  bad.replicas = 1;
  bad.template_spec.containers = {Ctr(RL({{"cpu", "-1"}}))};
  bool threw = false;
  try {
    FlattenV1Job(1, {{"Worker", bad}}, kNoPC, &f);
  } catch (const Error& e) {
    threw = e.code == PE_EINVAL;
  }
  CHECK(threw);
  CHECK(f.job_group_off.size() == 2 && f.cont_kind.size() == 2);   // all-or-nothing append
}

// a started PriorityClass informer and the deterministic tie policy
TEST_CPU(TestPriorityClassInformerAndTiePolicy) {
  ReplicaSpec m, w, l;
  m.replicas = 1;
  m.template_spec.priority_class_name = "";
  w.replicas = 4;
  w.template_spec.priority_class_name = "high";
  l.replicas = 1;
  l.template_spec.priority_class_name = "low";
  const std::map<ReplicaType, ReplicaSpec> reps = {{"Master", m}, {"Worker", w}, {"Launcher", l}};
  PriorityClassInformer inf;
  // informer not fed (the reference's never-started factory): every Get misses, all tie -> name asc
  CHECK((ReplicaOrderV1(reps, inf.Lister()) == std::vector<ReplicaType>{"Launcher", "Master", "Worker"}));
  inf.OnAdd("high", 1000);
  inf.OnAdd("low", -5);
  CHECK((ReplicaOrderV1(reps, inf.Lister()) == std::vector<ReplicaType>{"Worker", "Master", "Launcher"}));
  inf.OnUpdate("high", -10);
  CHECK((ReplicaOrderV1(reps, inf.Lister()) == std::vector<ReplicaType>{"Master", "Launcher", "Worker"}));
  inf.OnDelete("high");
  inf.OnDelete("low");
  // tie policy: listed types first in the given order, then name asc
  CHECK((ReplicaOrderV1(reps, inf.Lister(), V1OrderPolicy{{"Worker", "Master"}}) ==
         std::vector<ReplicaType>{"Worker", "Master", "Launcher"}));
  // priority still dominates the tie policy
  inf.OnAdd("low", 7);
  CHECK((ReplicaOrderV1(reps, inf.Lister(), V1OrderPolicy{{"Worker", "Master"}}) ==
         std::vector<ReplicaType>{"Launcher", "Worker", "Master"}));
  // the flattened CSR follows the order
  Flat f;
  FlattenV1Job(2, reps, inf.Lister(), &f, V1OrderPolicy{{"Worker"}});
  CHECK((f.group_replicas == std::vector<int32_t>{1, 4, 1}));   // Launcher(7), Worker(tie first), Master
}

TEST_CPU(TestGetTotalReplicas) {
  auto r = mnist(3);
  r["Worker"].replicas.reset();                   // nil counts as 1 (k8sutil.go:131-133)
  CHECK(GetTotalReplicas(r) == 2);
  // Go's int32 sum wraps: INT32_MAX + 1 (the nil Worker) is INT32_MIN
  r["Master"].replicas = INT32_MAX;
  CHECK(GetTotalReplicas(r) == INT32_MIN);
  r["Worker"].replicas = INT32_MAX;
  CHECK(GetTotalReplicas(r) == -2);
}

// framework_test.go:154-253 TestRunEnforceMLPolicyPlugins
TEST_CPU(TestRunEnforceMLPolicyPlugins) {
  struct TC {
    const char* name;
    std::optional<MLPolicy> policy;
    std::optional<int32_t> trainjob_nodes;
    int32_t want;
  } tcs[] = {
      {"plainml MLPolicy is applied to runtime.Info, TrainJob doesn't have numNodes", MLPolicy{100, MLPolicy::kPlainML},
       std::nullopt, 100},
      {"plainml MLPolicy is applied to runtime.Info, TrainJob has numNodes", MLPolicy{100, MLPolicy::kPlainML}, 30, 30},
      {"registry is empty", std::nullopt, std::nullopt, 10},
      {"mpi leaves replicas untouched (mpi.go:50-56)", MLPolicy{4, MLPolicy::kMPI}, 8, 10},
      {"torch without numNodes -> DefaultJobReplicas", MLPolicy{std::nullopt, MLPolicy::kTorch}, std::nullopt, 1},
  };
  for (auto& tc : tcs) {
    Info info;
    info.runtime_policy.ml_policy = tc.policy;
    info.scheduler.total_requests["initializer"] = {1, {}};
    info.scheduler.total_requests["trainer-node"] = {10, {}};
    TrainJob tj;
    tj.trainer_num_nodes = tc.trainjob_nodes;
    PlainML p;
    Torch t;
    MPI m;
    for (EnforceMLPolicyPlugin* plugin : std::vector<EnforceMLPolicyPlugin*>{&p, &t, &m}) CHECK(!plugin->EnforceMLPolicy(&info, &tj));
    CHECK(info.scheduler.total_requests["trainer-node"].replicas == tc.want);
    CHECK(info.scheduler.total_requests["initializer"].replicas == 1);
  }
}

TEST_CPU(TestEnforcePodGroupPolicyAndNeedsCreateOrUpdate) {
  Info info;
  info.runtime_policy.pod_group_policy = PodGroupPolicy{CoschedulingPodGroupPolicySource{120}};
  TrainJob tj;
  tj.name = "test-job";
  // coscheduling.go:91-101 (no engine call: construct with a dangling-free dummy by scope)
  if (info.runtime_policy.pod_group_policy) info.scheduler.pod_labels[CoScheduling::kPodGroupLabel] = tj.name;
  CHECK(info.scheduler.pod_labels["scheduling.x-k8s.io/pod-group"] == "test-job");
  PodGroup a, b;
  a.min_member = b.min_member = 31;
  a.min_resources = RL({{"cpu", "31"}});
  b.min_resources = RL({{"cpu", "31000m"}});
  CHECK(NeedsCreateOrUpdate(nullptr, a, false));
  CHECK(!NeedsCreateOrUpdate(&b, a, false));     // exists, not suspended
  CHECK(!NeedsCreateOrUpdate(&b, a, true));      // suspended, spec equal under Cmp
  b.min_member = 30;
  CHECK(NeedsCreateOrUpdate(&b, a, true));       // suspended and changed
}

// ------------------------------------------------------------------ GPU: v2 (pinned by reference tests)

// runtime_test.go:37-104 TestNewInfo "all arguments are specified"
TEST_GPU(TestNewInfo) {
  InfoOptions o;
  o.labels = {{"labelKey", "labelValue"}};
  o.annotations = {{"annotationKey", "annotationValue"}};
  PodSpec init, trainer;
  init.init_containers = {Ctr(RL({{"cpu", "5"}}), std::nullopt, std::string("Always"))};
  init.containers = {Ctr(RL({{"cpu", "10"}}))};
  trainer.init_containers = {Ctr(RL({{"cpu", "15"}}), std::nullopt, std::string("Always"))};
  trainer.containers = {Ctr(RL({{"cpu", "25"}}))};
  o.pod_spec_replicas = {{"initializer", 1, init}, {"trainer-node", 10, trainer}};
  Info info = NewInfo(eng(), o);
  CHECK(info.labels.at("labelKey") == "labelValue");
  CHECK(info.scheduler.total_requests.at("initializer").replicas == 1);
  CHECK(EqualResourceList(info.scheduler.total_requests.at("initializer").pod_requests, RL({{"cpu", "15"}})));
  CHECK(info.scheduler.total_requests.at("trainer-node").replicas == 10);
  CHECK(EqualResourceList(info.scheduler.total_requests.at("trainer-node").pod_requests, RL({{"cpu", "40"}})));
  Info empty = NewInfo(eng(), InfoOptions{});   // "all arguments are not specified"
  CHECK(empty.scheduler.total_requests.empty());
}

static PodSpec InitializerPod(const ResourceList& r) {   // wrapper.go:495-528 + :741-756
  PodSpec p;
  p.init_containers = {Ctr(r), Ctr(r)};
  p.containers = {Ctr(std::nullopt)};
  return p;
}
static PodSpec TrainerPod(const ResourceList& r) {       // wrapper.go:529-551 + :706-720
  PodSpec p;
  p.containers = {Ctr(r)};
  return p;
}

// buildObjects (core/trainingruntime.go:83-129): NewInfo -> EnforceMLPolicy -> EnforcePodGroupPolicy -> Build
static CoScheduling::BuildResult RunBuild(const ResourceList& res, std::optional<int32_t> runtime_nodes,
                                          std::optional<int32_t> trainjob_nodes, int32_t timeout, bool suspend,
                                          Info* info_out = nullptr) {
  InfoOptions o;
  o.ml_policy = MLPolicy{runtime_nodes, MLPolicy::kPlainML};
  o.pod_group_policy = PodGroupPolicy{CoschedulingPodGroupPolicySource{timeout}};
  o.pod_spec_replicas = {{"initializer", 1, InitializerPod(res)}, {"trainer-node", 1, TrainerPod(res)}};
  Info info = NewInfo(eng(), o);
  TrainJob tj;
  tj.name = "test-job";
  tj.ns = "default";
  tj.uid = "uid";
  tj.suspend = suspend;
  tj.trainer_num_nodes = trainjob_nodes;
  PlainML().EnforceMLPolicy(&info, &tj);
  CoScheduling cs(eng());
  CHECK(!cs.EnforcePodGroupPolicy(&info, &tj));
  CHECK(info.scheduler.pod_labels.at(CoScheduling::kPodGroupLabel) == "test-job");
  auto r = cs.Build(&info, &tj, nullptr);
  if (info_out) *info_out = info;
  return r;
}

// core/trainingruntime_test.go:51-98: runtime NumNodes 100, TrainJob 30 -> MinMember 31, cpu 31
TEST_GPU(TestTrainingRuntimeNewObjects) {
  auto r = RunBuild(RL({{"cpu", "1"}}), 100, 30, 120, true);
  CHECK(!r.error && r.object);
  CHECK(r.object->min_member == 31);
  CHECK(EqualResourceList(r.object->min_resources, RL({{"cpu", "31"}})));
  CHECK(r.object->schedule_timeout_seconds == 120);
  CHECK(r.object->owner_kind == "TrainJob" && r.object->owner_uid == "uid");
}

// core/clustertrainingruntime_test.go:47-83: NumNodes 100 from the runtime -> 101
TEST_GPU(TestClusterTrainingRuntimeNewObjects) {
  auto r = RunBuild(RL({{"cpu", "1"}}), 100, std::nullopt, 120, true);
  CHECK(r.object && r.object->min_member == 101);
  CHECK(EqualResourceList(r.object->min_resources, RL({{"cpu", "101"}})));
}

// test/integration/controller.v2/trainjob_controller_test.go:106-157: 101 CPU, 404Gi
TEST_GPU(TestIntegrationPodGroup) {
  auto r = RunBuild(RL({{"cpu", "1"}, {"memory", "4Gi"}}), 100, std::nullopt, 100, false);
  CHECK(r.object && r.object->min_member == 101);
  CHECK(EqualResourceList(r.object->min_resources, RL({{"cpu", "101"}, {"memory", "404Gi"}})));
  CHECK(r.object->schedule_timeout_seconds == 100);
}

// framework/core/framework_test.go:398-486: Build on a given runtime.Info
TEST_GPU(TestRunComponentBuilderPlugins) {
  Info info;
  info.runtime_policy.ml_policy = MLPolicy{10, MLPolicy::kPlainML};
  info.runtime_policy.pod_group_policy = PodGroupPolicy{CoschedulingPodGroupPolicySource{300}};
  info.trainer.num_nodes = 10;
  const ResourceList res = RL({{"cpu", "1"}, {"memory", "4Gi"}});
  info.scheduler.total_requests = {{"initializer", {1, res}}, {"trainer-node", {1, res}}};
  TrainJob tj;
  tj.name = "test-job";
  tj.uid = "uid";
  tj.trainer_num_nodes = 100;
  PlainML().EnforceMLPolicy(&info, &tj);
  CHECK(info.trainer.num_nodes == 100);
  CHECK(info.scheduler.total_requests.at("trainer-node").replicas == 100);
  CoScheduling cs(eng());
  cs.EnforcePodGroupPolicy(&info, &tj);
  auto r = cs.Build(&info, &tj, nullptr);
  CHECK(r.object && r.object->min_member == 101);
  CHECK(EqualResourceList(r.object->min_resources, RL({{"cpu", "101"}, {"memory", "404Gi"}})));
  CHECK(r.object->schedule_timeout_seconds == 300);
}

// job.go:250-313 + scheduling.go:32-73 through the GPU aggregation, both PodGroup flavours
TEST_GPU(TestSyncPodGroupV1) {
  JobMeta job;
  job.name = "pytorch-dist-mnist-nccl";
  job.ns = "kubeflow";
  job.uid = "uid-1";
  auto c = SyncPodGroupV1(eng(), GangScheduler::kSchedulerPlugins, job, mnist(1), nullptr, kNoPC, nullptr);
  CHECK(c.action == SyncPodGroupResult::kCreate && c.object.min_member == 2);
  CHECK(c.object.min_resources.at("nvidia.com/gpu").String() == "2");
  const std::string js = PodGroupJSON(c.object);
  CHECK(js.find("\"spec\":{\"minMember\":2,\"minResources\":{\"nvidia.com/gpu\":\"2\"}}") != std::string::npos);
  CHECK(js.find("\"ownerReferences\":[{\"apiVersion\":\"kubeflow.org/v1\",\"kind\":\"PyTorchJob\"") != std::string::npos);
  // Volcano: queue / priorityClass from the SchedulingPolicy, no timeout field
  SchedulingPolicy pol;
  pol.queue = "q1";
  pol.priority_class = "high";
  pol.schedule_timeout_seconds = 30;
  auto v = SyncPodGroupV1(eng(), GangScheduler::kVolcano, job, mnist(3), &pol, kNoPC, nullptr);
  CHECK(v.object.queue == "q1" && v.object.priority_class_name == "high" && !v.object.schedule_timeout_seconds);
  CHECK(PodGroupJSON(v.object).find("\"spec\":{\"minMember\":4,\"queue\":\"q1\",\"priorityClassName\":\"high\","
                                    "\"minResources\":{\"nvidia.com/gpu\":\"4\"}}") != std::string::npos);
  // existing Volcano PodGroup keeps its queue; an existing object is always updated
  PodGroup old = v.object;
  old.queue = "keep";
  auto u = SyncPodGroupV1(eng(), GangScheduler::kVolcano, job, mnist(3), &pol, kNoPC, &old);
  CHECK(u.action == SyncPodGroupResult::kUpdate && u.object.queue == "keep");
  auto same = SyncPodGroupV1(eng(), GangScheduler::kVolcano, job, mnist(3), &pol, kNoPC, &u.object);
  CHECK(same.action == SyncPodGroupResult::kUpdate);
  // MinResources given: used verbatim (job.go:267-269), printed as given
  pol.min_resources = RL({{"cpu", "1500m"}, {"memory", "1024Mi"}});
  auto g = SyncPodGroupV1(eng(), GangScheduler::kSchedulerPlugins, job, mnist(1), &pol, kNoPC, nullptr);
  CHECK(PodGroupJSON(g.object).find("\"minResources\":{\"cpu\":\"1500m\",\"memory\":\"1Gi\"},\"scheduleTimeoutSeconds\":30") !=
        std::string::npos);
  // mixed formats: DecimalSI first nonzero wins; 1G + 1Gi prints as plain digits
  ReplicaSpec a, b;
  a.replicas = 1;
  a.template_spec.containers = {Ctr(RL({{"memory", "1G"}}))};
  b.replicas = 1;
  b.template_spec.containers = {Ctr(RL({{"memory", "1Gi"}}))};
  auto mix = CalcPGMinResources(eng(), 2, {{"A", a}, {"B", b}}, kNoPC);
  CHECK(mix.at("memory").String() == "2073741824");
}

// framework_test.go:398-486 pin (101 CPU, 404Gi, timeout 300) as the wire object
TEST_GPU(TestBuildWireV2) {
  auto r = RunBuild(RL({{"cpu", "1"}, {"memory", "4Gi"}}), 100, std::nullopt, 300, false);
  CHECK(r.object);
  const std::string js = PodGroupJSON(*r.object);
  CHECK(js.find("\"spec\":{\"minMember\":101,\"minResources\":{\"cpu\":\"101\",\"memory\":\"404Gi\"},"
                "\"scheduleTimeoutSeconds\":300}") != std::string::npos);
  CHECK(js.find("\"apiVersion\":\"kubeflow.org/v2alpha1\",\"kind\":\"TrainJob\"") != std::string::npos);
}

// ResourcesPerNode vs TotalRequests.  Reference behaviour (option off): the
// PodGroup counts the runtime's trainer requests even though the pods run with ResourcesPerNode.
TEST_GPU(TestResourcesPerNodeTotalRequests) {
  PodSpec trainer;
  Container tc = Ctr(RL({{"cpu", "1"}, {"memory", "4Gi"}}));
  tc.name = "trainer";
  trainer.containers = {tc, Ctr(RL({{"cpu", "100m"}}))};   // a second (sidecar-style) container keeps its own
  TrainJob tj;
  tj.name = "rpn";
  tj.uid = "u";
  tj.trainer_num_nodes = 10;
  tj.resources_per_node = ResourceRequirements{RL({{"cpu", "2"}, {"memory", "8Gi"}}), std::nullopt};
  auto run = [&](bool fix) {
    InfoOptions o;
    o.ml_policy = MLPolicy{std::nullopt, MLPolicy::kTorch};
    o.pod_group_policy = PodGroupPolicy{CoschedulingPodGroupPolicySource{60}};
    o.pod_spec_replicas = {{"trainer-node", 1, trainer}};
    Info info = NewInfo(eng(), o);
    CHECK(!ApplyTotalRequestsOptions(eng(), TotalRequestsOptions{fix}, &info, &tj, trainer));
    Torch().EnforceMLPolicy(&info, &tj);
    return CoScheduling(eng()).Build(&info, &tj, nullptr);
  };
  auto ref = run(false);   // 10 x (1 + 0.1) cpu, 10 x 4Gi
  CHECK(ref.object && ref.object->min_member == 10);
  CHECK(EqualResourceList(ref.object->min_resources, RL({{"cpu", "11"}, {"memory", "40Gi"}})));
  auto fixed = run(true);  // 10 x (2 + 0.1) cpu, 10 x 8Gi
  CHECK(fixed.object && fixed.object->min_member == 10);
  CHECK(EqualResourceList(fixed.object->min_resources, RL({{"cpu", "21"}, {"memory", "80Gi"}})));
  PodSpec applied = ApplyTrainerResourcesPerNode(trainer, tj);
  CHECK(applied.containers[0].requests->at("cpu").Equal(Quantity::Parse("2")) && !applied.containers[0].limits);
  CHECK(applied.containers[1].requests->at("cpu").Equal(Quantity::Parse("100m")));
}

// The order decides which pods count toward minMember (util.go:126-141)
TEST_GPU(TestCalcPGMinResourcesTiePolicy) {
  ReplicaSpec m, w;
  m.replicas = 1;
  m.template_spec.containers = {Ctr(RL({{"cpu", "4"}}))};
  w.replicas = 3;
  w.template_spec.containers = {Ctr(RL({{"cpu", "1"}}))};
  const std::map<ReplicaType, ReplicaSpec> reps = {{"Master", m}, {"Worker", w}};
  PriorityClassInformer inf;
  auto dflt = CalcPGMinResources(eng(), 2, reps, inf.Lister());   // Master then one Worker
  CHECK(dflt.at("cpu").Equal(Quantity::Parse("5")));
  auto wfirst = CalcPGMinResources(eng(), 2, reps, inf.Lister(), V1OrderPolicy{{"Worker"}});   // two Workers
  CHECK(wfirst.at("cpu").Equal(Quantity::Parse("2")));
  w.template_spec.priority_class_name = "hp";
  inf.OnAdd("hp", 100);
  auto pri = CalcPGMinResources(eng(), 2, {{"Master", m}, {"Worker", w}}, inf.Lister());
  CHECK(pri.at("cpu").Equal(Quantity::Parse("2")));
}

TEST_GPU(TestBuildNilPolicyAndExistingPodGroup) {
  CoScheduling cs(eng());
  Info info;
  TrainJob tj;
  auto none = cs.Build(&info, &tj, nullptr);     // coscheduling.go:104-106 -> (nil, nil)
  CHECK(!none.object && !none.error);
  Info made;
  auto r = RunBuild(RL({{"cpu", "1"}}), 3, std::nullopt, 60, false, &made);
  CHECK(r.object);
  auto again = cs.Build(&made, &tj, &*r.object); // exists and not suspended -> nothing to apply
  CHECK(!again.object && !again.error);
}

// ------------------------------------------------------------------ GPU: v1 (hand-derived, parity unpinned)

TEST_GPU(TestCalcPGMinResourcesMnist) {
  for (int n : {1, 3, 7, 15}) {
    auto r = mnist(n);
    auto pg = CalcPodGroupSpecV1(eng(), r, nullptr, kNoPC);
    CHECK(pg.min_member == 1 + n);
    CHECK(EqualResourceList(pg.min_resources, RL({{"nvidia.com/gpu", std::to_string(1 + n).c_str()}})));
  }
}

TEST_GPU(TestCalcPGMinResourcesSdkGangSpec) {
  // sdk/python/test/e2e/test_e2e_pytorchjob.py:54-95,342-348: limits {memory 2Gi, cpu 0.8}
  ReplicaSpec m, w;
  m.replicas = w.replicas = 1;
  m.template_spec.containers = w.template_spec.containers = {Ctr(std::nullopt, RL({{"memory", "2Gi"}, {"cpu", "0.8"}}))};
  std::map<ReplicaType, ReplicaSpec> r = {{"Master", m}, {"Worker", w}};
  for (int32_t min_avail : {10, 2}) {
    SchedulingPolicy sp;
    sp.min_available = min_avail;
    auto pg = CalcPodGroupSpecV1(eng(), r, &sp, kNoPC);
    CHECK(pg.min_member == min_avail);
    CHECK(EqualResourceList(pg.min_resources, RL({{"cpu", "1600m"}, {"memory", "4Gi"}})));
  }
  SchedulingPolicy verbatim;
  verbatim.min_resources = RL({{"cpu", "7"}});
  CHECK(EqualResourceList(CalcPodGroupSpecV1(eng(), r, &verbatim, kNoPC).min_resources, RL({{"cpu", "7"}})));
}

TEST_GPU(TestCalcPGMinResourcesBatchAndOverflow) {
  std::vector<V1Job> jobs;
  for (int n = 0; n < 1000; ++n) jobs.push_back({1 + n % 16, mnist(n % 16)});
  auto out = CalcPGMinResourcesBatch(eng(), jobs, kNoPC);
  for (int n = 0; n < 1000; ++n)
    CHECK(EqualResourceList(out[n], RL({{"nvidia.com/gpu", std::to_string(1 + n % 16).c_str()}})));
  ReplicaSpec w;
  w.replicas = 4;
  w.template_spec.containers = {Ctr(RL({{"memory", "4611686018427387904"}}))};   // 2^62 bytes x 4
  bool threw = false;
  try {
    CalcPGMinResources(eng(), 4, {{"Worker", w}}, kNoPC);
  } catch (const Error& e) {
    threw = e.code == PE_EOVERFLOW;
  }
  CHECK(threw);
}

// Verdict r5 item 2: keys beyond the four engine dimensions reach the GPU (tests/golden/wide_keys.json
// cases 1-2 and the v2 sidecar case, hand-derived); only an int64 overflow is the reference's.
TEST_GPU(TestCalcPGMinResourcesWideKeys) {
  ReplicaSpec m, w;
  m.replicas = 1;
  m.template_spec.containers = {Ctr(RL({{"cpu", "2"}, {"memory", "8Gi"}, {"hugepages-2Mi", "1Gi"}, {"rdma/hca", "1"},
                                        {"nvidia.com/gpu", "1"}}))};
  w.replicas = 3;
  w.template_spec.containers = {Ctr(RL({{"cpu", "2"}, {"memory", "8Gi"}, {"hugepages-2Mi", "512Mi"}, {"rdma/hca", "1"},
                                        {"nvidia.com/gpu", "1"}}))};
  auto pg = CalcPodGroupSpecV1(eng(), {{"Master", m}, {"Worker", w}}, nullptr, kNoPC);
  CHECK(pg.min_member == 4);
  CHECK(EqualResourceList(pg.min_resources, RL({{"cpu", "8"}, {"memory", "32Gi"}, {"hugepages-2Mi", "2560Mi"},
                                                {"rdma/hca", "4"}, {"nvidia.com/gpu", "4"}})));
  CHECK(pg.min_resources.at("hugepages-2Mi").String() == "2560Mi");
  ReplicaSpec a, b;
  a.replicas = 1;
  a.template_spec.containers = {Ctr(RL({{"nvidia.com/gpu", "1"}, {"cpu", "1"}}))};
  b.replicas = 2;
  b.template_spec.containers = {Ctr(RL({{"amd.com/gpu", "8"}, {"cpu", "1500u"}}))};
  auto pg2 = CalcPodGroupSpecV1(eng(), {{"Master", a}, {"Worker", b}}, nullptr, kNoPC);
  CHECK(EqualResourceList(pg2.min_resources, RL({{"nvidia.com/gpu", "1"}, {"amd.com/gpu", "16"}, {"cpu", "1003m"}})));
  CHECK(pg2.min_resources.at("cpu").String() == "1003m");
  // v2: a sidecar in micro-cores, an extended key, pod overhead; 2 trainer nodes
  InfoOptions o;
  PodSpec pod;
  pod.init_containers = {Ctr(RL({{"cpu", "1500u"}, {"example.com/fpga", "1"}}), std::nullopt, std::string("Always"))};
  pod.containers = {Ctr(RL({{"cpu", "2"}, {"memory", "1Gi"}}))};
  pod.overhead = RL({{"cpu", "100m"}});
  o.pod_spec_replicas = {{"trainer-node", 1, pod}};
  o.ml_policy = MLPolicy{2, MLPolicy::kPlainML};
  o.pod_group_policy = PodGroupPolicy{CoschedulingPodGroupPolicySource{}};
  Info info = NewInfo(eng(), o);
  TrainJob tj;
  tj.name = "wide";
  PlainML().EnforceMLPolicy(&info, &tj);
  CoScheduling cs(eng());
  auto r = cs.Build(&info, &tj, nullptr);
  CHECK(r.object && !r.error);
  if (r.object) {
    CHECK(r.object->min_member == 2);
    CHECK(EqualResourceList(r.object->min_resources,
                            RL({{"cpu", "4203m"}, {"example.com/fpga", "2"}, {"memory", "2Gi"}})));
  }
  // 21 keys: two key slices of one call
  ResourceList many;
  for (int i = 0; i < 20; ++i) many["example.com/r" + std::to_string(100 + i)] = Quantity::Parse("1");
  many["cpu"] = Quantity::Parse("1");
  ReplicaSpec z;
  z.replicas = 5;
  z.template_spec.containers = {Ctr(many)};
  ResourceList want;
  for (auto& kv : many) want[kv.first] = Quantity::Parse("5");
  CHECK(EqualResourceList(CalcPGMinResources(eng(), 5, {{"Worker", z}}, kNoPC), want));
  // an int64 sum overflow stays the one refused case
  ReplicaSpec h;
  h.replicas = 2;
  h.template_spec.containers = {Ctr(RL({{"example.com/huge", "5e18"}})), Ctr(RL({{"example.com/huge", "1"}}))};
  bool threw = false;
  try {
    CalcPGMinResources(eng(), 2, {{"Worker", h}}, kNoPC);
  } catch (const Error& e) {
    threw = e.code == PE_EOVERFLOW;
  }
  CHECK(threw);
}

// ------------------------------------------------------------------ GPU: node inventory (8f row 3)

static Node MkNode(const char* name, const char* cpu, const char* mem, const char* gpu, const char* req_cpu,
                   const char* req_mem, uint32_t labels = 0) {
  Node n;
  n.name = name;
  n.allocatable = RL({{"cpu", cpu}, {"memory", mem}, {"amd.com/gpu", gpu}, {"pods", "110"}});
  n.requested = RL({{"cpu", req_cpu}, {"memory", req_mem}});
  n.label_bits = labels;
  return n;
}

static std::vector<int64_t> Residuals(Engine& e, int64_t slots) {
  std::vector<int64_t> r((size_t)PE_DIMS * slots);
  CHECK(pe_read_residuals(e.ctx(), r.data()) == PE_OK);
  return r;
}

TEST_GPU(TestNodeInventoryInformer) {
  Engine e(0, "amd.com/gpu");
  NodeInventory inv(e, 6);
  inv.OnAdd(MkNode("cpu-a", "64", "256Gi", "0", "8", "32Gi"));
  inv.OnAdd(MkNode("gpu-a", "128", "1Ti", "8", "0", "0", 1));
  inv.OnAdd(MkNode("cpu-b", "32", "128Gi", "0", "31", "1Gi"));
  CHECK(inv.Flush() == 3 && inv.Pending() == 0);
  CHECK(*inv.SlotOf("cpu-a") == 0 && *inv.SlotOf("gpu-a") == 1 && *inv.SlotOf("cpu-b") == 2);
  auto r = Residuals(e, 6);
  CHECK(r[0 * 6 + 0] == 56000 && r[1 * 6 + 0] == (224LL << 30));   // cpu milli, memory bytes
  CHECK(r[2 * 6 + 1] == 8 && r[0 * 6 + 2] == 1000);
  CHECK(r[0 * 6 + 3] == INT64_MIN);                                 // empty slot: nothing fits

  // delete + add reuse the lowest free slot; update rewrites in place; one flush for all three
  inv.OnDelete("gpu-a");
  inv.OnAdd(MkNode("gpu-b", "192", "2Ti", "8", "16", "64Gi", 1));
  inv.OnUpdate(MkNode("cpu-a", "64", "256Gi", "0", "60", "32Gi"));
  CHECK(inv.Flush() == 3);
  CHECK(*inv.SlotOf("gpu-b") == 1 && !inv.SlotOf("gpu-a") && inv.Size() == 3);
  r = Residuals(e, 6);
  CHECK(r[0 * 6 + 1] == 176000 && r[2 * 6 + 1] == 8 && r[0 * 6 + 0] == 4000);

  // the fit mask sees the live inventory: cpu 2 + mem 1Gi fits cpu-b? no (1 core left); cpu-a yes
  const int64_t req[2 * PE_DIMS] = {2000, 1LL << 30, 0, 0, 1000, 1LL << 30, 1, 0};
  const uint32_t need[2] = {0, 1};
  int64_t counts[2] = {-1, -1};
  CHECK(pe_fit_mask(e.ctx(), 2, req, need, counts, nullptr, nullptr) == PE_OK);
  CHECK(counts[0] == 2 && counts[1] == 1);                          // cpu-a + gpu-b; gpu-b only
  uint64_t rows[2];
  CHECK(pe_fit_mask_rows(e.ctx(), 0, 2, rows) == PE_OK);
  CHECK(rows[0] == 0b011 && rows[1] == 0b010);

  // a node whose quantity has no exact canonical value changes nothing; a full table refuses
  bool threw = false;
  try {
    inv.OnAdd(MkNode("bad", "0.0001", "1Gi", "0", "0", "0"));
  } catch (const Error& err) {
    threw = err.code == PE_EINVAL;
  }
  CHECK(threw && inv.Pending() == 0 && !inv.SlotOf("bad"));
  for (int i = 0; i < 3; ++i) inv.OnAdd(MkNode(("n" + std::to_string(i)).c_str(), "8", "8Gi", "0", "0", "0"));
  threw = false;
  try {
    inv.OnAdd(MkNode("overflow", "8", "8Gi", "0", "0", "0"));
  } catch (const Error& err) {
    threw = err.code == PE_ENOMEM;
  }
  CHECK(threw && inv.Size() == 6 && inv.Flush() == 3);
}

int main(int argc, char** argv) {
  bool cpu = true, gpu = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--gpu")) { cpu = false; gpu = true; }
    if (!std::strcmp(argv[i], "--all")) { cpu = gpu = true; }
  }
  for (auto& c : cases()) {
    if ((c.gpu && !gpu) || (!c.gpu && !cpu)) continue;
    const int before = g_fail;
    ++g_run;
    try {
      c.fn();
    } catch (const Error& e) {
      std::fprintf(stderr, "  FAIL %s: kf::Error %d %s\n", c.name, e.code, e.msg.c_str());
      ++g_fail;
    } catch (const QuantityError& e) {
      std::fprintf(stderr, "  FAIL %s: QuantityError %s\n", c.name, e.msg.c_str());
      ++g_fail;
    }
    std::printf("%s %s\n", g_fail == before ? "ok  " : "FAIL", c.name);
  }
  std::printf("%d cases, %d failed checks\n", g_run, g_fail);
  return g_fail ? 1 : 0;
}
