// Host-side mirror of the reference's interfaces for the PodGroup hot path, in C++ (the reference
// is compiled Go; no Go toolchain exists in this pipeline).  Names, argument meaning and error
// behaviour follow the Go code so the tests read like the reference's own; every number is
// computed by libplacement on the GPU through include/placement.h -- this layer only flattens
// object graphs into the ABI's CSR arrays and builds result objects.
//
//   kf::CalcPGMinResources  <- pkg/controller.v1/common/util.go:108-145
//   kf::GetTotalReplicas    <- pkg/util/k8sutil/k8sutil.go:126-137
//   kf::CalcPodGroupSpecV1  <- pkg/controller.v1/common/job.go:250-277 (minMember / MinResources)
//   kf::NewInfo             <- pkg/runtime.v2/runtime.go:105-145 (TotalRequests via kueue formula)
//   kf::PlainML/Torch/MPI   <- pkg/runtime.v2/framework/plugins/{plainml,torch,mpi} EnforceMLPolicy
//   kf::CoScheduling        <- pkg/runtime.v2/framework/plugins/coscheduling/coscheduling.go:58-153
#pragma once
#include <stdint.h>

#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "placement.h"
#include "quantity.h"

namespace kf {

// ------------------------------------------------------------------ API types (input schema slice)
// pkg/apis/kubeflow.org/v1/common_types.go:96-110,194-251; k8s core/v1 Container/PodSpec subset
struct Container {
  std::string name;
  std::optional<ResourceList> requests;  // nil vs empty matters for v1 (util.go:90-92)
  std::optional<ResourceList> limits;
  std::optional<std::string> restart_policy;  // "Always" on an init container = sidecar
};

struct PodSpec {
  std::vector<Container> containers;
  std::vector<Container> init_containers;
  std::optional<ResourceList> overhead;
  std::string priority_class_name;
};

using ReplicaType = std::string;

struct ReplicaSpec {
  std::optional<int32_t> replicas;
  PodSpec template_spec;
};

struct SchedulingPolicy {
  std::optional<int32_t> min_available;
  std::string queue;
  std::optional<ResourceList> min_resources;
  std::string priority_class;
  std::optional<int32_t> schedule_timeout_seconds;
};

struct PriorityClass {
  int32_t value = 0;
};
// util.go:106 PriorityClassGetFunc; std::nullopt plays the (nil, err) return
using PriorityClassGetFunc = std::function<std::optional<PriorityClass>(const std::string&)>;

// v2 (pkg/apis/kubeflow.org/v2alpha1/trainingruntime_types.go:103-180, trainjob_types.go:169-200)
struct MLPolicy {
  enum Source { kPlainML, kTorch, kMPI };
  std::optional<int32_t> num_nodes;
  Source source = kPlainML;
};
struct CoschedulingPodGroupPolicySource {
  std::optional<int32_t> schedule_timeout_seconds;
};
struct PodGroupPolicy {
  std::optional<CoschedulingPodGroupPolicySource> coscheduling;
};
struct ResourceRequirements {
  std::optional<ResourceList> requests, limits;
};
struct TrainJob {
  std::string name, ns, uid;
  bool suspend = false;
  std::optional<int32_t> trainer_num_nodes;
  std::optional<ResourceRequirements> resources_per_node;   // trainjob_types.go:192 Trainer.ResourcesPerNode
  std::map<std::string, std::string> labels, annotations;
};

// pkg/runtime.v2/runtime.go:28-62
struct TotalResourceRequest {
  int32_t replicas = 0;
  ResourceList pod_requests;
};
struct RuntimePolicy {
  std::optional<MLPolicy> ml_policy;
  std::optional<PodGroupPolicy> pod_group_policy;
};
struct Info {
  std::map<std::string, std::string> labels, annotations;
  RuntimePolicy runtime_policy;
  struct {
    std::optional<int32_t> num_nodes;
  } trainer;
  struct {
    std::map<std::string, std::string> pod_labels;
    std::map<std::string, TotalResourceRequest> total_requests;
  } scheduler;
};

// Which PodGroup API the operator writes: --gang-scheduler-name (pkg/controller.v1/common/
// job_controller.go GangSchedulerVolcano / scheduler-plugins default; v2 always scheduler-plugins)
enum class GangScheduler { kSchedulerPlugins, kVolcano };

// The PodGroup the operator creates: scheduler-plugins v1alpha1 (the fields coscheduling.go:119-133
// and job.go:302-310 set) or Volcano v1beta1 (job.go:285-299: queue, priorityClassName, minResources
// as a pointer).  The owner reference is the job's controller reference
// (job_controller.go:221-233 GenOwnerReference / ctrlutil.SetControllerReference): controller and
// blockOwnerDeletion true.
struct PodGroup {
  GangScheduler flavour = GangScheduler::kSchedulerPlugins;
  std::string name, ns;
  int32_t min_member = 0;
  ResourceList min_resources;
  std::optional<int32_t> schedule_timeout_seconds;   // scheduler-plugins only
  std::string queue, priority_class_name;            // Volcano only
  std::map<std::string, std::string> labels, annotations;
  std::string owner_api_version, owner_kind, owner_name, owner_uid;
};

// The object as the operator's client sends it to the API server: Go's JSON encoding of the
// scheduler-plugins / Volcano PodGroup types (struct field order, omitempty, map keys sorted,
// quantities through Quantity.String(), metav1.Time zero values as null).  SURVEY 8f row 1.
std::string PodGroupJSON(const PodGroup& pg);

// ------------------------------------------------------------------ engine handle

struct Error {
  int code;  // PE_E* or PE_EINVAL for host-side validation
  std::string msg;
};

// Resource key <-> engine dimension (0 cpu, 1 memory, 2 accelerator, 3 ephemeral-storage)
struct Dims {
  std::string gpu = "amd.com/gpu";
  int dim_of(const std::string& resource) const;  // -1: no engine dimension for this key
  std::string name_of(int dim) const;
};

class Engine {
 public:
  explicit Engine(int device_id = 0, std::string gpu_resource_name = "amd.com/gpu");
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
  pe_ctx* ctx() const { return ctx_; }
  const Dims& dims() const { return dims_; }

 private:
  pe_ctx* ctx_ = nullptr;
  Dims dims_;
};

// ------------------------------------------------------------------ priority classes
// In the reference the PriorityClass lister's shared informer factory is never started
// (pytorchjob_controller.go:73-86 builds it, nothing calls Start), so every Get misses and every
// replica type gets priority 0 with a warning (util.go:112-119); the tie is then broken by Go map
// iteration order through a non-stable sort.Sort (util.go:29-48,124): random.  Two explicit fixes:
//
// PriorityClassInformer -- the started informer's store: the PriorityClass watch handlers feed it,
// Lister() answers Get(name) from it (miss / "" -> nullopt -> priority 0, as the Go lister errors).
class PriorityClassInformer {
 public:
  void OnAdd(const std::string& name, int32_t value) { values_[name] = value; }
  void OnUpdate(const std::string& name, int32_t value) { values_[name] = value; }
  void OnDelete(const std::string& name) { values_.erase(name); }
  bool HasSynced() const { return true; }
  PriorityClassGetFunc Lister() const;   // reads the live store (valid while the informer lives)

 private:
  std::map<std::string, int32_t> values_;
};

// V1OrderPolicy -- the deterministic tie policy: among replica types of equal priority, the types
// listed in tie_order come first, in that order; the rest by type name ascending (the default,
// what the kernel fixtures and the oracle's canonical order use).  E.g. {"Master", "Launcher",
// "Chief"} counts leader pods toward minMember before workers.
struct V1OrderPolicy {
  std::vector<ReplicaType> tie_order;
};
// The CalcPGMinResources type order under a policy (priority desc, then the tie policy).
std::vector<ReplicaType> ReplicaOrderV1(const std::map<ReplicaType, ReplicaSpec>& replicas,
                                        const PriorityClassGetFunc& pcGetFunc, const V1OrderPolicy& order = {});

// ------------------------------------------------------------------ v1

int32_t GetTotalReplicas(const std::map<ReplicaType, ReplicaSpec>& replicas);

// util.go:108.  Any resource key (a per-call key table, pe_pg_min_resources_keys).  Throws kf::Error
// {PE_EOVERFLOW} when a sum or a value has no int64 at its key's scale (Go would switch to inf.Dec:
// the one case a caller hands to the reference), {PE_EINVAL} on a negative quantity.
ResourceList CalcPGMinResources(Engine& eng, int32_t minMember, const std::map<ReplicaType, ReplicaSpec>& replicas,
                                const PriorityClassGetFunc& pcGetFunc, const V1OrderPolicy& order = {});

struct V1Job {
  int32_t min_member;
  std::map<ReplicaType, ReplicaSpec> replicas;
};
// One kernel launch for a batch of jobs (the throughput form of the same rule).
std::vector<ResourceList> CalcPGMinResourcesBatch(Engine& eng, const std::vector<V1Job>& jobs,
                                                  const PriorityClassGetFunc& pcGetFunc, const V1OrderPolicy& order = {});

// job.go:250-277: minMember = MinAvailable ?? GetTotalReplicas; MinResources verbatim if set.
struct PodGroupSpecV1 {
  int32_t min_member;
  ResourceList min_resources;
};
PodGroupSpecV1 CalcPodGroupSpecV1(Engine& eng, const std::map<ReplicaType, ReplicaSpec>& replicas,
                                  const SchedulingPolicy* policy, const PriorityClassGetFunc& pcGetFunc,
                                  const V1OrderPolicy& order = {});

// Print format of each MinResources key as Go's AddResourceList leaves it (util.go:79-104): a new
// key deep-copies the first quantity, Quantity.Add adopts the addend's format while the running
// value is 0 -- so a key prints in the format of its first nonzero contribution (all zero: the
// last one).  Host-side metadata only; the values come from the GPU.
std::map<std::string, Format> MinResourcesFormatsV1(int32_t minMember, const std::map<ReplicaType, ReplicaSpec>& replicas,
                                                    const PriorityClassGetFunc& pcGetFunc,
                                                    const V1OrderPolicy& order = {});

// v1 gang branch + SyncPodGroup (job.go:250-313, scheduling.go:32-73): the PodGroup the job
// controller creates or updates for one job.
struct JobMeta {
  std::string name, ns, uid;
  std::string api_version = "kubeflow.org/v1", kind = "PyTorchJob";
  std::map<std::string, std::string> annotations;
};
struct SyncPodGroupResult {
  enum Action { kCreate, kUpdate } action;
  PodGroup object;
};
// existing = the PodGroup GetPodGroup returned (nullptr = NotFound).  A new PodGroup takes the
// job's name, namespace, annotations and controller reference.  For an existing one the spec is
// refilled in place and the result is ALWAYS kUpdate: SyncPodGroup compares `&podGroup` (a
// *metav1.Object) with `podGroup` (a metav1.Object) through cmp.Diff, which never reports equal
// (scheduling.go:38-44) -- reproduced.  Volcano keeps a non-empty queue already on the object
// (job.go:287-289).  MinResources: SchedulingPolicy.MinResources verbatim, else
// CalcPGMinResources on the GPU, printed in MinResourcesFormatsV1's formats.
SyncPodGroupResult SyncPodGroupV1(Engine& eng, GangScheduler flavour, const JobMeta& job,
                                  const std::map<ReplicaType, ReplicaSpec>& replicas, const SchedulingPolicy* policy,
                                  const PriorityClassGetFunc& pcGetFunc, const PodGroup* existing,
                                  const V1OrderPolicy& order = {});

// ------------------------------------------------------------------ v2

struct PodSpecReplica {
  std::string name;
  int32_t replicas;
  PodSpec pod_spec;
};
struct InfoOptions {
  std::map<std::string, std::string> labels, annotations;
  std::optional<MLPolicy> ml_policy;
  std::optional<PodGroupPolicy> pod_group_policy;
  std::vector<PodSpecReplica> pod_spec_replicas;
};
// runtime.go:115-145: TotalRequests[name] = {replicas, kueue TotalRequests(podSpec)} -- the pod
// formula runs in the pg_min_resources kernel (PE_MODE_V2, one entry per group, replicas 1).
Info NewInfo(Engine& eng, const InfoOptions& opts);

// jobset/builder.go:138-163 (Builder.Trainer): the TrainJob's Trainer.ResourcesPerNode replaces the
// resources of the "trainer" container (constants.ContainerTrainer) of the trainer-node pod.
PodSpec ApplyTrainerResourcesPerNode(const PodSpec& runtime_trainer_pod, const TrainJob& trainJob);

// the reference computes TotalRequests["trainer-node"] from the RUNTIME's pod spec
// (runtime.go:133-134; plainml.go:63-66 and torch.go:122-125 carry "TODO: Add support for total
// requests from the TrainJob's ResourcesPerNode"), while the JobSet it launches runs the pods with
// ResourcesPerNode -- so the PodGroup's MinResources can disagree with the pods it gates.  Opt-in
// fix (default off = the reference's behaviour): when the TrainJob sets ResourcesPerNode, recompute
// the trainer-node pod requests on the GPU from ApplyTrainerResourcesPerNode(runtime pod).  The
// replica count (MLPolicy rewrite) is untouched.  Call after NewInfo, before Build.
struct TotalRequestsOptions {
  bool from_resources_per_node = false;
};
std::optional<Error> ApplyTotalRequestsOptions(Engine& eng, const TotalRequestsOptions& opts, Info* info,
                                               const TrainJob* trainJob, const PodSpec& runtime_trainer_pod);

class Plugin {
 public:
  virtual ~Plugin() = default;
  virtual std::string Name() const = 0;
};

// framework/interface.go:45-48
class EnforceMLPolicyPlugin : public Plugin {
 public:
  virtual std::optional<Error> EnforceMLPolicy(Info* info, const TrainJob* trainJob) = 0;
};

class PlainML : public EnforceMLPolicyPlugin {  // plainml.go:45-76
 public:
  std::string Name() const override { return "PlainML"; }
  std::optional<Error> EnforceMLPolicy(Info* info, const TrainJob* trainJob) override;
};
class Torch : public EnforceMLPolicyPlugin {    // torch.go:52-135 (replica rewrite only)
 public:
  std::string Name() const override { return "Torch"; }
  std::optional<Error> EnforceMLPolicy(Info* info, const TrainJob* trainJob) override;
};
class MPI : public EnforceMLPolicyPlugin {      // mpi.go:50-56: no-op
 public:
  std::string Name() const override { return "MPI"; }
  std::optional<Error> EnforceMLPolicy(Info*, const TrainJob*) override { return std::nullopt; }
};

// coscheduling.go: implements EnforcePodGroupPolicyPlugin + ComponentBuilderPlugin
class CoScheduling : public Plugin {
 public:
  static constexpr const char* kName = "CoScheduling";              // coscheduling.go:67
  static constexpr const char* kPodGroupLabel = "scheduling.x-k8s.io/pod-group";
  explicit CoScheduling(Engine& eng) : eng_(eng) {}
  std::string Name() const override { return kName; }
  std::optional<Error> EnforcePodGroupPolicy(Info* info, const TrainJob* trainJob);   // :91-101
  struct BuildResult {
    std::optional<PodGroup> object;  // (nil, nil) <=> no object and no error
    std::optional<Error> error;
  };
  // :103-148. `existing` = the PodGroup the client Get returned (nullptr = NotFound).
  BuildResult Build(const Info* info, const TrainJob* trainJob, const PodGroup* existing);
  // Batch form: one kernel launch aggregates every (info, trainJob) pair.
  std::vector<BuildResult> BuildBatch(const std::vector<const Info*>& infos,
                                      const std::vector<const TrainJob*>& trainJobs,
                                      const std::vector<const PodGroup*>& existing);

 private:
  Engine& eng_;
};

bool NeedsCreateOrUpdate(const PodGroup* old, const PodGroup& pg, bool suspended);  // :150-153

// ------------------------------------------------------------------ node inventory
// The Node informer's event-handler side of pe_update_nodes: node name -> slot map, lowest-free-slot
// reuse, and a pending delta batch flushed in one call.  A Node carries status.allocatable and the
// summed requests of the pods bound to it (the scheduler cache's view); keys without an engine
// dimension (pods, hugepages-*) are not part of the fit and are ignored.
struct Node {
  std::string name;
  ResourceList allocatable;
  ResourceList requested;
  uint32_t label_bits = 0;   // the node's labels as the engine's label bits (placement.h `need`)
  int32_t island = -1;
};

class NodeInventory {
 public:
  // Loads `slots` empty slots on the engine (nothing fits a slot until a node arrives in it).
  NodeInventory(Engine& eng, int64_t slots);
  void OnAdd(const Node& node);              // lowest free slot; Error{PE_ENOMEM} when every slot is used
  void OnUpdate(const Node& node);           // rewrites the node's slot (an unknown node is added)
  void OnDelete(const std::string& name);    // empties the slot (unknown names are ignored)
  int64_t Flush();                           // one pe_update_nodes call; returns the entries sent
  std::optional<int64_t> SlotOf(const std::string& name) const;
  int64_t Size() const { return (int64_t)slot_of_.size(); }
  int64_t Pending() const { return (int64_t)p_slot_.size(); }

 private:
  void stage(int64_t slot, const Node* node);   // nullptr: remove
  Engine& eng_;
  int64_t slots_;
  std::map<std::string, int64_t> slot_of_;
  std::set<int64_t> free_;
  std::vector<int64_t> p_slot_, p_cap_, p_used_;
  std::vector<uint8_t> p_op_;
  std::vector<uint32_t> p_lab_;
  std::vector<int32_t> p_isl_;
};

// ------------------------------------------------------------------ flattening (exposed for tests)

// The CSR of one pe_pg_min_resources_keys batch over a per-call KEY TABLE: every ResourceName the
// containers name (the reference sums any key: util.go:80-103, coscheduling.go:112-116), numbered in
// first-seen order.  The quantities stay exact here; run time picks each key's decimal scale (the
// finest exponent its nonzero quantities need, Quantity::Exp10) and converts them to int64 counts of
// 10^scale units -- a value with no int64 at its key's scale makes its job an overflow (inf.Dec in Go).
struct Flat {
  std::vector<int32_t> job_group_off{0}, min_member, group_replicas, group_cont_off{0};
  std::vector<uint8_t> cont_kind;          // PE_KIND_*
  std::vector<int32_t> ent_off{0};         // container c's entries: [ent_off[c], ent_off[c + 1])
  std::vector<int32_t> ent_key;            // key id of each entry
  std::vector<Quantity> ent_q;
  std::vector<std::string> keys;           // key id -> ResourceName
  std::map<std::string, int32_t> key_id;
  std::vector<int> Scales() const;         // per key id
};
// Each call appends exactly one job (V1Job / Info) or one group (V2PodGroup) or nothing (throws
// Error{PE_EINVAL} on a negative quantity).
void FlattenV1Job(int32_t minMember, const std::map<ReplicaType, ReplicaSpec>& replicas,
                  const PriorityClassGetFunc& pcGetFunc, Flat* out, const V1OrderPolicy& order = {});
void FlattenV2PodGroup(int32_t replicas, const PodSpec& pod, Flat* out);
void FlattenV2Info(const Info& info, Flat* out);

}  // namespace kf
