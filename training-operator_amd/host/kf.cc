#include "kf.h"

#include <algorithm>
#include <utility>

namespace kf {

// ------------------------------------------------------------------ engine

Engine::Engine(int device_id, std::string gpu_resource_name) {
  dims_.gpu = std::move(gpu_resource_name);
  pe_config cfg{};
  cfg.device_id = device_id;
  cfg.rank = 0;
  cfg.world_size = 1;
  cfg.gpu_resource_name = dims_.gpu.c_str();
  const int rc = pe_create(&cfg, &ctx_);
  if (rc != PE_OK) throw Error{rc, "pe_create failed (no GPU: the engine has no CPU fallback)"};
}

Engine::~Engine() { pe_destroy(ctx_); }

int Dims::dim_of(const std::string& r) const {
  if (r == "cpu") return 0;
  if (r == "memory") return 1;
  if (r == gpu) return 2;
  if (r == "ephemeral-storage") return 3;
  return -1;
}

std::string Dims::name_of(int d) const {
  static const char* n[] = {"cpu", "memory", nullptr, "ephemeral-storage"};
  return d == 2 ? gpu : n[d];
}

// ------------------------------------------------------------------ flattening

static void add_record(const ResourceList* rl, int kind, Flat* out) {
  if (rl) {
    for (const auto& kv : *rl) {
      if (kv.second.Negative()) throw Error{PE_EINVAL, kv.first + "=" + kv.second.String() + " is negative"};
      auto it = out->key_id.find(kv.first);
      if (it == out->key_id.end()) {
        it = out->key_id.emplace(kv.first, (int32_t)out->keys.size()).first;
        out->keys.push_back(kv.first);
      }
      out->ent_key.push_back(it->second);
      out->ent_q.push_back(kv.second);
    }
  }
  out->cont_kind.push_back((uint8_t)kind);
  out->ent_off.push_back((int32_t)out->ent_key.size());
}

std::vector<int> Flat::Scales() const {
  std::vector<int> sc(keys.size(), 0);
  std::vector<bool> seen(keys.size(), false);
  for (size_t e = 0; e < ent_key.size(); ++e) {
    if (ent_q[e].IsZero()) continue;
    const int k = ent_key[e];
    const int x = ent_q[e].Exp10();
    sc[k] = seen[k] ? std::min(sc[k], x) : x;
    seen[k] = true;
  }
  return sc;
}

static void end_group(int32_t replicas, Flat* out) {
  out->group_replicas.push_back(replicas);
  out->group_cont_off.push_back((int32_t)out->cont_kind.size());
}

static void end_job(int32_t min_member, Flat* out) {
  out->min_member.push_back(min_member);
  out->job_group_off.push_back((int32_t)out->group_replicas.size());
}

// util.go:110-124: priority from the PriorityClass lister (error/nil -> 0), sorted DESC.  Go's
// sort.Sort leaves equal priorities in map-iteration order (random); we apply V1OrderPolicy.
std::vector<ReplicaType> ReplicaOrderV1(const std::map<ReplicaType, ReplicaSpec>& replicas,
                                        const PriorityClassGetFunc& pcGetFunc, const V1OrderPolicy& order) {
  struct Ent {
    int32_t pri;
    size_t rank;   // position in tie_order, or tie_order.size() for unlisted types
    ReplicaType t;
  };
  std::vector<Ent> pri;
  for (const auto& kv : replicas) {
    std::optional<PriorityClass> pc;
    if (pcGetFunc) pc = pcGetFunc(kv.second.template_spec.priority_class_name);
    const size_t rank = (size_t)(std::find(order.tie_order.begin(), order.tie_order.end(), kv.first) -
                                 order.tie_order.begin());
    pri.push_back({pc ? pc->value : 0, rank, kv.first});
  }
  std::sort(pri.begin(), pri.end(), [](const Ent& a, const Ent& b) {
    if (a.pri != b.pri) return a.pri > b.pri;
    if (a.rank != b.rank) return a.rank < b.rank;
    return a.t < b.t;
  });
  std::vector<ReplicaType> out;
  for (auto& p : pri) out.push_back(p.t);
  return out;
}

PriorityClassGetFunc PriorityClassInformer::Lister() const {
  return [this](const std::string& name) -> std::optional<PriorityClass> {
    auto it = values_.find(name);
    if (it == values_.end()) return std::nullopt;   // lister NotFound -> priority 0
    return PriorityClass{it->second};
  };
}

// Roll the arrays back to their sizes at entry if a record throws (one job is all-or-nothing).
struct FlatTxn {
  Flat* f;
  size_t j, g, c, r;
  bool done = false;
  explicit FlatTxn(Flat* out)
      : f(out), j(out->job_group_off.size()), g(out->group_replicas.size()), c(out->cont_kind.size()),
        r(out->ent_key.size()) {}
  ~FlatTxn() {
    if (done) return;
    f->job_group_off.resize(j);
    f->min_member.resize(j - 1);
    f->group_replicas.resize(g);
    f->group_cont_off.resize(g + 1);
    f->cont_kind.resize(c);
    f->ent_off.resize(c + 1);
    f->ent_key.resize(r);
    f->ent_q.resize(r);
    // (a key first seen in the rolled-back records stays in the table: it is simply never present)
  }
};

void FlattenV1Job(int32_t minMember, const std::map<ReplicaType, ReplicaSpec>& replicas,
                  const PriorityClassGetFunc& pcGetFunc, Flat* out, const V1OrderPolicy& order) {
  FlatTxn txn(out);
  for (const ReplicaType& t : ReplicaOrderV1(replicas, pcGetFunc, order)) {
    const ReplicaSpec& spec = replicas.at(t);
    for (const Container& c : spec.template_spec.containers) {
      // AddResourceList (util.go:79-104): Requests keys, or Limits only when Requests is nil
      const ResourceList* rl = c.requests ? &*c.requests : (c.limits ? &*c.limits : nullptr);
      add_record(rl, PE_KIND_CONTAINER, out);
    }
    end_group(spec.replicas ? *spec.replicas : -1, out);
  }
  end_job(minMember, out);
  txn.done = true;
}

void FlattenV2PodGroup(int32_t replicas, const PodSpec& pod, Flat* out) {
  FlatTxn txn(out);
  for (const Container& c : pod.init_containers) {
    const bool sidecar = c.restart_policy && *c.restart_policy == "Always";
    add_record(c.requests ? &*c.requests : nullptr, sidecar ? PE_KIND_SIDECAR : PE_KIND_INIT, out);
  }
  for (const Container& c : pod.containers) add_record(c.requests ? &*c.requests : nullptr, PE_KIND_CONTAINER, out);
  if (pod.overhead) add_record(&*pod.overhead, PE_KIND_OVERHEAD, out);
  end_group(replicas, out);
  txn.done = true;
}

void FlattenV2Info(const Info& info, Flat* out) {
  FlatTxn txn(out);
  for (const auto& kv : info.scheduler.total_requests) {
    add_record(&kv.second.pod_requests, PE_KIND_CONTAINER, out);
    end_group(kv.second.replicas, out);
  }
  end_job(0, out);
  txn.done = true;
}

// ------------------------------------------------------------------ aggregation through the ABI

struct AggOut {
  std::vector<std::string> keys;
  std::vector<int> scale;        // per key: results are counts of 10^scale
  std::vector<int64_t> res;      // [J][keys]
  std::vector<uint8_t> present;  // [J][keys] 0 / 1
  std::vector<uint8_t> overflow;
  std::vector<int32_t> members;
};

// One pe_pg_min_resources_keys call per slice of <= PE_MAX_KEYS keys (keys never interact; every
// slice returns the same members).  A value with no int64 at its key's scale marks its job overflowed
// on the host (its records carry 0), exactly like a sum the kernel flags.
static AggOut run_agg(Engine& eng, int mode, const Flat& f) {
  const int64_t J = (int64_t)f.job_group_off.size() - 1;
  const int64_t C = (int64_t)f.cont_kind.size();
  const int nk = (int)f.keys.size();
  AggOut o;
  o.keys = f.keys;
  o.scale = f.Scales();
  o.res.assign((size_t)J * nk, 0);
  o.present.assign((size_t)J * nk, 0);
  o.overflow.assign((size_t)J, 0);
  o.members.assign((size_t)J, 0);
  if (J == 0) return o;
  std::vector<int64_t> val(f.ent_q.size(), 0);
  for (int64_t j = 0; j < J; ++j)
    for (int32_t g = f.job_group_off[j]; g < f.job_group_off[j + 1]; ++g)
      for (int32_t c = f.group_cont_off[g]; c < f.group_cont_off[g + 1]; ++c)
        for (int32_t e = f.ent_off[c]; e < f.ent_off[c + 1]; ++e) {
          const std::optional<int64_t> v = f.ent_q[e].Scaled(o.scale[f.ent_key[e]]);
          if (v) val[e] = *v;
          else o.overflow[j] = 1;
        }
  std::vector<int64_t> req, res((size_t)J * PE_MAX_KEYS);
  std::vector<uint32_t> flags((size_t)C);
  std::vector<uint16_t> pres((size_t)J);
  std::vector<uint8_t> ovf((size_t)J);
  for (int lo = 0; lo < std::max(nk, 1); lo += PE_MAX_KEYS) {
    const int n = std::max(1, std::min(PE_MAX_KEYS, nk - lo));   // (no key at all: one empty key for members)
    req.assign((size_t)C * n, 0);
    for (int64_t c = 0; c < C; ++c) {
      uint32_t fl = (uint32_t)f.cont_kind[c] << PE_KEYS_KIND_SHIFT;
      for (int32_t e = f.ent_off[c]; e < f.ent_off[c + 1]; ++e) {
        const int k = f.ent_key[e] - lo;
        if (k < 0 || k >= n || lo + k >= nk) continue;
        req[(size_t)c * n + k] = val[e];
        fl |= 1u << k;
      }
      flags[c] = fl;
    }
    const int rc = pe_pg_min_resources_keys(eng.ctx(), mode, J, n, f.job_group_off.data(), f.min_member.data(),
                                            f.group_replicas.data(), f.group_cont_off.data(), req.data(),
                                            flags.data(), res.data(), pres.data(), o.members.data(), ovf.data());
    if (rc != PE_OK && rc != PE_EOVERFLOW) throw Error{rc, pe_last_error(eng.ctx())};
    for (int64_t j = 0; j < J; ++j) {
      o.overflow[j] |= ovf[j];
      for (int k = 0; k < n && lo + k < nk; ++k) {
        o.res[(size_t)j * nk + lo + k] = res[(size_t)j * n + k];
        o.present[(size_t)j * nk + lo + k] = (uint8_t)(pres[j] >> k & 1);
      }
    }
  }
  return o;
}

static ResourceList to_list(const AggOut& o, int64_t j, const std::map<std::string, Format>* formats = nullptr) {
  if (o.overflow[j]) throw Error{PE_EOVERFLOW, "int64 overflow: the reference would switch to inf.Dec"};
  ResourceList rl;
  const size_t nk = o.keys.size();
  for (size_t k = 0; k < nk; ++k) {
    if (!o.present[j * nk + k]) continue;
    const std::string& key = o.keys[k];
    const auto f = formats ? formats->find(key) : std::map<std::string, Format>::const_iterator{};
    const Format fmt = formats && f != formats->end() ? f->second : key == "cpu" ? Format::kDecimalSI : Format::kBinarySI;
    rl[key] = Quantity::FromScaled(o.res[j * nk + k], o.scale[k], fmt);
  }
  return rl;
}

// Quantity.Add's format rule (quantity.go Add: `if q.i.value == 0 { q.Format = y.Format }`, and the
// same for the inf.Dec branch): the running sum adopts the addend's format while it is still 0.
struct FormatAcc {
  std::map<std::string, Format> fmt;
  std::map<std::string, bool> nonzero;
  void add(const std::string& key, const Quantity& q, bool first_copies) {
    auto it = fmt.find(key);
    if (it == fmt.end()) {
      // AddResourceList deep-copies the first quantity; Build's zero Quantity{} adopts it on Add
      fmt[key] = q.format();
      nonzero[key] = !q.IsZero();
      (void)first_copies;
      return;
    }
    if (!nonzero[key]) it->second = q.format();
    if (!q.IsZero()) nonzero[key] = true;
  }
};

// ------------------------------------------------------------------ v1

int32_t GetTotalReplicas(const std::map<ReplicaType, ReplicaSpec>& replicas) {
  uint32_t total = 0;   // Go int32 addition wraps; signed overflow would be UB here, so add unsigned
  for (const auto& kv : replicas) total += (uint32_t)(kv.second.replicas ? *kv.second.replicas : 1);  // k8sutil.go:131-133
  return (int32_t)total;
}

std::map<std::string, Format> MinResourcesFormatsV1(int32_t minMember, const std::map<ReplicaType, ReplicaSpec>& replicas,
                                                    const PriorityClassGetFunc& pcGetFunc,
                                                    const V1OrderPolicy& order) {
  // util.go:126-141 walk: only counted pods add, pods of one type are identical, so one pass per
  // type that counts at least one pod gives the same first-nonzero / last-zero answer
  FormatAcc acc;
  int64_t pod_cnt = 0;
  for (const ReplicaType& t : ReplicaOrderV1(replicas, pcGetFunc, order)) {
    const ReplicaSpec& spec = replicas.at(t);
    if (!spec.replicas) continue;
    const int64_t k = std::min<int64_t>(*spec.replicas, std::max<int64_t>(0, (int64_t)minMember - pod_cnt));
    if (k <= 0) continue;
    pod_cnt += k;
    for (int64_t pod = 0; pod < std::min<int64_t>(k, 2); ++pod)   // a 2nd pod only re-adds the same formats
      for (const Container& c : spec.template_spec.containers) {
        const ResourceList* rl = c.requests ? &*c.requests : (c.limits ? &*c.limits : nullptr);
        if (rl)
          for (const auto& kv : *rl) acc.add(kv.first, kv.second, true);
      }
  }
  return acc.fmt;
}

ResourceList CalcPGMinResources(Engine& eng, int32_t minMember, const std::map<ReplicaType, ReplicaSpec>& replicas,
                                const PriorityClassGetFunc& pcGetFunc, const V1OrderPolicy& order) {
  Flat f;
  FlattenV1Job(minMember, replicas, pcGetFunc, &f, order);
  const auto formats = MinResourcesFormatsV1(minMember, replicas, pcGetFunc, order);
  return to_list(run_agg(eng, PE_MODE_V1, f), 0, &formats);
}

std::vector<ResourceList> CalcPGMinResourcesBatch(Engine& eng, const std::vector<V1Job>& jobs,
                                                  const PriorityClassGetFunc& pcGetFunc, const V1OrderPolicy& order) {
  Flat f;
  for (const V1Job& j : jobs) FlattenV1Job(j.min_member, j.replicas, pcGetFunc, &f, order);
  AggOut o = run_agg(eng, PE_MODE_V1, f);
  std::vector<ResourceList> out;
  for (size_t j = 0; j < jobs.size(); ++j) {
    const auto formats = MinResourcesFormatsV1(jobs[j].min_member, jobs[j].replicas, pcGetFunc, order);
    out.push_back(to_list(o, (int64_t)j, &formats));
  }
  return out;
}

PodGroupSpecV1 CalcPodGroupSpecV1(Engine& eng, const std::map<ReplicaType, ReplicaSpec>& replicas,
                                  const SchedulingPolicy* policy, const PriorityClassGetFunc& pcGetFunc,
                                  const V1OrderPolicy& order) {
  PodGroupSpecV1 pg;
  pg.min_member = GetTotalReplicas(replicas);                                    // job.go:251
  if (policy && policy->min_available) pg.min_member = *policy->min_available;   // job.go:258-260
  if (policy && policy->min_resources) pg.min_resources = *policy->min_resources;  // job.go:267-269
  else pg.min_resources = CalcPGMinResources(eng, pg.min_member, replicas, pcGetFunc, order);  // job.go:275-277
  return pg;
}

// ------------------------------------------------------------------ v2

Info NewInfo(Engine& eng, const InfoOptions& opts) {
  Info info;
  info.labels = opts.labels;
  info.annotations = opts.annotations;
  info.runtime_policy.ml_policy = opts.ml_policy;
  info.runtime_policy.pod_group_policy = opts.pod_group_policy;
  if (opts.pod_spec_replicas.empty()) return info;
  Flat f;
  for (const PodSpecReplica& r : opts.pod_spec_replicas) {
    FlattenV2PodGroup(1, r.pod_spec, &f);   // per-pod requests: one group of 1 replica per job
    end_job(0, &f);
  }
  AggOut o = run_agg(eng, PE_MODE_V2, f);
  for (size_t i = 0; i < opts.pod_spec_replicas.size(); ++i) {
    const PodSpecReplica& r = opts.pod_spec_replicas[i];
    // Print formats through kueue's merges (containers, then sidecar / init containers, then
    // overhead, by the Add rule).  kueue v0.6.3 is not in the container: this order is an
    // assumption ("parity unpinned"); the values are exact either way.
    FormatAcc acc;
    for (const Container& c : r.pod_spec.containers)
      if (c.requests)
        for (const auto& kv : *c.requests) acc.add(kv.first, kv.second, true);
    for (const Container& c : r.pod_spec.init_containers)
      if (c.requests)
        for (const auto& kv : *c.requests) acc.add(kv.first, kv.second, true);
    if (r.pod_spec.overhead)
      for (const auto& kv : *r.pod_spec.overhead) acc.add(kv.first, kv.second, true);
    info.scheduler.total_requests[r.name] =
        TotalResourceRequest{r.replicas, to_list(o, (int64_t)i, &acc.fmt)};
  }
  return info;
}

PodSpec ApplyTrainerResourcesPerNode(const PodSpec& pod, const TrainJob& trainJob) {
  PodSpec out = pod;
  if (!trainJob.resources_per_node) return out;
  for (Container& c : out.containers)
    if (c.name == "trainer") {   // constants.ContainerTrainer
      c.requests = trainJob.resources_per_node->requests;
      c.limits = trainJob.resources_per_node->limits;
    }
  return out;
}

std::optional<Error> ApplyTotalRequestsOptions(Engine& eng, const TotalRequestsOptions& opts, Info* info,
                                               const TrainJob* trainJob, const PodSpec& runtime_trainer_pod) {
  if (!opts.from_resources_per_node || !info || !trainJob || !trainJob->resources_per_node) return std::nullopt;
  auto it = info->scheduler.total_requests.find("trainer-node");   // constants.JobTrainerNode
  if (it == info->scheduler.total_requests.end()) return std::nullopt;
  try {
    InfoOptions o;
    o.pod_spec_replicas = {{"trainer-node", 1, ApplyTrainerResourcesPerNode(runtime_trainer_pod, *trainJob)}};
    it->second.pod_requests = NewInfo(eng, o).scheduler.total_requests.at("trainer-node").pod_requests;
  } catch (const Error& e) {
    return e;
  }
  return std::nullopt;
}

static std::optional<Error> rewrite_trainer_replicas(Info* info, const TrainJob* trainJob) {
  std::optional<int32_t> num_nodes = info->runtime_policy.ml_policy->num_nodes;
  if (trainJob && trainJob->trainer_num_nodes) num_nodes = trainJob->trainer_num_nodes;
  info->trainer.num_nodes = num_nodes;
  auto it = info->scheduler.total_requests.find("trainer-node");   // constants.JobTrainerNode
  if (it != info->scheduler.total_requests.end()) it->second.replicas = num_nodes ? *num_nodes : 1;
  return std::nullopt;
}

std::optional<Error> PlainML::EnforceMLPolicy(Info* info, const TrainJob* trainJob) {
  if (!info || !info->runtime_policy.ml_policy || info->runtime_policy.ml_policy->source != MLPolicy::kPlainML)
    return std::nullopt;
  return rewrite_trainer_replicas(info, trainJob);
}

std::optional<Error> Torch::EnforceMLPolicy(Info* info, const TrainJob* trainJob) {
  if (!info || !info->runtime_policy.ml_policy || info->runtime_policy.ml_policy->source != MLPolicy::kTorch)
    return std::nullopt;
  return rewrite_trainer_replicas(info, trainJob);
}

std::optional<Error> CoScheduling::EnforcePodGroupPolicy(Info* info, const TrainJob* trainJob) {
  if (!info || !info->runtime_policy.pod_group_policy || !trainJob) return std::nullopt;
  info->scheduler.pod_labels[kPodGroupLabel] = trainJob->name;
  return std::nullopt;
}

bool NeedsCreateOrUpdate(const PodGroup* old, const PodGroup& pg, bool suspended) {
  if (!old) return true;
  if (!suspended) return false;
  const bool spec_equal = old->min_member == pg.min_member && EqualResourceList(old->min_resources, pg.min_resources) &&
                          old->schedule_timeout_seconds == pg.schedule_timeout_seconds;
  return !spec_equal || old->labels != pg.labels || old->annotations != pg.annotations;
}

std::vector<CoScheduling::BuildResult> CoScheduling::BuildBatch(const std::vector<const Info*>& infos,
                                                                const std::vector<const TrainJob*>& trainJobs,
                                                                const std::vector<const PodGroup*>& existing) {
  std::vector<BuildResult> out(infos.size());
  std::vector<size_t> idx;
  Flat f;
  for (size_t i = 0; i < infos.size(); ++i) {
    const Info* info = infos[i];
    if (!info || !info->runtime_policy.pod_group_policy || !info->runtime_policy.pod_group_policy->coscheduling ||
        !trainJobs[i])
      continue;  // coscheduling.go:104-106: (nil, nil)
    try {
      FlattenV2Info(*info, &f);
      idx.push_back(i);
    } catch (const Error& e) {
      out[i].error = e;
    }
  }
  AggOut o;
  try {
    o = run_agg(eng_, PE_MODE_V2, f);
  } catch (const Error& e) {
    for (size_t k : idx) out[k].error = e;
    return out;
  }
  for (size_t n = 0; n < idx.size(); ++n) {
    const size_t i = idx[n];
    PodGroup pg;
    pg.name = trainJobs[i]->name;
    pg.ns = trainJobs[i]->ns;
    pg.min_member = o.members[n];
    try {
      pg.min_resources = to_list(o, (int64_t)n);
    } catch (const Error& e) {
      out[i].error = e;
      continue;
    }
    // print formats: totalResources[k] starts as a zero Quantity{} and Adds quantity * replicas
    // (coscheduling.go:110-116); Go ranges TotalRequests in map order (random), we in name order
    FormatAcc acc;
    for (const auto& kv : infos[i]->scheduler.total_requests)
      for (const auto& q : kv.second.pod_requests) {
        Quantity scaled = q.second.IsZero() || kv.second.replicas == 0 ? Quantity::FromScaled(0, 0, q.second.format())
                                                                       : q.second;
        acc.add(q.first, scaled, false);
      }
    for (auto& kv : pg.min_resources) {
      auto f = acc.fmt.find(kv.first);
      if (f != acc.fmt.end()) kv.second = kv.second.WithFormat(f->second);
    }
    pg.schedule_timeout_seconds = infos[i]->runtime_policy.pod_group_policy->coscheduling->schedule_timeout_seconds;
    pg.owner_api_version = "kubeflow.org/v2alpha1";   // SetControllerReference (coscheduling.go:134)
    pg.owner_kind = "TrainJob";
    pg.owner_name = trainJobs[i]->name;
    pg.owner_uid = trainJobs[i]->uid;
    if (NeedsCreateOrUpdate(existing.empty() ? nullptr : existing[i], pg, trainJobs[i]->suspend)) out[i].object = pg;
  }
  return out;
}

CoScheduling::BuildResult CoScheduling::Build(const Info* info, const TrainJob* trainJob, const PodGroup* existing) {
  return BuildBatch({info}, {trainJob}, {existing})[0];
}

// ------------------------------------------------------------------ v1 SyncPodGroup (8f row 1)

SyncPodGroupResult SyncPodGroupV1(Engine& eng, GangScheduler flavour, const JobMeta& job,
                                  const std::map<ReplicaType, ReplicaSpec>& replicas, const SchedulingPolicy* policy,
                                  const PriorityClassGetFunc& pcGetFunc, const PodGroup* existing,
                                  const V1OrderPolicy& order) {
  // job.go:251-277
  int32_t min_member = GetTotalReplicas(replicas);
  std::string queue = "default", priority_class;
  std::optional<int32_t> timeout;
  std::optional<ResourceList> min_resources;
  if (policy) {
    if (policy->min_available) min_member = *policy->min_available;
    if (!policy->queue.empty()) queue = policy->queue;
    if (!policy->priority_class.empty()) priority_class = policy->priority_class;
    if (policy->min_resources) min_resources = *policy->min_resources;
    if (policy->schedule_timeout_seconds) timeout = policy->schedule_timeout_seconds;
  }
  if (!min_resources) min_resources = CalcPGMinResources(eng, min_member, replicas, pcGetFunc, order);

  SyncPodGroupResult r;
  if (existing) {
    r.action = SyncPodGroupResult::kUpdate;   // scheduling.go:38-44: the cmp.Diff never matches
    r.object = *existing;
  } else {
    r.action = SyncPodGroupResult::kCreate;   // scheduling.go:49-56
    r.object = PodGroup{};
    r.object.name = job.name;
    r.object.ns = job.ns;
    r.object.annotations = job.annotations;
    r.object.owner_api_version = job.api_version;
    r.object.owner_kind = job.kind;
    r.object.owner_name = job.name;
    r.object.owner_uid = job.uid;
  }
  PodGroup& pg = r.object;
  pg.flavour = flavour;
  // the fill replaces the whole Spec (job.go:291-297, 306-310)
  pg.min_member = min_member;
  pg.min_resources = *min_resources;
  if (flavour == GangScheduler::kVolcano) {
    if (!pg.queue.empty()) queue = pg.queue;   // job.go:287-289: the object's queue wins
    pg.queue = queue;
    pg.priority_class_name = priority_class;
    pg.schedule_timeout_seconds.reset();
  } else {
    pg.schedule_timeout_seconds = timeout;
    pg.queue.clear();
    pg.priority_class_name.clear();
  }
  return r;
}

// ------------------------------------------------------------------ PodGroup JSON (8f row 1)

static void json_str(std::string& o, const std::string& s) {
  // encoding/json: HTML-safe escaping by default (<, >, & as \u00XX), \n \r \t, other controls \u00XX
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  for (size_t i = 0; i < s.size(); ++i) {
    const unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20 || c == '<' || c == '>' || c == '&') {
          o += "\\u00";
          o.push_back(hex[c >> 4]);
          o.push_back(hex[c & 15]);
        } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
                   ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
          o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";   // U+2028 / U+2029
          i += 2;
        } else {
          o.push_back((char)c);
        }
    }
  }
  o.push_back('"');
}

static void json_map(std::string& o, const std::map<std::string, std::string>& m) {
  o.push_back('{');
  bool first = true;
  for (const auto& kv : m) {   // Go sorts map keys
    if (!first) o.push_back(',');
    first = false;
    json_str(o, kv.first);
    o.push_back(':');
    json_str(o, kv.second);
  }
  o.push_back('}');
}

static void json_resources(std::string& o, const ResourceList& rl) {
  std::map<std::string, std::string> m;
  for (const auto& kv : rl) m[kv.first] = kv.second.String();
  json_map(o, m);
}

std::string PodGroupJSON(const PodGroup& pg) {
  const bool volcano = pg.flavour == GangScheduler::kVolcano;
  std::string o = "{\"kind\":\"PodGroup\",\"apiVersion\":";
  json_str(o, volcano ? "scheduling.volcano.sh/v1beta1" : "scheduling.x-k8s.io/v1alpha1");
  // metav1.ObjectMeta, declaration order; creationTimestamp is a struct (omitempty never drops it)
  o += ",\"metadata\":{\"name\":";
  json_str(o, pg.name);
  if (!pg.ns.empty()) {
    o += ",\"namespace\":";
    json_str(o, pg.ns);
  }
  o += ",\"creationTimestamp\":null";
  if (!pg.labels.empty()) {
    o += ",\"labels\":";
    json_map(o, pg.labels);
  }
  if (!pg.annotations.empty()) {
    o += ",\"annotations\":";
    json_map(o, pg.annotations);
  }
  if (!pg.owner_kind.empty()) {
    o += ",\"ownerReferences\":[{\"apiVersion\":";
    json_str(o, pg.owner_api_version);
    o += ",\"kind\":";
    json_str(o, pg.owner_kind);
    o += ",\"name\":";
    json_str(o, pg.owner_name);
    o += ",\"uid\":";
    json_str(o, pg.owner_uid);
    o += ",\"controller\":true,\"blockOwnerDeletion\":true}]";
  }
  o += "},\"spec\":{";
  std::string spec;
  auto field = [&](const char* name) {
    if (!spec.empty()) spec.push_back(',');
    spec += "\"";
    spec += name;
    spec += "\":";
  };
  if (pg.min_member != 0) {   // int32 omitempty
    field("minMember");
    spec += std::to_string(pg.min_member);
  }
  if (volcano) {
    // v1beta1.PodGroupSpec: minMember, minTaskMember, queue, priorityClassName, minResources (*ResourceList)
    if (!pg.queue.empty()) {
      field("queue");
      json_str(spec, pg.queue);
    }
    if (!pg.priority_class_name.empty()) {
      field("priorityClassName");
      json_str(spec, pg.priority_class_name);
    }
    field("minResources");   // a non-nil pointer: written even when the list is empty
    json_resources(spec, pg.min_resources);
  } else {
    // v1alpha1.PodGroupSpec: minMember, minResources (map, omitempty), scheduleTimeoutSeconds (*int32)
    if (!pg.min_resources.empty()) {
      field("minResources");
      json_resources(spec, pg.min_resources);
    }
    if (pg.schedule_timeout_seconds) {
      field("scheduleTimeoutSeconds");
      spec += std::to_string(*pg.schedule_timeout_seconds);
    }
  }
  o += spec;
  // status of a new object: every field omitempty except scheduler-plugins' scheduleStartTime (metav1.Time)
  o += volcano ? "},\"status\":{}}" : "},\"status\":{\"scheduleStartTime\":null}}";
  return o;
}

// ------------------------------------------------------------------ node inventory

NodeInventory::NodeInventory(Engine& eng, int64_t slots) : eng_(eng), slots_(slots) {
  if (slots < 0) throw Error{PE_EINVAL, "slots < 0"};
  std::vector<int64_t> zero((size_t)PE_DIMS * (size_t)slots, 0);
  int rc = pe_load_nodes(eng_.ctx(), slots, zero.data(), zero.data(), nullptr, nullptr);
  if (rc != PE_OK) throw Error{rc, pe_last_error(eng_.ctx())};
  std::vector<int64_t> ids((size_t)slots);
  for (int64_t i = 0; i < slots; ++i) ids[i] = i;
  std::vector<uint8_t> ops((size_t)slots, (uint8_t)PE_NODE_REMOVE);
  rc = pe_update_nodes(eng_.ctx(), slots, ids.data(), ops.data(), nullptr, nullptr, nullptr, nullptr);
  if (rc != PE_OK) throw Error{rc, pe_last_error(eng_.ctx())};
  for (int64_t i = 0; i < slots; ++i) free_.insert(free_.end(), i);
}

void NodeInventory::stage(int64_t slot, const Node* node) {
  int64_t cap[PE_DIMS] = {0, 0, 0, 0}, used[PE_DIMS] = {0, 0, 0, 0};
  if (node) {
    const Dims& dims = eng_.dims();
    auto conv = [&](const ResourceList& rl, int64_t* out) {
      for (const auto& kv : rl) {
        const int d = dims.dim_of(kv.first);
        if (d < 0) continue;
        try {
          out[d] = kv.second.Canonical(kv.first);
        } catch (const QuantityError& e) {
          throw Error{PE_EINVAL, "node " + node->name + ": " + e.msg};
        }
      }
    };
    conv(node->allocatable, cap);   // converted before anything is staged: a bad node changes nothing
    conv(node->requested, used);
  }
  p_slot_.push_back(slot);
  p_op_.push_back((uint8_t)(node ? PE_NODE_SET : PE_NODE_REMOVE));
  p_cap_.insert(p_cap_.end(), cap, cap + PE_DIMS);
  p_used_.insert(p_used_.end(), used, used + PE_DIMS);
  p_lab_.push_back(node ? node->label_bits : 0u);
  p_isl_.push_back(node ? node->island : -1);
}

void NodeInventory::OnAdd(const Node& node) {
  if (slot_of_.count(node.name)) return OnUpdate(node);
  if (free_.empty()) throw Error{PE_ENOMEM, "node inventory full (" + std::to_string(slots_) + " slots)"};
  const int64_t slot = *free_.begin();
  stage(slot, &node);
  free_.erase(free_.begin());
  slot_of_[node.name] = slot;
}

void NodeInventory::OnUpdate(const Node& node) {
  auto it = slot_of_.find(node.name);
  if (it == slot_of_.end()) return OnAdd(node);
  stage(it->second, &node);
}

void NodeInventory::OnDelete(const std::string& name) {
  auto it = slot_of_.find(name);
  if (it == slot_of_.end()) return;
  stage(it->second, nullptr);
  free_.insert(it->second);
  slot_of_.erase(it);
}

int64_t NodeInventory::Flush() {
  const int64_t n = (int64_t)p_slot_.size();
  if (n == 0) return 0;
  const int rc = pe_update_nodes(eng_.ctx(), n, p_slot_.data(), p_op_.data(), p_cap_.data(), p_used_.data(),
                                 p_lab_.data(), p_isl_.data());
  if (rc != PE_OK) throw Error{rc, pe_last_error(eng_.ctx())};
  p_slot_.clear();
  p_op_.clear();
  p_cap_.clear();
  p_used_.clear();
  p_lab_.clear();
  p_isl_.clear();
  return n;
}

std::optional<int64_t> NodeInventory::SlotOf(const std::string& name) const {
  auto it = slot_of_.find(name);
  if (it == slot_of_.end()) return std::nullopt;
  return it->second;
}

}  // namespace kf
