// C ABI of the host resolver (include/placement.h, "Host resolver").  Pure C++: no device.
#include <cstring>
#include <new>
#include <vector>

#include "pe_resolver.h"
#include "placement.h"

struct pe_resolver {
  // the resolver keeps pointers into these copies, so they must outlive it
  std::vector<int32_t> jgo, prio, cnt;
  std::vector<int64_t> req;
  std::vector<uint32_t> need;
  pe::Resolver* r = nullptr;
  std::vector<pe::GroupCands> cands;
  std::vector<pe::Update> updates;
  int64_t n_nodes = PE_MAX_NODES;   // listed and seeded node ids must lie below (pe_resolver_set_nodes)
  ~pe_resolver() { delete r; }
};

extern "C" {

int pe_resolver_create(int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority,
                       const int32_t* group_count, const int64_t* group_req, const uint32_t* group_need,
                       pe_resolver** out) {
  if (!out || n_jobs < 0 || (n_jobs > 0 && (!job_group_off || !priority))) return PE_EINVAL;
  *out = nullptr;
  try {
    pe_resolver* h = new pe_resolver();
    h->jgo.assign(job_group_off, job_group_off + (n_jobs > 0 ? n_jobs + 1 : 0));
    if (h->jgo.empty()) h->jgo.push_back(0);
    const int64_t G = h->jgo.back();
    for (int64_t j = 0; j < n_jobs; ++j)
      if (h->jgo[j + 1] < h->jgo[j]) {
        delete h;
        return PE_EINVAL;
      }
    if (G > 0 && (!group_count || !group_req)) {
      delete h;
      return PE_EINVAL;
    }
    h->prio.assign(priority, priority + n_jobs);
    h->cnt.assign(group_count, group_count + G);
    h->req.assign(group_req, group_req + G * PE_DIMS);
    if (group_need) h->need.assign(group_need, group_need + G);
    else h->need.assign((size_t)G, 0u);
    for (int64_t g = 0; g < G; ++g)
      if (h->cnt[g] < 0) {
        delete h;
        return PE_EINVAL;
      }
    for (int64_t v : h->req)
      if (v < 0) {
        delete h;
        return PE_EINVAL;
      }
    h->r = new pe::Resolver(n_jobs, h->jgo.data(), h->prio.data(), h->cnt.data(), h->req.data(), h->need.data());
    *out = h;
    return PE_OK;
  } catch (const std::bad_alloc&) {
    return PE_ENOMEM;
  }
}

void pe_resolver_destroy(pe_resolver* r) { delete r; }

int pe_resolver_set_nodes(pe_resolver* r, int64_t n_nodes) {
  if (!r || n_nodes < 0 || n_nodes > PE_MAX_NODES) return PE_EINVAL;
  r->n_nodes = n_nodes;
  return PE_OK;
}

int pe_resolver_done(const pe_resolver* r) { return r && r->r->done() ? 1 : 0; }

int pe_resolver_next_window(pe_resolver* r, int32_t max_groups, int64_t max_pods, int32_t* out_groups,
                            int32_t* out_n) {
  if (!r || !out_groups || !out_n || max_groups <= 0 || max_pods <= 0) return PE_EINVAL;
  std::vector<int32_t> g;
  r->r->next_window(max_groups, max_pods, g);
  std::memcpy(out_groups, g.data(), g.size() * sizeof(int32_t));
  *out_n = (int32_t)g.size();
  return PE_OK;
}

int pe_resolver_resolve(pe_resolver* r, int32_t n_groups, const int32_t* groups, const uint8_t* blob,
                        int32_t n_shards, int32_t topk, int64_t* out_updates, int64_t max_updates,
                        int64_t* out_n_updates, int32_t* out_consumed) {
  return pe_resolver_resolve_seeded(r, n_groups, groups, blob, n_shards, topk, 0, nullptr, out_updates, max_updates,
                                    out_n_updates, out_consumed);
}

int pe_resolver_resolve_seeded(pe_resolver* r, int32_t n_groups, const int32_t* groups, const uint8_t* blob,
                               int32_t n_shards, int32_t topk, int64_t n_seeds, const int64_t* seeds,
                               int64_t* out_updates, int64_t max_updates, int64_t* out_n_updates,
                               int32_t* out_consumed) {
  if (!r || n_groups < 0 || n_shards < 1 || topk < 1 || !out_n_updates || !out_consumed) return PE_EINVAL;
  if (n_groups > 0 && (!groups || !blob)) return PE_EINVAL;
  if (n_seeds < 0 || (n_seeds > 0 && !seeds)) return PE_EINVAL;
  for (int64_t i = 0; i < n_seeds; ++i)
    if (seeds[i * 6] < 0 || seeds[i * 6] >= r->n_nodes || seeds[i * 6 + 5] < 0 || seeds[i * 6 + 5] > 0xFFFFFFFFll)
      return PE_EINVAL;
  try {
    std::vector<int32_t> g(groups, groups + n_groups);
    for (int32_t x : g)
      if (x < 0 || x >= (int32_t)r->cnt.size()) return PE_EINVAL;
    // every header, node id and key order is checked before the resolver moves (PE_EINVAL, no update)
    pe::parse_window(blob, n_shards, n_groups, topk, r->cands, false, r->n_nodes);
    std::vector<pe::Update> seed((size_t)n_seeds);
    for (int64_t i = 0; i < n_seeds; ++i) {
      seed[i].gid = seeds[i * 6];
      for (int d = 0; d < 4; ++d) seed[i].res[d] = seeds[i * 6 + 1 + d];
      seed[i].labels = (uint32_t)seeds[i * 6 + 5];
    }
    r->updates.clear();
    const bool consumed = r->r->resolve(g, r->cands, r->updates, n_seeds > 0 ? &seed : nullptr);
    if ((int64_t)r->updates.size() > max_updates || (!out_updates && !r->updates.empty())) return PE_EINVAL;
    for (size_t i = 0; i < r->updates.size(); ++i) {
      out_updates[i * 5] = r->updates[i].gid;
      for (int d = 0; d < 4; ++d) out_updates[i * 5 + 1 + d] = r->updates[i].res[d];
    }
    *out_n_updates = (int64_t)r->updates.size();
    *out_consumed = consumed ? 1 : 0;
    return PE_OK;
  } catch (const std::bad_alloc&) {
    return PE_ENOMEM;
  } catch (const pe::CorruptList&) {
    return PE_EINVAL;
  } catch (const std::exception&) {   // (nothing else may cross the C boundary)
    return PE_EINVAL;
  }
}

int pe_resolver_results(const pe_resolver* r, int32_t* out_pod_node, int32_t* out_job_status) {
  if (!r) return PE_EINVAL;
  if (out_pod_node) std::memcpy(out_pod_node, r->r->pod_node().data(), r->r->pod_node().size() * sizeof(int32_t));
  if (out_job_status)
    std::memcpy(out_job_status, r->r->job_status().data(), r->r->job_status().size() * sizeof(int32_t));
  return PE_OK;
}

}  // extern "C"
