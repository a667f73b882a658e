// Host half of the greedy gang placement: sequential, exact resolution of one scan window.
//
// The GPU scans a WINDOW of upcoming groups (identical-pod sets) against one residual snapshot
// and returns, per group, the exact list of the best K clean-node keys plus a limit (every clean
// node with key < limit is listed).  Placements inside the window only change the nodes they
// touch ("dirty" nodes); the resolver re-scores those exactly on the host, so for every pod
//     argmin over all nodes = min(best dirty key, first non-dirty listed key)
// which is the sequential rule of SURVEY.md Appendix B bit for bit.  When a group's list runs
// dry and no dirty node beats its limit, the window ends (NEED_RESCAN): updates are flushed to
// the device and the next window rescans from the current pod.  Pure C++, no HIP: the same code
// runs behind every shard (all ranks resolve identically) and under the CPU tests.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <unordered_map>
#include <vector>

namespace pe {

constexpr int RD = 4;

struct NodeState {
  int64_t res[RD];
  uint32_t labels;
};

// One candidate, byte-identical to the device's CandRec (labels in the low half of a u64), so a
// single-shard window blob is read in place.
struct Cand {
  uint64_t key;
  int64_t res[RD];
  uint32_t labels;
  uint32_t pad_;
};
static_assert(sizeof(Cand) == 48, "Cand must match the 48-B device record");

struct GroupCands {
  const Cand* data = nullptr;  // ascending keys, all clean at the snapshot
  size_t n = 0;
  uint64_t limit = ~0ull;      // every clean node with key < limit is listed
  std::vector<Cand> own;       // storage when the list is a copy (shard merge, or copy_blob)
  size_t size() const { return n; }
  const Cand& operator[](size_t i) const { return data[i]; }
};

struct Update {
  int64_t gid;
  int64_t res[RD];
  uint32_t labels;
};

// Position of the resolver in the (priority-ordered) pod sequence.
struct Cursor {
  int64_t oi = 0;  // position in the job order
  int32_t g = 0;   // group index
  int32_t p = 0;   // next pod of the group
  bool operator==(const Cursor& o) const { return oi == o.oi && g == o.g && p == o.p; }
};

uint64_t score_of(const int64_t left[RD]);
uint64_t key_of(const int64_t res[RD], uint32_t labels, const int64_t q[RD], uint32_t need, uint64_t gid);

// Merge per-shard candidate lists of one group into the global exact list (limit = min).
void merge_shards(const std::vector<const GroupCands*>& parts, GroupCands& out);

// Window blob = n_shards consecutive shard blocks, each n_groups x (16-B header {int32 n,
// int32 flags, uint64 limit} + K x 48-B records {u64 key, i64 res[4], u64 labels}) -- exactly
// what the merge kernel writes.  Parses and merges the shards into cands[n_groups].
// With one shard and copy_blob = false the lists point INTO the blob, which must outlive them.
void parse_window(const uint8_t* blob, int n_shards, int n_groups, int K, std::vector<GroupCands>& cands,
                  bool copy_blob = false);

// Nodes modified since the window's snapshot, as flat struct-of-arrays so the per-group re-score
// is one branch-free (vectorisable) loop; gid -> slot is a direct-mapped array grown on demand.
class DirtySet {
 public:
  int32_t find(int64_t gid) const { return gid < (int64_t)slot_.size() ? slot_[gid] : -1; }
  int32_t upsert(int64_t gid, const NodeState& st);
  void set(int32_t i, const NodeState& st);
  void mark(int32_t i) { touched[i] = 1; }
  NodeState get(int32_t i) const;
  size_t size() const { return gid.size(); }
  void clear();
  // keys of every dirty node for request (q, need) -> out (NO_KEY where it does not fit)
  void keys(const int64_t q[RD], uint32_t need, std::vector<uint64_t>& out) const;
  uint64_t key_at(int32_t i, const int64_t q[RD], uint32_t need) const;
  std::vector<int64_t> gid, r0, r1, r2, r3;
  std::vector<uint32_t> lab;
  std::vector<uint8_t> touched;   // changed in this window (seeded entries start untouched)

 private:
  std::vector<int32_t> slot_;
};

class Resolver {
 public:
  Resolver(int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority, const int32_t* group_count,
           const int64_t* group_req, const uint32_t* group_need);

  bool done() const { return oi_ >= (int64_t)order_.size(); }
  // Groups (global ids, count > 0) of the next window, starting at the cursor (or at `from`);
  // *end receives the cursor just past the window (where it stands if the window is consumed).
  void next_window(int max_groups, int64_t max_pods, std::vector<int32_t>& groups);
  void next_window_from(const Cursor& from, int max_groups, int64_t max_pods, std::vector<int32_t>& groups,
                        Cursor* end) const;
  Cursor cursor() const { return Cursor{oi_, g_, p_}; }
  // Resolve with candidates for exactly the groups returned by next_window (same order).
  // Appends the residual updates to flush; returns true if the whole window was consumed.
  // seed (pipelined form): nodes changed since the snapshot the candidates were scanned on, with
  // their current state -- they start dirty, so the lists' clean entries stay exact; only nodes
  // changed in THIS window are returned as updates.
  bool resolve(const std::vector<int32_t>& groups, const std::vector<GroupCands>& cands,
               std::vector<Update>& updates, const std::vector<Update>* seed = nullptr);

  const std::vector<int32_t>& pod_node() const { return pod_node_; }
  const std::vector<int32_t>& job_status() const { return job_status_; }
  int64_t jobs_placed() const { return jobs_placed_; }
  int64_t jobs_failed() const { return jobs_failed_; }
  int64_t pods_placed() const { return pods_placed_; }
  int64_t rescans() const { return rescans_; }
  int64_t n_pods() const { return (int64_t)pod_node_.size(); }

 private:
  void finish_job(bool ok);
  void advance_group();

  int64_t J_;
  const int32_t* jgo_;
  const int32_t* cnt_;
  const int64_t* req_;
  const uint32_t* need_;
  std::vector<int64_t> order_;
  std::vector<int64_t> pod_off_;
  std::vector<int32_t> pod_node_;
  std::vector<int32_t> job_status_;
  // cursor
  int64_t oi_ = 0;  // position in order_
  int32_t g_ = 0;   // global group index inside the current job
  int32_t p_ = 0;   // next pod of group g_
  // window state
  DirtySet dirty_;
  std::vector<uint64_t> dk_;
  // nodes touched by the current job (exact current residuals, survive window flushes)
  std::unordered_map<int64_t, NodeState> job_nodes_;
  int64_t jobs_placed_ = 0, jobs_failed_ = 0, pods_placed_ = 0, rescans_ = 0;
};

}  // namespace pe
