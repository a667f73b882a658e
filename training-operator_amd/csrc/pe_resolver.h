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
#include <sched.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <sys/mman.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <memory>
#include <new>
#include <stdexcept>
#include <thread>
#include <unordered_map>
#include <vector>

namespace pe {

constexpr int RD = 4;

// One cache line per node: the host mirror is read at random node ids (one DRAM miss each, the
// next candidates prefetched); 40-B records straddled two lines for half the ids, and the second
// line was never prefetched.  PE_NODESTATE_ALIGN=8 restores the packed 40-B record (A/B builds).
#ifndef PE_NODESTATE_ALIGN
#define PE_NODESTATE_ALIGN 64
#endif
struct alignas(PE_NODESTATE_ALIGN) NodeState {
  int64_t res[RD];
  uint32_t labels;
};

// Allocator of the host mirror (one 64-B record per node of the global inventory, 64 MB at 1M nodes,
// read at random ids by the resolver): 2 MiB-aligned and marked MADV_HUGEPAGE, so its reads do not
// also miss the TLB (4 KiB pages: 16k pages for 1M nodes, several times the L2 TLB).  Small arrays
// and PE_NO_HUGE=1 (A/B) take ordinary pages.
template <class T>
struct HugeAlloc {
  using value_type = T;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U>&) {}
  T* allocate(size_t n) {
    constexpr size_t kHuge = (size_t)2 << 20;
    size_t bytes = n * sizeof(T);
    const bool huge = bytes >= 2 * kHuge && !getenv("PE_NO_HUGE");
    size_t align = alignof(T) < 64 ? 64 : alignof(T);
    if (huge) {
      bytes = (bytes + kHuge - 1) / kHuge * kHuge;
      align = kHuge;
    }
    void* p = nullptr;
    if (posix_memalign(&p, align, bytes ? bytes : align) != 0) throw std::bad_alloc();
    if (huge) (void)madvise(p, bytes, MADV_HUGEPAGE);
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t) { free(p); }
  template <class U>
  bool operator==(const HugeAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const HugeAlloc<U>&) const { return false; }
};

// One candidate record of the pe_resolver_* ABI blob (placement.h): key + the node's residual
// snapshot, labels in the low half of a u64.
struct Cand {
  uint64_t key;
  int64_t res[RD];
  uint32_t labels;
  uint32_t pad_;
};
static_assert(sizeof(Cand) == 48, "Cand must match the 48-B ABI record");

// Host copy of the inventory the engine keeps next to the device shard(s): state (residuals +
// labels) of every node of the GLOBAL inventory by id, current at the window's snapshot for every
// clean node.  Key-only candidate lists read their nodes' states here (one cache line per node).
struct Mirror {
  const NodeState* nodes = nullptr;
  int64_t n = 0;
};

// One group's candidate list: either records (data) or keys whose states come from a Mirror.
// Key lists of several shards are merged lazily: the resolver reads a list from its head and
// usually stops after a few entries, so only the consumed prefix is ever merged.
struct GroupCands {
  const Cand* data = nullptr;      // ascending keys, all clean at the snapshot
  const uint64_t* keys = nullptr;  // key-only form (engine windows), one shard
  bool keyed = false;              // key-only (keys, or the lazy shard merge below)
  size_t n = 0;
  uint64_t limit = ~0ull;          // every clean node with key < limit is listed
  std::vector<Cand> own;           // storage when the list is a copy (record shard merge, copy_blob)
  // lazy k-way merge of per-shard key lists (each ascending, cut at limit)
  std::vector<const uint64_t*> part;
  std::vector<size_t> part_n;
  mutable std::vector<size_t> head;
  mutable std::vector<uint64_t> merged;
  size_t size() const { return n; }
  uint64_t key(size_t i) const {
    if (keys) return keys[i];
    if (!keyed) return data[i].key;
    while (merged.size() <= i) {
      size_t best = 0;
      uint64_t bk = ~0ull;
      for (size_t r = 0; r < part.size(); ++r)
        if (head[r] < part_n[r] && part[r][head[r]] < bk) {
          bk = part[r][head[r]];
          best = r;
        }
      ++head[best];
      merged.push_back(bk);
    }
    return merged[i];
  }
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

// A candidate list the resolver cannot trust: a header count outside [0, K] (it would read past the
// group's slot), a listed node id outside the inventory, or (record blobs) keys out of order.  The
// blobs may arrive over any transport (placement.h), so they are checked, never read past: the
// pe_resolver_* ABI reports PE_EINVAL (before any update is written), pe_place_greedy PE_EHIP.
struct CorruptList : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Window blob = n_shards consecutive shard blocks, each n_groups x (16-B header {int32 n,
// int32 flags, uint64 limit} + K x 48-B records {u64 key, i64 res[4], u64 labels}) -- exactly
// what the merge kernel writes.  Parses and merges the shards into cands[n_groups].
// With one shard and copy_blob = false the lists point INTO the blob, which must outlive them.
// Every header and record is validated (CorruptList): 0 <= n <= K, node id (key bits 0-23) <
// n_nodes, keys strictly ascending within a shard list.
void parse_window(const uint8_t* blob, int n_shards, int n_groups, int K, std::vector<GroupCands>& cands,
                  bool copy_blob = false, int64_t n_nodes = (int64_t)1 << 24);
// Key-only window blob (the engine's device format): per shard, per group a 16-B header + K u64
// keys.  Lists point into the blob when n_shards == 1.  Headers are validated (0 <= n <= K); the
// listed node ids are checked where the resolver reads their mirror state (Resolver::resolve).
void parse_window_keys(const uint8_t* blob, int n_shards, int n_groups, int K, std::vector<GroupCands>& cands);

// Pipelined walk windows (engine, one shard): the device writes each group's key list straight
// into pinned host memory and SIGNALS it -- keys, n and limit first, then header.flags = the
// window's generation (system-scope release).  The feed hands the groups to the resolver as they
// arrive, so resolving starts when the first group is done instead of when the slowest one is.
// Only the resolver thread parses (fills cands[w], then publishes parsed() with release); the
// seed helper reads groups below parsed() only.
// A rank's lists never arrived in a zero-copy exchange window (the engine reports PE_ERCCL)
struct ExchangeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
// A window of the RCCL transport did not arrive within PE_RCCL_TIMEOUT_S -- its collective is stuck
// (a peer lost mid-batch keeps the stream busy, so the feed's idle test never fires): the engine
// aborts the communicator and reports PE_ERCCL
struct CollectiveTimeout : ExchangeError {
  using ExchangeError::ExchangeError;
};

class WindowFeed {
 public:
  void reset(const uint8_t* blob, int n_groups, int K, uint32_t gen, std::vector<GroupCands>* cands);
  size_t parsed() const { return parsed_.load(std::memory_order_acquire); }
  size_t size() const { return n_; }
  // resolver thread: parse every group signalled so far (never blocks)
  void advance();
  // resolver thread: block until group w is parsed.  While spinning, idle(user) is called every
  // few thousand polls; false aborts (throws std::runtime_error).
  void wait(size_t w);
  bool (*idle)(void*) = nullptr;
  void* idle_user = nullptr;
  // > 0: wait() gives up after this many seconds blocked on one group, busy device or not, and
  // throws CollectiveTimeout (the RCCL transport; the other transports have bounds of their own).
  // on_timeout(timeout_user), when set, runs first, at the throw site: the engine starts the
  // communicator's abort there, before the unwinding waits for anything (advice r5)
  double timeout_s = 0;
  void (*on_timeout)(void*) = nullptr;
  void* timeout_user = nullptr;
  double spin_ms() const { return spin_ms_; }   // time spent blocked in wait() since reset
 private:
  bool signalled(size_t w) const;
  const uint8_t* blob_ = nullptr;
  size_t n_ = 0, gb_ = 0;
  uint32_t gen_ = 0;
  std::vector<GroupCands>* cands_ = nullptr;
  std::atomic<size_t> parsed_{0};
  double spin_ms_ = 0;
  int K_ = 0;
};

// Node id -> small index, open addressing (linear probing) sized to the live entries: the dirty
// set and a job's nodes hold hundreds of ids out of up to 2^24, so the table stays in L1/L2 where a
// direct-mapped array over all ids would miss in cache on every lookup.
class IdMap {
 public:
  int32_t find(int64_t id) const {
    if (n_ == 0) return -1;
    for (size_t h = hash(id);; h = (h + 1) & mask_) {
      if (keys_[h] == id) return vals_[h];
      if (keys_[h] < 0) return -1;
    }
  }
  // value of id, inserting `v` if absent
  int32_t insert(int64_t id, int32_t v) {
    if (2 * (n_ + 1) > keys_.size()) grow();
    for (size_t h = hash(id);; h = (h + 1) & mask_) {
      if (keys_[h] == id) return vals_[h];
      if (keys_[h] < 0) {
        keys_[h] = id;
        vals_[h] = v;
        ++n_;
        return v;
      }
    }
  }
  // forget every id (the caller lists them: O(entries), not O(table))
  template <class It>
  void clear(It b, It e) {
    if (4 * n_ < keys_.size() / 4 && keys_.size() > 1024) {   // far too big after a burst: shrink
      keys_.assign(1024, -1);
      vals_.assign(1024, -1);
      mask_ = 1023;
    } else {
      pos_.clear();
      for (; b != e; ++b)   // tombstones first, so the remaining ids' probe chains stay intact
        for (size_t h = hash(*b);; h = (h + 1) & mask_)
          if (keys_[h] == *b) {
            keys_[h] = -2;
            pos_.push_back(h);
            break;
          }
      for (size_t h : pos_) keys_[h] = -1;
    }
    n_ = 0;
  }

 private:
  size_t hash(int64_t id) const { return (size_t)(((uint64_t)id * 0x9E3779B97F4A7C15ull) >> 40) & mask_; }
  void grow() {
    std::vector<int64_t> ok = std::move(keys_);
    std::vector<int32_t> ov = std::move(vals_);
    const size_t cap = std::max<size_t>(1024, ok.size() * 2);
    keys_.assign(cap, -1);
    vals_.assign(cap, -1);
    mask_ = cap - 1;
    n_ = 0;
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i] >= 0) insert(ok[i], ov[i]);
  }
  std::vector<int64_t> keys_;
  std::vector<int32_t> vals_;
  std::vector<size_t> pos_;
  size_t mask_ = 0, n_ = 0;
};

// A vector whose resize() leaves new elements uninitialised: the key scans write every slot they
// report, and re-growing the slot list to the dirty set's size zero-filled ~1 KB per group.
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
using IdxVec = std::vector<int32_t, NoInitAlloc<int32_t>>;

// Nodes modified since the window's snapshot, as flat struct-of-arrays so the per-group re-score
// is one branch-free (vectorisable) loop; gid -> slot is a small hash map.  The columns share one
// allocation, one count and one capacity: an append is one capacity test and seven stores (seven
// vector push_backs were seven tests and size updates per placement).
class DirtySet {
 public:
  DirtySet() = default;
  DirtySet(const DirtySet&) = delete;
  DirtySet& operator=(const DirtySet&) = delete;
  DirtySet(DirtySet&& o) noexcept { swap(o); }
  DirtySet& operator=(DirtySet&& o) noexcept {
    swap(o);
    return *this;
  }
  ~DirtySet() { ::operator delete(buf_, std::align_val_t(64)); }
  void swap(DirtySet& o) noexcept;
  int32_t find(int64_t gid) const { return slot_.find(gid); }
  // membership only: one bit per node id (128 KiB per 1M ids, cache-resident), the candidate
  // lists' skip test
  bool contains(int64_t gid) const {
    const size_t w = (size_t)gid >> 6;
    return w < bits_.size() && (bits_[w] >> (gid & 63) & 1);
  }
  int32_t upsert(int64_t gid, const NodeState& st);
  void set(int32_t i, const NodeState& st);
  NodeState get(int32_t i) const;
  size_t size() const { return n_; }
  void clear();
  // keys of every dirty node for request (q, need) -> out (NO_KEY where it does not fit).  Keys
  // >= `limit` may be reported as NO_KEY: a node whose node-only key K(n) (below) rules out a key
  // < limit is not scored (K(n) >= (s(q) << 24) for a fit, key >= K(n) - ((s(q) + 2) << 24)).
  // `idx` receives the slots that were scored (the rest are NO_KEY in out).
  void keys(const int64_t q[RD], uint32_t need, uint64_t limit, std::vector<uint64_t>& out, IdxVec& idx) const;
  // the fitting slots' keys for (q, need): their slots -> idx, their keys -> out at those slots
  // (out elsewhere is left as it was; the K(n) range test above leaves out nodes that cannot have a
  // key < limit); returns the smallest.  AVX-512 where the CPU has it (8 nodes per step), else
  // keys() + a scalar pass.
  uint64_t keys_all(const int64_t q[RD], uint32_t need, uint64_t limit, std::vector<uint64_t>& out,
                    IdxVec& idx) const;
  uint64_t key_at(int32_t i, const int64_t q[RD], uint32_t need) const;
  // the columns, size() entries each
  int64_t *gid = nullptr, *r0 = nullptr, *r1 = nullptr, *r2 = nullptr, *r3 = nullptr;
  uint32_t* lab = nullptr;
  uint64_t* kn = nullptr;   // K(n) = (S(n) << 24) | gid, or ~0 (saturating / negative: always scored)

 private:
  void grow();
  size_t n_ = 0, cap_ = 0;
  void* buf_ = nullptr;
  IdMap slot_;
  std::vector<uint64_t> bits_;
};

// CPUs that share cpu's L3 (Linux sysfs); false if unknown.
bool l3_cpus(int cpu, cpu_set_t* set);
// A CPU of the (k mod n)-th of the n L3 domains that `allowed` touches (domains ordered by their
// first allowed CPU); -1 if unknown.
int l3_pick(const cpu_set_t& allowed, int k);

// Per window group: the smallest keys over the window's SEEDS (nodes changed since the lists'
// snapshot, their current state known at the window start), below the group's limit.
struct SeedTop {
  static constexpr int kTop = 32;
  int n = 0;                 // keys in key[], ascending
  bool truncated = false;    // more seed keys lie below the limit than kTop
  size_t head = 0;           // the group list's first entry that is not a seed
  uint64_t key[kTop];
};

// Scores the seeds of a pipelined window for every group of the window, in group order, on a
// helper thread that runs ahead of the resolver: the seeds stay untouched until the resolver
// changes them, so a seed's key computed from its window-start state is current until then
// (the resolver skips the entries of seeds it has changed and scores those itself).  The
// resolver never waits: a group whose top is not ready yet is scored on the resolver's thread.
class SeedScorer {
 public:
  SeedScorer() = default;
  ~SeedScorer();
  SeedScorer(const SeedScorer&) = delete;
  SeedScorer& operator=(const SeedScorer&) = delete;
  // Main thread: start scoring a window (seeds, cands and the request arrays must stay unchanged
  // until stop()).
  void start(const DirtySet* seeds, const std::vector<int32_t>* groups, const std::vector<GroupCands>* cands,
             const int64_t* scan_req, const uint32_t* need, const WindowFeed* feed = nullptr,
             const NodeState* mirror = nullptr, int64_t mirror_n = 0);
  bool ready(size_t wi) const { return slots_[wi].gen.load(std::memory_order_acquire) == gen_; }
  const SeedTop& top(size_t wi) const { return slots_[wi].top; }
  // the resolver is at group wi: the helper skips what it would finish too late
  void at(size_t wi) { main_wi_.store(wi, std::memory_order_relaxed); }
  void stop();   // cancel the window and wait until the helper is idle
  // CPUs of the helper thread (applied now, or when the thread starts); without a call the helper
  // takes the L3 of the CPU that starts it
  void pin(const cpu_set_t& set);
  // one group's top (any thread; out / idx are the caller's scratch)
  static void compute(const DirtySet& seeds, const GroupCands& gc, const int64_t q[RD], uint32_t need, SeedTop& top,
                      std::vector<uint64_t>& out, IdxVec& idx);

 private:
  void loop();
  std::unique_ptr<std::thread> th_;
  bool have_pin_ = false;
  cpu_set_t pin_set_;
  std::atomic<int> state_{0};            // 0 idle, 1 window posted, 2 cancel, 3 exit
  // One slot per window group, its own cache lines: the ready generation sits on the same line as
  // the top's head and first keys, so the resolver's check-and-read of a group is one line handed
  // over from the helper (flags packed 16 to a line ping-ponged between the two cores).
  struct alignas(64) TopSlot {
    std::atomic<uint32_t> gen{0};   // == gen_: top is final for this window
    SeedTop top;
  };
  std::unique_ptr<TopSlot[]> slots_;
  size_t cap_ = 0;
  uint32_t gen_ = 0;                                  // window generation (written before posting)
  std::atomic<size_t> main_wi_{0};
  // long idle: the helper sleeps on park_cv_ (parked_ set) instead of spinning a core between calls
  static constexpr int kParkAfter = 1 << 16;
  std::atomic<bool> parked_{false};
  std::mutex park_mu_;
  std::condition_variable park_cv_;
  const DirtySet* seeds_ = nullptr;
  const std::vector<int32_t>* groups_ = nullptr;
  const std::vector<GroupCands>* cands_ = nullptr;
  const WindowFeed* feed_ = nullptr;   // groups at or above feed_->parsed() are not there yet
  // host mirror: the helper reads the states of each group's first non-seed list entries, so the
  // resolver finds those lines in a cache of its CCD (a cross-core hit) instead of in DRAM
  const NodeState* mirror_ = nullptr;
  int64_t mirror_n_ = 0;
#ifndef PE_WARM_STATES
#define PE_WARM_STATES 4
#endif
  static constexpr int kWarmStates = PE_WARM_STATES;
  volatile int64_t warm_sink_ = 0;   // (keeps the reads)
  const int64_t* req_ = nullptr;
  const uint32_t* need_ = nullptr;
  std::vector<uint64_t> out_;
  IdxVec idx_;
};

class Resolver {
 public:
  Resolver(int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority, const int32_t* group_count,
           const int64_t* group_req, const uint32_t* group_need);
  // A new batch on the same object: every per-batch state cleared, allocations (and the seed helper
  // thread) kept -- a fresh resolver per batch page-faulted its ~1 MB of arrays and started a thread.
  void reset(int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority, const int32_t* group_count,
             const int64_t* group_req, const uint32_t* group_need);
  void pin_helper(const cpu_set_t& set) { scorer_.pin(set); }

  bool done() const { return oi_ >= (int64_t)order_.size(); }
  // Groups (global ids, count > 0) of the next window, starting at the cursor (or at `from`);
  // *end receives the cursor just past the window (where it stands if the window is consumed).
  void next_window(int max_groups, int64_t max_pods, std::vector<int32_t>& groups);
  void next_window_from(const Cursor& from, int max_groups, int64_t max_pods, std::vector<int32_t>& groups,
                        Cursor* end) const;
  Cursor cursor() const { return Cursor{oi_, g_, p_}; }
  // states of key-only candidates (must stay valid and current while resolving such lists)
  void set_mirror(const Mirror& m) { mirror_ = m; }
  // Resolve with candidates for exactly the groups returned by next_window (same order).
  // Appends the residual updates to flush; returns true if the whole window was consumed.
  // seed (pipelined form): nodes changed since the snapshot the candidates were scanned on, with
  // their current state -- they start dirty, so the lists' clean entries stay exact; only nodes
  // changed in THIS window are returned as updates.
  // feed (pipelined walk windows): cands fill in as the device signals each group (see WindowFeed).
  bool resolve(const std::vector<int32_t>& groups, const std::vector<GroupCands>& cands,
               std::vector<Update>& updates, const std::vector<Update>* seed = nullptr, WindowFeed* feed = nullptr);

  // The request a group's candidate lists are scanned for: the pod request, or count x request
  // for an island group (need bit 31: its pods are placed as one unit on one node).
  const int64_t* scan_req(int64_t g) const { return &qeff_[(size_t)g * RD]; }
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
  std::vector<int64_t> qeff_;    // [G][4] scan request (island groups: count x request)
  std::vector<uint8_t> unit_;    // [G] 1 = island group, 2 = island group whose summed request overflows
  Mirror mirror_;
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
  IdxVec dki_;   // dirty slots with a key for the current group (argmin runs over these)
  std::vector<size_t> head_;   // per window group: its list's first entry not known to be dirty
  // pipelined windows: the seeds live here (not in dirty_, which then holds the window's own
  // changes only); their per-group keys come from the scorer's helper thread
  DirtySet seeds_;
  // the previous resolve's changes (its dirty set, kept instead of cleared): the next pipelined
  // window's seeds are exactly those updates, so the set is taken over as is (no re-insertion)
  DirtySet prev_;
  bool prev_ok_ = false;
  // dirty_ OR seeds_ during a resolve, one bitmap: the list-skip test (every list entry the resolver
  // looks at) is one bit instead of a bit in each set; cleared entry by entry when the resolve ends
  std::vector<uint64_t> any_;
  void any_set(int64_t g) {
    const size_t w = (size_t)g >> 6;
    if (w >= any_.size()) any_.resize(std::max(w + 1, 2 * any_.size()), 0);
    any_[w] |= 1ull << (g & 63);
  }
  bool any_has(int64_t g) const {
    const size_t w = (size_t)g >> 6;
    return w < any_.size() && (any_[w] >> (g & 63) & 1);
  }
  std::vector<uint64_t> sk_out_;
  IdxVec sk_idx_;
  std::vector<uint64_t> sfull_;      // a group's every seed key below the limit (truncated top)
  SeedScorer scorer_;                // declared after what its thread reads: stopped first
  // A failed job's nodes are restored from their CURRENT states, looked up only then (rollbacks are
  // rare; no per-placement bookkeeping): the window's dirty set, else the mirror (which follows every
  // resolved window), else -- record-form lists without a mirror (pe_resolver_* ABI) -- the last state
  // this resolver gave the node in an earlier window (changed_).
  NodeState current_state(int64_t gid) const;
  // (cleared when a job finishes: only the in-flight job can roll back what they record)
  IdMap changed_slot_;
  std::vector<NodeState> changed_;
  std::vector<int64_t> changed_gid_;
  int64_t jobs_placed_ = 0, jobs_failed_ = 0, pods_placed_ = 0, rescans_ = 0;
};

}  // namespace pe
