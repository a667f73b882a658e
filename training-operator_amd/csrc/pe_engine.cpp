// libplacement: context, device-resident inventory, C ABI entry points (include/placement.h).
//
// One context = one process = one GPU = one contiguous shard of the node inventory.  The
// inventory lives on the device as int64 struct-of-arrays res[4][stride] (+ labels, islands),
// so every kernel streams each dimension coalesced.  Sharded contexts exchange per-group
// candidate lists with one RCCL all-gather per scan window (or a host callback in tests).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <deque>
#include <condition_variable>
#include <atomic>
#include <chrono>
#include <exception>
#include <functional>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "pe_hostx.h"
#include "pe_kernels.h"
#include "pe_merge.h"
#include "pe_resolver.h"
#include "placement.h"

namespace {

using pe::ReqRec;

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  // flags: hipExtMallocWithFlags flags (hipDeviceMallocContiguous falls back to a plain hipMalloc
  // when the driver cannot provide it)
  hipError_t ensure(size_t count, unsigned flags = 0) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    hipError_t e = hipErrorOutOfMemory;
    if (flags) {
      e = hipExtMallocWithFlags((void**)&p, bytes, flags);
      if (e != hipSuccess) (void)hipGetLastError();
    }
    if (e != hipSuccess) e = hipMalloc((void**)&p, bytes);
    if (e == hipSuccess) n = count;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// Pinned host buffer.  Coherent (fine-grained) ones are also read and written by kernels directly
// (dev = the device-side address): per-window inputs and the candidate blob skip the copy engines.
template <class T>
struct HostBuf {
  T* p = nullptr;
  T* dev = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t count, unsigned flags = hipHostMallocDefault) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), flags);
    // zeroed: several of these buffers carry completion flags (signalled groups, the aggregation
    // flag) that a recycled allocation could otherwise hold from an earlier engine's generations
    if (e == hipSuccess) std::memset((void*)p, 0, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&dev, p, 0);
    if (e == hipSuccess) n = count;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    n = 0;
  }
};
constexpr unsigned kZeroCopy = hipHostMallocCoherent | hipHostMallocMapped;

// One helper thread that runs a posted task while the caller does other work (pipelined greedy:
// the next window's launches are issued while the host resolves the current one).  Spin handoff:
// the wake-up of a sleeping thread would cost about as much as the launches it hides.
class SpinWorker {
 public:
  explicit SpinWorker(int device) : th_([this, device] {
    (void)hipSetDevice(device);   // the current device is per thread
    loop();
  }) {}
  ~SpinWorker() {
    while (state_.load(std::memory_order_acquire) == 1) _mm_pause();   // a posted task finishes first
    state_.store(3, std::memory_order_release);
    th_.join();
  }
  void pin(const cpu_set_t& set) { (void)pthread_setaffinity_np(th_.native_handle(), sizeof(set), &set); }
  void post(std::function<void()> f) {
    task_ = std::move(f);
    err_ = nullptr;
    posted_ = true;
    state_.store(1, std::memory_order_release);
  }
  bool busy() const { return state_.load(std::memory_order_acquire) == 1; }   // a posted task not done yet
  bool failed() const { return state_.load(std::memory_order_acquire) == 2 && err_ != nullptr; }
  void wait() {   // rethrows what the task threw; returns at once when nothing is posted
    if (!posted_) return;
    posted_ = false;
    for (int spin = 0; state_.load(std::memory_order_acquire) != 2; ++spin)
      if (spin < 4096) _mm_pause();
      else std::this_thread::yield();   // the helper is not running (oversubscribed host)
    state_.store(0, std::memory_order_relaxed);
    if (err_) std::rethrow_exception(err_);
  }

 private:
  void loop() {
    int idle = 0;
    for (;;) {
      const int st = state_.load(std::memory_order_acquire);
      if (st == 3) return;
      if (st != 1) {
        if (++idle < 4096) _mm_pause();
        else std::this_thread::yield();   // long idle (host resolving): let others run
        continue;
      }
      idle = 0;
      try {
        task_();
      } catch (...) {
        err_ = std::current_exception();
      }
      state_.store(2, std::memory_order_release);
    }
  }
  std::atomic<int> state_{0};
  bool posted_ = false;   // (the posting thread's own view: a task posted and not waited for yet)
  std::function<void()> task_;
  std::exception_ptr err_;
  std::thread th_;   // last: starts after the members above exist
};

// A SpinWorker with a queue: post() does not wait for the previous task (up to kCap in flight), the
// tasks run in order on the thread, wait() waits for all of them.  After a task threw, the rest are
// skipped and wait() rethrows.  (The host-merged zero-copy exchange: the main thread posts each
// window's merge as it launches the window, without waiting for the previous merge to finish.)
class SpinQueue {
 public:
  static constexpr unsigned kCap = 8;
  explicit SpinQueue(int device) : th_([this, device] {
    (void)hipSetDevice(device);
    loop();
  }) {}
  ~SpinQueue() {
    while (busy()) _mm_pause();
    stop_.store(true, std::memory_order_release);
    th_.join();
  }
  void pin(const cpu_set_t& set) { (void)pthread_setaffinity_np(th_.native_handle(), sizeof(set), &set); }
  void post(std::function<void()> f) {
    const unsigned t = tail_.load(std::memory_order_relaxed);
    while (t - head_.load(std::memory_order_acquire) >= kCap) _mm_pause();   // full: the oldest first
    q_[t % kCap] = std::move(f);
    tail_.store(t + 1, std::memory_order_release);
  }
  bool busy() const { return head_.load(std::memory_order_acquire) != tail_.load(std::memory_order_acquire); }
  bool failed() const { return failed_.load(std::memory_order_acquire); }
  void wait() {   // every posted task done; rethrows the first error (once)
    for (int spin = 0; busy(); ++spin)
      if (spin < 4096) _mm_pause();
      else std::this_thread::yield();
    if (failed_.load(std::memory_order_acquire)) {
      failed_.store(false, std::memory_order_relaxed);
      std::exception_ptr e = err_;
      err_ = nullptr;
      if (e) std::rethrow_exception(e);
    }
  }

 private:
  void loop() {
    int idle = 0;
    for (;;) {
      const unsigned h = head_.load(std::memory_order_relaxed);
      if (h == tail_.load(std::memory_order_acquire)) {
        if (stop_.load(std::memory_order_acquire)) return;
        if (++idle < 4096) _mm_pause();
        else std::this_thread::yield();
        continue;
      }
      idle = 0;
      if (!failed_.load(std::memory_order_relaxed)) {
        try {
          q_[h % kCap]();
        } catch (...) {
          err_ = std::current_exception();
          failed_.store(true, std::memory_order_release);
        }
      }
      q_[h % kCap] = nullptr;
      head_.store(h + 1, std::memory_order_release);
    }
  }
  std::function<void()> q_[kCap];
  std::atomic<unsigned> head_{0}, tail_{0};
  std::atomic<bool> failed_{false}, stop_{false};
  std::exception_ptr err_;
  std::thread th_;   // last: starts after the members above exist
};


struct PeError {
  int code;
  std::string msg;
};

[[noreturn]] void raise(int code, const std::string& msg) { throw PeError{code, msg}; }

void hipchk(hipError_t e, const char* what) {
  if (e != hipSuccess) raise(PE_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

void ncclchk(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) raise(PE_ERCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

// Bound of the communicator set-up: PE_RCCL_INIT_TIMEOUT_S seconds (default 120).
double rccl_init_timeout_ms() {
  const char* e = std::getenv("PE_RCCL_INIT_TIMEOUT_S");
  const double s = e ? std::atof(e) : 120.0;
  return (s > 0 ? s : 120.0) * 1e3;
}

// ncclCommInitRank with a time bound: a rank whose peers never arrive (a wrong comm_id, a dead
// peer) gets PE_ERCCL instead of hanging in the bootstrap, which has no timeout of its own.  The
// blocking call runs on a helper thread; past the bound the call is abandoned: the thread stays
// behind (detached) and destroys the communicator itself if the peers ever do arrive.  (A
// non-blocking communicator, ncclConfig_t.blocking = 0, still blocked in the bootstrap on this
// RCCL, and ncclCommAbort of a set-up in progress waits for it: profiles/r10_rccl_init.txt.)
ncclComm_t comm_init_bounded(int device, int world, const ncclUniqueId& id, int rank, double timeout_ms) {
  struct State {
    std::mutex m;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclResult_t r = ncclSuccess;
    ncclComm_t comm = nullptr;
  };
  auto st = std::make_shared<State>();
  std::thread([st, device, world, id, rank] {
    (void)hipSetDevice(device);   // the current device is per thread
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, world, id, rank);
    std::lock_guard<std::mutex> lk(st->m);
    if (st->abandoned) {
      if (r == ncclSuccess && c) (void)ncclCommDestroy(c);
      return;
    }
    st->r = r;
    st->comm = c;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->m);
  if (!st->cv.wait_for(lk, std::chrono::duration<double, std::milli>(timeout_ms), [&] { return st->done; })) {
    st->abandoned = true;
    raise(PE_ERCCL, "ncclCommInitRank: the " + std::to_string(world) + " ranks did not meet within " +
                        std::to_string((int)(timeout_ms / 1e3)) + " s (PE_RCCL_INIT_TIMEOUT_S)");
  }
  ncclchk(st->r, "ncclCommInitRank");
  return st->comm;
}

// Bound of one RCCL window of the greedy: PE_RCCL_TIMEOUT_S seconds (default 60) blocked on a window
// whose all-gather has not completed (a peer lost mid-batch) -- then the communicator is aborted and
// the call returns PE_ERCCL.
double rccl_timeout_s() {
  const char* e = std::getenv("PE_RCCL_TIMEOUT_S");
  const double s = e ? std::atof(e) : 60.0;
  return s > 0 ? s : 60.0;
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// pe_config.fit_path_mask bits
constexpr int kMaxMergers = 7;   // zero-copy exchange: merge helper threads per rank (at most)
constexpr int PATH_I64 = 1, PATH_I32 = 2, PATH_CODED = 4, PATH_NO_THERM = 8, PATH_PLANES = 16, PATH_PLANES_BLOCKS = 32,
              PATH_LDS = 64;
constexpr int PATHS_ALL = PATH_I64 | PATH_I32 | PATH_CODED | PATH_PLANES | PATH_LDS;

// One segment of the packed aggregation batch (pe_kernels.h AggSegHdr).
struct AggSeg {
  int64_t j0;
  int32_t nj, ng, nc;
  int64_t bytes;
  bool narrow;            // the request section narrowed (pe_kernels.h agg_seg_layout), shifts in sh
  uint8_t sh[pe::AGG_MAX_KEYS];
};

}  // namespace

struct pe_ctx {
  std::mutex mu;
  int device = 0;
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  // a greedy window's collective timed out: the communicator was handed to comm_abort (ncclCommAbort
  // on its own thread -- it returns once the device work it aborts has drained) and every later
  // sharded call fails with PE_ERCCL; the caller rebuilds the context (e.g. on the host exchange)
  bool comm_aborted = false;
  std::thread comm_abort;
  std::unique_ptr<pe::Resolver> resolver;   // the greedy's host resolver, reset per batch
  pe_allgather_fn exchange = nullptr;
  void* exchange_user = nullptr;
  void* zc_hx = nullptr;   // the shared-memory exchange whose zero-copy use the ranks agreed on (zc_ok)
  bool zc_ok = false;
  int topk = 256, window_groups = 112;
  bool pipeline = true;   // greedy: scan window w+1 while the host resolves window w (greedy_flags bit0 = off)
  int64_t window_pods = 1024;
  int64_t max_nodes = 0;
  std::string gpu_name, err;
  hipStream_t stream = nullptr;
  // inventory shard
  int64_t n_total = 0, begin = 0, end = 0, Ns = 0, stride = 0;
  bool loaded = false;
  // host mirror of the GLOBAL inventory (node states by id, and the reset copy): the greedy
  // windows ship candidate keys only and the resolver reads node states here
  std::vector<pe::NodeState, pe::HugeAlloc<pe::NodeState>> m_nodes, m_nodes0;   // (2 MiB pages: random reads)
  DevBuf<int64_t> res0, res;
  DevBuf<uint32_t> labels;
  DevBuf<int32_t> island;
  DevBuf<pe::NodeUpd> n_upd;   // pe_update_nodes staging
  // fit mask
  int64_t fit_J = 0, fit_Jp = 0, Wn = 0, Wt = 0;
  bool fit_uploaded = false;
  DevBuf<ReqRec> fit_jobs;
  DevBuf<pe::ReqRec32> fit_jobs32;
  DevBuf<int32_t> res32;
  bool fit32 = false;      // batch is exactly representable in 32 bits (see ReqRec32)
  int fit_shift[pe::D] = {0, 0, 0, 0};
  int fit_path = 0;        // 0 int64 compare, 1 int32 compare, 2 dictionary-coded, 3 bit planes, 4 LDS digit planes
  // LDS digit-plane path (pe_kernels.h LdsSpec): spec, node-block geometry, codes, ranks
  pe::LdsSpec lds{};
  int lds_W = 4;                          // u32 words per lane per plane: block = 2048 W nodes
  int lds_shape[4] = {0, 0, 0, 0};        // fields with 4 / 3 / 2 / 1 digit levels (kernel template)
  int64_t lds_nblk = 0, lds_R = 1, lds_Tpad = 0, lds_npad = 0, lds_pitch = 0;   // pitch in u64 words
  DevBuf<pe::LdsSpec> lds_spec_d;
  DevBuf<int64_t> lds_vals;
  DevBuf<uint16_t> lds_codes;
  DevBuf<uint32_t> lds_ranks, lds_aux, lds_slots;   // lds_slots: the fit kernel's per-job u32 count slots
  DevBuf<uint32_t> lds_rows;                         // the job (mask row) of each count slot, ~0 = none
  int num_cu = 256;
  int fit_path_mask = PATHS_ALL;   // allowed paths (pe_config.fit_path_mask)
  pe::PlaneSpec plane{};
  int64_t pl_nblk = 0;                   // planes path: 8192-node blocks
  bool pl_rows = true;                   // planes path: row-major sweep kernel (else block-major streams)
  int64_t pl_R = 1;                      // row-major kernel: job phases of the uploaded batch
  int64_t pl_pitch = 0;                  // row-major mask pitch in 8192-node blocks (>= pl_nblk)
  // A batch with more than PL_MAX distinct (dimension, value) pairs is split into plane sets of at
  // most PL_MAX pairs each (row-major layout only); each set is encoded and swept on its own by
  // the indexed-row kernel, its jobs' codes carrying their mask rows.
  struct PlaneSet {
    pe::PlaneSpec spec;
    int64_t J, R, Jr, off;   // jobs, phases, phase stride, first code / count slot
  };
  std::vector<PlaneSet> pl_sets;        // empty: one set (ctx->plane, the rows kernel)
  DevBuf<pe::PlaneSpec> pl_specs_d;     // multi-set: the sets' specs and {off, J, Jr} on the device
  DevBuf<int64_t> pl_meta_d;
  std::vector<int64_t> pl_cnt_row;      // multi-set: count slot -> job row (-1: padding)
  int64_t pl_counts_n = 0;              // count slots of the planes path
  DevBuf<uint32_t> planes;
  DevBuf<uint64_t> plane_jobs;
  pe::CodeSpec code{};
  int64_t code_Jp = 0, node_stride = 0;
  DevBuf<int64_t> code_vals;
  DevBuf<uint32_t> code_needs, code_jobs, code_x;
  DevBuf<uint64_t> mask;
  DevBuf<unsigned long long> counts;
  HostBuf<unsigned long long> h_counts;
  // aggregation: segmented batch and outputs in pinned, device-mapped host memory (pe_kernels.h
  // AggSegHdr); the device-resident arrays below only serve the PE_AGG_DEVICE=1 A/B path
  HostBuf<uint8_t> a_stage, a_outh;
  DevBuf<uint8_t> a_dstage;              // large batches: the packed batch DMA'd to the device chunk by chunk
  hipStream_t a_h2d = nullptr;           // ... on this copy stream (the kernels wait on its events)
  std::vector<hipEvent_t> a_ev_h2d;
  HostBuf<int64_t> a_segoff;
  HostBuf<uint32_t> a_flag;
  std::vector<hipEvent_t> a_ev;   // large batches: one per chunk (its outputs are copied out when it is done)
  DevBuf<uint32_t> a_ctr;   // latency launches: blocks done (the last one stores the flag)
  uint32_t agg_gen = 0;
  std::vector<std::vector<AggSeg>> agg_segs;   // per planning range, reused across calls (no allocation per call)
  std::vector<AggSeg> agg_all;                 // all segments in order
  DevBuf<int32_t> a_jgo, a_mm, a_rep, a_gco, a_mem;
  DevBuf<int64_t> a_req, a_out;
  DevBuf<uint8_t> a_fl, a_pres, a_ovf;
  // greedy
  DevBuf<ReqRec> g_groups;
  DevBuf<uint64_t> g_cand, g_bound;
  DevBuf<int32_t> g_cnt;
  DevBuf<uint8_t> g_out, g_gath;
  DevBuf<int64_t> g_upd;
  DevBuf<uint64_t> g_kn;   // scan: node-only score terms K(n) (prep_nodes), refreshed by apply
  DevBuf<uint32_t> g_lo;   // scan: lo20(r1) / lo24(r3), [2][stride]
  HostBuf<ReqRec> h_groups, h_groups2;   // h_groups2: the window requests of blob buffer 1 (signalled walk)
  HostBuf<ReqRec> h_groupsx[2];           // blob buffers 2, 3 (pipeline depth 2, 3)
  HostBuf<uint8_t> h_outx[2];             // blob buffers 2, 3
  HostBuf<int64_t> h_updx[2];             // update staging slots 1, 2 (pipeline depth 2, 3)
  uint32_t walk_gen = 0;                  // generation of the last signalled walk window (never 0)
  int pin_cpu = -2;                       // greedy thread pinning at world > 1: a CPU of this rank's L3 (-2: not chosen yet)
  HostBuf<uint8_t> h_out, h_out2, h_own;   // h_out2: the pipelined loop's second blob buffer (h_outx: 3rd, 4th)
  HostBuf<uint8_t> h_merged;                // host-exchange windows: the device-merged lists
  HostBuf<uint8_t> h_xg[4];                 // pipelined host exchange: the gathered lists of blob buffer b
  std::vector<const uint64_t*> x_lists;     // host merge of the gathered lists (exchange thread scratch)
  std::vector<int32_t> x_ns, x_hd;
  HostBuf<int64_t> h_upd;
  // greedy sorted walk (pe_kernels.h WalkIndex; the default window path, greedy_flags bit1 = full scan)
  bool walk = true;
  int64_t resort_nodes = 20480;  // re-sort once this many applied updates joined the overlay
  int64_t w_est = 0;             // updates applied since the last sort (>= overlay size)
  // two index sets: the walks read ws[w_cur]; the next one is rebuilt on the side stream w_s2
  // (lowest priority) while the walks go on (walk_resort_async), then taken over (walk_switch)
  struct WalkSet {
    DevBuf<uint64_t> sk, rmin;
    DevBuf<int64_t> sr, rmax;
    DevBuf<uint32_t> sl, pos, ror, inovl, ovidx, ovlab;
    DevBuf<int64_t> ovres;
    DevBuf<uint64_t> ovkn;
    DevBuf<int32_t> ovl, ovln;
    void release() {
      sk.release(); rmin.release(); sr.release(); rmax.release(); sl.release(); pos.release(); ror.release();
      inovl.release(); ovidx.release(); ovlab.release(); ovres.release(); ovkn.release(); ovl.release(); ovln.release();
    }
  } ws[2];
  int w_cur = 0;
  bool w_pending = false;        // ws[1 - w_cur] is being rebuilt on w_s2
  int64_t w_pend_est = 0;        // updates applied since that rebuild's snapshot
  int64_t w_pend_windows = 0;    // windows launched while that rebuild was pending
  hipStream_t w_s2 = nullptr;
  hipEvent_t w_ev_snap = nullptr, w_ev_done = nullptr;
  DevBuf<uint64_t> w_kin;
  DevBuf<uint32_t> w_slow;       // saturating nodes of the side-stream rebuild (walk_switch adds them)
  DevBuf<uint8_t> w_temp;
  DevBuf<uint32_t> w_flush;   // PE_WALK_FLUSH: 512 MiB rewritten before each walk (cold-cache diagnostics)
  DevBuf<unsigned long long> w_stat;   // walk counters of the current pe_place_greedy (rounds, overlay)
  DevBuf<uint64_t> g_xstatus;          // zero-copy exchange: the window's wait status (launch_xwait)
  pe_stats stats{};

  ~pe_ctx() {
    (void)hipSetDevice(device);
    if (comm_abort.joinable()) comm_abort.join();
    if (stream) (void)hipStreamSynchronize(stream);
    res0.release(); res.release(); labels.release(); island.release(); n_upd.release();
    fit_jobs.release(); fit_jobs32.release(); res32.release(); mask.release();
    code_vals.release(); code_needs.release(); code_jobs.release(); code_x.release(); counts.release(); h_counts.release();
    planes.release(); plane_jobs.release();
    lds_spec_d.release(); lds_vals.release(); lds_codes.release(); lds_ranks.release(); lds_aux.release(); lds_slots.release(); lds_rows.release();
    a_stage.release(); a_outh.release(); a_segoff.release(); a_flag.release(); a_ctr.release();
    for (hipEvent_t e : a_ev) (void)hipEventDestroy(e);
    if (a_h2d) (void)hipStreamSynchronize(a_h2d);
    for (hipEvent_t e : a_ev_h2d) (void)hipEventDestroy(e);
    if (a_h2d) (void)hipStreamDestroy(a_h2d);
    a_dstage.release();
    a_jgo.release(); a_mm.release(); a_rep.release(); a_gco.release(); a_mem.release();
    a_req.release(); a_out.release(); a_fl.release(); a_pres.release(); a_ovf.release();
    g_groups.release(); g_cand.release(); g_bound.release(); g_cnt.release(); g_out.release(); g_gath.release();
    g_upd.release(); g_kn.release(); g_lo.release(); h_groups.release(); h_groups2.release(); h_out.release(); h_out2.release(); h_own.release(); h_merged.release(); h_upd.release();
    for (auto& x : h_xg) x.release();
    for (int i = 0; i < 2; ++i) {
      h_groupsx[i].release();
      h_outx[i].release();
      h_updx[i].release();
    }
    if (w_s2) (void)hipStreamSynchronize(w_s2);
    for (auto& x : ws) x.release();
    w_kin.release(); w_slow.release(); w_temp.release(); w_stat.release(); w_flush.release(); g_xstatus.release();
    if (w_ev_snap) (void)hipEventDestroy(w_ev_snap);
    if (w_ev_done) (void)hipEventDestroy(w_ev_done);
    if (w_s2) (void)hipStreamDestroy(w_s2);
    if (comm) (void)ncclCommDestroy(comm);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

// A collective timed out (pe::CollectiveTimeout): abort the communicator without blocking the caller.
// ncclCommAbort raises the communicator's abort flag, which the stuck collective kernel polls, and then
// frees its resources (the frees wait for the device work in flight); on its own thread, so the call
// that timed out returns PE_ERCCL within the bound; pe_destroy joins it.
void rccl_abort(pe_ctx* ctx) {
  if (!ctx->comm) return;
  ncclComm_t c = ctx->comm;
  ctx->comm = nullptr;
  ctx->comm_aborted = true;
  const int dev = ctx->device;
  ctx->comm_abort = std::thread([c, dev] {
    (void)hipSetDevice(dev);
    (void)ncclCommAbort(c);
  });
}

// Every ABI entry runs its body through here: lock, select device, map exceptions to codes.
template <class F>
int guarded(pe_ctx* ctx, F&& body) {
  if (!ctx) return PE_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->err.clear();
  try {
    hipchk(hipSetDevice(ctx->device), "hipSetDevice");
    return body();
  } catch (const PeError& e) {
    ctx->err = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    ctx->err = "host allocation failed";
    return PE_ENOMEM;
  } catch (const pe::CollectiveTimeout& e) {   // an RCCL window's all-gather never completed
    ctx->err = e.what();
    rccl_abort(ctx);
    return PE_ERCCL;
  } catch (const pe::ExchangeError& e) {   // a zero-copy window's peer lists never arrived
    ctx->err = e.what();
    return PE_ERCCL;
  } catch (const std::runtime_error& e) {   // pe::WindowFeed: a walk group the device never signalled
    ctx->err = e.what();
    return PE_EHIP;
  } catch (...) {
    ctx->err = "unexpected C++ exception";
    return PE_EINVAL;
  }
}

void need_ptr(const void* p, const char* name) {
  if (!p) raise(PE_EINVAL, std::string(name) + " is NULL");
}

// Persistent helpers for the batch planning (pe_jobs_upload is on the batch's path; creating and
// joining a thread per task cost tens of us each).  run(n, f): f(0) on the caller, f(1 .. n-1) on
// up to 7 pool threads, returns when all are done, rethrows the first exception.  The threads
// sleep on a condition variable between calls; the pool lives for the process.
// PE_NO_POOL=1: a thread per task instead (A/B).
class PlanPool {
 public:
  static constexpr int kMax = 16;
  static PlanPool& get() {
    static PlanPool* p = new PlanPool();   // never destroyed: its threads may still wait at exit
    return *p;
  }
  void run(int n, const std::function<void(int)>& f) {
    n = std::max(1, std::min(n, kMax));
    std::vector<std::exception_ptr> err((size_t)n);
    if (n > 1 && std::getenv("PE_NO_POOL")) {
      std::vector<std::thread> th;
      for (int t = 1; t < n; ++t)
        th.emplace_back([&, t] {
          try {
            f(t);
          } catch (...) {
            err[(size_t)t] = std::current_exception();
          }
        });
      try {
        f(0);
      } catch (...) {
        err[0] = std::current_exception();
      }
      for (auto& x : th) x.join();
    } else if (n > 1) {
      std::lock_guard<std::mutex> serial(call_mu_);   // one planning call at a time on the pool
      {
        std::lock_guard<std::mutex> lk(mu_);
        while ((int)th_.size() < n - 1) {
          const int id = (int)th_.size();
          th_.emplace_back([this, id] { loop(id); });
        }
        task_ = &f;
        errs_ = &err;
        want_ = n - 1;
        left_ = n - 1;
        ++gen_;
        agen_.store(gen_, std::memory_order_release);
      }
      cv_.notify_all();
      try {
        f(0);
      } catch (...) {
        err[0] = std::current_exception();
      }
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [this] { return left_ == 0; });
      task_ = nullptr;
    } else {
      try {
        f(0);
      } catch (...) {
        err[0] = std::current_exception();
      }
    }
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  }

 private:
  // A worker that just finished spins for up to spin_us() before it sleeps on the condition variable:
  // a chunked call dispatches plan / pack / copy-out back to back (24 dispatches in a 1M-job
  // aggregation), and a futex wake-up per dispatch cost ~50 us each.
  static int spin_us() {   // PE_POOL_SPIN_US (0..2000, default 150; A/B)
    static const int v = [] {
      const char* e = std::getenv("PE_POOL_SPIN_US");
      return e ? std::max(0, std::min(2000, std::atoi(e))) : 150;
    }();
    return v;
  }
  void loop(int id) {
    uint64_t seen = 0;
    bool ran = false;
    for (;;) {
      const std::function<void(int)>* f;
      std::vector<std::exception_ptr>* errs;
      if (ran && spin_us() > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned i = 1; agen_.load(std::memory_order_acquire) == seen; ++i) {
          _mm_pause();
          if ((i & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us())) break;
        }
      }
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        ran = id < want_;
        if (!ran) continue;   // not needed for this call
        f = task_;
        errs = errs_;
      }
      try {
        (*f)(id + 1);
      } catch (...) {
        (*errs)[(size_t)id + 1] = std::current_exception();
      }
      std::lock_guard<std::mutex> lk(mu_);
      if (--left_ == 0) done_cv_.notify_one();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> th_;
  const std::function<void(int)>* task_ = nullptr;
  std::vector<std::exception_ptr>* errs_ = nullptr;
  int want_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  std::atomic<uint64_t> agen_{0};   // gen_, for the spinning workers (written under mu_)
};

// The first index in [0, n) where bad(i) holds, or n: chunks of 4096 reduced branch-free (the
// loops vectorise), on the planning pool for large arrays (the aggregation validates ~10^7 values
// per call).
template <class Bad>
int64_t first_bad(int64_t n, Bad bad) {
  constexpr int64_t kChunk = 4096;
  auto scan = [&](int64_t b, int64_t e) -> int64_t {
    for (int64_t c = b; c < e; c += kChunk) {
      const int64_t ce = std::min(e, c + kChunk);
      bool any = false;
      for (int64_t i = c; i < ce; ++i) any |= bad(i);
      if (any)
        for (int64_t i = c; i < ce; ++i)
          if (bad(i)) return i;
    }
    return e;
  };
  if (n < (int64_t(1) << 20)) return scan(0, n);
  constexpr int kT = 8;
  int64_t first[kT];
  PlanPool::get().run(kT, [&](int t) {
    const int64_t b = n * t / kT, e = n * (t + 1) / kT;
    const int64_t r = scan(b, e);
    first[t] = r < e ? r : n;
  });
  int64_t r = n;
  for (int t = 0; t < kT; ++t) r = std::min(r, first[t]);
  return r;
}

void check_req(const int64_t* req, int64_t n, const char* what) {
  const int64_t i = first_bad(n * pe::D, [req](int64_t k) { return req[k] < 0; });
  if (i < n * pe::D) raise(PE_EINVAL, std::string(what) + ": negative request at index " + std::to_string(i));
}

void check_offsets(const int32_t* off, int64_t n, int64_t limit, const char* what) {
  if (off[0] != 0) raise(PE_EINVAL, std::string(what) + "[0] must be 0");
  if (first_bad(n, [off](int64_t i) { return off[i + 1] < off[i]; }) < n)
    raise(PE_EINVAL, std::string(what) + " is not monotonic");
  if (limit >= 0 && off[n] > limit) raise(PE_EINVAL, std::string(what) + " exceeds its array");
}

// body(j0, j1) over [0, n) in contiguous chunks: on up to 8 threads for large batches (the batch
// planning is on the upload's path), inline for small ones.  Exceptions are rethrown here.
template <class Body>
void parallel_for(int64_t n, Body body) {
  const int64_t nt = n < 32768 ? 1 : std::min<int64_t>(8, std::max(1u, std::thread::hardware_concurrency()));
  if (nt <= 1) {
    body(0, n);
    return;
  }
  PlanPool::get().run((int)nt, [&](int t) { body(n * t / nt, n * (t + 1) / nt); });
}

void fill_req(ReqRec& r, const int64_t* q, uint32_t need) {
  std::memset(&r, 0, sizeof(r));
  for (int d = 0; d < pe::D; ++d) r.q[d] = q[d];
  r.need = need;
}

}  // namespace

extern "C" {

int pe_abi_version(void) { return PE_ABI_VERSION; }

int pe_comm_id(uint8_t out[PE_COMM_ID_BYTES]) {
  if (!out) return PE_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return PE_ERCCL;
  static_assert(sizeof(id) <= PE_COMM_ID_BYTES, "unique id size");
  std::memset(out, 0, PE_COMM_ID_BYTES);
  std::memcpy(out, &id, sizeof(id));
  return PE_OK;
}

int pe_create(const pe_config* cfg, pe_ctx** out) {
  if (!cfg || !out) return PE_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PE_ENODEV;
  if (cfg->world_size < 1 || cfg->rank < 0 || cfg->rank >= cfg->world_size) return PE_EINVAL;
  if (cfg->max_nodes < 0 || cfg->max_nodes > PE_MAX_NODES) return PE_EINVAL;
  pe_ctx* ctx = new (std::nothrow) pe_ctx();
  if (!ctx) return PE_ENOMEM;
  int dev = cfg->device_id;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev >= ndev) {
    delete ctx;
    return PE_EINVAL;
  }
  ctx->device = dev;
  ctx->rank = cfg->rank;
  ctx->world = cfg->world_size;
  ctx->exchange = cfg->exchange;
  ctx->exchange_user = cfg->exchange_user;
  ctx->max_nodes = cfg->max_nodes > 0 ? cfg->max_nodes : PE_MAX_NODES;
  ctx->topk = cfg->topk > 0 ? std::min(cfg->topk, pe::MG_CAP) : 256;
  // 112 groups per window (round 5, 4 interleaved reps on the bench batch: 128 / 112 / 104 / 96 groups
  // 9.53 / 9.25 / 9.53 / 9.50 ms per batch, host 7.98 / 7.65 / 7.70 / 7.38 ms -- smaller windows shrink
  // the resolver's dirty sets, below ~112 the walk + apply chain per window outlasts the resolve)
  ctx->window_groups = cfg->window_groups > 0 ? cfg->window_groups : 112;
  ctx->window_pods = cfg->window_pods > 0 ? cfg->window_pods : 1024;
  ctx->gpu_name = cfg->gpu_resource_name ? cfg->gpu_resource_name : "amd.com/gpu";
  ctx->fit_path_mask = cfg->fit_path_mask & (PATHS_ALL | PATH_NO_THERM | PATH_PLANES_BLOCKS);
  ctx->pl_rows = !(ctx->fit_path_mask & PATH_PLANES_BLOCKS);
  ctx->pipeline = (cfg->greedy_flags & 1) == 0;
  // the walk's block holds K + 1 <= WK_ROUND selected keys; larger K takes the full scan + merge
  ctx->walk = (cfg->greedy_flags & 2) == 0 && ctx->topk + 1 <= pe::WK_ROUND;
  if (cfg->resort_nodes < 0) raise(PE_EINVAL, "resort_nodes < 0");
  ctx->resort_nodes = cfg->resort_nodes > 0 ? cfg->resort_nodes : 20480;   // (profiles/r12_async_resort.txt)
  if (!(ctx->fit_path_mask & PATHS_ALL)) ctx->fit_path_mask |= PATHS_ALL;   // no kernel bits = all kernels
  ctx->fit_path_mask |= PATH_I64;                                           // always available
  int rc = PE_OK;
  try {
    hipchk(hipSetDevice(dev), "hipSetDevice");
    hipchk(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking), "hipStreamCreate");
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
      ctx->num_cu = ncu;
    // RCCL whenever shards exchange without a host callback; a comm_id at world_size 1 also
    // builds a 1-rank communicator (exercises the RCCL window path on a single GPU)
    if (!ctx->exchange && (ctx->world > 1 || cfg->comm_id)) {
      if (!cfg->comm_id) raise(PE_EINVAL, "world_size > 1 needs comm_id or an exchange callback");
      ncclUniqueId id;
      std::memcpy(&id, cfg->comm_id, sizeof(id));
      ctx->comm = comm_init_bounded(ctx->device, ctx->world, id, ctx->rank, rccl_init_timeout_ms());
    }
  } catch (const PeError& e) {
    rc = e.code;
  }
  if (rc != PE_OK) {
    delete ctx;
    return rc;
  }
  *out = ctx;
  return PE_OK;
}

void pe_destroy(pe_ctx* ctx) { delete ctx; }

const char* pe_last_error(const pe_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// A node's device / mirror labels: the caller's bits 0-30, bit 31 = the node has an xGMI island
// (PE_LABEL_ISLAND, what an island group's need requires).
static uint32_t node_labels(const uint32_t* labels, const int32_t* island, int64_t i) {
  const uint32_t l = labels ? labels[i] : 0u;
  const bool has = island && island[i] >= 0;
  return (l & ~PE_LABEL_ISLAND) | (has ? PE_LABEL_ISLAND : 0u);
}

int pe_load_nodes(pe_ctx* ctx, int64_t n, const int64_t* cap, const int64_t* used, const uint32_t* labels,
                  const int32_t* island) {
  return guarded(ctx, [&]() -> int {
    if (n < 0 || n > ctx->max_nodes) raise(PE_EINVAL, "node count out of range");
    if (n > 0) {
      need_ptr(cap, "cap");
      need_ptr(used, "used");
    }
    ctx->n_total = n;
    ctx->begin = n * ctx->rank / ctx->world;
    ctx->end = n * (ctx->rank + 1) / ctx->world;
    ctx->Ns = ctx->end - ctx->begin;
    ctx->stride = round_up(std::max<int64_t>(ctx->Ns, 1), 256);
    const size_t cells = (size_t)pe::D * (size_t)ctx->stride;
    std::vector<int64_t> r(cells, pe::NEVER);
    std::vector<uint32_t> lab((size_t)ctx->stride, 0u);
    std::vector<int32_t> isl((size_t)ctx->stride, -1);
    for (int d = 0; d < pe::D; ++d)
      for (int64_t i = 0; i < ctx->Ns; ++i) {
        const int64_t g = ctx->begin + i;
        const int64_t c = cap[d * n + g], u = used[d * n + g];
        if (c < 0 || u < 0) raise(PE_EINVAL, "negative capacity/usage");
        r[(size_t)d * ctx->stride + i] = c - u;
      }
    for (int64_t i = 0; i < ctx->Ns; ++i) {
      lab[i] = node_labels(labels, island, ctx->begin + i);
      isl[i] = island ? island[ctx->begin + i] : -1;
    }
    ctx->m_nodes.assign((size_t)n, pe::NodeState{});
    for (int d = 0; d < pe::D; ++d)
      for (int64_t g = 0; g < n; ++g) {
        if (cap[d * n + g] < 0 || used[d * n + g] < 0) raise(PE_EINVAL, "negative capacity/usage");
        ctx->m_nodes[g].res[d] = cap[d * n + g] - used[d * n + g];
      }
    for (int64_t g = 0; g < n; ++g) ctx->m_nodes[g].labels = node_labels(labels, island, g);
    ctx->m_nodes0 = ctx->m_nodes;
    hipchk(ctx->res0.ensure(cells), "alloc res0");
    hipchk(ctx->res.ensure(cells), "alloc res");
    hipchk(ctx->labels.ensure((size_t)ctx->stride), "alloc labels");
    hipchk(ctx->island.ensure((size_t)ctx->stride), "alloc island");
    hipchk(hipMemcpyAsync(ctx->res0.p, r.data(), cells * 8, hipMemcpyHostToDevice, ctx->stream), "H2D res0");
    hipchk(hipMemcpyAsync(ctx->res.p, r.data(), cells * 8, hipMemcpyHostToDevice, ctx->stream), "H2D res");
    hipchk(hipMemcpyAsync(ctx->labels.p, lab.data(), lab.size() * 4, hipMemcpyHostToDevice, ctx->stream), "H2D lab");
    hipchk(hipMemcpyAsync(ctx->island.p, isl.data(), isl.size() * 4, hipMemcpyHostToDevice, ctx->stream), "H2D isl");
    hipchk(hipStreamSynchronize(ctx->stream), "sync load");
    ctx->loaded = true;
    return PE_OK;
  });
}

int pe_update_nodes(pe_ctx* ctx, int64_t n, const int64_t* slots, const uint8_t* op, const int64_t* cap,
                    const int64_t* used, const uint32_t* labels, const int32_t* island) {
  return guarded(ctx, [&]() -> int {
    if (!ctx->loaded) raise(PE_ESTATE, "no inventory loaded");
    if (n < 0) raise(PE_EINVAL, "n < 0");
    if (n == 0) return PE_OK;
    need_ptr(slots, "slots");
    need_ptr(op, "op");
    // validate the whole batch first: nothing is applied unless every entry is valid
    bool any_set = false;
    for (int64_t i = 0; i < n; ++i) {
      if (slots[i] < 0 || slots[i] >= ctx->n_total) raise(PE_EINVAL, "slot out of range");
      if (op[i] != PE_NODE_SET && op[i] != PE_NODE_REMOVE) raise(PE_EINVAL, "unknown node op");
      any_set |= op[i] == PE_NODE_SET;
    }
    if (any_set) {
      need_ptr(cap, "cap");
      need_ptr(used, "used");
      for (int64_t i = 0; i < n; ++i)
        if (op[i] == PE_NODE_SET)
          for (int d = 0; d < pe::D; ++d)
            if (cap[i * pe::D + d] < 0 || used[i * pe::D + d] < 0) raise(PE_EINVAL, "negative capacity/usage");
    }
    // the host mirror takes every entry in order (global inventory)
    for (int64_t i = 0; i < n; ++i) {
      const int64_t g = slots[i];
      pe::NodeState& m = ctx->m_nodes[g];
      for (int d = 0; d < pe::D; ++d)
        m.res[d] = op[i] == PE_NODE_SET ? cap[i * pe::D + d] - used[i * pe::D + d] : pe::NEVER;
      m.labels = op[i] == PE_NODE_SET ? node_labels(labels, island, i) : 0u;
      ctx->m_nodes0[g] = m;
    }
    // last entry per slot wins; keep only this shard's slots
    std::unordered_map<int64_t, int64_t> last;
    last.reserve((size_t)n * 2);
    for (int64_t i = 0; i < n; ++i)
      if (slots[i] >= ctx->begin && slots[i] < ctx->end) last[slots[i]] = i;
    std::vector<pe::NodeUpd> upd;
    upd.reserve(last.size());
    for (int64_t i = 0; i < n; ++i) {
      auto it = last.find(slots[i]);
      if (it == last.end() || it->second != i) continue;
      pe::NodeUpd u{};
      u.local = slots[i] - ctx->begin;
      if (op[i] == PE_NODE_SET) {
        for (int d = 0; d < pe::D; ++d) u.res[d] = cap[i * pe::D + d] - used[i * pe::D + d];
        u.labels = node_labels(labels, island, i);
        u.island = island ? island[i] : -1;
      } else {
        for (int d = 0; d < pe::D; ++d) u.res[d] = pe::NEVER;
        u.labels = 0u;
        u.island = -1;
      }
      upd.push_back(u);
    }
    if (upd.empty()) return PE_OK;
    hipchk(ctx->n_upd.ensure(upd.size()), "alloc node updates");
    hipchk(hipMemcpyAsync(ctx->n_upd.p, upd.data(), upd.size() * sizeof(pe::NodeUpd), hipMemcpyHostToDevice,
                          ctx->stream),
           "H2D node updates");
    hipchk(pe::launch_scatter_nodes(ctx->stream, ctx->res.p, ctx->res0.p, ctx->stride, ctx->labels.p, ctx->island.p,
                                    ctx->n_upd.p, (int64_t)upd.size()),
           "launch scatter_nodes");
    hipchk(hipStreamSynchronize(ctx->stream), "sync node updates");   // the host vector dies here
    return PE_OK;
  });
}

int pe_reset_residuals(pe_ctx* ctx) {
  return guarded(ctx, [&]() -> int {
    if (!ctx->loaded) raise(PE_ESTATE, "no inventory loaded");
    hipchk(hipMemcpyAsync(ctx->res.p, ctx->res0.p, (size_t)pe::D * ctx->stride * 8, hipMemcpyDeviceToDevice,
                          ctx->stream),
           "D2D reset");
    ctx->m_nodes = ctx->m_nodes0;
    return PE_OK;
  });
}

int pe_shard_range(const pe_ctx* ctx, int64_t* begin, int64_t* end) {
  if (!ctx || !begin || !end) return PE_EINVAL;
  *begin = ctx->begin;
  *end = ctx->end;
  return PE_OK;
}

int pe_comm_ranks(const pe_ctx* ctx, int32_t* nranks) {
  if (!ctx || !nranks) return PE_EINVAL;
  *nranks = 0;
  if (!ctx->comm) return PE_OK;
  int n = 0;
  if (ncclCommCount(ctx->comm, &n) != ncclSuccess) return PE_ERCCL;
  *nranks = n;
  return PE_OK;
}

int pe_read_residuals(pe_ctx* ctx, int64_t* res_out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx->loaded) raise(PE_ESTATE, "no inventory loaded");
    need_ptr(res_out, "res_out");
    for (int d = 0; d < pe::D; ++d)
      hipchk(hipMemcpyAsync(res_out + (size_t)d * ctx->Ns, ctx->res.p + (size_t)d * ctx->stride,
                            (size_t)ctx->Ns * 8, hipMemcpyDeviceToHost, ctx->stream),
             "D2H res");
    hipchk(hipStreamSynchronize(ctx->stream), "sync read");
    return PE_OK;
  });
}

}  // extern "C"

namespace {

// Wait for the one-segment aggregation kernel's flag (pinned host memory, written after its outputs).
// The stream is polled now and then: a faulted kernel surfaces as its HIP error, a kernel that ended
// without the flag as PE_EHIP.
void agg_wait_flag(pe_ctx* ctx, uint32_t gen) {
  for (unsigned spin = 1;; ++spin) {
    if (__atomic_load_n(ctx->a_flag.p, __ATOMIC_ACQUIRE) == gen) return;
    _mm_pause();
    if ((spin & 1023) == 0) {
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipErrorNotReady) continue;
      hipchk(e, "aggregation kernel");
      if (__atomic_load_n(ctx->a_flag.p, __ATOMIC_ACQUIRE) == gen) return;
      raise(PE_EHIP, "aggregation kernel finished without signalling");
    }
  }
}

// The r2 call path (device copies of the six input arrays, four D2H copies): PE_AGG_DEVICE=1 A/B.
void agg_device_path(pe_ctx* ctx, int32_t mode, int64_t n_jobs, int64_t G, int64_t C, const int32_t* job_group_off,
                     const int32_t* min_member, const int32_t* group_replicas, const int32_t* group_cont_off,
                     const int64_t* cont_req, const uint8_t* cont_flags, int64_t* out_min_res, uint8_t* out_present,
                     int32_t* out_members, uint8_t* out_overflow) {
  if (C > 0) check_req(cont_req, C, "cont_req");
  hipStream_t s = ctx->stream;
  hipchk(ctx->a_jgo.ensure(n_jobs + 1), "alloc");
  hipchk(ctx->a_mm.ensure(n_jobs), "alloc");
  hipchk(ctx->a_rep.ensure(G), "alloc");
  hipchk(ctx->a_gco.ensure(G + 1), "alloc");
  hipchk(ctx->a_req.ensure((size_t)C * pe::D), "alloc");
  hipchk(ctx->a_fl.ensure(C), "alloc");
  hipchk(ctx->a_out.ensure((size_t)n_jobs * pe::D), "alloc");
  hipchk(ctx->a_pres.ensure(n_jobs), "alloc");
  hipchk(ctx->a_mem.ensure(n_jobs), "alloc");
  hipchk(ctx->a_ovf.ensure(n_jobs), "alloc");
  hipchk(hipMemcpyAsync(ctx->a_jgo.p, job_group_off, (n_jobs + 1) * 4, hipMemcpyHostToDevice, s), "H2D");
  if (mode == PE_MODE_V1) hipchk(hipMemcpyAsync(ctx->a_mm.p, min_member, n_jobs * 4, hipMemcpyHostToDevice, s), "H2D");
  if (G > 0) {
    hipchk(hipMemcpyAsync(ctx->a_rep.p, group_replicas, G * 4, hipMemcpyHostToDevice, s), "H2D");
    hipchk(hipMemcpyAsync(ctx->a_gco.p, group_cont_off, (G + 1) * 4, hipMemcpyHostToDevice, s), "H2D");
  }
  if (C > 0) {
    hipchk(hipMemcpyAsync(ctx->a_req.p, cont_req, (size_t)C * pe::D * 8, hipMemcpyHostToDevice, s), "H2D");
    hipchk(hipMemcpyAsync(ctx->a_fl.p, cont_flags, C, hipMemcpyHostToDevice, s), "H2D");
  }
  hipchk(pe::launch_pg_min_resources(s, mode, n_jobs, ctx->a_jgo.p, ctx->a_mm.p, ctx->a_rep.p, ctx->a_gco.p,
                                     ctx->a_req.p, ctx->a_fl.p, ctx->a_out.p, ctx->a_pres.p, ctx->a_mem.p, ctx->a_ovf.p),
         "launch pg_min_resources");
  hipchk(hipMemcpyAsync(out_min_res, ctx->a_out.p, (size_t)n_jobs * pe::D * 8, hipMemcpyDeviceToHost, s), "D2H");
  hipchk(hipMemcpyAsync(out_present, ctx->a_pres.p, n_jobs, hipMemcpyDeviceToHost, s), "D2H");
  hipchk(hipMemcpyAsync(out_members, ctx->a_mem.p, n_jobs * 4, hipMemcpyDeviceToHost, s), "D2H");
  hipchk(hipMemcpyAsync(out_overflow, ctx->a_ovf.p, n_jobs, hipMemcpyDeviceToHost, s), "D2H");
  hipchk(hipStreamSynchronize(s), "sync pg_min_resources");
}

// Per-key OR of rows x 4 int64 request records (the narrowing test of a segment, below)
__attribute__((target("avx2"))) void or_rows4(const int64_t* q, int64_t rows, uint64_t orv[4]) {
  __m256i a = _mm256_setzero_si256(), b = _mm256_setzero_si256();
  int64_t r = 0;
  for (; r + 2 <= rows; r += 2) {
    a = _mm256_or_si256(a, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(q + r * 4)));
    b = _mm256_or_si256(b, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(q + r * 4 + 4)));
  }
  if (r < rows) a = _mm256_or_si256(a, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(q + r * 4)));
  _mm256_storeu_si256(reinterpret_cast<__m256i*>(orv), _mm256_or_si256(a, b));
}

// rows x 4 int64 records -> rows x 4 u32 of value >> sh[key] (the values are known to fit)
// NT: non-temporal stores (dst 16-B aligned): the staging buffer is written once and read by the DMA
// engine, so no line of it is read for ownership first (the pack's host-memory traffic is otherwise
// read + RFO + write)
template <bool NT>
__attribute__((target("avx2"))) void narrow_rows4(uint32_t* dst, const int64_t* q, int64_t rows, const uint8_t sh[4]) {
  const __m256i vs = _mm256_set_epi64x(sh[3], sh[2], sh[1], sh[0]);
  const __m256i even = _mm256_set_epi32(7, 5, 3, 1, 6, 4, 2, 0);
  for (int64_t r = 0; r < rows; ++r) {
    const __m256i v = _mm256_srlv_epi64(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(q + r * 4)), vs);
    const __m128i lo = _mm256_castsi256_si128(_mm256_permutevar8x32_epi32(v, even));
    if constexpr (NT) _mm_stream_si128(reinterpret_cast<__m128i*>(dst + r * 4), lo);
    else _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + r * 4), lo);
  }
}

// memcpy into a 16-B aligned staging section with non-temporal stores (whole 16-B chunks; the tail
// with plain stores)
__attribute__((target("avx2"))) void nt_copy(void* dst, const void* src, size_t bytes) {
  uint8_t* d = static_cast<uint8_t*>(dst);
  const uint8_t* s = static_cast<const uint8_t*>(src);
  size_t i = 0;
  for (; i + 16 <= bytes; i += 16)
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i), _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i)));
  if (i < bytes) std::memcpy(d + i, s + i, bytes - i);
}

// dst[0, n) = src[0, n) and the OR of all values (its sign says whether any is negative), in one
// pass: the aggregation's request records are validated while they are packed.
template <bool NT>
__attribute__((target("avx2"))) int64_t copy_or_i64(int64_t* dst, const int64_t* src, int64_t n) {
  __m256i acc = _mm256_setzero_si256();
  int64_t i = 0;
  for (; i + 4 <= n; i += 4) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    if constexpr (NT) {   // (dst 16-B aligned: two 16-B streams)
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), _mm256_castsi256_si128(v));
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 2), _mm256_extracti128_si256(v, 1));
    } else {
      _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i), v);
    }
    acc = _mm256_or_si256(acc, v);
  }
  alignas(32) int64_t lanes[4];
  _mm256_store_si256(reinterpret_cast<__m256i*>(lanes), acc);
  int64_t any = lanes[0] | lanes[1] | lanes[2] | lanes[3];
  for (; i < n; ++i) {
    dst[i] = src[i];
    any |= src[i];
  }
  return any;
}

// Grow-only pinned buffer (a 1M-job batch needs ~170 MB; hipHostMalloc costs ms, so keep it).
template <class T>
void ensure_pinned(HostBuf<T>& b, size_t count, const char* what) {
  if (count <= b.n && b.p) return;
  hipchk(b.ensure(std::max(count, b.n + b.n / 2), kZeroCopy), what);
}

// Call path (pe_kernels.h AggSegHdr): validate + pack the batch into segments of <= 256 jobs in a
// pinned, device-mapped staging buffer (on the planning pool for large batches), one block per
// segment (the segment comes into LDS in one round of coalesced 16-B loads), outputs written by the
// kernel straight into a pinned buffer in the caller's layout, then copied out.  Up to 8192 jobs: one
// launch reading the pinned segments over PCIe, the host waiting on a flag the kernel stores in pinned
// memory (the operator's per-reconcile call: one job).  Larger batches: chunks planned, packed, DMA'd
// to the device and launched one after another (below).
// ak / n_keys: the fixed four dimensions ({4, 1}, n_keys 4) or a per-call key table of n_keys <= 16
// keys padded to ak.nd (pe_pg_min_resources_keys); cont_flags / out_present are u8 or u32 / u16.
int agg_call(pe_ctx* ctx, int32_t mode, int64_t n_jobs, pe::AggKeys ak, int n_keys, const int32_t* job_group_off,
                    const int32_t* min_member, const int32_t* group_replicas, const int32_t* group_cont_off,
                    const int64_t* cont_req, const void* cont_flags_v, int64_t* out_min_res, void* out_present_v,
                    int32_t* out_members, uint8_t* out_overflow) {
  const uint8_t* cont_flags = static_cast<const uint8_t*>(cont_flags_v);
  uint8_t* out_present = static_cast<uint8_t*>(out_present_v);
  const bool wide = ak.fb != 1;
  const int ND = ak.nd;
  const int pb = wide ? 2 : 1;   // presence bytes per job out
  return guarded(ctx, [&]() -> int {
    if (mode != PE_MODE_V1 && mode != PE_MODE_V2) raise(PE_EINVAL, "mode must be PE_MODE_V1 or PE_MODE_V2");
    if (n_jobs < 0) raise(PE_EINVAL, "n_jobs < 0");
    if (n_jobs == 0) return PE_OK;
    need_ptr(job_group_off, "job_group_off");
    need_ptr(out_min_res, "out_min_res");
    need_ptr(out_present, "out_present");
    need_ptr(out_members, "out_members");
    need_ptr(out_overflow, "out_overflow");
    if (mode == PE_MODE_V1) need_ptr(min_member, "min_member");
    check_offsets(job_group_off, n_jobs, -1, "job_group_off");
    const int64_t G = job_group_off[n_jobs];
    if (G > 0) {
      need_ptr(group_replicas, "group_replicas");
      need_ptr(group_cont_off, "group_cont_off");
      check_offsets(group_cont_off, G, -1, "group_cont_off");
    }
    const int64_t C = G > 0 ? group_cont_off[G] : 0;
    if (C > 0) {
      need_ptr(cont_req, "cont_req");
      need_ptr(cont_flags, "cont_flags");
    }
    if (wide && C > 0) {   // a key table's flags: presence bits of the call's keys and the kind only
      const uint32_t allowed = ((n_keys >= 32 ? 0u : (1u << n_keys)) - 1u) | (3u << PE_KEYS_KIND_SHIFT);
      const uint32_t* f32 = static_cast<const uint32_t*>(cont_flags_v);
      for (int64_t c = 0; c < C; ++c)
        if (f32[c] & ~allowed)
          raise(PE_EINVAL, "cont_flags[" + std::to_string(c) + "]: presence bit past n_keys or unknown bits");
    }
    if (!wide && std::getenv("PE_AGG_DEVICE")) {
      agg_device_path(ctx, mode, n_jobs, G, C, job_group_off, min_member, group_replicas, group_cont_off, cont_req,
                      cont_flags, out_min_res, out_present, out_members, out_overflow);
    } else {
      const bool v1 = mode == PE_MODE_V1;
      const int32_t* gco = G > 0 ? group_cont_off : nullptr;
      // PE_AGG_TRACE=1: phase times of the call on stderr (diagnostics)
      const bool trace = std::getenv("PE_AGG_TRACE") != nullptr;
      auto now = [] { return std::chrono::steady_clock::now(); };
      const auto tt0 = now();
      double t_pack = 0;
      // 1. segments, per job range (one range below 32k jobs; segments never span ranges)
      // PE_AGG_THREADS (1..16, default 8): host threads planning / packing / copying out a large batch
      static const int kAggT = [] {
        const char* e = std::getenv("PE_AGG_THREADS");
        return e ? std::max(1, std::min(PlanPool::kMax, std::atoi(e))) : 8;
      }();
      const int T = n_jobs < 32768 ? 1 : kAggT;
      // Calls of <= kLatJobs jobs are one launch the host waits on through the kernel's flag; up to
      // 2048 jobs with segments of 32 jobs, so a 256-job call spreads its ~40 KB over 8 CUs (one
      // CU's zero-copy reads come in at a few GB/s: 41 KB through one block took ~27 us, 8 blocks
      // 19 us); larger batches take 256-job segments, above kLatJobs in chunks with a stream sync.
      // PE_AGG_SEG_JOBS overrides the segment size (A/B, profiles/r10_agg_latency.txt).
      constexpr int64_t kLatJobs = 8192;
      int64_t seg_jobs = n_jobs <= 2048 ? 32 : pe::AGG_SEG_JOBS;   // (8192 jobs: 94 us with 256, 112 with 32)
      if (const char* e = std::getenv("PE_AGG_SEG_JOBS")) seg_jobs = std::max<int64_t>(1, std::min<int64_t>(pe::AGG_SEG_JOBS, std::atoll(e)));
      // Large batches run in chunks (PE_AGG_CHUNKS, 1..64, default 8): chunk k's segments are planned
      // and packed by the planning pool while chunk k - 1 crosses PCIe, so the link starts after the
      // first chunk's plan and pack instead of the whole batch's plan (0.3 ms of a 1M-job call).
      static const int64_t kChunks = [] {
        const char* e = std::getenv("PE_AGG_CHUNKS");
        return e ? std::max<int64_t>(1, std::min<int64_t>(64, std::atoll(e))) : 8;
      }();
      const int64_t CH = n_jobs > kLatJobs && T > 1 ? kChunks : 1;
      // PE_AGG_ONE_PLAN=1 (A/B): the whole batch planned before the first chunk is packed
      static const bool one_plan = std::getenv("PE_AGG_ONE_PLAN") != nullptr;
      auto& segs = ctx->agg_segs;
      if (segs.size() < (size_t)T) segs.resize((size_t)T);
      // A segment's requests cross narrowed (pe_kernels.h agg_seg_layout) when every key's values span
      // <= 32 bits above their common trailing zeros, none is negative, and it saves bytes; else as the
      // caller's int64 records.  PE_AGG_WIDE=1: never narrowed (A/B).
      static const bool no_narrow = std::getenv("PE_AGG_WIDE") != nullptr;
      auto narrow_seg = [&](AggSeg& sg) {
        sg.narrow = false;
        if (no_narrow || sg.nc == 0 ||
            pe::agg_req_bytes(sg.nc, ND, true) >= pe::agg_req_bytes(sg.nc, ND, false))
          return;
        const int64_t* q = cont_req + (int64_t)gco[job_group_off[sg.j0]] * n_keys;
        uint64_t orv[pe::AGG_MAX_KEYS] = {0};
        if (n_keys == 4) {
          or_rows4(q, sg.nc, orv);
        } else {
          for (int64_t c = 0; c < sg.nc; ++c)
            for (int k = 0; k < n_keys; ++k) orv[k] |= (uint64_t)q[c * n_keys + k];
        }
        for (int k = 0; k < ND; ++k) {
          const uint64_t v = k < n_keys ? orv[k] : 0;
          if (v >> 63) return;   // a negative request: the wide pack reports it
          const int tz = v ? __builtin_ctzll(v) : 0;
          if (v && 63 - __builtin_clzll(v) - tz > 31) return;
          sg.sh[k] = (uint8_t)tz;
        }
        sg.narrow = true;
        int64_t off[7];
        pe::agg_seg_layout(sg.nj, sg.ng, sg.nc, v1, off, ak, true);
        sg.bytes = off[6];
      };
      auto plan = [&](int t, int64_t pa, int64_t pb) {   // thread t's share of jobs [pa, pb)
        const int64_t ja = pa + (pb - pa) * t / T, jb = pa + (pb - pa) * (t + 1) / T;
        auto& out = segs[(size_t)t];
        out.clear();
        int64_t off[7];
        for (int64_t j = ja; j < jb;) {
          AggSeg sg{j, 0, 0, 0, 0, false, {}};
          while (j < jb && sg.nj < seg_jobs) {
            const int64_t g0 = job_group_off[j], g1 = job_group_off[j + 1];
            const int64_t nc = gco ? (int64_t)gco[g1] - gco[g0] : 0;
            pe::agg_seg_layout(sg.nj + 1, sg.ng + (g1 - g0), sg.nc + nc, v1, off, ak);
            if (sg.nj > 0 && off[6] > pe::AGG_SEG_BYTES) break;
            ++sg.nj;
            sg.ng += (int32_t)(g1 - g0);
            sg.nc += (int32_t)nc;
            sg.bytes = off[6];
            ++j;
          }
          narrow_seg(sg);
          out.push_back(sg);
        }
      };
      auto& all = ctx->agg_all;   // every planned segment so far, in job order
      all.clear();
      // chunk c: plan jobs [n c / CH, n (c + 1) / CH), its segments appended to all and their offsets to so
      int64_t* so = nullptr;
      auto plan_chunk = [&](int64_t c) {   // (c = -1: every job, in one pass)
        const int64_t pa = c < 0 ? 0 : n_jobs * c / CH, pb = c < 0 ? n_jobs : n_jobs * (c + 1) / CH;
        if (T == 1) plan(0, pa, pb);
        else PlanPool::get().run(T, [&](int t) { plan(t, pa, pb); });
        const size_t k0 = all.size();
        for (int t = 0; t < T; ++t) all.insert(all.end(), segs[t].begin(), segs[t].end());
        if (so)
          for (size_t k = k0; k < all.size(); ++k) so[k + 1] = so[k] + all[k].bytes;
      };
      // Pinned staging sized before the first chunk is planned (a chunked call writes chunk 0 before the
      // rest is planned): raw section bytes plus at most 8 + 5 x 15 B of padding and a header per
      // segment; a segment ends at seg_jobs jobs, at a chunk or thread boundary, or where it and the
      // next job would pass AGG_SEG_BYTES -- each job's bytes are in at most two such sums.
      const int64_t raw = n_jobs * 8 + G * 8 + C * (8 * ND + ak.fb);
      const int64_t seg_cap = n_jobs / seg_jobs + 2 * raw / (pe::AGG_SEG_BYTES - 128) + CH * T + 2;
      const int64_t seg_over = (int64_t)sizeof(pe::AggSegHdr) + 8 + 5 * 15;
      int64_t nseg = 0, total = 0;
      if (CH == 1 || one_plan) {
        plan_chunk(-1);
        nseg = (int64_t)all.size();
        ensure_pinned(ctx->a_segoff, (size_t)nseg + 1, "alloc pinned segment offsets");
        so = ctx->a_segoff.p;
        so[0] = 0;
        for (int64_t k = 0; k < nseg; ++k) so[k + 1] = so[k] + all[(size_t)k].bytes;
        total = so[nseg];
      } else {
        ensure_pinned(ctx->a_segoff, (size_t)seg_cap + 1, "alloc pinned segment offsets");
        so = ctx->a_segoff.p;
        so[0] = 0;
        total = raw + seg_cap * seg_over;   // (an upper bound: the staging capacity)
      }
      int64_t oo[4];
      pe::agg_out_layout(n_jobs, oo, ak);
      const int64_t out_bytes = oo[3] + pe::agg_r16(n_jobs);
      ensure_pinned(ctx->a_stage, (size_t)total, "alloc pinned aggregation batch");
      ensure_pinned(ctx->a_outh, (size_t)out_bytes, "alloc pinned aggregation outputs");
      if (!ctx->a_flag.p) {
        hipchk(ctx->a_flag.ensure(16, kZeroCopy), "alloc pinned flag");
        // pinned memory may come back recycled (e.g. the flag of an engine destroyed earlier): clear
        // it, and start the generations past whatever it held, so no stale value matches a wait
        __atomic_store_n(ctx->a_flag.p, 0u, __ATOMIC_RELEASE);
        ctx->agg_gen = 0;
      }
      if (!ctx->a_ctr.p) {
        hipchk(ctx->a_ctr.ensure(1), "alloc done counter");
        hipchk(hipMemsetAsync(ctx->a_ctr.p, 0, 4, ctx->stream), "memset done counter");
      }
      const auto tt1 = now();
      // 2. pack (and the negative-request check, on the copied values); 3. launch
      int64_t bad[PlanPool::kMax];
      std::fill(bad, bad + PlanPool::kMax, INT64_MAX);
      // non-temporal stores for the request records of large calls (PE_AGG_NO_NT=1: plain stores, A/B)
      static const bool nt_env = std::getenv("PE_AGG_NO_NT") == nullptr;
      const bool nt = nt_env && n_jobs > kLatJobs;
      auto pack = [&](int64_t s0, int64_t s1, int64_t& badv) {
        struct Fence {   // the streamed lines are globally visible before the pack returns (the DMA reads them)
          bool on;
          ~Fence() {
            if (on) _mm_sfence();
          }
        } fence{nt};
        for (int64_t k = s0; k < s1; ++k) {
          const AggSeg& sg = all[(size_t)k];
          uint8_t* b = ctx->a_stage.p + so[k];
          pe::AggSegHdr h{};
          h.j0 = sg.j0;
          h.nj = sg.nj;
          h.ng = sg.ng;
          h.nc = sg.nc;
          const int32_t g0 = job_group_off[sg.j0];
          h.g0 = g0;
          h.c0 = sg.ng > 0 ? gco[g0] : 0;
          h.narrow = sg.narrow ? 1 : 0;
          std::memcpy(b, &h, sizeof(h));
          int64_t off[7];
          pe::agg_seg_layout(sg.nj, sg.ng, sg.nc, v1, off, ak, sg.narrow);
          // offsets copied as they are (the kernel rebases by h.g0 / h.c0): every section is a memcpy
          auto copy = [nt](void* d, const void* src, size_t bytes) {
            if (nt) nt_copy(d, src, bytes);
            else std::memcpy(d, src, bytes);
          };
          copy(b + off[0], job_group_off + sg.j0, (size_t)(sg.nj + 1) * 4);
          if (v1) copy(b + off[1], min_member + sg.j0, (size_t)sg.nj * 4);
          if (sg.ng > 0) {
            copy(b + off[2], group_replicas + g0, (size_t)sg.ng * 4);
            const int32_t c0 = h.c0;
            copy(b + off[3], gco + g0, (size_t)(sg.ng + 1) * 4);
            if (sg.nc > 0) {
              const int64_t* q = cont_req + (int64_t)c0 * n_keys;
              const int64_t nq = (int64_t)sg.nc * n_keys;
              int64_t any;
              if (sg.narrow) {   // (no negative value: narrow_seg checked)
                std::memcpy(b + off[4], sg.sh, 16);
                uint32_t* d = reinterpret_cast<uint32_t*>(b + off[4] + 16);
                if (n_keys == 4 && ND == 4) {
                  if (nt) narrow_rows4<true>(d, q, sg.nc, sg.sh);
                  else narrow_rows4<false>(d, q, sg.nc, sg.sh);
                } else {
                  for (int32_t c = 0; c < sg.nc; ++c) {
                    for (int k = 0; k < n_keys; ++k)
                      d[(int64_t)c * ND + k] = (uint32_t)((uint64_t)q[(int64_t)c * n_keys + k] >> sg.sh[k]);
                    for (int k = n_keys; k < ND; ++k) d[(int64_t)c * ND + k] = 0;
                  }
                }
                any = 0;
              } else if (n_keys == ND) {
                any = nt ? copy_or_i64<true>(reinterpret_cast<int64_t*>(b + off[4]), q, nq)   // one pass
                         : copy_or_i64<false>(reinterpret_cast<int64_t*>(b + off[4]), q, nq);
              } else {   // a key table narrower than its kernel: rows padded with zeros (never present)
                int64_t* d = reinterpret_cast<int64_t*>(b + off[4]);
                int64_t acc = 0;
                for (int32_t c = 0; c < sg.nc; ++c) {
                  for (int k = 0; k < n_keys; ++k) acc |= d[(int64_t)c * ND + k] = q[(int64_t)c * n_keys + k];
                  for (int k = n_keys; k < ND; ++k) d[(int64_t)c * ND + k] = 0;
                }
                any = acc;
              }
              copy(b + off[5], cont_flags + (int64_t)c0 * ak.fb, (size_t)sg.nc * ak.fb);
              if (any < 0 && badv == INT64_MAX)
                for (int64_t i = 0; i < nq; ++i)
                  if (q[i] < 0) {
                    badv = (int64_t)c0 * n_keys + i;
                    break;
                  }
            }
          } else {
            reinterpret_cast<int32_t*>(b + off[3])[0] = 0;   // (h.c0 = 0)
          }
        }
      };
      uint8_t* const od = ctx->a_outh.dev;
      const uint8_t* oh = ctx->a_outh.p;
      auto unpack = [&](int64_t a, int64_t e) {   // outputs of jobs [a, e) into the caller's arrays
        if (n_keys == ND) {
          std::memcpy(out_min_res + a * n_keys, oh + oo[0] + a * 8 * ND, (size_t)(e - a) * 8 * ND);
        } else {
          const int64_t* src = reinterpret_cast<const int64_t*>(oh + oo[0]);
          for (int64_t j = a; j < e; ++j) std::memcpy(out_min_res + j * n_keys, src + j * ND, (size_t)n_keys * 8);
        }
        std::memcpy(out_members + a, oh + oo[1] + a * 4, (size_t)(e - a) * 4);
        std::memcpy(out_present + a * pb, oh + oo[2] + a * pb, (size_t)(e - a) * pb);
        std::memcpy(out_overflow + a, oh + oo[3] + a, (size_t)(e - a));
      };
      int64_t unpacked = 0;   // jobs [0, unpacked) already copied out
      int64_t first_neg = INT64_MAX;
      double t_launch = 0, t_wait = 0;
      if (n_jobs <= kLatJobs) {   // latency path: one launch, the host waits on the flag
        const auto tp = now();
        pack(0, nseg, bad[0]);
        first_neg = bad[0];
        t_pack = std::chrono::duration<double, std::milli>(now() - tp).count();
        if (first_neg == INT64_MAX) {
          if (++ctx->agg_gen == 0) ++ctx->agg_gen;
          const auto tl = now();
          if (nseg == 1 && total <= pe::AGG_KARG_BYTES && !std::getenv("PE_AGG_NO_KARG")) {
            // the segment in the kernel arguments (no zero-copy read; PE_AGG_NO_KARG=1: A/B)
            static thread_local pe::AggKarg karg;   // (512 B)
            std::memcpy(karg.b, ctx->a_stage.p, (size_t)total);
            hipchk(pe::launch_pg_agg_karg(ctx->stream, mode, karg, total, od, n_jobs, ctx->a_flag.dev, ctx->agg_gen, ak),
                   "launch pg_agg_karg");
          } else {
            hipchk(pe::launch_pg_agg_segments(ctx->stream, mode, ctx->a_stage.dev,
                                              nseg == 1 ? nullptr : ctx->a_segoff.dev, nseg, total, od, n_jobs,
                                              ctx->a_flag.dev, ctx->agg_gen, ctx->a_ctr.p, ak),
                   "launch pg_agg_segments");
          }
          const auto tw = now();
          agg_wait_flag(ctx, ctx->agg_gen);
          t_launch = std::chrono::duration<double, std::milli>(tw - tl).count();
          t_wait = std::chrono::duration<double, std::milli>(now() - tw).count();
        }
      } else {
        // chunks of segments, each planned and packed by the planning pool and launched at once: chunk
        // k's segments cross PCIe while the host plans and packs chunk k + 1, and chunk k - 1's outputs
        // are copied out once its kernel is done (an event per chunk).  The input crosses as one DMA per
        // chunk (a copy engine on its own stream, pinned -> device; the chunk's kernel waits on its event
        // and reads the segments from HBM): the copy engine streams the link at its rate, where the
        // kernels' own zero-copy reads reached ~2/3 of it beside their output writes (round 5: 3.35 ms
        // of kernel for a 2.2 ms input stream).  Outputs stay zero-copy writes into pinned memory: the
        // link's other direction.  PE_AGG_ZEROCOPY=1: the kernels read the pinned batch directly (A/B).
        const bool dma = !std::getenv("PE_AGG_ZEROCOPY");
        while ((int64_t)ctx->a_ev.size() < CH) {
          hipEvent_t e;
          hipchk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
          ctx->a_ev.push_back(e);
        }
        if (dma) {
          hipchk(ctx->a_dstage.ensure((size_t)total), "alloc device aggregation batch");
          if (!ctx->a_h2d) hipchk(hipStreamCreateWithFlags(&ctx->a_h2d, hipStreamNonBlocking), "stream");
          while ((int64_t)ctx->a_ev_h2d.size() < CH) {
            hipEvent_t e;
            hipchk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
            ctx->a_ev_h2d.push_back(e);
          }
        }
        const uint8_t* const blob = dma ? ctx->a_dstage.p : ctx->a_stage.dev;
        int64_t prev_s0 = -1, prev_s1 = -1, prev_c = -1;   // prev_c: event of the last launched chunk
        auto job_end = [&](int64_t s1) { return all[(size_t)s1 - 1].j0 + all[(size_t)s1 - 1].nj; };
        for (int64_t c = 0; c < CH && first_neg == INT64_MAX; ++c) {
          const auto tp = now();
          const bool planned = CH == 1 || one_plan;   // (every chunk planned above)
          const int64_t s0 = planned ? nseg * c / CH : (int64_t)all.size();
          if (!planned) plan_chunk(c);
          const int64_t s1 = planned ? nseg * (c + 1) / CH : (int64_t)all.size();
          if (!planned && (s1 > seg_cap || so[s1] > total))   // (the bounds above hold by construction)
            raise(PE_ENOMEM, "aggregation staging bound exceeded");
          if (s1 == s0) continue;
          if (T == 1) pack(s0, s1, bad[0]);
          else PlanPool::get().run(T, [&](int t) { pack(s0 + (s1 - s0) * t / T, s0 + (s1 - s0) * (t + 1) / T, bad[t]); });
          t_pack += std::chrono::duration<double, std::milli>(now() - tp).count();
          first_neg = *std::min_element(bad, bad + T);
          if (first_neg != INT64_MAX) break;
          if (dma) {   // the chunk's bytes at the same offsets in the device copy (seg_off stays valid)
            hipchk(hipMemcpyAsync(ctx->a_dstage.p + so[s0], ctx->a_stage.p + so[s0], (size_t)(so[s1] - so[s0]),
                                  hipMemcpyHostToDevice, ctx->a_h2d),
                   "H2D aggregation chunk");
            hipchk(hipEventRecord(ctx->a_ev_h2d[(size_t)c], ctx->a_h2d), "event record");
            hipchk(hipStreamWaitEvent(ctx->stream, ctx->a_ev_h2d[(size_t)c], 0), "stream wait");
          }
          hipchk(pe::launch_pg_agg_segments(ctx->stream, mode, blob, ctx->a_segoff.dev + s0, s1 - s0, 0, od,
                                            n_jobs, nullptr, 0, nullptr, ak),
                 "launch pg_agg_segments");
          hipchk(hipEventRecord(ctx->a_ev[(size_t)c], ctx->stream), "event record");
          if (prev_s1 > prev_s0) {   // the previous chunk's outputs, while this chunk runs
            hipchk(hipEventSynchronize(ctx->a_ev[(size_t)prev_c]), "event sync");
            const int64_t ja = all[(size_t)prev_s0].j0, jb = job_end(prev_s1);
            parallel_for(jb - ja, [&](int64_t a, int64_t e) { unpack(ja + a, ja + e); });
            unpacked = jb;
          }
          prev_s0 = s0;
          prev_s1 = s1;
          prev_c = c;
        }
        nseg = (int64_t)all.size();
        hipchk(hipStreamSynchronize(ctx->stream), "sync pg_agg_segments");
        ctx->stats.agg_segments += nseg;
        ctx->stats.agg_wire_bytes += nseg > 0 ? so[nseg] : 0;
        for (int64_t k = 0; k < nseg; ++k) ctx->stats.agg_narrow_segments += all[(size_t)k].narrow ? 1 : 0;   // (also before an EINVAL:
                                                                             // launched chunks read the batch)
      }
      if (first_neg != INT64_MAX) raise(PE_EINVAL, "cont_req: negative request at index " + std::to_string(first_neg));
      const auto tt2 = now();
      if (T == 1) unpack(unpacked, n_jobs);
      else parallel_for(n_jobs - unpacked, [&](int64_t a, int64_t e) { unpack(unpacked + a, unpacked + e); });
      if (trace) {
        const auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
          return std::chrono::duration<double, std::milli>(b - a).count();
        };
        std::fprintf(stderr, "agg: J %lld segs %lld bytes %lld | plan %.4f ms, pack %.4f ms, pack+launch+wait %.4f ms "
                             "(launch call %.4f, flag wait %.4f), unpack %.4f ms\n",
                     (long long)n_jobs, (long long)nseg, (long long)total, ms(tt0, tt1), t_pack, ms(tt1, tt2), t_launch,
                     t_wait, ms(tt2, now()));
      }
    }
    const void* o1 = std::memchr(out_overflow, 1, (size_t)n_jobs);
    if (o1) {
      ctx->err = "int64 overflow in job " + std::to_string(static_cast<const uint8_t*>(o1) - out_overflow);
      return PE_EOVERFLOW;
    }
    return PE_OK;
  });
}

}  // namespace

extern "C" {

int pe_pg_min_resources(pe_ctx* ctx, int32_t mode, int64_t n_jobs, const int32_t* job_group_off,
                        const int32_t* min_member, const int32_t* group_replicas, const int32_t* group_cont_off,
                        const int64_t* cont_req, const uint8_t* cont_flags, int64_t* out_min_res,
                        uint8_t* out_present, int32_t* out_members, uint8_t* out_overflow) {
  return agg_call(ctx, mode, n_jobs, pe::AggKeys{4, 1}, 4, job_group_off, min_member, group_replicas, group_cont_off,
                  cont_req, cont_flags, out_min_res, out_present, out_members, out_overflow);
}

int pe_pg_min_resources_keys(pe_ctx* ctx, int32_t mode, int64_t n_jobs, int32_t n_keys, const int32_t* job_group_off,
                             const int32_t* min_member, const int32_t* group_replicas, const int32_t* group_cont_off,
                             const int64_t* cont_req, const uint32_t* cont_flags, int64_t* out_min_res,
                             uint16_t* out_present, int32_t* out_members, uint8_t* out_overflow) {
  if (n_keys < 1 || n_keys > PE_MAX_KEYS) {
    if (ctx) ctx->err = "n_keys must be in [1, " + std::to_string(PE_MAX_KEYS) + "]";
    return PE_EINVAL;
  }
  const pe::AggKeys ak{n_keys <= 4 ? 4 : n_keys <= 8 ? 8 : 16, 4};
  return agg_call(ctx, mode, n_jobs, ak, n_keys, job_group_off, min_member, group_replicas, group_cont_off, cont_req,
                  cont_flags, out_min_res, out_present, out_members, out_overflow);
}

// ------------------------------------------------------------------ fit mask

// The batch's dictionary, built once per upload and shared by every fit path's planning: per field
// (dims 0-3, field 4 = label need) the distinct values ascending and each job's index into them.
// One hashing pass per field (first-seen ids), then only the distinct values are sorted -- O(J)
// for the usual few-valued batches instead of five O(J log J) sorts.
struct BatchDict {
  static constexpr int F = pe::D + 1;
  std::vector<int64_t> vals[F];
  std::vector<uint32_t> rank[F];
};

extern "C++" {   // (this part of the file sits in the ABI's extern "C" block)
template <class V>
static void dict_field(int64_t n, V value, std::vector<int64_t>& vals, std::vector<uint32_t>& rank) {
  size_t cap = 64;
  while (cap < 2 * (size_t)n) cap *= 2;
  std::vector<int64_t> keys(cap);
  std::vector<uint32_t> ids(cap, UINT32_MAX);
  const size_t mask = cap - 1;
  vals.clear();
  rank.resize((size_t)n);
  for (int64_t j = 0; j < n; ++j) {
    const int64_t v = value(j);
    size_t h = (size_t)(((uint64_t)v * 0x9E3779B97F4A7C15ull) >> 32) & mask;
    while (ids[h] != UINT32_MAX && keys[h] != v) h = (h + 1) & mask;
    if (ids[h] == UINT32_MAX) {
      keys[h] = v;
      ids[h] = (uint32_t)vals.size();
      vals.push_back(v);
    }
    rank[j] = ids[h];
  }
  // order the distinct values: (value, first-seen id) pairs, LSD radix (11-bit digits, passes whose
  // digit is constant skipped) for many values, a comparison sort for few
  const size_t m = vals.size();
  std::vector<std::pair<uint64_t, uint32_t>> pr(m), tmp;
  for (size_t i = 0; i < m; ++i) pr[i] = {(uint64_t)vals[i] ^ (1ull << 63), (uint32_t)i};   // signed order
  if (m < 4096) {
    std::sort(pr.begin(), pr.end());
  } else {
    tmp.resize(m);
    uint64_t orv = 0, andv = ~0ull;
    for (const auto& e : pr) {
      orv |= e.first;
      andv &= e.first;
    }
    for (int sh = 0; sh < 64; sh += 11) {
      if ((((orv ^ andv) >> sh) & 0x7FF) == 0) continue;   // every value has the same digit here
      size_t cnt[2049] = {0};
      for (const auto& e : pr) ++cnt[((e.first >> sh) & 0x7FF) + 1];
      for (int b = 0; b < 2048; ++b) cnt[b + 1] += cnt[b];
      for (const auto& e : pr) tmp[cnt[(e.first >> sh) & 0x7FF]++] = e;
      pr.swap(tmp);
    }
  }
  std::vector<uint32_t> pos(m);
  for (size_t i = 0; i < m; ++i) {
    pos[pr[i].second] = (uint32_t)i;
    vals[i] = (int64_t)(pr[i].first ^ (1ull << 63));
  }
  for (int64_t j = 0; j < n; ++j) rank[j] = pos[rank[j]];
}
}  // extern "C++"

static void build_dict(BatchDict& bd, int64_t n_jobs, const int64_t* req, const uint32_t* need) {
  auto field = [&](int f) {
    if (f < pe::D)
      dict_field(n_jobs, [&](int64_t j) { return req[j * pe::D + f]; }, bd.vals[f], bd.rank[f]);
    else
      dict_field(n_jobs, [&](int64_t j) { return (int64_t)(need ? need[j] : 0u); }, bd.vals[f], bd.rank[f]);
  };
  if (n_jobs < 16384) {
    for (int f = 0; f < BatchDict::F; ++f) field(f);
    return;
  }
  // large batches: the five independent fields on five threads (the upload is on the batch's path)
  PlanPool::get().run(BatchDict::F, [&](int f) { field(f); });
}

// Dictionary codes of one batch (pe_kernels.h, CodeSpec): per dimension the sorted distinct request
// values, per job their ranks packed with guard bits; label needs must form an inclusion chain.
// Returns false when the batch does not fit the 32-bit code word (the compare paths take it).
static bool build_codes(pe_ctx* ctx, int64_t n_jobs, const BatchDict& bd) {
  if (n_jobs == 0) return false;
  const std::vector<int64_t>* vals = bd.vals;
  for (int d = 0; d < pe::D; ++d)
    if ((int)vals[d].size() >= pe::CODE_MAXV) return false;
  if ((int)bd.vals[4].size() >= pe::CODE_MAXV) return false;
  std::vector<uint32_t> needs;
  for (int64_t v : bd.vals[4]) needs.push_back((uint32_t)v);
  std::sort(needs.begin(), needs.end(), [](uint32_t a, uint32_t b) {
    return __builtin_popcount(a) != __builtin_popcount(b) ? __builtin_popcount(a) < __builtin_popcount(b) : a < b;
  });
  // need dictionary index -> position in the inclusion chain
  std::vector<uint32_t> need_pos(bd.vals[4].size());
  for (size_t i = 0; i < bd.vals[4].size(); ++i)
    need_pos[i] = (uint32_t)(std::find(needs.begin(), needs.end(), (uint32_t)bd.vals[4][i]) - needs.begin());
  if ((int)needs.size() >= pe::CODE_MAXV) return false;
  for (size_t i = 0; i + 1 < needs.size(); ++i)
    if ((needs[i] & needs[i + 1]) != needs[i]) return false;   // not a chain under inclusion
  pe::CodeSpec sp{};
  int therm_bits = 0;
  for (int f = 0; f < pe::CODE_FIELDS; ++f) therm_bits += f < pe::D ? (int)vals[f].size() : (int)needs.size();
  // thermometer fields (one bit per distinct value) when they fit 31 bits -- bit 31 stays free for
  // the never-fitting padding jobs -- else log-width SWAR fields with guard bits
  sp.therm = (ctx->fit_path_mask & PATH_NO_THERM) == 0 && therm_bits <= 31 ? 1 : 0;
  int off = 0;
  for (int f = 0; f < pe::CODE_FIELDS; ++f) {
    const int k = f < pe::D ? (int)vals[f].size() : (int)needs.size();
    const int bits = 32 - __builtin_clz((unsigned)k);
    sp.nvals[f] = k;
    sp.width[f] = sp.therm ? k : bits + 1;
    sp.off[f] = off;
    off += sp.width[f];
  }
  if (off > 32) return false;
  sp.guard = 0;
  if (!sp.therm)
    for (int f = 0; f < pe::CODE_FIELDS; ++f) sp.guard |= 1u << (sp.off[f] + sp.width[f] - 1);
  const int64_t Jp = round_up(n_jobs, pe::FC_JT);
  // padding jobs never fit: SWAR code M (every field fails); thermometer ~Y with bit 31 cleared
  std::vector<uint32_t> jc((size_t)Jp, sp.therm ? ~(1u << 31) : sp.guard);
  for (int64_t j = 0; j < n_jobs; ++j) {
    uint32_t c = 0;
    for (int d = 0; d < pe::D; ++d) c |= (bd.rank[d][j] + 1) << sp.off[d];
    c |= (need_pos[bd.rank[4][j]] + 1) << sp.off[4];
    if (sp.therm) {
      uint32_t y = 0;   // one bit per field: rank c <=> bit c-1
      for (int f = 0; f < pe::CODE_FIELDS; ++f) {
        const uint32_t r = (c >> sp.off[f]) & ((1u << sp.width[f]) - 1);   // ranks < 2^width here
        y |= 1u << (sp.off[f] + r - 1);
      }
      c = ~y;
    }
    jc[j] = c;
  }
  std::vector<int64_t> vt((size_t)pe::D * pe::CODE_MAXV, INT64_MAX);
  for (int d = 0; d < pe::D; ++d) std::copy(vals[d].begin(), vals[d].end(), vt.begin() + (size_t)d * pe::CODE_MAXV);
  std::vector<uint32_t> nt((size_t)pe::CODE_MAXV, 0xFFFFFFFFu);
  std::copy(needs.begin(), needs.end(), nt.begin());
  ctx->code = sp;
  ctx->code_Jp = Jp;
  ctx->node_stride = round_up(std::max<int64_t>(ctx->Ns, 1), 64 * pe::FC_CH);
  hipchk(ctx->code_vals.ensure(vt.size()), "alloc code vals");
  hipchk(ctx->code_needs.ensure(nt.size()), "alloc code needs");
  hipchk(ctx->code_jobs.ensure(jc.size()), "alloc code jobs");
  hipchk(ctx->code_x.ensure((size_t)ctx->node_stride), "alloc code x");
  hipchk(hipMemcpyAsync(ctx->code_vals.p, vt.data(), vt.size() * 8, hipMemcpyHostToDevice, ctx->stream), "H2D vals");
  hipchk(hipMemcpyAsync(ctx->code_needs.p, nt.data(), nt.size() * 4, hipMemcpyHostToDevice, ctx->stream), "H2D needs");
  hipchk(hipMemcpyAsync(ctx->code_jobs.p, jc.data(), jc.size() * 4, hipMemcpyHostToDevice, ctx->stream), "H2D codes");
  return true;
}

// Bit planes of one batch (pe_kernels.h, PlaneSpec): one plane per distinct request value of each
// dimension and per distinct label need, each job selecting five.  Any int64 values and any need
// sets.  A batch with more than PL_MAX distinct (dimension, value) pairs is split into plane sets
// (row-major layout only, at most PL_MAX_SETS); returns false when it cannot be held either way.
constexpr int PL_MAX_SETS = 256;
constexpr int64_t PL_SETS_BYTES = int64_t(2) << 30;   // planes of all sets (4 MiB per set at 1M nodes)

static bool build_planes(pe_ctx* ctx, int64_t n_jobs, const BatchDict& bd, bool allow_sets) {
  if (n_jobs == 0) return false;
  constexpr int F = pe::D + 1;
  const std::vector<int64_t>* vals = bd.vals;
  int64_t off[F], P = 0;
  for (int f = 0; f < F; ++f) {
    off[f] = P;
    P += (int64_t)vals[f].size();
  }
  if (P > pe::PL_MAX && !allow_sets) return false;
  // pair id (global over the fields) of each job's five selections (the plane-set path)
  std::vector<int32_t> pid;
  if (P > pe::PL_MAX) {
    pid.resize((size_t)n_jobs * F);
    parallel_for(n_jobs, [&](int64_t j0, int64_t j1) {
      for (int64_t j = j0; j < j1; ++j)
        for (int f = 0; f < F; ++f) pid[(size_t)j * F + f] = (int32_t)(off[f] + bd.rank[f][j]);
    });
  }
  auto pair_spec = [&](int64_t p, int& kind, int64_t& val) {
    int f = F - 1;
    while (off[f] > p) --f;
    kind = f;
    val = vals[f][(size_t)(p - off[f])];
  };
  // field f's plane index sits at bits 0/7/14/21 (dims) and 32 (need) as 4 x index (register offset)
  auto field_shift = [](int f) { return f < pe::D ? 7 * f : 32; };
  ctx->pl_nblk = (std::max<int64_t>(ctx->Ns, 1) + pe::PL_BLK - 1) / pe::PL_BLK;
  // row-major mask pitch in blocks (PE_ROW_PITCH_BLOCKS: a study knob; the words past nblk are
  // never written)
  static const int64_t pitch_env = std::getenv("PE_ROW_PITCH_BLOCKS") ? std::atoll(std::getenv("PE_ROW_PITCH_BLOCKS")) : 0;
  ctx->pl_pitch = std::max(ctx->pl_nblk, pitch_env);
  // phases of a set of J jobs: one wave per SIMD (1024 on 256 CUs) = nblk x R; codes phase-major.
  // (Padding the row to 1024 / R blocks, i.e. an aligned 1 MiB store window, was measured no
  // faster: profiles/r5c_row_pitch.txt.)
  // PE_PL_WAVES / PE_PL_JPW (A/B studies): a fixed wave count, or R from a jobs-per-wave target
  static const int64_t pl_waves = std::getenv("PE_PL_WAVES") ? std::max(1ll, std::atoll(std::getenv("PE_PL_WAVES"))) : 1024;
  static const int64_t pl_jpw = std::getenv("PE_PL_JPW") ? std::max(1ll, std::atoll(std::getenv("PE_PL_JPW"))) : 0;
  auto phases = [&](int64_t J, int64_t& R, int64_t& Jr) {
    R = ctx->pl_rows ? std::min<int64_t>(J, std::max<int64_t>(1, pl_waves / ctx->pl_nblk)) : 1;
    if (ctx->pl_rows && pl_jpw) R = std::min<int64_t>(J, std::max<int64_t>(R, (J + pl_jpw - 1) / pl_jpw));
    Jr = ctx->pl_rows ? ((J + R - 1) / R + 3) / 4 * 4 : J;   // = the kernel's phase stride
  };
  std::vector<uint64_t> jc;
  ctx->pl_sets.clear();
  ctx->pl_cnt_row.clear();
  if (P <= pe::PL_MAX) {   // one set: every pair is a plane
    pe::PlaneSpec sp{};
    for (int64_t p = 0; p < P; ++p) {
      int kind;
      pair_spec(p, kind, sp.val[sp.n]);
      sp.kind[sp.n++] = kind;
    }
    ctx->plane = sp;
    hipchk(ctx->pl_specs_d.ensure(1), "alloc plane spec");
    hipchk(hipMemcpyAsync(ctx->pl_specs_d.p, &ctx->plane, sizeof(pe::PlaneSpec), hipMemcpyHostToDevice, ctx->stream),
           "H2D plane spec");
    int64_t R, Jr;
    phases(n_jobs, R, Jr);
    // each job's code straight into its phase-major slot (row-major kernel) or job order
    jc.assign((size_t)(ctx->pl_rows ? R * Jr : n_jobs), 0);
    parallel_for(n_jobs, [&](int64_t j0, int64_t j1) {
      for (int64_t j = j0; j < j1; ++j) {
        uint64_t c = 0;
        for (int f = 0; f < F; ++f) c |= (uint64_t)(4 * (off[f] + bd.rank[f][j])) << field_shift(f);
        jc[ctx->pl_rows ? (size_t)((j % R) * Jr + j / R) : (size_t)j] = c;
      }
    });
    ctx->pl_R = R;
    ctx->pl_counts_n = R * Jr;
  } else {
    if (!allow_sets || !ctx->pl_rows || n_jobs >= (int64_t(1) << 24)) return false;
    // Sets: jobs ordered by their selections, the field with the most distinct values first, then
    // swept greedily; a set closes when the next job would take it past PL_MAX planes.
    int ford[F];
    for (int f = 0; f < F; ++f) ford[f] = f;
    std::sort(ford, ford + F, [&](int x, int y) { return vals[x].size() > vals[y].size(); });
    std::vector<int64_t> order((size_t)n_jobs);
    for (int64_t j = 0; j < n_jobs; ++j) order[j] = j;
    std::sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
      for (int f : ford)
        if (pid[(size_t)x * F + f] != pid[(size_t)y * F + f]) return pid[(size_t)x * F + f] < pid[(size_t)y * F + f];
      return x < y;
    });
    std::vector<int32_t> stamp((size_t)P, -1), local((size_t)P, 0);
    std::vector<std::vector<int64_t>> members;
    std::vector<std::vector<uint64_t>> codes;
    std::vector<pe::PlaneSpec> specs;
    int cur = -1, ncur = 0;
    for (int64_t j : order) {
      int add = 0;
      for (int f = 0; f < F; ++f) add += cur < 0 || stamp[pid[(size_t)j * F + f]] != cur;
      if (cur < 0 || ncur + add > pe::PL_MAX) {
        if ((int)specs.size() == PL_MAX_SETS ||
            (int64_t)(specs.size() + 1) * ctx->pl_nblk * pe::PL_MAX * 64 * pe::PL_R * 4 > PL_SETS_BYTES)
          return false;
        ++cur;
        ncur = 0;
        members.emplace_back();
        codes.emplace_back();
        specs.push_back(pe::PlaneSpec{});
      }
      uint64_t c = (uint64_t)j << 40;   // the job's mask row
      for (int f = 0; f < F; ++f) {
        const int32_t p = pid[(size_t)j * F + f];
        if (stamp[p] != cur) {
          stamp[p] = cur;
          local[p] = ncur++;
          pe::PlaneSpec& sp = specs[cur];
          int kind;
          pair_spec(p, kind, sp.val[sp.n]);
          sp.kind[sp.n++] = kind;
        }
        c |= (uint64_t)(4 * local[p]) << field_shift(f);
      }
      members[cur].push_back(j);
      codes[cur].push_back(c);
    }
    // each set's jobs in row order: the sweep's stores in flight then stay in a narrow band of
    // rows (the partition order scattered them over the whole mask)
    for (size_t t = 0; t < members.size(); ++t) {
      std::vector<size_t> ix(members[t].size());
      for (size_t i = 0; i < ix.size(); ++i) ix[i] = i;
      std::sort(ix.begin(), ix.end(), [&](size_t x, size_t y) { return members[t][x] < members[t][y]; });
      std::vector<int64_t> m2(ix.size());
      std::vector<uint64_t> c2(ix.size());
      for (size_t i = 0; i < ix.size(); ++i) {
        m2[i] = members[t][ix[i]];
        c2[i] = codes[t][ix[i]];
      }
      members[t].swap(m2);
      codes[t].swap(c2);
    }
    // one launch sweeps every set: the phase count is common (one wave per SIMD over nblk blocks)
    const int64_t R = std::max<int64_t>(1, 1024 / ctx->pl_nblk);
    int64_t total = 0;
    std::vector<int64_t> meta;
    for (size_t t = 0; t < specs.size(); ++t) {
      pe_ctx::PlaneSet st{specs[t], (int64_t)members[t].size(), R, 0, total};
      st.Jr = ((st.J + R - 1) / R + 3) / 4 * 4;
      total += R * st.Jr;
      ctx->pl_sets.push_back(st);
      meta.insert(meta.end(), {st.off, st.J, st.Jr});
    }
    hipchk(ctx->pl_specs_d.ensure(specs.size()), "alloc plane specs");
    hipchk(ctx->pl_meta_d.ensure(meta.size()), "alloc plane set meta");
    hipchk(hipMemcpyAsync(ctx->pl_specs_d.p, specs.data(), specs.size() * sizeof(pe::PlaneSpec),
                          hipMemcpyHostToDevice, ctx->stream),
           "H2D plane specs");
    hipchk(hipMemcpyAsync(ctx->pl_meta_d.p, meta.data(), meta.size() * 8, hipMemcpyHostToDevice, ctx->stream),
           "H2D plane set meta");
    hipchk(hipStreamSynchronize(ctx->stream), "sync plane sets");   // the host vectors die here
    jc.assign((size_t)total, 0);
    ctx->pl_cnt_row.assign((size_t)total, -1);
    for (size_t t = 0; t < specs.size(); ++t) {
      const pe_ctx::PlaneSet& st = ctx->pl_sets[t];
      for (int64_t i = 0; i < st.J; ++i) {
        const size_t k = (size_t)(st.off + (i % st.R) * st.Jr + i / st.R);
        jc[k] = codes[t][i];
        ctx->pl_cnt_row[k] = members[t][i];
      }
    }
    ctx->pl_R = 1;
    ctx->pl_counts_n = total;
  }
  hipchk(ctx->planes.ensure((size_t)std::max<size_t>(ctx->pl_sets.size(), 1) * ctx->pl_nblk * pe::PL_MAX * 64 *
                            pe::PL_R),
         "alloc planes");
  hipchk(ctx->plane_jobs.ensure(jc.size()), "alloc plane jobs");
  hipchk(hipMemcpyAsync(ctx->plane_jobs.p, jc.data(), jc.size() * 8, hipMemcpyHostToDevice, ctx->stream),
         "H2D plane jobs");
  return true;
}

// LDS digit planes of one batch (pe_kernels.h LdsSpec): per dimension with >= 2 distinct values a
// digit field of L levels (chosen with the node-block size W to minimise plane reads per job within
// the LDS budget), dimensions with one value folded into the need planes, one plane per distinct
// need -- or, with single-level fields crossed into them, one per (need, crossed values): a job then
// reads one plane for its labels and those fields.  Returns false when no configuration fits 160 KiB
// of LDS (the other paths take the batch).  PE_LDS_W=1|2|4 forces the block size, PE_LDS_MAXL=1..4
// caps the levels, PE_LDS_CROSS=0 crosses nothing (tuning / tests).
static bool build_lds(pe_ctx* ctx, int64_t n_jobs, const BatchDict& bd) {
  if (n_jobs == 0 || ctx->Ns == 0) return false;
  const std::vector<int64_t>* vals = bd.vals;
  std::vector<uint32_t> needs;
  for (int64_t v : bd.vals[4]) needs.push_back((uint32_t)v);   // ascending
  if ((int)needs.size() > pe::LD_MAXNEED) return false;
  pe::LdsSpec sp{};
  int fdim[pe::LD_MAXF];
  for (int d = 0; d < pe::D; ++d) {
    if (vals[d].size() == 1) {
      sp.fold_dim[sp.nfold] = d;
      sp.fold_val[sp.nfold++] = vals[d][0];
    } else {
      fdim[sp.nf++] = d;
    }
  }
  // planes of a field with m values at L levels (lower levels base B, top level whatever is left):
  // level 0 has B planes, levels 1 .. L-2 B + 1 (their GE(c + 1) is read too), the top m / B^(L-1) + 2
  auto plan = [](int64_t m, int L, int64_t& B) -> int64_t {
    if (L == 1) {
      B = m;
      return m;
    }
    int64_t best = INT64_MAX;
    for (int64_t b = 2; b <= m; ++b) {
      int64_t low = 1;
      for (int k = 1; k < L; ++k) low *= b;
      const int64_t T = m / low + 1;
      const int64_t p = (T + 1) + (L - 2) * (b + 1) + b;
      if (p < best) {
        best = p;
        B = b;
      }
      if (low / b * b * b > 4 * m + 4) break;   // past the square-ish optimum
    }
    return best;
  };
  int maxl = pe::LD_MAXL;
  if (const char* e = std::getenv("PE_LDS_MAXL")) maxl = std::max(1, std::min(pe::LD_MAXL, std::atoi(e)));
  int forced_w = 0;
  if (const char* e = std::getenv("PE_LDS_W")) forced_w = std::atoi(e);
  const int64_t nneed = (int64_t)needs.size();
  bool cross = true;
  if (const char* e = std::getenv("PE_LDS_CROSS")) cross = std::atoi(e) != 0;
  int bestW = 0, bestL[pe::LD_MAXF] = {1, 1, 1, 1}, bestX = 0;   // bestX: bit i = field i crossed
  int64_t bestB[pe::LD_MAXF] = {0, 0, 0, 0};
  double bestCost = 1e300;
  for (int W : {4, 2, 1}) {
    if (forced_w && W != forced_w) continue;
    const int64_t budget = 163840 / (256 * W);
    int combos = 1;
    for (int i = 0; i < sp.nf; ++i) combos *= maxl;
    for (int cix = 0; cix < combos; ++cix) {
      int L[pe::LD_MAXF];
      int64_t B[pe::LD_MAXF], P[pe::LD_MAXF];
      bool ok = true;
      for (int i = 0, x = cix; i < sp.nf; ++i, x /= maxl) {
        L[i] = 1 + x % maxl;
        const int64_t m = (int64_t)vals[fdim[i]].size();
        if (L[i] > 1 && m < 4) L[i] = 1;
        if (L[i] == 4 && W == 1) ok = false;     // four-level kernels exist for W >= 2 only
        P[i] = plan(m, L[i], B[i]);
      }
      if (!ok) continue;
      // crossed sets: the k single-level fields with the fewest values, k = 0 .. all of them
      int one[pe::LD_MAXF], n1 = 0;
      for (int i = 0; i < sp.nf; ++i)
        if (L[i] == 1) one[n1++] = i;
      std::sort(one, one + n1, [&](int a, int b) { return vals[fdim[a]].size() < vals[fdim[b]].size(); });
      // a crossing must not cost the second workgroup per CU (LDS <= 80 KiB) the uncrossed plan has:
      // store-bound batches need the waves more than the plane read they save ("many": R 4 -> 2, 90 KB,
      // 2.32 -> 2.68 ms when crossing pushed the LDS past half the CU's)
      int64_t planes0 = nneed;
      for (int i = 0; i < sp.nf; ++i) planes0 += P[i];
      const int64_t half = 81920 / (256 * W);
      for (int k = 0; k <= (cross ? n1 : 0); ++k) {
        int xs = 0;
        int64_t xprod = 1;
        for (int t = 0; t < k; ++t) {
          xs |= 1 << one[t];
          xprod *= (int64_t)vals[fdim[one[t]]].size();
        }
        int64_t planes = nneed * xprod, reads = 1, entries = 0, nfk = 0;
        for (int i = 0; i < sp.nf; ++i) {
          if (xs >> i & 1) continue;
          planes += P[i];
          reads += 2 * L[i] - 1;
          entries += L[i];
          ++nfk;
        }
        if (entries > pe::LD_NEED_SLOT || planes > budget || planes > 65535) continue;
        if (k > 0 && planes > half && planes0 <= half) continue;
        // per job and 8192 nodes, in CU cycles: LDS plane reads (b128 / b64 / read2st64_b64: 4 per
        // KiB, b32: 8) -- the kernel's bound -- plus its VALU at ~0.6 CU cycles per wave instruction:
        // per entry a readlane half and an address, ~6 fixed, and the three-input combines (2 per
        // extra level and word, 4 per 8192 nodes whatever W)
        const double valu = (4.0 / W) * (1.5 * (double)entries + 6.0) + 4.0 * (double)(reads - 1 - nfk + nfk / 2);
        const double cost = reads * (W == 1 ? 8.0 : 4.0) + 0.625 * valu;
        if (cost < bestCost - 1e-9) {
          bestCost = cost;
          bestW = W;
          bestX = xs;
          for (int i = 0; i < sp.nf; ++i) {
            bestL[i] = L[i];
            bestB[i] = B[i];
          }
        }
      }
    }
  }
  if (!bestW) return false;
  // fields in the kernel's order: four-level first, then three-, two- and single-level; the crossed
  // fields last (they keep a rank row but no digit planes)
  const int nx = __builtin_popcount(bestX);
  {
    int ord[pe::LD_MAXF] = {0, 1, 2, 3};
    auto key = [&](int x) { return (bestX >> x & 1) ? 0 : bestL[x]; };
    std::stable_sort(ord, ord + sp.nf, [&](int x, int y) { return key(x) > key(y); });
    int d2[pe::LD_MAXF], L2[pe::LD_MAXF];
    int64_t B2[pe::LD_MAXF];
    for (int i = 0; i < sp.nf; ++i) {
      d2[i] = fdim[ord[i]];
      L2[i] = bestL[ord[i]];
      B2[i] = bestB[ord[i]];
    }
    for (int i = 0; i < sp.nf; ++i) {
      fdim[i] = d2[i];
      bestL[i] = L2[i];
      bestB[i] = B2[i];
    }
  }
  sp.nf -= nx;
  int shape[4] = {0, 0, 0, 0};
  for (int i = 0; i < sp.nf; ++i) ++shape[4 - bestL[i]];
  // level specs, plane bases
  int32_t p = 0;
  int64_t voff = 0;
  std::vector<int64_t> allv;
  for (int i = 0; i < sp.nf; ++i) {
    const int64_t m = (int64_t)vals[fdim[i]].size(), B = bestB[i];
    const int L = bestL[i];
    sp.dim[i] = fdim[i];
    sp.L[i] = L;
    sp.voff[i] = voff;
    sp.m[i] = m;
    allv.insert(allv.end(), vals[fdim[i]].begin(), vals[fdim[i]].end());
    voff += m;
    for (int k = 0; k < L; ++k) {
      const bool top = k == L - 1;
      int64_t dv = 1;
      for (int t = 0; t < k; ++t) dv *= B;
      sp.div[i][k] = (uint32_t)dv;
      sp.mod[i][k] = top ? 0u : (uint32_t)B;
      if (L == 1) {
        sp.vlo[i][k] = 1;
        sp.nv[i][k] = (int32_t)m;
      } else {
        sp.vlo[i][k] = 0;
        sp.nv[i][k] = (int32_t)(top ? m / dv + 2 : (k == 0 ? B : B + 1));
      }
      sp.pbase[i][k] = p;
      p += sp.nv[i][k];
    }
  }
  sp.nx = nx;
  sp.xprod = 1;
  for (int x = 0; x < nx; ++x) {   // crossed fields: rank rows and values after the digit fields
    const int i = sp.nf + x;
    const int64_t m = (int64_t)vals[fdim[i]].size();
    sp.dim[i] = fdim[i];
    sp.L[i] = 1;
    sp.voff[i] = voff;
    sp.m[i] = m;
    allv.insert(allv.end(), vals[fdim[i]].begin(), vals[fdim[i]].end());
    voff += m;
    sp.xstride[x] = sp.xprod;
    sp.xprod *= (int32_t)m;
  }
  sp.need_pbase = p;
  sp.nneed = (int32_t)nneed;
  for (int64_t i = 0; i < nneed; ++i) sp.needs[i] = needs[i];
  sp.nplanes = p + (int32_t)(nneed * sp.xprod);
  // geometry: W words per lane, blocks of 2048 W nodes, R job phases for an even spread over the CUs
  const int W = bestW;
  const int64_t S = 2048 * W;
  const int64_t nblk = (ctx->Ns + S - 1) / S;
  const int64_t lds_bytes = (int64_t)sp.nplanes * S / 8;
  const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(2, 163840 / std::max<int64_t>(lds_bytes, 1)));
  const int64_t slots = (int64_t)ctx->num_cu * per_cu;
  // job phases R: every workgroup builds its block's planes before its share (1/R) of the jobs, so
  // minimise rounds(R) x (prologue + 1/R) -- the prologue being ~2 % of one block's full job sweep
  int64_t R = 1;
  double best_t = 1e300;
  for (int64_t r = 1; r <= 64 && (r == 1 || 16 * r <= n_jobs); ++r) {
    const int64_t rounds = (nblk * r + slots - 1) / slots;
    const double t = (double)rounds * (0.02 + 1.0 / (double)r);
    if (t < best_t - 1e-9) {
      best_t = t;
      R = r;
    }
  }
  if (const char* ev = std::getenv("PE_LDS_R")) R = std::max<int64_t>(1, std::atoll(ev));
  const int64_t Tmax = ((n_jobs + R - 1) / R + 15) / 16;
  const int64_t Tpad = round_up(std::max<int64_t>(Tmax, 1), 16);
  // job codes: u16 plane indices, per job first
  std::vector<uint16_t> jc((size_t)n_jobs * pe::LD_CODE, 0);
  parallel_for(n_jobs, [&](int64_t j0, int64_t j1) {
  for (int64_t j = j0; j < j1; ++j) {
    uint16_t* c = jc.data() + (size_t)j * pe::LD_CODE;
    for (int i = 0; i < sp.nf; ++i) {
      const int64_t rank = (int64_t)bd.rank[fdim[i]][j] + 1;
      const int o = pe::lds_field_off(i, shape[0], shape[1], shape[2]);
      if (sp.L[i] == 1) {
        c[o] = (uint16_t)(sp.pbase[i][0] + rank - 1);
      } else {
        int64_t x = rank;
        for (int k = 0; k < sp.L[i]; ++k) {
          const int64_t digit = sp.mod[i][k] ? x % sp.mod[i][k] : x;
          x = sp.mod[i][k] ? x / sp.mod[i][k] : 0;
          c[o + k] = (uint16_t)(sp.pbase[i][k] + digit);
        }
      }
    }
    int64_t xc = 0;   // the job's crossed values (0-based value index: the node's rank must exceed it)
    for (int x = 0; x < sp.nx; ++x) xc += (int64_t)bd.rank[fdim[sp.nf + x]][j] * sp.xstride[x];
    c[pe::lds_need_slot(shape[0], shape[1], shape[2], shape[3])] =
        (uint16_t)(sp.need_pbase + bd.rank[4][j] * sp.xprod + xc);
  }
  });
  // slot (r * 16 + w) * Tpad + t = job r + R (w + 16 t), the t-th of wave w's run in phase r (the
  // kernel's consumption order); each slot's job in lds_rows for the counts
  std::vector<uint16_t> codes((size_t)(R * 16 * Tpad * pe::LD_CODE), 0);
  std::vector<uint32_t> rows((size_t)(R * 16 * Tpad), ~0u);
  {
    int64_t pos = 0;
    for (int64_t v = 0; v < R * 16; ++v) {
      const int64_t r = v / 16, w = v % 16, j0 = r + R * w;
      const int64_t T = j0 < n_jobs ? (n_jobs - j0 + 16 * R - 1) / (16 * R) : 0;
      for (int64_t t = 0; t < T; ++t, ++pos) {
        const uint32_t j = (uint32_t)(j0 + 16 * R * t);
        std::memcpy(codes.data() + (size_t)((v * Tpad + t) * pe::LD_CODE), jc.data() + (size_t)j * pe::LD_CODE,
                    pe::LD_CODE * 2);
        rows[(size_t)(v * Tpad + t)] = j;
      }
    }
    if (pos != n_jobs) raise(PE_EINVAL, "lds: run lengths do not cover the batch");
  }
  if (std::getenv("PE_LDS_DEBUG")) {   // diagnostics: the chosen configuration
    std::fprintf(stderr, "lds: W %d nblk %lld R %lld planes %d need %d fold %d cross %d x %d |", W, (long long)nblk,
                 (long long)R, sp.nplanes, sp.nneed, sp.nfold, sp.nx, sp.xprod);
    for (int i = 0; i < sp.nf; ++i)
      std::fprintf(stderr, " dim %d m %lld L %d B %u", sp.dim[i], (long long)sp.m[i], sp.L[i], sp.mod[i][0]);
    std::fprintf(stderr, "\n");
  }
  ctx->lds = sp;
  ctx->lds_W = W;
  for (int i = 0; i < 4; ++i) ctx->lds_shape[i] = shape[i];
  ctx->lds_nblk = nblk;
  ctx->lds_R = R;
  ctx->lds_Tpad = Tpad;
  // (+ the kernel's per-block work-unit counters, zeroed with the slots every step)
  hipchk(ctx->lds_slots.ensure((size_t)R * 16 * Tpad + (size_t)ctx->lds_nblk), "alloc count slots");
  hipchk(ctx->lds_rows.ensure((size_t)R * 16 * Tpad), "alloc count rows");
  hipchk(hipMemcpyAsync(ctx->lds_rows.p, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, ctx->stream),
         "H2D lds rows");
  ctx->lds_npad = nblk * S;
  ctx->lds_pitch = nblk * S / 64;
  hipchk(ctx->lds_spec_d.ensure(1), "alloc lds spec");
  hipchk(ctx->lds_vals.ensure(std::max<size_t>(allv.size(), 1)), "alloc lds vals");
  hipchk(ctx->lds_codes.ensure(codes.size()), "alloc lds codes");
  hipchk(ctx->lds_ranks.ensure((size_t)std::max(sp.nf + sp.nx, 1) * ctx->lds_npad), "alloc lds ranks");
  hipchk(ctx->lds_aux.ensure((size_t)2 * ctx->lds_npad), "alloc lds aux");
  hipchk(hipMemcpyAsync(ctx->lds_spec_d.p, &ctx->lds, sizeof(pe::LdsSpec), hipMemcpyHostToDevice, ctx->stream),
         "H2D lds spec");
  if (!allv.empty())
    hipchk(hipMemcpyAsync(ctx->lds_vals.p, allv.data(), allv.size() * 8, hipMemcpyHostToDevice, ctx->stream),
           "H2D lds vals");
  hipchk(hipMemcpyAsync(ctx->lds_codes.p, codes.data(), codes.size() * 2, hipMemcpyHostToDevice, ctx->stream),
         "H2D lds codes");
  hipchk(hipStreamSynchronize(ctx->stream), "sync lds upload");   // the host vectors die here
  return true;
}

static void fit_upload(pe_ctx* ctx, int64_t n_jobs, const int64_t* req, const uint32_t* need) {
  if (n_jobs < 0) raise(PE_EINVAL, "n_jobs < 0");
  if (!ctx->loaded) raise(PE_ESTATE, "no inventory loaded");
  if (n_jobs > 0) {
    need_ptr(req, "req");
    check_req(req, n_jobs, "req");
  }
  const int64_t Jp = round_up(std::max<int64_t>(n_jobs, 1), pe::FM_JT);
  ctx->fit_J = n_jobs;
  ctx->fit_Jp = Jp;
  ctx->Wn = (ctx->Ns + 63) / 64;
  ctx->Wt = (ctx->Wn + 3) / 4;
  // one bit-plane set (register planes) > LDS digit planes > bit-plane sets > coded > int32 > int64
  const bool planes_ok = ctx->fit_path_mask & PATH_PLANES;
  ctx->fit_path = -1;
  if (n_jobs > 0 && (ctx->fit_path_mask & (PATH_PLANES | PATH_LDS | PATH_CODED))) {
    BatchDict bd;
    build_dict(bd, n_jobs, req, need);
    if (planes_ok && build_planes(ctx, n_jobs, bd, false)) ctx->fit_path = 3;
    else if ((ctx->fit_path_mask & PATH_LDS) && build_lds(ctx, n_jobs, bd)) ctx->fit_path = 4;
    else if (planes_ok && build_planes(ctx, n_jobs, bd, true)) ctx->fit_path = 3;
    else if ((ctx->fit_path_mask & PATH_CODED) && build_codes(ctx, n_jobs, bd)) ctx->fit_path = 2;
  }
  if (ctx->fit_path < 0) {
    // compare paths.  Exact 32-bit form: per dim the shift that brings the largest request below
    // 2^31, valid only if 2^shift divides every request of the batch in that dim
    bool use32 = true;
    for (int d = 0; d < pe::D && use32; ++d) {
      int64_t mx = 0, orv = 0;
      for (int64_t j = 0; j < n_jobs; ++j) {
        mx = std::max(mx, req[j * pe::D + d]);
        orv |= req[j * pe::D + d];
      }
      int sh = 0;
      while (sh < 62 && (mx >> sh) > (int64_t)INT32_MAX) ++sh;
      if (orv & ((int64_t(1) << sh) - 1)) use32 = false;
      ctx->fit_shift[d] = sh;
    }
    ctx->fit32 = use32 && (ctx->fit_path_mask & PATH_I32);
    ctx->fit_path = ctx->fit32 ? 1 : 0;
    if (ctx->fit32) {
      std::vector<pe::ReqRec32> r32((size_t)Jp);
      for (int64_t j = 0; j < Jp; ++j) {
        std::memset(&r32[j], 0, sizeof(pe::ReqRec32));
        for (int d = 0; d < pe::D; ++d)
          r32[j].q[d] = j < n_jobs ? (int32_t)(req[j * pe::D + d] >> ctx->fit_shift[d]) : INT32_MAX;
        r32[j].need = j < n_jobs ? (need ? need[j] : 0u) : 0xFFFFFFFFu;
      }
      hipchk(ctx->fit_jobs32.ensure(Jp), "alloc fit jobs32");
      hipchk(ctx->res32.ensure((size_t)pe::D * ctx->stride), "alloc res32");
      hipchk(hipMemcpyAsync(ctx->fit_jobs32.p, r32.data(), Jp * sizeof(pe::ReqRec32), hipMemcpyHostToDevice,
                            ctx->stream),
             "H2D fit jobs32");
      hipchk(hipStreamSynchronize(ctx->stream), "sync fit jobs32");   // the host vector dies here
    } else {
      std::vector<ReqRec> recs((size_t)Jp);
      for (int64_t j = 0; j < Jp; ++j) {
        if (j < n_jobs) fill_req(recs[j], req + j * pe::D, need ? need[j] : 0u);
        else {
          const int64_t never[pe::D] = {INT64_MAX, INT64_MAX, INT64_MAX, INT64_MAX};
          fill_req(recs[j], never, 0xFFFFFFFFu);
        }
      }
      hipchk(ctx->fit_jobs.ensure(Jp), "alloc fit jobs");
      hipchk(hipMemcpyAsync(ctx->fit_jobs.p, recs.data(), Jp * sizeof(ReqRec), hipMemcpyHostToDevice, ctx->stream),
             "H2D fit jobs");
      hipchk(hipStreamSynchronize(ctx->stream), "sync fit jobs");
    }
  }
  const size_t mask_words = ctx->fit_path == 4   ? (size_t)std::max<int64_t>(n_jobs, 1) * ctx->lds_pitch
                            : ctx->fit_path == 3 ? (size_t)std::max<int64_t>(n_jobs, 1) *
                                                       (ctx->pl_rows ? ctx->pl_pitch : ctx->pl_nblk) * 128
                            : ctx->fit_path == 2 ? (size_t)(ctx->code_Jp / 64) * ctx->node_stride
                                                 : (size_t)Jp * std::max<int64_t>(ctx->Wt, 1) * 4;
  static const unsigned mask_flags = std::getenv("PE_MASK_CONTIG") ? hipDeviceMallocContiguous : 0u;
  hipchk(ctx->mask.ensure(mask_words, mask_flags), "alloc fit mask");
  const int64_t n_counts = std::max<int64_t>(Jp, ctx->fit_path == 3 ? ctx->pl_counts_n : 0);
  // (+ the row sweep's per-block work-unit counters, zeroed with the counts every step)
  hipchk(ctx->counts.ensure(n_counts + (ctx->fit_path == 3 ? ctx->pl_nblk : 0)), "alloc fit counts");
  hipchk(ctx->h_counts.ensure(n_counts), "alloc pinned counts");
  hipchk(hipStreamSynchronize(ctx->stream), "sync fit upload");
  ctx->fit_uploaded = true;
}

static void fit_run(pe_ctx* ctx) {
  if (!ctx->fit_uploaded) raise(PE_ESTATE, "pe_jobs_upload first");
  const int64_t J = ctx->fit_J;
  // the single-plane-set encode zeroes the count slots itself (one launch fewer per step)
  const bool encode_zeroes = ctx->fit_path == 3 && ctx->pl_sets.empty() && J > 0 && ctx->Ns > 0 && ctx->pl_nblk > 0;
  if (!encode_zeroes)
    hipchk(hipMemsetAsync(ctx->counts.p, 0, ctx->counts.n * sizeof(unsigned long long), ctx->stream), "memset counts");
  if (J == 0 || ctx->Ns == 0) return;
  // enough waves to fill 256 CUs several times over; at most 16 tiles (4096 nodes) per wave
  const int64_t waves_y = (J + pe::FM_JT - 1) / pe::FM_JT;
  const int64_t want_x = std::max<int64_t>(1, (16384 + waves_y - 1) / waves_y);
  int64_t tpw = (ctx->Ns + 256 * want_x - 1) / (256 * want_x);
  tpw = std::min<int64_t>(16, std::max<int64_t>(1, tpw));
  if (ctx->fit_path == 4) {
    hipchk(hipMemsetAsync(ctx->lds_slots.p, 0, ((size_t)ctx->lds_R * 16 * ctx->lds_Tpad + ctx->lds_nblk) * 4, ctx->stream),
           "memset count slots");
    hipchk(pe::launch_node_ranks(ctx->stream, ctx->res.p, ctx->stride, ctx->labels.p, ctx->Ns, ctx->lds_npad,
                                 ctx->lds_spec_d.p, ctx->lds_vals.p, ctx->lds_ranks.p, ctx->lds_aux.p),
           "launch node_ranks");
    hipchk(pe::launch_fit_mask_lds(ctx->stream, ctx->lds_W, ctx->lds_shape, ctx->lds_spec_d.p, ctx->lds.nplanes,
                                   ctx->lds_ranks.p,
                                   ctx->lds_npad, ctx->lds_aux.p, ctx->lds_nblk, ctx->lds_codes.p, J,
                                   ctx->lds_R, ctx->lds_Tpad, ctx->lds_pitch * 8,
                                   reinterpret_cast<uint8_t*>(ctx->mask.p), ctx->lds_slots.p,
                                   std::getenv("PE_FIT_STATIC") ? nullptr
                                                                : ctx->lds_slots.p + (size_t)ctx->lds_R * 16 * ctx->lds_Tpad),
           "launch fit_mask_lds");
    hipchk(pe::launch_lds_counts(ctx->stream, ctx->lds_slots.p, ctx->lds_rows.p, ctx->lds_R * 16 * ctx->lds_Tpad,
                                 ctx->counts.p),
           "launch lds_counts");
    ctx->stats.fit_runs_lds += 1;
  } else if (ctx->fit_path == 3) {
    // ~16k waves: every 8192-node block times enough job ranges, at least 64 jobs per wave
    if (!ctx->pl_sets.empty()) {   // plane sets: one encode pass and one sweep for all of them
      const int ns = (int)ctx->pl_sets.size();
      hipchk(pe::launch_encode_planes_sets(ctx->stream, ctx->res.p, ctx->stride, ctx->labels.p, ctx->Ns, ctx->pl_nblk,
                                           ctx->pl_specs_d.p, ns, ctx->planes.p),
             "launch encode_planes_sets");
      hipchk(pe::launch_fit_mask_planes_sets(ctx->stream, ctx->planes.p, ctx->pl_nblk, ctx->plane_jobs.p,
                                             ctx->pl_meta_d.p, ns, ctx->pl_sets[0].R,
                                             reinterpret_cast<uint32_t*>(ctx->mask.p), ctx->counts.p, ctx->pl_pitch),
             "launch fit_mask_planes_sets");
      ctx->stats.fit_runs_planes += 1;
      ctx->stats.fit_runs_sets += 1;
      ctx->stats.fit_evals += J * ctx->Ns;
      return;
    }
    hipchk(pe::launch_encode_planes(ctx->stream, ctx->res.p, ctx->stride, ctx->labels.p, ctx->Ns, ctx->pl_nblk,
                                    ctx->plane, ctx->pl_specs_d.p, ctx->planes.p, ctx->counts.p, ctx->counts.n),
           "launch encode_planes");
    if (ctx->pl_rows) {
      // PE_FIT_STATIC=1: every wave keeps its own phase (no work units; A/B, read per call)
      unsigned long long* const units = std::getenv("PE_FIT_STATIC") ? nullptr : ctx->counts.p + ctx->pl_counts_n;
      hipchk(pe::launch_fit_mask_planes_rows(ctx->stream, ctx->planes.p, ctx->pl_nblk, ctx->plane_jobs.p, J, ctx->pl_R,
                                             reinterpret_cast<uint32_t*>(ctx->mask.p), ctx->counts.p, ctx->pl_pitch,
                                             units),
             "launch fit_mask_planes_rows");
    } else {
      const int64_t ranges = std::max<int64_t>(1, (16384 + ctx->pl_nblk - 1) / ctx->pl_nblk);
      const int64_t jpw = std::max<int64_t>(64, (J + ranges - 1) / ranges);
      hipchk(pe::launch_fit_mask_planes(ctx->stream, ctx->planes.p, ctx->pl_nblk, ctx->plane_jobs.p, J, jpw,
                                        reinterpret_cast<uint32_t*>(ctx->mask.p), ctx->counts.p),
             "launch fit_mask_planes");
    }
    ctx->stats.fit_runs_planes += 1;
  } else if (ctx->fit_path == 2) {
    const int64_t jblocks = ctx->code_Jp / pe::FC_JT;
    const int64_t want_x2 = std::max<int64_t>(1, (16384 + jblocks - 1) / jblocks);
    int64_t tpw2 = (ctx->Ns + 64 * pe::FC_CH * want_x2 - 1) / (64 * pe::FC_CH * want_x2);
    tpw2 = std::min<int64_t>(64, std::max<int64_t>(1, tpw2));
    hipchk(pe::launch_encode_nodes(ctx->stream, ctx->res.p, ctx->stride, ctx->labels.p, ctx->Ns, ctx->node_stride,
                                   ctx->code, ctx->code_vals.p, ctx->code_needs.p, ctx->code_x.p),
           "launch encode_nodes");
    hipchk(pe::launch_fit_mask_coded(ctx->stream, ctx->code.therm, ctx->code_x.p, ctx->Ns, ctx->node_stride, ctx->code_jobs.p,
                                     ~ctx->code.guard, J, tpw2, ctx->mask.p, ctx->counts.p),
           "launch fit_mask_coded");
    ctx->stats.fit_runs_coded += 1;
    ctx->stats.fit_runs_therm += ctx->code.therm;
  } else if (ctx->fit32) {
    hipchk(pe::launch_compress_res(ctx->stream, ctx->res.p, ctx->res32.p, ctx->stride, ctx->Ns, ctx->fit_shift),
           "launch compress_res");
    hipchk(pe::launch_fit_mask32(ctx->stream, ctx->res32.p, ctx->stride, ctx->labels.p, ctx->Ns, ctx->Wt,
                                 ctx->fit_jobs32.p, J, tpw, ctx->mask.p, ctx->counts.p),
           "launch fit_mask32");
    ctx->stats.fit_runs_i32 += 1;
  } else {
    hipchk(pe::launch_fit_mask(ctx->stream, ctx->res.p, ctx->stride, ctx->labels.p, ctx->Ns, ctx->Wt,
                               ctx->fit_jobs.p, J, tpw, ctx->mask.p, ctx->counts.p),
           "launch fit_mask");
    ctx->stats.fit_runs_i64 += 1;
  }
  ctx->stats.fit_evals += J * ctx->Ns;
}

static void fit_counts(pe_ctx* ctx, int64_t* out) {
  const int64_t J = ctx->fit_J;
  if (J == 0) return;
  if (ctx->fit_path == 3 && !ctx->pl_sets.empty()) {   // plane sets: slot -> row
    hipchk(hipMemcpyAsync(ctx->h_counts.p, ctx->counts.p, ctx->pl_counts_n * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, ctx->stream),
           "D2H counts");
    hipchk(hipStreamSynchronize(ctx->stream), "sync counts");
    for (int64_t k = 0; k < ctx->pl_counts_n; ++k)
      if (ctx->pl_cnt_row[k] >= 0) out[ctx->pl_cnt_row[k]] = (int64_t)ctx->h_counts.p[k];
    return;
  }
  const bool phased = ctx->fit_path == 3 && ctx->pl_rows;
  const int64_t R = phased ? ctx->pl_R : 1, Jr = phased ? ((J + R - 1) / R + 3) / 4 * 4 : J;
  hipchk(hipMemcpyAsync(ctx->h_counts.p, ctx->counts.p, R * Jr * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        ctx->stream),
         "D2H counts");
  hipchk(hipStreamSynchronize(ctx->stream), "sync counts");
  for (int64_t j = 0; j < J; ++j) out[j] = (int64_t)ctx->h_counts.p[(j % R) * Jr + j / R];
}

int pe_jobs_upload(pe_ctx* ctx, int64_t n_jobs, const int64_t* req, const uint32_t* need) {
  return guarded(ctx, [&]() -> int {
    fit_upload(ctx, n_jobs, req, need);
    return PE_OK;
  });
}

int pe_fit_mask_run(pe_ctx* ctx) {
  return guarded(ctx, [&]() -> int {
    fit_run(ctx);
    return PE_OK;
  });
}

int pe_fit_counts(pe_ctx* ctx, int64_t* out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx->fit_uploaded) raise(PE_ESTATE, "pe_jobs_upload first");
    need_ptr(out, "out_feasible_count");
    fit_counts(ctx, out);
    return PE_OK;
  });
}

int pe_fit_mask_rows(pe_ctx* ctx, int64_t row0, int64_t n_rows, uint64_t* out) {
  return guarded(ctx, [&]() -> int {
    if (!ctx->fit_uploaded) raise(PE_ESTATE, "pe_jobs_upload first");
    if (row0 < 0 || n_rows < 0 || row0 + n_rows > ctx->fit_J) raise(PE_EINVAL, "row range");
    if (n_rows == 0 || ctx->Wn == 0) return PE_OK;
    need_ptr(out, "out");
    if ((ctx->fit_path == 3 && ctx->pl_rows) || ctx->fit_path == 4) {   // row-major
      const int64_t pitch = ctx->fit_path == 4 ? ctx->lds_pitch : ctx->pl_pitch * 128;
      hipchk(hipMemcpy2DAsync(out, (size_t)ctx->Wn * 8, ctx->mask.p + (size_t)row0 * pitch, (size_t)pitch * 8,
                              (size_t)ctx->Wn * 8, (size_t)n_rows, hipMemcpyDeviceToHost, ctx->stream),
             "D2H mask rows");
      hipchk(hipStreamSynchronize(ctx->stream), "sync mask");
      return PE_OK;
    }
    if (ctx->fit_path == 3) {   // block-major: one strided copy per 8192-node block (128 u64 per row)
      for (int64_t b = 0; b * 128 < ctx->Wn; ++b) {
        const int64_t w = std::min<int64_t>(128, ctx->Wn - b * 128);
        hipchk(hipMemcpy2DAsync(out + b * 128, (size_t)ctx->Wn * 8, ctx->mask.p + ((size_t)b * ctx->fit_J + row0) * 128,
                                128 * 8, (size_t)w * 8, (size_t)n_rows, hipMemcpyDeviceToHost, ctx->stream),
               "D2H mask rows");
      }
      hipchk(hipStreamSynchronize(ctx->stream), "sync mask");
      return PE_OK;
    }
    if (ctx->fit_path == 2) {
      // bits-over-jobs layout: copy the 64-job bands, transpose the rows out
      const int64_t b0 = row0 / 64, b1 = (row0 + n_rows - 1) / 64;
      const size_t band = (size_t)ctx->node_stride;
      std::vector<uint64_t> bands((size_t)(b1 - b0 + 1) * band);
      hipchk(hipMemcpyAsync(bands.data(), ctx->mask.p + (size_t)b0 * band, bands.size() * 8, hipMemcpyDeviceToHost,
                            ctx->stream),
             "D2H mask");
      hipchk(hipStreamSynchronize(ctx->stream), "sync mask");
      for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t j = row0 + r;
        const uint64_t* bw = bands.data() + (size_t)(j / 64 - b0) * band;
        const int bit = (int)(j % 64);
        for (int64_t c = 0; c < ctx->Wn; ++c) {
          uint64_t word = 0;
          for (int i = 0; i < 64 && c * 64 + i < ctx->Ns; ++i) word |= ((bw[c * 64 + i] >> bit) & 1ull) << i;
          out[(size_t)r * ctx->Wn + c] = word;
        }
      }
      return PE_OK;
    }
    // copy the 16-row tile bands covering the rows, then untile into row-major
    const int64_t t0 = row0 / 16, t1 = (row0 + n_rows - 1) / 16;
    const size_t band = (size_t)ctx->Wt * 64;
    std::vector<uint64_t> tiles((size_t)(t1 - t0 + 1) * band);
    hipchk(hipMemcpyAsync(tiles.data(), ctx->mask.p + (size_t)t0 * band, tiles.size() * 8, hipMemcpyDeviceToHost,
                          ctx->stream),
           "D2H mask");
    hipchk(hipStreamSynchronize(ctx->stream), "sync mask");
    for (int64_t r = 0; r < n_rows; ++r)
      for (int64_t c = 0; c < ctx->Wn; ++c)
        out[(size_t)r * ctx->Wn + c] = tiles[(size_t)(pe::fm_word_index(row0 + r, c, ctx->Wt) - t0 * (int64_t)band)];
    return PE_OK;
  });
}

int pe_fit_mask(pe_ctx* ctx, int64_t n_jobs, const int64_t* req, const uint32_t* need, int64_t* out_feasible_count,
                const uint64_t** dev_mask, int64_t* words_per_row) {
  return guarded(ctx, [&]() -> int {
    fit_upload(ctx, n_jobs, req, need);
    fit_run(ctx);
    if (out_feasible_count) fit_counts(ctx, out_feasible_count);
    else hipchk(hipStreamSynchronize(ctx->stream), "sync fit");
    if (dev_mask) *dev_mask = ctx->mask.p;
    if (words_per_row) *words_per_row = ctx->Wn;
    return PE_OK;
  });
}

// ------------------------------------------------------------------ greedy placement

// The sorted-walk index of the shard over the current residuals (g_kn must be current): sort the
// walkable nodes by K(n), gather the sorted SoA copy and the round summaries, empty the overlay
// (then holding only the saturating nodes).
static pe::WalkIndex walk_index(pe_ctx* ctx, int set) {
  pe_ctx::WalkSet& x = ctx->ws[set];
  pe::WalkIndex w{};
  w.sk = x.sk.p;
  w.sr = x.sr.p;
  w.sl = x.sl.p;
  w.pos = x.pos.p;
  w.rmin = x.rmin.p;
  w.rmax = x.rmax.p;
  w.ror = x.ror.p;
  w.ovl = x.ovl.p;
  w.ovl_n = x.ovln.p;
  w.in_ovl = x.inovl.p;
  w.ovl_idx = x.ovidx.p;
  w.ovl_res = x.ovres.p;
  w.ovl_lab = x.ovlab.p;
  w.ovl_kn = x.ovkn.p;
  w.stat = ctx->w_stat.p;
  w.sstride = ctx->stride;
  w.nr = (ctx->Ns + pe::WK_ROUND - 1) / pe::WK_ROUND;
  return w;
}
static pe::WalkIndex walk_index(pe_ctx* ctx) { return walk_index(ctx, ctx->w_cur); }

// Index set `set` allocated and its overlay / pos cleared on stream s; returns the sort scratch size.
static size_t walk_set_prepare(pe_ctx* ctx, int set, hipStream_t s) {
  const int64_t Ns = ctx->Ns, st = std::max<int64_t>(ctx->stride, 1);
  const int64_t nr = std::max<int64_t>(1, (Ns + pe::WK_ROUND - 1) / pe::WK_ROUND);
  if (nr > pe::WK_MAXR) raise(PE_EINVAL, "shard too large for the sorted walk");
  pe_ctx::WalkSet& x = ctx->ws[set];
  hipchk(x.sk.ensure(st), "alloc walk keys");
  hipchk(ctx->w_kin.ensure(st), "alloc walk keys");
  hipchk(x.sr.ensure((size_t)pe::D * st), "alloc walk residuals");
  hipchk(x.sl.ensure(st), "alloc walk labels");
  hipchk(x.pos.ensure(st), "alloc walk pos");
  hipchk(x.rmin.ensure(nr), "alloc walk rounds");
  hipchk(x.rmax.ensure((size_t)pe::D * nr), "alloc walk rounds");
  hipchk(x.ror.ensure(nr), "alloc walk rounds");
  hipchk(x.ovl.ensure(st), "alloc overlay");
  hipchk(x.ovln.ensure(1), "alloc overlay");
  hipchk(x.inovl.ensure(st), "alloc overlay");
  hipchk(x.ovidx.ensure(st), "alloc overlay");
  hipchk(x.ovlab.ensure(st), "alloc overlay");
  hipchk(x.ovres.ensure((size_t)pe::D * st), "alloc overlay");
  hipchk(x.ovkn.ensure(st), "alloc overlay");
  size_t tb = 0;
  hipchk(pe::sort_keys_u64(nullptr, &tb, ctx->w_kin.p, x.sk.p, Ns, s), "sort size");
  hipchk(ctx->w_temp.ensure(tb), "alloc sort scratch");
  hipchk(hipMemsetAsync(x.ovln.p, 0, sizeof(int32_t), s), "memset overlay");
  hipchk(hipMemsetAsync(x.inovl.p, 0, (size_t)st * 4, s), "memset overlay");
  hipchk(hipMemsetAsync(x.pos.p, 0xFF, (size_t)st * 4, s), "memset pos");
  return tb;
}

// A side-stream rebuild still running is waited for and dropped (the caller rebuilds in line).
static void walk_drop_pending(pe_ctx* ctx) {
  if (!ctx->w_pending) return;
  hipchk(hipStreamSynchronize(ctx->w_s2), "sync walk rebuild");
  ctx->w_pending = false;
}

// In-line rebuild of the current set on the main stream (the walks after it wait for it).
static void walk_resort(pe_ctx* ctx) {
  walk_drop_pending(ctx);
  hipStream_t s = ctx->stream;
  const int64_t Ns = ctx->Ns;
  size_t tb = walk_set_prepare(ctx, ctx->w_cur, s);
  const pe::WalkIndex w = walk_index(ctx);
  hipchk(pe::launch_walk_prep(s, ctx->res.p, ctx->stride, Ns, ctx->g_kn.p, ctx->labels.p, ctx->w_kin.p, w),
         "launch walk_prep");
  hipchk(pe::sort_keys_u64(ctx->w_temp.p, &tb, ctx->w_kin.p, w.sk, Ns, s), "sort walk keys");
  hipchk(pe::launch_walk_build(s, ctx->res.p, ctx->stride, ctx->labels.p, Ns, (uint64_t)ctx->begin, w),
         "launch walk_build");
  ctx->w_est = 0;
  ctx->stats.resorts += 1;
}

// Rebuild the other set on the side stream from the residuals as of now (the main stream's point
// `snap`), while the main stream's walks keep using the current set: the applies after `snap`
// update both overlays (apply_kernel nx), and walk_switch drops their nodes' possibly torn sorted
// entries from the new set once it is built.  The side stream has the lowest priority, so the
// walks' blocks are dispatched first.  Correct for the same reason as the in-line rebuild: every
// node changed after the snapshot is in the new overlay with its current state, every other node's
// sorted entry and round summaries are exact (a torn entry only widens its round's summary).
static void walk_resort_async(pe_ctx* ctx) {
  if (!ctx->w_s2) {
    int least = 0, greatest = 0;
    hipchk(hipDeviceGetStreamPriorityRange(&least, &greatest), "stream priorities");
    hipchk(hipStreamCreateWithPriority(&ctx->w_s2, hipStreamNonBlocking, least), "side stream");
    hipchk(hipEventCreateWithFlags(&ctx->w_ev_snap, hipEventDisableTiming), "event");
    hipchk(hipEventCreateWithFlags(&ctx->w_ev_done, hipEventDisableTiming), "event");
  }
  hipStream_t s = ctx->stream, s2 = ctx->w_s2;
  const int nx = 1 - ctx->w_cur;
  const int64_t Ns = ctx->Ns;
  size_t tb = walk_set_prepare(ctx, nx, s);   // (cleared on the main stream: before any apply that writes it)
  hipchk(ctx->w_slow.ensure((size_t)std::max<int64_t>(ctx->stride, 1)), "alloc walk slow flags");
  hipchk(hipMemsetAsync(ctx->w_slow.p, 0, (size_t)std::max<int64_t>(ctx->stride, 1) * 4, s), "memset slow flags");
  hipchk(hipEventRecord(ctx->w_ev_snap, s), "event record");
  hipchk(hipStreamWaitEvent(s2, ctx->w_ev_snap, 0), "stream wait");
  const pe::WalkIndex w = walk_index(ctx, nx);
  hipchk(pe::launch_walk_prep(s2, ctx->res.p, ctx->stride, Ns, ctx->g_kn.p, ctx->labels.p, ctx->w_kin.p, w,
                              ctx->w_slow.p),
         "launch walk_prep");
  hipchk(pe::sort_keys_u64(ctx->w_temp.p, &tb, ctx->w_kin.p, w.sk, Ns, s2), "sort walk keys");
  hipchk(pe::launch_walk_build(s2, ctx->res.p, ctx->stride, ctx->labels.p, Ns, (uint64_t)ctx->begin, w),
         "launch walk_build");
  hipchk(hipEventRecord(ctx->w_ev_done, s2), "event record");
  ctx->w_pending = true;
  ctx->w_pend_est = 0;
  ctx->w_pend_windows = 0;
}

// Take over the side-stream rebuild (the main stream waits for it if it is not done yet).
static void walk_switch(pe_ctx* ctx) {
  hipStream_t s = ctx->stream;
  const int nx = 1 - ctx->w_cur;
  hipchk(hipStreamWaitEvent(s, ctx->w_ev_done, 0), "stream wait");
  hipchk(pe::launch_walk_switch(s, ctx->res.p, ctx->stride, ctx->labels.p, ctx->Ns, ctx->w_slow.p, walk_index(ctx, nx)),
         "launch walk_switch");
  ctx->w_cur = nx;
  ctx->w_pending = false;
  ctx->w_est = ctx->w_pend_est;
  ctx->stats.resorts += 1;
}

int pe_place_greedy(pe_ctx* ctx, int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority,
                    const int32_t* group_count, const int64_t* group_req, const uint32_t* group_need,
                    int32_t* out_pod_node, int32_t* out_job_status) {
  return guarded(ctx, [&]() -> int {
    const auto t0 = std::chrono::steady_clock::now();
    if (!ctx->loaded) raise(PE_ESTATE, "no inventory loaded");
    if (ctx->comm_aborted)
      raise(PE_ERCCL, "the RCCL communicator was aborted after a window's all-gather timed out; recreate the context");
    if (n_jobs < 0) raise(PE_EINVAL, "n_jobs < 0");
    if (n_jobs == 0) return PE_OK;
    need_ptr(job_group_off, "job_group_off");
    need_ptr(priority, "priority");
    need_ptr(out_job_status, "out_job_status");
    check_offsets(job_group_off, n_jobs, -1, "job_group_off");
    const int64_t G = job_group_off[n_jobs];
    int64_t P = 0;
    if (G > 0) {
      need_ptr(group_count, "group_count");
      need_ptr(group_req, "group_req");
      check_req(group_req, G, "group_req");
      for (int64_t g = 0; g < G; ++g) {
        if (group_count[g] < 0) raise(PE_EINVAL, "negative group_count");
        P += group_count[g];
      }
    }
    if (P > 0) need_ptr(out_pod_node, "out_pod_node");
    std::vector<uint32_t> no_need;
    if (!group_need) {
      no_need.assign((size_t)std::max<int64_t>(G, 1), 0u);
      group_need = no_need.data();
    }
    // Device preparation first (asynchronous): it runs while the host builds the resolver.
    hipchk(ctx->g_kn.ensure((size_t)std::max<int64_t>(ctx->stride, 1)), "alloc node keys");
    hipchk(ctx->g_lo.ensure((size_t)2 * std::max<int64_t>(ctx->stride, 1)), "alloc node lows");
    // residuals may have changed since the last call (reset, pe_update_nodes): one pass over the shard
    hipchk(pe::launch_prep_nodes(ctx->stream, ctx->res.p, ctx->stride, ctx->Ns, (uint64_t)ctx->begin, ctx->g_kn.p,
                                 ctx->g_lo.p),
           "launch prep_nodes");
    const bool walk = ctx->walk && ctx->Ns > 0;
    // Candidate lists that grow after a rescan (sorted walk): windows start with lists of topk keys;
    // once a window's lists ran out (a rescan: its groups consumed more list entries than it had --
    // whole-node gangs, all of a window's groups after the same few nodes), the rest of the batch walks
    // lists of 2 x topk.  Longer lists cost walk time (cfg3: 0.58 -> 1.25 ms of device wait at 512),
    // rescans cost a drained pipeline each (cfg4: 41 rescans at 256, none at 384).  The blob capacity
    // is the grown length from the start.  Sharded runs grow alike on every rank (each resolves every
    // window identically, so all switch at the same window): over a node's shared-memory segment when
    // its slots hold the grown stride (the host merge cuts at the window's length), and over RCCL, whose
    // windows are written, gathered and merged at the window's own list length (rccl_grow: the
    // all-gather moves k_win keys per group, not the capacity).  The decision depends on nothing a rank
    // holds alone (its shard may be empty): ctx->walk, the segment, the communicator.
    // PE_NO_LIST_GROWTH=1 keeps topk throughout on an UNSHARDED context (A/B; read per call) -- a
    // per-process variable cannot steer sharded ranks, which must agree on the stride.
    const bool rccl_path = ctx->comm && !ctx->exchange;   // the windows go through ncclAllGather (= !use_exchange below)
    const bool no_growth = ctx->world == 1 && !ctx->comm && std::getenv("PE_NO_LIST_GROWTH") != nullptr;
    const int K0 = ctx->topk;
    const int Kg = std::max(K0, std::min(2 * K0, pe::WK_ROUND - 1));
    pe_host_exchange* const hx_grow = ctx->world > 1 && pe::hx_is(ctx->exchange)
                                          ? static_cast<pe_host_exchange*>(ctx->exchange_user) : nullptr;
    const bool kgrow = ctx->walk && !no_growth &&
                       ((ctx->world == 1 && !ctx->comm) || rccl_path ||
                        (hx_grow && (size_t)ctx->window_groups * pe::cand_group_bytes(Kg) <= pe::hx_slot_bytes(hx_grow)));
    const bool rccl_grow = kgrow && rccl_path;
    const int K = kgrow ? Kg : K0;   // blob stride (list capacity)
    int k_win = K0;                  // list length walked (changed only while the helper threads are idle)
    // PE_ASYNC_RESORT=0: rebuild the walk index in line, on the main stream (A/B; read per call).
    // Otherwise the rebuild starts kResortEarly updates before the threshold on the side stream and
    // is taken over once done -- or waited for past kResortLate updates over the threshold.
    const bool async_resort = walk && !(std::getenv("PE_ASYNC_RESORT") && std::atoi(std::getenv("PE_ASYNC_RESORT")) == 0);
    const int64_t kResortEarly = std::min<int64_t>(4096, ctx->resort_nodes / 4);
    const int64_t kResortLate = std::max<int64_t>(1, ctx->resort_nodes / 2);
    const int64_t switch_delay = std::getenv("PE_WALK_SWITCH_DELAY") ? std::atoll(std::getenv("PE_WALK_SWITCH_DELAY")) : 0;
    hipchk(ctx->w_stat.ensure(2), "alloc walk counters");
    hipchk(hipMemsetAsync(ctx->w_stat.p, 0, 2 * sizeof(unsigned long long), ctx->stream), "memset walk counters");
    if (walk) walk_resort(ctx);
    const auto t_prep = std::chrono::steady_clock::now();
    // one resolver per context, reset per batch (its arrays and seed helper thread are reused)
    if (ctx->resolver) ctx->resolver->reset(n_jobs, job_group_off, priority, group_count, group_req, group_need);
    else ctx->resolver.reset(new pe::Resolver(n_jobs, job_group_off, priority, group_count, group_req, group_need));
    pe::Resolver& R = *ctx->resolver;
    R.set_mirror(pe::Mirror{ctx->m_nodes.data(), ctx->n_total});
    const auto t_res = std::chrono::steady_clock::now();
    // PE_DUMP_WINDOWS=<file>: record the batch and every window's groups + blob (host resolver
    // replay, tools/replay_resolver.cc); diagnostics only
    FILE* dump = nullptr;
    if (const char* dp = std::getenv("PE_DUMP_WINDOWS")) {
      dump = std::fopen(dp, "wb");
      if (dump) {
        const int64_t hdr[3] = {n_jobs, G, (int64_t)K};   // (the blob stride)
        std::fwrite(hdr, 8, 3, dump);
        std::fwrite(job_group_off, 4, (size_t)n_jobs + 1, dump);
        std::fwrite(priority, 4, (size_t)n_jobs, dump);
        std::fwrite(group_count, 4, (size_t)G, dump);
        std::fwrite(group_req, 8, (size_t)G * pe::D, dump);
        std::fwrite(group_need, 4, (size_t)G, dump);
        std::fwrite(&ctx->n_total, 8, 1, dump);   // the host mirror at the batch start
        std::fwrite(ctx->m_nodes.data(), sizeof(pe::NodeState), ctx->m_nodes.size(), dump);
      }
    }
    struct DumpClose { FILE*& f; ~DumpClose() { if (f) std::fclose(f); } } dump_close{dump};
    // PE_GREEDY_TRACE=1: per-window wait / resolve / post times, summarised on stderr (diagnostics)
    const bool trace = std::getenv("PE_GREEDY_TRACE") != nullptr;
    std::vector<double> tr_wait, tr_res, tr_post, tr_xspin, tr_xmerge, tr_xblock;
    int helper_cpu = -1;
    struct TraceOut {
      int& helper_cpu;
      const bool& on;
      std::vector<double>& a; std::vector<double>& b; std::vector<double>& c;
      std::vector<double>& d; std::vector<double>& e; std::vector<double>& f;
      ~TraceOut() {
        if (!on || a.empty()) return;
        auto pr = [](const char* n, std::vector<double>& v) {
          if (v.empty()) return;
          std::sort(v.begin(), v.end());
          double sum = 0;
          for (double x : v) sum += x;
          std::fprintf(stderr, "%s n %zu sum %.2f ms mean %.1f us p10 %.1f p50 %.1f p90 %.1f max %.1f\n", n, v.size(),
                       sum / 1e3, sum / v.size(), v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
        };
        pr("wait   ", a);
        pr("resolve", b);
        pr("post   ", c);
        pr("xspin  ", d);   // exchange thread: waiting for the ranks' signals, per window
        pr("xmerge ", e);   // exchange thread: merging, per window
        pr("xblock ", f);   // main thread: waiting for the exchange thread before posting
        auto sib = [](int cpu) {
          char path[128], buf[64] = {0};
          std::snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", cpu);
          FILE* f = std::fopen(path, "r");
          if (f) {
            if (!std::fgets(buf, sizeof buf, f)) buf[0] = 0;
            std::fclose(f);
          }
          buf[std::strcspn(buf, "\n")] = 0;
          return std::string(buf);
        };
        const int mc = sched_getcpu();
        std::fprintf(stderr, "cpus: main %d (siblings %s) helper %d (siblings %s)\n", mc, sib(mc).c_str(), helper_cpu,
                     helper_cpu >= 0 ? sib(helper_cpu).c_str() : "-");
      }
    } trace_out{helper_cpu, trace, tr_wait, tr_res, tr_post, tr_xspin, tr_xmerge, tr_xblock};
    int64_t dump_left = std::getenv("PE_DUMP_MAX_WINDOWS") ? std::atoll(std::getenv("PE_DUMP_MAX_WINDOWS")) : INT64_MAX;
    const size_t gb = pe::cand_group_bytes(K);
    const int Wmax = ctx->window_groups;
    const int Wpad = (int)round_up(Wmax, pe::SC_GT);
    const int nwaves = (int)std::max<int64_t>(1, (ctx->Ns + pe::SC_SPAN - 1) / pe::SC_SPAN);
    hipchk(ctx->g_groups.ensure(Wpad), "alloc groups");
    hipchk(ctx->h_groups.ensure(Wpad, kZeroCopy), "alloc pinned groups");
    hipchk(ctx->g_cand.ensure((size_t)Wpad * nwaves * 64), "alloc cand");
    hipchk(ctx->g_cnt.ensure((size_t)Wpad * nwaves), "alloc cnt");
    hipchk(ctx->g_bound.ensure((size_t)Wpad * nwaves), "alloc bound");
    hipchk(ctx->g_out.ensure((size_t)Wmax * gb), "alloc out");
    hipchk(ctx->h_out.ensure((size_t)Wmax * gb * ctx->world, kZeroCopy), "alloc pinned out");
    if (ctx->pipeline) hipchk(ctx->h_out2.ensure((size_t)Wmax * gb * ctx->world, kZeroCopy), "alloc pinned out");
    if (ctx->world > 1 || ctx->comm) {
      hipchk(ctx->g_gath.ensure((size_t)Wmax * gb * ctx->world), "alloc gather");
      hipchk(ctx->h_own.ensure((size_t)Wmax * gb, kZeroCopy), "alloc pinned own");
    }
    // PE_WALK_EVENTS=1: hipEvents around every walk launch, summed into stats.walk_ms (diagnostics:
    // the greedy roofline of bench.py; the events cost a few us of host time per window)
    const bool wev = walk && std::getenv("PE_WALK_EVENTS") != nullptr;
    // PE_WALK_FLUSH=1 (diagnostics, with PE_WALK_EVENTS: the COLD-cache greedy roofline): before every
    // walk launch a 512 MiB device buffer is rewritten, evicting the walk index (sorted keys, residual
    // copy, round summaries: ~50 MB at 1M nodes) from L2 and the 256 MiB Infinity Cache, so the walk
    // reads come from HBM.  The fill is outside the walk's events.
    const bool wflush = walk && std::getenv("PE_WALK_FLUSH") != nullptr;
    if (wflush) hipchk(ctx->w_flush.ensure((size_t)512 << 20), "alloc flush buffer");
    std::vector<std::pair<hipEvent_t, hipEvent_t>> walk_events;
    struct EventsFree {
      std::vector<std::pair<hipEvent_t, hipEvent_t>>& v;
      ~EventsFree() {
        for (auto& p : v) {
          (void)hipEventDestroy(p.first);
          (void)hipEventDestroy(p.second);
        }
      }
    } events_free{walk_events};
    int64_t walk_launch_groups = 0;
    std::vector<pe::GroupCands> cands;
    hipStream_t s = ctx->stream;
    const bool use_exchange = ctx->exchange && !(ctx->world == 1 && !ctx->comm);
    // The host exchange is a synchronous callback.  Pipelined, the launch helper runs it: after it
    // issued window w+1's scan it waits for the own lists, exchanges them and launches the device
    // merge, signalled per group like an RCCL window -- all while the host resolves window w.
    const bool pipelined = ctx->pipeline;
    // ---- one window on the device: group requests H2D, scan, merge, (RCCL all-gather), blob D2H
    int cb = 0;   // the blob buffer of the window being resolved
    std::unique_ptr<SpinWorker> worker;
    // The resolver, the seed scorer (pe_resolver.cpp) and the launch helper hand cache lines to each
    // other every window / group: keep the three on the CPUs that share this thread's L3 (one CCD)
    // for the call -- intersected with the caller's affinity, restored on return; PE_NO_PIN=1 skips.
    // With several ranks on one host (world > 1), rank r takes the (r mod n)-th of the n L3 domains
    // its affinity allows, so ranks do not pile their spinning threads onto one CCD.
    struct Pin {
      cpu_set_t old_set, l3;
      bool on = false;
      Pin(int rank, int world, int& picked) {
        if (std::getenv("PE_NO_PIN") || pthread_getaffinity_np(pthread_self(), sizeof(old_set), &old_set) != 0)
          return;
        if (world > 1 && picked == -2) picked = pe::l3_pick(old_set, rank);   // sysfs walk once per context
        const int cpu = world > 1 ? picked : sched_getcpu();
        if (!pe::l3_cpus(cpu, &l3)) return;
        CPU_AND(&l3, &l3, &old_set);
        on = CPU_COUNT(&l3) >= 3 && pthread_setaffinity_np(pthread_self(), sizeof(l3), &l3) == 0;
      }
      ~Pin() {
        if (on) (void)pthread_setaffinity_np(pthread_self(), sizeof(old_set), &old_set);
      }
    } pin(ctx->rank, ctx->world, ctx->pin_cpu);
    if (pipelined) {
      worker.reset(new SpinWorker(ctx->device));
      if (pin.on) worker->pin(pin.l3);
    }
    if (pin.on) R.pin_helper(pin.l3);
    // blob buffer b (0: h_out, 1: h_out2, 2-3: h_outx): the windows scanned ahead land in their own
    // buffers while the host still resolves from the current one's
    auto outbuf = [&](int b) { return b == 0 ? ctx->h_out.p : b == 1 ? ctx->h_out2.p : ctx->h_outx[b - 2].p; };
    auto outbufdev = [&](int b) { return b == 0 ? ctx->h_out.dev : b == 1 ? ctx->h_out2.dev : ctx->h_outx[b - 2].dev; };
    const bool direct_out = ctx->world == 1 && !ctx->comm;
    // Pipelined walk windows written in place are SIGNALLED per group (pe::WindowFeed): the host
    // takes each group's list when its block is done, not at a stream sync after the slowest block.
    // The window requests are then double-buffered like the blobs (a walk may still be running when
    // the next window's requests are written); seeing any group of window w signalled proves that
    // every earlier launch of the stream is complete (kernels of one stream run in order), which is
    // what the pinned update records need.  PE_NO_GROUP_SIGNAL=1: stream sync per window instead.
    // Multi-rank windows (RCCL all-gather, or the host exchange): the gathered shard lists are merged
    // on the device into one list per group (merge_shards), written into pinned host memory and
    // signalled like an unsharded walk window -- no D2H of every shard's lists, no host k-way merge.
    // PE_HOST_MERGE=1: the gathered blob is copied and merged lazily on the host instead.
    // (PE_HOST_MERGE=1 with a host exchange, measured: the lazy host merge doubled the resolve --
    // the seed helper cannot pre-skip merged lists -- 20.4 vs 8.9 ms per 2-rank cfg3 batch)
    // (merge_shards_kernel stages one header per rank in a wave's lanes: world <= MG_THREADS / 64;
    // wider sharded runs take the host merge)
    const bool dev_merge = !direct_out && (int64_t)ctx->world * K <= pe::MG_CAP &&
                           ctx->world <= pe::MG_THREADS / 64 && !std::getenv("PE_HOST_MERGE");
    // the shard merge kernel: at 1-2 ranks the rank merge (256-thread blocks, a cut of each list ranked,
    // no sort), from 3 ranks the top-K sort merge (1024-thread blocks) -- measured alone on one MI355X,
    // 112 groups of K = 256 (tools/bench_merge_dev.cc, profiles/r23_merge_dev.txt): rank 13.7 / 19.9 /
    // 35.0 / 102 us per window at 2 / 4 / 8 / 16 ranks, sort 18.0 / 14.8 / 15.2 / 19.3 us.
    // PE_MERGE_RANKED=1 / PE_MERGE_SORT=1 force one (A/B; the rank merge only where its LDS holds the lists).
    const bool ranked = (std::getenv("PE_MERGE_RANKED") || (ctx->world <= 2 && !std::getenv("PE_MERGE_SORT"))) &&
                        ctx->world <= pe::RM_MAX_WORLD && pe::merge_ranked_lds(ctx->world, K) <= pe::RM_MAX_LDS;
    auto* const merge_fn = ranked ? &pe::launch_merge_ranked : &pe::launch_merge_shards;
    const bool signalled = pipelined && !std::getenv("PE_NO_GROUP_SIGNAL") && (direct_out ? walk : dev_merge);
    // Zero-copy shared-memory exchange (pe_hostx.h): decided first, the pipeline depth depends on it.
    bool zc = false;
    pe_host_exchange* const hx = pe::hx_is(ctx->exchange) ? static_cast<pe_host_exchange*>(ctx->exchange_user) : nullptr;
    if (hx && use_exchange && pipelined && signalled && ctx->walk && !std::getenv("PE_NO_ZC_EXCHANGE")) {
      if (ctx->zc_hx != hx) {
        const uint8_t ok = ctx->world <= pe::HX_ZC_MAX_WORLD && pe::hx_zc_register(hx) &&
                                   (size_t)Wmax * gb <= pe::hx_slot_bytes(hx) ? 1 : 0;
        std::vector<uint8_t> all((size_t)ctx->world, 0);
        if (ctx->exchange(ctx->exchange_user, &ok, all.data(), 1) != 0) raise(PE_ERCCL, "exchange callback failed");
        ctx->zc_ok = std::all_of(all.begin(), all.end(), [](uint8_t v) { return v == 1; });
        ctx->zc_hx = hx;
      }
      zc = ctx->zc_ok;
      if (zc) hipchk(ctx->g_xstatus.ensure(1), "alloc exchange status");
    }
    // Pipeline depth D (signalled windows; PE_PIPE_DEPTH, 1..3, default 1): windows i+1 .. i+D are
    // scanned while window i is resolved (D + 1 blob / request buffers, D update staging slots).  (2
    // measured on a 2-rank host-exchange run: 36 vs 22 ms per cfg3 batch -- every dropped speculation
    // throws away two scans.)
    // A copying split exchange (below) reads this rank's lists from the one h_own buffer while the
    // walk of the next window would overwrite it: depth 1 there (only zero-copy windows go deeper).
    const bool copy_split = use_exchange && walk && !zc;
    const int depth = !pipelined ? 0 : !signalled || copy_split ? 1 : [&] {
      const char* e = std::getenv("PE_PIPE_DEPTH");
      return e ? std::min(3, std::max(1, std::atoi(e))) : 1;
    }();
    if (signalled) hipchk(ctx->h_groups2.ensure(Wpad, kZeroCopy), "alloc pinned groups");
    for (int b = 2; b <= depth; ++b) {
      hipchk(ctx->h_groupsx[b - 2].ensure(Wpad, kZeroCopy), "alloc pinned groups");
      hipchk(ctx->h_outx[b - 2].ensure((size_t)Wmax * gb * ctx->world, kZeroCopy), "alloc pinned out");
    }
    auto hgroups = [&](int b) -> HostBuf<ReqRec>& {
      return !signalled || b == 0 ? ctx->h_groups : b == 1 ? ctx->h_groups2 : ctx->h_groupsx[b - 2];
    };
    if (dev_merge && use_exchange && !pipelined)
      hipchk(ctx->h_merged.ensure((size_t)Wmax * gb, kZeroCopy), "alloc pinned merged");
    if (dev_merge && use_exchange && pipelined)
      for (int b = 0; b <= std::max(depth, 1); ++b)
        hipchk(ctx->h_xg[b].ensure((size_t)Wmax * gb * ctx->world, kZeroCopy), "alloc pinned gathered");
    const uint8_t* last_blob = nullptr;   // the parsed blob of the window being resolved (one list per group
                                          // unless the shards are merged on the host)
    uint32_t buf_gen[4] = {0, 0, 0, 0};
    int buf_k[4] = {K, K, K, K};   // the list stride each blob buffer's window was written with
    pe::WindowFeed feed;
    struct StreamIdle {
      hipStream_t s;
      const SpinQueue* x = nullptr;   // the exchange thread (split exchange): a merge it has not launched yet
      // a faulted walk / merge kernel surfaces as its own HIP error (PE_EHIP with the HIP string),
      // and a failed exchange as its own error, not as the feed's "never signalled"
      static bool stream_busy(hipStream_t s) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipErrorNotReady) return true;
        hipchk(e, "walk window stream");
        return false;
      }
      static bool busy(void* u) {
        auto* t = static_cast<StreamIdle*>(u);
        if (t->x && t->x->failed()) const_cast<SpinQueue*>(t->x)->wait();   // rethrows the exchange's error
        return (t->x && t->x->busy()) || stream_busy(t->s);
      }
    } stream_idle{s};
    feed.idle = &StreamIdle::busy;
    feed.idle_user = &stream_idle;
    // RCCL transport: every wait for the stream is bounded (PE_RCCL_TIMEOUT_S) -- a collective that
    // never completes keeps the stream busy, which the idle test above cannot tell from a slow walk
    const double coll_tmo = !use_exchange && ctx->comm ? rccl_timeout_s() : 0.0;
    feed.timeout_s = coll_tmo;
    // a timed-out window starts the communicator's abort where it is detected, before the unwinding
    // (the launch helper's and the events' clean-up) could wait on anything the stuck collective holds
    feed.on_timeout = [](void* u) { rccl_abort(static_cast<pe_ctx*>(u)); };
    feed.timeout_user = ctx;
    auto sync_stream = [&](const char* what) {
      if (coll_tmo <= 0) return hipchk(hipStreamSynchronize(s), what);
      const auto ts = std::chrono::steady_clock::now();
      for (unsigned spin = 1;; ++spin) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) return hipchk(e, what);
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
        if ((spin & 63) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count() > coll_tmo) {
          rccl_abort(ctx);   // (at the throw site: see feed.on_timeout)
          throw pe::CollectiveTimeout(std::string(what) + ": the stream did not drain within " +
                                      std::to_string(coll_tmo) +
                                      " s -- a window's all-gather is stuck (a peer stalled or was lost; PE_RCCL_TIMEOUT_S)");
        }
      }
    };
    // PE_TEST_STALL_WINDOW=n, PE_TEST_STALL_MS=m (test knob, RCCL transport): a one-thread kernel that
    // holds the stream for m ms (wall clock, bounded) is queued right before window n's all-gather --
    // a stand-in for a collective whose peer is gone
    const int64_t stall_window = std::getenv("PE_TEST_STALL_WINDOW") ? std::atoll(std::getenv("PE_TEST_STALL_WINDOW")) : -1;
    const int64_t stall_ticks = [] {
      const char* e = std::getenv("PE_TEST_STALL_MS");
      const double ms = e ? std::atof(e) : 0.0;
      return (int64_t)(std::min(std::max(ms, 0.0), 30000.0) * 1e5);   // wall_clock64: 100 MHz; at most 30 s
    }();
    double feed_spin_seen = 0;   // feed.spin_ms() already counted as device wait
    // A pipelined host exchange with device merge runs on its own thread (split_x): the launch helper
    // only launches window w+1's walk (its lists signalled into pinned memory), the exchange thread
    // waits for them, exchanges and launches the device merge, while the host resolves window w --
    // the resolver then waits for the merged groups' signals only, not for the whole chain.
    // Zero-copy shared-memory exchange (pe_hostx.h): each window's walk writes this rank's lists into
    // its slot of the registered segment and the shard merge, queued behind it, waits on the device
    // for every rank's signal of its group -- no exchange thread, no host barrier, no copies.  The
    // ranks agree on it once per context and segment (each says whether it could register the
    // segment); PE_NO_ZC_EXCHANGE=1 (every rank): the copying exchange below.  (zc is set above.)
    // a rank whose peer stalls: its wait gives up after PE_HX_GPU_TIMEOUT_S (default 60) and the
    // resolver raises (the merged lists come back with n = -1), the GPU is not held
    const int64_t zc_ticks = [] {
      const char* e = std::getenv("PE_HX_GPU_TIMEOUT_S");
      const double t = e ? std::atof(e) : 60.0;
      return (int64_t)((t > 0 ? t : 60.0) * 1e8);   // wall_clock64: 100 MHz
    }();
    // Merging a zero-copy window: by default on the host, by the exchange thread, group by group as
    // every rank's walk signals it into the segment (zc_host: no kernel, no PCIe read-back, the
    // resolver streams the merged groups as in an unsharded window); PE_ZC_DEV_MERGE=1 (A/B): a
    // one-block device wait and the merge kernel behind the walk (zc_dev).
    const bool zc_dev = zc && std::getenv("PE_ZC_DEV_MERGE");
    const bool zc_host = zc && !zc_dev;
    const bool split_x =
        use_exchange && pipelined && signalled && walk && !zc_dev && !std::getenv("PE_NO_SPLIT_EXCHANGE");
    std::unique_ptr<SpinQueue> xworker;
    // Zero-copy windows of 3+ ranks: the exchange thread's host merge grows with the world (8 ranks:
    // ~1-2 us per group against ~0.5 us of resolve; tools/bench_merge.cc), so the window's groups are
    // shared among the exchange thread and helpers, group w on thread w mod T (T = 1 + helpers: 2 up to
    // 4 ranks, 4 above; PE_XCHG_THREADS overrides).  The resolver still takes the groups in order.
    std::vector<std::unique_ptr<SpinWorker>> xmergers;
    if (split_x) {
      xworker.reset(new SpinQueue(ctx->device));
      if (pin.on) xworker->pin(pin.l3);
      stream_idle.x = xworker.get();
      if (zc && !std::getenv("PE_ZC_DEV_MERGE")) {
        int T = ctx->world <= 2 ? 1 : ctx->world <= 4 ? 2 : 4;
        if (const char* e = std::getenv("PE_XCHG_THREADS")) T = std::atoi(e);
        T = std::max(1, std::min(T, kMaxMergers + 1));
        for (int t = 1; t < T; ++t) {
          xmergers.emplace_back(new SpinWorker(ctx->device));
          if (pin.on) xmergers.back()->pin(pin.l3);
          xmergers.back()->post(&pe::merge_warm);   // (waited for before the first window's share)
        }
        xworker->post(&pe::merge_warm);
      }
    }
    struct XWait {   // every exit: the exchange thread's task is over before the buffers it uses go
      std::unique_ptr<SpinQueue>& w;
      ~XWait() {
        if (w) try {
            w->wait();
          } catch (...) {
          }
      }
    } xwait_exit{xworker};
    // PE_XCHG_HOST_MERGE=1 (A/B): the exchange thread merges the gathered lists on the host, group by
    // group, each signalled as written, instead of the device merge -- measured 36.7 vs 18.5 ms per
    // 2-rank cfg3 batch (the merge of world x K keys per group is host work the resolver waits on).
    // The rule is merge_shards_kernel's: the keys below the smallest shard limit, the K + 1 smallest
    // of them; limit = the (K+1)-th, else that minimum.
    const bool xhost_merge = use_exchange && dev_merge && std::getenv("PE_XCHG_HOST_MERGE");
    // merge_shards_kernel's rule on the host: the keys below the smallest shard limit, the K + 1
    // smallest of them (two shards: a branch-free two-way merge); group w of shard r at
    // gath + r * stride + w * gb
    auto host_merge_zc = [&](const uint8_t* gath, size_t stride, int w, uint8_t* out, uint32_t gen) {
      const int W = ctx->world;
      const int Kc = k_win;   // the merged list's length: the window's (the stride may be longer)
      uint8_t* og = out + (size_t)w * gb;
      uint64_t* dst = reinterpret_cast<uint64_t*>(og + sizeof(pe::CandHdr));
      uint64_t L = pe::NO_KEY;
      static_assert(pe::HX_ZC_MAX_WORLD >= pe::RM_MAX_WORLD, "zero-copy merge arrays");
      const uint64_t* lists[pe::HX_ZC_MAX_WORLD];   // (zero-copy windows: world <= HX_ZC_MAX_WORLD)
      int ns[pe::HX_ZC_MAX_WORLD];
      bool bad = false;
      for (int r = 0; r < W; ++r) {
        const uint8_t* g = gath + (size_t)r * stride + (size_t)w * gb;
        pe::CandHdr h;
        std::memcpy(&h, g, sizeof(h));
        L = std::min(L, h.limit);
        lists[r] = reinterpret_cast<const uint64_t*>(g + sizeof(h));
        bad |= h.n < 0 || h.n > K;   // a corrupt rank list: the merged group says so (never read past it)
        ns[r] = std::max(0, std::min(h.n, K));
      }
      uint64_t lim = L;
      const int m = bad ? pe::CAND_CORRUPT : pe::merge_rank_lists(lists, ns, W, L, Kc, dst, &lim);
      pe::CandHdr* hp = reinterpret_cast<pe::CandHdr*>(og);
      hp->n = m;
      hp->limit = bad ? 0 : lim;
      __atomic_store_n(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE);   // the group's signal, last
    };
    auto host_merge_group = [&](const uint8_t* gath, int Wg, int w, uint8_t* out, uint32_t gen) {
      const int W = ctx->world;
      std::vector<const uint64_t*>& lists = ctx->x_lists;
      std::vector<int32_t>& ns = ctx->x_ns;
      std::vector<int32_t>& hd = ctx->x_hd;
      lists.resize((size_t)W);
      ns.resize((size_t)W);
      hd.assign((size_t)W, 0);
      uint64_t L = pe::NO_KEY;
      bool bad = false;
      for (int r = 0; r < W; ++r) {
        const uint8_t* g = gath + ((size_t)r * Wg + w) * gb;
        pe::CandHdr h;
        std::memcpy(&h, g, sizeof(h));
        L = std::min(L, h.limit);
        lists[(size_t)r] = reinterpret_cast<const uint64_t*>(g + sizeof(h));
        bad |= h.n < 0 || h.n > K;   // a corrupt rank list: no key is taken, the group is marked below
        ns[(size_t)r] = std::max(0, std::min(h.n, K));
      }
      uint8_t* og = out + (size_t)w * gb;
      uint64_t* dst = reinterpret_cast<uint64_t*>(og + sizeof(pe::CandHdr));
      int m = bad ? pe::CAND_CORRUPT : 0;
      uint64_t lim = L;
      for (; !bad;) {
        int br = -1;
        uint64_t bk = L;   // (only keys below the smallest limit count)
        for (int r = 0; r < W; ++r)
          if (hd[(size_t)r] < ns[(size_t)r] && lists[(size_t)r][hd[(size_t)r]] < bk) {
            bk = lists[(size_t)r][hd[(size_t)r]];
            br = r;
          }
        if (br < 0) break;
        if (m == K) {   // a (K+1)-th key below the limit: it is the list's limit
          lim = bk;
          break;
        }
        dst[m++] = bk;
        ++hd[(size_t)br];
      }
      pe::CandHdr* hp = reinterpret_cast<pe::CandHdr*>(og);
      hp->n = m;
      hp->limit = lim;
      __atomic_store_n(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE);   // the group's signal, last
    };
    auto exchange_window = [&](int b, int Wg, uint32_t gen, bool own_direct, const SpinWorker* launcher,
                               const pe::HxWindow* hw = nullptr) {
      const size_t bytes = (size_t)Wg * gb;
      if (zc_host) {   // every rank's lists are in the segment: merge each group as all ranks signalled it
        const double tmo = pe::hx_timeout_s();
        const auto t0 = std::chrono::steady_clock::now();
        const int T = 1 + (int)xmergers.size();   // the exchange thread + its merge helpers, groups w = t mod T
        const size_t pf_bytes = pe::merge_read_bytes(ctx->world, k_win, gb);
        // one share of the window: groups t, t + T, ... (waited / merged / spun: this share's times)
        auto share = [&, hw, b, gen, Wg](int t, double* waited, double* spun, double* merged) {
          for (int w = t; w < Wg; w += T) {
            const auto ts = trace ? std::chrono::steady_clock::now() : t0;
            for (int r = 0; r < ctx->world; ++r) {
              const pe::CandHdr* h = reinterpret_cast<const pe::CandHdr*>(hw->host + (size_t)r * hw->slot + (size_t)w * gb);
              if (__atomic_load_n(&h->flags, __ATOMIC_ACQUIRE) == (int32_t)hw->gen) continue;
              const auto tw = std::chrono::steady_clock::now();
              for (unsigned spin = 1; __atomic_load_n(&h->flags, __ATOMIC_ACQUIRE) != (int32_t)hw->gen; ++spin) {
                _mm_pause();
                if ((spin & 4095) == 0) {
                  if (t == 0) {   // (HIP calls from the exchange thread only) a faulted walk of this rank: its own error
                    const hipError_t e = hipStreamQuery(s);
                    if (e != hipErrorNotReady) hipchk(e, "walk window stream");
                  }
                  if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > tmo)
                    throw pe::ExchangeError("host exchange: rank " + std::to_string(r) +
                                            "'s candidate lists never arrived (peer stalled or failed; PE_HX_TIMEOUT_S)");
                }
              }
              *waited += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
            }
            const auto tm = trace ? std::chrono::steady_clock::now() : t0;
            // this share's next groups on their way from DRAM (the device wrote them past the CPU caches;
            // a line fetched before the device's write is snooped out again, harmless) -- the heads the
            // merge reads, not whole slots -- and the output lines owned for writing
            for (int a = 1; a <= 2 && w + a * T < Wg; ++a) {
              const int wn = w + a * T;
              for (int r = 0; r < ctx->world; ++r) {
                const uint8_t* gl = hw->host + (size_t)r * hw->slot + (size_t)wn * gb;
                for (size_t o = 0; o < pf_bytes; o += 64) __builtin_prefetch(gl + o, 0, 3);
              }
              uint8_t* ol = outbuf(b) + (size_t)wn * gb;
              for (size_t o = 0; o < gb; o += 64) __builtin_prefetch(ol + o, 1, 3);
            }
            host_merge_zc(hw->host, hw->slot, w, outbuf(b), gen);
            if (trace) {
              *spun += std::chrono::duration<double, std::micro>(tm - ts).count();
              *merged += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tm).count();
            }
          }
        };
        struct Times {
          double waited = 0, spun = 0, merged = 0, busy = 0;   // busy: the share's wall time less its waits
        };
        Times tt[kMaxMergers + 1];
        auto timed_share = [&share](int t, Times* x) {
          const auto a = std::chrono::steady_clock::now();
          share(t, &x->waited, &x->spun, &x->merged);
          x->busy = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count() - x->waited;
        };
        for (int t = 1; t < T; ++t) {
          Times* x = &tt[t];
          xmergers[(size_t)t - 1]->wait();   // (the warm-up task, before the first window)
          xmergers[(size_t)t - 1]->post([&timed_share, t, x] { timed_share(t, x); });
        }
        std::exception_ptr err;
        try {
          timed_share(0, &tt[0]);
        } catch (...) {
          err = std::current_exception();
        }
        for (int t = 1; t < T; ++t) try {   // every helper is done with the window before it is released
            xmergers[(size_t)t - 1]->wait();
          } catch (...) {
            if (!err) err = std::current_exception();
          }
        if (err) std::rethrow_exception(err);
        double busy = 0, spun = 0, merged = 0;
        for (int t = 0; t < T; ++t) {
          busy = std::max(busy, tt[t].busy);   // the merge's critical path: the busiest share (they run side by side)
          spun += tt[t].spun;
          merged += tt[t].merged;
        }
        if (trace) {
          tr_xspin.push_back(spun);
          tr_xmerge.push_back(merged);
        }
        const double all_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        ctx->stats.xchg_merge_ms += busy;
        ctx->stats.xchg_wait_ms += std::max(0.0, all_ms - busy);   // the rest of the window's exchange: waiting
        pe::hx_zc_consumed(hx, *hw);
        return;
      }
      if (own_direct && ctx->Ns > 0) {   // every own group signalled: the lists are in h_own
        struct Idle {   // busy while the launcher has not launched the walk yet, or the stream runs
          const SpinWorker* l;
          hipStream_t s;
          static bool busy(void* u) {
            auto* x = static_cast<Idle*>(u);
            return (x->l && x->l->busy()) || StreamIdle::stream_busy(x->s);
          }
        } idle{launcher, s};
        pe::WindowFeed own;
        std::vector<pe::GroupCands> own_cands;
        own.idle = &Idle::busy;
        own.idle_user = &idle;
        own.reset(ctx->h_own.p, Wg, K, gen, &own_cands);
        own.wait((size_t)Wg - 1);
      } else {
        hipchk(hipMemcpyAsync(ctx->h_own.p, ctx->g_out.p, bytes, hipMemcpyDeviceToHost, s), "D2H cands");
        hipchk(hipStreamSynchronize(s), "sync own cands");
      }
      const auto tx = std::chrono::steady_clock::now();
      if (ctx->exchange(ctx->exchange_user, ctx->h_own.p, dev_merge ? ctx->h_xg[b].p : outbuf(b), bytes) != 0)
        raise(PE_ERCCL, "exchange callback failed");
      ctx->stats.xchg_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tx).count();
      if (xhost_merge) {
        const auto tm = std::chrono::steady_clock::now();
        for (int w = 0; w < Wg; ++w) host_merge_group(ctx->h_xg[b].p, Wg, w, outbuf(b), gen);
        ctx->stats.xchg_merge_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tm).count();
      } else if (dev_merge) {   // the gathered lists (pinned) merged on the device, signalled per group
        hipchk(merge_fn(s, ctx->h_xg[b].dev, ctx->world, Wg, K, outbufdev(b), gen, 0, nullptr, true),
               "launch merge_shards");
      }
    };
    // gen_in: the window's generation assigned by the caller (split exchange: the exchange thread
    // must know it before the launch); defer_x: leave the exchange to the exchange thread
    auto enqueue_window = [&](const std::vector<int32_t>& groups, int b, uint32_t gen_in = 0, bool defer_x = false,
                              const pe::HxWindow* hw_in = nullptr) {
      const int Wg = (int)groups.size();
      const int Wgp = (int)round_up(Wg, pe::SC_GT);
      const int Kw = rccl_grow ? k_win : K;   // the window's list stride (RCCL: its length, see rccl_grow)
      auto& hg = hgroups(b);
      for (int w = 0; w < Wgp; ++w) {
        const int g = groups[std::min(w, Wg - 1)];
        fill_req(hg.p[w], R.scan_req(g), group_need[g]);   // island groups: count x request
      }
      // unsharded: the kernel writes the blob straight into pinned host memory (no D2H copy); so does
      // a pipelined host exchange's walk (its own lists, signalled per group: no D2H, no stream sync)
      const bool own_direct = walk && use_exchange && pipelined && !zc;
      pe::HxWindow hw;   // zero-copy: this window's slots and their generation (every rank, every window)
      if (zc) {
        hw = hw_in ? *hw_in : pe::hx_zc_next(hx);
        if (zc_host && !pe::hx_zc_wait_reuse(hx, hw))   // (every rank read the window that used the slots)
          throw pe::ExchangeError("host exchange: a rank never finished reading a window (peer stalled or failed)");
      }
      uint8_t* const dst = zc           ? hw.dev + (size_t)ctx->rank * hw.slot
                           : direct_out ? outbufdev(b)
                           : own_direct ? ctx->h_own.dev
                                        : ctx->g_out.p;
      uint32_t gen = 0;   // signalled window: its generation (the walk's or the shard merge's)
      if (gen_in) {
        gen = gen_in;
      } else if (signalled || own_direct) {
        if (++ctx->walk_gen == 0) ++ctx->walk_gen;
        gen = ctx->walk_gen;
      }
      buf_gen[b] = gen;
      buf_k[b] = Kw;
      if (walk) {   // one 64-B request per block: read from pinned host memory, no H2D copy
        // PE_WALK_SWITCH_DELAY=n (test knob): take a finished rebuild over only after n windows ran
        // with it pending, so the dual overlay writes of those windows' applies are exercised
        if (ctx->w_pending && (ctx->w_est > ctx->resort_nodes + kResortLate ||
                               (ctx->w_pend_windows++ >= switch_delay && hipEventQuery(ctx->w_ev_done) == hipSuccess)))
          walk_switch(ctx);
        if (!ctx->w_pending) {
          if (async_resort && ctx->w_est > ctx->resort_nodes - kResortEarly) walk_resort_async(ctx);
          else if (ctx->w_est > ctx->resort_nodes) walk_resort(ctx);
        }
        std::pair<hipEvent_t, hipEvent_t> evp{nullptr, nullptr};
        if (wflush) hipchk(hipMemsetD32Async((hipDeviceptr_t)ctx->w_flush.p, ctx->walk_gen, (size_t)128 << 20, s), "flush");
        if (wev) {
          hipchk(hipEventCreate(&evp.first), "event");
          hipchk(hipEventCreate(&evp.second), "event");
          walk_events.push_back(evp);
          hipchk(hipEventRecord(evp.first, s), "event record");
        }
        hipchk(pe::launch_walk(s, hg.dev, Wg, k_win, walk_index(ctx), ctx->res.p, ctx->stride, ctx->labels.p, ctx->Ns,
                               (uint64_t)ctx->begin, dst, zc ? hw.gen : direct_out || own_direct ? gen : 0u, Kw),
               "launch walk");
        if (wev) hipchk(hipEventRecord(evp.second, s), "event record");
        walk_launch_groups += Wg;
      } else if (ctx->Ns > 0) {
        hipchk(hipMemcpyAsync(ctx->g_groups.p, hg.p, Wgp * sizeof(ReqRec), hipMemcpyHostToDevice, s), "H2D window");
        hipchk(pe::launch_scan(s, ctx->res.p, ctx->stride, ctx->labels.p, ctx->g_kn.p, ctx->g_lo.p, ctx->Ns,
                               (uint64_t)ctx->begin, ctx->g_groups.p, Wg, ctx->g_cand.p, ctx->g_cnt.p, ctx->g_bound.p,
                               nwaves),
               "launch scan");
        hipchk(pe::launch_merge(s, ctx->g_cand.p, ctx->g_cnt.p, ctx->g_bound.p, nwaves, K, dst, Wg),
               "launch merge");
      } else if (zc) {   // an empty shard: empty lists, signalled in stream order like a walk's
        hipchk(pe::launch_empty_groups(s, Wg, Kw, dst, hw.gen), "launch empty groups");
      } else {
        const size_t gbw = pe::cand_group_bytes(Kw);
        std::vector<uint8_t> empty((size_t)Wg * gbw, 0);
        for (int w = 0; w < Wg; ++w) {
          pe::CandHdr h{0, 0, pe::NO_KEY};
          std::memcpy(empty.data() + (size_t)w * gbw, &h, sizeof(h));
        }
        if (direct_out) {
          std::memcpy(outbuf(b), empty.data(), empty.size());
        } else {
          hipchk(hipMemcpyAsync(dst, empty.data(), empty.size(), hipMemcpyHostToDevice, s), "H2D empty");
          hipchk(hipStreamSynchronize(s), "sync empty");
        }
      }
      const size_t bytes = (size_t)Wg * pe::cand_group_bytes(Kw);
      if (direct_out) {
        // written in place
      } else if (zc_host) {   // the exchange thread (or, not deferred, this thread) merges on the host
        ctx->stats.xchg_zc_windows += 1;
        if (!defer_x) exchange_window(b, Wg, gen, false, nullptr, &hw);
      } else if (zc) {   // merged once every rank's walk signalled every group (pe_hostx.h)
        ctx->stats.xchg_zc_windows += 1;
        hipchk(pe::launch_xwait(s, hw.dev, ctx->world, Wg, K, (int64_t)hw.slot, hw.gen, zc_ticks, ctx->g_xstatus.p),
               "launch exchange wait");
        hipchk(merge_fn(s, hw.dev, ctx->world, Wg, K, outbufdev(b), gen, (int64_t)hw.slot,
                                       ctx->g_xstatus.p, true),
               "launch merge_shards");
      } else if (use_exchange) {
        if (!pipelined)
          hipchk(hipMemcpyAsync(ctx->h_own.p, ctx->g_out.p, bytes, hipMemcpyDeviceToHost, s), "D2H cands");
        else if (!defer_x)   // (the launch helper, or the main thread at a restart) exchange now
          exchange_window(b, Wg, gen, own_direct, nullptr);
      } else {
        if (stall_window >= 0 && ctx->stats.windows == stall_window && stall_ticks > 0)
          hipchk(pe::launch_stall(s, stall_ticks), "launch stall (test knob)");
        ncclchk(ncclAllGather(ctx->g_out.p, ctx->g_gath.p, bytes, ncclUint8, ctx->comm, s), "ncclAllGather");
        if (dev_merge)
          hipchk(merge_fn(s, ctx->g_gath.p, ctx->world, Wg, Kw, outbufdev(b), gen, 0, nullptr, false),   // (device lists)
                 "launch merge_shards");
        else
          hipchk(hipMemcpyAsync(outbuf(b), ctx->g_gath.p, bytes * ctx->world, hipMemcpyDeviceToHost, s),
                 "D2H gathered");
      }
      ctx->stats.windows += 1;
      ctx->stats.groups_scanned += Wg;
      if (!walk) ctx->stats.scan_evals += (int64_t)Wg * ctx->Ns;
    };
    // ---- wait for the window's blob (and run the host exchange when one is configured), parse it
    auto collect_window = [&](const std::vector<int32_t>& groups, int b) {
      const int Wg = (int)groups.size();
      const size_t bytes = (size_t)Wg * gb;
      const auto tw = std::chrono::steady_clock::now();
      if (signalled && buf_gen[b] != 0) {   // the first group's list (and so every earlier launch) is done
        last_blob = outbuf(b);
        feed.reset(outbuf(b), Wg, buf_k[b], buf_gen[b], &cands);
        feed.wait(0);
        feed_spin_seen = feed.spin_ms();
        const auto th = std::chrono::steady_clock::now();
        ctx->stats.greedy_wait_ms += std::chrono::duration<double, std::milli>(th - tw).count();
        if (trace) tr_wait.push_back(std::chrono::duration<double, std::micro>(th - tw).count());
        return;
      }
      sync_stream("sync window");
      last_blob = outbuf(b);
      if (use_exchange && !pipelined) {
        const auto tx = std::chrono::steady_clock::now();
        if (ctx->exchange(ctx->exchange_user, ctx->h_own.p, outbuf(b), bytes) != 0)
          raise(PE_ERCCL, "exchange callback failed");
        ctx->stats.xchg_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tx).count();
        if (dev_merge) {   // the gathered blob (pinned) merged by the device into h_merged
          hipchk(merge_fn(s, outbufdev(b), ctx->world, Wg, K, ctx->h_merged.dev, 0u, 0, nullptr, true),
                 "launch merge_shards");
          sync_stream("sync merge");
          last_blob = ctx->h_merged.p;
        }
      }
      const auto th = std::chrono::steady_clock::now();
      ctx->stats.greedy_wait_ms += std::chrono::duration<double, std::milli>(th - tw).count();
      if (trace) tr_wait.push_back(std::chrono::duration<double, std::micro>(th - tw).count());
      pe::parse_window_keys(last_blob, dev_merge ? 1 : ctx->world, Wg, buf_k[b], cands);   // lists point into the blob

      ctx->stats.greedy_host_ms +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th).count();
    };
    // ---- residual updates of this shard: the apply kernel reads the records from pinned staging
    //      slot `slot` (no H2D copy); a slot is rewritten only once a later launch is known to have
    //      started (a signalled group seen, or a stream sync) -- the pipelined loop below rotates D
    auto enqueue_apply = [&](const std::vector<pe::Update>& updates, int slot) {
      int64_t nu = 0;
      HostBuf<int64_t>& hu = slot == 0 ? ctx->h_upd : ctx->h_updx[slot - 1];
      hipchk(hu.ensure(std::max<size_t>(updates.size(), 1) * (pe::D + 1), kZeroCopy), "alloc pinned upd");
      for (const pe::Update& u : updates) {
        if (u.gid < ctx->begin || u.gid >= ctx->end) continue;
        int64_t* o = hu.p + nu * (pe::D + 1);
        o[0] = u.gid - ctx->begin;
        for (int d = 0; d < pe::D; ++d) o[1 + d] = u.res[d];
        ++nu;
      }
      if (nu > 0) {   // the kernel reads the pinned records directly (no H2D copy)
        const pe::WalkIndex w = walk_index(ctx);
        const pe::WalkIndex wn = walk_index(ctx, 1 - ctx->w_cur);   // (read only while a rebuild is pending)
        hipchk(pe::launch_apply(s, ctx->res.p, ctx->stride, hu.dev, nu, (uint64_t)ctx->begin, ctx->g_kn.p,
                                ctx->g_lo.p, ctx->labels.p, walk ? &w : nullptr,
                                walk && ctx->w_pending ? &wn : nullptr),
               "launch apply");
        ctx->w_est += nu;
        if (ctx->w_pending) {
          ctx->w_pend_est += nu;
          ctx->stats.walk_pend_updates += nu;   // applied into both index sets' overlays
        }
      }
    };
    auto timed_resolve = [&](const std::vector<int32_t>& groups, std::vector<pe::Update>& updates,
                             const std::vector<pe::Update>* seed) {
      if (dump && dump_left-- == 0) {   // PE_DUMP_MAX_WINDOWS reached
        std::fclose(dump);
        dump = nullptr;
      }
      if (dump) {   // {Wg, groups, blob, n_seed, seeds}: what this resolve call reads
        if (signalled) feed.wait(groups.size() - 1);   // (diagnostics: the whole blob first)
        const int32_t wg = (int32_t)groups.size(), ns = seed ? (int32_t)seed->size() : 0;
        std::fwrite(&wg, 4, 1, dump);
        std::fwrite(groups.data(), 4, (size_t)wg, dump);
        std::fwrite(last_blob, 1, (size_t)wg * gb * (dev_merge || direct_out ? 1 : ctx->world), dump);
        std::fwrite(&ns, 4, 1, dump);
        if (ns) std::fwrite(seed->data(), sizeof(pe::Update), (size_t)ns, dump);
      }
      const auto th = std::chrono::steady_clock::now();
      updates.clear();
      const bool fed = signalled && buf_gen[cb] != 0;
      const bool consumed = R.resolve(groups, cands, updates, seed, fed ? &feed : nullptr);
      // time the resolver spent blocked on groups not yet signalled is device wait, not host work
      const double spun = fed ? feed.spin_ms() - feed_spin_seen : 0.0;
      if (trace) tr_res.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - th).count() -
                                  spun * 1e3);
      for (const pe::Update& u : updates)          // the mirror follows every placement (all shards)
        for (int d = 0; d < pe::D; ++d) ctx->m_nodes[u.gid].res[d] = u.res[d];
      ctx->stats.greedy_host_ms +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th).count() - spun;
      ctx->stats.greedy_wait_ms += spun;
      return consumed;
    };

    // Pipelined (exact), depth D: while the host resolves window i, the device holds windows
    // i+1 .. i+D scanned (or scanning), each speculating that the windows before it are consumed.  A
    // window scanned after the updates of the epoch's windows < v were applied misses the changes of
    // windows v .. i-1, which its resolution takes as dirty seeds (their current states are known
    // here).  Each iteration the helper thread applies the previous window's updates and scans the
    // window D ahead into the next free buffer.  A window cut short, or a cursor that did not land
    // where the speculation started, syncs, applies everything and restarts from the cursor.
    // Staging-buffer reuse: the apply posted in iteration j is followed, in the same post, by the
    // scan of window j + D; the slot is written again in iteration j + D, when that window's first
    // group has been seen, i.e. after every earlier launch of the stream finished (with the early post
    // below, two slots: see early_post).  Blob / request buffer b is reused D + 1 windows later, after
    // the windows in between were resolved.
    struct Flight {
      std::vector<int32_t> groups;
      pe::Cursor end;
      int buf = 0;
      size_t ver = 0;   // updates of the epoch's windows [0, ver) were applied before its scan
    };
    std::deque<Flight> fl;
    std::vector<std::vector<pe::Update>> hist;   // updates of the epoch's resolved windows
    size_t n_app = 0;                             // of which posted for apply
    int next_buf = 0, upd_slot = 0;
    // Early post (signalled windows at depth 1, one rank or a non-split exchange; PE_EARLY_POST=0: off,
    // A/B; unsignalled windows share one request buffer, which the next walk may still read): once window i
    // landed, the helper is given apply(i) and the scan of window i + 2 at once -- queued behind the walk
    // of window i + 1 -- instead of after the first group of window i + 1 was seen, so the device never
    // idles while the host posts them.  The apply records then need two staging slots: apply(i) may be
    // written while apply(i - 1) has not run yet; the slot it reuses was read by apply(i - 2), which ran
    // before the walk of window i, all of whose groups were resolved.
    const bool early_post = signalled && depth == 1 && !split_x &&
                            !(std::getenv("PE_EARLY_POST") && std::atoi(std::getenv("PE_EARLY_POST")) == 0);
    const int upd_slots = early_post ? 2 : std::max(depth, 1);
    bool posted = false;   // the helper already has this iteration's task (early post)
    const int nbuf = std::max(depth, 1) + 1;
    auto add_flight = [&](const pe::Cursor& from) -> Flight* {   // main thread; nullptr: no window left
      Flight f;
      R.next_window_from(from, Wmax, ctx->window_pods, f.groups, &f.end);
      if (f.groups.empty()) return nullptr;
      f.buf = next_buf;
      next_buf = (next_buf + 1) % nbuf;
      f.ver = hist.size();
      fl.push_back(std::move(f));
      return &fl.back();
    };
    auto restart = [&]() {   // nothing in flight, every update applied: a fresh epoch at the cursor
      fl.clear();
      hist.clear();
      n_app = 0;
      next_buf = 0;
      Flight* f = add_flight(R.cursor());
      if (!f) return;
      if (split_x && zc_host) {
        // a zero-copy window: merged group by group on the exchange thread as in the loop below, so
        // the resolver starts on the first merged group (merging the whole window here first put the
        // walk's tail and the full merge in front of every batch start and every rescan)
        if (++ctx->walk_gen == 0) ++ctx->walk_gen;
        const uint32_t gen = ctx->walk_gen;
        const pe::HxWindow hw = pe::hx_zc_next(hx);
        enqueue_window(f->groups, f->buf, gen, true, &hw);
        const int b = f->buf, wg = (int)f->groups.size();
        xworker->post([&, b, wg, gen, hw] { exchange_window(b, wg, gen, true, worker.get(), &hw); });
      } else {
        enqueue_window(f->groups, f->buf);
      }
    };
    const auto t_setup = std::chrono::steady_clock::now();
    restart();
    std::vector<pe::Update> seed, upd;
    while (!fl.empty()) {
      Flight& cur = fl.front();
      cb = cur.buf;
      collect_window(cur.groups, cur.buf);       // cur's lists: snapshot = device state at its launch
      if (!pipelined) {
        if (!timed_resolve(cur.groups, upd, nullptr)) k_win = K;
        enqueue_apply(upd, 0);
        if (R.done()) break;
        fl.clear();
        next_buf = 0;
        if (Flight* f = add_flight(R.cursor())) enqueue_window(f->groups, f->buf);
        continue;
      }
      // the helper: previous windows' updates applied, then windows scanned up to D ahead
      std::vector<std::pair<const std::vector<pe::Update>*, int>> to_apply;
      std::vector<Flight*> to_scan;
      auto plan_post = [&]() {
        to_apply.clear();
        to_scan.clear();
        for (; n_app < hist.size(); ++n_app) {
          to_apply.emplace_back(&hist[n_app], upd_slot);
          upd_slot = (upd_slot + 1) % upd_slots;
        }
        while ((int)fl.size() < depth + 1)
          if (Flight* f = add_flight(fl.back().end)) to_scan.push_back(f);
          else break;
      };
      auto post_scan = [&]() {   // (the non-split helper task)
        worker->post([&, to_apply, to_scan] {
          const auto tp = std::chrono::steady_clock::now();
          if (trace) helper_cpu = sched_getcpu();
          for (const auto& a : to_apply) enqueue_apply(*a.first, a.second);
          for (Flight* f : to_scan) enqueue_window(f->groups, f->buf);
          if (trace) tr_post.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tp).count());
        });
      };
      if (posted) {
        posted = false;
      } else if (split_x) {
        plan_post();
        // generations assigned here, in launch order: the exchange thread waits for these windows' own
        // lists (signalled with them) while the launch helper launches the walks
        // (zero-copy: the windows' slots too, taken in the same order on every rank)
        struct XWin {
          int buf, wg;
          uint32_t gen;
          pe::HxWindow hw;
        };
        std::vector<XWin> xs;
        std::vector<std::pair<Flight*, XWin>> ws;
        for (Flight* f : to_scan) {
          if (++ctx->walk_gen == 0) ++ctx->walk_gen;
          xs.push_back(XWin{f->buf, (int)f->groups.size(), ctx->walk_gen, zc_host ? pe::hx_zc_next(hx) : pe::HxWindow{}});
          ws.emplace_back(f, xs.back());
        }
        const auto txb = std::chrono::steady_clock::now();
        // (the copying exchange: the previous window's exchange is over before the next one, its
        // buffers are shared; host-merged zero-copy windows queue up -- slot reuse is counted)
        if (!zc_host) xworker->wait();
        if (trace) tr_xblock.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - txb).count());
        worker->post([&, to_apply, ws] {
          const auto tp = std::chrono::steady_clock::now();
          if (trace) helper_cpu = sched_getcpu();
          for (const auto& a : to_apply) enqueue_apply(*a.first, a.second);
          for (const auto& w : ws)
            enqueue_window(w.first->groups, w.first->buf, w.second.gen, true, zc_host ? &w.second.hw : nullptr);
          if (trace) tr_post.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tp).count());
        });
        xworker->post([&, xs] {
          for (const XWin& x : xs) exchange_window(x.buf, x.wg, x.gen, true, worker.get(), zc_host ? &x.hw : nullptr);
        });
      } else {
        plan_post();
        post_scan();
      }
      // seeds: the changes of the windows resolved since cur's scan (later states overwrite)
      seed.clear();
      for (size_t k = cur.ver; k < hist.size(); ++k) seed.insert(seed.end(), hist[k].begin(), hist[k].end());
      bool consumed = false;
      try {
        consumed = timed_resolve(cur.groups, upd, &seed);
      } catch (...) {
        // the helper task still reads the flights and update sets: let it finish before the
        // unwinding frees them, then report the resolver's error (the helper's is secondary)
        try {
          worker->wait();
        } catch (...) {
        }
        if (xworker) xworker->wait();   // (a failed exchange is the cause: its error wins)
        throw;
      }
      worker->wait();
      const bool landed = consumed && R.cursor() == cur.end && fl.size() > 1;
      if (landed && !R.done()) {
        hist.push_back(std::move(upd));
        upd = {};
        fl.pop_front();
        if (early_post) {   // the next iteration's task, now
          plan_post();
          post_scan();
          posted = true;
        }
        continue;
      }
      // done, or speculation dropped: finish the device work, apply what is left, in order (one
      // launch per window: a node may be in several windows' updates)
      if (xworker) xworker->wait();   // (its merge launch first: it is stream work too)
      sync_stream("sync speculative");
      for (; n_app < hist.size(); ++n_app) {   // (depth > 1 only; slot 0 is rewritten after each)
        enqueue_apply(hist[n_app], 0);
        sync_stream("sync apply");
      }
      enqueue_apply(upd, 0);
      if (R.done()) break;
      if (!consumed) k_win = K;   // lists ran out: longer ones from here (the helper is idle now)
      restart();
    }
    const auto t_loop = std::chrono::steady_clock::now();
    if (xworker) xworker->wait();
    sync_stream("sync greedy");
    walk_drop_pending(ctx);   // (the next call rebuilds in line anyway)
    if (walk) {
      unsigned long long wc[2] = {0, 0};
      hipchk(hipMemcpy(wc, ctx->w_stat.p, sizeof(wc), hipMemcpyDeviceToHost), "D2H walk counters");
      ctx->stats.walk_rounds += (int64_t)wc[0];
      ctx->stats.walk_overlay += (int64_t)wc[1];
      ctx->stats.walk_groups += walk_launch_groups;
      ctx->stats.walk_prepass += walk_launch_groups * ((ctx->Ns + pe::WK_ROUND - 1) / pe::WK_ROUND);
      for (auto& p : walk_events) {
        float ms = 0.f;
        hipchk(hipEventElapsedTime(&ms, p.first, p.second), "event elapsed");
        ctx->stats.walk_ms += ms;
      }
    }
    if (P > 0) std::memcpy(out_pod_node, R.pod_node().data(), (size_t)P * 4);
    std::memcpy(out_job_status, R.job_status().data(), (size_t)n_jobs * 4);
    ctx->stats.rescans += R.rescans();
    ctx->stats.pods_placed += R.pods_placed();
    ctx->stats.jobs_placed += R.jobs_placed();
    ctx->stats.jobs_failed += R.jobs_failed();
    ctx->stats.last_greedy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (trace) {
      auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::micro>(b - a).count();
      };
      std::fprintf(stderr, "greedy phases (us): checks+prep %.0f resolver %.0f setup %.0f loop %.0f tail %.0f\n",
                   us(t0, t_prep), us(t_prep, t_res), us(t_res, t_setup), us(t_setup, t_loop),
                   us(t_loop, std::chrono::steady_clock::now()));
    }
    return PE_OK;
  });
}

int pe_fit_mask_layout(const pe_ctx* ctx, int32_t* layout) {
  if (!ctx || !layout) return PE_EINVAL;
  *layout = ctx->fit_path == 4   ? PE_MASK_ROWS
            : ctx->fit_path == 3 ? (ctx->pl_rows ? PE_MASK_ROWS : PE_MASK_NODE_BLOCKS)
            : ctx->fit_path == 2 ? PE_MASK_JOB_BITS
                                 : PE_MASK_NODE_TILES;
  return PE_OK;
}

int pe_fit_mask_row_pitch(const pe_ctx* ctx, int64_t* words) {
  if (!ctx || !words) return PE_EINVAL;
  *words = ctx->fit_path == 4 ? ctx->lds_pitch : ctx->fit_path == 3 && ctx->pl_rows ? ctx->pl_pitch * 128 : 0;
  return PE_OK;
}

int pe_synchronize(pe_ctx* ctx) {
  return guarded(ctx, [&]() -> int {
    hipchk(hipStreamSynchronize(ctx->stream), "sync");
    return PE_OK;
  });
}

void* pe_stream(pe_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int pe_get_stats(const pe_ctx* ctx, pe_stats* out) {
  if (!ctx || !out) return PE_EINVAL;
  *out = ctx->stats;
  return PE_OK;
}

int pe_reset_stats(pe_ctx* ctx) {
  if (!ctx) return PE_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->stats = pe_stats{};
  return PE_OK;
}

}  // extern "C"
