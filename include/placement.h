/*
 * placement.h -- C ABI of libplacement, the MI355X-native gang-placement engine.
 *
 * Drop-in boundary for the training operator's PodGroup / coscheduling hot path.  Plain C11:
 * plain pointers and sizes, no C++ or torch types, integer return codes, no exceptions or
 * aborts across the ABI.  The reference is Go; the binding a maintainer adds on the reference
 * side (cgo package pkg/placement/hip) is in INTEGRATION.md.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo root):
 *   pe_pg_min_resources(PE_MODE_V1, ...)
 *       pkg/controller.v1/common/util.go:108  func CalcPGMinResources(minMember int32,
 *           replicas map[ReplicaType]*ReplicaSpec, pcGetFunc PriorityClassGetFunc) *v1.ResourceList
 *       (called from pkg/controller.v1/common/job.go:275-277,455-457; AddResourceList util.go:79-104)
 *   pe_pg_min_resources(PE_MODE_V2, ...)
 *       pkg/runtime.v2/framework/plugins/coscheduling/coscheduling.go:103-118  (*CoScheduling).Build
 *       aggregation loop, fed by pkg/runtime.v2/runtime.go:115-145 NewInfo (kueue TotalRequests)
 *   pe_fit_mask / pe_fit_mask_run, pe_place_greedy
 *       NO reference function: node fit / score / placement is done by the external gang
 *       scheduler (scheduler-plugins coscheduling / Volcano) that consumes the PodGroup the
 *       operator writes (pkg/controller.v1/control/podgroup_control.go:36-54).  The rule is
 *       build-defined and exposed here so the plugin can answer
 *       feasibility / placement itself.
 *   pe_create / pe_destroy / pe_last_error
 *       lifetime of the plugin instance: pkg/runtime.v2/framework/plugins/registry.go:32-42
 *       factory + coscheduling.go:71-85 New(); errors follow framework.go:117-121 (first error
 *       stops the phase) -> every call returns a code and sets a message.
 *
 * Units (canonical int64): dim 0 cpu in milli-cores, dim 1 memory in
 * bytes, dim 2 accelerator count (resource name given by pe_config.gpu_resource_name), dim 3
 * ephemeral-storage in bytes.  Values must be >= 0; int64 overflow is flagged, never wrapped
 * (where Go's resource.Quantity would fall back to inf.Dec).
 *
 * Ownership: the caller owns every host pointer for the duration of the call only; the library
 * never retains them.  Device memory is library-owned; pointers it hands out stay valid until
 * the next call that re-sizes the same buffer, or pe_destroy.
 * Threading: one mutex per context; every call selects the context's device itself (callers
 * such as cgo goroutines may migrate between OS threads).
 */
#ifndef PLACEMENT_H_
#define PLACEMENT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PE_ABI_VERSION 7
#define PE_DIMS 4
#define PE_COMM_ID_BYTES 128
#define PE_MAX_NODES (1LL << 24) /* node ids live in the low 24 bits of the best-fit key */

enum {
  PE_OK = 0,
  PE_EINVAL = -1,    /* bad argument (negative request, ids out of range, null pointer) */
  PE_EOVERFLOW = -2, /* int64 overflow in an aggregation (per-job flags say which job) */
  PE_ENOMEM = -3,
  PE_EHIP = -4,      /* HIP runtime error, see pe_last_error */
  PE_ERCCL = -5,     /* RCCL error */
  PE_ESTATE = -6,    /* call order (e.g. fit mask before pe_load_nodes) */
  PE_ENODEV = -7     /* no usable GPU: the engine has no CPU fallback */
};

enum { PE_MODE_V1 = 1, PE_MODE_V2 = 2 };
enum { PE_JOB_PLACED = 0, PE_JOB_UNSCHEDULABLE = 1 };
/* xGMI islands (SURVEY.md Appendix B extension; BASELINE config 4).  Label bit 31 of every node is
 * the engine's: set iff the node has an island (island >= 0 at pe_load_nodes / pe_update_nodes;
 * the caller's bit 31 is replaced).  A greedy group whose need has bit 31 is an ISLAND GROUP: its
 * group_count pods are co-located on ONE node with an island, chosen as a unit -- the node with
 * the smallest Appendix-B key for the summed request count x request (exact int64; a sum that
 * overflows fits nowhere) -- and all of them land on it, or the job fails (all-or-nothing).
 * Islands are single nodes in this model (one 8-GPU node = one xGMI island). */
#define PE_LABEL_ISLAND 0x80000000u
#define PE_NEED_ISLAND PE_LABEL_ISLAND

/* container record flags for pe_pg_min_resources: bits 0-3 = which dims are present in the
 * container's ResourceList (keys with value 0 are present), bits 4-5 = kind */
#define PE_KIND_SHIFT 4
enum { PE_KIND_CONTAINER = 0, PE_KIND_INIT = 1, PE_KIND_SIDECAR = 2, PE_KIND_OVERHEAD = 3 };

/* Host all-gather used instead of RCCL when set (tests run several shards on one GPU):
 * gather `bytes` from every rank into recv[rank * bytes]; return 0 on success. */
typedef int (*pe_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);

/* Intra-node host exchange (no reference counterpart: the transport of the sharded greedy when the
 * ranks share one node and RCCL cannot be set up, e.g. several ranks on one GPU).  An all-gather
 * through a POSIX shared-memory segment `name` ("/..."), one barrier per call; rank 0 creates it,
 * the other ranks wait for it (PE_HX_TIMEOUT_S, default 300 s) and the last rank to attach unlinks
 * the name.  Use as pe_config.exchange = pe_host_exchange_allgather, exchange_user = the handle;
 * every rank must make the same sequence of calls with the same byte counts (<= max_bytes).  A peer
 * that does not arrive within PE_HX_TIMEOUT_S makes the call return PE_ERCCL. */
typedef struct pe_host_exchange pe_host_exchange;
int pe_host_exchange_open(const char* name, int32_t rank, int32_t world, size_t max_bytes, pe_host_exchange** out);
int pe_host_exchange_allgather(void* user, const void* send, void* recv, size_t bytes);
void pe_host_exchange_close(pe_host_exchange* hx);

typedef struct pe_ctx pe_ctx;

typedef struct {
  int32_t device_id;             /* HIP ordinal; -1 = the calling thread's current device */
  int32_t rank;                  /* inventory shard owned by this process, 0..world_size-1 */
  int32_t world_size;            /* shards of the node inventory (1 = unsharded) */
  const uint8_t* comm_id;        /* PE_COMM_ID_BYTES from pe_comm_id() on rank 0 (RCCL); at
                                    world_size 1 it builds a 1-rank communicator */
  pe_allgather_fn exchange;      /* optional host exchange replacing RCCL */
  void* exchange_user;
  int64_t max_nodes;             /* global inventory capacity (<= PE_MAX_NODES) */
  const char* gpu_resource_name; /* resource key of dim 2, e.g. "amd.com/gpu" (informational) */
  int32_t topk;                  /* best-fit candidates kept per group and window (0 = 256; above
                                    1023 the windows take the full scan instead of the sorted walk) */
  int32_t window_groups;         /* groups per scan window (0 = 112) */
  int64_t window_pods;           /* pods per scan window (0 = 1024) */
  int32_t fit_path_mask;         /* allowed fit-mask kernels: bit0 int64 compare, bit1 int32 compare,
                                    bit2 dictionary-coded, bit4 bit planes (batches with more than 32
                                    distinct request values split into plane sets); bit3 set = no thermometer
                                    form of the coded kernel; bit5 set = bit planes through the
                                    block-major kernel (PE_MASK_NODE_BLOCKS) instead of the row-major
                                    sweep (PE_MASK_ROWS); no kernel bit set = all kernels (the
                                    int64 path is always allowed) */
  int32_t greedy_flags;          /* bit0 set = sequential greedy windows.  Default (clear): pipelined --
                                    the GPU scans the next window while the host resolves the current
                                    one, and the current window's changes are seeded as dirty nodes
                                    into the next one's resolution (exact either way).
                                    bit1 set = every window scans all nodes of the shard (scan +
                                    merge kernels) instead of the sorted walk */
  int32_t resort_nodes;          /* sorted walk: rebuild the sorted index once this many node updates
                                    were applied since the last build (0 = 20480) */
} pe_config;

typedef struct {
  int64_t fit_evals;     /* job x node fit evaluations (fit mask) */
  int64_t scan_evals;    /* group x node key evaluations (greedy full scans, greedy_flags bit1) */
  int64_t windows;       /* greedy scan windows */
  int64_t rescans;       /* windows cut short because a candidate list ran dry */
  int64_t groups_scanned;
  int64_t pods_placed;
  int64_t jobs_placed;
  int64_t jobs_failed;
  double last_greedy_ms; /* wall time of the last pe_place_greedy */
  double greedy_wait_ms; /* host time blocked on window scans + transfers (cumulative) */
  double greedy_host_ms; /* host time parsing + resolving windows (cumulative) */
  int64_t fit_runs_i32;  /* fit-mask launches on the exact 32-bit path (scaled requests) */
  int64_t fit_runs_i64;  /* fit-mask launches on the general 64-bit path */
  int64_t fit_runs_coded; /* fit-mask launches on the dictionary-coded path (SWAR or thermometer) */
  int64_t fit_runs_therm; /* ... of which used the thermometer code (3 VALU per 64 evaluations) */
  int64_t fit_runs_planes; /* fit-mask launches on the bit-plane path (5-way AND per 32 nodes) */
  int64_t resorts;       /* sorted-walk index builds (greedy) */
  int64_t fit_runs_lds;  /* fit-mask launches on the LDS digit-plane path (any cardinality) */
  int64_t fit_runs_sets; /* ... bit-plane launches that swept more than one plane set */
  int64_t walk_rounds;   /* greedy sorted walk: 1024-entry rounds walked, summed over groups */
  int64_t walk_overlay;  /* greedy sorted walk: overlay entries evaluated, summed over groups */
  int64_t walk_groups;   /* greedy sorted walk: group blocks launched */
  int64_t walk_prepass;  /* greedy sorted walk: round summaries read (rounds x groups) */
  double walk_ms;        /* walk kernel time by hipEvents, only when PE_WALK_EVENTS=1 in the environment */
  int64_t walk_pend_updates; /* greedy sorted walk: node updates applied while a side-stream index rebuild
                                was pending (written into both index sets' overlays) */
  int64_t xchg_zc_windows;   /* multi-rank greedy windows exchanged zero-copy through the shared-memory
                                exchange's registered segment (no host copy, no host barrier) */
  /* (ABI 6) the host exchange's cost, summed over windows: time its thread waited for the ranks'
     lists (zero-copy: spinning on peers' group signals; copying: inside the all-gather callback) and
     time it spent merging them on the host (zero-copy windows) */
  double xchg_wait_ms;
  double xchg_merge_ms;
  /* (ABI 7) aggregation calls above 8192 jobs (the chunked path): segments packed, how many of them crossed with
     narrowed request records (value >> per-key shift in 32 bits), and the packed bytes that crossed to
     the device, cumulative */
  int64_t agg_segments;
  int64_t agg_narrow_segments;
  int64_t agg_wire_bytes;
} pe_stats;

int pe_abi_version(void);
/* RCCL unique id for a sharded context (call on rank 0, broadcast the bytes to every rank). */
int pe_comm_id(uint8_t out[PE_COMM_ID_BYTES]);
/* With a comm_id, pe_create waits for the RCCL communicator at most PE_RCCL_INIT_TIMEOUT_S seconds
 * (environment, default 120) and returns PE_ERCCL past that bound.  The abandoned set-up keeps
 * running on a detached thread (RCCL's bootstrap cannot be cancelled), so peers that arrive late may
 * still get a communicator whose collectives would hang.  PE_ERCCL on ANY rank is therefore a
 * collective decision: every rank must destroy its context (and, if it goes on, create a new one
 * with a host `exchange` or a fresh comm_id), as bench.py does through its gloo vote.  A process
 * that abandoned a set-up should leave with _exit(). */
int pe_create(const pe_config* cfg, pe_ctx** out);
void pe_destroy(pe_ctx* ctx);
const char* pe_last_error(const pe_ctx* ctx); /* valid until the next call on ctx */

/* Inventory: caller-owned host SoA [4][n] (row d = dim d) of the GLOBAL inventory; the context
 * keeps its shard [rank*n/world, (rank+1)*n/world) device-resident.  residual = cap - used. */
int pe_load_nodes(pe_ctx* ctx, int64_t n, const int64_t* cap, const int64_t* used, const uint32_t* labels,
                  const int32_t* island);
int pe_reset_residuals(pe_ctx* ctx); /* residual := cap - used (device-side copy) */
/* Incremental inventory ingestion (Node list/watch -> SoA deltas).  The
 * loaded inventory is a table of n_total slots; the caller (the Node informer's event handler)
 * keeps the node-name -> slot map and a free-slot list, so an added node takes a free slot, an
 * updated node rewrites its slot and a deleted node empties it.  Per update i:
 *   op[i] = PE_NODE_SET:    cap[i][4], used[i][4], labels[i], island[i] replace slot slots[i]; its
 *                           residual (and the pe_reset_residuals snapshot) becomes cap - used,
 *                           replacing whatever placements had taken from it
 *   op[i] = PE_NODE_REMOVE: the slot is empty (nothing fits it, no labels, island -1)
 * Later entries for the same slot win.  Every rank of a sharded context gets the whole batch and
 * scatters the slots of its own shard on the device.  The batch is validated before anything is
 * applied (slot out of range, unknown op, negative capacity/usage: PE_EINVAL, nothing changes).
 * labels / island may be NULL (0 / -1). */
enum { PE_NODE_SET = 0, PE_NODE_REMOVE = 1 };
int pe_update_nodes(pe_ctx* ctx, int64_t n, const int64_t* slots, const uint8_t* op, const int64_t* cap /*[n][4]*/,
                    const int64_t* used /*[n][4]*/, const uint32_t* labels, const int32_t* island);
int pe_shard_range(const pe_ctx* ctx, int64_t* begin, int64_t* end);
/* Ranks of the context's RCCL communicator (ncclCommCount); 0 when the shards exchange through the
 * host callback, or an unsharded context was created without a comm_id. */
int pe_comm_ranks(const pe_ctx* ctx, int32_t* nranks);
int pe_read_residuals(pe_ctx* ctx, int64_t* res_out /* [4][end-begin] of this shard */);

/* Batched PodGroup MinResources (one job per lane on the GPU).
 *   groups of job j: [job_group_off[j], job_group_off[j+1]); containers of group g:
 *   [group_cont_off[g], group_cont_off[g+1]); cont_req [C][4], cont_flags [C].
 *   V1: groups in CalcPGMinResources order (priority desc; ties: type name asc), group_replicas
 *       -1 = nil, only PE_KIND_CONTAINER records count, pods counted until min_member[j];
 *       out_members = pods counted.
 *   V2: group = runtime.Info TotalRequests entry with its pod's containers (kueue formula),
 *       out_members = sum of replicas (Go int32 wrap-around), min_member ignored (may be NULL).
 * Outputs per job: out_min_res[j][4], out_present[j] (bit d = key d present), out_members[j],
 * out_overflow[j] (1 = int64 overflow: the reference would have switched to inf.Dec; that job's
 * out_min_res values are then defined as 0, its presence bits and members are still exact).
 * Returns PE_EOVERFLOW if any job overflowed (outputs still written).  A negative request is
 * PE_EINVAL (the first offending index in pe_last_error); a large batch streams to the device in
 * chunks, so the outputs of jobs before the offending chunk may then be written. */
int pe_pg_min_resources(pe_ctx* ctx, int32_t mode, int64_t n_jobs, const int32_t* job_group_off,
                        const int32_t* min_member, const int32_t* group_replicas, const int32_t* group_cont_off,
                        const int64_t* cont_req, const uint8_t* cont_flags, int64_t* out_min_res,
                        uint8_t* out_present, int32_t* out_members, uint8_t* out_overflow);

/* (ABI 7) The same aggregation over a per-call KEY TABLE: any ResourceName the reference sums
 * (util.go:80-103 AddResourceList; coscheduling.go:112-116), not only the four engine dimensions --
 * hugepages-2Mi, rdma/hca, several accelerator names, cpu finer than 1m.  The caller numbers the
 * call's distinct keys 0..n_keys-1 (n_keys <= PE_MAX_KEYS; a batch with more keys takes one call
 * per key slice: keys never interact) and gives each key a decimal scale s_k of its choosing:
 * cont_req[c][k] is container c's quantity of key k as an exact int64 count of 10^s_k units (e.g.
 * s = -9 for "1500u" cpu = 1500000 x 1e-9; bytes at s = 0).  The engine sums the integers per key,
 * exactly as pe_pg_min_resources does per dimension, and the caller reads result k back at s_k.
 * A value with no exact int64 at s_k, or a sum that overflows int64 (out_overflow), is what Go
 * would hold in inf.Dec: the caller's fallback to the reference is for those jobs only.
 *   cont_flags[c] = presence bits 0..n_keys-1 (keys with value 0 are present) | kind << PE_KEYS_KIND_SHIFT
 *   out_min_res[J][n_keys], out_present[J] (bit k = key k present), out_members / out_overflow as above.
 * Other bits in cont_flags are PE_EINVAL. */
#define PE_MAX_KEYS 16
#define PE_KEYS_KIND_SHIFT 16
int pe_pg_min_resources_keys(pe_ctx* ctx, int32_t mode, int64_t n_jobs, int32_t n_keys, const int32_t* job_group_off,
                             const int32_t* min_member, const int32_t* group_replicas, const int32_t* group_cont_off,
                             const int64_t* cont_req, const uint32_t* cont_flags, int64_t* out_min_res,
                             uint16_t* out_present, int32_t* out_members, uint8_t* out_overflow);

/* What-if feasibility (config 5): bit (j, n) = fit(job j, node n) against the CURRENT residuals
 * of this shard, device-resident.  The kernel picks the fastest exact path for the batch and the
 * device layout follows it (pe_fit_mask_layout):
 *   PE_MASK_NODE_TILES (compare paths): word (j, c) holds nodes 64c..64c+63 (bit n%64) at
 *     ((j / 16) * Wt + c / 4) * 64 + (j % 16) * 4 + c % 4,   Wt = ceil(words_per_row / 4)
 *   PE_MASK_JOB_BITS (dictionary-coded path): word (b, n) holds jobs 64b..64b+63 (bit j%64) for
 *     node n at b * S + n,  S = shard nodes rounded up to 512
 *   PE_MASK_ROWS (bit-plane path, default): row-major, word (j, c) at j * P + c, P =
 *     pe_fit_mask_row_pitch (a whole number of 8192-node blocks, >= ceil(S / 8192) * 128 words;
 *     S = shard nodes; padding bits 0)
 *   PE_MASK_NODE_BLOCKS (bit-plane path, fit_path_mask bit5): word (j, c) at
 *     ((c / 128) * J + j) * 128 + c % 128, i.e. per 8192-node block a [J][128]-word slab
 * All layouts are written as whole 128-B lines.  pe_fit_mask_rows always hands rows back
 * row-major [n_rows][words_per_row].  Counts are per job over this shard (sum across shards).
 * One-shot form: upload + compute + counts to host; *dev_mask receives the device pointer. */
int pe_fit_mask(pe_ctx* ctx, int64_t n_jobs, const int64_t* req /*[j][4]*/, const uint32_t* need,
                int64_t* out_feasible_count, const uint64_t** dev_mask, int64_t* words_per_row);
/* Staged form (device-resident inputs, used by the benchmark): */
int pe_jobs_upload(pe_ctx* ctx, int64_t n_jobs, const int64_t* req, const uint32_t* need);
int pe_fit_mask_run(pe_ctx* ctx); /* asynchronous on the context stream */
int pe_fit_counts(pe_ctx* ctx, int64_t* out_feasible_count); /* synchronizes */
int pe_fit_mask_rows(pe_ctx* ctx, int64_t row0, int64_t n_rows, uint64_t* out /*[n_rows][words_per_row]*/);
enum { PE_MASK_NODE_TILES = 0, PE_MASK_JOB_BITS = 1, PE_MASK_NODE_BLOCKS = 2, PE_MASK_ROWS = 3 };
int pe_fit_mask_layout(const pe_ctx* ctx, int32_t* layout);
/* u64 words between consecutive job rows of the device mask in the PE_MASK_ROWS layout (0 for
 * the other layouts). */
int pe_fit_mask_row_pitch(const pe_ctx* ctx, int64_t* words);

/* Greedy best-fit all-or-nothing gang placement.  Jobs in (priority
 * desc, index asc) order, groups of a job in the given order, pods of a group identical.
 *   job_group_off[J+1], priority[J], group_count[G] (pods to place), group_req[G][4],
 *   group_need[G] (required label bits).
 * out_pod_node[sum(group_count)]: GLOBAL node id per pod slot (groups in input order), -1 = none.
 * out_job_status[J]: PE_JOB_PLACED / PE_JOB_UNSCHEDULABLE.  Residuals are updated in place
 * (successful placements stay; failed jobs are rolled back).  Every rank of a sharded context
 * must make the same call; all ranks return the same placements.  group_need bit 31
 * (PE_NEED_ISLAND) makes the group an island group (see PE_LABEL_ISLAND).
 * RCCL transport: a window whose all-gather does not complete within PE_RCCL_TIMEOUT_S seconds
 * (environment, default 60; a peer lost mid-batch) makes the call return PE_ERCCL; the context's
 * communicator is then aborted (ncclCommAbort, on a thread of its own: the call returns at once)
 * and every later sharded call on the context returns PE_ERCCL -- destroy it and rebuild (e.g. on a
 * pe_host_exchange), as bench.py does.  The host exchange's bound is PE_HX_TIMEOUT_S. */
int pe_place_greedy(pe_ctx* ctx, int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority,
                    const int32_t* group_count, const int64_t* group_req, const uint32_t* group_need,
                    int32_t* out_pod_node, int32_t* out_job_status);

/* ---- Host resolver: the host half of pe_place_greedy, exposed on its own so a caller (or a
 * CPU test) can drive the windowed protocol with candidate blobs it obtained elsewhere, e.g. one
 * blob per shard gathered over any transport.  No device is touched.
 * Window blob layout (what the device merge kernel writes, per shard, per window group):
 *   16-B header {int32 n; int32 flags; uint64 limit} + K records of 48 B
 *   {uint64 key; int64 res[4]; uint64 labels}; shards are concatenated.
 * Updates are returned as [n][5] int64 {global node id, res[0..3]} (absolute residuals).
 * An island group's (PE_NEED_ISLAND) lists must be scanned for group_count x request. */
typedef struct pe_resolver pe_resolver;
int pe_resolver_create(int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority,
                       const int32_t* group_count, const int64_t* group_req, const uint32_t* group_need,
                       pe_resolver** out);
void pe_resolver_destroy(pe_resolver* r);
/* (ABI 7) Inventory size for the id checks below (default PE_MAX_NODES).  Blobs may arrive over any
 * transport, so pe_resolver_resolve* validate every header and record before the resolver moves: a
 * header count outside [0, topk], a listed node id >= n_nodes or keys not strictly ascending within a
 * shard list (and a seed id >= n_nodes) return PE_EINVAL with no update written and the resolver's
 * position unchanged -- never a read past the blob. */
int pe_resolver_set_nodes(pe_resolver* r, int64_t n_nodes);
int pe_resolver_done(const pe_resolver* r); /* 1 when every job is decided */
int pe_resolver_next_window(pe_resolver* r, int32_t max_groups, int64_t max_pods, int32_t* out_groups,
                            int32_t* out_n);
int pe_resolver_resolve(pe_resolver* r, int32_t n_groups, const int32_t* groups, const uint8_t* blob,
                        int32_t n_shards, int32_t topk, int64_t* out_updates, int64_t max_updates,
                        int64_t* out_n_updates, int32_t* out_consumed);
/* Pipelined form (what pe_place_greedy does internally): the blob's lists were scanned on a
 * snapshot that misses some changes; seeds [n_seeds][6] = {global node id, res[0..3], labels} are
 * every node changed since that snapshot, with its CURRENT state (e.g. the previous window's
 * updates).  They count as dirty for the whole window and are scored by a helper thread ahead of
 * the resolution.  Updates returned as by pe_resolver_resolve (nodes this window changed). */
int pe_resolver_resolve_seeded(pe_resolver* r, int32_t n_groups, const int32_t* groups, const uint8_t* blob,
                               int32_t n_shards, int32_t topk, int64_t n_seeds, const int64_t* seeds,
                               int64_t* out_updates, int64_t max_updates, int64_t* out_n_updates,
                               int32_t* out_consumed);
int pe_resolver_results(const pe_resolver* r, int32_t* out_pod_node, int32_t* out_job_status);

int pe_synchronize(pe_ctx* ctx);
void* pe_stream(pe_ctx* ctx); /* hipStream_t the context launches on (for event timing) */
int pe_get_stats(const pe_ctx* ctx, pe_stats* out);
int pe_reset_stats(pe_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* PLACEMENT_H_ */
