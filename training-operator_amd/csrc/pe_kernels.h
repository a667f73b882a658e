// Device-side building blocks of libplacement (gfx950).  Host code in pe_engine.cpp launches
// these through the wrappers below; nothing here is part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pe {

constexpr int D = 4;                    // cpu milli, memory B, gpu count, ephemeral-storage B
constexpr uint64_t SCORE_MAX = (1ull << 40) - 1;
constexpr uint64_t NO_KEY = ~0ull;
constexpr int64_t NEVER = INT64_MIN;    // residual of padding nodes: nothing fits

// One request vector (a pod template / a fit-mask job), 64 B so a wave loads it with one
// scalar s_load_dwordx16 and it never straddles two scalar-cache lines.
struct alignas(64) ReqRec {
  int64_t q[D];
  uint32_t need;
  uint32_t pad_[7];
};
static_assert(sizeof(ReqRec) == 64, "ReqRec must be 64 B");

// Exact 32-bit form of a request batch: q32[d] = q[d] >> shift[d] where 2^shift[d] divides every
// request of the batch in dim d, so  q <= r  <=>  q32 <= sat32(floor(r / 2^shift))  (r's floor
// loses nothing because q is a multiple of 2^shift; r >= 2^31 saturates, r < 0 becomes -1).
struct alignas(32) ReqRec32 {
  int32_t q[D];
  uint32_t need;
  uint32_t pad_[3];
};
static_assert(sizeof(ReqRec32) == 32, "ReqRec32 must be 32 B");

// Per-group candidate list shipped to the host resolver: a header + K keys (ascending).  The keys
// carry the node id (low 24 bits); the host reads the node's residual snapshot from its own mirror
// of the inventory, so the device ships 8 B per candidate instead of a 48-B record.
struct CandHdr {
  int32_t n;       // valid keys (ascending)
  int32_t flags;   // merge: bit0 = overflowed LDS, list truncated to the exact minimum; signalled walk: the window generation, written last
  uint64_t limit;  // every clean node with key < limit is in the list
};
static_assert(sizeof(CandHdr) == 16, "CandHdr must be 16 B");
// CandHdr.n values that are not a count: a zero-copy exchange wait timed out (limit = the xwait status),
// and a merged group one of whose shard lists was corrupt (a shard header with n outside [0, K]).  The
// host resolver raises on either (pe_resolver.cpp parse_group_keys); it never reads past a list.
constexpr int32_t CAND_TIMEOUT = -1;
constexpr int32_t CAND_CORRUPT = -2;

__host__ __device__ inline size_t cand_group_bytes(int K) { return sizeof(CandHdr) + (size_t)K * sizeof(uint64_t); }

// ---- geometry shared by host and device
constexpr int FM_CH = 4;       // fit mask: 64-node chunks per wave tile (256 nodes in VGPRs)
constexpr int FM_JT = 256;     // fit mask: jobs per wave
constexpr int SC_M = 16;       // scan: nodes per lane (wave span 1024 nodes)
constexpr int SC_GT = 4;       // scan: groups per wave (top-2 state in registers)
constexpr int SC_SPAN = 64 * SC_M;
constexpr int SC_WPB = 16;     // scan: waves (group tiles) per block, all on one node span
constexpr int MG_CAP = 16384;  // merge / walk: LDS candidate capacity per group (128 KiB of keys)
constexpr int MG_THREADS = 1024;
constexpr int MG_SEL = 1024;   // merge: keys kept after the histogram cut (sorted instead of all)

// ---- PodGroup aggregation call path (pe_pg_min_resources).  The host packs the batch into
// SEGMENTS in one pinned, device-mapped staging buffer: a segment holds up to AGG_SEG_JOBS
// consecutive jobs with their groups and containers, offsets rebased to the segment, every
// section 16-B aligned, so one block copies its whole segment into LDS with one round trip of
// coalesced 16-B loads and runs one job per lane from LDS -- reading the pinned buffer over PCIe for
// calls up to 8192 jobs, a device copy (one DMA per chunk) for larger ones.  Outputs go straight into
// a pinned output buffer in the caller's layout.  A segment larger than AGG_SEG_BYTES (one job with
// very many groups / containers) is read in place.
constexpr int AGG_SEG_JOBS = 256;
constexpr int64_t AGG_SEG_BYTES = 48 * 1024;
struct AggSegHdr {
  int64_t j0;            // first job of the segment (index in the call's batch)
  int32_t nj, ng, nc;    // jobs, groups, containers
  int32_t g0, c0;        // the segment's first group / container: its jgo / gco sections hold the caller's
                         // absolute offsets (copied as they are), the kernel rebases
  int32_t narrow;        // 1: the request section is narrowed (agg_seg_layout), 0: nc x nd i64
};
static_assert(sizeof(AggSegHdr) == 32, "AggSegHdr must be 32 B");
__host__ __device__ inline int64_t agg_r16(int64_t x) { return (x + 15) & ~int64_t(15); }
// Key layout of a call: nd int64 values per container record and per job result, fb bytes of flags
// per container.  {4, 1}: the fixed engine dimensions (pe_pg_min_resources: presence bits 0-3 | kind
// << 4, u8 presence out); {4 | 8 | 16, 4}: a per-call key table (pe_pg_min_resources_keys: presence
// bits 0-15 | kind << 16, u16 presence out), n_keys rounded up to nd.
struct AggKeys {
  int nd = 4;
  int fb = 1;
};
constexpr int AGG_MAX_KEYS = 16;
// byte offsets of the sections in a segment: [0] jgo (nj+1 i32, absolute group ids), [1] min_member
// (nj i32, V1 only), [2] replicas (ng i32), [3] gco (ng+1 i32, absolute container ids), [4] req
// (nc x nd i64; narrowed: 16 shift bytes, then nc x nd u32), [5] flags (nc x fb), [6] = size.
// A narrowed request section holds value >> shift[key] in 32 bits, shift[key] = the fewest trailing
// zero bits of the key's values in the segment -- exact whenever every value of a key spans <= 32 bits
// above its shift (quantities in canonical units are: milli-cpu, memory in multiples of 2^k bytes),
// and half the bytes over PCIe.  The host narrows a segment only when it can, and when it pays.
__host__ __device__ inline int64_t agg_req_bytes(int64_t nc, int nd, bool narrow) {
  return narrow ? 16 + agg_r16(nc * 4 * nd) : nc * 8 * nd;
}
__host__ __device__ inline void agg_seg_layout(int64_t nj, int64_t ng, int64_t nc, bool v1, int64_t off[7],
                                               AggKeys ak = AggKeys{}, bool narrow = false) {
  off[0] = (int64_t)sizeof(AggSegHdr);
  off[1] = off[0] + agg_r16((nj + 1) * 4);
  off[2] = off[1] + (v1 ? agg_r16(nj * 4) : 0);
  off[3] = off[2] + agg_r16(ng * 4);
  off[4] = off[3] + agg_r16((ng + 1) * 4);
  off[5] = off[4] + agg_req_bytes(nc, ak.nd, narrow);
  off[6] = off[5] + agg_r16(nc * ak.fb);
}
// Output buffer layout (the caller's arrays back to back): res [J][nd] i64, members [J] i32,
// present [J] (u8, or u16 for a key table), overflow [J] u8, each 16-B aligned.
__host__ __device__ inline void agg_out_layout(int64_t J, int64_t off[4], AggKeys ak = AggKeys{}) {
  off[0] = 0;
  off[1] = agg_r16(J * 8 * ak.nd);
  off[2] = off[1] + agg_r16(J * 4);
  off[3] = off[2] + agg_r16(J * (ak.fb == 1 ? 1 : 2));
}

// ---- launch wrappers (return hipError_t of the launch)
// Segmented aggregation: nseg segments; segment s spans blob[seg_off[s], seg_off[s+1]) (seg_off
// may be NULL for one segment of nbytes0 bytes at blob[0]).  out = output buffer (agg_out_layout,
// J jobs).  flag != NULL (latency launches): every block publishes its outputs system-wide and counts
// itself in done_ctr (device memory, 0 between launches; unused for one block); the last one resets
// it and stores flag_val (release, system scope) -- the host waits on the flag, not on the stream.
hipError_t launch_pg_agg_segments(hipStream_t s, int mode, const uint8_t* blob, const int64_t* seg_off, int64_t nseg,
                                  int64_t nbytes0, uint8_t* out, int64_t J, uint32_t* flag, uint32_t flag_val,
                                  uint32_t* done_ctr, AggKeys ak = AggKeys{});
// One segment of <= AGG_KARG_BYTES (a multiple of 16) passed by value in the kernel arguments.
constexpr int64_t AGG_KARG_BYTES = 512;   // (a 3 KB argument block cost ~1.5 us more per launch call)
struct AggKarg {
  alignas(16) uint8_t b[AGG_KARG_BYTES];
};
hipError_t launch_pg_agg_karg(hipStream_t s, int mode, const AggKarg& blob, int64_t nbytes, uint8_t* out, int64_t J,
                              uint32_t* flag, uint32_t flag_val, AggKeys ak = AggKeys{});
hipError_t launch_pg_min_resources(hipStream_t s, int mode, int64_t n_jobs, const int32_t* job_group_off,
                                   const int32_t* min_member, const int32_t* group_replicas,
                                   const int32_t* group_cont_off, const int64_t* cont_req,
                                   const uint8_t* cont_flags, int64_t* out_res, uint8_t* out_present,
                                   int32_t* out_members, uint8_t* out_overflow);

// Device mask layout (tile-major, so every store writes whole 128-B lines): tiles of 16 jobs x 4
// words (256 nodes); word (j, c) -- bit n%64 of chunk c = n/64 = fit(job j, local node n) -- sits at
//   ((j / 16) * Wt + c / 4) * 64 + (j % 16) * 4 + c % 4,      Wt = ceil(ceil(Ns/64) / 4).
// Rows are padded to FM_JT, chunks to a multiple of 4; pe_fit_mask_rows returns row-major.
__host__ __device__ inline int64_t fm_word_index(int64_t j, int64_t c, int64_t Wt) {
  return ((j >> 4) * Wt + (c >> 2)) * 64 + (j & 15) * 4 + (c & 3);
}
hipError_t launch_fit_mask(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels,
                           int64_t Ns, int64_t Wt, const ReqRec* jobs, int64_t J, int64_t tiles_per_wave,
                           uint64_t* mask, unsigned long long* counts);

// 32-bit path: residuals compressed per fit run (res32 = sat32(res >> shift)), then the same kernel
// with v_cmp_le_i32 instead of the (quarter-rate) v_cmp_le_i64.
hipError_t launch_compress_res(hipStream_t s, const int64_t* res, int32_t* res32, int64_t stride, int64_t Ns,
                               const int* shift);
hipError_t launch_fit_mask32(hipStream_t s, const int32_t* res32, int64_t stride, const uint32_t* labels,
                             int64_t Ns, int64_t Wt, const ReqRec32* jobs, int64_t J, int64_t tiles_per_wave,
                             uint64_t* mask, unsigned long long* counts);

// ---- dictionary-coded SWAR path (fit mask).  Per batch the host ranks the distinct request
// values of each dimension (and a chain of label needs); field f of a node's 32-bit code word is
// (#batch values <= residual) + guard bit, the job's word holds its values' ranks.  Then
//   fit(j, n)  <=>  ((X[n] - C[j]) | ~M) == 0xFFFFFFFF   (every field keeps its guard bit)
// exactly, for all 4 dimensions and the labels at once.
constexpr int CODE_FIELDS = 5;   // cpu, memory, gpu, ephemeral, label-chain
constexpr int CODE_MAXV = 128;   // distinct values per field the device tables hold
struct CodeSpec {
  int off[CODE_FIELDS];
  int width[CODE_FIELDS];       // SWAR: code bits + 1 guard bit; thermometer: nvals bits
  int nvals[CODE_FIELDS];
  uint32_t guard;               // SWAR: M (guard bits); thermometer: unused
  int therm;                    // 1: thermometer fields, fit <=> (X | ~Y) == ~0 (3 VALU per 64 evals)
};
constexpr int FC_CH = 16;       // coded fit: 64-node chunks per wave tile (X in 16 VGPRs)
constexpr int FC_JT = 64;       // coded fit: jobs per wave (one 64-bit word per node)

// vals: [4][CODE_MAXV] sorted int64 request values; needs: [CODE_MAXV] label chain (inclusion order)
hipError_t launch_encode_nodes(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                               int64_t n_pad, CodeSpec spec, const int64_t* vals, const uint32_t* needs, uint32_t* X);
// Coded-path mask layout (bits over jobs): word (b, n) = jobs 64b..64b+63 at node n (bit j%64),
// stored at b * node_stride + n, node_stride = ceil(Ns/512)*512.
// therm = 0: jcode = C (ranks), k = ~M;   therm = 1: jcode = ~Y (one bit per field cleared), k unused
hipError_t launch_fit_mask_coded(hipStream_t s, int therm, const uint32_t* X, int64_t Ns, int64_t node_stride,
                                 const uint32_t* jcode, uint32_t not_guard, int64_t J, int64_t tiles_per_wave,
                                 uint64_t* mask, unsigned long long* counts);

// ---- bit-plane path (fit mask).  Per batch the host lists the distinct request values of each
// dimension and the distinct label needs; plane p of a node is one predicate, evaluated exactly in
// int64 when the planes are encoded:
//   kind d < 4:  res[d][n] >= val        kind 4:  (labels[n] & need) == need
// and is stored transposed, 32 nodes per u32 word (padding nodes 0).  A job selects one plane per
// dimension and one for its need, so for 32 nodes at once
//   fit word = P[i0] & P[i1] & P[i2] & P[i3] & P[i4]
// -- two v_bitop3 per 2048 (job, node) pairs per wave instead of one VALU op per 64.
constexpr int PL_MAX = 32;      // planes a batch may use (held in VGPRs, dynamic index via gpr_idx)
constexpr int PL_R = 4;         // u32 node words per lane: one 16-B store per job and lane
constexpr int PL_BLK = 64 * PL_R * 32;   // nodes per wave block (8192)
struct PlaneSpec {
  int32_t n;                    // planes in use
  int32_t kind[PL_MAX];         // 0..3 resource dimension, 4 label need
  int64_t val[PL_MAX];          // request value (kind < 4) or need bits (kind 4)
};
// planes: [nblk][PL_MAX][64 * PL_R] u32; word w of block b covers nodes b*PL_BLK + 32w .. +31
hipError_t launch_encode_planes(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels,
                                int64_t Ns, int64_t nblk, const PlaneSpec& spec, const PlaneSpec* spec_d,
                                uint32_t* planes, unsigned long long* zero = nullptr,
                                int64_t n_zero = 0);   // spec_d: the same spec on the device; + zero[0..n_zero)
// jcode[j] = 5 fields of 7 bits (dims 0..3 at bits 0/7/14/21, need at bit 32), each 4 x the plane index.  Mask block-major:
// u32 word w of row j (nodes 32w..32w+31) at (w / 256 * J + j) * 256 + w % 256, i.e. per 8192-node
// block a [J][1 KiB] slab.
hipError_t launch_fit_mask_planes(hipStream_t s, const uint32_t* planes, int64_t nblk, const uint64_t* jcode,
                                  int64_t J, int64_t jobs_per_wave, uint32_t* mask, unsigned long long* counts);
// Row-major form (the default): nblk x R persistent waves, one per SIMD, R job phases; wave
// (blk, r) takes jobs r, r+R, ...; u32 word w of row j at j * nblk * 256 + w.  jcode and counts are
// phase-major: entry r * Jr + i belongs to job r + R * i (Jr = ceil(J / R) rounded up to 4), so
// every wave reads and counts a contiguous run.
// pitch_blk >= nblk: mask row pitch in 8192-node blocks (1 KiB each; words past nblk are not written)
// unit_ctr (nblk zeroed counters, or nullptr): the waves of a block share its (phase, 64-job batch)
// units through the block's counter instead of each taking its own phase -- same rows, same counts.
hipError_t launch_fit_mask_planes_rows(hipStream_t s, const uint32_t* planes, int64_t nblk, const uint64_t* jcode,
                                       int64_t J, int64_t R, uint32_t* mask, unsigned long long* counts,
                                       int64_t pitch_blk, unsigned long long* unit_ctr = nullptr);
// Plane-set form (batches with more than PL_MAX distinct request values), all sets in one launch
// each: encode writes set t's planes at planes + t * nblk * PL_MAX * 256; the sweep has the rows
// kernel's grid (R phases common to all sets); set t's codes and counts start at meta[3t] (phase-
// major, stride meta[3t+2], meta[3t+1] jobs), each code carrying its job's mask row in bits 40-63.
hipError_t launch_encode_planes_sets(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels,
                                     int64_t Ns, int64_t nblk, const PlaneSpec* specs, int nsets, uint32_t* planes);
hipError_t launch_fit_mask_planes_sets(hipStream_t s, const uint32_t* planes, int64_t nblk, const uint64_t* jcode,
                                       const int64_t* meta, int nsets, int64_t R, uint32_t* mask,
                                       unsigned long long* counts, int64_t pitch_blk);

// ---- LDS digit-plane path (fit mask, any number of distinct request values).  Per dimension the
// host ranks the batch's distinct request values v_1 < ... < v_m; a job asks rank c (v_c = its
// request), a node has rank R = #{v_i <= residual}, and  q <= res  <=>  c <= R  exactly.  R >= c is
// decided digit by digit (mixed radix, most significant first): with threshold planes
// GE_k(v) = [digit_k(R) >= v],
//     [R >= c] = GE_top(c_top + 1) | (GE_top(c_top) & ( ... GE_0(c_0) ... ))
// so a field of m values costs L digit levels (m^(1/L)-ish planes each) and 2L - 1 plane reads per
// job; a single-level field is one plane per value.  Label needs are one plane each, and
// dimensions with a single requested value are folded into those.  Single-level fields may be
// CROSSED with the needs instead: one plane per (need, value of each crossed field), the AND of the
// label test and the crossed thresholds, so the job reads one plane for all of them.  The workgroup builds its node
// block's planes in LDS (scatter of the equality bits + suffix OR), then streams the jobs: per job
// a handful of LDS reads, AND/AND-OR combines, one store of the block's slice of the mask row.
constexpr int LD_MAXF = 4;        // digit fields (dimensions with >= 2 distinct values)
constexpr int LD_MAXL = 4;        // digit levels per field
constexpr int LD_MAXNEED = 64;    // distinct label needs
constexpr int LD_CODE = 16;       // u16 plane indices per job: field f's levels at lds_field_off(f) + k, then
                                  // the need plane at lds_need_slot (right after the fields: one readlane fewer)
constexpr int LD_NEED_SLOT = 15;  // the last slot: at most 15 field entries
// First code entry of field fi when the fields are ordered N4 four-level, N3 three-level, N2 two-level,
// then one-level (the kernel's template shape; the sum of the levels must stay <= LD_NEED_SLOT).
__host__ __device__ constexpr int lds_field_off(int fi, int n4, int n3, int n2) {
  return fi <= n4                ? 4 * fi
         : fi <= n4 + n3         ? 4 * n4 + 3 * (fi - n4)
         : fi <= n4 + n3 + n2    ? 4 * n4 + 3 * n3 + 2 * (fi - n4 - n3)
                                 : 4 * n4 + 3 * n3 + 2 * n2 + (fi - n4 - n3 - n2);
}
// The need plane's code entry: the first one after the fields, so that it shares the last field's
// dword (the kernel reads one dword per readlane) instead of sitting alone in the code's last dword.
__host__ __device__ constexpr int lds_need_slot(int n4, int n3, int n2, int n1) {
  return 4 * n4 + 3 * n3 + 2 * n2 + n1;
}
constexpr int LD_THREADS = 1024;  // 16 waves per workgroup, one node block per workgroup
struct LdsSpec {
  int32_t nf;                       // digit fields
  int32_t dim[LD_MAXF];             // resource dimension of field f
  int32_t L[LD_MAXF];               // digit levels of field f
  // level slot k (0 = least significant): digit = (R / div) % mod (mod 0 = no modulus); threshold
  // planes GE(v) for v in [vlo, vlo + nv) at planes pbase + v - vlo
  uint32_t div[LD_MAXF][LD_MAXL];
  uint32_t mod[LD_MAXF][LD_MAXL];
  int32_t pbase[LD_MAXF][LD_MAXL];
  int32_t vlo[LD_MAXF][LD_MAXL];
  int32_t nv[LD_MAXF][LD_MAXL];
  int32_t nneed, need_pbase, nplanes, nfold;
  // crossed single-level fields (ranks rows nf .. nf + nx - 1, dim / voff / m at nf + i): need plane
  // need_pbase + i * xprod + sum_f c_f * xstride[f] = need i AND rank_f >= c_f + 1 for every crossed f
  int32_t nx, xprod;
  int32_t xstride[LD_MAXF];
  uint32_t needs[LD_MAXNEED];
  int32_t fold_dim[D];              // single-valued dimensions folded into the need planes:
  int64_t fold_val[D];              // a node passes them iff res[fold_dim] >= fold_val
  int64_t voff[LD_MAXF];            // field f's sorted distinct values at vals[voff[f] .. voff[f] + m[f])
  int64_t m[LD_MAXF];
};
// ranks: [nf + nx][npad] u32 (npad = node blocks x S, padding nodes 0); aux: [2][npad] u32, row 0 = 1 for
// a shard node passing the folded dimensions (else 0), row 1 = its labels (0 for padding).
// spec: device copy.
hipError_t launch_node_ranks(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                             int64_t npad, const LdsSpec* spec, const int64_t* vals, uint32_t* ranks, uint32_t* aux);
// S = 2048 * W nodes per workgroup block (W u32 words per lane per plane); grid = nblk x R
// workgroups, wave w of workgroup (blk, r) takes jobs j = r + R (w + 16 t).  codes: LD_CODE u16 per
// job, job j's at position (r * 16 + w) * Tpad + t (Tpad >= the longest run, a multiple of 16).
// Mask row-major (PE_MASK_ROWS): row j at mask + j * pitch_bytes, block blk's S/8 bytes at + blk * S/8.
// slots: [R * 16 * Tpad] u32 count slots (zeroed by the caller), slot (r * 16 + w) * Tpad + t = job
// r + R (w + 16 t); launch_lds_counts turns them into per-job u64 counts through the slots' rows.  spec: device copy;
// nplanes = spec->nplanes.  shape = {N4, N3, N2, N1}: fields 0 .. N4-1 have 4 digit levels (W >= 2
// only), the next N3 three, then N2 two, the last N1 one.  The mask has J rows.
hipError_t launch_fit_mask_lds(hipStream_t s, int W, const int shape[4], const LdsSpec* spec, int nplanes,
                               const uint32_t* ranks, int64_t npad, const uint32_t* aux, int64_t nblk,
                               const uint16_t* codes, int64_t J, int64_t R, int64_t Tpad, int64_t pitch_bytes,
                               uint8_t* mask, uint32_t* slots, uint32_t* units = nullptr);   // units: nblk zeroed counters
hipError_t launch_lds_counts(hipStream_t s, const uint32_t* slots, const uint32_t* rows, int64_t nslots,
                             unsigned long long* counts);

// kn / lo: the node-only score terms of prep_nodes (K(n) = (S(n) << 24) | gid, lo20(r1), lo24(r3)),
// kept current by apply; see pe_kernels.hip node_prep for the exactness argument.
hipError_t launch_prep_nodes(hipStream_t s, const int64_t* res, int64_t stride, int64_t Ns, uint64_t id_base,
                             uint64_t* kn, uint32_t* lo /* [2][stride] */);
hipError_t launch_scan(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, const uint64_t* kn,
                       const uint32_t* lo, int64_t Ns, uint64_t id_base, const ReqRec* groups, int Wg, uint64_t* cand,
                       int32_t* cnt, uint64_t* bound, int nwaves);

hipError_t launch_merge(hipStream_t s, const uint64_t* cand, const int32_t* cnt, const uint64_t* bound,
                        int nwaves, int K, uint8_t* out, int Wg);

// ---- sorted walk (the default greedy window path).  The shard's nodes sorted by the node-only
// key K(n) = (S(n) << 24) | gid, copied into sorted SoA order and summarised per 1024-entry round
// (max residual per dimension, OR of labels, first key).  A fitting node has S(n) >= s(q), and its
// key is K(n) - ((s(q) + borrows) << 24) with borrows <= 2, so a group walks the rounds from the
// first that can hold K >= s(q) << 24 and stops once K + 1 collected keys lie below every key the
// unvisited rounds can produce.  Nodes changed since the sort (apply) and nodes whose terms can
// saturate form the overlay, evaluated in full by every group; their sorted entries are
// invalidated (WK_INVALID).  Negative-residual nodes fit nothing and appear in neither.
constexpr int WK_ROUND = 1024;          // sorted entries per round = walk threads per group
constexpr int WK_MAXR = 16384;          // rounds per shard (PE_MAX_NODES / WK_ROUND)
constexpr uint64_t WK_INVALID = ~0ull;
// Walk steps: one round at a time for the first WK_MULTI_AFTER rounds, then up to WK_MULTI candidate
// rounds per step (their loads in flight together, one barrier and one stop test per step).  Round 5
// (tools/walk_ab.py, interleaved, one box): 4 rounds per step after 4 single ones 43.8-45.7 us per
// launch, 2 after 1 39.1-40.2, 2 after 0 / 2 / 4 39.8-41.1, 3 after 2 41.1-42.1 -- with the stop test
// no longer rescanning every key, finer steps collect fewer surplus keys for the selection.
#ifndef WK_MULTI
#define WK_MULTI 2
#endif
#ifndef WK_MULTI_AFTER
#define WK_MULTI_AFTER 1
#endif
struct WalkIndex {
  uint64_t* sk;        // [Ns] sorted keys (WK_INVALID = not walked)
  int64_t* sr;         // [4][sstride] residuals in sorted order
  uint32_t* sl;        // [Ns] labels in sorted order
  uint32_t* pos;       // [stride] sorted index of each local node (~0u = none)
  uint64_t* rmin;      // [nr] first key of each round (at sort time)
  int64_t* rmax;       // [4][nr] max residual per dimension over the round's valid entries
  uint32_t* ror;       // [nr] OR of the round's labels
  int32_t* ovl;        // [stride] overlay local node ids
  int32_t* ovl_n;      // overlay size
  uint32_t* in_ovl;    // [stride] 1 = in the overlay
  uint32_t* ovl_idx;   // [stride] a node's overlay slot (valid while in_ovl)
  int64_t* ovl_res;    // [4][sstride] residuals by overlay slot (kept current by apply)
  uint32_t* ovl_lab;   // [stride] labels by overlay slot
  uint64_t* ovl_kn;    // [stride] K(n) of each overlay slot's state (node_prep; KEY_SLOW: always evaluated)
  unsigned long long* stat;   // nullable: [0] += rounds walked, [1] += overlay entries, per group
  int64_t sstride, nr;
};
// kin[n] = K(n) of a walkable node (no negative residual, not saturating), else WK_INVALID; the
// saturating ones are appended to the overlay (cleared by the caller beforehand) -- or, with `slow`
// (a rebuild on the side stream, whose overlay only the main stream's applies write), flagged in
// slow[n] for walk_switch to add.
hipError_t launch_walk_prep(hipStream_t s, const int64_t* res, int64_t stride, int64_t Ns, const uint64_t* kn,
                            const uint32_t* labels, uint64_t* kin, const WalkIndex& w, uint32_t* slow = nullptr);
// Takes over an index rebuilt on the side stream (pe_engine walk_resort_async), on the main stream
// once the rebuild is done: every node an apply moved into nx's overlay while it was rebuilt leaves
// nx's sorted walk (its entry may hold a state read mid-update), and the flagged saturating nodes
// join nx's overlay with their current state.
hipError_t launch_walk_switch(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                              const uint32_t* slow, const WalkIndex& nx);
// hipcub radix sort of n u64 keys (temp == nullptr: *temp_bytes = the scratch size needed).
hipError_t sort_keys_u64(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out, int64_t n, hipStream_t s);
// Sorted SoA copy, pos[], round summaries from the sorted keys w.sk.
hipError_t launch_walk_build(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                             uint64_t id_base, const WalkIndex& w);
// Multi-rank window: world gathered shard blobs (key lists) -> one list per group (the K smallest
// keys below the smallest shard limit, limit = the (K+1)-th or that minimum); gen != 0 signals each
// group as the walk does.  world * K <= MG_CAP.
// rank_stride: bytes between the ranks' blocks in gath (0 = Wg x cand_group_bytes(K), back to back; the
// shared-memory exchange's slots are further apart).  xstatus (zero-copy exchange, device word
// written by launch_xwait before it on the stream): nonzero = a rank's lists never arrived, every
// group is written with n = -1 and limit = *xstatus (signalled) instead of a list.
// sys_scope: the lists may sit in host memory other processes write (this kernel always reads so).
hipError_t launch_merge_shards(hipStream_t s, const uint8_t* gath, int world, int Wg, int K, uint8_t* out, uint32_t gen,
                               int64_t rank_stride = 0, const uint64_t* xstatus = nullptr, bool sys_scope = true);
// Zero-copy exchange: one block waits until every rank's header of every group (slot r at gath +
// r * rank_stride) carries in_gen, at most timeout_ticks of wall_clock64 (100 MHz); *xstatus = 0,
// or 1 << 63 | rank << 32 | the generation that rank's slot still held.
constexpr int XW_THREADS = 256;
hipError_t launch_xwait(hipStream_t s, const uint8_t* gath, int world, int Wg, int K, int64_t rank_stride,
                        uint32_t in_gen, int64_t timeout_ticks, uint64_t* xstatus);
// The same merge by rank (merge_ranked_kernel, the default): 256-thread blocks, the lists and the
// merged list in LDS (merge_ranked_lds bytes of dynamic LDS, at most RM_MAX_LDS), a cut of each list
// ranked by lock-step binary searches, no sort.  sys_scope = false: gath is device memory written by
// an earlier kernel of the stream (the RCCL all-gather), read with plain loads.
constexpr int RM_THREADS = 256, RM_MAX_WORLD = 16;
constexpr size_t RM_MAX_LDS = 64 * 1024;
size_t merge_ranked_lds(int world, int K);
hipError_t launch_merge_ranked(hipStream_t s, const uint8_t* gath, int world, int Wg, int K, uint8_t* out, uint32_t gen,
                               int64_t rank_stride = 0, const uint64_t* xstatus = nullptr, bool sys_scope = true);
// Wg empty lists (n = 0, limit = NO_KEY), signalled with gen
hipError_t launch_empty_groups(hipStream_t s, int Wg, int K, uint8_t* out, uint32_t gen);
// Test knob (PE_TEST_STALL_*): one thread that holds the stream for `ticks` of wall_clock64 (100 MHz),
// sleeping between polls -- bounded, so the stream always drains
hipError_t launch_stall(hipStream_t s, int64_t ticks);
// One block per group: overlay + walk, exact top-K keys and limit, same blob as merge.  gen != 0:
// each group's header.flags is set to gen after its keys, n and limit are visible to the host
// (system-scope release; out is pinned host memory the host polls per group).  K_stride: the blob's
// list capacity per group (cand_group_bytes(K_stride) apart; 0 = K), K <= K_stride.
hipError_t launch_walk(hipStream_t s, const ReqRec* groups, int Wg, int K, const WalkIndex& w, const int64_t* res,
                       int64_t stride, const uint32_t* labels, int64_t Ns, uint64_t id_base, uint8_t* out,
                       uint32_t gen = 0, int K_stride = 0);

// upd: [n] records {local node (i64), res[4]} -> res[d][node] = value (absolute)
// (kn, lo nullable: refreshed for the updated nodes when given; w nullable: the updated nodes
// leave the sorted walk and join its overlay; nx nullable: an index being rebuilt on the side
// stream -- the updated nodes join its overlay too, its sorted entries are left to walk_switch)
hipError_t launch_apply(hipStream_t s, int64_t* res, int64_t stride, const int64_t* upd, int64_t n, uint64_t id_base,
                        uint64_t* kn, uint32_t* lo, const uint32_t* labels, const WalkIndex* w,
                        const WalkIndex* nx = nullptr);

// Inventory delta for one slot of this shard (pe_update_nodes): residual written to both the
// live and the reset copy, labels and island replaced.  Slots are unique within a launch.
struct NodeUpd {
  int64_t local;
  int64_t res[D];
  uint32_t labels;
  int32_t island;
};
static_assert(sizeof(NodeUpd) == 48, "NodeUpd must be 48 B");
hipError_t launch_scatter_nodes(hipStream_t s, int64_t* res, int64_t* res0, int64_t stride, uint32_t* labels,
                                int32_t* island, const NodeUpd* upd, int64_t n);

}  // namespace pe
