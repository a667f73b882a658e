// Package hip binds libplacement, the MI355X gang-placement engine (include/placement.h), for the
// training operator.  Mechanically thin on purpose: one Go method per C entry point, Go slices
// pinned for the duration of the call and never retained by C, every non-zero return code turned
// into an error carrying pe_last_error.
//
// This file is the reference-side binding a maintainer adds as pkg/placement/hip.  There is no Go
// toolchain in the build pipeline that produced it (SURVEY.md sec. 0.3), so it is not compiled
// there; tests/test_go_binding.py checks that it calls every pe_* function of the header with the
// header's arity.
//
// Reference interfaces it serves (paths relative to the training-operator repo):
//
//	PGMinResources(ModeV1, ...)  pkg/controller.v1/common/util.go:108 CalcPGMinResources
//	PGMinResources(ModeV2, ...)  pkg/runtime.v2/framework/plugins/coscheduling/coscheduling.go:103-118 Build
//	New / Close                   the plugin instance lifetime, pkg/runtime.v2/framework/plugins/registry.go:32-42
package hip

/*
#cgo LDFLAGS: -lplacement
#include <stdlib.h>
#include "placement.h"

// The Go side cannot hand a Go func to C as a pe_allgather_fn; sharded contexts use RCCL
// (comm_id), which needs no callback, or the library's own shared-memory all-gather (HostExchange).
static pe_allgather_fn hx_allgather_fn(void) { return pe_host_exchange_allgather; }
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"

	corev1 "k8s.io/api/core/v1"
)

// Aggregation modes (PE_MODE_*).
const (
	ModeV1 = int(C.PE_MODE_V1) // CalcPGMinResources: priority order, pods counted up to minMember
	ModeV2 = int(C.PE_MODE_V2) // CoScheduling.Build: sum of Replicas x PodRequests
)

// Container record kinds (cont_flags bits 4-5) and the presence bits (0-3) of pe_pg_min_resources.
const (
	KindContainer = uint8(C.PE_KIND_CONTAINER)
	KindInit      = uint8(C.PE_KIND_INIT)
	KindSidecar   = uint8(C.PE_KIND_SIDECAR)
	KindOverhead  = uint8(C.PE_KIND_OVERHEAD)
	KindShift     = uint(C.PE_KIND_SHIFT)
)

// Job status of PlaceGreedy.
const (
	JobPlaced        = int32(C.PE_JOB_PLACED)
	JobUnschedulable = int32(C.PE_JOB_UNSCHEDULABLE)
	// LabelIsland is node label bit 31 (set by the engine when island >= 0); a greedy group whose
	// need carries NeedIsland is placed as one unit on one island node (placement.h).
	LabelIsland = uint32(C.PE_LABEL_ISLAND)
	NeedIsland  = uint32(C.PE_NEED_ISLAND)
)

// Node inventory update ops.
const (
	NodeSet    = uint8(C.PE_NODE_SET)
	NodeRemove = uint8(C.PE_NODE_REMOVE)
)

// Device mask layouts (FitMaskLayout).
const (
	MaskNodeTiles  = int32(C.PE_MASK_NODE_TILES)
	MaskJobBits    = int32(C.PE_MASK_JOB_BITS)
	MaskNodeBlocks = int32(C.PE_MASK_NODE_BLOCKS)
	MaskRows       = int32(C.PE_MASK_ROWS)
)

// Dims is the number of engine resource dimensions: cpu (milli), memory (B), the accelerator
// resource named in Config.GPUResourceName (count), ephemeral-storage (B).
const Dims = int(C.PE_DIMS)

// CommIDBytes is the size of an RCCL unique id (CommID).
const CommIDBytes = int(C.PE_COMM_ID_BYTES)

// ErrOverflow: an aggregation overflowed int64 -- the reference's resource.Quantity would have
// switched to inf.Dec.  The per-job Overflow flags say which job; the caller takes the exact
// reference path for those jobs.
var ErrOverflow = errors.New("placement: int64 overflow (reference would switch to inf.Dec)")

// ErrNoDevice: no usable GPU.  The engine has no CPU fallback.
var ErrNoDevice = errors.New("placement: no usable GPU")

// Config mirrors pe_config.  Zero values take the engine defaults.
type Config struct {
	DeviceID        int32  // HIP ordinal; -1 = the calling thread's current device
	Rank, WorldSize int32  // inventory shard of this process (WorldSize 0 = 1)
	CommID          []byte // CommIDBytes from CommID() on rank 0 (RCCL), for WorldSize > 1
	MaxNodes        int64
	GPUResourceName string // dim 2's resource key, e.g. "amd.com/gpu"
	TopK            int32
	WindowGroups    int32
	WindowPods      int64
	FitPathMask     int32
	GreedyFlags     int32
	ResortNodes     int32
	// HostExchange replaces RCCL for ranks of one node (e.g. when the communicator set-up failed on
	// some rank: PE_ERCCL there means every rank drops its engine and creates a new one).
	HostExchange *HostExchange
}

// HostExchange is pe_host_exchange: an all-gather through a POSIX shared-memory segment, for the
// ranks of one node.  Every rank opens the same name ("/..."); rank 0 creates the segment.
type HostExchange struct {
	h    *C.pe_host_exchange
	rank int32
	size int32
}

// OpenHostExchange opens (rank 0: creates) the segment; maxBytes bounds one rank's block per call
// (WindowGroups x (16 + 8 x TopK) for the greedy windows).  Passed as Config.HostExchange, the
// library recognises its own exchange and runs the greedy windows zero-copy: each rank's walk writes
// into the segment and an exchange thread merges every group on the host (Stats.xchg_zc_windows).
func OpenHostExchange(name string, rank, world int32, maxBytes int) (*HostExchange, error) {
	cn := C.CString(name)
	defer C.free(unsafe.Pointer(cn))
	x := &HostExchange{rank: rank, size: world}
	if rc := C.pe_host_exchange_open(cn, C.int32_t(rank), C.int32_t(world), C.size_t(maxBytes), &x.h); rc != C.PE_OK {
		return nil, fmt.Errorf("placement: pe_host_exchange_open: %d", int(rc))
	}
	runtime.SetFinalizer(x, (*HostExchange).Close)
	return x, nil
}

// Allgather gathers every rank's send block into recv (world x len(send) bytes, rank order).
func (x *HostExchange) Allgather(send, recv []byte) error {
	if len(recv) < int(x.size)*len(send) {
		return errors.New("placement: HostExchange.Allgather: recv too small")
	}
	var sp, rp unsafe.Pointer
	if len(send) > 0 {
		sp, rp = unsafe.Pointer(&send[0]), unsafe.Pointer(&recv[0])
	}
	if rc := C.pe_host_exchange_allgather(unsafe.Pointer(x.h), sp, rp, C.size_t(len(send))); rc != C.PE_OK {
		return fmt.Errorf("placement: pe_host_exchange_allgather: %d", int(rc))
	}
	runtime.KeepAlive(x) // the finalizer must not unmap the segment during the call
	return nil
}

// Close unmaps the segment.  Idempotent; the engines using it must be closed first.
func (x *HostExchange) Close() {
	if x.h != nil {
		C.pe_host_exchange_close(x.h)
		x.h = nil
	}
}

// Engine is one pe_ctx: a GPU, an inventory shard, a stream.  Safe for concurrent use (the
// context holds a mutex and selects its device on every call).
type Engine struct {
	ctx  *C.pe_ctx
	name *C.char
	// hx keeps the HostExchange the context was created with reachable for the context's lifetime:
	// its walks and exchange thread use the mapped segment, which HostExchange's finalizer unmaps.
	hx *HostExchange
}

// Stats mirrors pe_stats.
type Stats = C.pe_stats

func ptr64(s []int64) *C.int64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int64_t)(unsafe.Pointer(&s[0]))
}

func ptr32(s []int32) *C.int32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int32_t)(unsafe.Pointer(&s[0]))
}

func ptru32(s []uint32) *C.uint32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint32_t)(unsafe.Pointer(&s[0]))
}

func ptr8(s []uint8) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&s[0]))
}

func ptru64(s []uint64) *C.uint64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&s[0]))
}

// ABIVersion is PE_ABI_VERSION of the loaded library.
func ABIVersion() int { return int(C.pe_abi_version()) }

// CommID makes an RCCL unique id (rank 0; broadcast the bytes to every rank).
func CommID() ([]byte, error) {
	buf := make([]byte, CommIDBytes)
	if rc := C.pe_comm_id((*C.uint8_t)(unsafe.Pointer(&buf[0]))); rc != C.PE_OK {
		return nil, fmt.Errorf("placement: pe_comm_id: %d", int(rc))
	}
	return buf, nil
}

// New creates an engine context (pe_create).
func New(cfg Config) (*Engine, error) {
	e := &Engine{name: C.CString(cfg.GPUResourceName)}
	var c C.pe_config
	c.device_id = C.int32_t(cfg.DeviceID)
	c.rank = C.int32_t(cfg.Rank)
	c.world_size = C.int32_t(cfg.WorldSize)
	if c.world_size == 0 {
		c.world_size = 1
	}
	var id unsafe.Pointer
	if len(cfg.CommID) > 0 {
		if len(cfg.CommID) != CommIDBytes {
			C.free(unsafe.Pointer(e.name))
			return nil, fmt.Errorf("placement: comm id must be %d bytes", CommIDBytes)
		}
		id = C.CBytes(cfg.CommID)
		defer C.free(id)
		c.comm_id = (*C.uint8_t)(id)
	}
	c.max_nodes = C.int64_t(cfg.MaxNodes)
	c.gpu_resource_name = e.name
	c.topk = C.int32_t(cfg.TopK)
	c.window_groups = C.int32_t(cfg.WindowGroups)
	c.window_pods = C.int64_t(cfg.WindowPods)
	c.fit_path_mask = C.int32_t(cfg.FitPathMask)
	c.greedy_flags = C.int32_t(cfg.GreedyFlags)
	c.resort_nodes = C.int32_t(cfg.ResortNodes)
	if cfg.HostExchange != nil {
		c.exchange = C.hx_allgather_fn()
		c.exchange_user = unsafe.Pointer(cfg.HostExchange.h)
		e.hx = cfg.HostExchange
	}
	rc := C.pe_create(&c, &e.ctx)
	if rc != C.PE_OK {
		C.free(unsafe.Pointer(e.name))
		if rc == C.PE_ENODEV {
			return nil, ErrNoDevice
		}
		return nil, fmt.Errorf("placement: pe_create: %d", int(rc))
	}
	runtime.SetFinalizer(e, (*Engine).Close)
	return e, nil
}

// Close releases the context (pe_destroy).  Idempotent.
func (e *Engine) Close() {
	if e.ctx != nil {
		C.pe_destroy(e.ctx)
		e.ctx = nil
		C.free(unsafe.Pointer(e.name))
		e.hx = nil // the segment may be unmapped now (the caller's Close, or its finalizer)
	}
}

func (e *Engine) err(rc C.int, what string) error {
	switch rc {
	case C.PE_OK:
		return nil
	case C.PE_EOVERFLOW:
		return ErrOverflow
	case C.PE_ENODEV:
		return ErrNoDevice
	}
	return fmt.Errorf("placement: %s: %d: %s", what, int(rc), C.GoString(C.pe_last_error(e.ctx)))
}

// LoadNodes loads the GLOBAL inventory (SoA [4][n]: row d = dim d); the context keeps its shard.
func (e *Engine) LoadNodes(n int64, capacity, used []int64, labels []uint32, island []int32) error {
	if int64(len(capacity)) < int64(Dims)*n || int64(len(used)) < int64(Dims)*n {
		return fmt.Errorf("placement: LoadNodes: cap/used need %d values", int64(Dims)*n)
	}
	return e.err(C.pe_load_nodes(e.ctx, C.int64_t(n), ptr64(capacity), ptr64(used), ptru32(labels), ptr32(island)),
		"pe_load_nodes")
}

// ResetResiduals restores residual := cap - used on the device.
func (e *Engine) ResetResiduals() error { return e.err(C.pe_reset_residuals(e.ctx), "pe_reset_residuals") }

// UpdateNodes applies Node informer events: per entry NodeSet (cap/used [n][4], labels, island
// replace the slot) or NodeRemove.  Validated as a whole before anything changes.
func (e *Engine) UpdateNodes(slots []int64, ops []uint8, capacity, used []int64, labels []uint32, island []int32) error {
	if len(ops) != len(slots) {
		return errors.New("placement: UpdateNodes: one op per slot")
	}
	return e.err(C.pe_update_nodes(e.ctx, C.int64_t(len(slots)), ptr64(slots), ptr8(ops), ptr64(capacity), ptr64(used),
		ptru32(labels), ptr32(island)), "pe_update_nodes")
}

// ShardRange is this context's node range [begin, end).
func (e *Engine) ShardRange() (begin, end int64, err error) {
	var b, en C.int64_t
	if rc := C.pe_shard_range(e.ctx, &b, &en); rc != C.PE_OK {
		return 0, 0, e.err(rc, "pe_shard_range")
	}
	return int64(b), int64(en), nil
}

// CommRanks is the RCCL communicator size (0 without one).
func (e *Engine) CommRanks() (int32, error) {
	var n C.int32_t
	if rc := C.pe_comm_ranks(e.ctx, &n); rc != C.PE_OK {
		return 0, e.err(rc, "pe_comm_ranks")
	}
	return int32(n), nil
}

// ReadResiduals copies this shard's residuals ([4][end-begin]).
func (e *Engine) ReadResiduals() ([]int64, error) {
	b, en, err := e.ShardRange()
	if err != nil {
		return nil, err
	}
	out := make([]int64, int64(Dims)*(en-b))
	return out, e.err(C.pe_read_residuals(e.ctx, ptr64(out)), "pe_read_residuals")
}

// CSR is the flattened batch of pe_pg_min_resources (include/placement.h).
type CSR struct {
	JobGroupOff   []int32 // [J+1]
	MinMember     []int32 // [J] (v1)
	GroupReplicas []int32 // [G], -1 = nil (v1)
	GroupContOff  []int32 // [G+1]
	ContReq       []int64 // [C][4] canonical int64
	ContFlags     []uint8 // [C] presence bits 0-3 | kind << KindShift
}

// Agg holds the per-job results of PGMinResources.
type Agg struct {
	MinRes   []int64 // [J][4]
	Present  []uint8 // bit d = key d present (keys with value 0 included)
	Members  []int32
	Overflow []uint8 // 1 = int64 overflow: take the reference's exact path for this job
}

// PGMinResources aggregates a batch of PodGroups on the GPU.  Overflowed jobs are flagged, not an
// error: the batch's other jobs are exact.
func (e *Engine) PGMinResources(mode int, b *CSR) (*Agg, error) {
	J := len(b.JobGroupOff) - 1
	if J < 0 {
		return nil, errors.New("placement: JobGroupOff needs J+1 entries")
	}
	out := &Agg{make([]int64, Dims*J), make([]uint8, J), make([]int32, J), make([]uint8, J)}
	if J == 0 {
		return out, nil
	}
	rc := C.pe_pg_min_resources(e.ctx, C.int32_t(mode), C.int64_t(J), ptr32(b.JobGroupOff), ptr32(b.MinMember),
		ptr32(b.GroupReplicas), ptr32(b.GroupContOff), ptr64(b.ContReq), ptr8(b.ContFlags), ptr64(out.MinRes),
		ptr8(out.Present), ptr32(out.Members), ptr8(out.Overflow))
	if rc == C.PE_EOVERFLOW {
		return out, nil
	}
	return out, e.err(rc, "pe_pg_min_resources")
}

// MaxKeys is PE_MAX_KEYS: the keys of one pe_pg_min_resources_keys call (a batch with more takes one
// call per slice of keys; keys never interact).
const MaxKeys = int(C.PE_MAX_KEYS)

// KeysKindShift is PE_KEYS_KIND_SHIFT: the kind bits of a key-table container flag word.
const KeysKindShift = uint(C.PE_KEYS_KIND_SHIFT)

// KeyAgg holds the per-job results of PGMinResourcesKeys over the batch's key table.
type KeyAgg struct {
	Keys     []corev1.ResourceName
	Scale    []int32 // per key: MinRes values are counts of 10^Scale
	MinRes   []int64 // [J][len(Keys)]
	Present  []bool  // [J][len(Keys)] (keys with value 0 included)
	Members  []int32
	Overflow []uint8 // 1 = a sum (or a value) with no int64 at its key's scale: the reference's inf.Dec case
}

// PGMinResourcesKeys aggregates a batch over its per-call key table (pe_pg_min_resources_keys): any
// resource key, each at the finest decimal scale its quantities need (KeyCSR.Scales), one engine call
// per slice of MaxKeys keys.  A value with no int64 at its key's scale flags its job like an
// overflowed sum; flagged jobs are the caller's to hand to the reference.  Every other outcome is
// exact; an engine error is returned.
func (e *Engine) PGMinResourcesKeys(mode int, b *KeyCSR) (*KeyAgg, error) {
	J := len(b.JobGroupOff) - 1
	if J < 0 {
		return nil, errors.New("placement: JobGroupOff needs J+1 entries")
	}
	nk := len(b.Keys)
	out := &KeyAgg{Keys: b.Keys, Scale: b.Scales(), MinRes: make([]int64, J*nk), Present: make([]bool, J*nk),
		Members: make([]int32, J), Overflow: make([]uint8, J)}
	if J == 0 {
		return out, nil
	}
	val, jobOvf := b.scaledValues(out.Scale)
	for j := 0; j < J; j++ {
		out.Overflow[j] = jobOvf[j]
	}
	nc := len(b.ContKind)
	flags := make([]uint32, nc)
	pres := make([]uint16, J)
	ovf := make([]uint8, J)
	for lo := 0; lo < nk || (lo == 0 && nk == 0); lo += MaxKeys {
		n := nk - lo
		if n > MaxKeys {
			n = MaxKeys
		}
		if n < 1 {
			n = 1 // no key at all: one empty key, for Members
		}
		req := make([]int64, nc*n)
		res := make([]int64, J*n)
		for c := 0; c < nc; c++ {
			f := uint32(b.ContKind[c]) << KeysKindShift
			for x := b.EntOff[c]; x < b.EntOff[c+1]; x++ {
				k := int(b.EntKey[x]) - lo
				if k < 0 || k >= n || lo+k >= nk {
					continue
				}
				req[c*n+k] = val[x]
				f |= 1 << uint(k)
			}
			flags[c] = f
		}
		rc := C.pe_pg_min_resources_keys(e.ctx, C.int32_t(mode), C.int64_t(J), C.int32_t(n), ptr32(b.JobGroupOff),
			ptr32(b.MinMember), ptr32(b.GroupReplicas), ptr32(b.GroupContOff), ptr64(req), ptru32(flags), ptr64(res),
			(*C.uint16_t)(unsafe.Pointer(&pres[0])), ptr32(out.Members), ptr8(ovf))
		if rc != C.PE_OK && rc != C.PE_EOVERFLOW {
			return nil, e.err(rc, "pe_pg_min_resources_keys")
		}
		for j := 0; j < J; j++ {
			out.Overflow[j] |= ovf[j]
			for k := 0; k < n && lo+k < nk; k++ {
				out.MinRes[j*nk+lo+k] = res[j*n+k]
				out.Present[j*nk+lo+k] = pres[j]>>uint(k)&1 != 0
			}
		}
		if nk == 0 {
			break
		}
	}
	return out, nil
}

// FitMask evaluates every job against every node of the shard (device-resident mask); returns the
// per-job feasible counts of this shard and the mask's words per row.
func (e *Engine) FitMask(req []int64, need []uint32) (counts []int64, wordsPerRow int64, err error) {
	J := len(req) / Dims
	counts = make([]int64, J)
	var dev *C.uint64_t
	var wpr C.int64_t
	rc := C.pe_fit_mask(e.ctx, C.int64_t(J), ptr64(req), ptru32(need), ptr64(counts), &dev, &wpr)
	return counts, int64(wpr), e.err(rc, "pe_fit_mask")
}

// JobsUpload stages a fit batch on the device (plan + H2D); FitMaskRun evaluates it asynchronously;
// FitCounts synchronizes and returns the per-job counts.
func (e *Engine) JobsUpload(req []int64, need []uint32) error {
	return e.err(C.pe_jobs_upload(e.ctx, C.int64_t(len(req)/Dims), ptr64(req), ptru32(need)), "pe_jobs_upload")
}

func (e *Engine) FitMaskRun() error { return e.err(C.pe_fit_mask_run(e.ctx), "pe_fit_mask_run") }

func (e *Engine) FitCounts(nJobs int) ([]int64, error) {
	out := make([]int64, nJobs)
	return out, e.err(C.pe_fit_counts(e.ctx, ptr64(out)), "pe_fit_counts")
}

// FitMaskRows copies rows [row0, row0+nRows) of the mask, row-major [nRows][wordsPerRow].
func (e *Engine) FitMaskRows(row0, nRows, wordsPerRow int64) ([]uint64, error) {
	out := make([]uint64, nRows*wordsPerRow)
	return out, e.err(C.pe_fit_mask_rows(e.ctx, C.int64_t(row0), C.int64_t(nRows), ptru64(out)), "pe_fit_mask_rows")
}

// FitMaskLayout and FitMaskRowPitch describe the device mask (for callers that map it).
func (e *Engine) FitMaskLayout() (int32, error) {
	var l C.int32_t
	rc := C.pe_fit_mask_layout(e.ctx, &l)
	return int32(l), e.err(rc, "pe_fit_mask_layout")
}

func (e *Engine) FitMaskRowPitch() (int64, error) {
	var w C.int64_t
	rc := C.pe_fit_mask_row_pitch(e.ctx, &w)
	return int64(w), e.err(rc, "pe_fit_mask_row_pitch")
}

// Gangs is a greedy placement batch: jobs of groups of identical pods (include/placement.h).
type Gangs struct {
	JobGroupOff []int32  // [J+1]
	Priority    []int32  // [J]
	GroupCount  []int32  // [G] pods to place
	GroupReq    []int64  // [G][4]
	GroupNeed   []uint32 // [G] required label bits
}

func (g *Gangs) pods() int {
	n := 0
	for _, c := range g.GroupCount {
		n += int(c)
	}
	return n
}

// PlaceGreedy places the batch best-fit, all-or-nothing per job (SURVEY.md Appendix B).  Every rank
// of a sharded engine makes the same call and gets the same answer.
func (e *Engine) PlaceGreedy(g *Gangs) (podNode, jobStatus []int32, err error) {
	J := len(g.JobGroupOff) - 1
	podNode = make([]int32, g.pods())
	jobStatus = make([]int32, J)
	rc := C.pe_place_greedy(e.ctx, C.int64_t(J), ptr32(g.JobGroupOff), ptr32(g.Priority), ptr32(g.GroupCount),
		ptr64(g.GroupReq), ptru32(g.GroupNeed), ptr32(podNode), ptr32(jobStatus))
	return podNode, jobStatus, e.err(rc, "pe_place_greedy")
}

// Synchronize waits for the context's stream; Stream is its hipStream_t (for event timing).
func (e *Engine) Synchronize() error { return e.err(C.pe_synchronize(e.ctx), "pe_synchronize") }

func (e *Engine) Stream() unsafe.Pointer { return unsafe.Pointer(C.pe_stream(e.ctx)) }

// Stats and ResetStats: engine counters (fit evaluations, windows, placements, timings).
func (e *Engine) Stats() (Stats, error) {
	var s C.pe_stats
	rc := C.pe_get_stats(e.ctx, &s)
	return s, e.err(rc, "pe_get_stats")
}

func (e *Engine) ResetStats() error { return e.err(C.pe_reset_stats(e.ctx), "pe_reset_stats") }

// Resolver is the host half of the windowed greedy (pe_resolver_*), for callers that gather the
// per-shard candidate blobs over their own transport.  No device is touched.
type Resolver struct {
	r    *C.pe_resolver
	jobs int
	pods int
}

func NewResolver(g *Gangs) (*Resolver, error) {
	res := &Resolver{jobs: len(g.JobGroupOff) - 1, pods: g.pods()}
	rc := C.pe_resolver_create(C.int64_t(res.jobs), ptr32(g.JobGroupOff), ptr32(g.Priority), ptr32(g.GroupCount),
		ptr64(g.GroupReq), ptru32(g.GroupNeed), &res.r)
	if rc != C.PE_OK {
		return nil, fmt.Errorf("placement: pe_resolver_create: %d", int(rc))
	}
	return res, nil
}

func (r *Resolver) Close() {
	if r.r != nil {
		C.pe_resolver_destroy(r.r)
		r.r = nil
	}
}

// SetNodes bounds the node ids the blobs and seeds may list (pe_resolver_set_nodes): a blob from any
// transport with a header count outside [0, topK], an id >= nNodes or unsorted keys is then refused
// (PE_EINVAL) before the resolver moves.
func (r *Resolver) SetNodes(nNodes int64) error {
	if rc := C.pe_resolver_set_nodes(r.r, C.int64_t(nNodes)); rc != C.PE_OK {
		return fmt.Errorf("placement: pe_resolver_set_nodes: %d", int(rc))
	}
	return nil
}

func (r *Resolver) Done() bool { return C.pe_resolver_done(r.r) != 0 }

// NextWindow returns the global group ids of the next scan window.
func (r *Resolver) NextWindow(maxGroups int32, maxPods int64) ([]int32, error) {
	out := make([]int32, maxGroups)
	var n C.int32_t
	if rc := C.pe_resolver_next_window(r.r, C.int32_t(maxGroups), C.int64_t(maxPods), ptr32(out), &n); rc != C.PE_OK {
		return nil, fmt.Errorf("placement: pe_resolver_next_window: %d", int(rc))
	}
	return out[:n], nil
}

// Resolve consumes one window's blob (n_shards blocks, see placement.h) and returns the residual
// updates to flush ([n][5] = node id, res[4]) and whether the window was consumed.
func (r *Resolver) Resolve(groups []int32, blob []byte, nShards, topK int32) ([]int64, bool, error) {
	maxUpd := int64(2*r.pods + 64)
	upd := make([]int64, 5*maxUpd)
	var nu C.int64_t
	var consumed C.int32_t
	rc := C.pe_resolver_resolve(r.r, C.int32_t(len(groups)), ptr32(groups), ptr8(blob), C.int32_t(nShards),
		C.int32_t(topK), ptr64(upd), C.int64_t(maxUpd), &nu, &consumed)
	if rc != C.PE_OK {
		return nil, false, fmt.Errorf("placement: pe_resolver_resolve: %d", int(rc))
	}
	return upd[:5*int64(nu)], consumed != 0, nil
}

// ResolveSeeded is Resolve for the pipelined protocol: seeds ([n][6] int64: node id, res[0..3],
// labels) are the nodes changed since the snapshot the blob was scanned on, with current state.
func (r *Resolver) ResolveSeeded(groups []int32, blob []byte, nShards, topK int32, seeds []int64) ([]int64, bool, error) {
	if len(seeds)%6 != 0 {
		return nil, false, fmt.Errorf("placement: seeds must be [n][6]")
	}
	maxUpd := int64(2*r.pods + 64)
	upd := make([]int64, 5*maxUpd)
	var nu C.int64_t
	var consumed C.int32_t
	rc := C.pe_resolver_resolve_seeded(r.r, C.int32_t(len(groups)), ptr32(groups), ptr8(blob), C.int32_t(nShards),
		C.int32_t(topK), C.int64_t(len(seeds)/6), ptr64(seeds), ptr64(upd), C.int64_t(maxUpd), &nu, &consumed)
	if rc != C.PE_OK {
		return nil, false, fmt.Errorf("placement: pe_resolver_resolve_seeded: %d", int(rc))
	}
	return upd[:5*int64(nu)], consumed != 0, nil
}

// Results: the node of every pod slot (-1 = none) and every job's status.
func (r *Resolver) Results() (podNode, jobStatus []int32, err error) {
	podNode = make([]int32, r.pods)
	jobStatus = make([]int32, r.jobs)
	if rc := C.pe_resolver_results(r.r, ptr32(podNode), ptr32(jobStatus)); rc != C.PE_OK {
		return nil, nil, fmt.Errorf("placement: pe_resolver_results: %d", int(rc))
	}
	return podNode, jobStatus, nil
}
