/*
Engine-backed CalcPGMinResources: a drop-in for pkg/controller.v1/common/util.go:108 with the same
signature, wired in at job.go:455-457:

	func (jc *JobController) calcPGMinResources(minMember int32, replicas map[apiv1.ReplicaType]*apiv1.ReplicaSpec) *corev1.ResourceList {
		return jc.calcPGMinResourcesFn(minMember, replicas, jc.PriorityClassLister.Get)
	}
	// jc.calcPGMinResourcesFn = CalcPGMinResourcesEngine(engine, "nvidia.com/gpu") (or CalcPGMinResources)

The flattening restates util.go:108-145: one group per replica type in ReplicasPriority order
(priority desc; the reference breaks equal priorities by Go map order, which is random -- here by
type name, one of the orders the reference can produce), Replicas nil -> -1 (the type is skipped,
util.go:129), and per container the effective list AddResourceList adds (util.go:79-104): Requests,
or Limits only when the Requests map is nil (an empty non-nil map does not fall back).  Init
containers and pod overhead are not counted (util.go:138).  The engine counts pods up to minMember
exactly as the per-pod loop.  Every resource key is summed on the GPU (a per-call key table,
pe_pg_min_resources_keys: hugepages-*, rdma/*, any accelerator name, cpu finer than 1m), each at the
decimal scale its quantities need.  The ONE input handed to the reference's CalcPGMinResources is a
job whose sum has no int64 at its scale (Overflow: Go holds it in inf.Dec), so the answer is the
reference's for every input; an ENGINE error is never answered that way -- it is returned
(CalcPGMinResourcesEngineE, PGMinResourcesBatch) or counted and logged (EngineErrors).
*/
package common

import (
	"fmt"
	"sort"
	"sync/atomic"

	log "github.com/sirupsen/logrus"

	apiv1 "github.com/kubeflow/training-operator/pkg/apis/kubeflow.org/v1"
	"github.com/kubeflow/training-operator/pkg/placement/hip"
	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
)

// flattenV1 builds the one-job v1 CSR of CalcPGMinResources(minMember, replicas, pcGetFunc), and the
// print formats the reference's AddResourceList sums end with (hip.KeyFormatAcc, util.go:79-104): the
// same walk over the pods util.go:126-141 counts (a type's second pod only re-adds the formats of
// its first, so at most two per type are replayed).
func flattenV1(minMember int32, replicas map[apiv1.ReplicaType]*apiv1.ReplicaSpec,
	pcGetFunc PriorityClassGetFunc) (*hip.KeyCSR, *hip.KeyFormatAcc, error) {
	type typed struct {
		name     string
		priority int32
		spec     *apiv1.ReplicaSpec
	}
	order := make([]typed, 0, len(replicas))
	for t, replica := range replicas {
		rp := typed{name: string(t), spec: replica}
		if pc, err := pcGetFunc(replica.Template.Spec.PriorityClassName); err == nil && pc != nil {
			rp.priority = pc.Value // util.go:114-119: a failed lookup counts as priority 0
		}
		order = append(order, rp)
	}
	sort.SliceStable(order, func(i, j int) bool {
		if order[i].priority != order[j].priority {
			return order[i].priority > order[j].priority // ReplicasPriority.Less, util.go:42-44
		}
		return order[i].name < order[j].name
	})
	b := &hip.KeyCSR{}
	acc := &hip.KeyFormatAcc{}
	podCnt := int64(0)
	for _, t := range order {
		for _, c := range t.spec.Template.Spec.Containers {
			if err := b.AddContainer(effectiveList(c), hip.KindContainer); err != nil {
				return nil, nil, err
			}
		}
		replicasOrNil := int32(-1)
		if t.spec.Replicas != nil {
			replicasOrNil = *t.spec.Replicas
			k := int64(*t.spec.Replicas)
			if room := int64(minMember) - podCnt; room < k {
				k = room
			}
			for pod := int64(0); pod < k && pod < 2; pod++ {
				for _, c := range t.spec.Template.Spec.Containers {
					acc.AddList(effectiveList(c), 1)
				}
			}
			if k > 0 {
				podCnt += k
			}
		}
		b.EndGroup(replicasOrNil)
	}
	b.EndJob(minMember)
	return b, acc, nil
}

// effectiveList is what AddResourceList adds for a container: Requests, or Limits only when the
// Requests map is nil (util.go:90-92; an empty non-nil map does not fall back).
func effectiveList(c v1.Container) v1.ResourceList {
	if c.Resources.Requests == nil {
		return c.Resources.Limits
	}
	return c.Resources.Requests
}

// EngineErrors counts the engine failures (PE_EHIP, PE_ENODEV, a lost device ...) the v1-signature
// adapter below could not return to its caller.  Monitor it: every count is a log line and a PodGroup
// written with EngineErrorMinResources' answer, never an answer computed some other way.
var EngineErrors uint64

// EngineErrorResource is the resource the fail-closed answer asks for: no node offers it, so a gang
// scheduler that checks MinResources admits no gang of that PodGroup until a later reconcile (the
// operator resyncs, and SyncPodGroup always rewrites the PodGroup, job.go:308-313) computes the real
// minimum.
const EngineErrorResource v1.ResourceName = "placement.kubeflow.org/engine-error"

// EngineErrorMinResources is what CalcPGMinResourcesEngine answers for a job whose aggregation failed
// in the engine.  Default FailClosed: {EngineErrorResource: 1}, a minimum no cluster meets -- the gang
// waits instead of being admitted unchecked.  FailOpen (opt-in): an empty list, i.e. no minimum (the
// gang scheduler then checks nothing and may admit a gang that does not fit).  Production wiring
// returns the error instead: CalcPGMinResourcesEngineE or PGMinResourcesBatch (INTEGRATION.md section 2).
type EngineErrorPolicy int

const (
	FailClosed EngineErrorPolicy = iota
	FailOpen
)

var EngineErrorMinResources = FailClosed

func engineErrorAnswer() *v1.ResourceList {
	if EngineErrorMinResources == FailOpen {
		return &v1.ResourceList{}
	}
	return &v1.ResourceList{EngineErrorResource: *resource.NewQuantity(1, resource.DecimalSI)}
}

// CalcPGMinResourcesEngineE is CalcPGMinResources with the pod counting and the resource sums on the
// GPU, and the engine's failures returned.  Only an int64 OVERFLOW goes to the reference's
// CalcPGMinResources (util.go:108; the reference switches to inf.Dec there).  Every other outcome is
// the engine's: an engine error is returned as it is -- like the v2 plugin's Build -- so the reconcile
// fails and is retried (job.go:313's SyncPodGroup error path), and so is a flatten error (a negative
// quantity, which API validation never admits).  gpuName is kept for the signature of earlier wirings:
// every key is summed now, whatever its name.
func CalcPGMinResourcesEngineE(eng *hip.Engine, gpuName string) func(int32, map[apiv1.ReplicaType]*apiv1.ReplicaSpec,
	PriorityClassGetFunc) (*v1.ResourceList, error) {
	_ = gpuName
	return func(minMember int32, replicas map[apiv1.ReplicaType]*apiv1.ReplicaSpec, pcGetFunc PriorityClassGetFunc) (*v1.ResourceList, error) {
		csr, formats, ferr := flattenV1(minMember, replicas, pcGetFunc)
		if ferr != nil {
			return nil, fmt.Errorf("placement engine: CalcPGMinResources: %w", ferr)
		}
		agg, err := eng.PGMinResourcesKeys(hip.ModeV1, csr)
		if err != nil {
			return nil, fmt.Errorf("placement engine: CalcPGMinResources: %w", err)
		}
		if agg.Overflow[0] != 0 {
			return CalcPGMinResources(minMember, replicas, pcGetFunc), nil // the inf.Dec case: exact reference path
		}
		rl := agg.Unflatten(0, formats.Formats()) // printed as the reference's sums print
		return &rl, nil
	}
}

// CalcPGMinResourcesEngine keeps util.go:108's signature (no error result) for a one-line swap of
// jc.calcPGMinResourcesFn.  Like the reference it never returns nil.  An engine error cannot be
// returned through that signature, so it is counted in EngineErrors, logged, and answered per
// EngineErrorMinResources -- by default a minimum no node meets (fail closed), an empty list only when
// FailOpen is chosen -- never with the reference's CPU result.  Wire CalcPGMinResourcesEngineE instead
// where job.go can return the error (INTEGRATION.md section 2).
func CalcPGMinResourcesEngine(eng *hip.Engine, gpuName string) func(int32, map[apiv1.ReplicaType]*apiv1.ReplicaSpec,
	PriorityClassGetFunc) *v1.ResourceList {
	calc := CalcPGMinResourcesEngineE(eng, gpuName)
	return func(minMember int32, replicas map[apiv1.ReplicaType]*apiv1.ReplicaSpec, pcGetFunc PriorityClassGetFunc) *v1.ResourceList {
		rl, err := calc(minMember, replicas, pcGetFunc)
		if err != nil {
			atomic.AddUint64(&EngineErrors, 1)
			log.Errorf("CalcPGMinResources: %v (PodGroup MinResources answered per EngineErrorMinResources=%d; "+
				"EngineErrors=%d)", err, EngineErrorMinResources, atomic.LoadUint64(&EngineErrors))
			return engineErrorAnswer()
		}
		return rl
	}
}

// PGRequest is one CalcPGMinResources call of a batch (the arguments of util.go:108).
type PGRequest struct {
	MinMember int32
	Replicas  map[apiv1.ReplicaType]*apiv1.ReplicaSpec
	PcGetFunc PriorityClassGetFunc
}

// PGMinResourcesBatch is CalcPGMinResources for many jobs at once -- a resync of every job's
// PodGroup (job.go:455-457 called in a loop) -- with ONE engine call (per slice of hip.MaxKeys keys) for
// all the jobs.  Jobs whose sums overflow take the reference's CalcPGMinResources (the inf.Dec case,
// as CalcPGMinResourcesEngineE); a flatten error or an engine error fails the whole call (out is nil)
// and is returned.  out[i] is the answer for reqs[i], exactly the reference's.  The engine pays off
// above hip.BatchCrossoverJobs jobs.
func PGMinResourcesBatch(eng *hip.Engine, gpuName string, reqs []PGRequest) ([]*v1.ResourceList, error) {
	_ = gpuName
	out := make([]*v1.ResourceList, len(reqs))
	batch := &hip.KeyCSR{}
	formats := make([]*hip.KeyFormatAcc, 0, len(reqs))
	for i, r := range reqs {
		csr, f, ferr := flattenV1(r.MinMember, r.Replicas, r.PcGetFunc)
		if ferr != nil {
			return nil, fmt.Errorf("placement engine: PGMinResourcesBatch: request %d: %w", i, ferr)
		}
		batch.AppendJobs(csr)
		formats = append(formats, f)
	}
	if len(reqs) == 0 {
		return out, nil
	}
	agg, err := eng.PGMinResourcesKeys(hip.ModeV1, batch)
	if err != nil {
		return nil, fmt.Errorf("placement engine: PGMinResourcesBatch (%d jobs): %w", len(reqs), err)
	}
	for i, r := range reqs {
		if agg.Overflow[i] != 0 {
			out[i] = CalcPGMinResources(r.MinMember, r.Replicas, r.PcGetFunc) // the inf.Dec case: exact reference path
			continue
		}
		rl := agg.Unflatten(i, formats[i].Formats())
		out[i] = &rl
	}
	return out, nil
}
