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
exactly as the per-pod loop.  Inputs the tensor path does not hold exactly go to the reference's
CalcPGMinResources unchanged, so the answer is the reference's for every input.
*/
package common

import (
	"sort"

	apiv1 "github.com/kubeflow/training-operator/pkg/apis/kubeflow.org/v1"
	"github.com/kubeflow/training-operator/pkg/placement/hip"
	v1 "k8s.io/api/core/v1"
)

// flattenV1 builds the one-job v1 CSR of CalcPGMinResources(minMember, replicas, pcGetFunc), and the
// print formats the reference's AddResourceList sums end with (hip.FormatAcc, util.go:79-104): the
// same walk over the pods util.go:126-141 counts (a type's second pod only re-adds the formats of
// its first, so at most two per type are replayed).
func flattenV1(minMember int32, replicas map[apiv1.ReplicaType]*apiv1.ReplicaSpec, pcGetFunc PriorityClassGetFunc,
	gpuName string) (*hip.CSR, *hip.FormatAcc, error) {
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
	b := &hip.CSR{}
	acc := &hip.FormatAcc{}
	podCnt := int64(0)
	for _, t := range order {
		for _, c := range t.spec.Template.Spec.Containers {
			if err := b.AddContainer(effectiveList(c), hip.KindContainer, gpuName); err != nil {
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
					acc.AddList(effectiveList(c), gpuName, 1)
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

// CalcPGMinResourcesEngine returns a CalcPGMinResources with the pod counting and the resource sums
// on the GPU.  Like the reference it never returns nil.
func CalcPGMinResourcesEngine(eng *hip.Engine, gpuName string) func(int32, map[apiv1.ReplicaType]*apiv1.ReplicaSpec,
	PriorityClassGetFunc) *v1.ResourceList {
	return func(minMember int32, replicas map[apiv1.ReplicaType]*apiv1.ReplicaSpec, pcGetFunc PriorityClassGetFunc) *v1.ResourceList {
		csr, formats, err := flattenV1(minMember, replicas, pcGetFunc, gpuName)
		if err != nil {
			return CalcPGMinResources(minMember, replicas, pcGetFunc) // exact reference path
		}
		agg, err := eng.PGMinResources(hip.ModeV1, csr)
		if err != nil || agg.Overflow[0] != 0 {
			return CalcPGMinResources(minMember, replicas, pcGetFunc)
		}
		rl := agg.Unflatten(0, gpuName, formats.Formats()) // printed as the reference's sums print
		return &rl
	}
}

// PGRequest is one CalcPGMinResources call of a batch (the arguments of util.go:108).
type PGRequest struct {
	MinMember int32
	Replicas  map[apiv1.ReplicaType]*apiv1.ReplicaSpec
	PcGetFunc PriorityClassGetFunc
}

// PGMinResourcesBatch is CalcPGMinResources for many jobs at once -- a resync of every job's
// PodGroup (job.go:455-457 called in a loop) -- with ONE engine call for all the jobs the tensor path
// holds; the others (and any overflowed job) take the reference's CalcPGMinResources.  out[i] is the
// answer for reqs[i], exactly the reference's.  The engine pays off above hip.BatchCrossoverJobs jobs.
func PGMinResourcesBatch(eng *hip.Engine, gpuName string, reqs []PGRequest) []*v1.ResourceList {
	out := make([]*v1.ResourceList, len(reqs))
	batch := &hip.CSR{}
	idx := make([]int, 0, len(reqs))          // batch job -> request
	formats := make([]*hip.FormatAcc, 0, len(reqs))
	for i, r := range reqs {
		csr, f, err := flattenV1(r.MinMember, r.Replicas, r.PcGetFunc, gpuName)
		if err != nil {
			rl := CalcPGMinResources(r.MinMember, r.Replicas, r.PcGetFunc) // exact reference path
			out[i] = rl
			continue
		}
		batch.AppendJobs(csr)
		idx = append(idx, i)
		formats = append(formats, f)
	}
	if len(idx) == 0 {
		return out
	}
	agg, err := eng.PGMinResources(hip.ModeV1, batch)
	for j, i := range idx {
		r := reqs[i]
		if err != nil || agg.Overflow[j] != 0 {
			out[i] = CalcPGMinResources(r.MinMember, r.Replicas, r.PcGetFunc)
			continue
		}
		rl := agg.Unflatten(j, gpuName, formats[j].Formats())
		out[i] = &rl
	}
	return out
}
