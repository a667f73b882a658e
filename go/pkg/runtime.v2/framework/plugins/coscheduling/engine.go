/*
Engine-backed CoScheduling plugin: a drop-in for coscheduling.New in the v2 plugin registry.

The reference plugin is pkg/runtime.v2/framework/plugins/coscheduling/coscheduling.go.  This file is
added next to it (same package) and keeps everything but the aggregation: EnforcePodGroupPolicy,
the watch extension (ReconcilerBuilders, coscheduling.go:298-320), the indexers set up by New
(:71-85) and needsCreateOrUpdate (:150-153) are the reference's own.  Build (:103-148) computes
MinMember / MinResources (:108-118) with one pe_pg_min_resources_keys(PE_MODE_V2) call on the GPU
instead of the Quantity loop, over every resource key the TotalRequests name (a per-call key table,
each key at the decimal scale its quantities need).  The one object handed to the reference's Build
is one whose sum has no int64 at its scale (Overflow: the reference's inf.Dec case).

Registration (registry.go:32-42) -- the same name, so the framework's type assertions
(framework.go:53-77) see the same capabilities:

	func NewRegistryWithEngine(eng *hip.Engine, gpuName string) Registry {
		r := NewRegistry()
		r[coscheduling.Name] = coscheduling.NewWithEngine(eng, gpuName)
		return r
	}
*/
package coscheduling

import (
	"context"
	"sort"

	corev1 "k8s.io/api/core/v1"
	apierrors "k8s.io/apimachinery/pkg/api/errors"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/utils/ptr"
	"sigs.k8s.io/controller-runtime/pkg/client"
	ctrlutil "sigs.k8s.io/controller-runtime/pkg/controller/controllerutil"
	schedulerpluginsv1alpha1 "sigs.k8s.io/scheduler-plugins/apis/scheduling/v1alpha1"

	kubeflowv2 "github.com/kubeflow/training-operator/pkg/apis/kubeflow.org/v2alpha1"
	"github.com/kubeflow/training-operator/pkg/constants"
	"github.com/kubeflow/training-operator/pkg/placement/hip"
	runtime "github.com/kubeflow/training-operator/pkg/runtime.v2"
	"github.com/kubeflow/training-operator/pkg/runtime.v2/framework"
)

// EngineCoScheduling is CoScheduling with Build's aggregation on the GPU.
type EngineCoScheduling struct {
	*CoScheduling
	eng     *hip.Engine
	gpuName string
}

var _ framework.EnforcePodGroupPolicyPlugin = (*EngineCoScheduling)(nil)
var _ framework.WatchExtensionPlugin = (*EngineCoScheduling)(nil)
var _ framework.ComponentBuilderPlugin = (*EngineCoScheduling)(nil)

// NewWithEngine returns the plugin factory (registry.go:32's signature) of the engine-backed plugin.
func NewWithEngine(eng *hip.Engine, gpuName string) func(ctx context.Context, c client.Client,
	indexer client.FieldIndexer) (framework.Plugin, error) {
	return func(ctx context.Context, c client.Client, indexer client.FieldIndexer) (framework.Plugin, error) {
		p, err := New(ctx, c, indexer) // indexers + client exactly as the reference (coscheduling.go:71-85)
		if err != nil {
			return nil, err
		}
		return &EngineCoScheduling{CoScheduling: p.(*CoScheduling), eng: eng, gpuName: gpuName}, nil
	}
}

// flattenInfo turns info.TotalRequests into the engine's v2 CSR: one job, one group per entry
// (Replicas, and its PodRequests as one container record -- NewInfo has already applied kueue's
// TotalRequests, runtime.go:130-136).  Entries in name order: the sums do not depend on it, and the
// print formats (hip.FormatAcc: the first nonzero quantity x replicas Build adds per key) follow
// one of the orders the reference's map range can take.
func flattenInfo(info *runtime.Info) (*hip.KeyCSR, *hip.KeyFormatAcc, error) {
	names := make([]string, 0, len(info.TotalRequests))
	for name := range info.TotalRequests {
		names = append(names, name)
	}
	sort.Strings(names)
	b := &hip.KeyCSR{}
	acc := &hip.KeyFormatAcc{}
	for _, name := range names {
		trr := info.TotalRequests[name]
		if err := b.AddContainer(trr.PodRequests, hip.KindContainer); err != nil {
			return nil, nil, err
		}
		acc.AddList(trr.PodRequests, int64(trr.Replicas))
		b.EndGroup(trr.Replicas)
	}
	b.EndJob(0)
	return b, acc, nil
}

// unflatten is job 0's ResourceList, printed in the formats the reference's Build would print.
func unflatten(agg *hip.KeyAgg, formats *hip.KeyFormatAcc) corev1.ResourceList {
	return agg.Unflatten(0, formats.Formats())
}

// Build is coscheduling.go:103-148 with the aggregation (:108-118) on the engine; the PodGroup is
// emitted by buildPodGroup, the one copy of :119-147 both Builds call.
func (c *EngineCoScheduling) Build(ctx context.Context, obj client.Object, info *runtime.Info,
	trainJob *kubeflowv2.TrainJob) (client.Object, error) {
	if info == nil || info.RuntimePolicy.PodGroupPolicy == nil || info.RuntimePolicy.PodGroupPolicy.Coscheduling == nil || trainJob == nil {
		return nil, nil
	}
	csr, formats, ferr := flattenInfo(info)
	if ferr != nil {
		return nil, ferr // a negative quantity: API validation never admits one
	}
	agg, err := c.eng.PGMinResourcesKeys(hip.ModeV2, csr)
	if err != nil {
		return nil, err
	}
	if agg.Overflow[0] != 0 {
		return c.CoScheduling.Build(ctx, obj, info, trainJob) // the inf.Dec case: exact reference path
	}
	return c.CoScheduling.buildPodGroup(ctx, info, trainJob, agg.Members[0], unflatten(agg, formats))
}

// BuildBatch is Build for many TrainJobs at once (a resync of every TrainJob's PodGroup): ONE engine
// call (per slice of hip.MaxKeys keys) aggregates every (info, trainJob) pair, the PodGroups are then
// emitted one by one exactly as Build emits them; pairs whose sums overflow take the reference's
// Build (the inf.Dec case).  objs[i] / errs[i] answer (infos[i], trainJobs[i]).  The engine pays off
// above hip.BatchCrossoverJobs pairs; the C++ mirror's kf::CoScheduling::BuildBatch is the same loop.
func (c *EngineCoScheduling) BuildBatch(ctx context.Context, infos []*runtime.Info,
	trainJobs []*kubeflowv2.TrainJob) ([]client.Object, []error) {
	objs := make([]client.Object, len(infos))
	errs := make([]error, len(infos))
	batch := &hip.KeyCSR{}
	idx := make([]int, 0, len(infos))
	formats := make([]*hip.KeyFormatAcc, 0, len(infos))
	for i, info := range infos {
		if info == nil || info.RuntimePolicy.PodGroupPolicy == nil || info.RuntimePolicy.PodGroupPolicy.Coscheduling == nil ||
			trainJobs[i] == nil {
			continue // (nil, nil), as Build
		}
		csr, f, ferr := flattenInfo(info)
		if ferr != nil {
			errs[i] = ferr // a negative quantity, as Build
			continue
		}
		batch.AppendJobs(csr)
		idx = append(idx, i)
		formats = append(formats, f)
	}
	if len(idx) == 0 {
		return objs, errs
	}
	agg, err := c.eng.PGMinResourcesKeys(hip.ModeV2, batch)
	for j, i := range idx {
		switch {
		case err != nil:
			errs[i] = err
		case agg.Overflow[j] != 0:
			objs[i], errs[i] = c.CoScheduling.Build(ctx, nil, infos[i], trainJobs[i]) // the inf.Dec case
		default:
			objs[i], errs[i] = c.CoScheduling.buildPodGroup(ctx, infos[i], trainJobs[i], agg.Members[j],
				agg.Unflatten(j, formats[j].Formats()))
		}
	}
	return objs, errs
}

// buildPodGroup is the PodGroup emission of coscheduling.go:119-147 -- the object, its controller
// reference, the existing object's Get and needsCreateOrUpdate (:150-153) -- factored out of Build so
// that one copy serves both plugins.  The reference's Build ends in it after its own aggregation
// loop (INTEGRATION.md, "v2 plugin"):
//
//	return c.buildPodGroup(ctx, info, trainJob, totalMembers, totalResources)
func (c *CoScheduling) buildPodGroup(ctx context.Context, info *runtime.Info, trainJob *kubeflowv2.TrainJob,
	members int32, resources corev1.ResourceList) (client.Object, error) {
	newPG := &schedulerpluginsv1alpha1.PodGroup{
		TypeMeta: metav1.TypeMeta{
			APIVersion: schedulerpluginsv1alpha1.SchemeGroupVersion.String(),
			Kind:       constants.PodGroupKind,
		},
		ObjectMeta: metav1.ObjectMeta{
			Name:      trainJob.Name,
			Namespace: trainJob.Namespace,
		},
		Spec: schedulerpluginsv1alpha1.PodGroupSpec{
			ScheduleTimeoutSeconds: info.RuntimePolicy.PodGroupPolicy.Coscheduling.ScheduleTimeoutSeconds,
			MinMember:              members,
			MinResources:           resources,
		},
	}
	if err := ctrlutil.SetControllerReference(trainJob, newPG, c.scheme); err != nil {
		return nil, err
	}
	oldPG := &schedulerpluginsv1alpha1.PodGroup{}
	if err := c.client.Get(ctx, client.ObjectKeyFromObject(newPG), oldPG); err != nil {
		if !apierrors.IsNotFound(err) {
			return nil, err
		}
		oldPG = nil
	}
	if needsCreateOrUpdate(oldPG, newPG, ptr.Deref(trainJob.Spec.Suspend, false)) {
		return newPG, nil
	}
	return nil, nil
}
