package hip

// Object graph <-> engine CSR conversion shared by the v1 and v2 adapters (pure Go, no cgo).
// Canonical units (SURVEY.md Appendix A): cpu in milli-cores (exact iff the Quantity has no finer
// scale), memory / ephemeral-storage in bytes and the accelerator in units (exact iff integral).
// Anything else -- another resource key, an inexact or negative value -- is refused, and the
// adapters answer those objects with the reference's own arbitrary-precision code.

import (
	"fmt"

	corev1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
)

// DimNames are the resource keys of the four engine dimensions.
func DimNames(gpuName string) [4]corev1.ResourceName {
	return [4]corev1.ResourceName{corev1.ResourceCPU, corev1.ResourceMemory, corev1.ResourceName(gpuName),
		corev1.ResourceEphemeralStorage}
}

// ErrNotTensor: an input the int64 tensor path does not represent exactly.
type ErrNotTensor struct{ Reason string }

func (e *ErrNotTensor) Error() string { return "placement: not representable: " + e.Reason }

// Canonical is the engine's int64 for quantity q of dimension d.
func Canonical(d int, q resource.Quantity) (int64, error) {
	if q.Sign() < 0 {
		return 0, &ErrNotTensor{fmt.Sprintf("negative quantity %s", q.String())}
	}
	if d == 0 { // cpu: milli-cores, exact only if q has no finer scale than 1m
		m := q.MilliValue()
		if resource.NewMilliQuantity(m, q.Format).Cmp(q) != 0 {
			return 0, &ErrNotTensor{fmt.Sprintf("cpu %s is finer than 1m", q.String())}
		}
		return m, nil
	}
	v, ok := q.AsInt64()
	if !ok {
		return 0, &ErrNotTensor{fmt.Sprintf("%s is not an exact int64", q.String())}
	}
	return v, nil
}

// AddContainer appends one container record: its ResourceList's keys (present even when zero) and
// canonical values, with the record kind.  rl == nil is a record with no keys.
func (b *CSR) AddContainer(rl corev1.ResourceList, kind uint8, gpuName string) error {
	names := DimNames(gpuName)
	var vec [4]int64
	var present uint8
	for key, q := range rl {
		d := -1
		for i, n := range names {
			if n == key {
				d = i
			}
		}
		if d < 0 {
			return &ErrNotTensor{fmt.Sprintf("resource %q is not an engine dimension", key)}
		}
		v, err := Canonical(d, q)
		if err != nil {
			return err
		}
		vec[d] = v
		present |= 1 << uint(d)
	}
	b.ContReq = append(b.ContReq, vec[:]...)
	b.ContFlags = append(b.ContFlags, present|kind<<KindShift)
	return nil
}

// EndGroup closes the current group (replicas: -1 = nil, v1) and EndJob the current job.
func (b *CSR) EndGroup(replicas int32) {
	if len(b.GroupContOff) == 0 {
		b.GroupContOff = append(b.GroupContOff, 0)
	}
	b.GroupReplicas = append(b.GroupReplicas, replicas)
	b.GroupContOff = append(b.GroupContOff, int32(len(b.ContFlags)))
}

func (b *CSR) EndJob(minMember int32) {
	if len(b.JobGroupOff) == 0 {
		b.JobGroupOff = append(b.JobGroupOff, 0)
	}
	if len(b.GroupContOff) == 0 {
		b.GroupContOff = append(b.GroupContOff, 0)
	}
	b.MinMember = append(b.MinMember, minMember)
	b.JobGroupOff = append(b.JobGroupOff, int32(len(b.GroupReplicas)))
}

// Unflatten turns job j's result back into a ResourceList: one entry per present key (zero values
// included, as the reference's maps hold them).  formats, when given, is the Quantity format per
// dimension the reference's Add would have kept (the first contributing quantity's), so that
// String() prints identically; equality (Cmp) never depends on it.
func (a *Agg) Unflatten(j int, gpuName string, formats *[Dims]resource.Format) corev1.ResourceList {
	names := DimNames(gpuName)
	out := corev1.ResourceList{}
	for d := 0; d < Dims; d++ {
		if a.Present[j]&(1<<uint(d)) == 0 {
			continue
		}
		v := a.MinRes[j*Dims+d]
		f := resource.DecimalSI
		if d == 1 || d == 3 {
			f = resource.BinarySI
		}
		if formats != nil {
			f = formats[d]
		}
		if d == 0 {
			out[names[d]] = *resource.NewMilliQuantity(v, f)
		} else {
			out[names[d]] = *resource.NewQuantity(v, f)
		}
	}
	return out
}

// FormatAcc replays the print formats the reference's sums end with, per engine dimension, so that
// Unflatten's quantities print exactly as the reference's (values never depend on it):
//   - AddResourceList (util.go:79-104) deep-copies a key's first quantity (its format), then
//     Quantity.Add adopts the addend's format while the running value is still 0 (apimachinery
//     quantity.go Add: `if q.i.value == 0 { q.Format = y.Format }`, the same on the inf.Dec path);
//   - Build (coscheduling.go:108-118) starts each key from a zero Quantity{} and Adds
//     quantity.Mul(replicas), so the same rule holds (a product with 0 replicas is a zero addend).
// So a key prints in the format of its first nonzero contribution, or of the last one when all are
// zero -- the rule kf::FormatAcc / MinResourcesFormatsV1 implement in the C++ host mirror.
type FormatAcc struct {
	fmt     [Dims]resource.Format
	seen    [Dims]bool
	nonzero [Dims]bool
}

// Add one contribution of dimension d (zero = a zero-valued addend, e.g. a product with 0 replicas).
func (a *FormatAcc) Add(d int, q resource.Quantity, zero bool) {
	if !a.seen[d] {
		a.seen[d] = true
		a.fmt[d] = q.Format
		a.nonzero[d] = !zero
		return
	}
	if !a.nonzero[d] {
		a.fmt[d] = q.Format
	}
	if !zero {
		a.nonzero[d] = true
	}
}

// AddList adds every key of rl that is an engine dimension, scaled by `scale` for the zero test.
func (a *FormatAcc) AddList(rl corev1.ResourceList, gpuName string, scale int64) {
	names := DimNames(gpuName)
	for key, q := range rl {
		for d, n := range names {
			if n == key {
				a.Add(d, q, q.IsZero() || scale == 0)
			}
		}
	}
}

// Formats is Unflatten's formats argument (dimensions never added keep the defaults).
func (a *FormatAcc) Formats() *[Dims]resource.Format {
	out := [Dims]resource.Format{resource.DecimalSI, resource.BinarySI, resource.DecimalSI, resource.BinarySI}
	for d := 0; d < Dims; d++ {
		if a.seen[d] {
			out[d] = a.fmt[d]
		}
	}
	return &out
}

// AppendJobs appends every job of o (a CSR built for other jobs, e.g. one flattenV1 / flattenInfo
// result per object) to b, rebasing o's offsets: a resync of many PodGroups becomes ONE
// pe_pg_min_resources call.  Job j of o becomes job len(b.MinMember) + j of b.
func (b *CSR) AppendJobs(o *CSR) {
	if len(o.JobGroupOff) < 2 {
		return
	}
	if len(b.JobGroupOff) == 0 {
		b.JobGroupOff = append(b.JobGroupOff, 0)
	}
	if len(b.GroupContOff) == 0 {
		b.GroupContOff = append(b.GroupContOff, 0)
	}
	g0 := int32(len(b.GroupReplicas))
	c0 := int32(len(b.ContFlags))
	for _, v := range o.JobGroupOff[1:] {
		b.JobGroupOff = append(b.JobGroupOff, g0+v)
	}
	if len(o.GroupContOff) > 1 {
		for _, v := range o.GroupContOff[1:] {
			b.GroupContOff = append(b.GroupContOff, c0+v)
		}
	}
	b.MinMember = append(b.MinMember, o.MinMember...)
	b.GroupReplicas = append(b.GroupReplicas, o.GroupReplicas...)
	b.ContReq = append(b.ContReq, o.ContReq...)
	b.ContFlags = append(b.ContFlags, o.ContFlags...)
}

// BatchCrossoverJobs is the batch size above which one engine call beats the same arithmetic on
// one CPU core (bench.py `aggregation.crossover_jobs`, measured on the MI355X box: see
// INTEGRATION.md).  Below it a per-object call costs a kernel round trip over PCIe (~12 us) for
// work the CPU does in well under a microsecond, so callers with few objects keep the reference
// path; the batch entry points below take the engine for any size (the caller decides).
// Round-4 box run: 4096 jobs per call, GPU 51.8 us vs one core 59.6 us (3072: 45.9 vs 42.9).
const BatchCrossoverJobs = 4096
