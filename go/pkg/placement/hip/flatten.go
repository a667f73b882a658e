package hip

// Object graph <-> engine CSR conversion shared by the v1 and v2 adapters (pure Go, no cgo).
//
// KeyCSR (the adapters' form, pe_pg_min_resources_keys): any resource key -- the reference sums every
// ResourceName (util.go:80-103, coscheduling.go:112-116) -- numbered per call, each key at the finest
// decimal scale its quantities need, so every value is an exact int64 count of 10^scale units.  Only a
// value or a sum with no int64 at that scale (Go's inf.Dec case) is flagged for the reference.
//
// CSR (pe_pg_min_resources, the four fixed dimensions): canonical units (SURVEY.md Appendix A), cpu
// in milli-cores, memory / ephemeral-storage in bytes, one accelerator in units.

import (
	"fmt"
	"math/big"

	corev1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
)

// KeyCSR is the flattened batch of pe_pg_min_resources_keys: the job / group / container structure
// of CSR, and per container its (key, quantity) entries over the batch's key table.
type KeyCSR struct {
	JobGroupOff   []int32 // [J+1]
	MinMember     []int32 // [J] (v1)
	GroupReplicas []int32 // [G], -1 = nil (v1)
	GroupContOff  []int32 // [G+1]
	ContKind      []uint8 // [C] KindContainer / KindInit / KindSidecar / KindOverhead
	EntOff        []int32 // [C+1]: container c's entries are [EntOff[c], EntOff[c+1])
	EntKey        []int32 // key id of each entry
	EntQ          []resource.Quantity
	Keys          []corev1.ResourceName // key id -> name, first-seen order
	keyID         map[corev1.ResourceName]int32
}

func (b *KeyCSR) init() {
	if len(b.JobGroupOff) == 0 {
		b.JobGroupOff = append(b.JobGroupOff, 0)
	}
	if len(b.GroupContOff) == 0 {
		b.GroupContOff = append(b.GroupContOff, 0)
	}
	if len(b.EntOff) == 0 {
		b.EntOff = append(b.EntOff, 0)
	}
	if b.keyID == nil {
		b.keyID = map[corev1.ResourceName]int32{}
		for i, k := range b.Keys {
			b.keyID[k] = int32(i)
		}
	}
}

func (b *KeyCSR) key(name corev1.ResourceName) int32 {
	id, ok := b.keyID[name]
	if !ok {
		id = int32(len(b.Keys))
		b.keyID[name] = id
		b.Keys = append(b.Keys, name)
	}
	return id
}

// AddContainer appends one container record: every key of rl (present even when zero).  A negative
// quantity -- which API validation never admits into a PodSpec -- is an error, not a fallback.
func (b *KeyCSR) AddContainer(rl corev1.ResourceList, kind uint8) error {
	b.init()
	for name, q := range rl {
		if q.Sign() < 0 {
			return &ErrNotTensor{fmt.Sprintf("negative quantity %s=%s", name, q.String())}
		}
	}
	for name, q := range rl {
		b.EntKey = append(b.EntKey, b.key(name))
		b.EntQ = append(b.EntQ, q)
	}
	b.ContKind = append(b.ContKind, kind)
	b.EntOff = append(b.EntOff, int32(len(b.EntKey)))
	return nil
}

// EndGroup closes the current group (replicas: -1 = nil, v1) and EndJob the current job.
func (b *KeyCSR) EndGroup(replicas int32) {
	b.init()
	b.GroupReplicas = append(b.GroupReplicas, replicas)
	b.GroupContOff = append(b.GroupContOff, int32(len(b.ContKind)))
}

func (b *KeyCSR) EndJob(minMember int32) {
	b.init()
	b.MinMember = append(b.MinMember, minMember)
	b.JobGroupOff = append(b.JobGroupOff, int32(len(b.GroupReplicas)))
}

// AppendJobs appends every job of o (one flattenV1 / flattenInfo result per object) to b, rebasing the
// offsets and mapping o's key ids into b's key table: a resync of many PodGroups is ONE batch.
func (b *KeyCSR) AppendJobs(o *KeyCSR) {
	if len(o.JobGroupOff) < 2 {
		return
	}
	b.init()
	g0, c0, e0 := int32(len(b.GroupReplicas)), int32(len(b.ContKind)), int32(len(b.EntKey))
	for _, v := range o.JobGroupOff[1:] {
		b.JobGroupOff = append(b.JobGroupOff, g0+v)
	}
	for _, v := range o.GroupContOff[1:] {
		b.GroupContOff = append(b.GroupContOff, c0+v)
	}
	for _, v := range o.EntOff[1:] {
		b.EntOff = append(b.EntOff, e0+v)
	}
	for _, k := range o.EntKey {
		b.EntKey = append(b.EntKey, b.key(o.Keys[k]))
	}
	b.MinMember = append(b.MinMember, o.MinMember...)
	b.GroupReplicas = append(b.GroupReplicas, o.GroupReplicas...)
	b.ContKind = append(b.ContKind, o.ContKind...)
	b.EntQ = append(b.EntQ, o.EntQ...)
}

// exp10 is the exponent e of q = m * 10^e with m an integer not divisible by 10 (0 for zero): the
// finest decimal scale q needs.
func exp10(q resource.Quantity) int32 {
	d := q.AsDec()
	u := new(big.Int).Set(d.UnscaledBig())
	e := -int32(d.Scale())
	if u.Sign() == 0 {
		return 0
	}
	ten, r := big.NewInt(10), new(big.Int)
	for {
		qq := new(big.Int)
		qq.QuoRem(u, ten, r)
		if r.Sign() != 0 {
			return e
		}
		u = qq
		e++
	}
}

// scaled is q / 10^s when that is an exact int64 >= 0.
func scaled(q resource.Quantity, s int32) (int64, bool) {
	d := q.AsDec()
	u := new(big.Int).Set(d.UnscaledBig())
	if u.Sign() < 0 {
		return 0, false
	}
	k := -int32(d.Scale()) - s // q / 10^s = u * 10^k
	if k >= 0 {
		u.Mul(u, new(big.Int).Exp(big.NewInt(10), big.NewInt(int64(k)), nil))
	} else {
		r := new(big.Int)
		u.QuoRem(u, new(big.Int).Exp(big.NewInt(10), big.NewInt(int64(-k)), nil), r)
		if r.Sign() != 0 {
			return 0, false
		}
	}
	if !u.IsInt64() {
		return 0, false
	}
	return u.Int64(), true
}

// Scales is each key's decimal scale: the finest exponent of its nonzero quantities in the batch (0
// when it has none), so every quantity is an integer count of 10^scale.
func (b *KeyCSR) Scales() []int32 {
	sc := make([]int32, len(b.Keys))
	seen := make([]bool, len(b.Keys))
	for i, q := range b.EntQ {
		if q.IsZero() {
			continue
		}
		k, x := b.EntKey[i], exp10(q)
		if !seen[k] || x < sc[k] {
			sc[k] = x
		}
		seen[k] = true
	}
	return sc
}

// scaledValues converts every entry to its key's scale; a value with no int64 there flags its job
// (jobOvf), as an overflowed sum is flagged.
func (b *KeyCSR) scaledValues(scale []int32) (val []int64, jobOvf []uint8) {
	J := len(b.JobGroupOff) - 1
	val = make([]int64, len(b.EntQ))
	jobOvf = make([]uint8, J)
	for j := 0; j < J; j++ {
		for g := b.JobGroupOff[j]; g < b.JobGroupOff[j+1]; g++ {
			for c := b.GroupContOff[g]; c < b.GroupContOff[g+1]; c++ {
				for x := b.EntOff[c]; x < b.EntOff[c+1]; x++ {
					v, ok := scaled(b.EntQ[x], scale[b.EntKey[x]])
					if !ok {
						jobOvf[j] = 1
						continue
					}
					val[x] = v
				}
			}
		}
	}
	return val, jobOvf
}

// Unflatten turns job j's result back into a ResourceList: one entry per present key (zero values
// included), each NewScaledQuantity(value, scale) printed in the format the reference's sum ends with
// (KeyFormatAcc; DecimalSI when the key has none).
func (a *KeyAgg) Unflatten(j int, formats map[corev1.ResourceName]resource.Format) corev1.ResourceList {
	nk := len(a.Keys)
	out := corev1.ResourceList{}
	for k := 0; k < nk; k++ {
		if !a.Present[j*nk+k] {
			continue
		}
		q := *resource.NewScaledQuantity(a.MinRes[j*nk+k], resource.Scale(a.Scale[k]))
		if f, ok := formats[a.Keys[k]]; ok {
			q.Format = f
		}
		out[a.Keys[k]] = q
	}
	return out
}

// KeyFormatAcc is FormatAcc (below) for any resource key: the Quantity.Add format rule, per name.
type KeyFormatAcc struct {
	fmt     map[corev1.ResourceName]resource.Format
	nonzero map[corev1.ResourceName]bool
}

// Add one contribution of key name (zero = a zero-valued addend, e.g. a product with 0 replicas).
func (a *KeyFormatAcc) Add(name corev1.ResourceName, q resource.Quantity, zero bool) {
	if a.fmt == nil {
		a.fmt = map[corev1.ResourceName]resource.Format{}
		a.nonzero = map[corev1.ResourceName]bool{}
	}
	if _, seen := a.fmt[name]; !seen {
		a.fmt[name] = q.Format
		a.nonzero[name] = !zero
		return
	}
	if !a.nonzero[name] {
		a.fmt[name] = q.Format
	}
	if !zero {
		a.nonzero[name] = true
	}
}

// AddList adds every key of rl, scaled by `scale` for the zero test.
func (a *KeyFormatAcc) AddList(rl corev1.ResourceList, scale int64) {
	for name, q := range rl {
		a.Add(name, q, q.IsZero() || scale == 0)
	}
}

// Formats is Unflatten's formats argument.
func (a *KeyFormatAcc) Formats() map[corev1.ResourceName]resource.Format { return a.fmt }

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
