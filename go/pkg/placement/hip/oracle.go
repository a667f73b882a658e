package hip

// CPU oracle of the engine's best-fit rule (SURVEY.md Appendix B), in the plugin's own language and
// package: the "Go CPU oracle of the identical best-fit rule that lives in the same plugin" of the
// north star.  Pure Go, no cgo: a controller can cross-check the GPU answer of FitMask / PlaceGreedy
// on a sample (or answer without a GPU) with the same rule.  Function for function it restates
// oracle/oracle.c (the C oracle the repository's tests pin the GPU against, bit-exact):
//
//	fits          oracle.c fits
//	Score         oracle.c orc_score
//	Key           oracle.c node_key / orc_key
//	argminKey     oracle.c argmin_key
//	FitMaskCPU    oracle.c orc_fit_mask (row-major [J][ceil(N/64)] words)
//	PlaceGreedyCPU oracle.c orc_place_greedy (island groups, all-or-nothing rollback)
//
// Residuals are SoA [4][N] int64 (cpu milli, memory B, accelerators, ephemeral-storage B), node
// labels u32 (bit 31 = the node has an xGMI island, LabelIsland).  No reference function exists for
// this rule: the reference operator leaves placement to an external gang scheduler (SURVEY.md 0.2).

import (
	"math"
	"sort"
)

const (
	ScoreMax   = uint64(1)<<40 - 1 // score saturation (Appendix B)
	KeyShift   = 24                // key = score << KeyShift | node id
	NodeIDMask = uint64(1)<<KeyShift - 1
	MemShift   = 20 // memory term: leftover bytes >> 20 (1 MiB ~ 1 milli-cpu)
	GPUShift   = 20 // accelerator term: leftover count << 20 (packs GPU leftovers first)
	EphShift   = 24 // ephemeral-storage term: leftover bytes >> 24 (16 MiB)
	NoKey      = ^uint64(0)
)

// LabelIsland / NeedIsland mirror placement.h PE_LABEL_ISLAND / PE_NEED_ISLAND.
const (
	LabelIsland = uint32(0x80000000)
	NeedIsland  = LabelIsland
)

// fits: labels cover need and every request fits the residual (signed int64 compares).
func fits(res []int64, n, N int64, labels uint32, q *[Dims]int64, need uint32) bool {
	if labels&need != need {
		return false
	}
	for d := 0; d < Dims; d++ {
		if q[d] > res[int64(d)*N+n] {
			return false
		}
	}
	return true
}

// Score of the leftovers after a fit, computed in u64 and saturated at ScoreMax (oracle.c orc_score).
func Score(left *[Dims]int64) uint64 {
	a := uint64(left[0])
	b := uint64(left[1]) >> MemShift
	var c uint64
	if uint64(left[2]) >= 1<<20 {
		c = ScoreMax
	} else {
		c = uint64(left[2]) << GPUShift
	}
	e := uint64(left[3]) >> EphShift
	a, b, c, e = min64(a, ScoreMax), min64(b, ScoreMax), min64(c, ScoreMax), min64(e, ScoreMax)
	return min64(a+b+c+e, ScoreMax)
}

func min64(a, b uint64) uint64 {
	if a < b {
		return a
	}
	return b
}

// Key of node n (global id gid) for request (q, need): (Score << 24) | gid, NoKey when it does not fit.
func Key(res []int64, n, N int64, gid uint64, labels uint32, q *[Dims]int64, need uint32) uint64 {
	if !fits(res, n, N, labels, q, need) {
		return NoKey
	}
	var left [Dims]int64
	for d := 0; d < Dims; d++ {
		left[d] = res[int64(d)*N+n] - q[d]
	}
	return Score(&left)<<KeyShift | gid
}

// argminKey: the smallest key over all nodes (ties: the lowest node id, which the key carries).
func argminKey(res []int64, labels []uint32, N int64, q *[Dims]int64, need uint32) uint64 {
	best := NoKey
	for n := int64(0); n < N; n++ {
		if k := Key(res, n, N, uint64(n), labels[n], q, need); k < best {
			best = k
		}
	}
	return best
}

// FitMaskCPU is the what-if feasibility matrix (config 5): bit n%64 of word [j][n/64] = job j fits
// node n; counts[j] = nodes job j fits.  req is [J][4], need [J].
func FitMaskCPU(res []int64, labels []uint32, N int64, req []int64, need []uint32) (mask []uint64, counts []int64) {
	J := int64(len(need))
	W := (N + 63) / 64
	mask = make([]uint64, J*W)
	counts = make([]int64, J)
	for j := int64(0); j < J; j++ {
		var q [Dims]int64
		copy(q[:], req[j*Dims:(j+1)*Dims])
		for n := int64(0); n < N; n++ {
			if fits(res, n, N, labels[n], &q, need[j]) {
				mask[j*W+n/64] |= 1 << uint(n%64)
				counts[j]++
			}
		}
	}
	return mask, counts
}

func mulOvf(a, b int64) (int64, bool) {
	if a == 0 || b == 0 {
		return 0, false
	}
	c := a * b
	if c/b != a || (a == -1 && b == math.MinInt64) || (b == -1 && a == math.MinInt64) {
		return c, true
	}
	return c, false
}

// PlaceGreedyCPU is the sequential greedy best-fit gang placement, the engine's PlaceGreedy rule:
// jobs in (priority desc, index asc) order, groups in the given order, each pod on the argmin-key
// node; an island group (need bit 31) puts its count pods as one unit (count x request, overflow =
// fits nowhere) on one node; a job that cannot place a pod rolls back every pod it placed.  res
// ([4][N]) is updated in place.  Returns the per-pod node (-1 = none) in group-input order and the
// per-job status (JobPlaced / JobUnschedulable).
func PlaceGreedyCPU(res []int64, labels []uint32, N int64, jobGroupOff, priority, groupCount []int32,
	groupReq []int64, groupNeed []uint32) (podNode []int32, jobStatus []int32) {
	J := len(priority)
	G := int(jobGroupOff[J])
	podOff := make([]int64, G+1)
	for g := 0; g < G; g++ {
		c := int64(groupCount[g])
		if c < 0 {
			c = 0
		}
		podOff[g+1] = podOff[g] + c
	}
	podNode = make([]int32, podOff[G])
	for i := range podNode {
		podNode[i] = -1
	}
	jobStatus = make([]int32, J)
	order := make([]int, J)
	for j := range order {
		order[j] = j
	}
	sort.SliceStable(order, func(a, b int) bool { return priority[order[a]] > priority[order[b]] })
	take := func(n int64, q *[Dims]int64, sign int64) {
		for d := 0; d < Dims; d++ {
			res[int64(d)*N+n] -= sign * q[d]
		}
	}
	for _, j := range order {
		ok := true
		for g := jobGroupOff[j]; g < jobGroupOff[j+1] && ok; g++ {
			var q [Dims]int64
			copy(q[:], groupReq[int64(g)*Dims:int64(g+1)*Dims])
			if groupNeed[g]&NeedIsland != 0 {
				if groupCount[g] <= 0 {
					continue
				}
				var qe [Dims]int64
				ovf := false
				for d := 0; d < Dims; d++ {
					var o bool
					qe[d], o = mulOvf(q[d], int64(groupCount[g]))
					ovf = ovf || o
				}
				k := NoKey
				if !ovf {
					k = argminKey(res, labels, N, &qe, groupNeed[g])
				}
				if k == NoKey {
					ok = false
					break
				}
				n := int64(k & NodeIDMask)
				take(n, &qe, 1)
				for p := int64(0); p < int64(groupCount[g]); p++ {
					podNode[podOff[g]+p] = int32(n)
				}
				continue
			}
			for p := int64(0); p < int64(groupCount[g]); p++ {
				k := argminKey(res, labels, N, &q, groupNeed[g])
				if k == NoKey {
					ok = false
					break
				}
				n := int64(k & NodeIDMask)
				take(n, &q, 1)
				podNode[podOff[g]+p] = int32(n)
			}
		}
		if ok {
			jobStatus[j] = JobPlaced
			continue
		}
		// all-or-nothing: give back every pod of the job (an island group's pods share one node and
		// each gives back one request, count x request in all)
		for g := jobGroupOff[j]; g < jobGroupOff[j+1]; g++ {
			var q [Dims]int64
			copy(q[:], groupReq[int64(g)*Dims:int64(g+1)*Dims])
			for p := int64(0); p < int64(groupCount[g]); p++ {
				if n := podNode[podOff[g]+p]; n >= 0 {
					take(int64(n), &q, -1)
					podNode[podOff[g]+p] = -1
				}
			}
		}
		jobStatus[j] = JobUnschedulable
	}
	return podNode, jobStatus
}
