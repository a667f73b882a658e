// Engine-side view of the shared-memory exchange (pe_hostx.cpp): its zero-copy windows.
//
// With a pe_host_exchange as the exchange callback, the pipelined multi-rank greedy need not copy
// the lists through the host at all.  The segment is registered with HIP in every rank; each
// window's walk writes its rank's lists straight into its slot of the window's phase, signalled
// per group with the window's generation (the same on every rank: the n-th zero-copy window of
// the segment), and the rank's shard-merge kernel, queued right behind its walk, waits on the
// device for every rank's signal of its group before merging.  No host thread, no barrier, no
// copy: a group's merged list is signalled as soon as the last rank's walk wrote it.
//
// Two ways to merge (pe_engine.cpp): by default each rank's exchange thread polls the slot headers
// in host memory and merges group by group on the host, as soon as every rank's walk wrote the
// group (no kernel, no PCIe read-back); slot reuse then waits for every rank's consumed count.
// PE_ZC_DEV_MERGE=1: a one-block device wait plus the shard merge kernel queued behind the walk;
// there slot reuse needs no counter: window k + 2 reuses phase k & 1, and rank r's walk k + 2 runs
// after its merge k + 1 (one stream), which waited for every peer's walk k + 1, which ran after
// that peer's merge k (its stream) -- the last reader of rank r's window-k slot.
#pragma once
#include <cstddef>
#include <cstdint>

#include "placement.h"

namespace pe {

// the most ranks a segment runs zero-copy windows for (its consumed[] counters; pe_hostx.cpp)
constexpr int HX_ZC_MAX_WORLD = 32;

struct HxWindow {
  uint8_t* dev = nullptr;    // device address of the phase's slot 0 (slot r at dev + r * slot)
  uint8_t* host = nullptr;   // the same bytes, host address
  size_t slot = 0;           // bytes between the ranks' slots
  uint64_t index = 0;        // the window's number in the segment's zero-copy sequence
  uint32_t gen = 0;          // the window's signal generation, nonzero, equal on every rank
};

// is this exchange callback the shared-memory exchange (its user pointer a pe_host_exchange)?
bool hx_is(pe_allgather_fn fn);
// registers the segment with HIP (once per process and segment); false when that fails
bool hx_zc_register(pe_host_exchange* x);
size_t hx_slot_bytes(const pe_host_exchange* x);
// the next zero-copy window (every rank calls it once per window, in the same order)
HxWindow hx_zc_next(pe_host_exchange* x);
// Host-merged windows (the default, pe_engine.cpp): every rank's exchange thread reads all slots of
// a window, so a slot is rewritten (window index + 2, same phase) only after every rank said it
// read window index: hx_zc_consumed after the last group, hx_zc_wait_reuse before the walk that
// rewrites it (false: PE_HX_TIMEOUT_S passed).
bool hx_zc_wait_reuse(pe_host_exchange* x, const HxWindow& w);
void hx_zc_consumed(pe_host_exchange* x, const HxWindow& w);
double hx_timeout_s();

}  // namespace pe
