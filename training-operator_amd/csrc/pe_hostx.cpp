// Intra-node host exchange: the all-gather of the greedy windows' candidate lists through POSIX
// shared memory, for ranks of one node whose RCCL communicator could not be set up (include/
// placement.h pe_host_exchange_*).  It is a pe_allgather_fn, so the engine's pipelined multi-rank
// loop runs unchanged over it (the helper thread exchanges window w+1 while the host resolves w).
//
// Layout of the segment: a 4 KiB header (magic, world, slot bytes, attach count, two arrival
// counters), then four phases x world slots of `max_bytes`: phases 0-1 for the copying all-gather
// below, 2-3 for the engine's zero-copy windows (pe_hostx.h).  Call k of every rank uses phase
// p = k & 1: write the own block into slot [p][rank], count the arrival in ctr[p], wait until all
// world ranks arrived (ctr[p] == world * (k / 2 + 1)), copy the world slots out.  One barrier per
// call suffices: slot [p][r] is rewritten at call k + 2 only after barrier k + 1, which every rank
// reaches only after it copied call k's slots.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <immintrin.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "pe_hostx.h"
#include "placement.h"

namespace {

constexpr uint64_t kMagic = 0x70655f6878303031ull;   // "pe_hx001"
constexpr size_t kHdr = 4096;
constexpr int kZcMaxWorld = pe::HX_ZC_MAX_WORLD;

struct Hdr {
  std::atomic<uint64_t> magic;
  int32_t world;
  int32_t pad;
  uint64_t slot_bytes;
  std::atomic<int32_t> attached;
  alignas(64) std::atomic<uint64_t> ctr[2][8];   // ctr[p][0]; the rest pads to separate cache lines
  // zero-copy windows: consumed[r][0] = windows rank r has read every slot of (pe_hostx.h)
  alignas(64) std::atomic<uint64_t> consumed[kZcMaxWorld][8];
};
static_assert(sizeof(Hdr) <= kHdr, "header");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory atomics must be lock-free");

double timeout_s() {
  const char* e = std::getenv("PE_HX_TIMEOUT_S");
  const double s = e ? std::atof(e) : 300.0;
  return s > 0 ? s : 300.0;
}

}  // namespace

struct pe_host_exchange {
  Hdr* h = nullptr;
  uint8_t* data = nullptr;
  size_t map_bytes = 0;
  int32_t rank = 0, world = 1;
  uint64_t calls = 0;
  uint64_t zc_windows = 0;   // zero-copy windows issued (pe_hostx.h)
  int zc_reg = 0;            // 1: registered with HIP, -1: registration failed
  uint8_t* zc_dev = nullptr; // device address of the segment's data
  std::string name;
};

extern "C" {

int pe_host_exchange_open(const char* name, int32_t rank, int32_t world, size_t max_bytes, pe_host_exchange** out) {
  if (!name || !out || name[0] != '/' || world < 1 || rank < 0 || rank >= world || max_bytes == 0) return PE_EINVAL;
  *out = nullptr;
  const size_t slot = (max_bytes + 63) & ~(size_t)63;
  const size_t total = kHdr + 4 * (size_t)world * slot;
  int fd = -1;
  const auto t0 = std::chrono::steady_clock::now();
  auto waited = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  if (rank == 0) {
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return PE_ESTATE;   // the name exists: a stale or concurrent segment
    if (ftruncate(fd, (off_t)total) != 0) {
      close(fd);
      shm_unlink(name);
      return PE_ENOMEM;
    }
  } else {   // rank 0 creates it: wait for the segment, its size and its magic
    for (;;) {
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size == total) break;
        close(fd);
        fd = -1;
      }
      if (waited() > timeout_s()) return PE_ESTATE;
      usleep(1000);
    }
  }
  void* m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    if (rank == 0) shm_unlink(name);
    return PE_ENOMEM;
  }
  Hdr* h = static_cast<Hdr*>(m);
  if (rank == 0) {
    h->world = world;
    h->slot_bytes = slot;
    new (&h->attached) std::atomic<int32_t>(0);
    for (auto& c : h->ctr) new (&c[0]) std::atomic<uint64_t>(0);
    for (auto& c : h->consumed) new (&c[0]) std::atomic<uint64_t>(0);
    h->magic.store(kMagic, std::memory_order_release);
  } else {
    while (h->magic.load(std::memory_order_acquire) != kMagic) {
      if (waited() > timeout_s()) {
        munmap(m, total);
        return PE_ESTATE;
      }
      usleep(1000);
    }
    if (h->world != world || h->slot_bytes != slot) {
      munmap(m, total);
      return PE_EINVAL;
    }
  }
  // the last rank to attach removes the name: the mapping stays, nothing is left in /dev/shm
  if (h->attached.fetch_add(1, std::memory_order_acq_rel) + 1 == world) shm_unlink(name);
  auto* x = new (std::nothrow) pe_host_exchange;
  if (!x) {
    munmap(m, total);
    return PE_ENOMEM;
  }
  x->h = h;
  x->data = static_cast<uint8_t*>(m) + kHdr;
  x->map_bytes = total;
  x->rank = rank;
  x->world = world;
  x->name = name;
  *out = x;
  return PE_OK;
}

int pe_host_exchange_allgather(void* user, const void* send, void* recv, size_t bytes) {
  auto* x = static_cast<pe_host_exchange*>(user);
  if (!x || (!send && bytes) || (!recv && bytes)) return PE_EINVAL;
  const size_t slot = x->h->slot_bytes;
  if (bytes > slot) return PE_EINVAL;
  const int p = (int)(x->calls & 1);
  const uint64_t target = (uint64_t)x->world * (x->calls / 2 + 1);
  ++x->calls;
  uint8_t* base = x->data + (size_t)p * x->world * slot;
  if (bytes) std::memcpy(base + (size_t)x->rank * slot, send, bytes);
  std::atomic<uint64_t>& c = x->h->ctr[p][0];
  c.fetch_add(1, std::memory_order_acq_rel);   // release: the block is visible before the arrival
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0; c.load(std::memory_order_acquire) < target; ++spin) {
    if (spin < 4096) {
      _mm_pause();
      continue;
    }
    sched_yield();
    if ((spin & 1023) == 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s())
      return PE_ERCCL;   // a peer never arrived
  }
  for (int r = 0; r < x->world; ++r)
    if (bytes) std::memcpy(static_cast<uint8_t*>(recv) + (size_t)r * bytes, base + (size_t)r * slot, bytes);
  return PE_OK;
}

void pe_host_exchange_close(pe_host_exchange* x) {
  if (!x) return;
  if (x->zc_reg == 1) (void)hipHostUnregister(x->h);
  if (x->rank == 0) shm_unlink(x->name.c_str());   // (ENOENT once every rank attached)
  munmap(x->h, x->map_bytes);
  delete x;
}

}  // extern "C"

namespace pe {

bool hx_is(pe_allgather_fn fn) { return fn == &pe_host_exchange_allgather; }

bool hx_zc_register(pe_host_exchange* x) {
  if (!x || x->world > kZcMaxWorld) return false;
  if (x->zc_reg == 0) {
    void* dev = nullptr;
    x->zc_reg = -1;
    if (hipHostRegister(x->h, x->map_bytes, hipHostRegisterMapped | hipHostRegisterPortable) == hipSuccess) {
      if (hipHostGetDevicePointer(&dev, x->h, 0) == hipSuccess && dev) {
        x->zc_dev = static_cast<uint8_t*>(dev) + kHdr;
        x->zc_reg = 1;
      } else {
        (void)hipHostUnregister(x->h);
      }
    }
    (void)hipGetLastError();   // (a failed registration is an answer, not a sticky error)
  }
  return x->zc_reg == 1;
}

size_t hx_slot_bytes(const pe_host_exchange* x) { return x ? (size_t)x->h->slot_bytes : 0; }

HxWindow hx_zc_next(pe_host_exchange* x) {
  HxWindow w;
  const size_t slot = x->h->slot_bytes;
  const uint64_t k = x->zc_windows++;
  w.dev = x->zc_dev + (2 + (size_t)(k & 1)) * x->world * slot;
  w.host = x->data + (2 + (size_t)(k & 1)) * x->world * slot;
  w.index = k;
  w.slot = slot;
  w.gen = (uint32_t)(k % 0xFFFFFFFFull) + 1;   // (slot headers start zeroed: generation 0 is never current)
  return w;
}

}  // namespace pe

namespace pe {

bool hx_zc_wait_reuse(pe_host_exchange* x, const HxWindow& w) {
  if (w.index < 2) return true;
  const uint64_t need = w.index - 1;   // windows 0 .. index - 2 read by every rank
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < x->world; ++r)
    for (unsigned spin = 0; x->h->consumed[r][0].load(std::memory_order_acquire) < need; ++spin) {
      _mm_pause();
      if ((spin & 4095) == 4095 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s())
        return false;
    }
  return true;
}

void hx_zc_consumed(pe_host_exchange* x, const HxWindow& w) {
  x->h->consumed[x->rank][0].store(w.index + 1, std::memory_order_release);
}

double hx_timeout_s() { return timeout_s(); }

}  // namespace pe
