// Radix sort of the sorted-walk keys (pe_kernels.h WalkIndex), kept in its own translation unit so
// the rocPRIM templates compile once.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "pe_kernels.h"

namespace pe {

hipError_t sort_keys_u64(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out, int64_t n, hipStream_t s) {
  return rocprim::radix_sort_keys(temp, *temp_bytes, in, out, (size_t)n, 0, 64, s);
}

}  // namespace pe
