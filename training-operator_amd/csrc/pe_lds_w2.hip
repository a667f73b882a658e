// LDS digit-plane fit kernels of block size 4096 nodes (W = 2), every field shape.
#include "pe_lds_kernel.h"

namespace pe {

const void* lds_kernel_w2(int n4, int n3, int n2, int n1) { return lds_kernel_for<2>(n4, n3, n2, n1); }

}  // namespace pe
