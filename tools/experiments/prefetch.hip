// Cache warm-up: stream a byte range through the memory hierarchy so it is resident in the
// 256 MB MALL (Infinity Cache) before its consumer runs. Launched on a side stream / hipGraph
// branch next to a latency-bound kernel (decode attention) whose HBM pipe is otherwise idle,
// so the next GEMM's weights arrive from MALL instead of HBM. Few workgroups on purpose: it
// must not take CU slots from the kernel it overlaps. Loads are default-policy (allocating),
// 16 B per lane, 8 in flight per lane; the XOR sink keeps them from being optimised away.
#include "common.h"

namespace {
__global__ void __launch_bounds__(256) prefetch_kernel(const uint4* __restrict__ p, int64_t n16,
                                                       uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[i + j * stride];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == 0x9e3779b9u) *sink = acc;  // practically never taken; defeats dead-code elimination
}
}  // namespace

int launch_prefetch(const void* p, int64_t nbytes, int nwg, uint32_t* sink, hipStream_t stream) {
  if (nbytes < 16 || nwg < 1) return 0;
  hipLaunchKernelGGL(prefetch_kernel, dim3(nwg), dim3(256), 0, stream, (const uint4*)p, nbytes / 16, sink);
  return 0;
}
