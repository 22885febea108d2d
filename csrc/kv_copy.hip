// K8: paged-KV block copy. One launch copies a list of (src, dst) blocks across every layer of
// both caches (K [L][NB][Hkv*BS*D], V likewise): copy-on-write of a shared tail block, and deep
// snapshot forks (a "send back" continuation that must not share blocks with the live sequence).
// Grid (pairs, layers, 2 caches); each workgroup moves one block of one cache of one layer with
// 16-byte lanes — a block of Llama-3-8B is Hkv*BS*D*2 = 64 KiB, 16 B x 256 lanes x 16 iterations.
#include "common.h"

namespace {
__global__ void __launch_bounds__(256) kv_block_copy_kernel(uint16_t* __restrict__ k, uint16_t* __restrict__ v,
                                                            const int* __restrict__ src, const int* __restrict__ dst,
                                                            int64_t layer_stride, int64_t block_elems, int num_blocks) {
  const int p = blockIdx.x, l = blockIdx.y;
  uint16_t* base = (blockIdx.z == 0 ? k : v) + (size_t)l * layer_stride;
  const int s = src[p], d = dst[p];
  if (s < 0 || s >= num_blocks || d < 0 || d >= num_blocks || s == d) return;   // validated host-side too
  const uint4* from = reinterpret_cast<const uint4*>(base + (size_t)s * block_elems);
  uint4* to = reinterpret_cast<uint4*>(base + (size_t)d * block_elems);
  for (int64_t i = threadIdx.x; i < block_elems / 8; i += blockDim.x) to[i] = from[i];
}
}  // namespace

// k, v: [L, NB, block_elems] bf16; src/dst: device int32 [n]. block_elems % 8 == 0.
int launch_kv_block_copy(void* k, void* v, const int* src, const int* dst, int n, int L, int num_blocks,
                         int64_t block_elems, hipStream_t stream) {
  if (n <= 0) return 0;
  if (L <= 0 || block_elems <= 0 || block_elems % 8 || n > 65535 || L > 65535) return -1;
  hipLaunchKernelGGL(kv_block_copy_kernel, dim3(n, L, 2), dim3(256), 0, stream, (uint16_t*)k, (uint16_t*)v, src, dst,
                     (int64_t)num_blocks * block_elems, block_elems, num_blocks);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
