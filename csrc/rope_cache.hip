// K2: fused RoPE + paged KV-cache write.
//
// Input is the fused QKV projection row of each token ([Hq | Hkv | Hkv] x D, bf16).
// q and k are rotated with the Llama rotate-half convention using a host-precomputed
// fp32 cos|sin table (no on-device trig: cdna_hip_programming App. B "Element-wise"),
// q is written to its own [T, Hq, D] tensor, k is scattered to the paged key cache
// (chunk-major blocks, [blk][h][D/32][off][32]: common.h kc_elem) and v to the transposed value cache
// ([blk][h][D][off]) that the MFMA P.V B-operand reads with contiguous loads.
// One workgroup per token; each thread rotates 4 pairs (8-byte loads from both halves).
#include "common.h"

namespace {
template <bool ROPE>
__global__ void __launch_bounds__(256) rope_cache_kernel(
    uint16_t* __restrict__ q_out, const uint16_t* __restrict__ qkv, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, uint16_t* __restrict__ k_cache, uint16_t* __restrict__ v_cache,
    const int64_t* __restrict__ slots, int Hq, int Hkv, int D, int BS, int64_t qkv_stride) {
  const int t = blockIdx.x;
  const int64_t slot = slots[t];
  const int64_t blk = slot / BS;
  const int off = (int)(slot - blk * BS);
  const uint16_t* row = qkv + (size_t)t * qkv_stride;
  const int half = D >> 1;
  const int quads = half >> 2;  // 4-pair groups per head
  const float* cs = ROPE ? cos_sin + (size_t)positions[t] * D : nullptr;

  // q and k: (Hq + Hkv) heads x quads
  const int nqk = (Hq + Hkv) * quads;
  for (int i = threadIdx.x; i < nqk; i += blockDim.x) {
    const int h = i / quads;
    const int p = (i - h * quads) * 4;
    const uint16_t* src = row + (size_t)h * D;
    rt::short4 a = *reinterpret_cast<const rt::short4*>(src + p);
    rt::short4 b = *reinterpret_cast<const rt::short4*>(src + half + p);
    rt::short4 oa, ob;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x1 = rt::bf2f((uint16_t)a[j]), x2 = rt::bf2f((uint16_t)b[j]);
      if constexpr (ROPE) {
        const float c = cs[p + j], s = cs[half + p + j];
        const float y1 = x1 * c - x2 * s, y2 = x2 * c + x1 * s;
        x1 = y1;
        x2 = y2;
      }
      oa[j] = (short)rt::f2bf(x1);
      ob[j] = (short)rt::f2bf(x2);
    }
    // 4 dims p..p+3 (p % 4 == 0) never cross a 32-dim chunk
    uint16_t *da, *db;
    if (h < Hq) {
      da = q_out + ((size_t)t * Hq + h) * D + p;
      db = da + half;
    } else {
      uint16_t* kb = k_cache + ((size_t)blk * Hkv + (h - Hq)) * BS * D;
      da = kb + rt::kc_elem(BS, off, p);
      db = kb + rt::kc_elem(BS, off, half + p);
    }
    *reinterpret_cast<rt::short4*>(da) = oa;
    *reinterpret_cast<rt::short4*>(db) = ob;
  }
  // v: Hkv x D elements, transposed store (stride BS)
  const uint16_t* vsrc = row + (size_t)(Hq + Hkv) * D;
  const int nv = Hkv * D;
  for (int i = threadIdx.x; i < nv; i += blockDim.x) {
    const int h = i / D, d = i - h * D;
    v_cache[(((size_t)blk * Hkv + h) * D + d) * BS + off] = vsrc[i];
  }
}
}  // namespace

void launch_rope_cache(void* q_out, const void* qkv, const int64_t* positions, const float* cos_sin,
                       void* k_cache, void* v_cache, const int64_t* slots, int T, int Hq, int Hkv, int D, int BS,
                       int64_t qkv_stride, bool rope, hipStream_t stream) {
  if (T == 0) return;
  dim3 grid(T), block(256);
  if (rope)
    hipLaunchKernelGGL((rope_cache_kernel<true>), grid, block, 0, stream, (uint16_t*)q_out, (const uint16_t*)qkv,
                       positions, cos_sin, (uint16_t*)k_cache, (uint16_t*)v_cache, slots, Hq, Hkv, D, BS, qkv_stride);
  else
    hipLaunchKernelGGL((rope_cache_kernel<false>), grid, block, 0, stream, (uint16_t*)q_out, (const uint16_t*)qkv,
                       positions, cos_sin, (uint16_t*)k_cache, (uint16_t*)v_cache, slots, Hq, Hkv, D, BS, qkv_stride);
}
