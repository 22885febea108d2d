// Shared device helpers for the roundtable CDNA4 (gfx950) kernels.
// wave64 everywhere: reductions use __shfl_xor over 64 lanes; block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define RT_DEVICE __device__ __forceinline__

namespace rt {

constexpr int kWave = 64;

typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4 __attribute__((ext_vector_type(4)));
typedef float float4_ __attribute__((ext_vector_type(4)));
typedef float float16_ __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// bf16 <-> f32 by bit manipulation (round-to-nearest-even on the way down; NaN kept NaN).
RT_DEVICE float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
// f32 -> bf16 (RNE, NaN-preserving) on the gfx950 converter: one v_cvt_pk_bf16_f32 per PAIR.
// (A bit-twiddled RNE costs ~5 VALU + an exec-masked NaN branch per element — in the
// attention P conversion that was the largest VALU block of the loop.)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
RT_DEVICE uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
RT_DEVICE uint32_t pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}
// raw v_exp_f32 (2^x): exp2f adds a denormal-range rescale (cmp, 2 cndmask, add, ldexp) per call;
// softmax arguments are <= 0 and results below 2^-126 are negligible against the row sum
RT_DEVICE float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

template <typename T> struct DT;
template <> struct DT<uint16_t> {  // bf16 storage
  static RT_DEVICE float load(const uint16_t* p) { return bf2f(*p); }
  static RT_DEVICE void store(uint16_t* p, float v) { *p = f2bf(v); }
};
template <> struct DT<float> {
  static RT_DEVICE float load(const float* p) { return *p; }
  static RT_DEVICE void store(float* p, float v) { *p = v; }
};

RT_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
RT_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64). `scratch` >= 16 floats of LDS.
RT_DEVICE float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = (lane < nw) ? scratch[lane] : 0.f;
  return wave_sum(t);
}
RT_DEVICE float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = (lane < nw) ? scratch[lane] : -INFINITY;
  return wave_max(t);
}

// ---- paged K cache layout (round 6): every [block][kv head] K block is CHUNK-MAJOR,
// [D/32][BS keys][32 dims], not [BS keys][D]: the decode attention's MFMA A fragment for 32-dim
// chunk c (16 keys x 32 dims) is then 8 whole 128-B lines per load instruction instead of 16
// half lines (profiles/r06/attn_kchunk.md). The tensors keep their [NB, Hkv, BS, D] shape
// (same bytes per block); every K writer and reader goes through these two helpers.
RT_DEVICE int kc_elem(int BS, int key, int d) { return (d >> 5) * (BS * 32) + key * 32 + (d & 31); }
// flat 16-B chunk w of one K block -> (key, 16-B chunk c of that key's D-row)
RT_DEVICE void kc_chunk(int w, int BS, int& key, int& c) {
  const int c32 = w / (BS * 4), r = w - c32 * (BS * 4);
  key = r >> 2;
  c = c32 * 4 + (r & 3);
}

// ---- cross-workgroup hand-off I/O (MI355X_MICROARCH "Valid forms": every handed-off byte
// stored sc1 (write-through past the XCD L2) and loaded sc1 (L1-bypassing), 16 B per lane).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSC1 = 16;  // buffer cache-policy aux bit: scc -> sc1 on gfx94x/gfx950
RT_DEVICE __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
RT_DEVICE float4_ sc1_load4(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float4_, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kSC1));
}
RT_DEVICE void sc1_store4(__amdgpu_buffer_rsrc_t r, int byte_off, float4_ v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byte_off, 0, kSC1);
}

}  // namespace rt

#define RT_HIP_CHECK(expr)                                                              \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
    }                                                                                   \
  } while (0)
