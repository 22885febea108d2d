// K6: fused sampler — greedy / temperature / top-k / top-p in one kernel, graph-safe RNG.
//
// One 1024-thread workgroup per row (B <= 32 rows, V up to 128256: the row stays
// L2-resident across passes). Sampling is Gumbel-max: token = argmax(z_i + g_i) over the
// allowed set, z = (logit - max)/T, g_i = -log(-log(u_i)), u_i a counter-based hash of
// (seed, offset, i) — no RNG state, so a captured hipGraph replays deterministically
// and the stream of a knight depends only on (seed, knight, position) (the engine passes
// each row's token position as its offset). Top-k and top-p thresholds are found
// EXACTLY with a 4-pass 8-bit radix select over order-preserving float keys, weighted
// by count (top-k) or probability mass (top-p): no sort, no bisection.
// Bit-for-bit RNG twin: theroundtaible_amd/ops/reference.py::uniform_tensor.
#include "common.h"

namespace {
constexpr int NT = 1024;

RT_DEVICE uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
RT_DEVICE float gumbel(uint64_t key, uint32_t i) {
  const uint64_t z = mix64((uint64_t)i + key);
  const float u = ((float)(uint32_t)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
  return -__logf(-__logf(u));
}
RT_DEVICE uint32_t okey(float f) {  // order-preserving float -> uint32
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

template <typename T>
RT_DEVICE float ld(const T* p, int i) {
  return rt::DT<T>::load(p + i);
}

// Radix select: smallest key K such that weight(keys > K) < target <= weight(keys >= K),
// over elements with key >= floor_key. WEIGHTED: weight = exp(z); else weight = 1.
template <typename T, bool WEIGHTED>
RT_DEVICE uint32_t radix_select(const T* row, int V, float mx, float invT, uint32_t floor_key, float target,
                                float* hist, uint32_t* sh_u, float* sh_f) {
  uint32_t prefix = 0, mask = 0;
  float remaining = target;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += NT) hist[b] = 0.f;
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += NT) {
      const float z = (ld(row, i) - mx) * invT;
      const uint32_t k = okey(z);
      if (k >= floor_key && (k & mask) == prefix) {
        const float w = WEIGHTED ? __expf(z) : 1.f;
        atomicAdd(&hist[(k >> shift) & 0xFF], w);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float cum = 0.f;
      int sel = 0;
      for (int b = 255; b >= 0; --b) {
        if (cum + hist[b] >= remaining) {
          sel = b;
          break;
        }
        cum += hist[b];
        if (b == 0) sel = 0;  // rounding: fall back to the lowest bin
      }
      *sh_u = (uint32_t)sel;
      *sh_f = cum;
    }
    __syncthreads();
    prefix |= (*sh_u) << shift;
    mask |= 0xFFu << shift;
    remaining -= *sh_f;
    __syncthreads();
  }
  return prefix;
}

template <typename T>
__global__ void __launch_bounds__(NT) sample_kernel(int64_t* __restrict__ out, const T* __restrict__ logits, int V,
                                                    int64_t ld_row, const float* __restrict__ temperature,
                                                    const float* __restrict__ top_p, const int* __restrict__ top_k,
                                                    const int64_t* __restrict__ seeds,
                                                    const int64_t* __restrict__ offsets) {
  __shared__ float hist[256];
  __shared__ float red_f[32];
  __shared__ int red_i[32];
  __shared__ uint32_t sh_u;
  __shared__ float sh_f;
  const int b = blockIdx.x;
  const T* row = logits + (size_t)b * ld_row;
  const float temp = temperature[b];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  // pass 1: max (greedy: argmax directly)
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += NT) {
    const float v = ld(row, i);
    if (v > best) {  // i increasing per thread: keeps the lowest index on ties
      best = v;
      bi = i;
    }
  }
  auto argmax_reduce = [&](float& v, int& idx) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(idx, o, 64);
      if (ov > v || (ov == v && oi < idx)) {
        v = ov;
        idx = oi;
      }
    }
    if (lane == 0) {
      red_f[wid] = v;
      red_i[wid] = idx;
    }
    __syncthreads();
    v = lane < NT / 64 ? red_f[lane] : -INFINITY;
    idx = lane < NT / 64 ? red_i[lane] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(idx, o, 64);
      if (ov > v || (ov == v && oi < idx)) {
        v = ov;
        idx = oi;
      }
    }
    __syncthreads();
  };
  argmax_reduce(best, bi);
  if (!(temp > 0.f)) {
    if (threadIdx.x == 0) out[b] = bi;
    return;
  }
  const float mx = best;
  const float invT = 1.f / temp;
  uint32_t floor_key = 0;
  const int k = top_k[b];
  if (k > 0 && k < V) floor_key = radix_select<T, false>(row, V, mx, invT, 0u, (float)k, hist, &sh_u, &sh_f);
  const float p = top_p[b];
  if (p < 1.f) {
    float zs = 0.f;
    for (int i = threadIdx.x; i < V; i += NT) {
      const float z = (ld(row, i) - mx) * invT;
      if (okey(z) >= floor_key) zs += __expf(z);
    }
    zs = rt::block_sum(zs, red_f);
    __syncthreads();
    const uint32_t tp = radix_select<T, true>(row, V, mx, invT, floor_key, p * zs, hist, &sh_u, &sh_f);
    floor_key = tp > floor_key ? tp : floor_key;
  }
  const uint64_t key = mix64((uint64_t)seeds[b] ^ mix64((uint64_t)offsets[b]));
  float bv = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += NT) {
    const float z = (ld(row, i) - mx) * invT;
    if (okey(z) >= floor_key) {
      const float s = z + gumbel(key, (uint32_t)i);
      if (s > bv) {
        bv = s;
        bidx = i;
      }
    }
  }
  argmax_reduce(bv, bidx);
  if (threadIdx.x == 0) out[b] = bidx == 0x7fffffff ? bi : bidx;
}
}  // namespace

int launch_sample(int64_t* out, const void* logits, bool is_bf16, int B, int V, int64_t ld_row,
                  const float* temperature, const float* top_p, const int* top_k, const int64_t* seeds,
                  const int64_t* offsets, hipStream_t stream) {
  if (B == 0) return 0;
  if (is_bf16)
    hipLaunchKernelGGL(sample_kernel<uint16_t>, dim3(B), dim3(NT), 0, stream, out, (const uint16_t*)logits, V, ld_row,
                       temperature, top_p, top_k, seeds, offsets);
  else
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(NT), 0, stream, out, (const float*)logits, V, ld_row,
                       temperature, top_p, top_k, seeds, offsets);
  return 0;
}
