// K1: RMSNorm / fused residual-add + RMSNorm (+ LayerNorm variants for GPT-2), bf16 I/O, fp32 math.
//
// One workgroup per row. Each thread owns up to MAXC 16-byte chunks (8 bf16) held in
// registers between the reduction and the write, so a row is read exactly once
// (x and residual) and written once (out, residual): the kernel is HBM/latency bound and
// fully vectorized (global_load_dwordx4 / global_store_dwordx4, cdna_hip_programming G13).
#include "common.h"

namespace {
constexpr int MAXC = 4;  // chunks per thread: H <= 1024 threads * 4 * 8 = 32768

template <bool ADD, bool LN>
__global__ void __launch_bounds__(1024) norm_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ x,
                                                    uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
                                                    const uint16_t* __restrict__ b, int H, float eps) {
  __shared__ float scratch[32];
  const int row = blockIdx.x;
  const int nchunk = H >> 3;
  const uint16_t* xr = x + (size_t)row * H;
  uint16_t* rr = ADD ? res + (size_t)row * H : nullptr;
  float v[MAXC][8];
  float ss = 0.f, s1 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      rt::short8 a = *reinterpret_cast<const rt::short8*>(xr + c * 8);
      rt::short8 r;
      if constexpr (ADD) r = *reinterpret_cast<const rt::short8*>(rr + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float f = rt::bf2f((uint16_t)a[j]);
        if constexpr (ADD) {
          // round the residual sum to bf16 exactly as it is stored (matches the torch reference)
          f = rt::bf2f(rt::f2bf(f + rt::bf2f((uint16_t)r[j])));
          r[j] = (short)rt::f2bf(f);
        }
        v[i][j] = f;
        s1 += f;
        ss += f * f;
      }
      if constexpr (ADD) *reinterpret_cast<rt::short8*>(rr + c * 8) = r;
    }
  }
  float mean = 0.f, inv;
  if constexpr (LN) {
    mean = rt::block_sum(s1, scratch) / H;
    float var = rt::block_sum(ss, scratch) / H - mean * mean;
    inv = rsqrtf(fmaxf(var, 0.f) + eps);
  } else {
    inv = rsqrtf(rt::block_sum(ss, scratch) / H + eps);
  }
  uint16_t* orow = out + (size_t)row * H;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nchunk) {
      rt::short8 wv = *reinterpret_cast<const rt::short8*>(w + c * 8);
      rt::short8 bv;
      if constexpr (LN) bv = *reinterpret_cast<const rt::short8*>(b + c * 8);
      rt::short8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float y = (v[i][j] - mean) * inv * rt::bf2f((uint16_t)wv[j]);
        if constexpr (LN) y += rt::bf2f((uint16_t)bv[j]);
        o[j] = (short)rt::f2bf(y);
      }
      *reinterpret_cast<rt::short8*>(orow + c * 8) = o;
    }
  }
}

int norm_threads(int H) {
  int t = ((H / 8 + MAXC - 1) / MAXC + 63) / 64 * 64;
  int want = (H / 8 + 63) / 64 * 64;
  if (want <= 1024) t = want;
  if (t < 64) t = 64;
  if (t > 1024) t = 1024;
  return t;
}
}  // namespace

// H must be a multiple of 8 and <= 32768 (checked by the binding).
void launch_norm(void* out, const void* x, void* res, const void* w, const void* b, int rows, int H, float eps,
                 bool add, bool ln, hipStream_t stream) {
  dim3 grid(rows), block(norm_threads(H));
  auto o = (uint16_t*)out;
  auto xi = (const uint16_t*)x;
  auto r = (uint16_t*)res;
  auto wi = (const uint16_t*)w;
  auto bi = (const uint16_t*)b;
  if (add && ln) hipLaunchKernelGGL((norm_kernel<true, true>), grid, block, 0, stream, o, xi, r, wi, bi, H, eps);
  else if (add) hipLaunchKernelGGL((norm_kernel<true, false>), grid, block, 0, stream, o, xi, r, wi, bi, H, eps);
  else if (ln) hipLaunchKernelGGL((norm_kernel<false, true>), grid, block, 0, stream, o, xi, r, wi, bi, H, eps);
  else hipLaunchKernelGGL((norm_kernel<false, false>), grid, block, 0, stream, o, xi, r, wi, bi, H, eps);
}
