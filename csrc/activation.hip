// K5: SwiGLU (silu(gate) * up) and GELU-tanh; bf16 in/out, fp32 math, 16-byte vector I/O.
#include "common.h"

namespace {
RT_DEVICE float silu(float x) { return x / (1.f + __expf(-x)); }
RT_DEVICE float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

// grid-stride over [rows, I/8] chunks; x row = [gate(I) | up(I)]
__global__ void __launch_bounds__(256) silu_mul_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ x,
                                                       int rows, int I) {
  const int cpr = I >> 3;
  const int64_t total = (int64_t)rows * cpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cpr;
    const int c = (int)(i - r * cpr);
    const uint16_t* xr = x + r * 2 * I;
    rt::short8 g = *reinterpret_cast<const rt::short8*>(xr + c * 8);
    rt::short8 u = *reinterpret_cast<const rt::short8*>(xr + I + c * 8);
    rt::short8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (short)rt::f2bf(silu(rt::bf2f((uint16_t)g[j])) * rt::bf2f((uint16_t)u[j]));
    *reinterpret_cast<rt::short8*>(out + r * I + c * 8) = o;
  }
}

__global__ void __launch_bounds__(256) gelu_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ x,
                                                   int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    rt::short8 v = *reinterpret_cast<const rt::short8*>(x + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (short)rt::f2bf(gelu_tanh(rt::bf2f((uint16_t)v[j])));
    *reinterpret_cast<rt::short8*>(out + i * 8) = v;
  }
}

int grid_for(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 2048) g = 2048;  // 256 CUs x 8; grid-stride the rest (G11)
  if (g < 1) g = 1;
  return (int)g;
}
}  // namespace

void launch_silu_mul(void* out, const void* x, int rows, int I, hipStream_t stream) {
  if (rows == 0) return;
  hipLaunchKernelGGL(silu_mul_kernel, dim3(grid_for((int64_t)rows * (I / 8))), dim3(256), 0, stream,
                     (uint16_t*)out, (const uint16_t*)x, rows, I);
}

void launch_gelu(void* out, const void* x, int64_t n, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(n / 8)), dim3(256), 0, stream, (uint16_t*)out,
                     (const uint16_t*)x, n / 8);
}
