// Experiment: is a decode GEMM's time set by its bytes or by the busiest CU's tile count?
// gate_up has 896 16-column tiles on 256 CUs (3.5 per CU), qkv 384 (1.5 per CU). Time the
// production skinny kernel (skinny_core.h, M = 3) over tile counts around those: if 1024 tiles
// cost about what 896 cost, the last half-wave of tiles is what the GEMM waits for.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/exp_balance.hip -o build/exp_balance
#include "skinny_core.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace skinny;
using rt::short8;

namespace {
template <int PRO, int EPI, int NW, int U>
__global__ void __launch_bounds__(NW * 64) plain_kernel(GemmArgs p) {
  __shared__ GemmSmem<nacc<EPI>(), NW> sm;
  Stage<PRO, EPI, U> st0;
  gemm_tile<PRO, EPI, NW, U, false>(p, blockIdx.x, sm, st0, false, false);
}

__global__ void fill_kernel(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = rt::f2bf(((int)(h & 0xffff) - 32768) * (1.0f / 32768.f) * 0.02f);
  }
}

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                          \
    }                                                                                   \
  } while (0)
}  // namespace

int main() {
  const int M = 3, K = 4096;
  const int tiles[] = {256, 384, 448, 512, 640, 768, 896, 960, 1024, 1152, 1280};
  uint16_t *x, *out;
  CK(hipMalloc(&x, (size_t)16 * 16384 * 2));
  CK(hipMalloc(&out, (size_t)16 * 32768 * 2));
  hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, x, (size_t)16 * 16384, 7);
  // rotate over enough weight copies (>= 1 GiB) that the 256 MB MALL cannot serve repeats
  const int copies = 6;
  std::vector<uint16_t*> w(copies);
  const size_t wmax = (size_t)1280 * 16 * 2 * K;   // swiglu: 2 rows per output column
  for (int c = 0; c < copies; ++c) {
    CK(hipMalloc(&w[c], wmax * 2));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, w[c], wmax, 11 + c);
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int kind = 0; kind < 2; ++kind) {   // 0 swiglu 4x2 (gate_up), 1 norm 4x2 plain store (qkv-like)
    for (int t : tiles) {
      const int N = t * 16;
      auto launch = [&](int i) {
        GemmArgs p{out, x, (const short8*)w[i % copies], nullptr, M, N, K, N, 1e-5f, {}, nullptr, nullptr};
        if (kind == 0)
          hipLaunchKernelGGL((plain_kernel<PRO_NORM, EPI_SWIGLU, 4, 2>), dim3(t), dim3(256), 0, s, p);
        else
          hipLaunchKernelGGL((plain_kernel<PRO_NORM, EPI_STORE, 4, 2>), dim3(t), dim3(256), 0, s, p);
      };
      hipGraph_t g;
      hipGraphExec_t ge;
      const int R = 24;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < R; ++i) launch(i);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      const double us = best * 1e3 / R;
      const double bytes = (double)N * K * 2 * (kind == 0 ? 2 : 1);
      printf("%-8s tiles=%5d (%.2f per CU)  %7.2f us  %5.2f TB/s  %6.3f us per tile-per-CU\n",
             kind == 0 ? "swiglu" : "norm", t, t / 256.0, us, bytes / us / 1e6, us / (t / 256.0));
      fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
