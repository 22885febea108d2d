// Experiment: is a decode GEMM's time set by its bytes or by the busiest CU's tile count?
// gate_up has 896 16-column tiles on 256 CUs (3.5 per CU), qkv 384 (1.5 per CU). Time the
// production skinny kernel (skinny_core.h, M = 3) over tile counts around those: if 1024 tiles
// cost about what 896 cost, the last half-wave of tiles is what the GEMM waits for.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/exp_balance.hip -o build/exp_balance
#include "skinny_core.h"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
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

int main(int argc, char** argv) {
  const int M = 3;
  uint16_t *x, *out, *res;
  CK(hipMalloc(&x, (size_t)16 * 16384 * 2));
  CK(hipMalloc(&out, (size_t)16 * 131072 * 2));
  CK(hipMalloc(&res, (size_t)16 * 131072 * 2));
  hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, x, (size_t)16 * 16384, 7);
  hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, res, (size_t)16 * 131072, 9);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const bool layouts = argc > 1 && argv[1][0] == 'l';
  struct Shape { const char* name; int kind; int tiles; int K; };
  // kind 0 swiglu (norm, 4x2), 1 norm store (4x2), 2 plain resid (4x4)
  std::vector<Shape> shapes;
  if (layouts) {
    shapes = {{"o", 2, 256, 4096}, {"down", 2, 256, 14336}, {"qkv-like", 1, 384, 4096},
              {"gate_up", 0, 896, 4096}, {"lm_head", 1, 8016, 4096}};
  } else {
    for (int t : {256, 384, 448, 512, 640, 768, 896, 960, 1024, 1152, 1280}) shapes.push_back({"swiglu", 0, t, 4096});
    for (int t : {256, 384, 448, 512, 640, 768, 896, 960, 1024, 1152, 1280}) shapes.push_back({"norm", 1, t, 4096});
  }
  for (const Shape& sh : shapes) {
    const int t = sh.tiles, K = sh.K, N = t * 16;
    const size_t welems = (size_t)N * K * (sh.kind == 0 ? 2 : 1);
    const int copies = (int)std::max<size_t>(2, (size_t)(1.5e9 / (welems * 2.0)) + 1);
    std::vector<uint16_t*> w(copies);
    for (int c = 0; c < copies; ++c) {
      CK(hipMalloc(&w[c], welems * 2));
      hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, w[c], welems, 11 + c);
    }
    const int kms[] = {0, 1, 2, 3, 4, 5, 6, 7};   // tile-major, k-major, k-chunks of 2 .. 64 steps
    for (int kmi = 0; kmi < (layouts ? 8 : 1); ++kmi) {
      const int km = kms[kmi];
      auto launch = [&](int i) {
        GemmArgs p{sh.kind == 0 ? out : (sh.kind == 1 ? out : nullptr), x, (const short8*)w[i % copies],
                   sh.kind == 2 ? res : nullptr, M, N, K, N, 1e-5f, {}, nullptr, nullptr};
        p.kmajor = km;
        if (sh.kind == 0)
          hipLaunchKernelGGL((plain_kernel<PRO_NORM, EPI_SWIGLU, 4, 2>), dim3(t), dim3(256), 0, s, p);
        else if (sh.kind == 1)
          hipLaunchKernelGGL((plain_kernel<PRO_NORM, EPI_STORE, 4, 2>), dim3(t), dim3(256), 0, s, p);
        else
          hipLaunchKernelGGL((plain_kernel<PRO_PLAIN, EPI_RESID, 4, 4>), dim3(t), dim3(256), 0, s, p);
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
      char lay[32];
      snprintf(lay, sizeof lay, km == 0 ? "tile-major" : (km == 1 ? "k-major" : "k-chunk %d"), 1 << (km - 1));
      printf("%-9s %-11s tiles=%5d (%.2f per CU) K=%5d  %8.2f us  %5.2f TB/s\n", sh.name, layouts ? lay : "", t,
             t / 256.0, K, us, welems * 2.0 / us / 1e6);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
    for (auto p : w) CK(hipFree(p));
  }
  return 0;
}
