// Probe: what a short weight-streaming launch costs on MI355X as a function of workgroups, bytes
// per workgroup and bytes in flight per wave — the regime of tensor-parallel decode shards, where
// a GEMM streams only 4-30 MB and the launch is latency-bound rather than bandwidth-bound.
//
// Each workgroup streams its own contiguous chunk: NW waves, each lane one 16-B load per wave
// instruction (1 KiB per wave-load), U loads per wave in flight per stage, two stages (the same
// double-buffered pattern as csrc/skinny_core.h). The sum is reduced through LDS and one float
// per workgroup is written (keeps the loads live). 20 launches are captured in a hipGraph over
// buffers rotating through >= 1 GiB, so every launch reads cold weights; time per launch is the
// replay time / 20 (launch boundaries included, as in a decode step).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/probes/stream_probe tools/probes/stream_probe.hip
//   build/probes/stream_probe > stream_probe.csv
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef float float4_ __attribute__((ext_vector_type(4)));

template <int NW, int U>
__global__ void __launch_bounds__(NW * 64) stream_k(const float4_* __restrict__ w, long long per_wg_vec,
                                                     float* __restrict__ out) {
  __shared__ float red[NW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float4_* base = w + (long long)blockIdx.x * per_wg_vec;
  const int steps = (int)(per_wg_vec / 64);   // wave-loads of 1 KiB in this chunk
  float acc = 0.f;
  float4_ a[U], b[U];
  constexpr int SPAN = NW * U;
  int s = wid;
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(base + (long long)min(s + NW * u, steps - 1) * 64 + lane);
  for (; s < steps; s += 2 * SPAN) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      b[u] = __builtin_nontemporal_load(base + (long long)min(s + SPAN + NW * u, steps - 1) * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + NW * u < steps) acc += a[u][0] + a[u][1] + a[u][2] + a[u][3];
#pragma unroll
    for (int u = 0; u < U; ++u)
      a[u] = __builtin_nontemporal_load(base + (long long)min(s + 2 * SPAN + NW * u, steps - 1) * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + SPAN + NW * u < steps) acc += b[u][0] + b[u][1] + b[u][2] + b[u][3];
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) red[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < NW; ++i) t += red[i];
    out[blockIdx.x] = t;
  }
}

template <int NW, int U>
float run(const float4_* pool, long long pool_vec, int wgs, long long per_wg_bytes, float* out) {
  const long long per_wg_vec = per_wg_bytes / 16;
  const long long launch_vec = per_wg_vec * wgs;
  const int copies = (int)(pool_vec / launch_vec) < 20 ? (int)(pool_vec / launch_vec) : 20;
  if (copies < 2) return -1.f;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  constexpr int ITERS = 20;
  for (int i = 0; i < ITERS; ++i)
    hipLaunchKernelGGL((stream_k<NW, U>), dim3(wgs), dim3(NW * 64), 0, st, pool + (i % copies) * launch_vec,
                       per_wg_vec, out);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 6; ++r) {
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 0 && ms < best) best = ms;
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  CK(hipStreamDestroy(st));
  return best * 1000.f / ITERS;
}

int main() {
  const long long pool_bytes = 3LL << 30;
  float4_* pool;
  float* out;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMemset(pool, 0, pool_bytes));
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  const long long pool_vec = pool_bytes / 16;
  const int wgs_list[] = {48, 96, 112, 192, 224, 256, 384, 512, 768, 1024};
  const long long kb_list[] = {4, 8, 16, 32, 64, 128, 256};
  printf("nw,u,wgs,kb_per_wg,us,tbs\n");
  for (int wgs : wgs_list)
    for (long long kb : kb_list) {
      const long long bytes = kb * 1024;
      struct V {
        int nw, u;
        float us;
      } vs[] = {{4, 2, run<4, 2>(pool, pool_vec, wgs, bytes, out)},
                {4, 4, run<4, 4>(pool, pool_vec, wgs, bytes, out)},
                {8, 2, run<8, 2>(pool, pool_vec, wgs, bytes, out)},
                {8, 4, run<8, 4>(pool, pool_vec, wgs, bytes, out)},
                {16, 2, run<16, 2>(pool, pool_vec, wgs, bytes, out)},
                {16, 4, run<16, 4>(pool, pool_vec, wgs, bytes, out)}};
      for (auto& v : vs)
        printf("%d,%d,%d,%lld,%.2f,%.2f\n", v.nw, v.u, wgs, kb, v.us, v.us > 0 ? wgs * bytes / v.us / 1e6 : 0.0);
      fflush(stdout);
    }
  // the empty-ish floor: one trivial workgroup
  printf("# floor 1wg 1KB 4x2: %.2f us\n", run<4, 2>(pool, pool_vec, 1, 1024, out));
  CK(hipFree(pool));
  CK(hipFree(out));
  return 0;
}
