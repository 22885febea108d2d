// Experiment: overlap dependent decode GEMM launches across a kernel boundary.
//
// A decode layer's GEMMs are a strict chain (o -> gate_up -> down -> o ...), each a 8-40 µs
// weight stream whose first ~2-3 µs are a ramp (launch gap + first-load latency). Weights
// never depend on the previous kernel, so a consumer launched EARLY (on a second stream, no
// stream dependency on its producer) can put its first weight stage in flight, then wait on
// the producer's arrival counters (sharded by blockIdx % 8), and read the activations with sc1
// loads (the producer stores them sc1: MI355X_MICROARCH "Valid forms" row 1).
// Kernels alternate between two streams, so kernel i+1 may run beside kernel i but never
// beside kernel i-1 (same-stream order). Every poll is bounded (err word, never a hang).
//
// Modes: 0 plain launches one stream (the engine today), 1 chained kernels one stream
// (protocol cost without overlap), 2 chained kernels on two alternating streams; each eager
// and hipGraph-captured.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/exp_chain.hip -o build/exp_chain
#include "skinny_core.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace skinny;
using rt::short8;

namespace {
constexpr int SH = 8;                       // counter shards (blockIdx % 8 ~ XCD)
constexpr long long POLL_LIMIT = 1ll << 22; // x s_sleep(1): ~0.1-0.3 s, then give up

struct Chain {
  int* sig;        // [SH] this kernel's arrival counters (nullptr: last kernel)
  const int* wait; // [SH] producer's counters (nullptr: first kernel)
  int* wait_rw;    // same as wait, writable: reset by the last consumer to pass
  int wait_grid;   // producer grid size
  int* pass;       // consumer pass counter (1 word)
  int* err;
};

RT_DEVICE void chain_wait(const Chain& c) {
  if (threadIdx.x == 0) {   // one lane polls every shard (MI355X_MICROARCH polling-cost)
    long long it = 0;
    for (int s = 0; s < SH; ++s) {
      const int target = c.wait_grid / SH + (s < c.wait_grid % SH ? 1 : 0);
      while (__hip_atomic_load(c.wait + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(4);
        if (++it > POLL_LIMIT) {
          __hip_atomic_store(c.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s = SH;
          break;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // the last workgroup past the wait re-arms the producer's counters
    const int prev = __hip_atomic_fetch_add(c.pass, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (int)gridDim.x - 1) {
      for (int s = 0; s < SH; ++s) __hip_atomic_store(c.wait_rw + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c.pass, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

RT_DEVICE void chain_arrive(const Chain& c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && c.sig != nullptr)
    __hip_atomic_fetch_add(c.sig + (blockIdx.x % SH), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int PRO, int EPI, int NW, int U>
__global__ void __launch_bounds__(NW * 64) plain_kernel(GemmArgs p) {
  __shared__ GemmSmem<nacc<EPI>(), NW> sm;
  Stage<PRO, EPI, U> st0;
  gemm_tile<PRO, EPI, NW, U, false>(p, blockIdx.x, sm, st0, false, false);
}

template <int PRO, int EPI, int NW, int U, bool SC1>
__global__ void __launch_bounds__(NW * 64) chained_kernel(GemmArgs p, Chain c) {
  __shared__ GemmSmem<nacc<EPI>(), NW> sm;
  Stage<PRO, EPI, U> st0;
  const bool pre = c.wait != nullptr;
  if (pre) {
    gemm_prefetch<PRO, EPI, NW, U>(p, blockIdx.x, st0);
    chain_wait(c);
  }
  gemm_tile<PRO, EPI, NW, U, SC1>(p, blockIdx.x, sm, st0, pre, false);
  chain_arrive(c);
}

__global__ void fill_kernel(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const float f = ((int)(h & 0xffff) - 32768) * (1.0f / 32768.f) * 0.02f;
    p[i] = rt::f2bf(f);
  }
}

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);  \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

struct Op {
  int kind;  // 0 o (plain+resid), 1 gate_up (norm+swiglu), 2 down (plain+resid)
  GemmArgs a;
  int grid;
};

uint16_t* alloc_fill(size_t n, uint32_t seed) {
  uint16_t* p;
  CK(hipMalloc(&p, n * 2));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, p, n, seed);
  return p;
}
}  // namespace

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 8;   // layers
  const int M = argc > 2 ? atoi(argv[2]) : 3;
  const int H = 4096, I = 14336;
  std::vector<Op> ops;
  uint16_t* attn = alloc_fill((size_t)M * H, 1);
  uint16_t* res = alloc_fill((size_t)M * H, 2);
  uint16_t* hbuf = alloc_fill((size_t)M * I, 3);
  for (int l = 0; l < L; ++l) {
    uint16_t* wo = alloc_fill((size_t)H * H, 10 + l);
    uint16_t* wgu = alloc_fill((size_t)2 * I * H, 100 + l);
    uint16_t* wd = alloc_fill((size_t)H * I, 1000 + l);
    Op o{0, GemmArgs{res, attn, (const short8*)wo, res, M, H, H, H, 1e-5f, {}, nullptr, nullptr}, H / 16};
    Op gu{1, GemmArgs{hbuf, res, (const short8*)wgu, nullptr, M, I, H, I, 1e-5f, {}, nullptr, nullptr}, I / 16};
    Op dn{2, GemmArgs{res, hbuf, (const short8*)wd, res, M, H, I, H, 1e-5f, {}, nullptr, nullptr}, H / 16};
    ops.push_back(o);
    ops.push_back(gu);
    ops.push_back(dn);
  }
  const int n = (int)ops.size();
  int* ctr;   // per kernel: SH arrival shards + 1 pass word
  CK(hipMalloc(&ctr, (size_t)n * (SH + 1) * sizeof(int)));
  CK(hipMemset(ctr, 0, (size_t)n * (SH + 1) * sizeof(int)));
  int* err;
  CK(hipMalloc(&err, sizeof(int)));
  CK(hipMemset(err, 0, sizeof(int)));
  CK(hipDeviceSynchronize());

  hipStream_t sA, sB;
  CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
  hipEvent_t fork, join, t0, t1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));

  auto launch = [&](int mode) {
    const bool two = mode == 2 || mode == 4, sc1 = mode <= 2;
    if (two) {
      CK(hipEventRecord(fork, sA));
      CK(hipStreamWaitEvent(sB, fork, 0));
    }
    for (int i = 0; i < n; ++i) {
      const Op& op = ops[i];
      hipStream_t s = (two && (i & 1)) ? sB : sA;
      if (mode == 0) {
        if (op.kind == 0 || op.kind == 2)
          hipLaunchKernelGGL((plain_kernel<PRO_PLAIN, EPI_RESID, 4, 4>), dim3(op.grid), dim3(256), 0, s, op.a);
        else
          hipLaunchKernelGGL((plain_kernel<PRO_NORM, EPI_SWIGLU, 4, 2>), dim3(op.grid), dim3(256), 0, s, op.a);
      } else {
        Chain c{};
        c.sig = i + 1 < n ? ctr + (size_t)i * (SH + 1) : nullptr;
        c.wait = i > 0 ? ctr + (size_t)(i - 1) * (SH + 1) : nullptr;
        c.wait_rw = i > 0 ? ctr + (size_t)(i - 1) * (SH + 1) : nullptr;
        c.wait_grid = i > 0 ? ops[i - 1].grid : 0;
        c.pass = ctr + (size_t)i * (SH + 1) + SH;
        c.err = err;
        if (sc1) {
          if (op.kind == 0 || op.kind == 2)
            hipLaunchKernelGGL((chained_kernel<PRO_PLAIN, EPI_RESID, 4, 4, true>), dim3(op.grid), dim3(256), 0, s, op.a, c);
          else
            hipLaunchKernelGGL((chained_kernel<PRO_NORM, EPI_SWIGLU, 4, 2, true>), dim3(op.grid), dim3(256), 0, s, op.a, c);
        } else {
          if (op.kind == 0 || op.kind == 2)
            hipLaunchKernelGGL((chained_kernel<PRO_PLAIN, EPI_RESID, 4, 4, false>), dim3(op.grid), dim3(256), 0, s, op.a, c);
          else
            hipLaunchKernelGGL((chained_kernel<PRO_NORM, EPI_SWIGLU, 4, 2, false>), dim3(op.grid), dim3(256), 0, s, op.a, c);
        }
      }
    }
    if (two) {
      CK(hipEventRecord(join, sB));
      CK(hipStreamWaitEvent(sA, join, 0));
    }
  };

  double bytes = 0;
  for (auto& op : ops) bytes += (double)op.a.N * op.a.K * 2 * (op.kind == 1 ? 2 : 1);
  const char* names[5] = {"plain, one stream", "chained sc1, one stream", "chained sc1, two streams",
                          "chained nosc1, one (timing)", "chained nosc1, two (timing)"};
  for (int graph = 0; graph < 2; ++graph) {
    for (int mode = 0; mode < 5; ++mode) {
      hipGraphExec_t ge = nullptr;
      if (graph) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(sA, hipStreamCaptureModeGlobal));
        launch(mode);
        CK(hipStreamEndCapture(sA, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
      auto run = [&]() {
        if (graph) CK(hipGraphLaunch(ge, sA));
        else launch(mode);
      };
      for (int w = 0; w < 3; ++w) run();
      CK(hipStreamSynchronize(sA));
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        const int R = 10;
        CK(hipEventRecord(t0, sA));
        for (int r = 0; r < R; ++r) run();
        CK(hipEventRecord(t1, sA));
        CK(hipEventSynchronize(t1));
        float ms;
        CK(hipEventElapsedTime(&ms, t0, t1));
        best = ms / R < best ? ms / R : best;
      }
      int herr = 0;
      CK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
      printf("%-6s %-28s L=%d M=%d: %8.1f us per chain = %6.2f us per layer (%.2f TB/s) err=%d\n",
             graph ? "graph" : "eager", names[mode], L, M, best * 1e3, best * 1e3 / L, bytes / (best * 1e-3) / 1e12,
             herr);
      fflush(stdout);
      if (herr) {
        CK(hipMemset(err, 0, sizeof(int)));
        CK(hipMemset(ctr, 0, (size_t)n * (SH + 1) * sizeof(int)));
      }
      if (ge) CK(hipGraphExecDestroy(ge));
    }
  }
  return 0;
}
