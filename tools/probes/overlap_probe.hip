// Probe: can the launch + weight ramp of a dependent decode kernel hide under its producer?
//
// 1. Do two independent kernels captured on forked streams run CONCURRENTLY when the hipGraph
//    replays (or does the graph serialize its branches)? Two 1-workgroup kernels that each spin
//    ~20 us: ~20 us per replay = concurrent, ~40 = serialized.
// 2. A producer P (a weight stream of `pkb` KB per workgroup over 256 workgroups, the shape of a
//    tensor-parallel shard GEMM) followed by a consumer C (the same stream shape):
//      serial : P -> C on one stream (the kernel boundary);
//      early  : C on a forked stream with NO graph edge from P: every C workgroup first issues its
//               own weight loads, then waits (bounded poll, one lane, s_sleep) until P's last
//               workgroup has published its completion epoch (release fence + flag), then acquires
//               and consumes. The next replay's P waits the same way on C (a ring of two).
//    A time limit on every poll: on expiry the kernel records an error and proceeds (never a hang).
// Prints us per replay for each form; tools/probes/README notes what was concluded.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/probes/overlap_probe tools/probes/overlap_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef float float4_ __attribute__((ext_vector_type(4)));
constexpr long long POLL_LIMIT = 1 << 18;

__global__ void spin_k(long long ticks, unsigned* sink) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) sink[blockIdx.x] = 1u;
}

// one workgroup streams `vec` float4 of its chunk (4 waves x U=4 in flight, like the shard GEMMs)
__device__ float stream_chunk(const float4_* __restrict__ base, long long vec) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int steps = (int)(vec / 64);
  float acc = 0.f;
  for (int s = wid; s < steps; s += 4 * 4) {
    float4_ a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = __builtin_nontemporal_load(base + (long long)min(s + 4 * u, steps - 1) * 64 + lane);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (s + 4 * u < steps) acc += a[u][0] + a[u][1] + a[u][2] + a[u][3];
  }
  return acc;
}

// wait until *flag >= want (one lane, bounded), then acquire for the whole workgroup
__device__ void wait_flag(const unsigned* flag, unsigned want, int* err) {
  if (threadIdx.x == 0) {
    long long it = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > POLL_LIMIT) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
}

// the last workgroup out publishes `epoch` (release: every workgroup's stores written back first)
__device__ void signal_done(unsigned* done_ctr, unsigned* flag, unsigned epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1u) {
      __hip_atomic_store(done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct Sync {
  unsigned* ctr;      // [1] done counter of P, [2] done counter of C
  unsigned* flag;     // [0] P's published pair index + 1, [1] C's
  int* err;
};

__global__ void reset_k(Sync s) {
  if (threadIdx.x < 4) {
    s.ctr[threadIdx.x] = 0u;
    s.flag[threadIdx.x] = 0u;
  }
}

// mode 0: plain stream kernel (serial graph). mode 1: P of the early pair i, mode 2: C of pair i.
// P_i publishes i + 1 into flag[0]; C_i waits for flag[0] >= i + 1 (after issuing its own weight
// loads) and publishes i + 1 into flag[1]; P_i (i > 0) waits for flag[1] >= i (C_{i-1} read what
// P_i overwrites). Graph edges only within each stream (P_{i-1} -> P_i, C_{i-1} -> C_i).
__global__ void __launch_bounds__(256) stream_k(const float4_* __restrict__ w, long long per_wg_vec, float* out,
                                                int mode, int pair, Sync s) {
  const float4_* base = w + (long long)blockIdx.x * per_wg_vec;
  float acc = 0.f;
  if (mode == 2) {
    acc = stream_chunk(base, per_wg_vec);         // weights first: they do not depend on P
    wait_flag(s.flag + 0, (unsigned)pair + 1u, s.err);
    acc += out[(blockIdx.x * 7) % gridDim.x];     // the "activation" P wrote
  } else {
    if (mode == 1 && pair > 0) wait_flag(s.flag + 1, (unsigned)pair, s.err);
    acc = stream_chunk(base, per_wg_vec);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[(mode == 1 ? 0 : gridDim.x) + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  if (mode == 1) signal_done(s.ctr + 1, s.flag + 0, (unsigned)pair + 1u);
  if (mode == 2) signal_done(s.ctr + 2, s.flag + 1, (unsigned)pair + 1u);
}

float time_graph(hipGraphExec_t ge, hipStream_t st, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 0 && ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return best * 1000.f / iters;
}

int main() {
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  unsigned* sink;
  CK(hipMalloc(&sink, 4096));
  int clk = 0;
  CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, 0));   // kHz of wall_clock64()
  const long long cyc20 = (long long)clk * 20 / 1000;                     // ~20 us

  // ---- 1: branch concurrency ----
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    constexpr int IT = 10;
    for (int i = 0; i < IT; ++i) {
      CK(hipEventRecord(fork, s1));
      CK(hipStreamWaitEvent(s2, fork, 0));
      hipLaunchKernelGGL(spin_k, dim3(1), dim3(64), 0, s1, cyc20, sink);
      hipLaunchKernelGGL(spin_k, dim3(1), dim3(64), 0, s2, cyc20, sink + 64);
      CK(hipEventRecord(join, s2));
      CK(hipStreamWaitEvent(s1, join, 0));
    }
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const float tb = time_graph(ge, s1, IT);
    printf("branch concurrency: two ~20 us kernels per fork/join: %.2f us per pair (20 = concurrent, 40 = serial)\n",
           tb);
    fflush(stdout);
    if (tb > 30.f) {
      printf("graph branches serialize: the early-launch form would deadlock on its flags; skipped\n");
      return 0;
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }

  // ---- 2: serial vs early-launched consumer ----
  const long long pool_bytes = 2LL << 30;
  float4_* pool;
  float* out;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMemset(pool, 0, pool_bytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(out, 0, 1 << 20));
  Sync sy;
  CK(hipMalloc(&sy.ctr, 64));
  CK(hipMalloc(&sy.flag, 64));
  CK(hipMalloc(&sy.err, 64));
  CK(hipMemset(sy.err, 0, 64));
  const int wgs = 256;
  const long long kbs[] = {16, 64, 128};
  constexpr int IT = 10;   // P / C pairs per graph
  for (long long kb : kbs) {
    const long long per_wg_vec = kb * 1024 / 16;
    const long long launch_vec = per_wg_vec * wgs;
    const long long copies = (pool_bytes / 16) / launch_vec;
    auto buf = [&](int k) { return pool + (k % copies) * launch_vec; };
    float t_serial, t_early;
    {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
      for (int i = 0; i < IT; ++i) {
        hipLaunchKernelGGL(stream_k, dim3(wgs), dim3(256), 0, s1, buf(2 * i), per_wg_vec, out, 0, i, sy);
        hipLaunchKernelGGL(stream_k, dim3(wgs), dim3(256), 0, s1, buf(2 * i + 1), per_wg_vec, out, 0, i, sy);
      }
      CK(hipStreamEndCapture(s1, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      t_serial = time_graph(ge, s1, IT);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
    {
      hipGraph_t g;
      hipGraphExec_t ge;
      hipEvent_t fork, join;
      CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
      CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
      hipLaunchKernelGGL(reset_k, dim3(1), dim3(64), 0, s1, sy);
      CK(hipEventRecord(fork, s1));
      CK(hipStreamWaitEvent(s2, fork, 0));
      for (int i = 0; i < IT; ++i) {
        hipLaunchKernelGGL(stream_k, dim3(wgs), dim3(256), 0, s1, buf(2 * i), per_wg_vec, out, 1, i, sy);
        hipLaunchKernelGGL(stream_k, dim3(wgs), dim3(256), 0, s2, buf(2 * i + 1), per_wg_vec, out, 2, i, sy);
      }
      CK(hipEventRecord(join, s2));
      CK(hipStreamWaitEvent(s1, join, 0));
      CK(hipStreamEndCapture(s1, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      t_early = time_graph(ge, s1, IT);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      CK(hipEventDestroy(fork));
      CK(hipEventDestroy(join));
    }
    int err = 0;
    CK(hipMemcpy(&err, sy.err, sizeof(int), hipMemcpyDeviceToHost));
    printf("pair of 256 x %lld KB streams: serial %.2f us, early-launched consumer %.2f us per pair (poll expiry %d)\n",
           kb, t_serial, t_early, err);
    fflush(stdout);
  }
  CK(hipFree(pool));
  CK(hipFree(out));
  return 0;
}
