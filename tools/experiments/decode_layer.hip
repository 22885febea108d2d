// Persistent decode layer: one launch runs a whole transformer layer of the decode step —
//   P1 qkv (+RMSNorm, +RoPE, +paged K/V write)  -> P2 paged attention (split-KV + combine)
//   -> P3 o-proj (+residual) -> P4 gate_up (+RMSNorm, SwiGLU) -> P5 down (+residual)
// instead of five dependent launches.
//
// Why: at M <= 16 every phase is a short weight stream (5-40 µs) and each kernel boundary
// costs a launch gap plus a ramp to full bandwidth. Here the grid is one 8-wave workgroup
// per CU for the whole layer; phases hand off through device-scope arrival counters, and
// before waiting for a phase's inputs each workgroup already has the first weight records
// of its next tile in flight (weights never depend on activations), so HBM keeps streaming
// across the dependency.
//
// Hand-off protocol (MI355X_MICROARCH "Valid forms", row 1): every byte a later phase
// reads is stored sc1 (write-through) by its producer (skinny_core.h / attn_core.h SC1=true),
// every storing wave drains (vmcnt(0)) before a workgroup barrier, then ONE lane adds to the
// phase counter; a consumer's lane 0 polls the counter with sc1 loads (s_sleep between polls),
// the workgroup joins a barrier, and every load of handed-off bytes is an sc1 load.
// The workgroup whose final arrival completes the layer re-arms all counters to 0.
//
// Safety: the grid never exceeds the CU count and each workgroup needs a whole CU's worth
// of 8 waves x ~200 VGPRs, so every workgroup is resident at once (no waiting on an
// unscheduled producer). Every poll is bounded; on expiry the kernel sets *err and proceeds
// (wrong numbers, never a hang); the host checks the flag.
#include "attn_core.h"
#include "skinny_core.h"

namespace {
using rt::short8;
using namespace skinny;

constexpr int NWL = 8;        // waves per workgroup in every phase
constexpr int UL = 4;         // k-steps per wave per pipeline stage
constexpr int D = 128;        // head dim (Llama-3 / Mistral)
constexpr long long POLL_LIMIT = 1ll << 25;

enum : int { C_QKV = 0, C_ATT = 1, C_O = 2, C_GU = 3, C_END = 4, C_NUM = 5 };

struct LayerArgs {
  GemmArgs qkv, o, gu, dn;   // per-phase GEMM descriptors (SC1 variants)
  attn::AttnArgs at;
  int n_qkv, n_o, n_gu, n_dn;   // tiles per GEMM phase
  int n_items;                  // attention items = B * Hkv * splits
  int n_combine;                // attention outputs = B * Hkv
  int* sync;                    // [C_NUM] counters, zero at launch
  int* err;                     // set to 1 if a poll expired
  long long* stamps;            // optional [grid][NSTAMP] s_memrealtime per phase boundary (profiling)
};
constexpr int NSTAMP = 10;

RT_DEVICE void stamp(long long* stamps, int i) {
  if (stamps != nullptr && threadIdx.x == 0) {
    const long long t = (long long)__builtin_amdgcn_s_memrealtime();
    stamps[(size_t)blockIdx.x * NSTAMP + i] = t;
  }
}

union LayerSmem {
  GemmSmem<2, NWL> g2;
  GemmSmem<1, NWL> g1;
  attn::AttnSmem<D> at;
};

RT_DEVICE void arrive(int* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

RT_DEVICE void wait_for(const int* cnt, int target, int* err) {
  if (threadIdx.x == 0) {
    long long it = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > POLL_LIMIT) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(NWL * 64) decode_layer_kernel(LayerArgs P) {
  __shared__ LayerSmem sm;
  __shared__ int s_last;
  const int G = gridDim.x, w = blockIdx.x;
  int* sync = P.sync;
  stamp(P.stamps, 0);

  // ---- P1: qkv + RMSNorm + RoPE + K/V cache write (inputs from the previous launch) ----
  for (int t = w; t < P.n_qkv; t += G) {
    Stage<PRO_NORM, EPI_ROPE, UL> st;
    gemm_tile<PRO_NORM, EPI_ROPE, NWL, UL, true>(P.qkv, t, sm.g1, st, false, false);
    arrive(sync + C_QKV);
  }
  // ---- P2: attention (all q/k/v of the step must be in place) ----
  stamp(P.stamps, 1);
  wait_for(sync + C_QKV, P.n_qkv, P.err);
  stamp(P.stamps, 2);
  const int nbh = P.n_combine;
  for (int i = w; i < P.n_items; i += G) {
    const int bh = i % nbh, split = i / nbh;   // consecutive workgroups take different (seq, head)
    if (attn::attn_item<D, true>(P.at, bh, split, sm.at)) arrive(sync + C_ATT);
  }
  // ---- P3: o-proj + residual. Stage-0 weights go out before the wait. ----
  {
    Stage<PRO_PLAIN, EPI_RESID, UL> st;
    const bool has = w < P.n_o;
    if (has) gemm_prefetch<PRO_PLAIN, EPI_RESID, NWL, UL>(P.o, w, st);
    stamp(P.stamps, 3);
    wait_for(sync + C_ATT, P.n_combine, P.err);
    stamp(P.stamps, 4);
    for (int t = w; t < P.n_o; t += G) {
      gemm_tile<PRO_PLAIN, EPI_RESID, NWL, UL, true>(P.o, t, sm.g1, st, t == w, false);
      arrive(sync + C_O);
    }
  }
  // ---- P4: gate_up + RMSNorm + SwiGLU (needs the whole residual row) ----
  {
    Stage<PRO_NORM, EPI_SWIGLU, UL> st;
    if (w < P.n_gu) gemm_prefetch<PRO_NORM, EPI_SWIGLU, NWL, UL>(P.gu, w, st);
    stamp(P.stamps, 5);
    wait_for(sync + C_O, P.n_o, P.err);
    stamp(P.stamps, 6);
    for (int t = w; t < P.n_gu; t += G) {
      gemm_tile<PRO_NORM, EPI_SWIGLU, NWL, UL, true>(P.gu, t, sm.g2, st, t == w, false);
      arrive(sync + C_GU);
    }
  }
  // ---- P5: down + residual ----
  {
    Stage<PRO_PLAIN, EPI_RESID, UL> st;
    if (w < P.n_dn) gemm_prefetch<PRO_PLAIN, EPI_RESID, NWL, UL>(P.dn, w, st);
    stamp(P.stamps, 7);
    wait_for(sync + C_GU, P.n_gu, P.err);
    stamp(P.stamps, 8);
    for (int t = w; t < P.n_dn; t += G) gemm_tile<PRO_PLAIN, EPI_RESID, NWL, UL, true>(P.dn, t, sm.g1, st, t == w, false);
  }
  stamp(P.stamps, 9);
  // ---- the last workgroup out re-arms the counters (every workgroup is past all its waits) ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(sync + C_END, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == G - 1;
    if (s_last)
      for (int c = 0; c < C_NUM; ++c) __hip_atomic_store(sync + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
}  // namespace

int decode_layer_grid() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return cus;
}

// All pointers are device pointers; shapes: x/res [M, H], q [M, Hq, D], a [M, Hq*D], g [M, I].
int launch_decode_layer(void* res, void* q, void* a, void* g, const void* wqkv, const void* wo, const void* wgu,
                        const void* wd, const int64_t* positions, const float* cos_sin, void* k_cache, void* v_cache,
                        const int64_t* slots, const int* block_tables, const int* ctx_lens, float* part_o,
                        float* part_ml, int* split_counters, int* sync, int* err, long long* stamps, int M, int H,
                        int I, int Hq, int Hkv, int head_dim, int BS, int max_blocks, int num_splits, float eps,
                        float scale, hipStream_t stream) {
  if (head_dim != D || M < 1 || M > 16 || H % 32 || I % 32 || Hq % Hkv || Hq / Hkv > 16 || BS != 32) return -1;
  if (num_splits < 1 || num_splits > attn::MAXS) return -2;
  const int grid = decode_layer_grid();
  if (grid <= 0) return -3;
  const RopeEpi none{};
  const RopeEpi re{positions, cos_sin, (uint16_t*)k_cache, (uint16_t*)v_cache, slots, Hq, Hkv, D, BS};
  const int Nqkv = (Hq + 2 * Hkv) * D;
  LayerArgs P;
  P.qkv = GemmArgs{(uint16_t*)q, (const uint16_t*)res, (const short8*)wqkv, nullptr, M, Nqkv, H, 0, eps, re,
                   nullptr, nullptr};
  P.o = GemmArgs{nullptr, (const uint16_t*)a, (const short8*)wo, (uint16_t*)res, M, H, Hq * D, 0, eps, none,
                 nullptr, nullptr};
  P.gu = GemmArgs{(uint16_t*)g, (const uint16_t*)res, (const short8*)wgu, nullptr, M, I, H, I, eps, none, nullptr,
                  nullptr};
  P.dn = GemmArgs{nullptr, (const uint16_t*)g, (const short8*)wd, (uint16_t*)res, M, H, I, 0, eps, none, nullptr,
                  nullptr};
  P.at = attn::AttnArgs{(uint16_t*)a, (const uint16_t*)q, (const uint16_t*)k_cache, (const uint16_t*)v_cache,
                        block_tables, ctx_lens, part_o, part_ml, split_counters, Hq, Hkv, max_blocks,
                        scale * 1.4426950408889634f, num_splits};
  P.n_qkv = Nqkv / 16;
  P.n_o = H / 16;
  P.n_gu = I / 16;
  P.n_dn = H / 16;
  P.n_combine = M * Hkv;
  P.n_items = M * Hkv * num_splits;
  P.sync = sync;
  P.err = err;
  P.stamps = stamps;
  hipLaunchKernelGGL(decode_layer_kernel, dim3(grid), dim3(NWL * 64), 0, stream, P);
  return 0;
}
