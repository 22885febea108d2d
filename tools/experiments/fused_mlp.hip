// EXPERIMENT (launch folding redone fairly at shard shapes): the decode MLP
// of a tensor-parallel shard — gate_up (+RMSNorm, SwiGLU) then down (+residual) — as ONE
// persistent launch over ALL CUs, each phase laid out exactly as the product's separate launch:
//   phase 1: gate_up split-K (the product's tile/part mapping, S from splitk_parts: Llama-3-8B tp 8
//            = 112 tiles x 2 parts on 224 CUs; tp 4 = 224 whole tiles), the last arriver of a
//            tile combines its parts in index order and writes g write-through (sc1);
//   phase 2: down + residual, one 16-column tile per workgroup (256 tiles), its first weight
//            stage issued BEFORE the wait on phase 1 (weights never depend on activations).
// The phase hand-off is the persistent-kernel protocol of decode_layer.hip (drain + one arrival
// atomic per work item, a bounded sc1 poll, a workgroup barrier). Round 4's persistent LAYER
// ran gate_up on 112 CUs without split-K; this one gives both phases the whole chip, so the A/B
// against the two product launches isolates the kernel-boundary vs in-launch hand-off cost.
#include "skinny_core.h"

namespace {
using rt::short8;
using namespace skinny;

constexpr int NWM = 8;        // waves per workgroup (the product's split-K gate_up config)
constexpr int UM = 2;         // k-steps per wave per pipeline stage
constexpr int SPLIT_CTRS = 256;
constexpr long long POLL_LIMIT = 1ll << 25;

struct MlpArgs {
  GemmArgs gu, dn;
  int* ws;            // split workspace (product layout: SPLIT_CTRS counters, then part buffers)
  int S;              // gate_up parts per tile (1 = whole tiles)
  int n_gu, n_dn;     // tiles per phase
  int* sync;          // [2] counters, zero at launch (re-armed by the last workgroup out)
  int* err;
  int phases;         // diagnosis: 3 = both (the experiment), 1 = gate_up only, 2 = down only; +4 plain phase-1 stores;
                      // +8 no in-launch synchronisation at all (timing only: phase 2 may read stale g);
                      // +16 the hand-off and the exit re-arm on 8 sharded counters (round 6, below)
};

// Round 6: the 2.3x phase-1 anomaly. Phase 1 "alone" still ran the whole
// single-counter protocol: one arrival per item on ONE device-scope word (224 at tp 8), a poll by
// every workgroup on that word, and one exit arrival per workgroup on a second single word. The
// MI355X price list puts a 255 -> 1 fan-in on one counter at 3.6-4.5 us under streaming and a
// single-counter grid barrier at 7.4 us (MI355X_MICROARCH "fanin", "barrier-counter"). The sharded
// form below spreads arrivals over 8 words on separate 128-B lines, labelled by blockIdx % 8 (a
// label, not a placement assumption: the waiter sums all eight), so no word takes more than
// ceil(G / 8) arrivals; the exit re-arm is two-level (last of a shard -> top word).
constexpr int SH_STRIDE = 32;       // ints between shard words (128 B)
RT_DEVICE int* sh_arr(int* sync, int s) { return sync + SH_STRIDE * (1 + s); }
RT_DEVICE int* sh_exit(int* sync, int s) { return sync + SH_STRIDE * (9 + s); }
RT_DEVICE int* sh_top(int* sync) { return sync + SH_STRIDE * 17; }

RT_DEVICE void wait_sharded(int* sync, int target, int* err) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    long long it = 0;
    while (true) {
      int v = lane < 8 ? __hip_atomic_load(sh_arr(sync, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) v += __shfl_xor(v, o, 64);
      v = __shfl(v, 0, 64);              // every lane takes lane 0's total (a uniform exit)
      if (v >= target) break;
      __builtin_amdgcn_s_sleep(1);
      if (++it > POLL_LIMIT) {
        if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

union MlpSmem {
  GemmSmem<2, NWM> g2;
  GemmSmem<1, NWM> g1;
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
      __builtin_amdgcn_s_sleep(1);
      if (++it > POLL_LIMIT) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// ST1: phase-1 stores write-through (needed: phase 2 reads g from every XCD); false = diagnosis only
template <bool ST1>
__global__ void __launch_bounds__(NWM * 64) fused_mlp_kernel(MlpArgs P) {
  __shared__ MlpSmem sm;
  extern __shared__ float alds_dyn[];          // phase 2: [16] row sums, then the staged g rows
  const ALds al{reinterpret_cast<uint16_t*>(alds_dyn + 16), alds_dyn, P.dn.K + 8};
  const int G = gridDim.x, w = blockIdx.x;
  const int T = P.n_gu, S = P.S, items = (P.phases & 1) ? T * S : 0;
  for (int b = w; b < items; b += G) {
    if (S > 1) {
      int tile, part;
      if ((T & 7) == 0) {   // the product's placement: a tile's parts on one XCD
        const int j = b >> 3;
        tile = (j / S) * 8 + (b & 7);
        part = j % S;
      } else {
        tile = b / S;
        part = b % S;
      }
      const SplitX sx{reinterpret_cast<float*>(P.ws + SPLIT_CTRS) + (size_t)tile * S * SPLIT_STRIDE, P.ws + tile, part,
                      S};
      Stage<PRO_NORM, EPI_SWIGLU, UM> st;   // res came from an earlier launch: plain A loads
      gemm_tile<PRO_NORM, EPI_SWIGLU, NWM, UM, ST1, false, 0>(P.gu, tile, sm.g2, st, false, false, &sx);
    } else {
      Stage<PRO_NORM, EPI_SWIGLU, UM> st;
      gemm_tile<PRO_NORM, EPI_SWIGLU, NWM, UM, ST1, false, 0>(P.gu, b, sm.g2, st, false, false);
    }
    if (P.phases & 16) arrive(sh_arr(P.sync, w & 7));
    else if (!(P.phases & 8)) arrive(P.sync);
  }
  {
    Stage<PRO_PLAIN, EPI_RESID, UM> st;
    const int ndn = (P.phases & 2) ? P.n_dn : 0;
    if (w < ndn) gemm_prefetch<PRO_PLAIN, EPI_RESID, NWM, UM>(P.dn, w, st);
    if (P.phases & 16) wait_sharded(P.sync, items, P.err);
    else if (!(P.phases & 8)) wait_for(P.sync, items, P.err);
    // g was written in this launch: staged ONCE per tile into LDS with sc1 loads (ALDS), not an
    // sc1 load per k-step (phase 2 alone: 8.4 us with per-step sc1 loads vs 5.0 us as a launch);
    // res is stored plainly (the next launch reads it)
    for (int t = w; t < ndn; t += G) gemm_tile<PRO_PLAIN, EPI_RESID, NWM, UM, false, true, 1>(P.dn, t, sm.g1, st, t == w, false, nullptr, &al);
  }
  // the last workgroup out re-arms the counters (every workgroup is past its wait)
  if (P.phases & 8) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (P.phases & 16) {
      const int sh = w & 7, n_sh = (G - sh + 7) / 8, n_used = G < 8 ? G : 8;
      const int prev = __hip_atomic_fetch_add(sh_exit(P.sync, sh), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == n_sh - 1) {
        __hip_atomic_store(sh_exit(P.sync, sh), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int t = __hip_atomic_fetch_add(sh_top(P.sync), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == n_used - 1) {
          for (int k = 0; k < 8; ++k) __hip_atomic_store(sh_arr(P.sync, k), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(sh_top(P.sync), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else {
      const int prev = __hip_atomic_fetch_add(P.sync + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == G - 1) {
        __hip_atomic_store(P.sync, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(P.sync + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}
}  // namespace

// res [M, H] (in/out residual), g [M, I] scratch, wgu = shuffle_weight([gate; up] [2I, H], gamma, swiglu),
// wd = shuffle_weight(W_down [H, I]); ws = the product split workspace; S = gate_up parts (1 = none).
int launch_fused_mlp(void* res, void* g, const void* wgu, const void* wd, int* ws, int S, int* sync, int* err, int M,
                     int H, int I, float eps, int grid, int phases, hipStream_t stream) {
  if (M < 1 || M > 16 || H % 32 || I % 32 || S < 1 || grid < 1) return -1;
  const RopeEpi none{};
  MlpArgs P;
  P.gu = GemmArgs{(uint16_t*)g, (const uint16_t*)res, (const short8*)wgu, nullptr, M, I, H, I, eps, none, nullptr,
                  nullptr};
  P.dn = GemmArgs{nullptr, (const uint16_t*)g, (const short8*)wd, (uint16_t*)res, M, H, I, 0, eps, none, nullptr,
                  nullptr};
  P.ws = ws;
  P.S = S;
  P.n_gu = I / 16;
  P.n_dn = H / 16;
  P.sync = sync;
  P.err = err;
  P.phases = phases;
  if (phases & 4)   // diagnosis: plain phase-1 stores (wrong across XCDs, timing only)
    hipLaunchKernelGGL(fused_mlp_kernel<false>, dim3(grid), dim3(NWM * 64), alds_bytes(M, I), stream, P);
  else
    hipLaunchKernelGGL(fused_mlp_kernel<true>, dim3(grid), dim3(NWM * 64), alds_bytes(M, I), stream, P);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
