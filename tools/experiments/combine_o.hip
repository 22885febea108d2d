// EXPERIMENT (not adopted, profiles/r03/experiments_r03.md): K3 split combine + o-projection
// (+ residual) in ONE launch for the single-GPU decode step. Numerically exact vs the fp32 oracle
// (test_combine_o_gpu.py) but the driver bench measured 787.8 / 790.3 tok/s with it vs 840.5
// without (same box, alternating): the in-launch combine + grid barrier cost more than the
// separate combine launch they replace.
//
// The grouped decode attention leaves every split's partial (m, l, O) for the combine; the next
// op is the o-projection, a 256-tile skinny GEMM (one workgroup per CU) whose first weight round
// trip and launch ramp sit on the critical path. Here the o-GEMM's workgroups first put their
// tile's stage-0 weights in flight (weights never depend on activations), then combine a slice of
// the attention rows — unit = (row, 32-dim chunk), one unit per half workgroup, 8 dim-lanes x 16
// slot-lanes, shuffle + LDS merge in a fixed order — store them write-through (sc1), cross ONE
// grid barrier, and run the o tile reading the combined rows with sc1 loads (skinny_core.h
// SC1 = true; MI355X_MICROARCH "Valid forms" row 1: sc1 payload stores -> vmcnt(0) -> workgroup
// barrier -> one agent atomic; consumers poll, barrier, sc1 loads). Saves the combine launch
// (separate: ~4.9 us per layer at the driver config) and overlaps the o weights' first fetch
// with the combine.
//
// Residency: the grid is the o tile count, at most one workgroup per CU (256 for Llama-3-8B /
// Mistral-7B; wider o projections keep the separate combine), so every workgroup is resident at
// once and the barrier always completes; the wait is bounded anyway (on expiry *err is set and the kernel
// proceeds: wrong numbers, never a hang — the engine reads the flag at turn end). Only the
// single-GPU path uses it (tensor-parallel ranks keep the separate combine: their o-GEMM may
// already spin on peers in its epilogue).
#include "attn_core.h"
#include "skinny_core.h"

namespace {
using namespace skinny;
using attn::AttnArgs;

constexpr long long BAR_POLL_LIMIT = 1ll << 24;

struct CombineArgs {
  uint16_t* out;          // [B, Hq, D] attention output (combined rows written here)
  const float* part_o;    // [B, Hq, stride, D]
  const float* part_ml;   // [B, Hq, stride, 4]
  const int* groups;      // [B][3] or nullptr
  int stride, num_splits, B, Hq, Hkv;
  int* bar;               // [2] arrive / depart counters, zero between launches
  int* err;
};

RT_DEVICE void merge_state(float& M, float& L, float4_& O, float m2, float l2, float4_ o2) {
  if (!(l2 > 0.f)) return;
  const float Mc = fmaxf(M, m2);
  const float a = M == -INFINITY ? 0.f : exp2f(M - Mc), f = exp2f(m2 - Mc);
  O = O * a + f * o2;
  L = L * a + f * l2;
  M = Mc;
}

// one (row = b * Hq + head, 32-dim chunk) unit on the 128 threads `t` of a half workgroup
template <int D>
RT_DEVICE void combine_unit(const CombineArgs& c, int unit, bool live, int t, int half, float (*red)[2][8][6]) {
  constexpr int CH = D / 32;
  const int row = unit / CH, chunk = unit - row * CH;
  const int b = row / c.Hq;
  const int dl = t & 7, sl = t >> 3;             // 8 dim-lanes x 16 slot-lanes
  const int d0 = chunk * 32 + 4 * dl;
  const int G = c.Hq / c.Hkv;
  int n = 1;
  if (c.groups != nullptr) {
    const int b0 = c.groups[3 * b], nn = c.groups[3 * b + 1], sh = c.groups[3 * b + 2];
    if (!(nn < 1 || nn * G > 16 || b0 < 0 || b < b0 || b - b0 >= nn || sh < 0)) n = nn;   // as attn_item
  }
  const int nslots = n * c.num_splits;
  float M = -INFINITY, L = 0.f;
  float4_ O = {0.f, 0.f, 0.f, 0.f};
  if (nslots > 1) {
    const float* __restrict__ po = c.part_o + (size_t)row * c.stride * D;
    const float* __restrict__ pml = c.part_ml + (size_t)row * c.stride * 4;
    for (int s = sl; s < nslots; s += 16) {
      const float4_ ml = *reinterpret_cast<const float4_*>(pml + (size_t)s * 4);
      const float4_ o = *reinterpret_cast<const float4_*>(po + (size_t)s * D + d0);
      merge_state(M, L, O, ml[0], ml[1], o);
    }
  }
  // the 8 slot-lanes of a wave (lane bits 3..5), fixed order on both partners
#pragma unroll
  for (int x = 8; x < 64; x <<= 1) {
    const float m2 = __shfl_xor(M, x, 64), l2 = __shfl_xor(L, x, 64);
    float4_ o2;
#pragma unroll
    for (int i = 0; i < 4; ++i) o2[i] = __shfl_xor(O[i], x, 64);
    if (sl & (x >> 3)) {
      const float mm = M, ll = L;
      const float4_ oo = O;
      M = m2; L = l2; O = o2;
      merge_state(M, L, O, mm, ll, oo);
    } else {
      merge_state(M, L, O, m2, l2, o2);
    }
  }
  const int w = (t >> 6) & 1;                     // wave within the half
  if ((t & 63) < 8) {
    float* e = red[half][w][dl];
    e[0] = O[0]; e[1] = O[1]; e[2] = O[2]; e[3] = O[3]; e[4] = M; e[5] = L;
  }
  __syncthreads();
  if (live && nslots > 1 && t < 8) {              // rows without splits were written by attention
    const float* e = red[half][1][dl];
    merge_state(M, L, O, e[4], e[5], float4_{e[0], e[1], e[2], e[3]});
    const float inv = L > 0.f ? 1.f / L : 0.f;
    attn::store_bf16x4(c.out + (size_t)row * D + d0, O[0] * inv, O[1] * inv, O[2] * inv, O[3] * inv, true);
  }
  __syncthreads();
}

template <int D, int U>
__global__ void __launch_bounds__(256) combine_o_kernel(CombineArgs c, GemmArgs p) {
  __shared__ union {
    GemmSmem<1, 4> g;
    float red[2][2][8][6];
  } sm;
  // 1. this tile's first weight stage in flight before anything waits
  Stage<PRO_PLAIN, EPI_RESID, U> st0;
  gemm_prefetch<PRO_PLAIN, EPI_RESID, 4, U>(p, blockIdx.x, st0);
  // 2. combine units 2 * blockIdx.x + half, 2 * gridDim.x apart
  const int half = threadIdx.x >> 7, t = threadIdx.x & 127;
  const int units = c.B * c.Hq * (D / 32);
  for (int u0 = 2 * blockIdx.x; u0 < units; u0 += 2 * gridDim.x) {
    const int u = u0 + half;
    // both halves run the same number of workgroup barriers: a half past the last unit redoes
    // the last one without storing it
    combine_unit<D>(c, u < units ? u : units - 1, u < units, t, half, sm.red);
  }
  // 3. grid barrier: every combined row is visible before any tile reads it
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // MI355X_MICROARCH "Valid forms", table row 1 (no release / acquire: an agent release writes back
  // the XCD L2's dirty lines and 256 acquire pollers cut chip bandwidth): every combined byte was
  // stored sc1 and drained (vmcnt(0)) before the workgroup barrier, ONE lane adds to the counter,
  // the poll is an sc1 (relaxed agent) load, and every load of those bytes below is an sc1 load
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(c.bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long long it = 0;
    while (__hip_atomic_load(c.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (int)gridDim.x) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > BAR_POLL_LIMIT) {
        __hip_atomic_store(c.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    // the last workgroup past the barrier re-arms it for the next launch
    if (__hip_atomic_fetch_add(c.bar + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      __hip_atomic_store(c.bar + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c.bar, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  // 4. the o tile on the combined rows (sc1 activation loads), residual added in place
  gemm_tile<PRO_PLAIN, EPI_RESID, 4, U, true>(p, blockIdx.x, sm.g, st0, true, false);
}
}  // namespace

// attn_out [B, Hq, D] (uncombined rows hold the attention launch's partials in part_o / part_ml);
// Ws: shuffled o weight [N, Hq * D]; res [B, N] += attn . Wo^T. bar: 2 ints, zero; err: 1 int.
int launch_combine_o(void* attn_out, const float* part_o, const float* part_ml, const int* groups, int stride,
                     int num_splits, int B, int Hq, int Hkv, int D, const void* Ws, void* res, int N, int* bar,
                     int* err, hipStream_t stream) {
  if (B < 1 || B > 16 || D != 128 || Hq % Hkv || N % 16 || (Hq * D) % 32) return -1;
  if (((uintptr_t)attn_out & 15) || ((uintptr_t)Ws & 15)) return -2;
  const int tiles = N / 16;
  int cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -3;
  if (tiles > cus) return -4;   // one workgroup per CU: residency of the grid barrier, and the
                               // hand-off form measured for it (MI355X_MICROARCH "Valid forms")
  CombineArgs c{(uint16_t*)attn_out, part_o, part_ml, groups, stride, num_splits, B, Hq, Hkv, bar, err};
  const int K = Hq * D;
  GemmArgs p{nullptr, (const uint16_t*)attn_out, (const rt::short8*)Ws, (uint16_t*)res, B, N, K, N, 0.f,
             RopeEpi{}, nullptr, nullptr};
  hipLaunchKernelGGL((combine_o_kernel<128, 4>), dim3(tiles), dim3(256), 0, stream, c, p);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
