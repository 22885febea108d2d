// Decode-path linear layers (M <= 16 rows, up to 32 with plain / norm prologues): y[M,N] = x[M,K] . W[N,K]^T on MFMA, with the
// layer's elementwise work fused in, so a decode layer needs no separate norm/act kernels.
// The tile code (weight layout, pipeline, prologues, epilogues) lives in skinny_core.h and is
// shared with the persistent decode-layer kernel; this file holds the one-tile-per-workgroup
// launches, the weight shuffle, and the launchers.
//
// Fusions (details in skinny_core.h):
//   prologue NORM : RMSNorm with gamma folded into W and 1/rms(x_m) from the same A fragments
//                   (no extra pass, no atomics: deterministic).
//   prologue NORM_ADD: tensor-parallel residual + all-reduced partial, published by workgroup 0.
//   epilogue RESID: res[m,n] = bf16(acc + res[m,n])   (the residual add, in place)
//   epilogue SWIGLU: out[m,n] = silu(acc_gate) * acc_up,  W = [gate(I) ; up(I)]
//   epilogue ROPE  : the qkv projection. Its q/k weight rows are stored pair-interleaved per
//                   head (row 2i <- d=i, row 2i+1 <- d=i+D/2; `shuffle_weight(rope_heads=)`),
//                   so both halves of every rotate-half pair land in the same 16-column tile:
//                   the epilogue rotates them (fp32 cos|sin table), writes q to [M, Hq, D] and
//                   scatters k / v straight into the paged caches (k [blk][h][off][D], v
//                   transposed [blk][h][D][off]). Replaces the K2 rope/cache launch.
#include "skinny_core.h"

#include <cstdio>
#include <cstdlib>

namespace {
using rt::short8;
using namespace skinny;

template <int PRO, int EPI, int NW, int U>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_kernel(GemmArgs p) {
  __shared__ GemmSmem<nacc<EPI>(), NW> sm;
  Stage<PRO, EPI, U> st0;
  gemm_tile<PRO, EPI, NW, U, false>(p, blockIdx.x, sm, st0, false, blockIdx.x == 0);
}

// TN tiles per workgroup (skinny_core.h gemm_tiles): serving batches, M > 4
template <int PRO, int EPI, int NW, int U, int TN, int MB = 1>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_multi_kernel(GemmArgs p) {
  // two row blocks x (gate + up) x 4 tiles would not fit the static LDS: that variant is never
  // launched (the dispatcher caps SwiGLU at 2 tiles with two row blocks), compiled as 2 tiles
  constexpr int TNX = (MB == 2 && nacc<EPI>() == 2 && TN > 2) ? 2 : TN;
  __shared__ GemmSmemN<nacc<EPI>(), NW, TNX, MB> sm;
  gemm_tiles<PRO, EPI, NW, U, TNX, MB>(p, blockIdx.x * TNX, sm);
}


// the dynamic LDS of an ALDS launch: [16] row sums of squares, then the staged rows
RT_DEVICE ALds alds_view(int kspan) {
  extern __shared__ float alds_dyn[];
  return ALds{reinterpret_cast<uint16_t*>(alds_dyn + 16), alds_dyn, kspan + 8};
}

// The same launch with the A operand staged in LDS (skinny_core.h ALDS): tensor-parallel shard
// shapes, where the per-k-step activation loads, not HBM, bound the launch.
template <int PRO, int EPI, int NW, int U>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_alds_kernel(GemmArgs p) {
  __shared__ GemmSmem<nacc<EPI>(), NW> sm;
  Stage<PRO, EPI, U> st0;
  const ALds al = alds_view(p.K);
  gemm_tile<PRO, EPI, NW, U, false, true>(p, blockIdx.x, sm, st0, false, blockIdx.x == 0, nullptr, &al);
}

// CU-balanced launch for tile counts that are not a multiple of the CU count (gate_up of
// Llama-3-8B / Mistral-7B: 896 tiles on 256 CUs = 3.5 per CU, so half the CUs stream a 4th
// tile while the rest idle): the last R = T mod CUs tiles run as two K-halves each (SplitX in
// skinny_core.h), the other T - R whole. Every CU then gets the same bytes (3 tiles + one
// half-tile at 896/256). Workgroups [0, 2R) are the halves (dispatched first, so their
// hand-offs finish under the whole tiles' streams), [2R, T + R) the whole tiles.
// tools/exp_balance.hip: swiglu 768 / 896 / 1024 tiles = 31.0 / 37.6 / 40.5 us (896 is 1.8 us
// above the line through its neighbours).
constexpr int SPLIT_CTRS = 256;   // counter words at the head of the split workspace
template <int PRO, int EPI, int NW, int U>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_bal_kernel(GemmArgs p, int* __restrict__ ws, int R, int xpair) {
  __shared__ GemmSmem<nacc<EPI>(), NW> sm;
  Stage<PRO, EPI, U> st0;
  const int T = p.N / 16;
  const int b = blockIdx.x;
  if (b < 2 * R) {
    // the two halves of a tile on ONE XCD when R % 8 == 0 (blocks b and b + 8 of each group of 16:
    // round-robin dispatch puts both on XCD b % 8), so the combine reads same-XCD partials
    int r, idx;
    if (xpair && (R & 7) == 0) {
      r = (b >> 4) * 8 + (b & 7);
      idx = (b >> 3) & 1;
    } else {
      r = b >> 1;
      idx = b & 1;
    }
    const SplitX sx{reinterpret_cast<float*>(ws + SPLIT_CTRS) + (size_t)r * 2 * SPLIT_STRIDE, ws + r, idx, 2};
    gemm_tile<PRO, EPI, NW, U, false>(p, T - R + r, sm, st0, false, false, &sx);
  } else {
    gemm_tile<PRO, EPI, NW, U, false>(p, b - 2 * R, sm, st0, false, false);
  }
}

// Split-K launch for shapes with FEWER tiles than CUs — the tensor-parallel shard GEMMs (Llama-3-8B
// at tp 8: qkv 48 tiles, gate_up 112; tp 4: 96 / 224). One tile per workgroup would stream the
// weights with a fraction of the chip, so every tile's K range is cut into S parts (T x S
// workgroups, SplitX hand-off, last arriver combines in index order and runs the epilogue).
// Placement (speed only, never correctness): with T % 8 == 0 the S parts of a tile get block ids
// b, b + 8, ... — one XCD under round-robin dispatch, so the combine reads same-XCD partials.
// NORM_ADD: every part of tile 0 publishes its K range of x + x2.
template <int PRO, int EPI, int NW, int U, bool ALDS = false>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_splitk_kernel(GemmArgs p, int* __restrict__ ws, int S) {
  __shared__ GemmSmem<nacc<EPI>(), NW> sm;
  Stage<PRO, EPI, U> st0;
  const int T = p.N / 16;
  const int b = blockIdx.x;
  int tile, part;
  if ((T & 7) == 0) {
    const int j = b >> 3;
    tile = (j / S) * 8 + (b & 7);
    part = j % S;
  } else {
    tile = b / S;
    part = b % S;
  }
  const SplitX sx{reinterpret_cast<float*>(ws + SPLIT_CTRS) + (size_t)tile * S * SPLIT_STRIDE, ws + tile, part, S};
  if constexpr (ALDS) {
    const int ks = p.K / 32;
    const ALds al = alds_view(32 * ((ks + S - 1) / S + 1));
    gemm_tile<PRO, EPI, NW, U, false, true>(p, tile, sm, st0, false, tile == 0, &sx, &al);
  } else {
    gemm_tile<PRO, EPI, NW, U, false>(p, tile, sm, st0, false, tile == 0, &sx);
  }
}

// TN tiles per workgroup (gemm_tiles) with each group of TN tiles' K range cut into S parts (SplitX hand-off; group ids dealt as
// in skinny_gemm_splitk_kernel, so a group's parts share an XCD under round-robin dispatch)
template <int PRO, int EPI, int NW, int U, int TN, int MB = 1>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_multi_split_kernel(GemmArgs p, int* __restrict__ ws, int S) {
  __shared__ GemmSmemN<nacc<EPI>(), NW, TN, MB> sm;
  const int G = (p.N / 16 + TN - 1) / TN;
  const int b = blockIdx.x;
  int grp, part;
  if ((G & 7) == 0) {
    const int j = b >> 3;
    grp = (j / S) * 8 + (b & 7);
    part = j % S;
  } else {
    grp = b / S;
    part = b % S;
  }
  const SplitX sx{reinterpret_cast<float*>(ws + SPLIT_CTRS) + (size_t)grp * S * TN * MB * SPLIT_STRIDE, ws + grp, part,
                  S};
  gemm_tiles<PRO, EPI, NW, U, TN, MB>(p, grp * TN, sm, &sx);
}

int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cache[dev] = n > 0 ? n : -1;
  }
  return cache[dev] > 0 ? cache[dev] : 0;
}

// RT_WEIGHT_ORDER=0 pins tile-major weights everywhere (A/B against the shape rule; read once,
// so shuffle and GEMM launches of one process agree)
int forced_order() {
  static const int v = [] {
    const char* e = getenv("RT_WEIGHT_ORDER");
    return e ? atoi(e) : -1;
  }();
  return v;
}

// Ws[t][s][l][j] = W[16t + (l&15)][32s + 8(l>>4) + j] (optionally W * gamma[k] folded in)
// If rope_rows > 0, output row r < rope_rows takes source row h*D + (p>>1) + (p&1)*D/2
// (r = h*D + p): the pair-interleaved q/k order the ROPE epilogue expects.
// swiglu: N = 2I rows [gate; up], stored k-step-paired: Ws[t][s][h][l][j] = W[h*I + 16t + (l&15)][...]
__global__ void shuffle_kernel(short8* __restrict__ Ws, const uint16_t* __restrict__ W,
                               const uint16_t* __restrict__ gamma, int N, int K, int rope_rows, int D, int swiglu,
                               int force_order) {
  const int nsteps = K / 32;
  const int64_t total = (int64_t)(N / 16) * nsteps * 64;
  const int T = swiglu ? N / 32 : N / 16;   // output tiles (SwiGLU: gate + up rows per tile)
  const int order = force_order >= 0 ? force_order : weight_order(T, nsteps, swiglu != 0, rope_rows > 0);
  const int recs = swiglu ? 128 : 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i & 63);
    int64_t ts = i >> 6;
    int h = 0;
    if (swiglu) {
      h = (int)(ts & 1);
      ts >>= 1;
    }
    const int s = (int)(ts % nsteps);
    const int64_t t = ts / nsteps;
    int row = (int)(16 * t + (l & 15)) + h * (N / 2);
    if (row < rope_rows) {
      const int h = row / D, p = row - h * D;
      row = h * D + (p >> 1) + (p & 1) * (D >> 1);
    }
    const int k0 = 32 * s + 8 * (l >> 4);
    short8 v = *reinterpret_cast<const short8*>(W + (size_t)row * K + k0);
    if (gamma != nullptr) {
      const short8 gv = *reinterpret_cast<const short8*>(gamma + k0);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)rt::f2bf(rt::bf2f((uint16_t)v[j]) * rt::bf2f((uint16_t)gv[j]));
    }
    Ws[rec_index((int)t, s, T, nsteps, order, recs) + h * 64 + l] = v;
  }
}

// Exact inverse of shuffle_kernel's permutation (gamma, if any, stays folded): the row-major
// weight for the prefill GEMMs when only the shuffled copy is kept resident (70B on one GPU).
__global__ void unshuffle_kernel(uint16_t* __restrict__ W, const short8* __restrict__ Ws, int N, int K, int rope_rows,
                                 int D, int swiglu, int force_order) {
  const int nsteps = K / 32;
  const int64_t total = (int64_t)(N / 16) * nsteps * 64;
  const int T = swiglu ? N / 32 : N / 16;
  const int order = force_order >= 0 ? force_order : weight_order(T, nsteps, swiglu != 0, rope_rows > 0);
  const int recs = swiglu ? 128 : 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i & 63);
    int64_t ts = i >> 6;
    int h = 0;
    if (swiglu) {
      h = (int)(ts & 1);
      ts >>= 1;
    }
    const int s = (int)(ts % nsteps);
    const int64_t t = ts / nsteps;
    int row = (int)(16 * t + (l & 15)) + h * (N / 2);
    if (row < rope_rows) {
      const int hh = row / D, p = row - hh * D;
      row = hh * D + (p >> 1) + (p & 1) * (D >> 1);
    }
    const int k0 = 32 * s + 8 * (l >> 4);
    *reinterpret_cast<short8*>(W + (size_t)row * K + k0) = Ws[rec_index((int)t, s, T, nsteps, order, recs) + h * 64 + l];
  }
}
}  // namespace

int launch_unshuffle_weight(void* W, const void* Ws, int N, int K, int rope_rows, int D, int swiglu,
                            hipStream_t stream) {
  if (N % 16 || K % 32 || N <= 0 || K <= 0 || rope_rows > N || (rope_rows && (D <= 0 || D % 2)) ||
      (swiglu && (N / 2) % 16))
    return -1;
  const int64_t total = (int64_t)(N / 16) * (K / 32) * 64;
  const int64_t grid = (total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536;
  hipLaunchKernelGGL(unshuffle_kernel, dim3((unsigned)grid), dim3(256), 0, stream, (uint16_t*)W, (const short8*)Ws,
                     N, K, rope_rows, D, swiglu, forced_order());
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ALDS decision (skinny_core.h): RT_GEMM_ALDS=1 whenever the staged rows fit, =2 when they fit
// and the launch has at most one workgroup per CU, unset / 0 never. Staged rows + row sums
// <= 48 KB, so the workgroup stays under 64 KB of LDS.
constexpr int ALDS_MAX_BYTES = 48 * 1024;
bool use_alds(int M, int kspan, int wgs, int cus) {
  // default OFF: measured slower than the pipelined activation loads on every shard shape except
  // the NORM_ADD prologue, which the decode path no longer uses (tools/probes/gemm_variants.py,
  // profiles/r04/gemm_variants.md); RT_GEMM_ALDS=1 forces it, =2 is the "shard shapes" rule
  static const int mode = [] {
    const char* e = getenv("RT_GEMM_ALDS");
    return e ? atoi(e) : 0;
  }();
  if (mode == 0 || skinny::alds_bytes(M, kspan) > ALDS_MAX_BYTES) return false;
  return mode == 1 || (mode == 2 && cus > 0 && wgs <= cus);
}

int split_workspace_ints(int max_split_tiles) { return SPLIT_CTRS + max_split_tiles * 2 * SPLIT_STRIDE; }

// Split-K part count for a T-tile, ks-k-step GEMM on `cus` CUs (0 = no split-K): the most parts
// that keep every CU at one workgroup (profiles/r03/gemm_tp_shards_*), each part >= 8 k-steps,
// T x S capped by the workspace. RT_SPLITK=<S> pins S (1 = off),
// RT_SPLITK_TARGET=<wgs> = the r03-first rule S = ceil(wgs / T) (microbenchmark sweeps; read once).
int splitk_parts(int T, int ks, int cus, int64_t ws_ints) {
  static const int pinned = [] {
    const char* e = getenv("RT_SPLITK");
    return e ? atoi(e) : 0;
  }();
  static const int target_env = [] {
    const char* e = getenv("RT_SPLITK_TARGET");
    return e ? atoi(e) : 0;
  }();
  if (cus <= 0 || T >= cus || T > SPLIT_CTRS || pinned == 1) return 0;
  const int smax = ks / 8 < 16 ? ks / 8 : 16;
  int S;
  if (pinned > 1) {
    S = pinned;
  } else if (target_env > 0) {
    S = (target_env + T - 1) / T;
  } else {
    // at most ONE part per CU: T x S just above the CU count doubles some CUs, which costs more
    // than the split gains (r03 microbench, Llama-3-8B shards, us unsplit -> split: tp 8 qkv 48
    // tiles 8.70 -> 8.34 at S = 6 (288 WGs) / 11.26 at S = 11; tp 2 qkv 192 tiles 9.44 -> 10.85 at
    // S = 2; tp 4 gate_up 224 tiles 13.64 -> 14.18 at S = 2): S = floor(cus / T), so only shapes
    // with <= cus / 2 tiles split
    S = cus / T;
  }
  S = S < smax ? S : smax;
  while (S >= 2 && SPLIT_CTRS + (int64_t)T * S * SPLIT_STRIDE > ws_ints) --S;
  return S >= 2 ? S : 0;
}

int launch_skinny_gemm(void* out, const void* x, const void* Ws, void* res, int M, int N, int K, int ldo, float eps,
                       int pro, int epi, const void* rope, const void* x2, void* xo, hipStream_t stream,
                       int* split_ws, int64_t split_ws_ints, int split_mode) {
  if (pro == PRO_NORM_ADD && x2 == nullptr) return -5;
  // 17..32 rows: only the multi-tile launches below (two 16-row blocks per MFMA pass)
  if (M < 1 || M > 32 || K % 32 || N % 16) return -1;
  if (M > 16 && (pro == PRO_NORM_ADD || epi == EPI_AR)) return -1;
  RopeEpi re{};
  if (epi == EPI_ROPE) {
    if (rope == nullptr) return -3;
    re = *static_cast<const RopeEpi*>(rope);
    if (re.D % 16 || N != (re.Hq + 2 * re.Hkv) * re.D) return -4;
  }
  // split-K (split_mode bit 1) when the shape has fewer tiles than CUs: tensor-parallel shards
  if (split_ws != nullptr && (split_mode & 2) && M <= 16) {
    const int T = N / 16;
    const int S = splitk_parts(T, K / 32, device_cus(), split_ws_ints);
    if (S >= 2) {
      GemmArgs args{(uint16_t*)out, (const uint16_t*)x, (const short8*)Ws, (uint16_t*)res, M, N, K, ldo,
                    eps, re, (const uint16_t*)x2, (uint16_t*)xo};
      args.kmajor = forced_order();
      const dim3 grid(T * S);
      const int kspan = 32 * ((K / 32 + S - 1) / S + 1);
      const bool alds = use_alds(M, kspan, T * S, device_cus());
      const size_t lds = alds ? (size_t)skinny::alds_bytes(M, kspan) : 0;
      // (NW, U) of the split-K parts: 8 waves x 2 steps — one part per CU streams with twice
      // the bytes in flight of 4 waves (r03 microbench, Llama-3-8B tp 4 qkv 8.79 -> 7.98 us; tp 2/8
      // shards within noise; 4x4 no better: profiles/r03/gemm_tp_splitk_cfg_sweep.md).
      // RT_SPLITK_CFG=<NW>x<U> (8x2, 4x2, 4x4) pins it
      static const int skcfg = [] {
        const char* e = getenv("RT_SPLITK_CFG");
        int nw = 0, u = 0;
        if (!e || sscanf(e, "%dx%d", &nw, &u) != 2) return 802;
        return nw * 100 + u;
      }();
#define RT_SK(P, E)                                                                                                 \
  do {                                                                                                              \
    if (skcfg == 402)                                                                                               \
      hipLaunchKernelGGL((skinny_gemm_splitk_kernel<P, E, 4, 2>), grid, dim3(256), 0, stream, args, split_ws, S);  \
    else if (skcfg == 404)                                                                                          \
      hipLaunchKernelGGL((skinny_gemm_splitk_kernel<P, E, 4, 4>), grid, dim3(256), 0, stream, args, split_ws, S);  \
    else if (alds)                                                                                                  \
      hipLaunchKernelGGL((skinny_gemm_splitk_kernel<P, E, 8, 2, true>), grid, dim3(512), lds, stream, args, split_ws, \
                         S);                                                                                        \
    else                                                                                                            \
      hipLaunchKernelGGL((skinny_gemm_splitk_kernel<P, E, 8, 2>), grid, dim3(512), 0, stream, args, split_ws, S);  \
  } while (0)
      if (pro == PRO_PLAIN && epi == EPI_STORE) RT_SK(PRO_PLAIN, EPI_STORE);
      else if (pro == PRO_NORM && epi == EPI_STORE) RT_SK(PRO_NORM, EPI_STORE);
      else if (pro == PRO_NORM_ADD && epi == EPI_STORE) RT_SK(PRO_NORM_ADD, EPI_STORE);
      else if (pro == PRO_PLAIN && epi == EPI_RESID) RT_SK(PRO_PLAIN, EPI_RESID);
      else if (pro == PRO_NORM && epi == EPI_SWIGLU) RT_SK(PRO_NORM, EPI_SWIGLU);
      else if (pro == PRO_NORM_ADD && epi == EPI_SWIGLU) RT_SK(PRO_NORM_ADD, EPI_SWIGLU);
      else if (pro == PRO_NORM && epi == EPI_ROPE) RT_SK(PRO_NORM, EPI_ROPE);
      else if (pro == PRO_NORM_ADD && epi == EPI_ROPE) RT_SK(PRO_NORM_ADD, EPI_ROPE);
      else if (pro == PRO_PLAIN && epi == EPI_ROPE) RT_SK(PRO_PLAIN, EPI_ROPE);
      else if (pro == PRO_PLAIN && epi == EPI_SWIGLU) RT_SK(PRO_PLAIN, EPI_SWIGLU);
      else return -2;
#undef RT_SK
      return hipGetLastError() == hipSuccess ? 0 : -6;
    }
  }
  // Serving batches (M > 4): TN tiles per workgroup share each activation fragment (skinny_core.h
  // gemm_tiles), as long as the launch still covers 3/4 of the CUs. MI355X, Llama-3-8B, M = 16
  // (profiles/r05/gemm_multi_tile.md): lm_head 235.0 -> 163.2 us (TN 4), gate_up 42.1 -> 38.7
  // (TN 4), qkv 16.7 -> 13.5 (TN 2); o / down (256 tiles) lose with fewer workgroups and keep one
  // tile. RT_SKINNY_TN=<TN> (1 = off) pins the tile count, RT_SKINNY_TNCFG=<NW>x<U> the variant
  // (microbenchmarks); the M <= 4 decode path is unchanged.
  // A/B knob: the smallest M the multi-tile rule applies to (M = 3 gains nothing: the activation
  // fragments of 3 rows are L1 hits, profiles/r05/gemm_multi_tile.md); RT_SKINNY_TNS=2 forces the
  // two-tile K-split below 9 rows
  static const int tn_min_m = [] {
    const char* e = getenv("RT_SKINNY_TN_MINM");
    return e ? atoi(e) : 5;
  }();
  if ((M >= tn_min_m || M > 16) && (pro == PRO_PLAIN || pro == PRO_NORM) && epi != EPI_AR) {
    const int MB = M > 16 ? 2 : 1;
    static const int tn_env = [] {
      const char* e = getenv("RT_SKINNY_TN");
      return e ? atoi(e) : -1;
    }();
    static const int tncfg = [] {
      const char* e = getenv("RT_SKINNY_TNCFG");
      int nw = 0, u = 0;
      if (!e || sscanf(e, "%dx%d", &nw, &u) != 2) return 402;
      return nw * 100 + u;
    }();
    const int T16 = N / 16, cus = device_cus(), need = cus * 3 / 4;
    int tn = tn_env >= 0 ? tn_env : (cus <= 0 ? 1 : (T16 / 4 >= need ? 4 : (T16 / 2 >= need ? 2 : 1)));
    // LDS: two row blocks x (gate + up) x 4 tiles would not fit
    if (MB == 2) tn = tn >= 4 && epi != EPI_SWIGLU ? 4 : (tn >= 2 ? 2 : 1);
    // one tile per workgroup would still fill the chip (o / down: 256 tiles): two tiles per
    // workgroup over two K halves keep the workgroup count and halve the activation reads — from
    // 9 rows on (M = 16: down 28.8 -> 23.6 us, o 11.0 -> 10.6; M = 8: o 8.8 -> 10.0, down even,
    // profiles/r05/gemm_multi_tile.md). RT_SKINNY_TNS=0 keeps one tile.
    static const int tns_env = [] {
      const char* e = getenv("RT_SKINNY_TNS");
      return e ? atoi(e) : 1;
    }();
    const int G2 = (T16 + 1) / 2;
    if (tn == 1 && tn_env < 0 && tns_env && (M > 8 || tns_env == 2) && cus > 0 && T16 >= need && G2 <= SPLIT_CTRS && K / 32 >= 32 &&
        split_ws != nullptr && split_ws_ints >= (int64_t)SPLIT_CTRS + (int64_t)G2 * 2 * 2 * MB * SPLIT_STRIDE) {
      GemmArgs args{(uint16_t*)out, (const uint16_t*)x, (const short8*)Ws, (uint16_t*)res, M, N, K, ldo,
                    eps, re, nullptr, nullptr};
      args.kmajor = forced_order();
      const dim3 grid(G2 * 2);
#define RT_MS(P, E)                                                                                               \
  do {                                                                                                            \
    if (MB == 2)                                                                                                  \
      hipLaunchKernelGGL((skinny_gemm_multi_split_kernel<P, E, 4, 2, 2, 2>), grid, dim3(256), 0, stream, args,    \
                         split_ws, 2);                                                                            \
    else                                                                                                          \
      hipLaunchKernelGGL((skinny_gemm_multi_split_kernel<P, E, 4, 2, 2>), grid, dim3(256), 0, stream, args,       \
                         split_ws, 2);                                                                            \
  } while (0)
      if (pro == PRO_PLAIN && epi == EPI_STORE) RT_MS(PRO_PLAIN, EPI_STORE);
      else if (pro == PRO_NORM && epi == EPI_STORE) RT_MS(PRO_NORM, EPI_STORE);
      else if (pro == PRO_PLAIN && epi == EPI_RESID) RT_MS(PRO_PLAIN, EPI_RESID);
      else if (pro == PRO_NORM && epi == EPI_RESID) RT_MS(PRO_NORM, EPI_RESID);
      else if (pro == PRO_NORM && epi == EPI_SWIGLU) RT_MS(PRO_NORM, EPI_SWIGLU);
      else if (pro == PRO_PLAIN && epi == EPI_SWIGLU) RT_MS(PRO_PLAIN, EPI_SWIGLU);
      else if (pro == PRO_NORM && epi == EPI_ROPE) RT_MS(PRO_NORM, EPI_ROPE);
      else if (pro == PRO_PLAIN && epi == EPI_ROPE) RT_MS(PRO_PLAIN, EPI_ROPE);
      else return -2;
#undef RT_MS
      return hipGetLastError() == hipSuccess ? 0 : -6;
    }
    if (tn == 2 || tn == 4 || MB == 2) {
      GemmArgs args{(uint16_t*)out, (const uint16_t*)x, (const short8*)Ws, (uint16_t*)res, M, N, K, ldo,
                    eps, re, nullptr, nullptr};
      args.kmajor = forced_order();
      const int T = N / 16;
      const dim3 grid((T + tn - 1) / tn);
#define RT_MT(P, E)                                                                                               \
  do {                                                                                                            \
    if (MB == 2 && tn == 4)                                                                                       \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 4, 2, 4, 2>), grid, dim3(256), 0, stream, args);        \
    else if (MB == 2 && tn == 2)                                                                                  \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 4, 2, 2, 2>), grid, dim3(256), 0, stream, args);        \
    else if (MB == 2)                                                                                             \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 4, 2, 1, 2>), grid, dim3(256), 0, stream, args);        \
    else if (tn == 2 && tncfg == 802)                                                                             \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 8, 2, 2>), grid, dim3(512), 0, stream, args);           \
    else if (tn == 2 && tncfg == 404)                                                                             \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 4, 4, 2>), grid, dim3(256), 0, stream, args);           \
    else if (tn == 2)                                                                                             \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 4, 2, 2>), grid, dim3(256), 0, stream, args);           \
    else if (tncfg == 802)                                                                                        \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 8, 2, 4>), grid, dim3(512), 0, stream, args);           \
    else                                                                                                          \
      hipLaunchKernelGGL((skinny_gemm_multi_kernel<P, E, 4, 2, 4>), grid, dim3(256), 0, stream, args);           \
  } while (0)
      if (pro == PRO_PLAIN && epi == EPI_STORE) RT_MT(PRO_PLAIN, EPI_STORE);
      else if (pro == PRO_NORM && epi == EPI_STORE) RT_MT(PRO_NORM, EPI_STORE);
      else if (pro == PRO_PLAIN && epi == EPI_RESID) RT_MT(PRO_PLAIN, EPI_RESID);
      else if (pro == PRO_NORM && epi == EPI_RESID) RT_MT(PRO_NORM, EPI_RESID);
      else if (pro == PRO_NORM && epi == EPI_SWIGLU) RT_MT(PRO_NORM, EPI_SWIGLU);
      else if (pro == PRO_PLAIN && epi == EPI_SWIGLU) RT_MT(PRO_PLAIN, EPI_SWIGLU);
      else if (pro == PRO_NORM && epi == EPI_ROPE) RT_MT(PRO_NORM, EPI_ROPE);
      else if (pro == PRO_PLAIN && epi == EPI_ROPE) RT_MT(PRO_PLAIN, EPI_ROPE);
      else return -2;
#undef RT_MT
      return hipGetLastError() == hipSuccess ? 0 : -6;
    }
  }
  // CU-balanced variant (split_mode bit 0): whole plain/norm tiles + split remainder (not for
  // NORM_ADD, whose workgroup 0 publishes the whole K row). ROPE finishes its pairs after the
  // hand-off (partner = adjacent lane's combined sum); the decode path does not use it for qkv:
  // Llama-3-8B qkv (384 tiles) measured 11.02 us plain vs 12.28 us balanced
  // (profiles/experiments/README_r02.md)
  if (split_ws != nullptr && (split_mode & 1) && pro != PRO_NORM_ADD && (K / 32) % 2 == 0 && K >= 64) {
    const int cus = device_cus();
    const int T = N / 16;
    const int R = cus > 0 ? T % cus : 0;
    if (cus > 0 && T > cus && R > 0 && R <= SPLIT_CTRS && split_ws_ints >= split_workspace_ints(R)) {
      GemmArgs args{(uint16_t*)out, (const uint16_t*)x, (const short8*)Ws, (uint16_t*)res, M, N, K, ldo,
                    eps, re, nullptr, nullptr};
      args.kmajor = forced_order();
      const dim3 grid(T + R);
      // the two halves of a remainder tile on one XCD (RT_BAL_XCD=0: adjacent block ids, r02)
      static const int bal_xpair = !(getenv("RT_BAL_XCD") && getenv("RT_BAL_XCD")[0] == '0');
      if (pro == PRO_NORM && epi == EPI_ROPE)
        hipLaunchKernelGGL((skinny_gemm_bal_kernel<PRO_NORM, EPI_ROPE, 4, 2>), grid, dim3(256), 0, stream, args,
                           split_ws, R, bal_xpair);
      else if (pro == PRO_PLAIN && epi == EPI_ROPE)
        hipLaunchKernelGGL((skinny_gemm_bal_kernel<PRO_PLAIN, EPI_ROPE, 4, 2>), grid, dim3(256), 0, stream, args,
                           split_ws, R, bal_xpair);
      else if (pro == PRO_NORM && epi == EPI_SWIGLU)
        hipLaunchKernelGGL((skinny_gemm_bal_kernel<PRO_NORM, EPI_SWIGLU, 4, 2>), grid, dim3(256), 0, stream, args,
                           split_ws, R, bal_xpair);
      else if (pro == PRO_PLAIN && epi == EPI_SWIGLU)
        hipLaunchKernelGGL((skinny_gemm_bal_kernel<PRO_PLAIN, EPI_SWIGLU, 4, 2>), grid, dim3(256), 0, stream, args,
                           split_ws, R, bal_xpair);
      else if (pro == PRO_NORM && epi == EPI_STORE)
        hipLaunchKernelGGL((skinny_gemm_bal_kernel<PRO_NORM, EPI_STORE, 4, 2>), grid, dim3(256), 0, stream, args,
                           split_ws, R, bal_xpair);
      else if (pro == PRO_PLAIN && epi == EPI_STORE)
        hipLaunchKernelGGL((skinny_gemm_bal_kernel<PRO_PLAIN, EPI_STORE, 4, 2>), grid, dim3(256), 0, stream, args,
                           split_ws, R, bal_xpair);
      else if (pro == PRO_PLAIN && epi == EPI_RESID)
        hipLaunchKernelGGL((skinny_gemm_bal_kernel<PRO_PLAIN, EPI_RESID, 4, 2>), grid, dim3(256), 0, stream, args,
                           split_ws, R, bal_xpair);
      else
        return -2;
      return 0;
    }
  }
  // Variant = (waves per workgroup NW, k-steps per stage U). Since the pipeline's waits are
  // counted (skinny_core.h gemm_tile), 4 waves win on every decode shape: U = 2 for the wide
  // GEMMs (>= 384 column tiles: qkv 11.5, gate_up 39.0 us), U = 4 for the 256-tile o / down
  // (8.05 / 20.9 us; U = 2 loses there) — profiles/r01_microbench_v3_cfg_sweep.log, v4, v5
  // (4x1, 2x2, 2x4 lose on every shape).
  // Before the counted waits the narrow projections needed 8 waves to keep bytes in flight.
  // RT_SKINNY_CFG=<NW>x<U> (4x2, 8x2, 4x4, 8x4, 8x8, 4x8) pins one for microbenchmarks.
  static const int cfg_env = [] {
    const char* e = getenv("RT_SKINNY_CFG");
    if (!e) return 0;
    int nw = 0, u = 0;
    if (sscanf(e, "%dx%d", &nw, &u) != 2) return 0;
    return nw * 100 + u;
  }();
  // 129-224 tiles of >= 64 KB (tensor-parallel shards: tp2 qkv 192 tiles) stream on most of the
  // CUs: 8 waves keep twice the bytes in flight per CU (tp2 qkv norm+rope 7.86 -> 7.34 us;
  // tools/probes/stream_probe.hip 192 x 128 KB 8x2 6.53 / 4x4 6.99 us). Fewer tiles (48-96) stay
  // at 4 x 4: 16 x 2 streams faster there in the probe (48 x 128 KB 5.32 vs 6.00 us) but loses in
  // the GEMM (tp8 qkv 6.74 -> 7.24 us: the 16-wave LDS reduction and epilogue).
  const int T16 = N / 16;
  int cfg_shape = T16 >= 384 ? 402 : 404;
  if (K >= 2048 && T16 > 128 && T16 <= 224) cfg_shape = 802;
  const int cfg = cfg_env ? cfg_env : cfg_shape;
  dim3 grid(N / 16);
  const bool alds = !cfg_env && use_alds(M, K, N / 16, device_cus());
  const size_t lds = alds ? (size_t)skinny::alds_bytes(M, K) : 0;
#define RT_SG(P, E)                                                                                          \
  do {                                                                                                       \
    switch (cfg) {                                                                                           \
      case 402: RT_SGV(P, E, 4, 2); break;                                                                   \
      case 1602: RT_SGV(P, E, 16, 2); break;                                                                 \
      case 802: RT_SGV(P, E, 8, 2); break;                                                                   \
      case 408: RT_SGV(P, E, 4, 8); break;                                                                   \
      case 804: RT_SGV(P, E, 8, 4); break;                                                                   \
      case 808: RT_SGV(P, E, 8, 8); break;                                                                   \
      default: RT_SGV(P, E, 4, 4); break;                                                                    \
    }                                                                                                        \
  } while (0)
  GemmArgs args{(uint16_t*)out, (const uint16_t*)x, (const short8*)Ws, (uint16_t*)res, M, N, K, ldo,
                eps, re, (const uint16_t*)x2, (uint16_t*)xo};
  args.kmajor = forced_order();
#define RT_SGV(P, E, NWV, UV)                                                                                  \
  do {                                                                                                         \
    if (alds)                                                                                                  \
      hipLaunchKernelGGL((skinny_gemm_alds_kernel<P, E, NWV, UV>), grid, dim3(NWV * 64), lds, stream, args);   \
    else                                                                                                       \
      hipLaunchKernelGGL((skinny_gemm_kernel<P, E, NWV, UV>), grid, dim3(NWV * 64), 0, stream, args);          \
  } while (0)
  if (pro == PRO_PLAIN && epi == EPI_STORE) RT_SG(PRO_PLAIN, EPI_STORE);
  else if (pro == PRO_NORM && epi == EPI_STORE) RT_SG(PRO_NORM, EPI_STORE);
  else if (pro == PRO_PLAIN && epi == EPI_RESID) RT_SG(PRO_PLAIN, EPI_RESID);
  else if (pro == PRO_NORM && epi == EPI_SWIGLU) RT_SG(PRO_NORM, EPI_SWIGLU);
  else if (pro == PRO_PLAIN && epi == EPI_SWIGLU) RT_SG(PRO_PLAIN, EPI_SWIGLU);
  else if (pro == PRO_NORM && epi == EPI_ROPE) RT_SG(PRO_NORM, EPI_ROPE);
  else if (pro == PRO_PLAIN && epi == EPI_ROPE) RT_SG(PRO_PLAIN, EPI_ROPE);
  else if (pro == PRO_NORM_ADD && epi == EPI_STORE) RT_SG(PRO_NORM_ADD, EPI_STORE);
  else if (pro == PRO_NORM_ADD && epi == EPI_SWIGLU) RT_SG(PRO_NORM_ADD, EPI_SWIGLU);
  else if (pro == PRO_NORM_ADD && epi == EPI_ROPE) RT_SG(PRO_NORM_ADD, EPI_ROPE);
  else return -2;
#undef RT_SG
#undef RT_SGV
  return 0;
}

int launch_shuffle_weight(void* Ws, const void* W, const void* gamma, int N, int K, int rope_rows, int D, int swiglu,
                          hipStream_t stream) {
  if (K % 32 || N % 16 || rope_rows > N || (rope_rows > 0 && (D <= 0 || D % 2 || rope_rows % D))) return -1;
  if (swiglu && (N % 32 || rope_rows > 0)) return -1;
  const int64_t total = (int64_t)N * K / 8;
  int64_t grid = (total + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(shuffle_kernel, dim3((unsigned)grid), dim3(256), 0, stream, (short8*)Ws, (const uint16_t*)W,
                     (const uint16_t*)gamma, N, K, rope_rows, D, swiglu, forced_order());
  return 0;
}

int launch_skinny_gemm_rope(void* q_out, const void* x, const void* Ws, int M, int K, int pro, float eps,
                            const int64_t* positions, const float* cos_sin, void* k_cache, void* v_cache,
                            const int64_t* slots, int Hq, int Hkv, int D, int BS, const void* x2, void* xo,
                            hipStream_t stream, int* split_ws, int64_t split_ws_ints, int split_mode,
                            const float* bias) {
  const RopeEpi re{positions, cos_sin, (uint16_t*)k_cache, (uint16_t*)v_cache, slots, Hq, Hkv, D, BS, bias};
  return launch_skinny_gemm(q_out, x, Ws, nullptr, M, (Hq + 2 * Hkv) * D, K, 0, eps, pro, EPI_ROPE, &re, x2, xo,
                            stream, split_ws, split_ws_ints, split_mode);
}
