// K3: paged-KV decode attention (one query token per sequence), GQA, MFMA bf16, split-KV.
//
// Grid (B * Hkv, num_splits), 256 threads = 4 waves. A workgroup owns one (sequence, kv
// head, key range); its G = Hq/Hkv query heads share every K/V byte it loads (GQA
// packing: the G queries are the 16 MFMA columns, G <= 16).
//
// Per 32-key tile (= one cache block, BS = 32) each wave computes
//   S^T[32 keys x 16 q] = K . Q^T     4*(D/32)... 2 halves x D/32  mfma_f32_16x16x32_bf16
//   online softmax down each q column (in-register; 2 xor-shuffles per reduction)
//   O[16 q x D]        += P . V       D/16 mfma_f32_16x16x32_bf16
// The S^T accumulator of lane l already IS the A-operand fragment of P.V (keys permuted
// consistently on both operands), so P never leaves registers. K rows are read as
// 64 contiguous bytes per lane (d permuted consistently on K and Q); V is cached
// transposed per block ([D][32]) so its B-fragments are two 8-byte contiguous loads.
// Decode is HBM-bound: K/V go straight to VGPRs (cdna_hip_programming App. B "Attention
// decode") with the next tile's loads in flight while the current tile computes;
// LDS is used to merge the 4 waves' partial softmax states. Long contexts split the key
// range over workgroups; the last split to finish merges them (no second launch).
#include "common.h"

namespace {
using rt::bf16x8;
using rt::float4_;
using rt::short8;

constexpr int BS = 32;
constexpr int NW = 4;
constexpr float LOG2E = 1.4426950408889634f;

template <int D>
struct Tile {
  short8 k[2][D / 32];              // [half][chunk]: K rows 16h + r, d = (D/4)*g + 8c + j
  uint2 v[D / 16][2];               // [d-chunk][key group]: 4 keys each
};

template <int D>
RT_DEVICE void load_tile(Tile<D>& t, const uint16_t* __restrict__ kblk, const uint16_t* __restrict__ vblk, int r,
                         int g) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint16_t* kr = kblk + (16 * h + r) * D + (D / 4) * g;
#pragma unroll
    for (int c = 0; c < D / 32; ++c) t.k[h][c] = *reinterpret_cast<const short8*>(kr + 8 * c);
  }
#pragma unroll
  for (int e = 0; e < D / 16; ++e) {
    const uint16_t* vr = vblk + (16 * e + r) * BS;
    t.v[e][0] = *reinterpret_cast<const uint2*>(vr + 4 * g);
    t.v[e][1] = *reinterpret_cast<const uint2*>(vr + 16 + 4 * g);
  }
}

template <int D>
__global__ void __launch_bounds__(256) paged_decode_kernel(
    uint16_t* __restrict__ out, const uint16_t* __restrict__ q, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, const int* __restrict__ ctx_lens,
    float* __restrict__ part_o, float* __restrict__ part_ml, int* __restrict__ counters, int Hq, int Hkv,
    int max_blocks, float scale_log2, int num_splits) {
  __shared__ float s_m[NW][16];
  __shared__ float s_l[NW][16];
  __shared__ float s_o[NW][16][D + 4];

  const int bh = blockIdx.x;
  const int b = bh / Hkv, hk = bh - (bh / Hkv) * Hkv;
  const int split = blockIdx.y;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;

  const int ctx = ctx_lens[b];
  const int ntiles = (ctx + BS - 1) / BS;
  const int tps = (ntiles + num_splits - 1) / num_splits;
  const int t_begin = split * tps;
  const int t_end = min(ntiles, t_begin + tps);

  // Q^T fragments: column r = query head hk*G + r (zero for r >= G)
  short8 qf[D / 32];
  {
    const uint16_t* qr = q + ((size_t)b * Hq + hk * G + (r < G ? r : 0)) * D + (D / 4) * g;
#pragma unroll
    for (int c = 0; c < D / 32; ++c) {
      short8 v = *reinterpret_cast<const short8*>(qr + 8 * c);
      if (r >= G) v = short8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[c] = v;
    }
  }

  float4_ oacc[D / 16];
#pragma unroll
  for (int e = 0; e < D / 16; ++e) oacc[e] = float4_{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY;   // running max (log2 domain) of column r
  float lsum = 0.f;      // lane-partial running sum of column r

  const int* bt = block_tables + (size_t)b * max_blocks;
  const size_t blk_stride = (size_t)Hkv * BS * D;
  Tile<D> cur, nxt;
  int t = t_begin + wid;
  if (t < t_end) {
    const size_t base = (size_t)bt[t] * blk_stride + (size_t)hk * BS * D;
    load_tile<D>(cur, k_cache + base, v_cache + base, r, g);
  }
  for (; t < t_end; t += NW) {
    const int tn = t + NW;
    if (tn < t_end) {  // keep the next tile's loads in flight during this tile's math
      const size_t base = (size_t)bt[tn] * blk_stride + (size_t)hk * BS * D;
      load_tile<D>(nxt, k_cache + base, v_cache + base, r, g);
    }
    // ---- S^T = K Q^T ----
    float4_ s[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      s[h] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < D / 32; ++c)
        s[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, cur.k[h][c]),
                                                       __builtin_bit_cast(bf16x8, qf[c]), s[h], 0, 0, 0);
    }
    // ---- online softmax down column r ----
    const int key0 = t * BS;
    float tmax = -INFINITY;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = key0 + 16 * h + 4 * g + i;
        float v = s[h][i] * scale_log2;
        v = key < ctx ? v : -INFINITY;
        s[h][i] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = exp2f(m - mnew);  // m=-inf first time -> 0
    m = mnew;
    float psum = 0.f;
    short8 pa;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(s[h][i] - mnew);
        psum += p;
        pa[4 * h + i] = (short)rt::f2bf(p);
      }
    lsum = lsum * alpha + psum;
    // rows of O held by this lane are q = 4g + i: fetch their alphas from lanes 4g + i
    float al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) al[i] = __shfl(alpha, 4 * g + i, 64);
    // ---- O += P V ----
#pragma unroll
    for (int e = 0; e < D / 16; ++e) {
      float4_ o = oacc[e];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] *= al[i];
      uint4 vb;
      vb.x = cur.v[e][0].x;
      vb.y = cur.v[e][0].y;
      vb.z = cur.v[e][1].x;
      vb.w = cur.v[e][1].y;
      oacc[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pa),
                                                        __builtin_bit_cast(bf16x8, vb), o, 0, 0, 0);
    }
    cur = nxt;
  }
  // column-complete partial sum for q = r
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);

  // ---- merge the 4 waves through LDS ----
  if (g == 0) {
    s_m[wid][r] = m;
    s_l[wid][r] = lsum;
  }
#pragma unroll
  for (int e = 0; e < D / 16; ++e)
#pragma unroll
    for (int i = 0; i < 4; ++i) s_o[wid][4 * g + i][16 * e + r] = oacc[e][i];
  __syncthreads();

  // G x D outputs, 256 threads
  for (int idx = threadIdx.x; idx < G * D; idx += blockDim.x) {
    const int qi = idx / D, d = idx - qi * D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, s_m[w][qi]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float f = exp2f(s_m[w][qi] - M);
        L += f * s_l[w][qi];
        O += f * s_o[w][qi][d];
      }
    }
    const int head = hk * G + qi;
    if (num_splits == 1) {
      out[((size_t)b * Hq + head) * D + d] = rt::f2bf(L > 0.f ? O / L : 0.f);
    } else {
      // agent-scope relaxed atomic stores = write-through past this XCD's L2 (sc1), so the
      // combining workgroup, possibly on another XCD, reads them without any L2 writeback
      const size_t pi = ((size_t)b * Hq + head) * num_splits + split;
      __hip_atomic_store(part_o + pi * D + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(part_ml + pi * 2, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part_ml + pi * 2 + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (num_splits == 1) return;
  // ---- split-KV combine inside the launch: the last-arriving split of (b, hk) merges all
  // splits and re-arms the counter to 0 for the next launch (hipGraph replays need no memset
  // node). Protocol: every partial is an agent-scope atomic (sc1) store, each thread drains
  // its stores (vmcnt(0)) before the barrier, then one lane bumps the arrival counter; the
  // last arriver reads the partials with agent-scope atomic (sc1, L2-bypassing) loads.
  // A release/acquire fence pair would emit buffer_wbl2/buffer_inv of the whole L2 per
  // workgroup (measured: 2x slower kernel), which this avoids.
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(counters + bh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == num_splits - 1;
    if (s_last) __hip_atomic_store(counters + bh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  // Combine. Latency-bound (a few KB of L2-bypassing loads), so every load is issued
  // before any is consumed: (m, l) of all (head, split) pairs by distinct threads, then
  // per-split weights through LDS, then 8 independent part_o loads in flight per thread.
  auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  constexpr int MAXS = 64;
  __shared__ float s_w[16][MAXS];   // per (head, split) weight exp2(m_s - M) / L
  const size_t bh_q0 = (size_t)b * Hq + hk * G;
  for (int i = threadIdx.x; i < G * num_splits; i += blockDim.x) {
    const int qi = i / num_splits, s2 = i - qi * num_splits;
    const float* ml = part_ml + ((bh_q0 + qi) * num_splits + s2) * 2;
    const float m = ld(ml), l = ld(ml + 1);
    s_w[qi][s2] = l > 0.f ? m : -INFINITY;
    s_o[0][qi][s2] = l;  // reuse the (now idle) merge buffer for l
  }
  __syncthreads();
  if (threadIdx.x < G) {
    const int qi = threadIdx.x;
    float M = -INFINITY;
    for (int s2 = 0; s2 < num_splits; ++s2) M = fmaxf(M, s_w[qi][s2]);
    float L = 0.f;
    for (int s2 = 0; s2 < num_splits; ++s2) {
      const float f = (M == -INFINITY || s_w[qi][s2] == -INFINITY) ? 0.f : exp2f(s_w[qi][s2] - M);
      s_w[qi][s2] = f;
      L += f * s_o[0][qi][s2];
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    for (int s2 = 0; s2 < num_splits; ++s2) s_w[qi][s2] *= inv;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < G * D; idx += blockDim.x) {
    const int qi = idx / D, d = idx - qi * D;
    const float* po = part_o + (bh_q0 + qi) * num_splits * D + d;
    float O = 0.f;
    for (int s0 = 0; s0 < num_splits; s0 += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (s0 + j < num_splits) ? ld(po + (size_t)(s0 + j) * D) : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (s0 + j < num_splits) O = fmaf(s_w[qi][s0 + j], v[j], O);
    }
    out[(bh_q0 + qi) * D + d] = rt::f2bf(O);
  }
}

}  // namespace

// q [B, Hq, D]; k_cache [NB, Hkv, 32, D]; v_cache [NB, Hkv, D, 32]; block_tables [B, max_blocks] int32.
int launch_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                        const int* ctx_lens, float* part_o, float* part_ml, int* counters, int B, int Hq, int Hkv,
                        int D, int max_blocks, float scale, int num_splits, hipStream_t stream) {
  if (B == 0) return 0;
  if (Hq % Hkv || Hq / Hkv > 16) return -1;
  if (num_splits < 1) num_splits = 1;
  if (num_splits > 64 || (num_splits > 1 && num_splits > D + 4)) return -3;  // combine staging limits
  dim3 grid(B * Hkv, num_splits), block(256);
  const float sl2 = scale * LOG2E;
#define RT_DEC(DD)                                                                                               \
  hipLaunchKernelGGL((paged_decode_kernel<DD>), grid, block, 0, stream, (uint16_t*)out, (const uint16_t*)q,      \
                     (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, ctx_lens, part_o, part_ml, \
                     counters, Hq, Hkv, max_blocks, sl2, num_splits);
  if (D == 128) {
    RT_DEC(128)
  } else if (D == 64) {
    RT_DEC(64)
  } else {
    return -2;
  }
#undef RT_DEC
  return 0;
}
