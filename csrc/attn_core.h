// Device core of K3, paged-KV decode attention (one query token per sequence), GQA, MFMA bf16, split-KV.
//
// Grid (B * Hkv, num_splits), NW = 8 waves per workgroup. A workgroup owns one (sequence,
// kv head, key range); its G = Hq/Hkv query heads share every K/V byte it loads (GQA
// packing: the G queries are the 16 MFMA columns, G <= 16). The split count is chosen so the
// grid is ~one 8-wave workgroup per CU (ops.decode_splits): decode attention is a pure
// K/V stream, so what matters is bytes in flight per CU and few round trips per launch.
//
// Per 32-key tile (= one cache block, BS = 32) each wave computes
//   S^T[32 keys x 16 q] = K . Q^T     2 halves x D/32  mfma_f32_16x16x32_bf16
//   online softmax down each q column (in-register; 2 xor-shuffles per reduction)
//   O[16 q x D]        += P . V       D/16 mfma_f32_16x16x32_bf16
// K rows are fed to the MFMA in the order key(h, row) = 8*(row>>2) + 4h + (row&3), so lane
// (r, g) of the S^T accumulator holds keys 8g..8g+7 of column r — exactly the A-operand
// fragment of P.V (P never leaves registers) — and the matching B fragment of the
// transposed value cache ([D][32] per block) is ONE 16-byte load per lane per d-chunk.
// K blocks are chunk-major ([D/32][32 keys][32 dims]): each K load instruction reads 8 whole
// 128-B lines (d permuted consistently on K and Q).
// K/V go straight to VGPRs (cdna_hip_programming App. B "Attention decode") with the next
// tile's loads in flight while the current tile computes. The 8 waves' softmax states
// merge through LDS; the splits of one (sequence, kv head) are combined in the same launch
// by whichever workgroup arrives last (sc1 write-through hand-off, see below).
//
// Shared-prefix groups (the knights of one table share the discussion's KV blocks, see
// engine "shared" prompt layout): n consecutive sequences whose block tables start with the
// same `shared` blocks form a group. Their n*G query heads fill the MFMA columns together
// (3 knights x G=4 = 12 <= 16), so every shared K/V byte is read ONCE for the whole group.
// Work item of workgroup (b, kv head, split y), member index i = b - first:
//   virtual tiles = shared chunk (i*splits + y) of n*splits over [0, shared)   -> all columns
//                 + private split y of [shared, ctx_b) of sequence b            -> b's columns
// Each item leaves one partial (m, l, O) per column: member m collects n*splits partials
// (slot i*splits + y from every workgroup of the group) and the last arrival combines them.
#pragma once
#include "common.h"

namespace attn {
using rt::bf16x8;
using rt::float4_;
using rt::short8;

constexpr int BS = 32;
constexpr int NW = 8;
constexpr int MAXS = 64;  // max splits per (sequence, kv head)
constexpr float LOG2E = 1.4426950408889634f;

template <int D>
struct Tile {
  short8 k[2][D / 32];  // [half][chunk]: K row key(h, r), d = 32c + 8g + j (the same order of d for Q)
  short8 v[D / 16];     // [d-chunk]: V[keys 8g..8g+7][d = 16e + r]
};

// K/V load mode (LM bits, the round-6 stream study, attention_decode.hip): nontemporal loads
// (global_load ... nt, the cache policy of the weight streams) for the K tiles (LM_NTK) and the
// V tiles (LM_NTV). Right where every K/V byte is read once per launch (grouped launches, one row).
constexpr int LM_NTK = 1;
constexpr int LM_NTV = 2;
// LM_GLDS (A/B of VERDICT r5 #1b, RT_ATTN_LM=7): each wave stages its next K/V tile in a private
// 16-KB LDS slice by LDS-DMA (global_load_lds_dwordx4, lane-linear: lane l's 16 B of load i land
// at slice[i][l] and the same lane reads them back with ds_read_b128, so no swizzle and no bank
// conflict), then reads it into ONE register tile: 64 VGPRs less than the ping-pong pair, the
// same one tile in flight per wave during the math. The slices alias the merge buffers (a drain
// and a workgroup barrier separate the two uses).
constexpr int LM_GLDS = 4;

template <int D>
constexpr int tile_words() { return 2 * (D / 32) + D / 16; }   // 16-B loads per lane per tile

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <bool NT>
RT_DEVICE short8 ld16(const uint16_t* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const short8*>(p));
  else
    return *reinterpret_cast<const short8*>(p);
}

// One 32-key tile for lane (r, g). K blocks are chunk-major ([D/32][32 keys][32 dims], common.h
// kc_elem): the A fragment of half h, chunk c is key krow + 4h, dims 32c + 8g..+7, so one load
// instruction reads 16 keys x 64 B = 8 whole 128-B lines (4-key runs of 256 B). V blocks are
// [D][32 keys]: fragment e is dims 16e + r, keys 8g..8g+7, 1 KB contiguous per instruction.
// SC1: the block may hold K/V written earlier in the same launch (persistent kernel): sc1 loads.
template <int D, bool SC1, int LM = 0>
RT_DEVICE void load_tile(Tile<D>& t, const uint16_t* __restrict__ kblk, const uint16_t* __restrict__ vblk, int r,
                         int g) {
  const int krow = 8 * (r >> 2) + (r & 3);
  if constexpr (SC1) {
    const auto kr_ = rt::buf_rsrc(kblk), vr_ = rt::buf_rsrc(vblk);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int c = 0; c < D / 32; ++c)
        t.k[h][c] = __builtin_bit_cast(short8, rt::sc1_load4(kr_, 2 * (c * (BS * 32) + (krow + 4 * h) * 32 + 8 * g)));
#pragma unroll
    for (int e = 0; e < D / 16; ++e)
      t.v[e] = __builtin_bit_cast(short8, rt::sc1_load4(vr_, 2 * ((16 * e + r) * BS + 8 * g)));
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int c = 0; c < D / 32; ++c)
        t.k[h][c] = ld16<(LM & LM_NTK) != 0>(kblk + c * (BS * 32) + (krow + 4 * h) * 32 + 8 * g);
#pragma unroll
    for (int e = 0; e < D / 16; ++e) t.v[e] = ld16<(LM & LM_NTV) != 0>(vblk + (16 * e + r) * BS + 8 * g);
  }
}

struct AttnArgs {
  uint16_t* out;               // [B, Hq, D]
  const uint16_t* q;           // [B, Hq, D]
  const uint16_t* k_cache;     // [NB, Hkv, 32, D] bytes, each block chunk-major [D/32][32][32]
  const uint16_t* v_cache;     // [NB, Hkv, D, 32]
  const int* block_tables;     // [B, max_blocks]
  const int* ctx_lens;         // [B]
  float* part_o;               // [B, Hq, slot_stride, D]
  float* part_ml;              // [B, Hq, slot_stride, 4]
  int* counters;               // [B * Hkv], zero between launches
  int Hq, Hkv, max_blocks;
  float scale_log2;
  int num_splits;
  // shared-prefix groups, nullptr = every sequence on its own: per sequence {first sequence of
  // its group, group size n, shared full blocks}. n * G <= 16 (host-checked).
  const int* groups = nullptr;
  int slot_stride = 0;         // partial slots per (sequence, head) >= n * num_splits; 0 = num_splits
  int probe = 0;               // latency probe (microbench only, RT_ATTN_PROBE): stop after phase k
  int ext_combine = 0;         // 1: leave every partial for decode_combine_kernel (no in-launch combine)
  int xcd = 0;                 // 1: XCD-aware item order (attention_decode.hip), the launch's grid % 8 == 0
  int plain_partials = 0;      // 1 (ext_combine only): partials stay in the writer's L2 (plain stores)
  int lm = 0;                  // K/V load mode actually launched (LM_*), for the host's record
  // per-step work plan (attn_plan_kernel; nullptr = derive it in every launch): per item
  // (sequence, split), PLAN_HDR header ints then the item's block ids, plan_stride ints per item
  const int* plan = nullptr;
  int plan_stride = 0;
};

// The key range of work item (sequence b, split) — shared chunk of its group's prefix, then its
// private split — from the sequence's length and group record. attn_item derives it in every
// launch unless a per-step plan holds it (attn_plan_kernel, attention_decode.hip: computed once
// per decode step, read by every layer's launch in the same round trip as the block ids).
constexpr int PLAN_HDR = 8;
struct ItemRange {
  int b0, n, sh, ctx, sh_b, nsh, pr_b, nv;
};

RT_DEVICE ItemRange item_range(int ctx, int g0, int g1, int g2, bool grouped, int b, int split, int G, int GM,
                               int num_splits) {
  ItemRange it;
  const bool bad = !grouped | (g1 < 1) | (g1 * G > GM) | (g0 < 0) | (b < g0) | (b - g0 >= g1) | (g2 < 0);
  it.b0 = bad ? b : g0;   // no / malformed group record: run alone
  it.n = bad ? 1 : g1;
  it.sh = bad ? 0 : g2;
  it.ctx = ctx;
  const int mi = b - it.b0, nslots = it.n * num_splits, slot = mi * num_splits + split;
  const int ntiles = (ctx + BS - 1) / BS;
  // this workgroup's shared chunk (all members' columns) then its private split (own columns)
  const int sh_per = (it.sh + nslots - 1) / nslots;
  it.sh_b = min(it.sh, slot * sh_per);
  const int sh_e = min(it.sh, it.sh_b + sh_per);
  const int npr = max(0, ntiles - it.sh);
  const int pr_per = (npr + num_splits - 1) / num_splits;
  it.pr_b = it.sh + min(npr, split * pr_per);
  const int pr_e = it.sh + min(npr, split * pr_per + pr_per);
  it.nsh = sh_e - it.sh_b;
  it.nv = it.nsh + (pr_e - it.pr_b);
  return it;
}

// GM = max query columns the LDS is sized for (n * G <= GM). GM = 4 (Llama-3-8B, Mistral-7B,
// no groups) keeps the workgroup at ~26 KB so two fit a CU: 16 waves streaming K/V per CU.
template <int D, int GM = 16, int W = NW>
struct AttnSmem {
  float s_m[W][16];
  float s_l[W][16];
  float s_o[W][GM][D + 4];
  int s_last;                  // bit m: this workgroup combines member m
};

RT_DEVICE void store_bf16x4(uint16_t* dst, float a, float b_, float c, float d, bool sc1) {
  uint2 pk;
  pk.x = rt::pack2(a, b_);
  pk.y = rt::pack2(c, d);
  if (sc1)
    __hip_atomic_store(reinterpret_cast<uint64_t*>(dst), (uint64_t)pk.x | ((uint64_t)pk.y << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  else
    *reinterpret_cast<uint2*>(dst) = pk;
}

// One (sequence, kv head, key split) work item. Returns true when this workgroup wrote final
// output rows (no split, or the last-arriving split that combined them).
// W = waves per workgroup (8; 16 for grouped launches: twice the K/V in flight per CU and
// enough threads to combine a whole group's slots in one round trip).
// PP: ping-pong K/V tiles (two in flight per wave); false = the round-4 cur/nxt copy loop (A/B)
// LM: K/V load mode (LM_NTK / LM_NTV above)
template <int D, bool SC1, int GM = 16, int W = NW, bool PP = true, int LM = 0>
RT_DEVICE bool attn_item(const AttnArgs& P, int bh, int split, AttnSmem<D, GM, W>& S) {
  uint16_t* __restrict__ out = P.out;
  const uint16_t* __restrict__ q = P.q;
  const uint16_t* __restrict__ k_cache = P.k_cache;
  const uint16_t* __restrict__ v_cache = P.v_cache;
  const int* __restrict__ block_tables = P.block_tables;
  const int* __restrict__ ctx_lens = P.ctx_lens;
  float* __restrict__ part_o = P.part_o;
  float* __restrict__ part_ml = P.part_ml;
  int* __restrict__ counters = P.counters;
  const int Hq = P.Hq, Hkv = P.Hkv, max_blocks = P.max_blocks, num_splits = P.num_splits;
  const float scale_log2 = P.scale_log2;
  auto& s_m = S.s_m;
  auto& s_l = S.s_l;
  auto& s_o = S.s_o;
  int& s_last = S.s_last;

  const int b = bh / Hkv, hk = bh - (bh / Hkv) * Hkv;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int rseq = r / G, rhead = r - (r / G) * G;  // column r -> (member, head within the kv group)
  // reduction-dim order of the QK^T MFMAs: lane group g holds d = 32c + 8g.. of chunk c (the same
  // permutation of d for Q and K; it matches the chunk-major K block)
  const int kg = 8 * g, kc = 32;
  const bool grouped = P.groups != nullptr;
  ItemRange ir;
  // planned: the item's header and this wave's first 64 block ids are requested together, both
  // at addresses known at launch — one round trip ahead of the first K/V tile instead of two
  // (sequence record, then block table)
  const int* plan_ids = nullptr;
  const int maxt = P.plan_stride - PLAN_HDR;
  int blk_lane = 0;
  if (P.plan != nullptr) {
    const int* hdr = P.plan + (size_t)(b * num_splits + split) * P.plan_stride;
    plan_ids = hdr + PLAN_HDR;
    blk_lane = plan_ids[min(wid + W * lane, maxt - 1)];
    ir = ItemRange{hdr[0], hdr[1], hdr[2], hdr[3], hdr[4], hdr[5], hdr[6], hdr[7]};
  } else {
    // the sequence's length and its group record are requested together, before any test on
    // either (a short-circuit test made the compiler wait for one load before issuing the next:
    // two extra dependent trips ahead of the K/V stream)
    // branch-free: without groups the three record loads read ctx_lens[b] (valid, ignored)
    const int* gp = grouped ? P.groups + 3 * b : ctx_lens + b;
    const int go = grouped ? 1 : 0;
    ir = item_range(ctx_lens[b], gp[0], gp[go], gp[2 * go], grouped, b, split, G, GM, num_splits);
  }
  const int b0 = ir.b0, n = ir.n, ctx = ir.ctx;
  const int mi = b - b0, ncol = n * G;
  const int nslots = n * num_splits, slot = mi * num_splits + split;
  const int stride = P.slot_stride > 0 ? P.slot_stride : num_splits;

  if (P.probe == 1) {          // launch + metadata round trip only
    if (ctx == -12345) out[0] = 0;
    return false;
  }
  const int sh_b = ir.sh_b, pr_b = ir.pr_b, nsh = ir.nsh, nv = ir.nv;

  // Q^T fragments: column r = query head hk*G + rhead of member rseq (zero for r >= ncol)
  short8 qf[D / 32];
  {
    const bool live = r < ncol;
    const uint16_t* qr = q + ((size_t)(b0 + (live ? rseq : 0)) * Hq + hk * G + (live ? rhead : 0)) * D + kg;
#pragma unroll
    for (int c = 0; c < D / 32; ++c) {
      short8 v;
      if constexpr (SC1)   // uniform base + per-lane offset (a per-lane resource would waterfall)
        v = __builtin_bit_cast(short8, rt::sc1_load4(rt::buf_rsrc(q), (int)((qr - q) + kc * c) * 2));
      else
        v = *reinterpret_cast<const short8*>(qr + kc * c);
      if (!live) v = short8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[c] = v;
    }
  }

  float4_ oacc[D / 16];
#pragma unroll
  for (int e = 0; e < D / 16; ++e) oacc[e] = float4_{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY;  // running max (log2 domain) of column r
  float lsum = 0.f;     // lane-partial running sum of column r

  const size_t blk_stride = (size_t)Hkv * BS * D;
  // virtual tile v -> block-table entry: shared chunk tiles come from the group's first row
  auto bt_entry = [&](int v) -> int {
    return v < nsh ? block_tables[(size_t)b0 * max_blocks + sh_b + v]
                   : block_tables[(size_t)b * max_blocks + pr_b + (v - nsh)];
  };
  int v = wid;
  // Block ids of this wave's tiles (v = wid + W*j) are fetched one per lane (at j = 0, in flight
  // with Q, and refilled every 64 tiles, i.e. only past ~164K keys at 10 splits) and read out
  // with readlane: no dependent scalar load inside the loop. B=3, ctx 1500: 12.2 -> 11.2 us.
  // With a plan the j = 0 ids were requested with the item header (above).
  auto blk_of = [&](int tt) -> int {
    return tt < nv ? (plan_ids != nullptr && tt < maxt ? plan_ids[tt] : bt_entry(tt)) : 0;
  };
  // tile vn = wid + W*j into t (j: the wave's tile index, uniform)
  auto fetch = [&](Tile<D>& t, int vn, int j) {
    if ((j & 63) == 0 && !(j == 0 && plan_ids != nullptr && W * 64 <= maxt)) {
      const int tt = vn + W * lane;
      blk_lane = blk_of(tt);
    }
    const size_t base = (size_t)__builtin_amdgcn_readlane(blk_lane, j & 63) * blk_stride + (size_t)hk * BS * D;
    load_tile<D, SC1, LM>(t, k_cache + base, v_cache + base, r, g);
  };
  // one 32-key tile: S^T = K Q^T, online softmax down each column, O += P V
  auto step = [&](const Tile<D>& cur, int v) {
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
    // ---- online softmax down column r: lane holds keys 8g + 4h + i. Shared tiles are live
    // for every member's columns (full blocks); private tiles only for b's own, below ctx. ----
    const bool shared_t = v < nsh;
    const int t = shared_t ? sh_b + v : pr_b + (v - nsh);
    const int klim = shared_t ? (r < ncol ? 0x7fffffff : 0) : (rseq == mi && r < ncol ? ctx : 0);
    const int key0 = t * BS + 8 * g;
    float tmax = -INFINITY;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = s[h][i] * scale_log2;
        x = key0 + 4 * h + i < klim ? x : -INFINITY;
        s[h][i] = x;
        tmax = fmaxf(tmax, x);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float mref = mnew == -INFINITY ? 0.f : mnew;  // column with no live key yet: alpha = p = 0
    const float alpha = rt::fast_exp2(m - mref);         // m=-inf first time -> 0
    m = mnew;
    float psum = 0.f;
    rt::u32x4 pw;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float p0 = rt::fast_exp2(s[h][2 * i] - mref), p1 = rt::fast_exp2(s[h][2 * i + 1] - mref);
        psum += p0 + p1;
        pw[2 * h + i] = rt::pack2(p0, p1);
      }
    const short8 pa = __builtin_bit_cast(short8, pw);
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
      oacc[e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pa),
                                                        __builtin_bit_cast(bf16x8, cur.v[e]), o, 0, 0, 0);
    }
  };
  if constexpr ((LM & LM_GLDS) != 0 && !SC1) {
    short8* stg = reinterpret_cast<short8*>(&S) + (size_t)wid * tile_words<D>() * 64;
    const int krow = 8 * (r >> 2) + (r & 3);
    // tile vn (or, past the end, the wave's last tile again) -> the wave's LDS slice
    auto stage = [&](int vn, int j) {
      const bool past = vn >= nv;
      const int jj = past ? j - 1 : j;
      if (!past && (j & 63) == 0 && !(j == 0 && plan_ids != nullptr && W * 64 <= maxt)) blk_lane = blk_of(vn + W * lane);
      const size_t base = (size_t)__builtin_amdgcn_readlane(blk_lane, jj & 63) * blk_stride + (size_t)hk * BS * D;
      const uint16_t* kb = k_cache + base;
      const uint16_t* vb = v_cache + base;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // WAR: the slice's previous ds_reads are done
      int i = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < D / 32; ++c, ++i)
          __builtin_amdgcn_global_load_lds((glb_void*)(kb + c * (BS * 32) + (krow + 4 * h) * 32 + 8 * g),
                                           (lds_void*)(stg + i * 64), 16, 0, (LM & LM_NTK) ? 2 : 0);
#pragma unroll
      for (int e = 0; e < D / 16; ++e, ++i)
        __builtin_amdgcn_global_load_lds((glb_void*)(vb + (16 * e + r) * BS + 8 * g), (lds_void*)(stg + i * 64), 16, 0,
                                         (LM & LM_NTV) ? 2 : 0);
    };
    auto unstage = [&](Tile<D>& t) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the slice's LDS-DMA has landed
      int i = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < D / 32; ++c, ++i) t.k[h][c] = stg[i * 64 + lane];
#pragma unroll
      for (int e = 0; e < D / 16; ++e, ++i) t.v[e] = stg[i * 64 + lane];
    };
    Tile<D> t;
    if (v < nv) {
      stage(v, 0);
      int j = 1;
      while (true) {
        unstage(t);
        stage(v + W, j);        // unconditional (past the end: the same tile again), as PP
        step(t, v);
        v += W;
        ++j;
        if (v >= nv) break;
      }
    }
    // every wave's LDS-DMA drained before any wave writes the merge buffers over the slices
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else if constexpr (PP) {
    // Ping-pong over two named tiles, no `cur = nxt` copy, and the prefetch UNCONDITIONAL: with
    // the copy (and with a prefetch skipped past the range end) the compiler's wait counts had to
    // hold on every path, so each iteration waited for the NEXT tile's loads (vmcnt 15..0 before
    // the MFMAs) and a wave had one tile in flight — a full memory latency per tile. Here tile
    // j+1's 16 loads are always issued before tile j's math, which then waits with vmcnt(16):
    // two tiles (32 KB) in flight per wave. Past the end the prefetch re-reads the tile being
    // computed (an L2 hit, once per wave).
    auto prefetch = [&](Tile<D>& t, int vn, int j) {
      const bool past = vn >= nv;
      const int jj = past ? j - 1 : j;
      if (!past && (j & 63) == 0) {
        const int tt = vn + W * lane;
        blk_lane = blk_of(tt);
      }
      const size_t base = (size_t)__builtin_amdgcn_readlane(blk_lane, jj & 63) * blk_stride + (size_t)hk * BS * D;
      load_tile<D, SC1, LM>(t, k_cache + base, v_cache + base, r, g);
    };
    Tile<D> ta, tb;
    if (v < nv) {
      fetch(ta, v, 0);
      int j = 1;
      while (true) {
        prefetch(tb, v + W, j);
        step(ta, v);
        v += W;
        ++j;
        if (v >= nv) break;
        prefetch(ta, v + W, j);
        step(tb, v);
        v += W;
        ++j;
        if (v >= nv) break;
      }
    }
  } else {
    Tile<D> cur, nxt;
    if (v < nv) fetch(cur, v, 0);
    for (int j = 1; v < nv; v += W, ++j) {
      const int vn = v + W;
      if (vn < nv) fetch(nxt, vn, j);  // keep the next tile's loads in flight during this tile's math
      step(cur, v);
      cur = nxt;
    }
  }
  if (P.probe == 2) {          // + block ids, Q, every K/V tile and the math
    if (m == 12345.f && lsum == 1.f) out[0] = (uint16_t)oacc[0][0];
    return false;
  }
  // column-complete partial sum for q = r
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);

  // ---- merge the waves through LDS (only the ncol live query columns) ----
  if (g == 0) {
    s_m[wid][r] = m;
    s_l[wid][r] = lsum;
  }
#pragma unroll
  for (int e = 0; e < D / 16; ++e)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * g + i < ncol) s_o[wid][4 * g + i][16 * e + r] = oacc[e][i];
  __syncthreads();

  // (sequence, head) row of column c relative to the group's first row q0
  const size_t q0 = (size_t)b0 * Hq + hk * G;
  auto col_row = [&](int c) -> int { return (c / G) * Hq + (c - (c / G) * G); };
  const auto po_rsrc = rt::buf_rsrc(part_o + q0 * stride * D);
  const auto pml_rsrc = rt::buf_rsrc(part_ml + q0 * stride * 4);
  for (int it = threadIdx.x; it < ncol * (D / 4); it += blockDim.x) {
    const int qi = it / (D / 4), d0 = 4 * (it - qi * (D / 4));
    const int row = col_row(qi);
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; ++w) M = fmaxf(M, s_m[w][qi]);
    float L = 0.f;
    float4_ O = {0.f, 0.f, 0.f, 0.f};
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const float f = exp2f(s_m[w][qi] - M);
        L += f * s_l[w][qi];
        const float4_ ow = *reinterpret_cast<const float4_*>(&s_o[w][qi][d0]);
        O += f * ow;
      }
    }
    if (nslots == 1) {
      const float inv = L > 0.f ? 1.f / L : 0.f;
      store_bf16x4(out + (q0 + row) * D + d0, O[0] * inv, O[1] * inv, O[2] * inv, O[3] * inv, SC1);
    } else {
      if (P.plain_partials) {
        // read by the NEXT launch only (decode_combine_kernel): the kernel boundary orders them,
        // and plain stores keep the lines in this XCD's L2, where an XCD-aware combine reads them
        const size_t e = ((q0 + row) * stride + slot);
        *reinterpret_cast<float4_*>(part_o + e * D + d0) = O;
        if (d0 == 0) *reinterpret_cast<float4_*>(part_ml + e * 4) = float4_{M, L, 0.f, 0.f};
      } else {
        // partials leave as 16-B write-through (sc1) stores: the combining workgroup, possibly
        // on another XCD, reads them with sc1 loads and no L2 writeback/invalidate is needed
        rt::sc1_store4(po_rsrc, ((row * stride + slot) * D + d0) * 4, O);
        if (d0 == 0) rt::sc1_store4(pml_rsrc, (row * stride + slot) * 16, float4_{M, L, 0.f, 0.f});
      }
    }
  }
  if (nslots == 1) {
    __syncthreads();  // LDS is reused by the caller's next item
    return true;
  }
  if (P.ext_combine) {  // many slots: a separate, CU-parallel combine launch reads the partials
    __syncthreads();
    return false;
  }

  // ---- split-KV combine inside the launch (MI355X_MICROARCH "Valid forms", row 1): every
  // partial is stored sc1 and drained (vmcnt(0)) by each storing wave before the barrier;
  // one lane per member then bumps that member's (sequence, kv head) arrival counter; the
  // workgroup whose add returns nslots-1 combines the member, reading every partial with sc1
  // loads, and re-arms the counter for the next launch (hipGraph replays need no memset node).
  // A release/acquire fence pair instead would write back / invalidate caches per workgroup
  // (measured 2x slower).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) s_last = 0;
  __syncthreads();
  if ((int)threadIdx.x < n) {
    int* ctr = counters + (size_t)(b0 + threadIdx.x) * Hkv + hk;
    const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == nslots - 1) {
      __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicOr(&s_last, 1 << threadIdx.x);
    }
  }
  __syncthreads();
  const int mask = s_last;
  if (P.probe == 3) return false;   // + wave merge, partial stores, drain, arrival atomics
  if (mask == 0) return false;

  // One thread per output element (member head row, 4 dims); the RL = D/4 threads of a row are
  // consecutive lanes. Per chunk of RL slots each lane loads ONE slot's (m, l) (shared with the
  // row's other lanes by shuffles, not re-loaded by each) and its 4 dims of all RL partial O's.
  // The rows of the members being combined use nitems = nm * G * RL threads; the workgroup's
  // other threads are not idle: Q = blockDim / nitems thread groups take interleaved slot chunks
  // (chunk c -> group c % Q) and merge their (m, l, O) states through LDS, so a member with many
  // slots (small KV-head shards of a tensor-parallel knight: 3 knights x 64 splits = 192 slots)
  // needs ceil(nslots / (Q * RL)) dependent round trips instead of ceil(nslots / RL).
  constexpr int RL = D / 4;
  constexpr int SCR = W * GM * (D + 4);   // floats of s_o, reused as the merge scratch
  const int per_m = G * RL;
  const int nm = __popc(mask);
  const int nitems = nm * per_m;          // <= ncol * RL <= blockDim
  int Q = (int)blockDim.x / nitems;
  if (Q > 1 + SCR / (6 * nitems)) Q = 1 + SCR / (6 * nitems);
  Q = Q < 1 ? 1 : (1 << (31 - __clz(Q)));
  const int grp = threadIdx.x / nitems;
  const int it = threadIdx.x - grp * nitems;
  const int lr = threadIdx.x & (RL - 1);
  const int lane0 = (threadIdx.x & 63) & ~(RL - 1);
  float4_ O = {0.f, 0.f, 0.f, 0.f};
  float Mr = -INFINITY, Lr = 0.f;
  int row = 0, d0 = 0;
  if (grp < Q) {
    const int k = it / per_m;
    int mm = 0;
    for (int bits = mask, c = 0;; bits &= bits - 1) {   // k-th member set in the mask
      mm = __ffs(bits) - 1;
      if (c++ == k) break;
    }
    const int w = it - k * per_m;
    const int hj = w / RL;
    d0 = 4 * (w - hj * RL);
    row = mm * Hq + hj;
    for (int s0 = grp * RL; s0 < nslots; s0 += Q * RL) {
      const bool mine = s0 + lr < nslots;
      const float4_ mlq = mine ? rt::sc1_load4(pml_rsrc, (row * stride + s0 + lr) * 16)
                               : float4_{-INFINITY, 0.f, 0.f, 0.f};
      float4_ vv[RL];
#pragma unroll
      for (int j = 0; j < RL; ++j)
        vv[j] = s0 + j < nslots ? rt::sc1_load4(po_rsrc, ((row * stride + s0 + j) * D + d0) * 4)
                                : float4_{0.f, 0.f, 0.f, 0.f};
      float mc = mlq[1] > 0.f ? mlq[0] : -INFINITY;
#pragma unroll
      for (int x = 1; x < RL; x <<= 1) mc = fmaxf(mc, __shfl_xor(mc, x, 64));
      const float Mc = fmaxf(Mr, mc);
      if (Mc == -INFINITY) continue;                 // every slot of this chunk was empty
      const float a = Mr == -INFINITY ? 0.f : exp2f(Mr - Mc);
      O *= a;
      Lr *= a;
#pragma unroll
      for (int j = 0; j < RL; ++j) {
        const float mj = __shfl(mlq[0], lane0 + j, 64), lj = __shfl(mlq[1], lane0 + j, 64);
        if (lj > 0.f) {
          const float f = exp2f(mj - Mc);
          O += f * vv[j];
          Lr += f * lj;
        }
      }
      Mr = Mc;
    }
  }
  if (Q > 1) {   // merge the Q groups' states in group order (deterministic), group 0 stores
    float* scr = &S.s_o[0][0][0];
    __syncthreads();
    if (grp >= 1 && grp < Q) {
      float* e = scr + ((grp - 1) * nitems + it) * 6;
      e[0] = O[0]; e[1] = O[1]; e[2] = O[2]; e[3] = O[3]; e[4] = Mr; e[5] = Lr;
    }
    __syncthreads();
    if (grp == 0) {
      for (int q2 = 1; q2 < Q; ++q2) {
        const float* e = scr + ((q2 - 1) * nitems + it) * 6;
        const float Me = e[4];
        if (Me == -INFINITY || e[5] <= 0.f) continue;
        const float Mc = fmaxf(Mr, Me);
        const float a = Mr == -INFINITY ? 0.f : exp2f(Mr - Mc), f = exp2f(Me - Mc);
        O = O * a + f * float4_{e[0], e[1], e[2], e[3]};
        Lr = Lr * a + f * e[5];
        Mr = Mc;
      }
    }
  }
  if (grp == 0) {
    const float inv = Lr > 0.f ? 1.f / Lr : 0.f;
    store_bf16x4(out + (q0 + row) * D + d0, O[0] * inv, O[1] * inv, O[2] * inv, O[3] * inv, SC1);
  }
  __syncthreads();
  return true;
}
}  // namespace attn
