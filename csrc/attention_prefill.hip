// K4: varlen causal prefill attention over the paged KV cache (flash-style, MFMA bf16).
//
// Sequence s contributes queries q[cu_q[s] : cu_q[s+1]] at absolute positions
// start_pos[s] + i; they attend to cached keys [0, pos] (the resident prefix plus the
// chunk itself, already written by K2). This is the "delta prefill" of a knight turn.
//
// Grid (n_tiles, Hkv): a workgroup = one tile of query rows (host work list
// `tile_map` = (sequence, first row)) x one kv head; its 4 waves cover the G query
// heads of that kv head (GQA: one K/V tile load feeds all G heads):
//   G<=4: wave w -> head w%G, 16-row group w/G  (tile = 16*(4/G) rows)
//   G> 4: every wave 16 rows x HPW = ceil(G/4) heads (tile = 16 rows); a group that is not a
//         multiple of 4 (Qwen2.5: G = 7) leaves the last wave's surplus head slots idle
// K/V 32-key tiles are register-staged into LDS, double-buffered with one barrier per
// tile (async-STAGE split, cdna_hip_programming T14: the next tile's global loads are in
// flight during this tile's MFMAs). K rows are XOR-swizzled in 16-byte chunks and each
// lane's d-chunks are interleaved (chunk 4c+g) so the ds_read_b128 A-fragment reads are
// conflict-free; the transposed V tile uses 80-byte rows so the two ds_read_b64
// B-fragment reads per d-chunk are conflict-free. S^T = K.Q^T keeps P in the A-operand
// layout of P.V (no LDS round trip for P), as in the decode kernel.
#include "common.h"

#include <cstdlib>

namespace {
using rt::bf16x8;
using rt::float4_;
using rt::short8;

constexpr int BS = 32;
constexpr float LOG2E = 1.4426950408889634f;

template <int D>
struct PrefillCfg {
  static constexpr int NCH = D / 8;               // 16-byte chunks per K row
  static constexpr int KROW = D * 2;              // K tile row bytes
  static constexpr int VROW = BS * 2 + 16;        // V tile row bytes (64 + 16 pad)
  static constexpr int KBYTES = BS * KROW;
  static constexpr int VBYTES = D * VROW;
  static constexpr int STAGE = KBYTES + VBYTES;
  static constexpr int KLD = (BS * D * 2) / (256 * 16);  // 16-byte K loads per thread per tile
  static constexpr int VLD = (D * BS * 2) / (256 * 16);
};

template <int D, int HPW>
__global__ void __launch_bounds__(256) prefill_kernel(
    uint16_t* __restrict__ out, const uint16_t* __restrict__ q, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, const int* __restrict__ cu_q,
    const int* __restrict__ start_pos, const int* __restrict__ tile_map, int Hq, int Hkv, int max_blocks,
    float scale_log2, int rows_per_tile) {
  using C = PrefillCfg<D>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tile = blockIdx.x, hk = blockIdx.y;
  const int s = tile_map[2 * tile], row0 = tile_map[2 * tile + 1];
  const int q_begin = cu_q[s], q_end = cu_q[s + 1];
  const int sp = start_pos[s];
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;

  // wave -> (heads, rows)
  int head0, wrow0;
  if (HPW == 1) {
    const int Gw = G;  // G in {1,2,4}
    head0 = hk * G + (wid % Gw);
    wrow0 = row0 + 16 * (wid / Gw);
  } else {
    head0 = hk * G + wid * HPW;
    wrow0 = row0;
  }
  const int tile_rows_end = min(row0 + rows_per_tile, q_end);
  const int kmax = sp + (tile_rows_end - q_begin);  // keys [0, kmax)
  const int ntiles = (kmax + BS - 1) / BS;

  // this lane's query row (MFMA column r)
  const int my_row = wrow0 + r;
  const int my_row_c = min(my_row, q_end - 1);
  const int my_pos = sp + (my_row_c - q_begin);

  short8 qf[HPW][D / 32];
#pragma unroll
  for (int hh = 0; hh < HPW; ++hh) {
    // surplus head slot (HPW * 4 > G): read a valid head, never store it
    const int hq_ = min(head0 + hh, hk * G + G - 1);
    const uint16_t* qr = q + ((size_t)my_row_c * Hq + hq_) * D;
#pragma unroll
    for (int c = 0; c < D / 32; ++c) qf[hh][c] = *reinterpret_cast<const short8*>(qr + 8 * (4 * c + g));
  }
  float4_ oacc[HPW][D / 16];
  float m[HPW], lsum[HPW];
#pragma unroll
  for (int hh = 0; hh < HPW; ++hh) {
    m[hh] = -INFINITY;
    lsum[hh] = 0.f;
#pragma unroll
    for (int e = 0; e < D / 16; ++e) oacc[hh][e] = float4_{0.f, 0.f, 0.f, 0.f};
  }

  const int* bt = block_tables + (size_t)s * max_blocks;
  const size_t blk_stride = (size_t)Hkv * BS * D;
  const int tid = threadIdx.x;
  uint4 kreg[C::KLD], vreg[C::VLD];

  auto gload = [&](int t) {
    const size_t base = (size_t)bt[t] * blk_stride + (size_t)hk * BS * D;
    const uint4* kg = reinterpret_cast<const uint4*>(k_cache + base);
    const uint4* vg = reinterpret_cast<const uint4*>(v_cache + base);
#pragma unroll
    for (int i = 0; i < C::KLD; ++i) kreg[i] = kg[tid * C::KLD + i];
#pragma unroll
    for (int i = 0; i < C::VLD; ++i) vreg[i] = vg[tid * C::VLD + i];
  };
  auto lwrite = [&](int buf) {
    unsigned char* kb = smem + buf * C::STAGE;
    unsigned char* vb = kb + C::KBYTES;
#pragma unroll
    for (int i = 0; i < C::KLD; ++i) {
      const int ch = tid * C::KLD + i;  // 16-byte chunk of the chunk-major K block (common.h kc_chunk)
      int row, c;
      rt::kc_chunk(ch, BS, row, c);
      *reinterpret_cast<uint4*>(kb + row * C::KROW + 16 * (c ^ (row & (C::NCH - 1)))) = kreg[i];
    }
#pragma unroll
    for (int i = 0; i < C::VLD; ++i) {
      const int ch = tid * C::VLD + i;  // 4 chunks (64 B) per V row
      const int row = ch >> 2, c = ch & 3;
      *reinterpret_cast<uint4*>(vb + row * C::VROW + 16 * c) = vreg[i];
    }
  };

  if (ntiles > 0) {
    gload(0);
    lwrite(0);
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) gload(t + 1);
    const unsigned char* kb = smem + buf * C::STAGE;
    const unsigned char* vb = kb + C::KBYTES;
    // K A-fragments: rows 16h + r, chunks 4c + g (swizzled)
    short8 kf[2][D / 32];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 16 * h + r;
#pragma unroll
      for (int c = 0; c < D / 32; ++c)
        kf[h][c] = *reinterpret_cast<const short8*>(kb + row * C::KROW + 16 * ((4 * c + g) ^ (row & (C::NCH - 1))));
    }
    const int key0 = t * BS;
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) {
      float4_ sc[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        sc[h] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < D / 32; ++c)
          sc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf[h][c]),
                                                          __builtin_bit_cast(bf16x8, qf[hh][c]), sc[h], 0, 0, 0);
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = key0 + 16 * h + 4 * g + i;
          float v = sc[h][i] * scale_log2;
          v = (key <= my_pos) ? v : -INFINITY;
          sc[h][i] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mnew = fmaxf(m[hh], tmax);
      const float alpha = (mnew == -INFINITY) ? 1.f : rt::fast_exp2(m[hh] - mnew);
      m[hh] = mnew;
      float psum = 0.f;
      short8 pa;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = (mnew == -INFINITY) ? 0.f : rt::fast_exp2(sc[h][i] - mnew);
          psum += p;
          pa[4 * h + i] = (short)rt::f2bf(p);
        }
      lsum[hh] = lsum[hh] * alpha + psum;
      float al[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) al[i] = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
      for (int e = 0; e < D / 16; ++e) {
        const unsigned char* vr = vb + (16 * e + r) * C::VROW;
        const uint2 lo = *reinterpret_cast<const uint2*>(vr + 8 * g);
        const uint2 hi = *reinterpret_cast<const uint2*>(vr + 32 + 8 * g);
        uint4 vv;
        vv.x = lo.x;
        vv.y = lo.y;
        vv.z = hi.x;
        vv.w = hi.y;
        float4_ o = oacc[hh][e];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] *= al[i];
        oacc[hh][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, pa),
                                                              __builtin_bit_cast(bf16x8, vv), o, 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) lwrite(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds O[row 4g+i][d 16e+r]; normalize by the row's l (held by lane 4g+i)
#pragma unroll
  for (int hh = 0; hh < HPW; ++hh) {
    float l = lsum[hh];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float li = __shfl(l, 4 * g + i, 64);
      const int row = wrow0 + 4 * g + i;
      if (row < q_end && row < row0 + rows_per_tile && head0 + hh < hk * G + G) {
        uint16_t* orow = out + ((size_t)row * Hq + head0 + hh) * D;
        const float inv = li > 0.f ? 1.f / li : 0.f;
#pragma unroll
        for (int e = 0; e < D / 16; ++e) orow[16 * e + r] = rt::f2bf(oacc[hh][e][i] * inv);
      }
    }
  }
}
}  // namespace

int prefill32_rows(int G);
int launch_prefill32(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                     const int* cu_q, const int* start_pos, const int* tile_map, int n_tiles, int Hq, int Hkv,
                     int max_blocks, float scale, hipStream_t stream, int map_stride, const int* cmap, int n_split,
                     float* part_o, float* part_ml);

// D = 128 with G <= 8 (a non-power-of-two group in the next power of two of head slots) runs the
// 32x32-MFMA kernel (attention_prefill32.hip) unless
// ROUNDTABLE_PREFILL16=1; everything else this file's 16x16 kernel. The host tile map must use
// the rows of the kernel that will run, hence one function for both.
static bool use_prefill32(int G, int D) {
  static const bool off = getenv("ROUNDTABLE_PREFILL16") != nullptr;
  return !off && D == 128 && prefill32_rows(G) > 0;
}

int prefill_rows_per_tile(int G, int D) {
  if (use_prefill32(G, D)) return prefill32_rows(G);
  return G >= 4 ? 16 : 16 * (4 / G);
}

// q [T, Hq, D]; tile_map [n_tiles, 2] int32 (sequence, first row).
int launch_prefill(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                   const int* cu_q, const int* start_pos, const int* tile_map, int n_tiles, int Hq, int Hkv, int D,
                   int max_blocks, float scale, hipStream_t stream) {
  if (n_tiles == 0) return 0;
  const int G = Hq / Hkv;
  if (Hq % Hkv || G < 1 || G > 16) return -1;
  if (use_prefill32(G, D))
    return launch_prefill32(out, q, k_cache, v_cache, block_tables, cu_q, start_pos, tile_map, n_tiles, Hq, Hkv,
                            max_blocks, scale, stream, 2, nullptr, 0, nullptr, nullptr);
  const int rows = prefill_rows_per_tile(G, D);
  dim3 grid(n_tiles, Hkv), block(256);
  const float sl2 = scale * LOG2E;
#define RT_PF(DD, HH)                                                                                            \
  hipLaunchKernelGGL((prefill_kernel<DD, HH>), grid, block, 2 * PrefillCfg<DD>::STAGE, stream, (uint16_t*)out,   \
                     (const uint16_t*)q, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, cu_q, \
                     start_pos, tile_map, Hq, Hkv, max_blocks, sl2, rows)
  const int hpw = G > 4 ? (G + 3) / 4 : 1;
  if (D == 128) {
    if (hpw == 1) RT_PF(128, 1);
    else if (hpw == 2) RT_PF(128, 2);
    else if (hpw == 3) RT_PF(128, 3);
    else RT_PF(128, 4);
  } else if (D == 64) {
    if (hpw == 1) RT_PF(64, 1);
    else if (hpw == 2) RT_PF(64, 2);
    else if (hpw == 3) RT_PF(64, 3);
    else RT_PF(64, 4);
  } else {
    return -2;
  }
#undef RT_PF
  return 0;
}

// Key-split prefill (32x32 kernel only: D = 128, G <= 8): items [n_items, 5] (sequence,
// first row, first / end key tile, partial slot or -1), cmap [n_split, 4] (sequence, first row,
// first slot, parts). For launches with fewer tiles than CUs (tensor-parallel shards: one or two
// KV heads per rank), where whole tiles would leave most CUs idle.
int launch_prefill_split(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                         const int* cu_q, const int* start_pos, const int* items, int n_items, const int* cmap,
                         int n_split, float* part_o, float* part_ml, int Hq, int Hkv, int D, int max_blocks,
                         float scale, hipStream_t stream) {
  if (n_items == 0) return 0;
  const int G = Hq / Hkv;
  if (Hq % Hkv || !use_prefill32(G, D)) return -1;
  return launch_prefill32(out, q, k_cache, v_cache, block_tables, cu_q, start_pos, items, n_items, Hq, Hkv,
                          max_blocks, scale, stream, 5, cmap, n_split, part_o, part_ml);
}

int prefill_split_supported(int G, int D) { return use_prefill32(G, D) ? 1 : 0; }
