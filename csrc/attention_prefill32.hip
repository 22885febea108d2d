// K4 (D = 128): varlen causal prefill attention on 32x32x16 MFMAs.
//
// Same contract as attention_prefill.hip (queries q[cu_q[s]:cu_q[s+1]] at positions
// start_pos[s] + i attend to cached keys [0, pos]; K/V already in the paged cache), built for
// arithmetic intensity: each wave owns 32 query rows of one head and every K or V fragment it
// reads from LDS feeds a full 32x32x16 MFMA (four times the work per LDS byte of the 16x16
// kernel).
//
// Workgroup = 8 waves over G head slots (G a power of two >= the GQA group; surplus slots idle):
// wave w -> head slot w%G, rows row0 + 32*(w/G) .. +31 (256/G rows
// per workgroup: two waves per SIMD, each K/V tile feeds 8 x 32 query rows). Per 64-key
// tile (two cache blocks):
//   S^T[64 keys x 32 q] = K . Q^T      2 key blocks x 8 d-chunks   (A = K rows from LDS, B = Q^T regs)
//   online softmax down each q column (lane-local + one xor-32 shuffle)
//   O^T[128 d x 32 q] += V^T . P^T     4 d blocks x 4 key chunks   (A = V^T rows from LDS, B = P^T regs)
// K rows are read in the order key(rho) = rho with bits 2 and 3 swapped, which makes the S^T
// accumulator of lane (q, h) hold keys 16c + 8h + 0..7 of each 16-key chunk c — exactly the
// B-operand fragment of P^T — so P never leaves registers; O^T keeps every value of a query
// column in one lane, so the softmax rescale and the final 1/l are lane-local. V is cached
// transposed ([d][32 keys] per block), which is the A-operand order of V^T: one 16-byte LDS
// read per fragment. K/V tiles are register-staged into double-buffered LDS (one barrier
// per tile), K rows XOR-swizzled in 16-byte chunks, V^T rows padded to 144 B.
#include <cstdlib>

#include "common.h"

namespace {
using rt::bf16x8;
using rt::short8;
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int D = 128;
constexpr int BS = 32;          // cache block
constexpr int KT = 64;          // keys per tile
constexpr int KROW = D * 2;     // 256 B per K row
constexpr int VROW = KT * 2 + 16;  // 144 B per V^T row (64 keys + pad)
constexpr int KBYTES = KT * KROW;  // 16 KiB
constexpr int VBYTES = D * VROW;   // 18 KiB
constexpr int STAGE = KBYTES + VBYTES;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float RESCALE_LOG2 = 8.f;   // deferred-rescale slack (log2 units)

RT_DEVICE int swap23(int x) { return (x & ~12) | ((x & 4) << 1) | ((x & 8) >> 1); }

template <int NW>
struct Blocks {
  static constexpr int KL = KBYTES / (64 * NW * 16);
  static constexpr int VL = (D * KT * 2) / (64 * NW * 16);
  int k[KL], v[VL];   // cache block of each of this thread's K / V chunks of one tile

  // the block-table indirection is software-pipelined ahead of the K/V loads that use it, so
  // a tile's loads never wait on a dependent block-table load
  RT_DEVICE void fetch(const int* bt, int tile, int max_blocks, int tid) {
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const int bi = 2 * tile + (((tid * KL + i) >> 4) >> 5);
      k[i] = bt[bi < max_blocks ? bi : 0];
    }
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const int bi = 2 * tile + ((tid * VL + i) >> 9);
      v[i] = bt[bi < max_blocks ? bi : 0];
    }
  }
};

template <int NW>
struct Loader {
  // per thread: K 16 KiB / (64*NW) and V 16 KiB / (64*NW) bytes, 16 B per load
  static constexpr int KL = Blocks<NW>::KL;
  static constexpr int VL = Blocks<NW>::VL;
  rt::u32x4 k[KL], v[VL];   // native vectors: HIP's uint4 class defeats SROA (private-memory spill)

  RT_DEVICE void load(const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ v_cache,
                      const Blocks<NW>& b, size_t blk_stride, size_t head_off, int tid) {
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const int ch = tid * KL + i;          // 16-B chunk of the 64x128 K tile: block ch >> 9, whose
                                            // chunk-major bytes are read in order (common.h kc_chunk)
      k[i] = *reinterpret_cast<const rt::u32x4*>(k_cache + (size_t)b.k[i] * blk_stride + head_off + 8 * (ch & 511));
    }
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const int ch = tid * VL + i;          // 16-B chunk of the two [128 d][32 key] V blocks
      const int w = ch & 511, d = w >> 2, c = w & 3;
      v[i] = *reinterpret_cast<const rt::u32x4*>(v_cache + (size_t)b.v[i] * blk_stride + head_off + d * BS + 8 * c);
    }
  }
  RT_DEVICE void store(unsigned char* kb, unsigned char* vb, int tid) const {
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const int ch = tid * KL + i;
      int key, c;
      rt::kc_chunk(ch & 511, 32, key, c);
      const int row = ((ch >> 9) << 5) + key;
      *reinterpret_cast<rt::u32x4*>(kb + row * KROW + 16 * (c ^ (row & 15))) = k[i];
    }
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const int ch = tid * VL + i;
      const int half = ch >> 9;
      const int w = ch & 511, d = w >> 2, c = w & 3;
      *reinterpret_cast<rt::u32x4*>(vb + d * VROW + 64 * half + 16 * c) = v[i];
    }
  }
};

template <int G, int NW, int DEPTH>
__global__ void __launch_bounds__(NW * 64) prefill32_kernel(
    uint16_t* __restrict__ out, const uint16_t* __restrict__ q, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, const int* __restrict__ cu_q,
    const int* __restrict__ start_pos, const int* __restrict__ tile_map, int Hq, int Hkv, int max_blocks,
    float scale_log2, int rows_per_tile, int map_stride, float* __restrict__ part_o, float* __restrict__ part_ml) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];   // 68 KiB: static (> 64 KiB)
  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (id mod 8), so with
  // id = tile * Hkv + hk every workgroup of kv head hk lands on XCD hk (Hkv = 8): that head's
  // K/V (2 MiB at 4K tokens) stays in one XCD's 4 MiB L2 instead of streaming from MALL/HBM.
  const int tile = blockIdx.x / Hkv, hk = blockIdx.x - (blockIdx.x / Hkv) * Hkv;
  const int* item = tile_map + (size_t)map_stride * tile;
  const int s = item[0], row0 = item[1];
  const int q_begin = cu_q[s], q_end = cu_q[s + 1];
  const int sp = start_pos[s];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 31, h = lane >> 5;   // MFMA column (query) and k-half

  // G = head slots per kv head (a power of two); the real group Gr <= G (Qwen2.5: 7 in 8 slots,
  // Llama-3.2-3B: 3 in 4): a surplus slot's wave loads and barriers with the others, skips the
  // math and stores nothing
  const int Gr = Hq / Hkv, slot_h = wid % G;
  const bool head_ok = slot_h < Gr;
  const int head = hk * Gr + min(slot_h, Gr - 1);
  const int wrow0 = row0 + 32 * (wid / G);
  const int tile_rows_end = min(row0 + rows_per_tile, q_end);
  const int kmax = sp + (tile_rows_end - q_begin);  // keys [0, kmax) for the whole workgroup
  // key split (map_stride 5: sequence, first row, first / end key tile, partial slot): this
  // workgroup covers key tiles [tb, te) and leaves an unnormalised partial for the combine
  // launch (part >= 0), or the whole range and writes the output itself (part < 0)
  int tb = 0, te = (kmax + KT - 1) / KT, part = -1;
  if (map_stride == 5) {
    tb = item[2];
    te = min(item[3], te);
    part = item[4];
  }
  const int ntiles = max(0, te - tb);
  const int my_row = min(wrow0 + c, q_end - 1);
  const int my_pos = sp + (my_row - q_begin);
  // keys this wave can ever see (tiles past it are still loaded cooperatively, math skipped)
  const int wave_rows_end = min(wrow0 + 32, q_end);
  const int wave_kmax = head_ok ? sp + (wave_rows_end - q_begin) : 0;
  const int wave_min_pos = sp + (min(wrow0, q_end - 1) - q_begin);   // first row of the wave

  // Q^T B-fragments: lane (q = c, h) holds Q[q][16 dk + 8 h + j]
  short8 qf[D / 16];
  {
    const uint16_t* qr = q + ((size_t)my_row * Hq + head) * D + 8 * h;
#pragma unroll
    for (int dk = 0; dk < D / 16; ++dk) qf[dk] = *reinterpret_cast<const short8*>(qr + 16 * dk);
  }
  f16v o[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[db][i] = 0.f;
  float m = -INFINITY, lsum = 0.f;

  const int* bt = block_tables + (size_t)s * max_blocks;
  const size_t blk_stride = (size_t)Hkv * BS * D;
  const size_t head_off = (size_t)hk * BS * D;
  // one 64-key tile of the math: S^T = K Q^T, online softmax, O^T += V^T P^T
  auto compute_tile = [&](int tl, const unsigned char* kb, const unsigned char* vb) {
      const int t = tb + tl;   // absolute key tile
      if (tl < ntiles && t * KT < wave_kmax) {
        // ---- S^T = K Q^T (two 32-key blocks) ----
        f16v sc[2];
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int i = 0; i < 16; ++i) sc[blk][i] = 0.f;
        // the two key blocks' accumulation chains interleaved (independent MFMAs back to back)
#pragma unroll
        for (int dk = 0; dk < D / 16; ++dk) {
          const int ch = 2 * dk + h;
#pragma unroll
          for (int blk = 0; blk < 2; ++blk) {
            const int krow = 32 * blk + swap23(c);
            const short8 a = *reinterpret_cast<const short8*>(kb + krow * KROW + 16 * (ch ^ (krow & 15)));
            sc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                              __builtin_bit_cast(bf16x8, qf[dk]), sc[blk], 0, 0, 0);
          }
        }
        // ---- online softmax down column c: reg i of block blk holds key 64t + 32blk + 16(i>>3) + 8h + (i&7)
        float tmax = -INFINITY;
        if ((t + 1) * KT - 1 <= wave_min_pos) {   // whole tile visible to every row of the wave
#pragma unroll
          for (int blk = 0; blk < 2; ++blk)
#pragma unroll
            for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, sc[blk][i]);
        } else {                                  // diagonal tile: causal mask per element
#pragma unroll
          for (int blk = 0; blk < 2; ++blk)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int key = t * KT + 32 * blk + 16 * (i >> 3) + 8 * h + (i & 7);
              const float v = key <= my_pos ? sc[blk][i] : -INFINITY;
              sc[blk][i] = v;
              tmax = fmaxf(tmax, v);
            }
        }
        // scores stay raw: the scale (> 0) commutes with max and is folded into the FMA that
        // feeds exp2 below (one VALU op per score instead of a multiply pass plus a subtract)
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * scale_log2;
        // deferred rescale (guide T13): the running max moves only when some column's tile max
        // exceeds it by more than 2^RESCALE (then P <= 2^RESCALE, still exact enough in bf16 and
        // in the f32 sums). Wave-uniform branch, so most tiles skip the 64-multiply O rescale.
        if (__builtin_amdgcn_ballot_w64(tmax > m + RESCALE_LOG2) != 0) {
          const float mnew = fmaxf(m, tmax);
          const float alpha = (mnew == -INFINITY) ? 1.f : rt::fast_exp2(m - mnew);
          m = mnew;
          lsum *= alpha;
#pragma unroll
          for (int db = 0; db < D / 32; ++db)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[db][i] *= alpha;
        }
        short8 pf[4];   // P^T B-fragments per 16-key chunk
        float psum = 0.f;
        const float msub = (m == -INFINITY) ? 0.f : m;   // all-masked column so far: exp2(-inf) = 0
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
          rt::u32x4 w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float p0 = rt::fast_exp2(__builtin_fmaf(sc[kc >> 1][8 * (kc & 1) + 2 * j], scale_log2, -msub));
            const float p1 = rt::fast_exp2(__builtin_fmaf(sc[kc >> 1][8 * (kc & 1) + 2 * j + 1], scale_log2, -msub));
            psum += p0 + p1;
            w[j] = rt::pack2(p0, p1);
          }
          pf[kc] = __builtin_bit_cast(short8, w);
        }
        lsum += psum;
        // ---- O^T += V^T P^T ----
#pragma unroll
        for (int db = 0; db < D / 32; ++db) {
          // one d-block's 4 V^T fragments live at a time (16 VGPRs, not 64): keep the scheduler
          // from hoisting every block's LDS reads to the top
          __builtin_amdgcn_sched_barrier(0);
          const unsigned char* vr = vb + (32 * db + c) * VROW + 16 * h;
#pragma unroll
          for (int kc = 0; kc < 4; ++kc) {
            const short8 a = *reinterpret_cast<const short8*>(vr + 32 * kc);
            o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                            __builtin_bit_cast(bf16x8, pf[kc]), o[db], 0, 0, 0);
          }
        }
      }
  };

  // static priority for the second-dispatched half (waves NW/2..NW-1): the arbitration loser
  // on every VALU segment otherwise (MI355X_MICROARCH "Two waves per SIMD", item 4)
  if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  Blocks<NW> nb;
  if constexpr (DEPTH == 1) {
    // register staging one tile ahead: tile t+1's loads fly during tile t's math
    Loader<NW> ld;
    if (ntiles > 0) {
      nb.fetch(bt, tb, max_blocks, tid);
      ld.load(k_cache, v_cache, nb, blk_stride, head_off, tid);
      ld.store(smem, smem + KBYTES, tid);
      if (ntiles > 1) nb.fetch(bt, tb + 1, max_blocks, tid);
    }
    // Q^T and tile 0 landed: without this explicit drain the waitcnt pass, merging the
    // ntiles == 0 path at the loop header, waits on qf inside the loop with vmcnt(n..0) —
    // which also drains the next tile's prefetch every iteration (no copy/compute overlap).
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
      const int buf = t & 1;
      if (t + 1 < ntiles) {
        ld.load(k_cache, v_cache, nb, blk_stride, head_off, tid);
        if (t + 2 < ntiles) nb.fetch(bt, tb + t + 2, max_blocks, tid);
      }
      compute_tile(t, smem + buf * STAGE, smem + buf * STAGE + KBYTES);
      // buffer buf^1 held tile t-1, which every wave finished before the previous barrier
      if (t + 1 < ntiles) ld.store(smem + (buf ^ 1) * STAGE, smem + (buf ^ 1) * STAGE + KBYTES, tid);
      __syncthreads();
    }
  } else {
    // two register sets: tile t+2's loads are issued during tile t and written to LDS at the
    // end of tile t+1 — two tiles of math to cover the (L2 / MALL) latency. Loads past the
    // last tile are clamped to it (harmless re-reads) so every vmcnt count is static.
    Loader<NW> la, lb;
    Blocks<NW> nb2;                       // second block-id set: fetched a step before its use
    const int last = ntiles > 0 ? ntiles - 1 : 0;
    nb.fetch(bt, tb, max_blocks, tid);
    la.load(k_cache, v_cache, nb, blk_stride, head_off, tid);
    nb2.fetch(bt, tb + min(1, last), max_blocks, tid);
    lb.load(k_cache, v_cache, nb2, blk_stride, head_off, tid);
    nb.fetch(bt, tb + min(2, last), max_blocks, tid);
    la.store(smem, smem + KBYTES, tid);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    // per step the block-id fetch for tile t+3 is issued BEFORE tile t+2's K/V loads: the next
    // step waits only for that (older) fetch, never for the K/V loads still in flight
    auto step = [&](int t, Loader<NW>& issue, const Loader<NW>& write, const Blocks<NW>& use, Blocks<NW>& fill) {
      const int buf = t & 1;
      fill.fetch(bt, tb + min(t + 3, last), max_blocks, tid);
      issue.load(k_cache, v_cache, use, blk_stride, head_off, tid);   // tile min(t+2, last)
      compute_tile(t, smem + buf * STAGE, smem + buf * STAGE + KBYTES);   // no-op for t >= ntiles
      // unconditional (past the end it fills a buffer nobody reads): a branch here leaves the
      // loads pending on one path, and the waitcnt pass then drains them at the loop top
      write.store(smem + (buf ^ 1) * STAGE, smem + (buf ^ 1) * STAGE + KBYTES, tid);
      __syncthreads();
    };
    for (int t = 0; t < ntiles; t += 2) {   // branch-free pair of steps (an odd count runs one idle step)
      step(t, la, lb, nb, nb2);
      step(t + 1, lb, la, nb2, nb);
    }
  }

  // ---- epilogue: lane (q = c, h) holds O^T[d = 32db + 8b + 4h + j][q], reg i = 4b + j ----
  lsum += __shfl_xor(lsum, 32, 64);
  const int row = wrow0 + c;
  if (part >= 0) {
    // partial of this wave's 32 columns over its key range: O^T unnormalised (relative to the
    // running max m, log2 units), (m, l) per column; every column is written (the combine skips
    // rows past the tile)
    const size_t slot = (((size_t)part * Hkv + hk) * NW + wid) * 32 + c;
    float* po = part_o + slot * D;
#pragma unroll
    for (int db = 0; db < D / 32; ++db)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        *reinterpret_cast<rt::float4_*>(po + 32 * db + 8 * b + 4 * h) =
            rt::float4_{o[db][4 * b], o[db][4 * b + 1], o[db][4 * b + 2], o[db][4 * b + 3]};
    if (h == 0) *reinterpret_cast<float2*>(part_ml + 2 * slot) = make_float2(m, lsum);
    return;
  }
  if (head_ok && row < q_end && row < row0 + rows_per_tile) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    uint16_t* orow = out + ((size_t)row * Hq + head) * D;
#pragma unroll
    for (int db = 0; db < D / 32; ++db)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        uint2 pk;
        pk.x = rt::pack2(o[db][4 * b] * inv, o[db][4 * b + 1] * inv);
        pk.y = rt::pack2(o[db][4 * b + 2] * inv, o[db][4 * b + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * db + 8 * b + 4 * h) = pk;
      }
  }
}
// Combine of the key-split partials: one thread per (wave, column) of a split tile and 16 of its
// 128 dims (grid.y = D / 16), every part's (m, l) and O slice requested before the merge of a
// chunk; fixed part order (deterministic).
template <int G, int NW>
__global__ void __launch_bounds__(NW * 32) prefill32_combine_kernel(uint16_t* __restrict__ out,
                                                                    const int* __restrict__ cmap,
                                                                    const int* __restrict__ cu_q,
                                                                    const float* __restrict__ part_o,
                                                                    const float* __restrict__ part_ml, int Hq,
                                                                    int Hkv, int rows_per_tile) {
  const int st = blockIdx.x / Hkv, hk = blockIdx.x - (blockIdx.x / Hkv) * Hkv;
  const int w = threadIdx.x >> 5, c = threadIdx.x & 31;
  const int s = cmap[4 * st], row0 = cmap[4 * st + 1], p0 = cmap[4 * st + 2], np = cmap[4 * st + 3];
  const int row = row0 + 32 * (w / G) + c;
  const int Gr = Hq / Hkv;   // real group in G slots (prefill32_kernel)
  if (row >= cu_q[s + 1] || row >= row0 + rows_per_tile || w % G >= Gr) return;
  const int head = hk * Gr + (w % G);
  const int d0 = 16 * blockIdx.y;
  constexpr int PC = 4;   // parts per chunk of loads
  float M = -INFINITY, L = 0.f;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int pb = 0; pb < np; pb += PC) {
    float2 ml[PC];
    rt::float4_ ov[PC][4];
#pragma unroll
    for (int j = 0; j < PC; ++j) {
      const int p = p0 + min(pb + j, np - 1);
      const size_t slot = (((size_t)p * Hkv + hk) * NW + w) * 32 + c;
      ml[j] = *reinterpret_cast<const float2*>(part_ml + 2 * slot);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) ov[j][q4] = *reinterpret_cast<const rt::float4_*>(part_o + slot * 128 + d0 + 4 * q4);
    }
#pragma unroll
    for (int j = 0; j < PC; ++j) {
      if (pb + j >= np || !(ml[j].y > 0.f)) continue;
      const float Mc = fmaxf(M, ml[j].x);
      const float a = M == -INFINITY ? 0.f : exp2f(M - Mc), f = exp2f(ml[j].x - Mc);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[4 * q4 + i] = acc[4 * q4 + i] * a + f * ov[j][q4][i];
      L = L * a + f * ml[j].y;
      M = Mc;
    }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  uint16_t* orow = out + ((size_t)row * Hq + head) * 128 + d0;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    uint2 pk;
    pk.x = rt::pack2(acc[4 * q4] * inv, acc[4 * q4 + 1] * inv);
    pk.y = rt::pack2(acc[4 * q4 + 2] * inv, acc[4 * q4 + 3] * inv);
    *reinterpret_cast<uint2*>(orow + 4 * q4) = pk;
  }
}
}  // namespace

// head slots for group size G: the next power of two (surplus slots idle); 0 = unsupported
static int prefill32_slots(int G) {
  return G == 1 ? 1 : G == 2 ? 2 : G <= 4 ? 4 : G <= 8 ? 8 : 0;
}

// rows of one work tile for group size G (D = 128); 0 = unsupported (use attention_prefill.hip)
int prefill32_rows(int G) {
  const int slots = prefill32_slots(G);
  return slots ? 32 * 8 / slots : 0;   // 8 waves x 32 rows over the G heads' slots
}

// tile_map [n_tiles, map_stride]: map_stride 2 = (sequence, first row), every tile whole;
// map_stride 5 = key-split work items (+ first / end key tile, partial slot or -1) whose partial
// slots are merged by a second launch over cmap [n_split, 4] (sequence, first row, first slot,
// parts); part_o >= parts * Hkv * 8 * 32 * 128 floats, part_ml >= parts * Hkv * 8 * 32 * 2.
int launch_prefill32(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                     const int* cu_q, const int* start_pos, const int* tile_map, int n_tiles, int Hq, int Hkv,
                     int max_blocks, float scale, hipStream_t stream, int map_stride, const int* cmap, int n_split,
                     float* part_o, float* part_ml) {
  const int G = Hq / Hkv;
  const int rows = prefill32_rows(G);
  if (rows == 0) return -1;
  if (map_stride != 2 && map_stride != 5) return -2;
  if (map_stride == 5 && n_split > 0 && (cmap == nullptr || part_o == nullptr || part_ml == nullptr)) return -3;
  const float sl2 = scale * LOG2E;
  dim3 grid(n_tiles * Hkv);
  static const int depth = [] {
    const char* e = getenv("ROUNDTABLE_PREFILL_DEPTH");
    return (e && e[0] == '1') ? 1 : 2;
  }();
#define RT_P32(GG, NWV)                                                                                          \
  if (depth == 1) hipLaunchKernelGGL((prefill32_kernel<GG, NWV, 1>), grid, dim3(64 * NWV), 0, stream, (uint16_t*)out, \
                     (const uint16_t*)q, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, cu_q, \
                     start_pos, tile_map, Hq, Hkv, max_blocks, sl2, rows, map_stride, part_o, part_ml);          \
  else hipLaunchKernelGGL((prefill32_kernel<GG, NWV, 2>), grid, dim3(64 * NWV), 0, stream, (uint16_t*)out,              \
                     (const uint16_t*)q, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, cu_q, \
                     start_pos, tile_map, Hq, Hkv, max_blocks, sl2, rows, map_stride, part_o, part_ml);          \
  if (map_stride == 5 && n_split > 0)                                                                            \
    hipLaunchKernelGGL((prefill32_combine_kernel<GG, NWV>), dim3(n_split * Hkv, D / 16), dim3(32 * NWV), 0, stream, \
                       (uint16_t*)out, cmap, cu_q, (const float*)part_o, (const float*)part_ml, Hq, Hkv, rows)
  switch (prefill32_slots(G)) {
    case 1: RT_P32(1, 8); break;
    case 2: RT_P32(2, 8); break;
    case 4: RT_P32(4, 8); break;
    default: RT_P32(8, 8); break;
  }
#undef RT_P32
  return 0;
}
