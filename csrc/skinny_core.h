// Device core of the decode-path GEMMs (M <= 16 rows; 17..32 through gemm_tiles): shared by the standalone launches in
// gemm_skinny.hip and the persistent decode-layer kernel in decode_layer.hip.
//
// Weight layout ("fragment-shuffled", built once at load time by `shuffle_weight`):
//     Ws[N/16][K/32][64 lanes][8]   with  Ws[t][s][l][j] = W[16t + (l&15)][32s + 8(l>>4) + j]
// and for SwiGLU (W = [gate(I); up(I)], `swiglu=True`) the two halves paired per k-step:
//     Ws[I/16][K/32][2][64][8]      with  Ws[t][s][h][l][j] = W[h*I + 16t + (l&15)][32s + 8(l>>4) + j]
// i.e. exactly the order in which the 64 lanes of a wave hold the B operand of
// v_mfma_f32_16x16x32_bf16: every wave load instruction reads 1 KiB of contiguous HBM and a
// workgroup streams its 16-row panel front to back.
//
// One tile = 16 output columns (32 W rows for SwiGLU) x all of K; the NW waves of the
// workgroup take interleaved 32-deep k-steps (adjacent waves -> adjacent KiB), with the next
// U steps' loads issued before the current steps' MFMAs (register double-buffering). M is
// padded to the 16 MFMA rows. The waves' partial tiles are summed through LDS.
//
// Prologues:  PLAIN | NORM (RMSNorm: gamma folded into W, 1/rms from the same A fragments,
//             applied after the MFMAs) | NORM_ADD (A = bf16(x + x2): tensor-parallel residual
//             plus the all-reduced partial; workgroup 0 publishes the sum to `xo`).
// Epilogues:  STORE | RESID (res += y, in place) | SWIGLU (silu(gate) * up) |
//             ROPE (qkv: rotate q/k pairs, write q, scatter k/v into the paged caches) |
//             AR (tensor-parallel row-parallel output: the K9 one-shot all-reduce per tile —
//             push the bf16 tile to every rank's receive buffer, wait for the peers' copies of
//             the SAME tile, sum in rank order; csrc/oneshot_ar.hip).
// SC1 = true (persistent kernel): activations produced inside the same launch are read with
// sc1 loads and every output is stored sc1 (write-through), MI355X_MICROARCH "Valid forms".
#pragma once
#include "common.h"

namespace skinny {
using rt::bf16x8;
using rt::float4_;
using rt::short8;

enum : int { PRO_PLAIN = 0, PRO_NORM = 1, PRO_NORM_ADD = 2 };
enum : int { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_ROPE = 3, EPI_AR = 4 };

struct RopeEpi {
  const int64_t* positions;  // [M]
  const float* cos_sin;      // [max_pos][D]: cos(D/2) | sin(D/2)
  uint16_t* k_cache;
  uint16_t* v_cache;
  const int64_t* slots;      // [M]
  int Hq, Hkv, D, BS;
  const float* bias;         // [N] q/k/v bias in the epilogue's column order (Qwen2), or null
};

// EPI_AR: the K9 comm of csrc/oneshot_ar.hip (receive buffers [2 slots][world][cap] bf16 and
// per-tile flags [2][world][maxt] of every rank, the comm's call counter [epoch, done])
constexpr int AR_MAXW = 8;
struct ArEpi {
  uint16_t* data[AR_MAXW];
  uint32_t* tflags[AR_MAXW];
  uint64_t* ll[AR_MAXW];     // LL form: every rank's (data word, epoch) pair buffer
  uint32_t* ctr;
  int* err;
  long long poll_limit;
  int rank, world, cap, maxt;
  int use_ll;                // 1: exchange in the LL form (oneshot_ar.hip header), 0: push + fence + flag
};

struct GemmArgs {
  uint16_t* out;
  const uint16_t* x;
  const short8* Ws;
  uint16_t* res;
  int M, N, K, ldo;
  float eps;
  RopeEpi re;
  const uint16_t* x2;  // NORM_ADD
  uint16_t* xo;        // NORM_ADD: where workgroup `xo_wg` publishes x + x2
  // weight record order (see weight_order): -1 = the shape's rule, as shuffle_weight wrote it;
  // 0 / c > 0 pinned (layout experiments, tools/exp_balance.hip)
  int kmajor = -1;
  ArEpi ar{};           // EPI_AR only
};

template <int NACC, int NW>   // NACC = accumulators per lane (2 for SwiGLU gate + up)
struct GemmSmem {
  float red[NW][NACC][16][17];
  float sq[NW][16];
};
template <int EPI>
constexpr int nacc() { return EPI == EPI_SWIGLU ? 2 : 1; }

RT_DEVICE float silu(float x) { return x / (1.f + __expf(-x)); }

// Split tile: the K range of one 16-column tile runs as `n` workgroups (k-steps
// [ks*idx/n, ks*(idx+1)/n)); each leaves its row sums (v, up, sum of squares) in `part` with
// write-through stores, the last to arrive (tile counter) sums all n parts IN INDEX ORDER (the
// result does not depend on arrival order), runs the epilogue and re-arms the counter.
// Used by the CU-balanced launch (n = 2 for the remainder tiles) and by split-K (tensor-parallel
// shard shapes with fewer tiles than CUs). Per split tile: n x SPLIT_STRIDE floats.
constexpr int SPLIT_STRIDE = 16 * 16 * 2 + 16;   // v[16][16], up[16][16], ssq[16]
struct SplitX {
  float* part;    // this tile's [n][SPLIT_STRIDE]
  int* ctr;       // this tile's arrival counter (0 between launches)
  int idx;        // this workgroup's part
  int n;          // parts of the tile (>= 2)
};

// 16-bit store, optionally write-through (sc1) for consumers in the same launch
template <bool SC1>
RT_DEVICE void st16(uint16_t* p, float v) {
  if constexpr (SC1)
    __hip_atomic_store(p, rt::f2bf(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = rt::f2bf(v);
}
template <bool SC1>
RT_DEVICE float ld16(const uint16_t* p) {
  if constexpr (SC1)
    return rt::bf2f(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  else
    return rt::bf2f(*p);
}
// Activation fragment loads: SC1 goes through a buffer resource built from the UNIFORM tensor
// base (a per-lane base would force a readfirstlane waterfall loop) plus a per-lane byte offset.
struct XSrc {
  const uint16_t* base;            // plain path: this lane's row pointer
  __amdgpu_buffer_rsrc_t rsrc;     // SC1 path: whole-tensor resource
  int off;                         // SC1 path: this lane's byte offset
};
template <bool SC1>
RT_DEVICE XSrc make_xsrc(const uint16_t* tensor, size_t lane_elem) {
  XSrc x;
  x.base = tensor + lane_elem;
  if constexpr (SC1) {
    x.rsrc = rt::buf_rsrc(tensor);
    x.off = (int)(lane_elem * 2);
  } else {
    x.off = 0;
  }
  return x;
}
template <bool SC1>
RT_DEVICE short8 ld_x8(const XSrc& x, int elem) {
  if constexpr (SC1)
    return __builtin_bit_cast(short8, rt::sc1_load4(x.rsrc, x.off + elem * 2));
  else
    return *reinterpret_cast<const short8*>(x.base + elem);
}

// U = k-steps per wave per pipeline stage (x2 stages in flight)
template <int PRO, int EPI, int U>
struct Stage {
  short8 w[U];
  short8 w2[(EPI == EPI_SWIGLU) ? U : 1];
  short8 a[U];
  short8 b[(PRO == PRO_NORM_ADD) ? U : 1];
};

// short8 records per k-step of one tile (SwiGLU: gate + up)
template <int EPI>
constexpr size_t krec() { return (EPI == EPI_SWIGLU) ? 128 : 64; }

// Weight record order, chosen from the shape so that the shuffle (gemm_skinny.hip) and every
// GEMM launch agree without carrying a layout tag: 0 = tile-major (one contiguous panel per
// tile); c > 0 = k-chunks of 2^(c-1) steps (all tiles' chunks for one k range adjacent, so the
// concurrently streaming workgroups spread over every HBM channel instead of camping on a few
// long panels). tools/exp_balance.hip layouts, MI355X, M = 3: down (K 14336, 1 tile per CU)
// 20.97 -> 19.70 us k-major; qkv 11.25 -> 10.82 chunks of 4; gate_up 39.2-39.9 -> 38.7-39.0
// chunks of 16; lm_head 157.3 -> 148.3 chunks of 16; o (K 4096) unchanged, kept tile-major.
__host__ __device__ inline int weight_order(int tiles, int ksteps, bool swiglu, bool rope) {
  int order = 0;
  if (swiglu) order = 5;
  else if (rope) order = 3;
  else if (tiles >= 4096) order = 5;
  else if (ksteps >= 384) order = 1;
  if (order > 0 && ksteps % (1 << (order - 1)) != 0) order = 0;   // chunks must tile K exactly
  return order;
}

// index of the first record of (tile t, k-step s) in a layout of T tiles x ks steps
__host__ __device__ inline size_t rec_index(int t, int s, int T, int ks, int order, int recs) {
  if (order <= 0) return ((size_t)t * ks + s) * recs;
  const int lc = order - 1, C = 1 << lc;
  return ((size_t)(s >> lc) * T * C + (size_t)t * C + (s & (C - 1))) * recs;
}

struct WStride {
  int lc;          // log2(k-steps per chunk) (30: tile-major, one chunk)
  size_t cstride;  // records between consecutive chunks of one tile
  RT_DEVICE size_t off(int s, size_t rec) const {
    return (size_t)(s >> lc) * cstride + (size_t)(s & ((1 << lc) - 1)) * rec;
  }
};

template <int PRO, int EPI, int NW, int U>
RT_DEVICE void issue_w(Stage<PRO, EPI, U>& st, const short8* __restrict__ wt, const short8* __restrict__ wt2, int s0,
                       int nsteps, int lane, WStride ws) {
  // SwiGLU weights are stored k-step-paired ([tile][step][gate|up][64 lanes][8]): one wave streams
  // 2 KiB contiguous per step instead of two 1-KiB streams 117 MB apart (`wt2` unused)
#pragma unroll
  for (int u = 0; u < U; ++u) {
    // unconditional (steps past the end re-read the last one: an L2 hit) so hipcc counts the
    // loads and waits vmcnt(next stage) before a stage's MFMAs instead of draining vmcnt(0)
    const int s = min(s0 + NW * u, nsteps - 1);
    const size_t o = ws.off(s, krec<EPI>());
    st.w[u] = __builtin_nontemporal_load(wt + o + lane);
    if constexpr (EPI == EPI_SWIGLU) st.w2[u] = __builtin_nontemporal_load(wt + o + 64 + lane);
  }
}

// first record of `tile` and the distance between its k-steps, for either weight order
template <int EPI>
RT_DEVICE const short8* tile_base(const GemmArgs& p, int tile, WStride& ws) {
  const size_t T = (size_t)p.N / 16, ks = (size_t)p.K / 32;
  const int order = p.kmajor >= 0 ? p.kmajor : weight_order((int)T, (int)ks, EPI == EPI_SWIGLU, EPI == EPI_ROPE);
  if (order <= 0) {
    ws.lc = 30;
    ws.cstride = 0;
    return p.Ws + (size_t)tile * ks * krec<EPI>();
  }
  ws.lc = order - 1;
  const size_t chunk = (size_t)1 << ws.lc;
  ws.cstride = T * chunk * krec<EPI>();
  return p.Ws + (size_t)tile * chunk * krec<EPI>();
}

template <int PRO, int EPI, int NW, int U, bool SC1>
RT_DEVICE void issue_a(Stage<PRO, EPI, U>& st, const XSrc& xr, const XSrc& xr2, bool row_ok, int s0, int nsteps) {
  // unconditional as issue_w: lanes of rows >= M read row 0 (their MFMA rows and row sums are
  // never stored), steps past the end re-read the last one
  (void)row_ok;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int s = min(s0 + NW * u, nsteps - 1);
    st.a[u] = ld_x8<SC1>(xr, s * 32);
    if constexpr (PRO == PRO_NORM_ADD) st.b[u] = ld_x8<SC1>(xr2, s * 32);
  }
}

template <int PRO, int EPI, int NW, int U, bool SC1>
RT_DEVICE void consume(const Stage<PRO, EPI, U>& st, float4_& acc, float4_& acc2, float& ssq, int s0, int nsteps,
                       uint16_t* __restrict__ xo_r, const XSrc& xo_s) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (s0 + NW * u < nsteps) {
      short8 av = st.a[u];
      if constexpr (PRO == PRO_NORM_ADD) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          av[j] = (short)rt::f2bf(rt::bf2f((uint16_t)st.a[u][j]) + rt::bf2f((uint16_t)st.b[u][j]));
        if (xo_r != nullptr) {
          if constexpr (SC1) {
            rt::sc1_store4(xo_s.rsrc, xo_s.off + (s0 + NW * u) * 64, __builtin_bit_cast(float4_, av));
          } else {
            *reinterpret_cast<short8*>(xo_r + (s0 + NW * u) * 32) = av;
          }
        }
      }
      const bf16x8 a = __builtin_bit_cast(bf16x8, av);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, st.w[u]), acc, 0, 0, 0);
      if constexpr (EPI == EPI_SWIGLU)
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, st.w2[u]), acc2, 0, 0, 0);
      if constexpr (PRO != PRO_PLAIN) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = rt::bf2f((uint16_t)av[j]);
          ssq = fmaf(f, f, ssq);
        }
      }
    }
  }
}

// ---- A operand staged in LDS (ALDS) -------------------------------------------------------
// With the activation fragments loaded from global memory, every k-step of every wave issues one
// 16-B/lane activation load (two for NORM_ADD) beside its weight load: 2-3x the vector-memory
// instructions of the weight stream, through the CU's one texture path. At tensor-parallel shard
// shapes (few KB to ~100 KB of weights per workgroup) that — not HBM — bounds the launch
// (tools/probes/stream_probe.hip: a pure 16-B/lane stream of 192 x 128 KB takes 6.5 us, the
// tp2 qkv GEMM of the same bytes 9.6 us). ALDS stages rows [0, M) of the workgroup's K range
// ONCE (NORM_ADD: the bf16 sum x + x2, published to `xo` by the publishing workgroup; NORM /
// NORM_ADD: each row's sum of squares, from the same values), then every k-step reads its A
// fragment with one ds_read_b128 — the global loads of the k-loop are the weights alone.
struct ALds {
  uint16_t* a;     // [M][astride] bf16
  float* ssq;      // [16] sum of squares of each staged row (NORM / NORM_ADD)
  int astride;     // elements per staged row: K range + 8 (rows 4 banks apart)
};
constexpr int ALDS_BATCH = 8;   // 16-B loads per lane in flight while staging one row

// Rows are spread over the waves (row m on wave m % NW); within a row the 64 lanes take 16-B
// units, ALDS_BATCH per lane per round trip (clamped re-reads at the tail are L2 hits, never
// stored twice).
template <int PRO, int NW, bool SC1A = false>
RT_DEVICE void stage_a(const GemmArgs& p, int s_lo, int nsteps, const ALds& L, uint16_t* __restrict__ xo) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int K = p.K, kb = s_lo * 32, n8 = (nsteps - s_lo) * 4;
  for (int m = wid; m < p.M; m += NW) {
    const uint16_t* xr = p.x + (size_t)m * K + kb;
    const uint16_t* x2r = PRO == PRO_NORM_ADD ? p.x2 + (size_t)m * K + kb : xr;
    uint16_t* dst = L.a + (size_t)m * L.astride;
    float ss = 0.f;
    for (int u0 = 0; u0 < n8; u0 += 64 * ALDS_BATCH) {
      short8 a[ALDS_BATCH], b[ALDS_BATCH];
#pragma unroll
      for (int j = 0; j < ALDS_BATCH; ++j) {
        const int u = min(u0 + 64 * j + lane, n8 - 1);
        if constexpr (SC1A)   // rows written earlier in this launch (persistent phases)
          a[j] = __builtin_bit_cast(short8, rt::sc1_load4(rt::buf_rsrc(p.x), (int)((xr - p.x) + 8 * u) * 2));
        else
          a[j] = *reinterpret_cast<const short8*>(xr + 8 * u);
        if constexpr (PRO == PRO_NORM_ADD) b[j] = *reinterpret_cast<const short8*>(x2r + 8 * u);
      }
#pragma unroll
      for (int j = 0; j < ALDS_BATCH; ++j) {
        const int u = u0 + 64 * j + lane;
        short8 av = a[j];
        if constexpr (PRO == PRO_NORM_ADD) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            av[e] = (short)rt::f2bf(rt::bf2f((uint16_t)a[j][e]) + rt::bf2f((uint16_t)b[j][e]));
        }
        if (u < n8) {
          *reinterpret_cast<short8*>(dst + 8 * u) = av;
          if (PRO == PRO_NORM_ADD && xo != nullptr) *reinterpret_cast<short8*>(xo + (size_t)m * K + kb + 8 * u) = av;
          if constexpr (PRO != PRO_PLAIN) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float f = rt::bf2f((uint16_t)av[e]);
              ss = fmaf(f, f, ss);
            }
          }
        }
      }
    }
    if constexpr (PRO != PRO_PLAIN) {
      ss = rt::wave_sum(ss);
      if (lane == 0) L.ssq[m] = ss;
    }
  }
}

template <int PRO, int EPI, int NW, int U>
RT_DEVICE void consume_lds(const Stage<PRO, EPI, U>& st, float4_& acc, float4_& acc2, int s0, int nsteps,
                           const uint16_t* __restrict__ arow) {
  // arow = this lane's staged row + 8g - 32 s_lo: the A fragment of k-step s is arow[32 s .. +8)
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (s0 + NW * u < nsteps) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, *reinterpret_cast<const short8*>(arow + (s0 + NW * u) * 32));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, st.w[u]), acc, 0, 0, 0);
      if constexpr (EPI == EPI_SWIGLU)
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, st.w2[u]), acc2, 0, 0, 0);
    }
  }
}

// dynamic LDS bytes of the ALDS staging for M rows of a K range of `kspan` elements
__host__ __device__ inline int alds_bytes(int M, int kspan) { return 64 + M * (kspan + 8) * 2; }

// Stage-0 weight prefetch of `tile` for the calling wave (no activation loads): lets a
// persistent kernel put a tile's first weight bytes in flight before its inputs are ready.
template <int PRO, int EPI, int NW, int U>
RT_DEVICE void gemm_prefetch(const GemmArgs& p, int tile, Stage<PRO, EPI, U>& st0) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nsteps = p.K / 32;
  WStride sstride;
  const short8* wt = tile_base<EPI>(p, tile, sstride);
  const short8* wt2 = nullptr;
  issue_w<PRO, EPI, NW, U>(st0, wt, wt2, wid, nsteps, lane, sstride);
}

// EPI_AR: one tile's share of the K9 one-shot all-reduce, run by the workgroup that computed it
// (a row-parallel decode GEMM needs no separate all-reduce launch). The value every rank
// contributes is the bf16-rounded tile, exactly what the standalone K9 kernel would have been
// given, and the copies are summed in fp32 in rank order, so the result is bit-identical to
// GEMM (STORE) + K9 on every rank. Protocol as oneshot_ar.hip: remote 16-B pushes -> system
// fence -> one flag per (peer, tile) -> bounded wait on the peers' flags of this tile in our own
// memory -> sum. The last workgroup out advances the comm's call counter (graph-replayable).
// Slot reuse: before this call writes slot (epoch & 1) again, every workgroup of the previous
// call saw each peer's flag of that call, which the peer raised after its call before it (the
// slot's last reader) had completed.
template <int NW>
RT_DEVICE void ar_exchange(const GemmArgs& p, int tile, float v, int m, int n, bool live,
                           GemmSmem<1, NW>& sm) {
  const ArEpi& ar = p.ar;
  const int M = p.M, N = p.N;
  const uint32_t epoch = __hip_atomic_load(ar.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int slot = (int)(epoch & 1u);
  uint16_t* stage = reinterpret_cast<uint16_t*>(&sm.red[0][0][0][0]);   // [16 rows][16 cols] bf16
  __syncthreads();                         // every wave is done reading the reduction buffers
  const uint16_t mine = rt::f2bf(v);
  if (live) stage[m * 16 + n] = mine;
  __syncthreads();
  const int t = threadIdx.x;
  if (ar.use_ll) {
    // LL form: each 2-column word of the tile travels with the epoch in one 8-byte store; the
    // receiver polls its rank's pairs directly (no fence, no tile flag)
    const size_t rs = (size_t)ar.cap / 2;
    const uint64_t tag = (uint64_t)epoch << 32;
    for (int q = t; q < 8 * M * ar.world; q += blockDim.x) {
      const int dst = q / (8 * M), rem = q - dst * 8 * M, row = rem >> 3, c2 = rem & 7;
      const uint32_t w = *reinterpret_cast<const uint32_t*>(stage + row * 16 + 2 * c2);
      uint64_t* d = ar.ll[dst] + ((size_t)slot * ar.world + ar.rank) * rs + ((size_t)row * N + tile * 16) / 2 + c2;
      __hip_atomic_store(d, tag | w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (live) {
      const uint64_t* own = ar.ll[ar.rank] + (size_t)slot * ar.world * rs + ((size_t)m * N + tile * 16) / 2 + (n >> 1);
      uint64_t q[AR_MAXW];
#pragma unroll
      for (int r = 0; r < AR_MAXW; ++r)
        if (r < ar.world && r != ar.rank)
          q[r] = __hip_atomic_load(own + (size_t)r * rs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < AR_MAXW; ++r) {
        if (r >= ar.world) continue;
        if (r == ar.rank) {
          acc += rt::bf2f(mine);
          continue;
        }
        long long it = 0;
        while ((uint32_t)(q[r] >> 32) != epoch) {
          __builtin_amdgcn_s_sleep(1);
          if (++it > ar.poll_limit) {
            __hip_atomic_store(ar.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          q[r] = __hip_atomic_load(own + (size_t)r * rs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint32_t w = (uint32_t)q[r];
        acc += rt::bf2f((uint16_t)((n & 1) ? (w >> 16) : (w & 0xffffu)));
      }
      if (p.res != nullptr) {
        uint16_t* rp = p.res + (size_t)m * N + tile * 16 + n;
        *rp = rt::f2bf(rt::bf2f(*rp) + rt::bf2f(rt::f2bf(acc)));
      } else {
        p.out[(size_t)m * p.ldo + tile * 16 + n] = rt::f2bf(acc);
      }
    }
    __syncthreads();
    if (t == 0) {
      const uint32_t prev = __hip_atomic_fetch_add(ar.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gridDim.x - 1u) {
        __hip_atomic_store(ar.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ar.ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  // 1. push: row m of the tile = 32 B = two 16-B stores per destination rank
  if (t < 2 * M * ar.world) {
    const int dst = t / (2 * M), rem = t - dst * 2 * M, row = rem >> 1, half = rem & 1;
    const uint4 val = *reinterpret_cast<const uint4*>(stage + row * 16 + half * 8);
    uint16_t* d = ar.data[dst] + ((size_t)slot * ar.world + ar.rank) * ar.cap + (size_t)row * N + tile * 16 + half * 8;
    *reinterpret_cast<uint4*>(d) = val;
  }
  // 2. release: all pushes complete before any flag of this tile is raised
  __threadfence_system();
  __syncthreads();
  if (t < ar.world)
    __hip_atomic_store(ar.tflags[t] + ((size_t)slot * ar.world + ar.rank) * ar.maxt + tile, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every rank's copy of this tile (bounded: on expiry flag the error, proceed)
  if (t < ar.world) {
    const uint32_t* f = ar.tflags[ar.rank] + ((size_t)slot * ar.world + t) * ar.maxt + tile;
    long long it = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > ar.poll_limit) {
        __hip_atomic_store(ar.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
  // 4. sum the world copies in rank order (fp32), store the bf16 result
  if (live) {
    const uint16_t* own = ar.data[ar.rank] + (size_t)slot * ar.world * ar.cap + (size_t)m * N + tile * 16 + n;
    float acc = 0.f;
    for (int r = 0; r < ar.world; ++r) acc += rt::bf2f(r == ar.rank ? mine : own[(size_t)r * ar.cap]);
    if (p.res != nullptr) {   // residual form: res = bf16(res + bf16(sum)), in place
      uint16_t* rp = p.res + (size_t)m * N + tile * 16 + n;
      *rp = rt::f2bf(rt::bf2f(*rp) + rt::bf2f(rt::f2bf(acc)));
    } else {
      p.out[(size_t)m * p.ldo + tile * 16 + n] = rt::f2bf(acc);
    }
  }
  // 5. the last workgroup out advances the call counter (every workgroup has read it)
  __syncthreads();
  if (t == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(ar.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1u) {
      __hip_atomic_store(ar.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ar.ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One 16-column tile. `st0` may hold this tile's prefetched stage-0 weights (prefetched=true).
// `publish_xo`: this workgroup writes the NORM_ADD sum to p.xo.
// AC (persistent kernels): coherence of the ACTIVATION loads apart from the stores — -1 = as SC1,
// 0 = plain (the activation came from an earlier launch), 1 = sc1 (produced in this launch). With
// ALDS, AC = 1 stages the rows with sc1 loads once, then reads LDS.
template <int PRO, int EPI, int NW, int U, bool SC1, bool ALDS = false, int AC = -1>
RT_DEVICE void gemm_tile(const GemmArgs& p, int tile, GemmSmem<nacc<EPI>(), NW>& sm, Stage<PRO, EPI, U>& st0,
                         bool prefetched,
                         bool publish_xo, const SplitX* sx = nullptr, const ALds* al = nullptr) {
  constexpr bool SC1A = AC < 0 ? SC1 : AC != 0;
  static_assert(!(ALDS && SC1 && AC < 0), "an LDS-staged A operand in a persistent launch needs an explicit AC");
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int M = p.M, N = p.N, K = p.K;
  const int ksteps = K / 32;
  // k-step range of this workgroup: all of K, or one part of a split tile. `nsteps` below is
  // the range END (loads clamp to it), `s_lo` its start.
  const int s_lo = sx != nullptr ? (int)((long)ksteps * sx->idx / sx->n) : 0;
  const int nsteps = sx != nullptr ? (int)((long)ksteps * (sx->idx + 1) / sx->n) : ksteps;
  const bool row_ok = r < M;
  const size_t lane_elem = (size_t)(row_ok ? r : 0) * K + 8 * g;
  const XSrc xr = make_xsrc<SC1A>(p.x, lane_elem);
  const XSrc xr2 = make_xsrc<SC1A>(PRO == PRO_NORM_ADD ? p.x2 : p.x, lane_elem);
  uint16_t* xo_r =
      (PRO == PRO_NORM_ADD && publish_xo && row_ok && p.xo != nullptr) ? p.xo + (size_t)r * K + 8 * g : nullptr;
  const XSrc xo_s = make_xsrc<SC1A>(PRO == PRO_NORM_ADD && p.xo != nullptr ? p.xo : p.x, lane_elem);
  WStride sstride;
  const short8* wt = tile_base<EPI>(p, tile, sstride);
  const short8* wt2 = nullptr;

  float4_ acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
  float ssq = 0.f;
  Stage<PRO, EPI, U> st1;
  // stages of this wave: s = wid + NW*U*j < nsteps. Both halves of a pair sit in ONE basic
  // block (a break between them lets MachineSink move each stage's loads down next to their
  // consumer); every issue is unconditional, so the waits are counted, not vmcnt(0).
  constexpr int SPAN = NW * U;
  const int w0 = s_lo + wid;   // this wave's first k-step
  const int nst = w0 < nsteps ? (nsteps - w0 + SPAN - 1) / SPAN : 0;
  if (!prefetched) issue_w<PRO, EPI, NW, U>(st0, wt, wt2, w0, nsteps, lane, sstride);
  const uint16_t* arow = nullptr;
  if constexpr (ALDS) {
    // stage-0 weights are in flight; stage A once (its loads overlap theirs), then the k-loop
    stage_a<PRO, NW, SC1A>(p, s_lo, nsteps, *al,
                     (PRO == PRO_NORM_ADD && publish_xo && p.xo != nullptr) ? p.xo : nullptr);
    __syncthreads();
    arow = al->a + (size_t)(row_ok ? r : 0) * al->astride + 8 * g - 32 * s_lo;
  } else {
    issue_a<PRO, EPI, NW, U, SC1A>(st0, xr, xr2, row_ok, w0, nsteps);
  }
  // Epilogue operands that do not depend on the GEMM are loaded NOW, so their round trips hide
  // under the k-loop instead of following the last MFMA: the residual element (RESID) and the
  // K/V slot, position and cos/sin pair (ROPE). Unconditional, rows clamped (no branch for the
  // waitcnt pass to merge); the epilogue thread (em, en) is the one that uses them.
  const int em = min((int)(threadIdx.x >> 4), M - 1), en = threadIdx.x & 15;
  float e_res = 0.f, e_c = 0.f, e_s = 0.f, e_b = 0.f, e_bp = 0.f;
  int64_t e_slot = 0;
  if constexpr (EPI == EPI_RESID) e_res = ld16<SC1>(p.res + (size_t)em * N + tile * 16 + en);
  if constexpr (EPI == EPI_ROPE) {
    const RopeEpi& re = p.re;
    const int pp = (tile * 16 + en) % re.D;
    e_slot = re.slots[em];
    const float* cs = re.cos_sin + (size_t)re.positions[em] * re.D;
    e_c = cs[pp >> 1];
    e_s = cs[(re.D >> 1) + (pp >> 1)];
    if (re.bias != nullptr) {   // this column's bias and its rotate-half partner's (column ^ 1)
      e_b = re.bias[tile * 16 + en];
      e_bp = re.bias[(tile * 16 + en) ^ 1];
    }
  }
  int j = 0;
  if constexpr (ALDS) {
    for (; j + 1 < nst; j += 2) {
      const int s = w0 + SPAN * j;
      issue_w<PRO, EPI, NW, U>(st1, wt, wt2, s + SPAN, nsteps, lane, sstride);
      consume_lds<PRO, EPI, NW, U>(st0, acc, acc2, s, nsteps, arow);
      issue_w<PRO, EPI, NW, U>(st0, wt, wt2, s + 2 * SPAN, nsteps, lane, sstride);
      consume_lds<PRO, EPI, NW, U>(st1, acc, acc2, s + SPAN, nsteps, arow);
    }
    if (j < nst) consume_lds<PRO, EPI, NW, U>(st0, acc, acc2, w0 + SPAN * j, nsteps, arow);
  } else {
    for (; j + 1 < nst; j += 2) {
      const int s = w0 + SPAN * j;
      issue_w<PRO, EPI, NW, U>(st1, wt, wt2, s + SPAN, nsteps, lane, sstride);
      issue_a<PRO, EPI, NW, U, SC1A>(st1, xr, xr2, row_ok, s + SPAN, nsteps);
      consume<PRO, EPI, NW, U, SC1A>(st0, acc, acc2, ssq, s, nsteps, xo_r, xo_s);
      issue_w<PRO, EPI, NW, U>(st0, wt, wt2, s + 2 * SPAN, nsteps, lane, sstride);
      issue_a<PRO, EPI, NW, U, SC1A>(st0, xr, xr2, row_ok, s + 2 * SPAN, nsteps);
      consume<PRO, EPI, NW, U, SC1A>(st1, acc, acc2, ssq, s + SPAN, nsteps, xo_r, xo_s);
    }
    if (j < nst) consume<PRO, EPI, NW, U, SC1A>(st0, acc, acc2, ssq, w0 + SPAN * j, nsteps, xo_r, xo_s);
  }

  // C layout: acc[i] = C[m = 4g + i][n = r]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sm.red[wid][0][4 * g + i][r] = acc[i];
    if constexpr (EPI == EPI_SWIGLU) sm.red[wid][(EPI == EPI_SWIGLU) ? 1 : 0][4 * g + i][r] = acc2[i];
  }
  if constexpr (PRO != PRO_PLAIN && !ALDS) {
    ssq += __shfl_xor(ssq, 16, 64);
    ssq += __shfl_xor(ssq, 32, 64);
    if (g == 0) sm.sq[wid][r] = ssq;
  }
  __syncthreads();
  const int m = threadIdx.x >> 4, n = threadIdx.x & 15;
  const bool live = threadIdx.x < 256 && m < M;
  float v = 0.f, ss = 0.f, up = 0.f;
  if (live) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      v += sm.red[w][0][m][n];
      if constexpr (PRO != PRO_PLAIN && !ALDS) ss += sm.sq[w][m];
      if constexpr (EPI == EPI_SWIGLU) up += sm.red[w][(EPI == EPI_SWIGLU) ? 1 : 0][m][n];
    }
    if constexpr (PRO != PRO_PLAIN && ALDS) ss = al->ssq[m];
  }
  if (sx != nullptr) {   // split tile: hand this part's sums over, the last arrival finishes
    // hand-off (MI355X_MICROARCH, sc1 table row 1): 4-B sc1 payload stores -> every wave's
    // vmcnt(0) -> barrier -> one agent atomic add; the last adder's waves load sc1 after the
    // barrier that publishes its LDS flag
    float* mine = sx->part + sx->idx * SPLIT_STRIDE;
    if (live) {
      __hip_atomic_store(mine + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (EPI == EPI_SWIGLU)
        __hip_atomic_store(mine + 256 + threadIdx.x, up, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (n == 0) __hip_atomic_store(mine + 512 + m, ss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(sx->ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = prev == sx->n - 1;
      sm.sq[0][0] = last ? 1.f : 0.f;   // LDS flag: this workgroup arrived last
      if (last) __hip_atomic_store(sx->ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (sm.sq[0][0] == 0.f) return;   // not last: another workgroup finishes the tile
    if (live) {
      const float v_own = v, up_own = up, ss_own = ss;
      v = up = ss = 0.f;
      for (int i = 0; i < sx->n; ++i) {   // fixed order: bit-identical whoever arrives last
        const float* pi = sx->part + i * SPLIT_STRIDE;
        const bool own = i == sx->idx;
        v += own ? v_own : __hip_atomic_load(pi + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (EPI == EPI_SWIGLU)
          up += own ? up_own : __hip_atomic_load(pi + 256 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (PRO != PRO_PLAIN)
          ss += own ? ss_own : __hip_atomic_load(pi + 512 + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // ROPE: the rotate-half partner (column n ^ 1, same row) is the adjacent lane's finished sum,
  // whole or split alike (thread = 16 m + n); every lane takes part in the shuffle
  float vpartner = 0.f;
  if constexpr (EPI == EPI_ROPE) vpartner = __shfl_xor(v, 1, 64);
  if (live) {
    float inv = 1.f;
    if constexpr (PRO != PRO_PLAIN) inv = rsqrtf(ss / (float)K + p.eps);
    v *= inv;
    const int col = tile * 16 + n;
    if constexpr (EPI == EPI_SWIGLU) {
      up *= inv;
      st16<SC1>(p.out + (size_t)m * p.ldo + col, silu(v) * up);
    } else if constexpr (EPI == EPI_RESID) {
      uint16_t* rp = p.res + (size_t)m * N + col;
      st16<SC1>(rp, v + e_res);
    } else if constexpr (EPI == EPI_ROPE) {
      const RopeEpi& re = p.re;
      const int D = re.D, half = D >> 1;
      const int h = col / D, pp = col - h * D;
      const int64_t slot = e_slot;
      const int64_t blk = slot / re.BS;
      const int off = (int)(slot - blk * re.BS);
      v += e_b;
      if (h < re.Hq + re.Hkv) {
        const float partner = fmaf(vpartner, inv, e_bp);
        const int i = pp >> 1, hi = pp & 1;
        const float c = e_c, sn = e_s;
        // pair (x1 = d i, x2 = d i+D/2): y1 = x1 c - x2 s ; y2 = x2 c + x1 s
        const float y = hi ? fmaf(v, c, partner * sn) : fmaf(v, c, -partner * sn);
        const int d = i + hi * half;
        uint16_t* dst = (h < re.Hq) ? p.out + ((size_t)m * re.Hq + h) * D + d
                                    : re.k_cache + ((size_t)blk * re.Hkv + (h - re.Hq)) * re.BS * D +
                                          rt::kc_elem(re.BS, off, d);
        st16<SC1>(dst, y);
      } else {
        const int hv = h - re.Hq - re.Hkv;
        st16<SC1>(re.v_cache + (((size_t)blk * re.Hkv + hv) * D + pp) * re.BS + off, v);
      }
    } else if constexpr (EPI == EPI_AR) {
      // stored after the exchange below
    } else {
      st16<SC1>(p.out + (size_t)m * p.ldo + col, v);
    }
  }
  if constexpr (EPI == EPI_AR) ar_exchange<NW>(p, tile, v, m, n, live, sm);
  __syncthreads();  // LDS reduction buffers are reused by the next tile
}

// ---- TN tiles per workgroup (serving batches, M > 4) ----------------------------------------
// At M = 16 every k-step's activation fragment is 16 distinct rows, 1 KiB per wave — as many
// bytes as its weight fragment — and a one-tile workgroup streams the whole activation matrix
// through its CU for 16 output columns (lm_head, M = 16: 8016 tiles x 128 KiB of activation
// reads per step; 235 us vs 148 us at M = 3). Here each workgroup owns TN consecutive tiles:
// one activation fragment per k-step feeds TN MFMAs (TN weight streams), the activation reads
// fall TN-fold. MB = 2 row blocks (17..32 rows): every weight fragment feeds both blocks' MFMAs,
// so a 32-row batch streams the weights once. Plain / NORM prologues, STORE / RESID / SWIGLU /
// ROPE epilogues, optional K split, no SC1 (one launch per GEMM); the M <= 4 decode path keeps
// gemm_tile.
template <int NACC, int NW, int TN, int MB>
struct GemmSmemN {
  float red[NW][NACC * TN * MB][16][17];
  float sq[NW][16 * MB];
};

template <int PRO, int EPI, int U, int TN, int MB>
struct StageN {
  short8 w[U][TN];
  short8 w2[(EPI == EPI_SWIGLU) ? U : 1][(EPI == EPI_SWIGLU) ? TN : 1];
  short8 a[U][MB];
};

template <int PRO, int EPI, int NW, int U, int TN, int MB>
RT_DEVICE void issue_wn(StageN<PRO, EPI, U, TN, MB>& st, const short8* const* wt, int s0, int nsteps, int lane,
                        WStride ws) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int s = min(s0 + NW * u, nsteps - 1);   // unconditional, as issue_w
    const size_t o = ws.off(s, krec<EPI>());
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      st.w[u][t] = __builtin_nontemporal_load(wt[t] + o + lane);
      if constexpr (EPI == EPI_SWIGLU) st.w2[u][t] = __builtin_nontemporal_load(wt[t] + o + 64 + lane);
    }
  }
}

template <int PRO, int EPI, int NW, int U, int TN, int MB>
RT_DEVICE void issue_an(StageN<PRO, EPI, U, TN, MB>& st, const XSrc* xr, int s0, int nsteps) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int b = 0; b < MB; ++b) st.a[u][b] = ld_x8<false>(xr[b], min(s0 + NW * u, nsteps - 1) * 32);
}

// acc / acc2: [TN][MB] accumulators, ssq: [MB]
template <int PRO, int EPI, int NW, int U, int TN, int MB>
RT_DEVICE void consume_n(const StageN<PRO, EPI, U, TN, MB>& st, float4_ (*acc)[MB], float4_ (*acc2)[MB], float* ssq,
                         int s0, int nsteps) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (s0 + NW * u < nsteps) {
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, st.a[u][b]);
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, st.w[u][t]), acc[t][b], 0, 0, 0);
          if constexpr (EPI == EPI_SWIGLU)
            acc2[t][b] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, st.w2[u][t]), acc2[t][b], 0, 0, 0);
        }
        if constexpr (PRO != PRO_PLAIN) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float f = rt::bf2f((uint16_t)st.a[u][b][j]);
            ssq[b] = fmaf(f, f, ssq[b]);
          }
        }
      }
    }
  }
}

// Tiles tile0 .. tile0 + TN - 1 (those >= N / 16 are computed on a clamped copy, never stored).
// `sx` (optional): this workgroup runs part sx->idx of sx->n K ranges of the TN tiles; partial
// sums are handed over as in gemm_tile (sx->part holds [n][TN][MB][SPLIT_STRIDE]) and the last
// arrival sums the parts in index order and runs the epilogue — the o / down shapes (256 tiles)
// keep a workgroup per CU while each workgroup reads the activations for two tiles.
template <int PRO, int EPI, int NW, int U, int TN, int MB>
RT_DEVICE void gemm_tiles(const GemmArgs& p, int tile0, GemmSmemN<nacc<EPI>(), NW, TN, MB>& sm,
                          const SplitX* sx = nullptr) {
  static_assert(PRO == PRO_PLAIN || PRO == PRO_NORM, "multi-tile launches: plain / norm prologues");
  static_assert(EPI != EPI_AR, "multi-tile launches: no all-reduce epilogue");
  constexpr int NA = nacc<EPI>();
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int M = p.M, N = p.N, K = p.K;
  const int T = N / 16, ksteps = K / 32;
  const int s_lo = sx != nullptr ? (int)((long)ksteps * sx->idx / sx->n) : 0;
  const int nsteps = sx != nullptr ? (int)((long)ksteps * (sx->idx + 1) / sx->n) : ksteps;
  XSrc xr[MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    const int row = 16 * b + r;
    xr[b] = make_xsrc<false>(p.x, (size_t)(row < M ? row : 0) * K + 8 * g);   // rows >= M read row 0
  }
  WStride sstride;
  const short8* wt[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) wt[t] = tile_base<EPI>(p, min(tile0 + t, T - 1), sstride);

  float4_ acc[TN][MB], acc2[TN][MB];
  float ssq[MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    ssq[b] = 0.f;
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[t][b] = acc2[t][b] = float4_{0.f, 0.f, 0.f, 0.f};
  }
  StageN<PRO, EPI, U, TN, MB> st0, st1;
  constexpr int SPAN = NW * U;
  const int w0 = s_lo + wid;
  const int nst = w0 < nsteps ? (nsteps - w0 + SPAN - 1) / SPAN : 0;
  issue_wn<PRO, EPI, NW, U, TN, MB>(st0, wt, w0, nsteps, lane, sstride);
  issue_an<PRO, EPI, NW, U, TN, MB>(st0, xr, w0, nsteps);
  // epilogue operands independent of the GEMM, loaded under the k-loop (as gemm_tile); the
  // epilogue thread (em, en) of row block b owns row 16 b + em
  const int em = threadIdx.x >> 4, en = threadIdx.x & 15;
  float e_res[TN][MB], e_c[TN][MB], e_s[TN][MB], e_b[TN], e_bp[TN];
  int64_t e_slot[MB];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    e_b[t] = e_bp[t] = 0.f;
    if constexpr (EPI == EPI_ROPE) {
      const int c = min(tile0 + t, T - 1) * 16 + en;
      if (p.re.bias != nullptr) {
        e_b[t] = p.re.bias[c];
        e_bp[t] = p.re.bias[c ^ 1];
      }
    }
  }
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    const int row = min(16 * b + em, M - 1);
    e_slot[b] = 0;
    if constexpr (EPI == EPI_ROPE) e_slot[b] = p.re.slots[row];
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int tt = min(tile0 + t, T - 1);
      e_res[t][b] = e_c[t][b] = e_s[t][b] = 0.f;
      if constexpr (EPI == EPI_RESID) e_res[t][b] = ld16<false>(p.res + (size_t)row * N + tt * 16 + en);
      if constexpr (EPI == EPI_ROPE) {
        const RopeEpi& re = p.re;
        const int pp = (tt * 16 + en) % re.D;
        const float* cs = re.cos_sin + (size_t)re.positions[row] * re.D;
        e_c[t][b] = cs[pp >> 1];
        e_s[t][b] = cs[(re.D >> 1) + (pp >> 1)];
      }
    }
  }
  int j = 0;
  for (; j + 1 < nst; j += 2) {
    const int s = w0 + SPAN * j;
    issue_wn<PRO, EPI, NW, U, TN, MB>(st1, wt, s + SPAN, nsteps, lane, sstride);
    issue_an<PRO, EPI, NW, U, TN, MB>(st1, xr, s + SPAN, nsteps);
    consume_n<PRO, EPI, NW, U, TN, MB>(st0, acc, acc2, ssq, s, nsteps);
    issue_wn<PRO, EPI, NW, U, TN, MB>(st0, wt, s + 2 * SPAN, nsteps, lane, sstride);
    issue_an<PRO, EPI, NW, U, TN, MB>(st0, xr, s + 2 * SPAN, nsteps);
    consume_n<PRO, EPI, NW, U, TN, MB>(st1, acc, acc2, ssq, s + SPAN, nsteps);
  }
  if (j < nst) consume_n<PRO, EPI, NW, U, TN, MB>(st0, acc, acc2, ssq, w0 + SPAN * j, nsteps);

  // C layout per (tile, row block): acc[t][b][i] = C[m = 16 b + 4g + i][n = r]
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sm.red[wid][(NA * t) * MB + b][4 * g + i][r] = acc[t][b][i];
        if constexpr (EPI == EPI_SWIGLU) sm.red[wid][(NA * t + 1) * MB + b][4 * g + i][r] = acc2[t][b][i];
      }
  if constexpr (PRO != PRO_PLAIN) {
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      float q = ssq[b];
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (g == 0) sm.sq[wid][16 * b + r] = q;
    }
  }
  __syncthreads();
  const int m = threadIdx.x >> 4, n = threadIdx.x & 15;
  const bool thr = threadIdx.x < 256;
  float ss[MB], vs[TN][MB], ups[TN][MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    ss[b] = 0.f;
    const bool live = thr && 16 * b + m < M;
#pragma unroll
    for (int t = 0; t < TN; ++t) vs[t][b] = ups[t][b] = 0.f;
    if (live) {
      if constexpr (PRO != PRO_PLAIN) {
#pragma unroll
        for (int w = 0; w < NW; ++w) ss[b] += sm.sq[w][16 * b + m];
      }
#pragma unroll
      for (int t = 0; t < TN; ++t)
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          vs[t][b] += sm.red[w][(NA * t) * MB + b][m][n];
          if constexpr (EPI == EPI_SWIGLU) ups[t][b] += sm.red[w][(NA * t + 1) * MB + b][m][n];
        }
    }
  }
  if (sx != nullptr) {   // hand-off as gemm_tile: sc1 payload -> vmcnt(0) -> barrier -> one add
    float* mine = sx->part + (size_t)sx->idx * TN * MB * SPLIT_STRIDE;
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      if (thr && 16 * b + m < M) {
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          float* q = mine + (size_t)(t * MB + b) * SPLIT_STRIDE;
          __hip_atomic_store(q + threadIdx.x, vs[t][b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if constexpr (EPI == EPI_SWIGLU)
            __hip_atomic_store(q + 256 + threadIdx.x, ups[t][b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (n == 0)
          __hip_atomic_store(mine + (size_t)b * SPLIT_STRIDE + 512 + m, ss[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(sx->ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = prev == sx->n - 1;
      sm.sq[0][0] = last ? 1.f : 0.f;
      if (last) __hip_atomic_store(sx->ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (sm.sq[0][0] == 0.f) return;   // not last: another workgroup finishes the tiles
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      if (!(thr && 16 * b + m < M)) continue;
      float ss_sum = 0.f;
      float v_sum[TN], up_sum[TN];
#pragma unroll
      for (int t = 0; t < TN; ++t) v_sum[t] = up_sum[t] = 0.f;
      for (int i = 0; i < sx->n; ++i) {   // fixed order: bit-identical whoever arrives last
        const float* pi = sx->part + (size_t)i * TN * MB * SPLIT_STRIDE;
        const bool own = i == sx->idx;
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          const float* q = pi + (size_t)(t * MB + b) * SPLIT_STRIDE;
          v_sum[t] += own ? vs[t][b] : __hip_atomic_load(q + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if constexpr (EPI == EPI_SWIGLU)
            up_sum[t] += own ? ups[t][b]
                             : __hip_atomic_load(q + 256 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if constexpr (PRO != PRO_PLAIN)
          ss_sum += own ? ss[b]
                        : __hip_atomic_load(pi + (size_t)b * SPLIT_STRIDE + 512 + m, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
      }
      ss[b] = ss_sum;
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        vs[t][b] = v_sum[t];
        ups[t][b] = up_sum[t];
      }
    }
  }
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    const int row = 16 * b + m;
    const bool live = thr && row < M;
    float inv = 1.f;
    if constexpr (PRO != PRO_PLAIN) inv = rsqrtf(ss[b] / (float)K + p.eps);
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int tile = tile0 + t;
      float v = vs[t][b];
      const float up = ups[t][b];
      float vpartner = 0.f;
      if constexpr (EPI == EPI_ROPE) vpartner = __shfl_xor(v, 1, 64);   // every lane takes part
      if (live && tile < T) {
        v *= inv;
        const int col = tile * 16 + n;
        if constexpr (EPI == EPI_SWIGLU) {
          st16<false>(p.out + (size_t)row * p.ldo + col, silu(v) * (up * inv));
        } else if constexpr (EPI == EPI_RESID) {
          st16<false>(p.res + (size_t)row * N + col, v + e_res[t][b]);
        } else if constexpr (EPI == EPI_ROPE) {
          const RopeEpi& re = p.re;
          const int D = re.D, half = D >> 1;
          const int h = col / D, pp = col - h * D;
          const int64_t blk = e_slot[b] / re.BS;
          const int off = (int)(e_slot[b] - blk * re.BS);
          v += e_b[t];
          if (h < re.Hq + re.Hkv) {
            const float partner = fmaf(vpartner, inv, e_bp[t]);
            const int i = pp >> 1, hi = pp & 1;
            const float y = hi ? fmaf(v, e_c[t][b], partner * e_s[t][b]) : fmaf(v, e_c[t][b], -partner * e_s[t][b]);
            const int d = i + hi * half;
            uint16_t* dst = (h < re.Hq) ? p.out + ((size_t)row * re.Hq + h) * D + d
                                        : re.k_cache + ((size_t)blk * re.Hkv + (h - re.Hq)) * re.BS * D +
                                              rt::kc_elem(re.BS, off, d);
            st16<false>(dst, y);
          } else {
            const int hv = h - re.Hq - re.Hkv;
            st16<false>(re.v_cache + (((size_t)blk * re.Hkv + hv) * D + pp) * re.BS + off, v);
          }
        } else {
          st16<false>(p.out + (size_t)row * p.ldo + col, v);
        }
      }
    }
  }
}
}  // namespace skinny
