// Decode-path linear layers (M <= 16 rows): y[M,N] = x[M,K] . W[N,K]^T on MFMA, with the
// layer's elementwise work fused in, so a decode layer needs no separate norm/act kernels.
//
// Weight layout ("fragment-shuffled", built once at load time by `shuffle_weight`):
//     Ws[N/16][K/32][64 lanes][8]   with  Ws[t][s][l][j] = W[16t + (l&15)][32s + 8(l>>4) + j]
// i.e. exactly the order in which the 64 lanes of a wave hold the B operand of
// v_mfma_f32_16x16x32_bf16. Every wave load instruction therefore reads 1 KiB of
// contiguous HBM and a workgroup streams its 16-row panel front to back — decode GEMMs
// are pure weight streams, so this is the whole game (on 288 GB HBM the extra copy next
// to the row-major prefill weights is affordable: +16 GB for an 8B knight).
//
// One workgroup = 16 output columns (32 W rows for SwiGLU) x all of K; its 4 waves take
// interleaved 32-deep k-steps (adjacent waves -> adjacent KiB), with the next UNROLL
// steps' loads issued before the current steps' MFMAs (register double-buffering). M is
// padded to the 16 MFMA rows. The waves' partial tiles are summed through LDS.
//
// Fusions:
//   prologue NORM : RMSNorm of the residual stream. The norm weight gamma is folded into W
//                   at load time, and 1/rms(x_m) factors out of the k-sum, so the kernel
//                   feeds raw x to the MFMA, accumulates sum(x^2) from the same fragments,
//                   and scales row m of the result by rsqrt(ss_m/K + eps) in the epilogue
//                   (no extra pass, no atomics: deterministic).
//   epilogue RESID: res[m,n] = bf16(acc + res[m,n])   (the residual add, in place)
//   epilogue SWIGLU: out[m,n] = silu(acc_gate) * acc_up,  W = [gate(I) ; up(I)]
//   epilogue ROPE  : the qkv projection. Its q/k weight rows are stored pair-interleaved per
//                   head (row 2i <- d=i, row 2i+1 <- d=i+D/2; `shuffle_weight(rope_heads=)`),
//                   so both halves of every rotate-half pair land in the same 16-column tile:
//                   the epilogue rotates them (fp32 cos|sin table), writes q to [M, Hq, D] and
//                   scatters k / v straight into the paged caches (k [blk][h][off][D], v
//                   transposed [blk][h][D][off]). Replaces the K2 rope/cache launch.
#include "common.h"

#include <cstdio>
#include <cstdlib>

namespace {
using rt::bf16x8;
using rt::float4_;
using rt::short8;


// PRO_NORM_ADD (tensor-parallel decode): the A operand is bf16(x + x2) — the residual plus the
// all-reduced row-parallel partial — and workgroup 0 writes that sum to `xo` (the next residual).
enum : int { PRO_PLAIN = 0, PRO_NORM = 1, PRO_NORM_ADD = 2 };
enum : int { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_ROPE = 3 };

struct RopeEpi {
  const int64_t* positions;  // [M]
  const float* cos_sin;      // [max_pos][D]: cos(D/2) | sin(D/2)
  uint16_t* k_cache;
  uint16_t* v_cache;
  const int64_t* slots;      // [M]
  int Hq, Hkv, D, BS;
};

RT_DEVICE float silu(float x) { return x / (1.f + __expf(-x)); }

// U = k-steps per wave per pipeline stage (x2 stages in flight)
template <int PRO, int EPI, int U>
struct Stage {
  short8 w[U];
  short8 w2[(EPI == EPI_SWIGLU) ? U : 1];
  short8 a[U];
  short8 b[(PRO == PRO_NORM_ADD) ? U : 1];
};

template <int PRO, int EPI, int NW, int U>
RT_DEVICE void issue(Stage<PRO, EPI, U>& st, const short8* __restrict__ wt, const short8* __restrict__ wt2,
                     const uint16_t* __restrict__ xr, const uint16_t* __restrict__ xr2, bool row_ok, int s0,
                     int nsteps, int lane) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int s = s0 + NW * u;
    if (s < nsteps) {
      st.w[u] = __builtin_nontemporal_load(wt + (size_t)s * 64 + lane);
      if constexpr (EPI == EPI_SWIGLU) st.w2[u] = __builtin_nontemporal_load(wt2 + (size_t)s * 64 + lane);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int s = s0 + NW * u;
    st.a[u] = (row_ok && s < nsteps) ? *reinterpret_cast<const short8*>(xr + s * 32) : short8{0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (PRO == PRO_NORM_ADD)
      st.b[u] = (row_ok && s < nsteps) ? *reinterpret_cast<const short8*>(xr2 + s * 32) : short8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

template <int PRO, int EPI, int NW, int U>
RT_DEVICE void consume(const Stage<PRO, EPI, U>& st, float4_& acc, float4_& acc2, float& ssq, int s0, int nsteps,
                       uint16_t* __restrict__ xo_r) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (s0 + NW * u < nsteps) {
      short8 av = st.a[u];
      if constexpr (PRO == PRO_NORM_ADD) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          av[j] = (short)rt::f2bf(rt::bf2f((uint16_t)st.a[u][j]) + rt::bf2f((uint16_t)st.b[u][j]));
        if (xo_r != nullptr) *reinterpret_cast<short8*>(xo_r + (s0 + NW * u) * 32) = av;
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

template <int PRO, int EPI, int NW, int U>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ x,
                                                          const short8* __restrict__ Ws, uint16_t* __restrict__ res,
                                                          int M, int N, int K, int ldo, float eps, RopeEpi re,
                                                          const uint16_t* __restrict__ x2, uint16_t* __restrict__ xo) {
  __shared__ float red[NW][(EPI == EPI_SWIGLU) ? 2 : 1][16][17];
  __shared__ float sq[NW][16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int tile = blockIdx.x;
  const int nsteps = K / 32;
  const bool row_ok = r < M;
  const uint16_t* xr = x + (size_t)(row_ok ? r : 0) * K + 8 * g;
  const uint16_t* xr2 = (PRO == PRO_NORM_ADD) ? x2 + (size_t)(row_ok ? r : 0) * K + 8 * g : nullptr;
  // workgroup 0 publishes the summed residual (rows < M only)
  uint16_t* xo_r = (PRO == PRO_NORM_ADD && blockIdx.x == 0 && row_ok && xo != nullptr) ? xo + (size_t)r * K + 8 * g
                                                                                      : nullptr;
  const short8* wt = Ws + (size_t)tile * nsteps * 64;
  const short8* wt2 = (EPI == EPI_SWIGLU) ? Ws + (size_t)(N / 16 + tile) * nsteps * 64 : nullptr;

  float4_ acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
  float ssq = 0.f;
  Stage<PRO, EPI, U> st0, st1;
  int s = wid;
  issue<PRO, EPI, NW, U>(st0, wt, wt2, xr, xr2, row_ok, s, nsteps, lane);
  for (;;) {
    const int sn = s + NW * U;
    if (sn < nsteps) issue<PRO, EPI, NW, U>(st1, wt, wt2, xr, xr2, row_ok, sn, nsteps, lane);
    consume<PRO, EPI, NW, U>(st0, acc, acc2, ssq, s, nsteps, xo_r);
    if (sn >= nsteps) break;
    s = sn;
    const int sn2 = s + NW * U;
    if (sn2 < nsteps) issue<PRO, EPI, NW, U>(st0, wt, wt2, xr, xr2, row_ok, sn2, nsteps, lane);
    consume<PRO, EPI, NW, U>(st1, acc, acc2, ssq, s, nsteps, xo_r);
    if (sn2 >= nsteps) break;
    s = sn2;
  }

  // C layout: acc[i] = C[m = 4g + i][n = r]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[wid][0][4 * g + i][r] = acc[i];
    if constexpr (EPI == EPI_SWIGLU) red[wid][(EPI == EPI_SWIGLU) ? 1 : 0][4 * g + i][r] = acc2[i];
  }
  if constexpr (PRO != PRO_PLAIN) {
    ssq += __shfl_xor(ssq, 16, 64);
    ssq += __shfl_xor(ssq, 32, 64);
    if (g == 0) sq[wid][r] = ssq;
  }
  __syncthreads();
  const int m = threadIdx.x >> 4, n = threadIdx.x & 15;
  if (threadIdx.x < 256 && m < M) {
    float v = 0.f, ss = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      v += red[w][0][m][n];
      if constexpr (PRO != PRO_PLAIN) ss += sq[w][m];
    }
    float inv = 1.f;
    if constexpr (PRO != PRO_PLAIN) inv = rsqrtf(ss / (float)K + eps);
    v *= inv;
    const int col = tile * 16 + n;
    if constexpr (EPI == EPI_SWIGLU) {
      const int u1 = (EPI == EPI_SWIGLU) ? 1 : 0;
      float up = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) up += red[w][u1][m][n];
      up *= inv;
      out[(size_t)m * ldo + col] = rt::f2bf(silu(v) * up);
    } else if constexpr (EPI == EPI_RESID) {
      uint16_t* rp = res + (size_t)m * N + col;
      *rp = rt::f2bf(v + rt::bf2f(*rp));
    } else if constexpr (EPI == EPI_ROPE) {
      const int D = re.D, half = D >> 1;
      const int h = col / D, p = col - h * D;
      const int64_t slot = re.slots[m];
      const int64_t blk = slot / re.BS;
      const int off = (int)(slot - blk * re.BS);
      if (h < re.Hq + re.Hkv) {
        float partner = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) partner += red[w][0][m][n ^ 1];
        partner *= inv;
        const int i = p >> 1, hi = p & 1;
        const float* cs = re.cos_sin + (size_t)re.positions[m] * D;
        const float c = cs[i], sn = cs[half + i];
        // pair (x1 = d i, x2 = d i+D/2): y1 = x1 c - x2 s ; y2 = x2 c + x1 s
        const float y = hi ? fmaf(v, c, partner * sn) : fmaf(v, c, -partner * sn);
        const int d = i + hi * half;
        uint16_t* dst = (h < re.Hq) ? out + ((size_t)m * re.Hq + h) * D + d
                                    : re.k_cache + (((size_t)blk * re.Hkv + (h - re.Hq)) * re.BS + off) * D + d;
        *dst = rt::f2bf(y);
      } else {
        const int hv = h - re.Hq - re.Hkv;
        re.v_cache[(((size_t)blk * re.Hkv + hv) * D + p) * re.BS + off] = rt::f2bf(v);
      }
    } else {
      out[(size_t)m * ldo + col] = rt::f2bf(v);
    }
  }
}

// Ws[t][s][l][j] = W[16t + (l&15)][32s + 8(l>>4) + j] (optionally W * gamma[k] folded in)
// If rope_rows > 0, output row r < rope_rows takes source row h*D + (p>>1) + (p&1)*D/2
// (r = h*D + p): the pair-interleaved q/k order the ROPE epilogue expects.
__global__ void shuffle_kernel(short8* __restrict__ Ws, const uint16_t* __restrict__ W,
                               const uint16_t* __restrict__ gamma, int N, int K, int rope_rows, int D) {
  const int nsteps = K / 32;
  const int64_t total = (int64_t)(N / 16) * nsteps * 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i & 63);
    const int64_t ts = i >> 6;
    const int s = (int)(ts % nsteps);
    const int64_t t = ts / nsteps;
    int row = (int)(16 * t + (l & 15));
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
    Ws[i] = v;
  }
}
}  // namespace

int launch_skinny_gemm(void* out, const void* x, const void* Ws, void* res, int M, int N, int K, int ldo, float eps,
                       int pro, int epi, const void* rope, const void* x2, void* xo, hipStream_t stream) {
  if (pro == PRO_NORM_ADD && x2 == nullptr) return -5;
  if (M < 1 || M > 16 || K % 32 || N % 16) return -1;
  RopeEpi re{};
  if (epi == EPI_ROPE) {
    if (rope == nullptr) return -3;
    re = *static_cast<const RopeEpi*>(rope);
    if (re.D % 16 || N != (re.Hq + 2 * re.Hkv) * re.D) return -4;
  }
  // Variant = (waves per workgroup NW, k-steps per stage U). Few column tiles (o/down/qkv
  // projections: <= ~1.5 workgroups per CU) -> 8 waves so each CU keeps enough weight
  // bytes in flight; wide GEMMs (gate_up, lm_head) -> 4. RT_SKINNY_CFG=<NW>x<U> (4x4, 8x4,
  // 8x8, 4x8) pins one for microbenchmarks (tools/microbench.py).
  static const int cfg_env = [] {
    const char* e = getenv("RT_SKINNY_CFG");
    if (!e) return 0;
    int nw = 0, u = 0;
    if (sscanf(e, "%dx%d", &nw, &u) != 2) return 0;
    return nw * 100 + u;
  }();
  const int cfg = cfg_env ? cfg_env : ((N / 16) >= 768 ? 404 : 804);
  dim3 grid(N / 16);
#define RT_SG(P, E)                                                                                          \
  do {                                                                                                       \
    switch (cfg) {                                                                                           \
      case 408: RT_SGV(P, E, 4, 8); break;                                                                   \
      case 804: RT_SGV(P, E, 8, 4); break;                                                                   \
      case 808: RT_SGV(P, E, 8, 8); break;                                                                   \
      default: RT_SGV(P, E, 4, 4); break;                                                                    \
    }                                                                                                        \
  } while (0)
#define RT_SGV(P, E, NWV, UV)                                                                                \
  hipLaunchKernelGGL((skinny_gemm_kernel<P, E, NWV, UV>), grid, dim3(NWV * 64), 0, stream, (uint16_t*)out,  \
                     (const uint16_t*)x, (const short8*)Ws, (uint16_t*)res, M, N, K, ldo, eps, re,               \
                     (const uint16_t*)x2, (uint16_t*)xo)
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

int launch_shuffle_weight(void* Ws, const void* W, const void* gamma, int N, int K, int rope_rows, int D,
                          hipStream_t stream) {
  if (K % 32 || N % 16 || rope_rows > N || (rope_rows > 0 && (D <= 0 || D % 2 || rope_rows % D))) return -1;
  const int64_t total = (int64_t)N * K / 8;
  int64_t grid = (total + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(shuffle_kernel, dim3((unsigned)grid), dim3(256), 0, stream, (short8*)Ws, (const uint16_t*)W,
                     (const uint16_t*)gamma, N, K, rope_rows, D);
  return 0;
}

int launch_skinny_gemm_rope(void* q_out, const void* x, const void* Ws, int M, int K, int pro, float eps,
                            const int64_t* positions, const float* cos_sin, void* k_cache, void* v_cache,
                            const int64_t* slots, int Hq, int Hkv, int D, int BS, const void* x2, void* xo,
                            hipStream_t stream) {
  const RopeEpi re{positions, cos_sin, (uint16_t*)k_cache, (uint16_t*)v_cache, slots, Hq, Hkv, D, BS};
  return launch_skinny_gemm(q_out, x, Ws, nullptr, M, (Hq + 2 * Hkv) * D, K, 0, eps, pro, EPI_ROPE, &re, x2, xo,
                            stream);
}
