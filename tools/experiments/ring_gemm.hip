// EXPERIMENT (microbenchmark only): decode GEMM (M <= 16) with a dedicated LOADER wave streaming
// weights into an LDS ring by LDS-DMA (global_load_lds_dwordx4, no VGPRs) and CONSUMER waves doing
// the MFMAs from LDS. Question it answers for the persistent-layer design (README "Where the
// remaining decode time goes"): can one workgroup per CU keep the HBM stream running across tile
// epilogues when only the consumers ever drain their own memory ops?
//
// Layout: the fragment-shuffled weights of skinny_core.h (one k-step of a 16-column tile = 1 KiB,
// lane-linear). Ring: NSLOT slots x KSC k-steps. Protocol (all in LDS, no workgroup barrier
// after the prologue, so the loader never waits for consumers except for a free slot):
//   loader : chunk g -> slot g % NSLOT; waits freecnt[slot] >= NCONS * (g / NSLOT); issues KSC
//            glds; once chunk g - DEPTH has landed (counted vmcnt) publishes full[slot] = g + 1.
//   consumer q: waits full[slot] >= g + 1, reads its k-steps' fragments (ds_read_b128), MFMAs with
//            the activation fragments (prefetched two chunks ahead), releases the slot (LDS add).
//   per tile: consumers leave partials in LDS (double-buffered by tile parity); the last of the
//            NCONS to arrive sums them and stores the 16 output columns.
#include "common.h"

namespace {
using rt::bf16x8;
using rt::float4_;
using rt::short8;

constexpr int NCONS = 4;      // consumer waves
// variants (microbenchmark sweep): KSC = k-steps per ring slot, NSLOT slots, DEPTH = chunks the
// loader keeps in flight before publishing, AUX = cache policy of the LDS-DMA loads (2 = nt)

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

RT_DEVICE int lds_load(const int* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }

// Loader-side LDS flag access through asm: a compiler-visible LDS access after global_load_lds
// makes hipcc wait vmcnt(0) first (the DMA writes LDS), which would serialise the whole ring.
RT_DEVICE uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
RT_DEVICE int lds_read_asm(const int* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
RT_DEVICE void lds_add_asm(int* p, int v) {
  asm volatile("ds_add_u32 %0, %1" : : "v"(lds_addr(p)), "v"(v) : "memory");
}

template <int N>
RT_DEVICE void wait_vmcnt() {   // s_waitcnt vmcnt(N), other counters untouched
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int KSC, int NSLOT>
struct RingSmem {
  short8 ring[NSLOT][KSC][64];
  float red[2][NCONS][16][17];
  int full[NSLOT];
  int freecnt[NSLOT];
  int done[2];
};

template <int KSC, int NSLOT, int DEPTH, int AUX, int NL>
__global__ void __launch_bounds__(64 * (NL + NCONS)) ring_gemm_kernel(uint16_t* __restrict__ out,
                                                                    const uint16_t* __restrict__ x,
                                                                    const short8* __restrict__ Ws, int M, int N, int K) {
  __shared__ RingSmem<KSC, NSLOT> sm;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nsteps = K / 32, nchunks = nsteps / KSC, ntiles = N / 16;
  if (threadIdx.x < NSLOT) {
    sm.full[threadIdx.x] = 0;
    sm.freecnt[threadIdx.x] = 0;
  }
  if (threadIdx.x < 2) sm.done[threadIdx.x] = 0;
  __syncthreads();

  if (wid < NL) {
    // ---------------- loaders: loader l streams k-steps j = l, l + NL, ... of every chunk ----------------
    constexpr int PL = KSC / NL;
    int g = 0;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
      const short8* wt = Ws + (size_t)t * nsteps * 64;
      for (int c = 0; c < nchunks; ++c, ++g) {
        const int s = g % NSLOT;
        if (g >= NSLOT) {
          const int need = NCONS * (g / NSLOT);
          while (lds_read_asm(&sm.freecnt[s]) < need) __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int j = wid + NL * u;
          __builtin_amdgcn_global_load_lds((glb_void*)(wt + (size_t)(c * KSC + j) * 64 + lane),
                                           (lds_void*)&sm.ring[s][j][0], 16, 0, AUX);
        }
        if (g >= DEPTH) {
          wait_vmcnt<DEPTH * PL>();
          if (lane == 0) lds_add_asm(&sm.full[(g - DEPTH) % NSLOT], 1);
        }
      }
    }
    wait_vmcnt<0>();
    if (lane == 0)
      for (int h = (g > DEPTH ? g - DEPTH : 0); h < g; ++h) lds_add_asm(&sm.full[h % NSLOT], 1);
    return;
  }

  // ---------------- consumers ----------------
  const int q = wid - NL, r = lane & 15, gq = lane >> 4;
  const uint16_t* xr = x + (size_t)(r < M ? r : 0) * K + 8 * gq;
  constexpr int PER = KSC / NCONS;   // k-steps per consumer per chunk
  int g = 0, tl = 0;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x, ++tl) {
    float4_ acc = {0.f, 0.f, 0.f, 0.f};
    short8 xc[PER], xn[PER];   // activation fragments of this chunk / the next (static indices)
    // unconditional loads (rows >= M read row 0, whose products land in output rows never
    // stored; the chunk index is clamped) so hipcc can count them and wait vmcnt(PER), not 0
    auto load_x = [&](short8* dst, int c) {
      const int cc = c < nchunks ? c : nchunks - 1;
#pragma unroll
      for (int u = 0; u < PER; ++u)
        dst[u] = *reinterpret_cast<const short8*>(xr + (cc * KSC + q + NCONS * u) * 32);
    };
    // one chunk: its ring slot -> registers, release, MFMAs with `xa`; the loads of chunk c + 1 go
    // to the other buffer first (two chunks per loop turn: no register copies, so the only waits
    // are for the buffer being consumed)
    auto step = [&](int c, const short8* xa, short8* xnext) {
      load_x(xnext, c + 1);
      const int s = g % NSLOT;
      while (lds_load(&sm.full[s]) < NL * (g / NSLOT + 1)) __builtin_amdgcn_s_sleep(1);
      short8 w[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) w[u] = sm.ring[s][q + NCONS * u][lane];
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): fragments are in registers before the release
      if (lane == 0) __atomic_fetch_add(&sm.freecnt[s], 1, __ATOMIC_RELAXED);
#pragma unroll
      for (int u = 0; u < PER; ++u)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xa[u]),
                                                      __builtin_bit_cast(bf16x8, w[u]), acc, 0, 0, 0);
      ++g;
    };
    load_x(xc, 0);
    int c = 0;
    for (; c + 1 < nchunks; c += 2) {
      step(c, xc, xn);
      step(c + 1, xn, xc);
    }
    if (c < nchunks) step(c, xc, xn);
    // partials -> LDS; the last consumer to arrive sums and stores
    const int par = tl & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) sm.red[par][q][4 * gq + i][r] = acc[i];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    int last = 0;
    if (lane == 0) last = __atomic_fetch_add(&sm.done[par], 1, __ATOMIC_ACQ_REL) == NCONS * (tl / 2 + 1) - 1;
    last = __shfl(last, 0, 64);
    if (last) {
      for (int e = lane; e < 16 * M; e += 64) {
        const int m = e >> 4, n = e & 15;
        float v = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < NCONS; ++w2) v += sm.red[par][w2][m][n];
        out[(size_t)m * N + t * 16 + n] = rt::f2bf(v);
      }
    }
  }
}
}  // namespace

int launch_ring_gemm(void* out, const void* x, const void* Ws, int M, int N, int K, int grid, int variant,
                     hipStream_t stream) {
  if (M < 1 || M > 16 || N % 16 || K % (32 * 8)) return -1;
  if (grid <= 0) grid = N / 16;
  const dim3 g(grid);
  auto* o = (uint16_t*)out;
  auto* xx = (const uint16_t*)x;
  auto* w = (const short8*)Ws;
#define RT_RG(KS, NS, DP, AX, NLV) \
  hipLaunchKernelGGL((ring_gemm_kernel<KS, NS, DP, AX, NLV>), g, dim3(64 * (NLV + NCONS)), 0, stream, o, xx, w, M, N, K)
  switch (variant) {
    case 1: RT_RG(8, 12, 6, 2, 1); break;
    case 2: RT_RG(8, 16, 7, 2, 1); break;
    case 3: RT_RG(8, 16, 12, 2, 2); break;
    case 4: RT_RG(8, 16, 12, 2, 4); break;
    case 5: RT_RG(8, 16, 14, 2, 8); break;
    default: RT_RG(8, 12, 6, 0, 1); break;
  }
#undef RT_RG
  return 0;
}
