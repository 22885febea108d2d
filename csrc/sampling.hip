// K6: fused sampler — greedy / temperature / top-k / top-p, graph-safe RNG, multi-CU.
//
// Sampling is Gumbel-max: token = argmax(z_i + g_i) over the allowed set, z = (logit - max)/T,
// g_i = -log(-log(u_i)), u_i a counter-based hash of (seed, offset, i): no RNG state, so a
// captured hipGraph replays deterministically and a knight's stream depends only on
// (seed, knight, position) (the engine passes each row's token position as `offset`).
//
// Each row is split into C chunks handled by C workgroups (a single workgroup per row is
// LDS-atomic-bound: 2 x 128K histogram atomics on one CU), in six graph-capturable launches:
//   1 stats  : per-chunk max/argmax, and the chunk's best Gumbel score over ALL tokens (B x C)
//   2 accept : fast path. j* = argmax(z + g) over the whole vocabulary is the nucleus sample
//              whenever j* lies in the nucleus, i.e. when the mass of the tokens strictly more
//              likely than j* is below p * total (then the argmax over the nucleus is j*).
//              j* is itself a softmax draw, so that holds with probability >= top_p (95 % at
//              top_p 0.95). One pass sums both masses; the last-arriving chunk decides, writes
//              the token and raises the row's `done` flag. Greedy and unfiltered rows finish
//              here too; launches 3-6 return at once for a done row.  (grid B x C)
//   3 hist   : coarse 2048-bin histogram of z over [-ZR, 0] (count + probability mass),
//              chunk-local in LDS then merged with one global atomic per non-empty bin
//   4 select : per row, block-scan the histogram -> the bin where top-k (count) or top-p
//              (mass) crosses                                          (grid B)
//   5 refine : 2048-bin sub-histogram of that one bin                 (grid B x C)
//   6 final  : threshold from the sub-histogram, Gumbel-argmax over the chunk, then the
//              last-arriving chunk of each row reduces the partials   (grid B x C)
// Threshold resolution ZR/4M ~ 7e-6 in z; every pass uses 16-byte vector loads (G13).
// Bit-for-bit RNG twin: theroundtaible_amd/ops/reference.py::uniform_tensor.
#include "common.h"

namespace {
constexpr int NB = 2048;
constexpr int NT = 256;
constexpr int C = 32;       // chunks (workgroups) per row
constexpr float ZR = 30.f;  // exp(-30) * 128K < 1e-8 of the mass: ignored

// per-row workspace layout (floats / ints interchangeable, 4 bytes each)
constexpr int W_MAX = 0;                 // [C] chunk max
constexpr int W_ARG = W_MAX + C;         // [C] chunk argmax (int)
constexpr int W_GV = W_ARG + C;          // [C] chunk best Gumbel score v/T + g
constexpr int W_GI = W_GV + C;           // [C] its token (int)
// [W_HC, W_ROW) is zeroed by launch 1 (its chunks write only the words above)
constexpr int W_HC = W_GI + C;           // [NB] coarse count
constexpr int W_HM = W_HC + NB;          // [NB] coarse mass
constexpr int W_SC = W_HM + NB;          // [NB] sub count
constexpr int W_SM = W_SC + NB;          // [NB] sub mass
constexpr int W_SEL = W_SM + NB;         // bsel(int), by_count(int), need(float), row max(float)
constexpr int W_PV = W_SEL + 4;          // [C] partial score
constexpr int W_PI = W_PV + C;           // [C] partial index (int)
constexpr int W_CNT = W_PI + C;          // arrival counter (int)
constexpr int W_DONE = W_CNT + 1;        // row sampled by the accept pass (int)
constexpr int W_CNT2 = W_CNT + 2;        // accept-pass arrival counter (int)
constexpr int W_SUM = W_CNT + 4;         // mass above j*, total mass (accept-pass accumulators)
constexpr int W_ROW = W_SUM + 4;         // floats per row

RT_DEVICE uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
RT_DEVICE float gumbel(uint64_t key, uint32_t i) {
  const uint64_t z = mix64((uint64_t)i + key);
  const float u = ((float)(uint32_t)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
  return -__logf(-__logf(u));
}

template <typename T, bool VEC, typename F>
RT_DEVICE void for_chunk(const T* row, int lo, int hi, F&& f) {
  // lo is a multiple of 8 (chunk boundaries are), so the vector path stays aligned
  if constexpr (VEC && sizeof(T) == 2) {
    const int nv = (hi - lo) >> 3;
    const rt::short8* p = reinterpret_cast<const rt::short8*>(row + lo);
    for (int c = threadIdx.x; c < nv; c += NT) {
      const rt::short8 v = p[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) f(lo + c * 8 + j, rt::bf2f((uint16_t)v[j]));
    }
    for (int i = lo + (nv << 3) + threadIdx.x; i < hi; i += NT) f(i, rt::DT<T>::load(row + i));
  } else if constexpr (VEC) {
    const int nv = (hi - lo) >> 2;
    const float4* p = reinterpret_cast<const float4*>(row + lo);
    for (int c = threadIdx.x; c < nv; c += NT) {
      const float4 v = p[c];
      f(lo + c * 4 + 0, v.x);
      f(lo + c * 4 + 1, v.y);
      f(lo + c * 4 + 2, v.z);
      f(lo + c * 4 + 3, v.w);
    }
    for (int i = lo + (nv << 2) + threadIdx.x; i < hi; i += NT) f(i, rt::DT<T>::load(row + i));
  } else {
    for (int i = lo + threadIdx.x; i < hi; i += NT) f(i, rt::DT<T>::load(row + i));
  }
}

struct ArgMax {
  float v;
  int i;
};
RT_DEVICE void am_merge(ArgMax& a, float v, int i) {
  if (v > a.v || (v == a.v && i < a.i)) {
    a.v = v;
    a.i = i;
  }
}
RT_DEVICE ArgMax block_argmax(ArgMax a, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am_merge(a, __shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64));
  __syncthreads();
  if (lane == 0) {
    sv[wid] = a.v;
    si[wid] = a.i;
  }
  __syncthreads();
  ArgMax b{lane < NT / 64 ? sv[lane] : -INFINITY, lane < NT / 64 ? si[lane] : 0x7fffffff};
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am_merge(b, __shfl_xor(b.v, o, 64), __shfl_xor(b.i, o, 64));
  return b;
}

RT_DEVICE void chunk_range(int V, int c, int& lo, int& hi) {
  const int per = ((V + C - 1) / C + 7) & ~7;
  lo = min(V, c * per);
  hi = min(V, lo + per);
}

RT_DEVICE float row_max(const float* ws) {
  float m = -INFINITY;
  for (int c = 0; c < C; ++c) m = fmaxf(m, ws[W_MAX + c]);
  return m;
}

// ---- 1: chunk max / argmax -----------------------------------------------------------------
template <typename T, bool VEC>
__global__ void __launch_bounds__(NT) smp_stats(float* __restrict__ ws, const T* __restrict__ logits, int V,
                                                int64_t ld, const float* __restrict__ temperature,
                                                const int64_t* __restrict__ seeds,
                                                const int64_t* __restrict__ offsets) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int b = blockIdx.x, c = blockIdx.y;
  float* w = ws + (size_t)b * W_ROW;
  // zero this chunk's share of the row's histogram / counter region (replaces a per-call
  // memset launch; launches 2-5 are stream-ordered after this one)
  {
    const int z0 = W_HC, zn = W_ROW - W_HC, per = (zn + C - 1) / C;
    const int lo_z = z0 + c * per, hi_z = min(z0 + zn, lo_z + per);
    for (int i = lo_z + threadIdx.x; i < hi_z; i += NT) w[i] = 0.f;
  }
  int lo, hi;
  chunk_range(V, c, lo, hi);
  ArgMax a{-INFINITY, 0x7fffffff};
  const float temp = temperature[b];
  if (temp > 0.f) {   // also the chunk's best Gumbel score over every token (accept pass)
    const float invT = 1.f / temp;
    const uint64_t key = mix64((uint64_t)seeds[b] ^ mix64((uint64_t)offsets[b]));
    ArgMax gb{-INFINITY, 0x7fffffff};
    for_chunk<T, VEC>(logits + (size_t)b * ld, lo, hi, [&](int i, float v) {
      am_merge(a, v, i);
      am_merge(gb, v * invT + gumbel(key, (uint32_t)i), i);
    });
    gb = block_argmax(gb, sv, si);
    if (threadIdx.x == 0) {
      w[W_GV + c] = gb.v;
      reinterpret_cast<int*>(w)[W_GI + c] = gb.i;
    }
  } else {
    for_chunk<T, VEC>(logits + (size_t)b * ld, lo, hi, [&](int i, float v) { am_merge(a, v, i); });
  }
  a = block_argmax(a, sv, si);
  if (threadIdx.x == 0) {
    w[W_MAX + c] = a.v;
    reinterpret_cast<int*>(w)[W_ARG + c] = a.i;
  }
}

// ---- 2: accept pass (fast path, see the header) -------------------------------------------------
template <typename T, bool VEC>
__global__ void __launch_bounds__(NT) smp_accept(int64_t* __restrict__ out, float* __restrict__ ws,
                                                 const T* __restrict__ logits, int V, int64_t ld,
                                                 const float* __restrict__ temperature,
                                                 const float* __restrict__ top_p, const int* __restrict__ top_k) {
  __shared__ float red[8];
  const int b = blockIdx.x, c = blockIdx.y;
  float* w = ws + (size_t)b * W_ROW;
  int* wi = reinterpret_cast<int*>(w);
  const float temp = temperature[b];
  const int k = top_k[b];
  const float p = top_p[b];
  const bool use_k = k > 0 && k < V;
  if (!(temp > 0.f) || (!use_k && !(p < 1.f))) {   // greedy, or nothing filtered: decided now
    if (c == 0 && threadIdx.x == 0) {
      ArgMax r{-INFINITY, 0x7fffffff};
      for (int j = 0; j < C; ++j) {
        if (temp > 0.f) am_merge(r, w[W_GV + j], wi[W_GI + j]);
        else am_merge(r, w[W_MAX + j], wi[W_ARG + j]);
      }
      if (r.i < 0 || r.i >= V) {   // no finite score: the row argmax
        r = ArgMax{-INFINITY, 0x7fffffff};
        for (int j = 0; j < C; ++j) am_merge(r, w[W_MAX + j], wi[W_ARG + j]);
      }
      out[b] = r.i;
      wi[W_DONE] = 1;
    }
    return;
  }
  if (use_k) return;   // top-k rows take the histogram path
  ArgMax g{-INFINITY, 0x7fffffff};
  for (int j = 0; j < C; ++j) am_merge(g, w[W_GV + j], wi[W_GI + j]);
  if (g.i < 0 || g.i >= V) return;   // no finite score: the histogram path decides
  const float mx = row_max(w), invT = 1.f / temp;
  const T* row = logits + (size_t)b * ld;
  const float vj = rt::DT<T>::load(row + g.i);
  int lo, hi;
  chunk_range(V, c, lo, hi);
  float above = 0.f, total = 0.f;
  for_chunk<T, VEC>(row, lo, hi, [&](int, float v) {
    const float e = __expf((v - mx) * invT);
    total += e;
    above += v > vj ? e : 0.f;
  });
  above = rt::block_sum(above, red);
  total = rt::block_sum(total, red);
  if (threadIdx.x == 0) {
    atomicAdd(&w[W_SUM], above);
    atomicAdd(&w[W_SUM + 1], total);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(&wi[W_CNT2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == C - 1) {   // every chunk's sums are in: decide the row
      const float A = __hip_atomic_load(&w[W_SUM], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const float Z = __hip_atomic_load(&w[W_SUM + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (A < p * Z) {
        out[b] = g.i;
        __hip_atomic_store(&wi[W_DONE], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ---- 2 / 4: (sub-)histograms ---------------------------------------------------------------
template <typename T, bool VEC, bool SUB>
__global__ void __launch_bounds__(NT) smp_hist(float* __restrict__ ws, const T* __restrict__ logits, int V, int64_t ld,
                                               const float* __restrict__ temperature, const float* __restrict__ top_p,
                                               const int* __restrict__ top_k) {
  __shared__ float hc[NB], hm[NB];
  const int b = blockIdx.x, c = blockIdx.y;
  float* w = ws + (size_t)b * W_ROW;
  const float temp = temperature[b];
  const int k = top_k[b];
  if (!(temp > 0.f) || !((k > 0 && k < V) || top_p[b] < 1.f)) return;
  if (reinterpret_cast<const int*>(w)[W_DONE]) return;   // sampled by the accept pass
  int bsel = 0;
  if constexpr (SUB) {
    bsel = reinterpret_cast<const int*>(w)[W_SEL];
    if (bsel >= NB) return;
  }
  for (int i = threadIdx.x; i < NB; i += NT) {
    hc[i] = 0.f;
    hm[i] = 0.f;
  }
  __syncthreads();
  const float mx = row_max(w), invT = 1.f / temp, scale = NB / ZR;
  const float top_edge = -(float)bsel / scale;
  const float sub = scale * NB;
  int lo, hi;
  chunk_range(V, c, lo, hi);
  for_chunk<T, VEC>(logits + (size_t)b * ld, lo, hi, [&](int, float v) {
    const float z = (v - mx) * invT;
    const float fb = -z * scale;
    if constexpr (SUB) {
      if (fb >= (float)bsel && fb < (float)(bsel + 1)) {
        int sb = (int)((top_edge - z) * sub);
        sb = sb < 0 ? 0 : (sb >= NB ? NB - 1 : sb);
        atomicAdd(&hc[sb], 1.f);
        atomicAdd(&hm[sb], __expf(z));
      }
    } else if (fb < (float)NB) {
      const int bin = (int)fb;
      atomicAdd(&hc[bin], 1.f);
      atomicAdd(&hm[bin], __expf(z));
    }
  });
  __syncthreads();
  float* gc = w + (SUB ? W_SC : W_HC);
  float* gm = w + (SUB ? W_SM : W_HM);
  for (int i = threadIdx.x; i < NB; i += NT) {
    if (hc[i] != 0.f) {
      atomicAdd(gc + i, hc[i]);
      atomicAdd(gm + i, hm[i]);
    }
  }
}

// First bin whose inclusive prefix of `a` reaches ta or of `bm` reaches tb (1024 threads, 2 bins each).
RT_DEVICE int first_crossing(const float* a, const float* bm, float ta, float tb, float* scr, int* res, float* pa,
                             float* pb) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const float a0 = a[2 * t], a1 = a[2 * t + 1], b0 = bm[2 * t], b1 = bm[2 * t + 1];
  float sa = a0 + a1, sb = b0 + b1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float xa = __shfl_up(sa, o, 64), xb = __shfl_up(sb, o, 64);
    if (lane >= o) {
      sa += xa;
      sb += xb;
    }
  }
  __syncthreads();
  if (lane == 63) {
    scr[wid] = sa;
    scr[32 + wid] = sb;
  }
  if (t == 0) *res = NB;
  __syncthreads();
  float oa = 0.f, ob = 0.f;
  for (int w = 0; w < wid; ++w) {
    oa += scr[w];
    ob += scr[32 + w];
  }
  const float ia = oa + sa, ib = ob + sb, ea = ia - a0 - a1, eb = ib - b0 - b1;
  int cross = NB;
  if (ea + a0 >= ta || eb + b0 >= tb) cross = 2 * t;
  else if (ia >= ta || ib >= tb) cross = 2 * t + 1;
  if (cross < NB) atomicMin(res, cross);
  __syncthreads();
  const int cb = *res;
  if (cb < NB && (cb >> 1) == t) {
    *pa = (cb & 1) ? ea + a0 : ea;
    *pb = (cb & 1) ? eb + b0 : eb;
  }
  __syncthreads();
  return cb;
}

// ---- 3: select the threshold bin ---------------------------------------------------------------
__global__ void __launch_bounds__(1024) smp_select(float* __restrict__ ws, int V, const float* __restrict__ temperature,
                                                   const float* __restrict__ top_p, const int* __restrict__ top_k) {
  __shared__ float scr[64];
  __shared__ int sres;
  __shared__ float spa, spb;
  const int b = blockIdx.x;
  float* w = ws + (size_t)b * W_ROW;
  int* wi = reinterpret_cast<int*>(w);
  const int k = top_k[b];
  const float p = top_p[b];
  if (!(temperature[b] > 0.f) || !((k > 0 && k < V) || p < 1.f) || wi[W_DONE]) {
    if (threadIdx.x == 0) wi[W_SEL] = NB;
    return;
  }
  const float* hc = w + W_HC;
  const float* hm = w + W_HM;
  float tm = 0.f;
  for (int i = threadIdx.x; i < NB; i += 1024) tm += hm[i];
  tm = rt::block_sum(tm, scr);
  __syncthreads();
  const bool use_k = k > 0 && k < V;
  const float tk = use_k ? (float)k : 3.0e38f;
  int bk = NB;
  float pre_c = 0.f, zk_mass = tm;
  if (use_k) {
    bk = first_crossing(hc, hm, tk, 3.0e38f, scr, &sres, &spa, &spb);
    if (bk < NB) {
      zk_mass = spb + hm[bk];
      pre_c = spa;
    }
  }
  const float tp = p < 1.f ? p * zk_mass : 3.0e38f;
  int bp = NB;
  float pre_m = 0.f;
  if (p < 1.f) {
    bp = first_crossing(hc, hm, 3.0e38f, tp, scr, &sres, &spa, &spb);
    pre_m = spb;
  }
  if (threadIdx.x == 0) {
    if (bk <= bp) {
      wi[W_SEL] = bk;
      wi[W_SEL + 1] = 1;
      w[W_SEL + 2] = tk - pre_c;
    } else {
      wi[W_SEL] = bp;
      wi[W_SEL + 1] = 0;
      w[W_SEL + 2] = tp - pre_m;
    }
  }
}

// ---- 5: threshold + Gumbel argmax + last-arriver reduction --------------------------------------
template <typename T, bool VEC>
__global__ void __launch_bounds__(1024) smp_final(int64_t* __restrict__ out, float* __restrict__ ws,
                                                  const T* __restrict__ logits, int V, int64_t ld,
                                                  const float* __restrict__ temperature,
                                                  const int64_t* __restrict__ seeds,
                                                  const int64_t* __restrict__ offsets) {
  __shared__ float scr[64];
  __shared__ int sres;
  __shared__ float spa, spb;
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ int last;
  const int b = blockIdx.x, c = blockIdx.y;
  float* w = ws + (size_t)b * W_ROW;
  int* wi = reinterpret_cast<int*>(w);
  const float temp = temperature[b];
  if (wi[W_DONE]) return;   // greedy / unfiltered / accepted: out[b] written by launch 2
  const float mx = row_max(w), invT = 1.f / temp, scale = NB / ZR;
  float zthr = -INFINITY;
  const int bsel = wi[W_SEL];
  if (bsel < NB) {
    const bool by_count = wi[W_SEL + 1] != 0;
    const float need = w[W_SEL + 2];
    const int cb = by_count ? first_crossing(w + W_SC, w + W_SM, need, 3.0e38f, scr, &sres, &spa, &spb)
                            : first_crossing(w + W_SC, w + W_SM, 3.0e38f, need, scr, &sres, &spa, &spb);
    const int cc = cb < NB ? cb : NB - 1;
    zthr = -(float)bsel / scale - (float)(cc + 1) / (scale * NB);
  }
  const uint64_t key = mix64((uint64_t)seeds[b] ^ mix64((uint64_t)offsets[b]));
  int lo, hi;
  chunk_range(V, c, lo, hi);
  ArgMax a{-INFINITY, 0x7fffffff};
  // 1024 threads walk the chunk (NT is 256 in for_chunk's stride: walk 4 sub-ranges)
  const T* row = logits + (size_t)b * ld;
  for (int i = lo + threadIdx.x; i < hi; i += 1024) {
    const float z = (rt::DT<T>::load(row + i) - mx) * invT;
    if (z >= zthr) am_merge(a, z + gumbel(key, (uint32_t)i), i);
  }
  // block argmax over 16 waves
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am_merge(a, __shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64));
  if (lane == 0) {
    sv[wid] = a.v;
    si[wid] = a.i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ArgMax bm{-INFINITY, 0x7fffffff};
    for (int j = 0; j < 16; ++j) am_merge(bm, sv[j], si[j]);
    // publish this chunk's partial with sc1 (write-through) stores, drain them, then count
    // arrivals; the last arriver reads every partial with sc1 loads (MI355X_MICROARCH "Valid
    // forms" row 1: no L2 writeback/invalidate fences needed)
    __hip_atomic_store(&w[W_PV + c], bm.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&wi[W_PI + c], bm.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(&wi[W_CNT], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (prev == C - 1);
    if (last) {
      ArgMax r{-INFINITY, 0x7fffffff};
      for (int j = 0; j < C; ++j)
        am_merge(r, __hip_atomic_load(&w[W_PV + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&wi[W_PI + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (r.i == 0x7fffffff) {  // empty allowed set (rounding): fall back to the row argmax
        for (int j = 0; j < C; ++j) am_merge(r, w[W_MAX + j], wi[W_ARG + j]);
      }
      out[b] = r.i;
    }
  }
}
}  // namespace

int sample_workspace_floats(int B) { return B * W_ROW; }

int launch_sample(int64_t* out, const void* logits, bool is_bf16, int B, int V, int64_t ld_row,
                  const float* temperature, const float* top_p, const int* top_k, const int64_t* seeds,
                  const int64_t* offsets, float* ws, hipStream_t stream) {
  if (B == 0) return 0;
  const size_t esz = is_bf16 ? 2 : 4;
  const bool vec = ((uintptr_t)logits % 16 == 0) && ((ld_row * esz) % 16 == 0);
  const dim3 g2(B, C);
#define RT_SMP(TT, VV)                                                                                              \
  do {                                                                                                              \
    hipLaunchKernelGGL((smp_stats<TT, VV>), g2, dim3(NT), 0, stream, ws, (const TT*)logits, V, ld_row,             \
                       temperature, seeds, offsets);                                                                \
    hipLaunchKernelGGL((smp_accept<TT, VV>), g2, dim3(NT), 0, stream, out, ws, (const TT*)logits, V, ld_row,        \
                       temperature, top_p, top_k);                                                                  \
    hipLaunchKernelGGL((smp_hist<TT, VV, false>), g2, dim3(NT), 0, stream, ws, (const TT*)logits, V, ld_row,        \
                       temperature, top_p, top_k);                                                                  \
    hipLaunchKernelGGL(smp_select, dim3(B), dim3(1024), 0, stream, ws, V, temperature, top_p, top_k);              \
    hipLaunchKernelGGL((smp_hist<TT, VV, true>), g2, dim3(NT), 0, stream, ws, (const TT*)logits, V, ld_row,         \
                       temperature, top_p, top_k);                                                                  \
    hipLaunchKernelGGL((smp_final<TT, VV>), g2, dim3(1024), 0, stream, out, ws, (const TT*)logits, V, ld_row,       \
                       temperature, seeds, offsets);                                                                \
  } while (0)
  if (is_bf16) {
    if (vec) RT_SMP(uint16_t, true);
    else RT_SMP(uint16_t, false);
  } else {
    if (vec) RT_SMP(float, true);
    else RT_SMP(float, false);
  }
#undef RT_SMP
  return 0;
}
