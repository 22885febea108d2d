// K6: fused sampler — greedy / temperature / top-k / top-p, graph-safe RNG — and, in the
// captured decode step, the step's bookkeeping, in ONE launch (r02: six sampler launches +
// decode_advance = 47 us per step, profiles/r03/prof8.md).
//
// Sampling is Gumbel-max: token = argmax(z_i + g_i) over the allowed set, z = (logit - max)/T,
// g_i = -log(-log(u_i)), u_i a counter-based hash of (seed, offset, i): no RNG state, so a
// captured hipGraph replays deterministically and a knight's stream depends only on
// (seed, knight, position) (the engine passes each row's token position as `offset`).
//
// Grid (B, C): C workgroups per row stream one chunk each (chunk max / argmax, and the chunk's
// best Gumbel score over ALL its tokens), publish those 4 words write-through, and take a
// ticket; the row's LAST-arriving workgroup (the "decider", MI355X_MICROARCH sc1 hand-off
// table row 1) finishes the row alone:
//   * greedy / unfiltered rows: reduce the C chunk records;
//   * top-p rows, fast path: j* = argmax(z + g) over the whole vocabulary is the nucleus sample
//     whenever the mass of the tokens strictly more likely than j* is below p * total (then the
//     argmax over the nucleus is j*); j* is itself a softmax draw, so that holds with
//     probability >= top_p. One pass of the decider over the row sums both masses;
//   * otherwise (top-k, or a rejected j*): a 2048-bin histogram of z in LDS (count + mass) ->
//     the crossing bin -> a 2048-bin sub-histogram of that bin -> threshold -> Gumbel argmax over
//     the allowed set, all by the decider (coarse bins over the row's own z range, at most
//     [-ZR, 0]; threshold resolution range / 4M <= 7e-6 in z).
// The decider then writes the token and, with bookkeeping on (sample_advance), the decode_advance
// + decode_prep work of its row (out[step, b], ids, positions, lengths, next K/V slot, sampler
// offset, embedding row); the last decider of the launch bumps `step`. Every counter re-arms
// itself, so the workspace is zeroed once (ops.sample_workspace) and replays need no memset.
// Bit-for-bit RNG twin: theroundtaible_amd/ops/reference.py::uniform_tensor.
#include "common.h"

#include <cstdlib>

namespace {
constexpr int NB = 2048;
constexpr int NT = 512;     // threads per workgroup
constexpr int NWV = NT / 64;
constexpr int C = 32;       // chunks (workgroups) per row
constexpr float ZR = 30.f;  // exp(-30) * 128K < 1e-8 of the mass: ignored

// per-row workspace (4-byte words, floats / ints interchangeable)
constexpr int W_MAX = 0;                 // [C] chunk max
constexpr int W_ARG = W_MAX + C;         // [C] chunk argmax (int)
constexpr int W_GV = W_ARG + C;          // [C] chunk best Gumbel score v/T + g
constexpr int W_GI = W_GV + C;           // [C] its token (int)
constexpr int W_MIN = W_GI + C;          // [C] chunk min
constexpr int W_CNT = W_MIN + C;         // arrival ticket (int), re-armed by the decider
constexpr int W_SC = W_CNT + 1;          // histogram grid scale for the next launch (float, 0 = default)
constexpr int W_KB = W_CNT + 4;          // [C] chunk's top histogram bin floor(max * scale) (int)
constexpr int HB = 128;                  // histogram bins per chunk (the last one: everything lower)
constexpr float BW = 16.f;               // bins per unit of z = logit / T
constexpr int W_HIST = W_KB + C;         // [C][HB] chunk mass per bin, relative to the chunk max
// top-k rows with k <= KMAX: every chunk publishes its own top-k tokens (ties at its k-th key
// included up to LCAP), sorted by token id; the decider merges the C lists
constexpr int KMAX = 64;
constexpr int LCAP = 96;
constexpr int W_TKN = W_HIST + C * HB;   // [C] list length | truncated << 16 (int)
constexpr int W_TKK = W_TKN + C;         // [C] the chunk's k-th largest order key (int)
constexpr int W_TKL = W_TKK + C;         // [C][LCAP] order keys (int)
constexpr int W_TKI = W_TKL + C * LCAP;  // [C][LCAP] token ids (int)
constexpr int W_ROW = W_TKI + C * LCAP;  // words per row; after the B rows: the rows-done ticket
// LDS pool: the decider's histograms (hc, hm, hci, hmi) or, on top-k list rows, the chunk's
// order keys (phase 1) / the merged lists (decider)
constexpr int POOL_BYTES = NB * 4 * 3 + NB * 8;
constexpr int POOLK = POOL_BYTES / 4;
constexpr int NALLOW = NT;               // list path: at most this many allowed tokens (else the histogram path)
// which branch decided a row (RT_SMP_PROBE=5 writes it in place of the token; + PATH_EXACT_PASS
// when the accept test needed its exact pass over the row)
constexpr int PATH_PLAIN = 0, PATH_ACCEPT = 1, PATH_RESCAN = 2, PATH_CANDIDATES = 3, PATH_HISTOGRAM = 4,
              PATH_EXACT_PASS = 10;

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

// f(i, v) over [lo, hi) of a row, NT-strided, 16-byte loads when aligned (lo % 8 == 0)
template <typename T, bool VEC, typename F>
RT_DEVICE void for_range(const T* row, int lo, int hi, F&& f) {
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

// f(i, v) over a whole row [0, V): the decider's passes stream 256 KB on ONE CU, so every lane
// keeps UNR 16-byte loads in flight before consuming them (a load-use loop would pay one
// memory round trip per 16 bytes per lane).
template <typename T, bool VEC, typename F>
RT_DEVICE void for_row(const T* row, int V, F&& f) {
  if constexpr (VEC && sizeof(T) == 2) {
    constexpr int UNR = 8;
    const int nv = V >> 3;
    const rt::short8* p = reinterpret_cast<const rt::short8*>(row);
    int c0 = threadIdx.x;
    for (; c0 + (UNR - 1) * NT < nv; c0 += UNR * NT) {
      rt::short8 v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[u] = p[c0 + u * NT];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) f((c0 + u * NT) * 8 + j, rt::bf2f((uint16_t)v[u][j]));
    }
    for (int c = c0; c < nv; c += NT) {
      const rt::short8 v = p[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) f(c * 8 + j, rt::bf2f((uint16_t)v[j]));
    }
    for (int i = (nv << 3) + threadIdx.x; i < V; i += NT) f(i, rt::DT<T>::load(row + i));
  } else {
    for_range<T, VEC>(row, 0, V, f);
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
// Wave reductions on DPP lane permutes (VALU, a few cycles each) instead of ds_bpermute shuffles
// (an LDS round trip each): xor 1 and xor 2 as quad permutes, then the half-row and row mirrors
// pair the quads and the 8-lane halves (every lane of a 16-lane row then holds the row's
// result), and the four rows are read out with readlane (wave-uniform result). Fixed pairing
// order: deterministic.
constexpr int DPP_QUAD_1032 = 0xB1, DPP_QUAD_2301 = 0x4E, DPP_ROW_HALF_MIRROR = 0x141, DPP_ROW_MIRROR = 0x140;
template <int CTRL>
RT_DEVICE float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
RT_DEVICE int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
RT_DEVICE float rl(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}
RT_DEVICE float wave_sum_dpp(float v) {
  v += dpp_f<DPP_QUAD_1032>(v);
  v += dpp_f<DPP_QUAD_2301>(v);
  v += dpp_f<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_f<DPP_ROW_MIRROR>(v);
  return (rl(v, 0) + rl(v, 16)) + (rl(v, 32) + rl(v, 48));
}
RT_DEVICE float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f<DPP_QUAD_1032>(v));
  v = fmaxf(v, dpp_f<DPP_QUAD_2301>(v));
  v = fmaxf(v, dpp_f<DPP_ROW_HALF_MIRROR>(v));
  v = fmaxf(v, dpp_f<DPP_ROW_MIRROR>(v));
  return fmaxf(fmaxf(rl(v, 0), rl(v, 16)), fmaxf(rl(v, 32), rl(v, 48)));
}
RT_DEVICE ArgMax wave_argmax_dpp(ArgMax a) {
  am_merge(a, dpp_f<DPP_QUAD_1032>(a.v), dpp_i<DPP_QUAD_1032>(a.i));
  am_merge(a, dpp_f<DPP_QUAD_2301>(a.v), dpp_i<DPP_QUAD_2301>(a.i));
  am_merge(a, dpp_f<DPP_ROW_HALF_MIRROR>(a.v), dpp_i<DPP_ROW_HALF_MIRROR>(a.i));
  am_merge(a, dpp_f<DPP_ROW_MIRROR>(a.v), dpp_i<DPP_ROW_MIRROR>(a.i));
  ArgMax r{rl(a.v, 0), __builtin_amdgcn_readlane(a.i, 0)};
#pragma unroll
  for (int q = 16; q < 64; q += 16) am_merge(r, rl(a.v, q), __builtin_amdgcn_readlane(a.i, q));
  return r;
}
// block reductions: one value per wave through LDS, then every thread folds the NWV values in
// wave order (no second shuffle level)
RT_DEVICE float block_sum_dpp(float v, float* scr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum_dpp(v);
  __syncthreads();
  if (lane == 0) scr[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < NWV; ++w) t += scr[w];
  return t;
}
RT_DEVICE float block_max_dpp(float v, float* scr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_max_dpp(v);
  __syncthreads();
  if (lane == 0) scr[wid] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int w = 0; w < NWV; ++w) t = fmaxf(t, scr[w]);
  return t;
}
RT_DEVICE ArgMax block_argmax(ArgMax a, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  a = wave_argmax_dpp(a);
  __syncthreads();
  if (lane == 0) {
    sv[wid] = a.v;
    si[wid] = a.i;
  }
  __syncthreads();
  ArgMax b{sv[0], si[0]};
#pragma unroll
  for (int w = 1; w < NWV; ++w) am_merge(b, sv[w], si[w]);
  return b;
}

RT_DEVICE void chunk_range(int V, int c, int& lo, int& hi) {
  const int per = ((V + C - 1) / C + 7) & ~7;
  lo = min(V, c * per);
  hi = min(V, lo + per);
}

// order-preserving unsigned key of a float (larger value -> larger key; -inf > 0 = "no entry").
// lo = 16 for bf16 rows: the key's low half carries no order and is cleared, so equal values have
// equal keys whatever their sign (a negative value's ~u would otherwise set the low half to 0xFFFF
// and every tie at a threshold t with a clear low half would compare ABOVE t)
RT_DEVICE uint32_t okey(float v, int lo) {
  const uint32_t u = __float_as_uint(v);
  return ((u & 0x80000000u) ? ~u : (u | 0x80000000u)) & ~((1u << lo) - 1u);
}
RT_DEVICE float okey_value(uint32_t k, int lo) {
  return __uint_as_float(((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k) & ~((1u << lo) - 1u));
}

// The largest t with #{i < n : keys[i] >= t} >= need (the need-th largest key; need <= n), two
// bits per step, down to bit lo (16 for bf16 values: their keys' low half carries no order).
// Counts are wave ballots (a compare + a scalar popcount per key, no shuffles), one barrier per
// step (scr: 2 x 3 x NWV ints, alternating so a step never overwrites what a slower wave reads).
RT_DEVICE uint32_t kth_key(const uint32_t* keys, int n, int need, int lo, int* scr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t t = 0;
  int par = 0;
  for (int bit = 30; bit >= lo; bit -= 2, par ^= 1) {
    const uint32_t c1 = t | (1u << bit), c2 = t | (2u << bit), c3 = t | (3u << bit);
    int n1 = 0, n2 = 0, n3 = 0;
    for (int i0 = 0; i0 < n; i0 += 8 * NT) {
      uint32_t kk[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + (int)threadIdx.x + j * NT;
        kk[j] = i < n ? keys[i] : 0u;     // 0: below every value's key
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        n1 += __popcll(__ballot(kk[j] >= c1));
        n2 += __popcll(__ballot(kk[j] >= c2));
        n3 += __popcll(__ballot(kk[j] >= c3));
      }
    }
    int* sc = scr + par * 3 * NWV;
    if (lane == 0) {
      sc[wid] = n1;
      sc[NWV + wid] = n2;
      sc[2 * NWV + wid] = n3;
    }
    __syncthreads();
    n1 = n2 = n3 = 0;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      n1 += sc[w];
      n2 += sc[NWV + w];
      n3 += sc[2 * NWV + w];
    }
    t = n3 >= need ? c3 : (n2 >= need ? c2 : (n1 >= need ? c1 : t));
  }
  __syncthreads();   // the caller may rewrite keys / scr
  return t;
}

// First bin whose inclusive prefix of `a` reaches ta or of `bm` reaches tb (NT threads, NB/NT
// bins each); *pa / *pb = the exclusive prefixes before it. Returns NB when none crosses.
RT_DEVICE int first_crossing(const float* a, const float* bm, float ta, float tb, float* scr, int* res, float* pa,
                             float* pb) {
  constexpr int BPT = NB / NT;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  float la[BPT], lb[BPT], sa = 0.f, sb = 0.f;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    la[j] = a[BPT * t + j];
    lb[j] = bm[BPT * t + j];
    sa += la[j];
    sb += lb[j];
  }
  const float ta_own = sa, tb_own = sb;
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
    scr[NWV + wid] = sb;
  }
  if (t == 0) *res = NB;
  __syncthreads();
  float ca = 0.f, cb = 0.f;
  for (int w = 0; w < wid; ++w) {
    ca += scr[w];
    cb += scr[NWV + w];
  }
  ca += sa - ta_own;     // exclusive prefix before this thread's first bin
  cb += sb - tb_own;
  int cross = NB;
  float ea = 0.f, eb = 0.f;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    if (cross == NB && (ca + la[j] >= ta || cb + lb[j] >= tb)) {
      cross = BPT * t + j;
      ea = ca;
      eb = cb;
    }
    ca += la[j];
    cb += lb[j];
  }
  if (cross < NB) atomicMin(res, cross);
  __syncthreads();
  const int cbin = *res;
  if (cbin < NB && cross == cbin) {
    *pa = ea;
    *pb = eb;
  }
  __syncthreads();
  return cbin;
}

// Top-p slow path without a histogram (the rejected-j* case, ~1 - top_p of the rows):
// a token is inside the nucleus iff the mass of the tokens strictly more likely than it is below
// p * total (the reference's sorted-cumsum cut, restated), the same test the accept pass made for
// j*. Candidates = the chunks' best Gumbel tokens in score order; c1 = j* is out. ONE pass
// measures the mass above the next NC candidates; the first one inside, c*, is the answer unless
// a non-best token of a chunk ranked above c* (those chunks' bests are out) scores higher and is
// inside: those chunks are rescanned, their tokens' nucleus test decided from the known
// values (>= an inside candidate's value: in; <= an outside one's: out). Returns the token,
// or -1 when some token stays undecided or no candidate is inside (the histogram path decides).
constexpr int NC = 4;
template <typename T, bool VEC>
RT_DEVICE int nucleus_by_candidates(const T* row, int V, float mx, float invT, float pz, float vj, uint64_t key,
                                    const float* s_gv, const int* s_gi, float* sv, int* si, float* red) {
  __shared__ int s_ord[C];
  __shared__ float s_cv[NC];
  __shared__ int s_flag;
  if (threadIdx.x < C) {   // rank of chunk j's best by (score desc, index asc)
    const int j = threadIdx.x;
    int r = 0;
    for (int q = 0; q < C; ++q)
      r += (s_gv[q] > s_gv[j] || (s_gv[q] == s_gv[j] && s_gi[q] < s_gi[j])) ? 1 : 0;
    s_ord[r] = j;
  }
  __syncthreads();
  if (threadIdx.x < NC) {
    const int gi = s_gi[s_ord[1 + threadIdx.x]];
    s_cv[threadIdx.x] = (gi >= 0 && gi < V) ? rt::DT<T>::load(row + gi) : INFINITY;
  }
  if (threadIdx.x == 0) s_flag = 0;
  __syncthreads();
  float cv[NC], acc[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    cv[k] = s_cv[k];
    acc[k] = 0.f;
  }
  for_row<T, VEC>(row, V, [&](int, float v) {
    const float e = __expf((v - mx) * invT);
#pragma unroll
    for (int k = 0; k < NC; ++k) acc[k] += v > cv[k] ? e : 0.f;
  });
  int kstar = -1;
  float v_in = INFINITY, v_out = vj;   // known: values >= v_in are inside, <= v_out outside
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const float m = block_sum_dpp(acc[k], red);
    const bool ok = cv[k] != INFINITY && m < pz;
    if (ok) {
      if (kstar < 0) kstar = k;
      v_in = fminf(v_in, cv[k]);
    } else if (cv[k] != INFINITY) {
      v_out = fmaxf(v_out, cv[k]);
    }
  }
  if (kstar < 0) return -1;
  const int cs = s_ord[1 + kstar];
  ArgMax best{s_gv[cs], s_gi[cs]};
  __shared__ float s_uv[NC], s_us[NC];
  __shared__ int s_ui[NC];
  // chunks ranked above c* (their bests are outside): any token beating c* must be checked
  for (int q = 0; q <= kstar; ++q) {
    int lo, hi;
    chunk_range(V, s_ord[q], lo, hi);
    for_range<T, VEC>(row, lo, hi, [&](int i, float v) {
      const float sc = v * invT + gumbel(key, (uint32_t)i);
      if (sc > s_gv[cs] || (sc == s_gv[cs] && i < s_gi[cs])) {
        if (v >= v_in) {
          am_merge(best, sc, i);
        } else if (v > v_out) {             // undecided from the known values: test it exactly
          const int u = atomicAdd(&s_flag, 1);
          if (u < NC) {
            s_uv[u] = v;
            s_us[u] = sc;
            s_ui[u] = i;
          }
        }
      }
    });
  }
  best = block_argmax(best, sv, si);
  __syncthreads();
  const int nu = s_flag;
  if (nu > NC) return -1;
  if (nu > 0) {   // one more pass: the mass above each undecided token
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      cv[k] = k < nu ? s_uv[k] : INFINITY;
      acc[k] = 0.f;
    }
    for_row<T, VEC>(row, V, [&](int, float v) {
      const float e = __expf((v - mx) * invT);
#pragma unroll
      for (int k = 0; k < NC; ++k) acc[k] += v > cv[k] ? e : 0.f;
    });
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const float m = block_sum_dpp(acc[k], red);
      if (k < nu && m < pz) am_merge(best, s_us[k], s_ui[k]);
    }
  }
  return best.i;
}

struct SampleArgs {
  int64_t* tok;                 // [B] sampled ids
  float* ws;                    // B * W_ROW + 4 words, zero before the first launch (self re-arming)
  const void* logits;
  int V;
  int64_t ld;
  const float* temperature;
  const float* top_p;
  const int* top_k;
  const int64_t* seeds;
  int64_t* offsets;             // read by every workgroup; rewritten by the deciders (adv)
  int B;
  // decode-step bookkeeping (adv = 1): decode_advance + next-step decode_prep of each row
  int adv;
  int64_t* out;                 // [max_steps, B]
  int64_t* ids;
  int64_t* positions;
  int* ctx_lens;
  int64_t* step;
  int max_steps;
  int64_t* slots;               // prep (res != nullptr)
  uint16_t* res;
  const int* block_tables;
  const uint16_t* embed;
  int max_blocks, BS, H;
  int64_t vocab;
  int probe;                    // microbench only (RT_SMP_PROBE): 1 = stop before the slow path,
                                // 2 = after its coarse histogram, 3 = after the sub-histogram,
                                // 5 = full sampler, but tok[b] = the path that decided (PATH_*)
};

template <typename T, bool VEC>
__global__ void __launch_bounds__(NT) smp_kernel(SampleArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char pool[POOL_BYTES];
  float* hc = reinterpret_cast<float*>(pool);
  float* hm = hc + NB;
  // histogram accumulators: INTEGER LDS atomics (count, and mass in 32.32 fixed point) — LDS
  // float atomic adds serialize per lane on gfx950 (r03 probe: a 128K-token coarse pass took
  // 320 us on one workgroup), the integer ones do not
  unsigned* hci = reinterpret_cast<unsigned*>(hm + NB);
  unsigned long long* hmi = reinterpret_cast<unsigned long long*>(hci + NB);
  uint32_t* okeys = reinterpret_cast<uint32_t*>(pool);
  __shared__ int s_cnt3[2 * 3 * NWV], s_ln, s_lt;
  __shared__ uint32_t s_tk[LCAP];
  __shared__ int s_ti[LCAP];
  __shared__ uint32_t s_lk[LCAP];
  __shared__ int s_li[LCAP];
  __shared__ float sv[NWV], red[2 * NWV + 2];
  __shared__ int si[NWV];
  __shared__ float s_max[C], s_gv[C], s_min[C];
  __shared__ int s_arg[C], s_gi[C];
  __shared__ int s_last, s_res, s_kb[C], s_lump, s_rescan_c[C];
  __shared__ float s_sc[C];
  __shared__ float s_pa, s_pb;
  const int b = blockIdx.x, c = blockIdx.y;
  float* w = a.ws + (size_t)b * W_ROW;
  int* wi = reinterpret_cast<int*>(w);
  const T* row = static_cast<const T*>(a.logits) + (size_t)b * a.ld;
  const int V = a.V;
  int lo, hi;
  chunk_range(V, c, lo, hi);
  // this thread's first 16 B of the chunk, requested before the parameter loads (the chunk
  // pass cannot start until `temperature` arrives; its first round trip overlaps that one)
  rt::short8 pv{};
  bool has_pv = false;
  if constexpr (VEC && sizeof(T) == 2) {
    if ((int)threadIdx.x < ((hi - lo) >> 3)) {
      pv = *reinterpret_cast<const rt::short8*>(row + lo + 8 * threadIdx.x);
      has_pv = true;
    }
  }
  // f(i, v) over the chunk [lo, hi), the preloaded vector first (used by both chunk sweeps)
  auto for_chunk = [&](auto&& f) {
    if constexpr (VEC && sizeof(T) == 2) {
      const int nv = (hi - lo) >> 3;
      if (has_pv) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f(lo + 8 * (int)threadIdx.x + j, rt::bf2f((uint16_t)pv[j]));
      }
      const rt::short8* pp = reinterpret_cast<const rt::short8*>(row + lo);
      for (int cc = threadIdx.x + NT; cc < nv; cc += NT) {
        const rt::short8 v = pp[cc];
#pragma unroll
        for (int j = 0; j < 8; ++j) f(lo + cc * 8 + j, rt::bf2f((uint16_t)v[j]));
      }
      for (int i = lo + (nv << 3) + threadIdx.x; i < hi; i += NT) f(i, rt::DT<T>::load(row + i));
    } else {
      for_range<T, VEC>(row, lo, hi, f);
    }
  };
  const float temp = a.temperature[b];
  const int64_t off = a.offsets[b];
  const int64_t st = a.adv ? *a.step : 0;
  // grid scale of this row's histograms (bins per logit unit): chosen by the previous launch's
  // decider from the row's value span (0 before the first launch: the default)
  const float sgrid = __hip_atomic_load(&w[W_SC], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int k = a.top_k[b];
  const float p = a.top_p[b];
  // the decider's step bookkeeping inputs come with the parameters (row b's decider is their
  // only writer, after every ticket of the row): no dependent trip at the end of the launch
  const int64_t pos_b = a.adv ? a.positions[b] : 0;
  const int ctx_b = a.adv ? a.ctx_lens[b] : 0;
  // the deciders rewrite offsets / step / the grid scale: every read of them completes before
  // this workgroup's ticket (below), and the deciders write only after every ticket of their
  // row / launch (one wait for all the parameter loads)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t key = mix64((uint64_t)a.seeds[b] ^ mix64((uint64_t)off));
  const float invT = temp > 0.f ? 1.f / temp : 0.f;
  const bool use_k = k > 0 && k < V;
  // top-p rows (no top-k): every chunk also publishes a histogram of its tokens' mass on a grid
  // aligned across chunks (bin = floor(logit * scale)), which decides the accept test below
  // without another pass over the row for all but the rows whose j* shares a bin with the cut
  const bool hist = temp > 0.f && p < 1.f && !use_k;
  const float sbin = sgrid > 0.f ? sgrid : invT * BW;
  // top-k rows with a small k: chunk top-k lists (the decider needs no pass over the row)
  const int per = ((V + C - 1) / C + 7) & ~7;
  const bool full = a.probe == 0 || a.probe == 5;
  const bool lst = temp > 0.f && use_k && k <= KMAX && per <= POOLK && full;
  constexpr int KLO = sizeof(T) == 2 ? 16 : 0;

  // ---- 1: chunk records ----
  ArgMax am{-INFINITY, 0x7fffffff}, gb{-INFINITY, 0x7fffffff};
  float mn = INFINITY;
  if (temp > 0.f) {
    for_chunk([&](int i, float v) {
      am_merge(am, v, i);
      mn = fminf(mn, v);
      am_merge(gb, v * invT + gumbel(key, (uint32_t)i), i);
      if (lst) okeys[i - lo] = okey(v, KLO);
    });
    gb = block_argmax(gb, sv, si);
    mn = -block_max_dpp(-mn, red);
  } else {
    for_chunk([&](int i, float v) { am_merge(am, v, i); });
  }
  am = block_argmax(am, sv, si);
  if (hist) {
    // second sweep of the (L2-resident) chunk: mass exp((v - chunk max) / T) per bin, integer
    // LDS atomics in 32.32 fixed point (float LDS atomics serialize on gfx950)
    const float cmax = am.v;
    const float ktop = floorf(cmax * sbin);
    for (int i = threadIdx.x; i < HB; i += NT) hmi[i] = 0ull;
    __syncthreads();
    if (cmax > -INFINITY) {
      for_chunk([&](int, float v) {
        const float e = __expf((v - cmax) * invT);
        if (e > 0.f) {
          const float kr = fminf(fmaxf(ktop - floorf(v * sbin), 0.f), (float)(HB - 1));
          atomicAdd(&hmi[(int)kr], (unsigned long long)(e * 4294967296.f));
        }
      });
    }
    __syncthreads();
    for (int i = threadIdx.x; i < HB; i += NT)
      __hip_atomic_store(&w[W_HIST + c * HB + i], (float)(hmi[i] >> 8) * (1.f / 16777216.f), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0)
      __hip_atomic_store(&wi[W_KB + c], cmax > -INFINITY ? (int)ktop : -(1 << 30), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every thread's histogram stores complete before thread 0's ticket
  }
  if (lst) {
    // this chunk's k-th largest key Kc; list = every token above it, then its ties up to LCAP,
    // published sorted by token id (the atomic slot order is not deterministic)
    const int n = hi - lo;
    const int need = min(k, n);
    uint32_t kc = 0;
    if (need > 0) kc = kth_key(okeys, n, need, KLO, s_cnt3);
    if (threadIdx.x == 0) s_ln = s_lt = 0;
    __syncthreads();
    if (need > 0) {   // one pass: keys above kc (fewer than need <= KMAX < LCAP) and ties apart
      for (int i0 = 0; i0 < n; i0 += 8 * NT) {
        uint32_t kk[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + (int)threadIdx.x + j * NT;
          kk[j] = i < n ? okeys[i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + (int)threadIdx.x + j * NT;
          if (kk[j] > kc) {   // fewer than need <= KMAX < LCAP such keys; bounded all the same
            const int sl = atomicAdd(&s_ln, 1);
            if (sl < LCAP) {
              s_lk[sl] = kk[j];
              s_li[sl] = lo + i;
            }
          } else if (kk[j] == kc && i < n) {
            const int sl = atomicAdd(&s_lt, 1);
            if (sl < LCAP) {
              s_tk[sl] = kk[j];
              s_ti[sl] = lo + i;
            }
          }
        }
      }
      __syncthreads();
      const int g = s_ln;
      for (int q = threadIdx.x; q < min(s_lt, LCAP - g); q += NT) {
        s_lk[g + q] = s_tk[q];
        s_li[g + q] = s_ti[q];
      }
      __syncthreads();
      if (threadIdx.x == 0) s_ln = g + s_lt;
    }
    __syncthreads();
    const int len = min(s_ln, LCAP);
    if ((int)threadIdx.x < len) {
      const int mi = s_li[threadIdx.x];
      int r = 0;
      for (int j = 0; j < len; ++j) r += s_li[j] < mi;
      __hip_atomic_store(&wi[W_TKL + c * LCAP + r], (int)s_lk[threadIdx.x], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&wi[W_TKI + c * LCAP + r], mi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
      __hip_atomic_store(&wi[W_TKN + c], len | (s_ln > LCAP ? 1 << 16 : 0), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&wi[W_TKK + c], (int)kc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every thread's list stores complete before thread 0's ticket
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(&w[W_MIN + c], mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&w[W_MAX + c], am.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&wi[W_ARG + c], am.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&w[W_GV + c], gb.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&wi[W_GI + c], gb.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(&wi[W_CNT], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == C - 1;
    if (s_last) __hip_atomic_store(&wi[W_CNT], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;

  // ---- 2: the decider ----
  // ONE round trip for everything the chunks published: records, grid tops and (top-p rows)
  // the 4096 histogram words, 8 per thread
  float hv[C * HB / NT];
  if (threadIdx.x < C) {
    const int j = threadIdx.x;
    s_max[j] = __hip_atomic_load(&w[W_MAX + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_arg[j] = __hip_atomic_load(&wi[W_ARG + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_gv[j] = __hip_atomic_load(&w[W_GV + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_gi[j] = __hip_atomic_load(&wi[W_GI + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_min[j] = __hip_atomic_load(&w[W_MIN + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (hist) s_kb[j] = __hip_atomic_load(&wi[W_KB + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (hist) {
#pragma unroll
    for (int q = 0; q < C * HB / NT; ++q)
      hv[q] = __hip_atomic_load(&w[W_HIST + threadIdx.x + q * NT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // top-k list rows: the C lists (6 + 6 words per thread) in the same round trip
  __shared__ int s_tkn[C], s_tkk[C], s_ccnt[C], s_fb;
  uint32_t* lk = okeys;                                   // [C][LCAP] merged lists
  int* li = reinterpret_cast<int*>(okeys + C * LCAP);
  uint32_t* ak = okeys + 2 * C * LCAP;                    // [NALLOW] allowed tokens, id order
  int* ai = reinterpret_cast<int*>(ak + NALLOW);
  float* aw = reinterpret_cast<float*>(ai + NALLOW);
  constexpr int LQ = C * LCAP / NT;
  if (lst) {
    int lkr[LQ], lir[LQ];
    if (threadIdx.x < C) {
      s_tkn[threadIdx.x] = __hip_atomic_load(&wi[W_TKN + threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_tkk[threadIdx.x] = __hip_atomic_load(&wi[W_TKK + threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      lkr[q] = __hip_atomic_load(&wi[W_TKL + threadIdx.x + q * NT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lir[q] = __hip_atomic_load(&wi[W_TKI + threadIdx.x + q * NT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < LQ; ++q) {   // entries past a chunk's length: key 0 (below every value's key)
      const int e = threadIdx.x + q * NT, cc = e / LCAP;
      lk[e] = e - cc * LCAP < (s_tkn[cc] & 0xffff) ? (uint32_t)lkr[q] : 0u;
      li[e] = lir[q];
    }
  }
  __syncthreads();
  ArgMax ra{-INFINITY, 0x7fffffff}, g{-INFINITY, 0x7fffffff};
  float rmin = INFINITY;
  for (int j = 0; j < C; ++j) {
    am_merge(ra, s_max[j], s_arg[j]);
    am_merge(g, s_gv[j], s_gi[j]);
    rmin = fminf(rmin, s_min[j]);
  }
  const float mx = ra.v;
  int tok;
  int path = PATH_PLAIN;
  if (!(temp > 0.f)) {
    tok = ra.i;
  } else if (!use_k && !(p < 1.f)) {
    tok = (g.i >= 0 && g.i < V) ? g.i : ra.i;     // no finite score: the row argmax
  } else {
    bool accepted = false;
    int cand = -1;
    if (!use_k && g.i >= 0 && g.i < V) {   // fast path: is j* inside the nucleus?
      const float vj = rt::DT<T>::load(row + g.i);
      // bounds on the mass strictly above j* from the chunk histograms: bins above j*'s bin are
      // above it, its own bin (and a chunk's open-ended last bin reaching it) may or may not be
      const float kj = floorf(vj * sbin);
      float lo_m = 0.f, mid_m = 0.f, tot_m = 0.f;
      if (threadIdx.x < C) s_sc[threadIdx.x] = __expf((s_max[threadIdx.x] - mx) * invT);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < C * HB / NT; ++q) {
        const int e = threadIdx.x + q * NT, cc = e / HB, kk = e - cc * HB;
        const float m = hv[q] * s_sc[cc];
        const float kb = (float)(s_kb[cc] - kk);   // this bin's grid index (the last bin: its top)
        tot_m += m;
        if (kk < HB - 1) {
          lo_m += kb > kj ? m : 0.f;
          mid_m += kb == kj ? m : 0.f;
        } else {
          mid_m += kb >= kj ? m : 0.f;
        }
      }
      lo_m = block_sum_dpp(lo_m, red);
      mid_m = block_sum_dpp(mid_m, red);
      tot_m = block_sum_dpp(tot_m, red);
      float pz = p * tot_m;
      bool decided = lo_m + mid_m < pz || lo_m >= pz;
      accepted = lo_m + mid_m < pz;
      if (!decided) {   // j* shares its bin with the cut: the exact test, one pass
        float above = 0.f, total = 0.f;
        for_row<T, VEC>(row, V, [&](int, float v) {
          const float e = __expf((v - mx) * invT);
          total += e;
          above += v > vj ? e : 0.f;
        });
        above = block_sum_dpp(above, red);
        total = block_sum_dpp(total, red);
        pz = p * total;
        accepted = above < pz;
      }
      path = (accepted ? PATH_ACCEPT : PATH_RESCAN) + (decided ? 0 : PATH_EXACT_PASS);
      if (!accepted && full) {
        // rejected j*: the nucleus cut from the SAME histograms, merged on the common z grid
        // (bin g = kmax - floor(v / T * BW), 0 = top). With the crossing bin g*, tokens in bins
        // above it are inside the nucleus, below it outside, in it undecided. A chunk's best
        // Gumbel token inside the nucleus is its best allowed one; chunks whose best is not are
        // rescanned (tokens above g* only). Exact unless an undecided token (bin g*, or an
        // open-ended last bin reaching g*) could win: then the candidate / histogram paths.
        int kmx = -(1 << 30);
        for (int j = 0; j < C; ++j) kmx = max(kmx, s_kb[j]);
        for (int i = threadIdx.x; i < NB; i += NT) hmi[i] = 0ull;
        if (threadIdx.x == 0) s_lump = NB;
        __syncthreads();
        for (int q = 0; q < C * HB / NT; ++q) {   // re-read (L2): hv is not kept live across the passes
          const int e = threadIdx.x + q * NT, cc = e / HB, kk = e - cc * HB;
          const float m = __hip_atomic_load(&w[W_HIST + e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * s_sc[cc];
          const int gb = kmx - (s_kb[cc] - kk);
          if (m > 0.f) {
            if (kk == HB - 1 || gb >= NB) atomicMin(&s_lump, min(gb, NB - 1));   // open-ended: its top
            else atomicAdd(&hmi[gb], (unsigned long long)(m * 4294967296.f));
          }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < NB; i += NT) {
          hc[i] = 0.f;
          hm[i] = (float)(hmi[i] >> 8) * (1.f / 16777216.f);
        }
        __syncthreads();
        const int gst = first_crossing(hc, hm, 3.0e38f, pz, red, &s_res, &s_pa, &s_pb);
        if (gst < NB && s_lump > gst) {
          if (threadIdx.x < C) {
            const int j = threadIdx.x, gi = s_gi[j];
            const int gb = (gi >= 0 && gi < V) ? kmx - (int)floorf(rt::DT<T>::load(row + gi) * sbin) : NB;
            s_rescan_c[j] = gb < gst ? 0 : 1;
          }
          __syncthreads();
          ArgMax win{-INFINITY, 0x7fffffff}, amb{-INFINITY, 0x7fffffff};
          for (int j = 0; j < C; ++j)
            if (!s_rescan_c[j]) am_merge(win, s_gv[j], s_gi[j]);   // every thread: same merge order
          for (int j = 0; j < C; ++j) {
            if (!s_rescan_c[j]) continue;
            int clo, chi;
            chunk_range(V, j, clo, chi);
            // two accumulators updated by selects (a branch choosing one of two structs makes the
            // compiler address them through scratch)
            float wv = win.v, av = amb.v;
            int wi = win.i, ai = amb.i;
            for_range<T, VEC>(row, clo, chi, [&](int i, float v) {
              const int gb = kmx - (int)floorf(v * sbin);
              if (gb <= gst) {
                const float sc = v * invT + gumbel(key, (uint32_t)i);
                const bool in = gb < gst;
                const bool bw = in && (sc > wv || (sc == wv && i < wi));
                const bool ba = !in && (sc > av || (sc == av && i < ai));
                wv = bw ? sc : wv;
                wi = bw ? i : wi;
                av = ba ? sc : av;
                ai = ba ? i : ai;
              }
            });
            win = ArgMax{wv, wi};
            amb = ArgMax{av, ai};
          }
          win = block_argmax(win, sv, si);
          amb = block_argmax(amb, sv, si);
          if (win.i != 0x7fffffff && (amb.v < win.v || (amb.v == win.v && amb.i > win.i))) cand = win.i;
        }
        if (cand < 0) {
          cand = nucleus_by_candidates<T, VEC>(row, V, mx, invT, pz, vj, key, s_gv, s_gi, sv, si, red);
          path += PATH_CANDIDATES - PATH_RESCAN;
        }
      }
    }
    if (lst) {
      // top-k from the chunk lists: the union holds every chunk's top k, so its k-th largest key
      // is the row's; every allowed token (key >= kg) is listed unless a chunk dropped ties AT kg
      const uint32_t kg = kth_key(lk, C * LCAP, k, KLO, s_cnt3);
      if (threadIdx.x == 0) s_fb = 0;
      __syncthreads();
      if (threadIdx.x < C && (s_tkn[threadIdx.x] >> 16) && (uint32_t)s_tkk[threadIdx.x] == kg) s_fb = 1;
      __syncthreads();
      if (!s_fb && !(p < 1.f)) {
        ArgMax r{-INFINITY, 0x7fffffff};
        for (int e = threadIdx.x; e < C * LCAP; e += NT) {
          const uint32_t kk = lk[e];
          if (kk >= kg) am_merge(r, (okey_value(kk, KLO) - mx) * invT + gumbel(key, (uint32_t)li[e]), li[e]);
        }
        r = block_argmax(r, sv, si);
        cand = r.i != 0x7fffffff ? r.i : -1;
      } else if (!s_fb) {
        // top-p inside the top-k set: compact the allowed tokens in id order (lists are sorted by
        // id, chunks in id order; each wave ranks 4 chunks with ballots), then the exact test —
        // mass strictly above a token < p * allowed mass — and the Gumbel argmax over the nucleus
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        constexpr int CPW = C / NWV, RPC = (LCAP + 63) / 64;
        int pos[CPW][RPC];
#pragma unroll
        for (int q = 0; q < CPW; ++q) {
          const int cc = wid * CPW + q;
          int run = 0;
#pragma unroll
          for (int r = 0; r < RPC; ++r) {
            const int j = lane + 64 * r;
            const bool al = j < LCAP && lk[cc * LCAP + j] >= kg;
            const unsigned long long m = __ballot(al);
            pos[q][r] = al ? run + __popcll(m & ((1ull << lane) - 1ull)) : -1;
            run += __popcll(m);
          }
          if (lane == 0) s_ccnt[cc] = run;
        }
        __syncthreads();
        int tot = 0;
        for (int j = 0; j < C; ++j) tot += s_ccnt[j];
        if (tot <= NALLOW) {
#pragma unroll
          for (int q = 0; q < CPW; ++q) {
            const int cc = wid * CPW + q;
            int base = 0;
            for (int j = 0; j < cc; ++j) base += s_ccnt[j];
#pragma unroll
            for (int r = 0; r < RPC; ++r) {
              if (pos[q][r] >= 0) {
                const int e = cc * LCAP + lane + 64 * r;
                ak[base + pos[q][r]] = lk[e];
                ai[base + pos[q][r]] = li[e];
                aw[base + pos[q][r]] = __expf((okey_value(lk[e], KLO) - mx) * invT);
              }
            }
          }
          __syncthreads();
          const int t = threadIdx.x;
          const float my_w = t < tot ? aw[t] : 0.f;
          const float zsum = block_sum_dpp(my_w, red);
          ArgMax r{-INFINITY, 0x7fffffff};
          if (t < tot) {
            const uint32_t mk = ak[t];
            float above = 0.f;
            for (int j = 0; j < tot; ++j) above += ak[j] > mk ? aw[j] : 0.f;
            if (above < p * zsum) am_merge(r, (okey_value(mk, KLO) - mx) * invT + gumbel(key, (uint32_t)ai[t]), ai[t]);
          }
          r = block_argmax(r, sv, si);
          cand = r.i != 0x7fffffff ? r.i : -1;
        }
      }
      __syncthreads();   // the histogram path below reuses the pool
    }
    if (accepted || cand >= 0 || a.probe == 1) {
      tok = accepted ? g.i : (cand >= 0 ? cand : ra.i);
    } else {
      // ---- slow path: histogram threshold, then the Gumbel argmax over the allowed set ----
      path = (path / PATH_EXACT_PASS) * PATH_EXACT_PASS + PATH_HISTOGRAM;
      // coarse bins span the row's actual z range [zlo, 0] (not a fixed [-ZR, 0]): the values
      // spread over all NB bins, so the LDS atomics of one workgroup rarely collide
      const float zlo = fmaxf(-ZR, fminf((rmin - mx) * invT, -1e-3f));
      const float scale = NB / (-zlo * 1.0001f + 1e-6f);   // the row minimum lands inside the last bin
      for (int i = threadIdx.x; i < NB; i += NT) {
        hci[i] = 0u;
        hmi[i] = 0ull;
      }
      __syncthreads();
      for_row<T, VEC>(row, V, [&](int, float v) {
        const float z = (v - mx) * invT;
        const float fb = -z * scale;
        if (fb < (float)NB) {
          const int bin = (int)fb;
          atomicAdd(&hci[bin], 1u);
          atomicAdd(&hmi[bin], (unsigned long long)(__expf(z) * 4294967296.f));
        }
      });
      __syncthreads();
      for (int i = threadIdx.x; i < NB; i += NT) {
        hc[i] = (float)hci[i];
        hm[i] = (float)(hmi[i] >> 8) * (1.f / 16777216.f);
      }
      __syncthreads();
      if (a.probe == 2) {
        if (threadIdx.x == 0) a.tok[b] = ra.i + (hc[0] == -1.f);
        return;
      }
      float tm = 0.f;
      for (int i = threadIdx.x; i < NB; i += NT) tm += hm[i];
      tm = block_sum_dpp(tm, red);
      const float tk = use_k ? (float)k : 3.0e38f;
      int bk = NB;
      float pre_c = 0.f, zk_mass = tm;
      if (use_k) {
        bk = first_crossing(hc, hm, tk, 3.0e38f, red, &s_res, &s_pa, &s_pb);
        if (bk < NB) {
          zk_mass = s_pb + hm[bk];
          pre_c = s_pa;
        }
      }
      const float tp = p < 1.f ? p * zk_mass : 3.0e38f;
      int bp = NB;
      float pre_m = 0.f;
      if (p < 1.f) {
        bp = first_crossing(hc, hm, 3.0e38f, tp, red, &s_res, &s_pa, &s_pb);
        pre_m = s_pb;
      }
      int bsel;
      bool by_count;
      float need;
      if (bk <= bp) {
        bsel = bk;
        by_count = true;
        need = tk - pre_c;
      } else {
        bsel = bp;
        by_count = false;
        need = tp - pre_m;
      }
      float zthr = -INFINITY;
      if (bsel < NB) {   // sub-histogram of the selected bin
        __syncthreads();
        for (int i = threadIdx.x; i < NB; i += NT) {
          hci[i] = 0u;
          hmi[i] = 0ull;
        }
        __syncthreads();
        const float top_edge = -(float)bsel / scale, sub = scale * NB;
        for_row<T, VEC>(row, V, [&](int, float v) {
          const float z = (v - mx) * invT;
          const float fb = -z * scale;
          if (fb >= (float)bsel && fb < (float)(bsel + 1)) {
            int sb = (int)((top_edge - z) * sub);
            sb = sb < 0 ? 0 : (sb >= NB ? NB - 1 : sb);
            atomicAdd(&hci[sb], 1u);
            atomicAdd(&hmi[sb], (unsigned long long)(__expf(z) * 4294967296.f));
          }
        });
        __syncthreads();
        for (int i = threadIdx.x; i < NB; i += NT) {
          hc[i] = (float)hci[i];
          hm[i] = (float)(hmi[i] >> 8) * (1.f / 16777216.f);
        }
        __syncthreads();
        if (a.probe == 3) {
          if (threadIdx.x == 0) a.tok[b] = ra.i + (hc[0] == -1.f);
          return;
        }
        const int cb = by_count ? first_crossing(hc, hm, need, 3.0e38f, red, &s_res, &s_pa, &s_pb)
                                : first_crossing(hc, hm, 3.0e38f, need, red, &s_res, &s_pa, &s_pb);
        const int cc = cb < NB ? cb : NB - 1;
        zthr = -(float)bsel / scale - (float)(cc + 1) / (scale * NB);
      }
      // Gumbel argmax over the allowed set {z >= zthr}. A chunk's best score over ALL its tokens
      // (s_gv / s_gi, from the stats phase) is also its best allowed one whenever that token is
      // allowed; only the chunks whose best is not (the rejected j*'s, ~1 - top_p of the others)
      // are scanned again. Scores s_gv = v/T + g differ from z + g by the row constant mx/T.
      ArgMax r{-INFINITY, 0x7fffffff};
      __shared__ int s_rescan[C];
      __shared__ int s_nres;
      if (threadIdx.x == 0) s_nres = 0;
      __syncthreads();
      if (threadIdx.x < C) {
        const int j = threadIdx.x, gi = s_gi[j];
        const bool ok = gi >= 0 && gi < V && (rt::DT<T>::load(row + gi) - mx) * invT >= zthr;
        if (!ok) s_rescan[atomicAdd(&s_nres, 1)] = j;
      }
      __syncthreads();
      for (int j = 0; j < C; ++j) {
        const int gi = s_gi[j];
        bool listed = false;
        for (int q = 0; q < s_nres; ++q) listed |= s_rescan[q] == j;
        if (!listed) am_merge(r, s_gv[j] - mx * invT, gi);     // every thread: same merge order
      }
      for (int q = 0; q < s_nres; ++q) {
        int clo, chi;
        chunk_range(V, s_rescan[q], clo, chi);
        for_range<T, VEC>(row, clo, chi, [&](int i, float v) {
          const float z = (v - mx) * invT;
          if (z >= zthr) am_merge(r, z + gumbel(key, (uint32_t)i), i);
        });
      }
      r = block_argmax(r, sv, si);
      tok = r.i == 0x7fffffff ? ra.i : r.i;     // empty allowed set (rounding): the row argmax
    }
  }

  // ---- 3: the token and this row's step bookkeeping ----
  if (hist && threadIdx.x == 0) {
    // next launch's grid: HB - 2 bins over the row's span (at most 8 / invT, where the mass
    // below is < e^-8 of the top token's), so a near-flat distribution (random-init weights)
    // still spreads over the bins instead of landing in one or two; never so fine that
    // floor(v * scale) leaves the int range
    const float span = fmaxf(fminf(mx - rmin, 8.f / invT), 1e-4f);
    const float sn = fminf((float)(HB - 2) / span, 1e6f / (fabsf(mx) + fabsf(rmin) + 1.f));
    __hip_atomic_store(&w[W_SC], sn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int64_t pn = pos_b + 1;
  int64_t blk = 0;
  // the next K/V slot's block-table entry (thread 0) and the next step's embedding row (every
  // lane, 16 B) are requested together: one round trip for both
  if (a.adv && a.slots != nullptr && threadIdx.x == 0) {   // past the table the slot is never used
    const int64_t bi = pn / a.BS;
    if (bi < a.max_blocks) blk = a.block_tables[(size_t)b * a.max_blocks + bi];
  }
  if (a.adv && a.res != nullptr) {
    int64_t t = tok < 0 ? 0 : (tok >= a.vocab ? a.vocab - 1 : tok);
    const int row8 = a.H / 8;
    const uint4* src = reinterpret_cast<const uint4*>(a.embed) + (size_t)t * row8;
    uint4* dst = reinterpret_cast<uint4*>(a.res) + (size_t)b * row8;
    for (int i = threadIdx.x; i < row8; i += NT) dst[i] = src[i];
  }
  if (threadIdx.x == 0) {
    a.tok[b] = a.probe == 5 ? path : tok;
    if (a.adv) {
      if (st < a.max_steps) a.out[st * a.B + b] = tok;
      a.ids[b] = tok;
      a.positions[b] = pn;
      a.ctx_lens[b] = ctx_b + 1;
      if (a.slots != nullptr) {
        a.slots[b] = blk * a.BS + pn % a.BS;
        a.offsets[b] = pn + 1;
      }
    }
  }
  if (a.adv && threadIdx.x == 0) {   // the last decider of the launch advances the step counter
    int* done = reinterpret_cast<int*>(a.ws) + (size_t)a.B * W_ROW;
    const int prev = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == a.B - 1) {
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *a.step = st + 1;
    }
  }
}
}  // namespace

int sample_workspace_floats(int B) { return B * W_ROW + 4; }

int launch_sample(int64_t* out, const void* logits, bool is_bf16, int B, int V, int64_t ld_row,
                  const float* temperature, const float* top_p, const int* top_k, const int64_t* seeds,
                  const int64_t* offsets, float* ws, hipStream_t stream, const void* advance) {
  if (B == 0) return 0;
  if (V < 1) return -1;
  const size_t esz = is_bf16 ? 2 : 4;
  const bool vec = ((uintptr_t)logits % 16 == 0) && ((ld_row * esz) % 16 == 0);
  SampleArgs a{};
  if (advance != nullptr) a = *static_cast<const SampleArgs*>(advance);
  a.tok = out;
  a.ws = ws;
  a.logits = logits;
  a.V = V;
  a.ld = ld_row;
  a.temperature = temperature;
  a.top_p = top_p;
  a.top_k = top_k;
  a.seeds = seeds;
  a.offsets = const_cast<int64_t*>(offsets);
  a.B = B;
  static const int probe = getenv("RT_SMP_PROBE") ? atoi(getenv("RT_SMP_PROBE")) : 0;
  a.probe = probe;
  const dim3 g(B, C);
  if (is_bf16) {
    if (vec) hipLaunchKernelGGL((smp_kernel<uint16_t, true>), g, dim3(NT), 0, stream, a);
    else hipLaunchKernelGGL((smp_kernel<uint16_t, false>), g, dim3(NT), 0, stream, a);
  } else {
    if (vec) hipLaunchKernelGGL((smp_kernel<float, true>), g, dim3(NT), 0, stream, a);
    else hipLaunchKernelGGL((smp_kernel<float, false>), g, dim3(NT), 0, stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The captured decode step's sampler + bookkeeping (decode_advance + decode_prep semantics).
int launch_sample_advance(int64_t* tok, const void* logits, bool is_bf16, int B, int V, int64_t ld_row,
                          const float* temperature, const float* top_p, const int* top_k, const int64_t* seeds,
                          int64_t* offsets, float* ws, int64_t* out, int64_t* ids, int64_t* positions, int* ctx_lens,
                          int64_t* step, int max_steps, int64_t* slots, void* res, const int* block_tables,
                          const void* embed, int max_blocks, int BS, int H, int64_t vocab, hipStream_t stream) {
  const bool prep = res != nullptr;
  if (prep && (slots == nullptr || block_tables == nullptr || embed == nullptr || H % 8 || BS <= 0 ||
               max_blocks <= 0 || vocab <= 0))
    return -3;
  SampleArgs a{};
  a.adv = 1;
  a.out = out;
  a.ids = ids;
  a.positions = positions;
  a.ctx_lens = ctx_lens;
  a.step = step;
  a.max_steps = max_steps;
  a.slots = prep ? slots : nullptr;
  a.res = (uint16_t*)res;
  a.block_tables = block_tables;
  a.embed = (const uint16_t*)embed;
  a.max_blocks = max_blocks;
  a.BS = BS;
  a.H = H;
  a.vocab = vocab;
  return launch_sample(tok, logits, is_bf16, B, V, ld_row, temperature, top_p, top_k, seeds, offsets, ws, stream, &a);
}
