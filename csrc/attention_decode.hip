// K3: paged-KV decode attention (one query token per sequence), GQA, MFMA bf16, split-KV.
// The work-item code is in attn_core.h (shared with the persistent decode-layer kernel); this
// file holds the grid launch: blockIdx = (sequence x kv head, key split).
#include "attn_core.h"

#include <cstdlib>

namespace {
using namespace attn;

// XCD-aware item order (p.xcd): blocks are dealt round-robin over the 8 XCDs (block b runs on
// the XCD of b % 8, the same class->XCD map in consecutive launches: tools/probes/xcc_probe.hip),
// so item j = (lin % 8) * (nwg / 8) + lin / 8 gives each XCD a contiguous run of items. Items are
// ordered kv head slowest: one kv head's (sequence, split) items, whose partials its rows'
// combine reads, share an XCD — and decode_combine_kernel orders its rows the same way. A
// different placement changes only speed.
RT_DEVICE int xcd_item(int lin, int nwg) { return (lin & 7) * (nwg >> 3) + (lin >> 3); }

// the LDS-DMA staged form (LM_GLDS) puts each wave's K/V slice over the merge buffers
template <int D, int GM, int W, int LM>
union DecodeSmem {
  AttnSmem<D, GM, W> m;
  short8 stage[(LM & LM_GLDS) ? W * tile_words<D>() * 64 : 1];
};

template <int D, int GM, int W = NW, bool PP = true, int LM = 0>
__global__ void __launch_bounds__(W * 64) paged_decode_kernel(AttnArgs p) {
  static_assert(sizeof(DecodeSmem<D, GM, W, LM>) <= 160 * 1024, "LDS of one CU");
  __shared__ DecodeSmem<D, GM, W, LM> sm_;
  auto& sm = sm_.m;
  int bh = blockIdx.x, split = blockIdx.y;
  if (p.xcd) {
    const int ns = gridDim.y, nb = gridDim.x / p.Hkv;
    const int j = xcd_item(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * ns);
    const int hk = j / (nb * ns), rem = j - hk * (nb * ns);
    const int b = rem / ns;
    split = rem - b * ns;
    bh = b * p.Hkv + hk;
  }
  attn_item<D, false, GM, W, PP, LM>(p, bh, split, sm);
}

// Per-step work plan: one workgroup per item (sequence b, split) writes the item's key range
// (item_range, exactly as attn_item derives it) and its block ids. A decode step runs this once;
// every layer's attention launch then requests an item header and its first block ids together
// at launch-known addresses — one dependent round trip ahead of the K/V stream instead of two.
__global__ void __launch_bounds__(256) attn_plan_kernel(AttnArgs p, int G, int GM, int* __restrict__ plan) {
  const int b = blockIdx.x, split = blockIdx.y;
  const bool grouped = p.groups != nullptr;
  const int* gp = grouped ? p.groups + 3 * b : p.ctx_lens + b;
  const int go = grouped ? 1 : 0;
  const ItemRange it = item_range(p.ctx_lens[b], gp[0], gp[go], gp[2 * go], grouped, b, split, G, GM, p.num_splits);
  int* hdr = plan + (size_t)(b * p.num_splits + split) * p.plan_stride;
  if (threadIdx.x == 0) {
    hdr[0] = it.b0; hdr[1] = it.n; hdr[2] = it.sh; hdr[3] = it.ctx;
    hdr[4] = it.sh_b; hdr[5] = it.nsh; hdr[6] = it.pr_b; hdr[7] = it.nv;
  }
  const int lim = min(it.nv, p.plan_stride - PLAN_HDR);
  for (int tt = threadIdx.x; tt < lim; tt += blockDim.x)
    hdr[PLAN_HDR + tt] = tt < it.nsh ? p.block_tables[(size_t)it.b0 * p.max_blocks + it.sh_b + tt]
                                     : p.block_tables[(size_t)b * p.max_blocks + it.pr_b + (tt - it.nsh)];
}

// Split-KV combine as its own launch, for launches with many partial slots per query row
// (tensor-parallel shards: 1-2 KV heads per rank -> 32-64 splits so the K/V stream still
// covers the CUs; a table of 3 knights then leaves 3 x 64 = 192 slots per row). The in-launch
// combine runs on the ONE last-arriving workgroup, whose CU reads every partial of the row
// (cross-XCD hand-off reads ~65 GB/s per CU, MI355X_MICROARCH handoff-payload): 23 us for 192
// slots at 4 query heads (r03 probe). Here every (row, 32-dim chunk) gets its own workgroup of
// 8 dim-lanes x NSL slot-lanes (NSL = blockDim / 8, sized by the host to the row's slots, <= 128),
// each lane owning SPL slots whose loads are ALL issued before the first merge: one round trip
// per launch instead of one per 32 slots (round 3: 6 dependent trips at 192 slots, 6.6 us), and
// that trip overlaps the group-record lookup (the host's slot bound needs no record).
// Merge order is fixed (lane-local slots in index order, then xor-shuffle pairs, then a tree
// over the waves through LDS), so the result does not depend on timing.
// Partials were stored write-through by the previous launch: the kernel boundary orders them.
template <int D, int SPL>
__global__ void __launch_bounds__(1024) decode_combine_kernel(AttnArgs p) {
  const int G = p.Hq / p.Hkv;
  int row = blockIdx.x;                        // b * Hq + query head
  int chunk = blockIdx.y;
  if (p.xcd) {   // rows of one kv head on the XCD that ran its attention items (xcd_item)
    const int nc = gridDim.y, nb = gridDim.x / p.Hq;
    const int j = xcd_item(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * nc);
    const int per_h = nb * G * nc;
    const int hk = j / per_h, r1 = j - hk * per_h;
    const int bb = r1 / (G * nc), r2 = r1 - bb * (G * nc);
    const int hh = r2 / nc;
    chunk = r2 - hh * nc;
    row = bb * p.Hq + hk * G + hh;
  }
  const int b = row / p.Hq;
  const int dl = threadIdx.x & 7, sl = threadIdx.x >> 3;
  const int nsl = blockDim.x >> 3;
  const int d0 = chunk * 32 + 4 * dl;
  const int stride = p.slot_stride > 0 ? p.slot_stride : p.num_splits;
  // the host's sizing: every split of every member of the largest group (slots past the row's
  // own count are inside the row's stride and loaded, never merged)
  const int nmax = p.groups != nullptr ? min(stride, (16 / G) * p.num_splits) : p.num_splits;
  const float* __restrict__ po = p.part_o + (size_t)row * stride * D;
  const float* __restrict__ pml = p.part_ml + (size_t)row * stride * 4;
  // the group record and the first chunk's partials are independent: both requests go out
  // before either is used, the vector loads first (the compiler waits for a conditional block's
  // scalar loads at its end; round 3 paid the group lookup as a trip ahead of the partials)
  float4_ mlv[SPL], ov[SPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int s = min(sl + j * nsl, nmax - 1);
    mlv[j] = *reinterpret_cast<const float4_*>(pml + (size_t)s * 4);
    ov[j] = *reinterpret_cast<const float4_*>(po + (size_t)s * D + d0);
  }
  int b0 = 0, nn = 1, sh = 0;
  if (p.groups != nullptr) {
    b0 = p.groups[3 * b];
    nn = p.groups[3 * b + 1];
    sh = p.groups[3 * b + 2];
  }
  int n = 1;
  if (p.groups != nullptr && !(nn < 1 || nn * G > 16 || b0 < 0 || b < b0 || b - b0 >= nn || sh < 0))
    n = nn;                                    // as attn_item
  const int nslots = n * p.num_splits;
  if (nslots == 1) return;                     // written directly by the attention launch
  float M = -INFINITY, L = 0.f;
  float4_ O = {0.f, 0.f, 0.f, 0.f};
  auto merge = [&](float m2, float l2, float4_ o2) {
    if (!(l2 > 0.f)) return;
    const float Mc = fmaxf(M, m2);
    const float a = M == -INFINITY ? 0.f : exp2f(M - Mc), f = exp2f(m2 - Mc);
    O = O * a + f * o2;
    L = L * a + f * l2;
    M = Mc;
  };
#pragma unroll
  for (int j = 0; j < SPL; ++j)
    if (sl + j * nsl < nslots) merge(mlv[j][0], mlv[j][1], ov[j]);
  // more chunks only for rows with more slots than the host sized for (not reached when the
  // group record is well-formed: n * G <= 16)
  for (int base = SPL * nsl; base < nslots; base += SPL * nsl) {
#pragma unroll
    for (int j = 0; j < SPL; ++j) {            // every load of the chunk in flight before any merge
      const int s = min(base + sl + j * nsl, nslots - 1);
      mlv[j] = *reinterpret_cast<const float4_*>(pml + (size_t)s * 4);
      ov[j] = *reinterpret_cast<const float4_*>(po + (size_t)s * D + d0);
    }
#pragma unroll
    for (int j = 0; j < SPL; ++j)
      if (base + sl + j * nsl < nslots) merge(mlv[j][0], mlv[j][1], ov[j]);
  }
  // the 8 slot-lanes of a wave (lane bits 3..5), then the waves through LDS; fixed order
  auto xmerge = [&](int x, bool upper) {
    const float m2 = __shfl_xor(M, x, 64), l2 = __shfl_xor(L, x, 64);
    float4_ o2;
#pragma unroll
    for (int i = 0; i < 4; ++i) o2[i] = __shfl_xor(O[i], x, 64);
    if (upper) {   // the upper partner takes the lower's state first: same order on both
      const float mm = M, ll = L;
      const float4_ oo = O;
      M = m2; L = l2; O = o2;
      merge(mm, ll, oo);
    } else {
      merge(m2, l2, o2);
    }
  };
#pragma unroll
  for (int x = 8; x < 64; x <<= 1) xmerge(x, sl & (x >> 3));
  __shared__ float red[16][8][6];
  const int wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  if ((threadIdx.x & 63) < 8) {
    float* e = red[wave][dl];
    e[0] = O[0]; e[1] = O[1]; e[2] = O[2]; e[3] = O[3]; e[4] = M; e[5] = L;
  }
  __syncthreads();
  // the waves' states as a tree on the first wave: lane (w, dl) of 8 groups takes waves w and
  // w + 8, then three xor steps — 4 dependent merges instead of nwaves - 1
  if (threadIdx.x < 64) {
    const int w = threadIdx.x >> 3;
    M = -INFINITY; L = 0.f; O = float4_{0.f, 0.f, 0.f, 0.f};
    if (w < nwaves) {
      const float* e = red[w][dl];
      merge(e[4], e[5], float4_{e[0], e[1], e[2], e[3]});
    }
    if (w + 8 < nwaves) {
      const float* e = red[w + 8][dl];
      merge(e[4], e[5], float4_{e[0], e[1], e[2], e[3]});
    }
#pragma unroll
    for (int x = 8; x < 64; x <<= 1) xmerge(x, w & (x >> 3));
    if (w == 0) {
      const float inv = L > 0.f ? 1.f / L : 0.f;
      store_bf16x4(p.out + (size_t)row * D + d0, O[0] * inv, O[1] * inv, O[2] * inv, O[3] * inv, false);
    }
  }
}
}  // namespace


// q [B, Hq, D]; k_cache [NB, Hkv, 32, D] (chunk-major blocks, common.h kc_elem); v_cache [NB, Hkv, D, 32]; block_tables [B, max_blocks] int32;
// defer_combine: leave the separate combine to the caller (*deferred = 1 when it was needed);
// part_o >= B*Hq*slot_stride*D floats, part_ml >= B*Hq*slot_stride*4 floats, counters >= B*Hkv ints
// (zeroed once). groups: nullptr or [B][3] {first, n, shared blocks} (shared-prefix groups,
// attn_core.h); slot_stride >= max n * num_splits (0 = num_splits, no groups).
int launch_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                        const int* ctx_lens, float* part_o, float* part_ml, int* counters, int B, int Hq, int Hkv,
                        int D, int max_blocks, float scale, int num_splits, const int* groups, int slot_stride,
                        hipStream_t stream, int defer_combine, int* deferred, const int* plan, int plan_stride) {
  if (deferred != nullptr) *deferred = 0;
  if (B == 0) return 0;
  if (Hq % Hkv || Hq / Hkv > 16) return -1;
  if (num_splits < 1) num_splits = 1;
  if (num_splits > MAXS) return -3;
  dim3 grid(B * Hkv, num_splits), block(NW * 64);
  const float sl2 = scale * LOG2E;
  if (groups != nullptr && slot_stride < num_splits) return -4;
  AttnArgs args{(uint16_t*)out, (const uint16_t*)q, (const uint16_t*)k_cache, (const uint16_t*)v_cache,
                      block_tables, ctx_lens, part_o, part_ml, counters, Hq, Hkv, max_blocks, sl2, num_splits,
                      groups, groups != nullptr ? slot_stride : 0};
  static const int probe = getenv("RT_ATTN_PROBE") ? atoi(getenv("RT_ATTN_PROBE")) : 0;
  args.probe = probe;
  if (plan != nullptr) {
    if (plan_stride <= PLAN_HDR) return -5;
    args.plan = plan;
    args.plan_stride = plan_stride;
  }
  // separate combine launch from this many splits on (RT_ATTN_EXT_SPLITS pins it; 0 = never):
  // r03 probes, 3 knights x 40K shared keys: in-launch combine 8.7 us at 16 splits (48 slots),
  // 23 us at 64 (192 slots); whole launch(es), grouped B=3: tp8 shard 32.6 -> 14.9 us (64
  // splits), tp1 41.0 -> 38.7 us (8 splits) — the extra boundary costs less than the serial
  // combine on one CU at every measured split count (profiles/r03/attn_ext_combine.md)
  static const int ext_min = getenv("RT_ATTN_EXT_SPLITS") ? atoi(getenv("RT_ATTN_EXT_SPLITS")) : 2;
  args.ext_combine = (ext_min > 0 && num_splits >= ext_min && probe == 0) ? 1 : 0;
  // A/B knobs (profiles/r05/attn_xcd_ab.md): XCD-aware item order in both launches, and plain
  // (L2-resident) partial stores for the separate combine
  static const int xcd_env = getenv("RT_ATTN_XCD") ? atoi(getenv("RT_ATTN_XCD")) : 0;
  // latency decomposition only (microbench): the attention launch without its combine launch
  static const bool skip_combine = getenv("RT_ATTN_SKIP_COMBINE") && atoi(getenv("RT_ATTN_SKIP_COMBINE")) == 1;
  static const int plain_env = getenv("RT_ATTN_PLAIN_PARTIALS") ? atoi(getenv("RT_ATTN_PLAIN_PARTIALS")) : 0;
  const bool hk_split_ok = Hkv % 8 == 0 || 8 % Hkv == 0;
  args.xcd = (xcd_env && (B * Hkv * num_splits) % 8 == 0 && (B * Hq * (D / 32)) % 8 == 0 && hk_split_ok) ? 1 : 0;
  args.plain_partials = (plain_env && args.ext_combine && !defer_combine) ? 1 : 0;
  const int G = Hq / Hkv;
  // a group's n*G columns need the 16-column LDS merge buffers
  // K/V loop form (attn_core.h PP): the copy-free ping-pong wins where a workgroup streams many
  // tiles (Llama-3-8B tp 1, 8 KV heads: 3 knights x 22K shared keys 29.6 -> 28.7 us, 40K 41.1 ->
  // 40.8 us) and loses ~0.3 us on the short ranges of 1-2 KV-head shards (tp 4 / 8), which keep the
  // copy loop (profiles/r05/attn_pingpong_ab.md). RT_ATTN_PP=0 / 1 pins it (A/B).
  static const int pp_env = getenv("RT_ATTN_PP") ? atoi(getenv("RT_ATTN_PP")) : -1;
  const bool pp = pp_env >= 0 ? pp_env != 0 : Hkv >= 4;
  // K/V load mode (attn_core.h LM_*): nontemporal K and V loads. With the chunk-major K blocks,
  // tp 1, 3 knights x 22K / 40K shared keys 27.6 -> 25.4 / 41.9 -> 37.8 us; rows with distinct
  // contexts B = 1 25K 25.9 -> 23.7, B = 3 25K 59.3 -> 55.3, B = 16 2K 31.0 -> 28.6; tp 8 shard even
  // (profiles/r06/attn_kchunk.md). The one loser: ungrouped rows that read the SAME blocks (3 rows
  // over one 22K prefix without groups, 33.5 -> 35.4: the 2nd / 3rd reads no longer hit L2 / MALL)
  // — the engine decodes shared prefixes as groups, so that case does not arise there.
  // RT_ATTN_LM pins the mode (0 = default policy, 1 = K nt, 2 = V nt, 3 = both; A/B; 7 = both
  // through the LDS-DMA staged loop, ping-pong form only).
  static const int lm_env = getenv("RT_ATTN_LM") ? atoi(getenv("RT_ATTN_LM")) : (LM_NTK | LM_NTV);
  const int lm = (lm_env & LM_GLDS) && pp ? 7 : lm_env & 3;
  args.lm = lm;
#define RT_PD3(DV, PPV, LMV)                                                                                          \
  do {                                                                                                                \
    if (groups != nullptr) hipLaunchKernelGGL((paged_decode_kernel<DV, 16, NW, PPV, LMV>), grid, block, 0, stream, args); \
    else if (G <= 4) hipLaunchKernelGGL((paged_decode_kernel<DV, 4, NW, PPV, LMV>), grid, block, 0, stream, args);   \
    else if (G <= 8) hipLaunchKernelGGL((paged_decode_kernel<DV, 8, NW, PPV, LMV>), grid, block, 0, stream, args);   \
    else hipLaunchKernelGGL((paged_decode_kernel<DV, 16, NW, PPV, LMV>), grid, block, 0, stream, args);              \
  } while (0)
#define RT_PD2(DV, PPV)                             \
  do {                                              \
    if (lm == 0) RT_PD3(DV, PPV, 0);                \
    else if (lm == 1) RT_PD3(DV, PPV, 1);           \
    else if (lm == 2) RT_PD3(DV, PPV, 2);           \
    else if (lm == 3 || !PPV) RT_PD3(DV, PPV, 3);   \
    else RT_PD3(DV, PPV, 7);                        \
  } while (0)
#define RT_PD(DV) do { if (pp) RT_PD2(DV, true); else RT_PD2(DV, false); } while (0)
  // (16-wave grouped workgroups were measured and rejected: __launch_bounds__(1024) caps the item
  // at 128 VGPRs, it spills, and half the CUs stream — 22K shared keys 25.0 -> 41.6 us at 6 splits,
  // profiles/r06/attn_kchunk.md)
  if (D == 128) RT_PD(128);
  else if (D == 64) RT_PD(64);
  else return -2;
#undef RT_PD
#undef RT_PD2
#undef RT_PD3
  if (args.ext_combine && defer_combine && D == 128) {
    // the caller runs the combine inside the next launch (combine_o.hip: combine + o-projection)
    if (deferred != nullptr) *deferred = 1;
  } else if (args.ext_combine && !skip_combine) {
    // slots per row: every split of every member of the largest group (groups: n * G <= 16)
    const int nmax = groups != nullptr ? min(slot_stride, (16 / G) * num_splits) : num_splits;
    // slot-lanes (x 8 dim-lanes) per workgroup, capped at 32 (RT_COMBINE_NSL): fewer, wider lanes
    // (8 slots each for a tp 8 table's 256-slot bound) beat 128 lanes x 2 — 4 waves to dispatch
    // and merge instead of 16; tp 8 grouped attention + combine 12.4 -> 11.6 us
    // (profiles/r04/combine_lanes_ab.md)
    static const int nsl_cap = [] {
      const char* e = getenv("RT_COMBINE_NSL");
      const int v = e ? atoi(e) : 32;
      return (v >= 8 && v <= 128 && v % 8 == 0) ? v : 32;
    }();
    int nsl = min(nsl_cap, (nmax + 7) / 8 * 8);
    int spl = (nmax + nsl - 1) / nsl;                       // slots per lane per chunk
    spl = spl <= 1 ? 1 : (spl <= 2 ? 2 : (spl <= 4 ? 4 : 8));
    if ((nmax + spl - 1) / spl < nsl) nsl = ((nmax + spl - 1) / spl + 7) / 8 * 8;
    const dim3 cgrid(B * Hq, D / 32), cblock(8 * nsl);
#define RT_CB(DV)                                                                                   \
  do {                                                                                              \
    if (spl <= 1) hipLaunchKernelGGL((decode_combine_kernel<DV, 1>), cgrid, cblock, 0, stream, args); \
    else if (spl <= 2) hipLaunchKernelGGL((decode_combine_kernel<DV, 2>), cgrid, cblock, 0, stream, args); \
    else if (spl <= 4) hipLaunchKernelGGL((decode_combine_kernel<DV, 4>), cgrid, cblock, 0, stream, args); \
    else hipLaunchKernelGGL((decode_combine_kernel<DV, 8>), cgrid, cblock, 0, stream, args);          \
  } while (0)
    if (D == 128) RT_CB(128);
    else RT_CB(64);
#undef RT_CB
  }
  return 0;
}

// The per-step plan for launch_paged_decode's ``plan`` (same B, heads, num_splits, groups, block
// tables and lengths as the launches that read it): plan >= B * num_splits * plan_stride ints.
int launch_attn_plan(int* plan, int plan_stride, const int* block_tables, const int* ctx_lens, const int* groups,
                     int B, int Hq, int Hkv, int max_blocks, int num_splits, hipStream_t stream) {
  if (B == 0) return 0;
  if (Hq % Hkv || Hq / Hkv > 16 || num_splits < 1 || num_splits > MAXS || plan_stride <= PLAN_HDR) return -1;
  AttnArgs args{};
  args.block_tables = block_tables;
  args.ctx_lens = ctx_lens;
  args.max_blocks = max_blocks;
  args.num_splits = num_splits;
  args.groups = groups;
  args.plan_stride = plan_stride;
  hipLaunchKernelGGL(attn_plan_kernel, dim3(B, num_splits), dim3(256), 0, stream, args, Hq / Hkv, 16, plan);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
