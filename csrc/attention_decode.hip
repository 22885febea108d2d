// K3: paged-KV decode attention (one query token per sequence), GQA, MFMA bf16, split-KV.
// The work-item code is in attn_core.h (shared with the persistent decode-layer kernel); this
// file holds the grid launch: blockIdx = (sequence x kv head, key split).
#include "attn_core.h"

#include <cstdlib>

namespace {
using namespace attn;

template <int D, int GM, int W = NW>
__global__ void __launch_bounds__(W * 64) paged_decode_kernel(AttnArgs p) {
  __shared__ AttnSmem<D, GM, W> sm;
  attn_item<D, false, GM, W>(p, blockIdx.x, blockIdx.y, sm);
}
}  // namespace


// q [B, Hq, D]; k_cache [NB, Hkv, 32, D]; v_cache [NB, Hkv, D, 32]; block_tables [B, max_blocks] int32;
// part_o >= B*Hq*slot_stride*D floats, part_ml >= B*Hq*slot_stride*4 floats, counters >= B*Hkv ints
// (zeroed once). groups: nullptr or [B][3] {first, n, shared blocks} (shared-prefix groups,
// attn_core.h); slot_stride >= max n * num_splits (0 = num_splits, no groups).
int launch_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                        const int* ctx_lens, float* part_o, float* part_ml, int* counters, int B, int Hq, int Hkv,
                        int D, int max_blocks, float scale, int num_splits, const int* groups, int slot_stride,
                        hipStream_t stream) {
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
  const int G = Hq / Hkv;
  // a group's n*G columns need the 16-column LDS merge buffers
#define RT_PD(DV)                                                                                  \
  do {                                                                                             \
    if (groups != nullptr) hipLaunchKernelGGL((paged_decode_kernel<DV, 16>), grid, block, 0, stream, args); \
    else if (G <= 4) hipLaunchKernelGGL((paged_decode_kernel<DV, 4>), grid, block, 0, stream, args);   \
    else if (G <= 8) hipLaunchKernelGGL((paged_decode_kernel<DV, 8>), grid, block, 0, stream, args); \
    else hipLaunchKernelGGL((paged_decode_kernel<DV, 16>), grid, block, 0, stream, args);         \
  } while (0)
  if (D == 128) RT_PD(128);
  else if (D == 64) RT_PD(64);
  else return -2;
#undef RT_PD
  return 0;
}
