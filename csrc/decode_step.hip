// Per-token bookkeeping of the captured decode step, fused into two tiny launches (was ~12
// PyTorch elementwise kernels ≈ 45 µs per token, profiles/r01_*_v3*.md):
//
//   decode_prep    : slot[b]   = block_tables[b][pos/BS] * BS + pos % BS   (K/V write slot)
//                    offset[b] = pos + 1                                   (sampler RNG offset)
//                    res[b, :] = embed[ids[b], :]                          (embedding gather)
//   decode_advance : out[step, b] = next[b]; ids[b] = next[b]; pos[b] += 1; ctx[b] += 1;
//                    step += 1                                              (after sampling)
//                    and, given the prep operands, the NEXT step's decode_prep from the new
//                    ids / positions (the captured step then has one bookkeeping launch; the
//                    first step of a turn is prepped once, outside the graph)
//
// Everything the next replay needs stays on the device, so a hipGraph replay takes no host
// input. One workgroup per batch row; the embedding row copy is 16 B per lane.
#include "common.h"

namespace {
__global__ void __launch_bounds__(256) decode_prep_kernel(
    int64_t* __restrict__ slots, int64_t* __restrict__ offsets, uint16_t* __restrict__ res,
    const int64_t* __restrict__ ids, const int64_t* __restrict__ positions, const int* __restrict__ block_tables,
    const uint16_t* __restrict__ embed, int max_blocks, int BS, int H, int64_t vocab) {
  const int b = blockIdx.x;
  const int64_t pos = positions[b];
  if (threadIdx.x == 0) {
    const int64_t bi = pos / BS;   // past the table: a slot that is never written
    const int64_t blk = bi < max_blocks ? block_tables[(size_t)b * max_blocks + bi] : 0;
    slots[b] = blk * BS + pos % BS;
    offsets[b] = pos + 1;
  }
  int64_t tok = ids[b];
  tok = tok < 0 ? 0 : (tok >= vocab ? vocab - 1 : tok);
  const uint4* src = reinterpret_cast<const uint4*>(embed + (size_t)tok * H);
  uint4* dst = reinterpret_cast<uint4*>(res + (size_t)b * H);
  for (int i = threadIdx.x; i < H / 8; i += blockDim.x) dst[i] = src[i];
}

struct PrepArgs {   // next-step prep (all null: advance only)
  int64_t* slots;
  int64_t* offsets;
  uint16_t* res;
  const int* block_tables;
  const uint16_t* embed;
  int max_blocks, BS, H;
  int64_t vocab;
};

__global__ void __launch_bounds__(256) decode_advance_kernel(int64_t* __restrict__ out, int64_t* __restrict__ ids,
                                                             int64_t* __restrict__ positions, int* __restrict__ ctx_lens,
                                                             int64_t* __restrict__ step, const int64_t* __restrict__ next,
                                                             int B, int max_steps, PrepArgs pa) {
  const int64_t st = *step;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int64_t t = next[b];
    if (st < max_steps) out[st * B + b] = t;
    ids[b] = t;
    const int64_t p = positions[b] + 1;
    positions[b] = p;
    ctx_lens[b] += 1;
    if (pa.slots != nullptr) {   // past the table (a turn's last step) the slot is never used
      const int64_t bi = p / pa.BS;
      const int64_t blk = bi < pa.max_blocks ? pa.block_tables[(size_t)b * pa.max_blocks + bi] : 0;
      pa.slots[b] = blk * pa.BS + p % pa.BS;
      pa.offsets[b] = p + 1;
    }
  }
  if (pa.res != nullptr) {       // next step's embedding rows, 16 B per lane
    const int row8 = pa.H / 8;
    for (int i = threadIdx.x; i < B * row8; i += blockDim.x) {
      const int b = i / row8, j = i - b * row8;
      int64_t tok = next[b];
      tok = tok < 0 ? 0 : (tok >= pa.vocab ? pa.vocab - 1 : tok);
      reinterpret_cast<uint4*>(pa.res)[(size_t)b * row8 + j] =
          reinterpret_cast<const uint4*>(pa.embed)[(size_t)tok * row8 + j];
    }
  }
  __syncthreads();  // every lane has read *step before lane 0 bumps it
  if (threadIdx.x == 0) *step = st + 1;
}
}  // namespace

int launch_decode_prep(int64_t* slots, int64_t* offsets, void* res, const int64_t* ids, const int64_t* positions,
                       const int* block_tables, const void* embed, int B, int max_blocks, int BS, int H,
                       int64_t vocab, hipStream_t stream) {
  if (B <= 0) return 0;
  if (H % 8) return -1;
  hipLaunchKernelGGL(decode_prep_kernel, dim3(B), dim3(256), 0, stream, slots, offsets, (uint16_t*)res, ids,
                     positions, block_tables, (const uint16_t*)embed, max_blocks, BS, H, vocab);
  return 0;
}

int launch_decode_advance(int64_t* out, int64_t* ids, int64_t* positions, int* ctx_lens, int64_t* step,
                          const int64_t* next, int B, int max_steps, int64_t* slots, int64_t* offsets, void* res,
                          const int* block_tables, const void* embed, int max_blocks, int BS, int H, int64_t vocab,
                          hipStream_t stream) {
  if (B <= 0) return 0;
  const bool prep = res != nullptr;
  if (prep && (slots == nullptr || offsets == nullptr || block_tables == nullptr || embed == nullptr || H % 8 ||
               BS <= 0 || max_blocks <= 0 || vocab <= 0))
    return -1;
  const PrepArgs pa{prep ? slots : nullptr, prep ? offsets : nullptr, (uint16_t*)res, block_tables,
                    (const uint16_t*)embed, max_blocks, BS, H, vocab};
  hipLaunchKernelGGL(decode_advance_kernel, dim3(1), dim3(256), 0, stream, out, ids, positions, ctx_lens, step, next,
                     B, max_steps, pa);
  return 0;
}

// ---- debug variant: paging guard (ROUNDTABLE_DEBUG_CHECKS=1) ------------------------
// Validates, on the device and inside the captured step, the paging metadata every later kernel
// of the step dereferences — host asserts cannot see the slots / lengths the graph advances
// itself. Violations OR a code into err[0]; the host reads it at its sync points:
//   1 = ctx_len outside [1, max_blocks * BS]     2 = block-table entry outside [0, num_blocks)
//   4 = write slot != block_tables[pos / BS] * BS + pos % BS    8 = ctx_len != position + 1
namespace {
__global__ void __launch_bounds__(256) paging_guard_kernel(const int* __restrict__ block_tables,
                                                           const int* __restrict__ ctx_lens,
                                                           const int64_t* __restrict__ positions,
                                                           const int64_t* __restrict__ slots, int* __restrict__ err,
                                                           int max_blocks, int num_blocks, int BS) {
  const int b = blockIdx.x;
  const int ctx = ctx_lens[b];
  const int* bt = block_tables + (size_t)b * max_blocks;
  int code = 0;
  if (ctx < 1 || ctx > max_blocks * BS) code |= 1;
  const int nt = min((max(ctx, 0) + BS - 1) / BS, max_blocks);
  for (int t = threadIdx.x; t < nt; t += blockDim.x) {
    const int blk = bt[t];
    if (blk < 0 || blk >= num_blocks) code |= 2;
  }
  if (threadIdx.x == 0 && positions != nullptr) {
    const int64_t pos = positions[b];
    if (pos + 1 != ctx) code |= 8;
    if (slots != nullptr && pos >= 0 && pos / BS < max_blocks) {
      const int64_t want = (int64_t)bt[pos / BS] * BS + pos % BS;
      if (slots[b] != want) code |= 4;
    }
  }
  if (code) atomicOr(err, code);
}
}  // namespace

int launch_paging_guard(const int* block_tables, const int* ctx_lens, const int64_t* positions, const int64_t* slots,
                        int* err, int B, int max_blocks, int num_blocks, int BS, hipStream_t stream) {
  if (B <= 0) return 0;
  if (max_blocks <= 0 || BS <= 0) return -1;
  hipLaunchKernelGGL(paging_guard_kernel, dim3(B), dim3(256), 0, stream, block_tables, ctx_lens, positions, slots, err,
                     max_blocks, num_blocks, BS);
  return 0;
}
