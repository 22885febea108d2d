// Host-side argument validation of the HIP launchers, built with AddressSanitizer +
// UndefinedBehaviorSanitizer on the HOST code only (GPU ASan / xnack+ is not
// available on the MI355X pool). Every case below must be rejected BEFORE any HIP call, so
// the binary runs on a machine without a GPU. Build + run: tests/test_native_host_sanitizers.py.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

int launch_skinny_gemm(void* out, const void* x, const void* Ws, void* res, int M, int N, int K, int ldo, float eps,
                       int pro, int epi, const void* rope, const void* x2, void* xo, hipStream_t stream,
                       int* split_ws, int64_t split_ws_ints, int split_mode);
int splitk_parts(int T, int ks, int cus, int64_t ws_ints);
int launch_shuffle_weight(void* Ws, const void* W, const void* gamma, int N, int K, int rope_rows, int D, int swiglu,
                          hipStream_t stream);
int launch_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                        const int* ctx_lens, float* part_o, float* part_ml, int* counters, int B, int Hq, int Hkv,
                        int D, int max_blocks, float scale, int num_splits, const int* groups, int slot_stride,
                        hipStream_t stream, int defer_combine, int* deferred, const int* plan = nullptr,
                        int plan_stride = 0);
int launch_paging_guard(const int* block_tables, const int* ctx_lens, const int64_t* positions, const int64_t* slots,
                        int* err, int B, int max_blocks, int num_blocks, int BS, hipStream_t stream);
int launch_decode_advance(int64_t* out, int64_t* ids, int64_t* positions, int* ctx_lens, int64_t* step,
                          const int64_t* next, int B, int max_steps, int64_t* slots, int64_t* offsets, void* res,
                          const int* block_tables, const void* embed, int max_blocks, int BS, int H, int64_t vocab,
                          hipStream_t stream);
int prefill32_rows(int G);
int launch_kv_block_copy(void* k, void* v, const int* src, const int* dst, int n, int L, int num_blocks,
                         int64_t block_elems, hipStream_t stream);
int launch_unshuffle_weight(void* W, const void* Ws, int N, int K, int rope_rows, int D, int swiglu,
                            hipStream_t stream);

static int failures = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

int main() {
  // decode GEMM: M outside [1, 32] (17..32 only with plain / norm prologues and no all-reduce), K not a
  // multiple of 32, N not a multiple of 16, missing operands
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 0, 16, 64, 16, 1e-5f, 0, 0, nullptr, nullptr,
                            nullptr, nullptr, nullptr, 0, 3) == -1);
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 33, 16, 64, 16, 1e-5f, 0, 0, nullptr, nullptr,
                            nullptr, nullptr, nullptr, 0, 3) == -1);
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 17, 16, 64, 16, 1e-5f, 2, 0, nullptr, nullptr,
                            nullptr, nullptr, nullptr, 0, 3) == -5);   // NORM_ADD without its operand
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 17, 16, 64, 16, 1e-5f, 2, 0, nullptr, (const void*)1,
                            nullptr, nullptr, nullptr, 0, 3) == -1);   // NORM_ADD above 16 rows
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 3, 16, 48, 16, 1e-5f, 0, 0, nullptr, nullptr,
                            nullptr, nullptr, nullptr, 0, 3) == -1);
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 3, 24, 64, 24, 1e-5f, 0, 0, nullptr, nullptr,
                            nullptr, nullptr, nullptr, 0, 3) == -1);
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 3, 16, 64, 16, 1e-5f, 2, 0, nullptr, nullptr,
                            nullptr, nullptr, nullptr, 0, 3) == -5);   // NORM_ADD without its second operand
  EXPECT(launch_skinny_gemm(nullptr, nullptr, nullptr, nullptr, 3, 16, 64, 16, 1e-5f, 0, 3, nullptr, nullptr,
                            nullptr, nullptr, nullptr, 0, 3) == -3);   // ROPE epilogue without its parameters
  // split-K part choice: only with fewer tiles than CUs, >= 8 k-steps per part, within the workspace
  EXPECT(splitk_parts(384, 128, 256, 1 << 20) == 0);          // tp=1 qkv: tiles >= CUs, no split
  EXPECT(splitk_parts(48, 128, 256, 1 << 20) >= 2);           // tp=8 qkv shard
  EXPECT(splitk_parts(48, 8, 256, 1 << 20) == 0);             // one part of 8 k-steps only
  EXPECT(splitk_parts(48, 128, 256, 256 + 2 * 528 * 48 - 1) == 0);   // workspace below 2 parts
  EXPECT(splitk_parts(100, 128, 0, 1 << 20) == 0);            // unknown CU count
  EXPECT(launch_shuffle_weight(nullptr, nullptr, nullptr, 16, 48, 0, 0, 0, nullptr) == -1);
  EXPECT(launch_shuffle_weight(nullptr, nullptr, nullptr, 32, 64, 64, 128, 0, nullptr) == -1);   // rope rows > N
  EXPECT(launch_shuffle_weight(nullptr, nullptr, nullptr, 48, 64, 0, 0, 1, nullptr) == -1);      // SwiGLU halves of 24 rows
  // decode attention: group size, head dim, split range
  EXPECT(launch_paged_decode(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 2, 30, 8,
                             128, 4, 0.1f, 4, nullptr, 0, nullptr, 0, nullptr) == -1);
  EXPECT(launch_paged_decode(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 2, 64, 2,
                             128, 4, 0.1f, 4, nullptr, 0, nullptr, 0, nullptr) == -1);   // G = 32 > 16
  EXPECT(launch_paged_decode(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 2, 32, 8,
                             128, 4, 0.1f, 65, nullptr, 0, nullptr, 0, nullptr) == -3);  // splits > MAXS
  EXPECT(launch_paged_decode(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 32, 8,
                             128, 4, 0.1f, 4, nullptr, 0, nullptr, 0, nullptr) == 0);    // empty batch: no launch
  static const int grp[3] = {0, 1, 0};
  EXPECT(launch_paged_decode(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 2, 32, 8,
                             128, 4, 0.1f, 4, grp, 2, nullptr, 0, nullptr) == -4);   // group slots < splits
  // K8 block copy: empty list launches nothing; unaligned block size / empty layer set refused
  EXPECT(launch_kv_block_copy(nullptr, nullptr, nullptr, nullptr, 0, 32, 16, 8192, nullptr) == 0);
  EXPECT(launch_kv_block_copy(nullptr, nullptr, nullptr, nullptr, 2, 32, 16, 8190, nullptr) == -1);
  EXPECT(launch_kv_block_copy(nullptr, nullptr, nullptr, nullptr, 2, 0, 16, 8192, nullptr) == -1);
  // weight unshuffle: N%16, K%32, rope rows beyond N
  EXPECT(launch_unshuffle_weight(nullptr, nullptr, 24, 64, 0, 0, 0, nullptr) == -1);
  EXPECT(launch_unshuffle_weight(nullptr, nullptr, 32, 48, 0, 0, 0, nullptr) == -1);
  EXPECT(launch_unshuffle_weight(nullptr, nullptr, 32, 64, 64, 128, 0, nullptr) == -1);
  EXPECT(launch_paging_guard(nullptr, nullptr, nullptr, nullptr, nullptr, 2, 0, 16, 32, nullptr) == -1);
  EXPECT(launch_paging_guard(nullptr, nullptr, nullptr, nullptr, nullptr, 0, 4, 16, 32, nullptr) == 0);
  EXPECT(launch_decode_advance(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 8, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, 0, nullptr) == 0);
  // prefill tile geometry
  // (a group that is not a power of two takes the next power of two of head slots: G = 3 -> 4,
  // G = 7 -> 8; past 8 the 16x16 kernel runs)
  EXPECT(prefill32_rows(4) == 64 && prefill32_rows(8) == 32 && prefill32_rows(1) == 256 && prefill32_rows(3) == 64 &&
         prefill32_rows(7) == 32 && prefill32_rows(5) == 32 && prefill32_rows(12) == 0 && prefill32_rows(16) == 0);
  std::printf("host_check: %d failure(s)\n", failures);
  return failures ? 1 : 0;
}
