// pybind11 bindings: torch tensors -> raw HIP launchers on the current HIP stream
// (so every kernel is captured by torch.cuda.graph / hipGraph like any torch op).
// Every entry point validates dtype / device / contiguity / shape BEFORE launching:
// a hand-written kernel must never see operands its grid does not assume.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <vector>

void launch_norm(void* out, const void* x, void* res, const void* w, const void* b, int rows, int H, float eps,
                 bool add, bool ln, hipStream_t stream);
void launch_rope_cache(void* q_out, const void* qkv, const int64_t* positions, const float* cos_sin, void* k_cache,
                       void* v_cache, const int64_t* slots, int T, int Hq, int Hkv, int D, int BS, int64_t qkv_stride,
                       bool rope, hipStream_t stream);
void launch_silu_mul(void* out, const void* x, int rows, int I, hipStream_t stream);
void launch_gelu(void* out, const void* x, int64_t n, hipStream_t stream);
int launch_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                        const int* ctx_lens, float* part_o, float* part_ml, int* counters, int B, int Hq, int Hkv,
                        int D, int max_blocks, float scale, int num_splits, const int* groups, int slot_stride,
                        hipStream_t stream, int defer_combine, int* deferred, const int* plan, int plan_stride);
int launch_attn_plan(int* plan, int plan_stride, const int* block_tables, const int* ctx_lens, const int* groups,
                     int B, int Hq, int Hkv, int max_blocks, int num_splits, hipStream_t stream);
int prefill_rows_per_tile(int G, int D);
int launch_prefill_split(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                         const int* cu_q, const int* start_pos, const int* items, int n_items, const int* cmap,
                         int n_split, float* part_o, float* part_ml, int Hq, int Hkv, int D, int max_blocks,
                         float scale, hipStream_t stream);
int prefill_split_supported(int G, int D);
int launch_prefill(void* out, const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                   const int* cu_q, const int* start_pos, const int* tile_map, int n_tiles, int Hq, int Hkv, int D,
                   int max_blocks, float scale, hipStream_t stream);
int launch_sample(int64_t* out, const void* logits, bool is_bf16, int B, int V, int64_t ld_row,
                  const float* temperature, const float* top_p, const int* top_k, const int64_t* seeds,
                  const int64_t* offsets, float* ws, hipStream_t stream, const void* advance);
int launch_sample_advance(int64_t* tok, const void* logits, bool is_bf16, int B, int V, int64_t ld_row,
                          const float* temperature, const float* top_p, const int* top_k, const int64_t* seeds,
                          int64_t* offsets, float* ws, int64_t* out, int64_t* ids, int64_t* positions, int* ctx_lens,
                          int64_t* step, int max_steps, int64_t* slots, void* res, const int* block_tables,
                          const void* embed, int max_blocks, int BS, int H, int64_t vocab, hipStream_t stream);
int sample_workspace_floats(int B);

int launch_skinny_gemm(void* out, const void* x, const void* Ws, void* res, int M, int N, int K, int ldo, float eps,
                       int pro, int epi, const void* rope, const void* x2, void* xo, hipStream_t stream,
                       int* split_ws, int64_t split_ws_ints, int split_mode);
int split_workspace_ints(int max_split_tiles);
int splitk_parts(int T, int ks, int cus, int64_t ws_ints);
int launch_skinny_gemm_rope(void* q_out, const void* x, const void* Ws, int M, int K, int pro, float eps,
                            const int64_t* positions, const float* cos_sin, void* k_cache, void* v_cache,
                            const int64_t* slots, int Hq, int Hkv, int D, int BS, const void* x2, void* xo,
                            hipStream_t stream, int* split_ws, int64_t split_ws_ints, int split_mode,
                            const float* bias);
int launch_decode_prep(int64_t* slots, int64_t* offsets, void* res, const int64_t* ids, const int64_t* positions,
                       const int* block_tables, const void* embed, int B, int max_blocks, int BS, int H,
                       int64_t vocab, hipStream_t stream);
int launch_paging_guard(const int* block_tables, const int* ctx_lens, const int64_t* positions, const int64_t* slots,
                        int* err, int B, int max_blocks, int num_blocks, int BS, hipStream_t stream);
int launch_decode_advance(int64_t* out, int64_t* ids, int64_t* positions, int* ctx_lens, int64_t* step,
                          const int64_t* next, int B, int max_steps, int64_t* slots, int64_t* offsets, void* res,
                          const int* block_tables, const void* embed, int max_blocks, int BS, int H, int64_t vocab,
                          hipStream_t stream);
int oneshot_create(int world, int rank, int cap_elems, char* handles);
int oneshot_open(int id, const char* all_handles);
int oneshot_capacity(int id);
int oneshot_allreduce(int id, void* inout, int n, void* res, hipStream_t stream);
int oneshot_gemm_ar(int id, void* out, const void* x, const void* Ws, int M, int N, int K, void* res,
                    hipStream_t stream);
int oneshot_allgather(int id, const void* in, void* out, int rows, int shard, hipStream_t stream);
int oneshot_gather_capacity();
int oneshot_handle_bytes();
int oneshot_error(int id);
int oneshot_clear_error(int id);
int oneshot_set_poll_limit(int id, long long limit);
int oneshot_set_ll(int id, int on);
long long oneshot_epoch(int id);
int oneshot_resync(int id, long long epoch);
int sim_comm_spin(long long ticks, int nb, hipStream_t stream);
void oneshot_destroy(int id);
int launch_shuffle_weight(void* Ws, const void* W, const void* gamma, int N, int K, int rope_rows, int D, int swiglu,
                          hipStream_t stream);
int launch_kv_block_copy(void* k, void* v, const int* src, const int* dst, int n, int L, int num_blocks,
                         int64_t block_elems, hipStream_t stream);
int launch_unshuffle_weight(void* W, const void* Ws, int N, int K, int rope_rows, int D, int swiglu,
                            hipStream_t stream);


namespace {
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_gpu(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_bf16(const torch::Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bfloat16");
}
void check_type(const torch::Tensor& t, torch::ScalarType st, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == st, name, " has wrong dtype");
}

void norm_common(torch::Tensor& out, const torch::Tensor& x, torch::Tensor* res, const torch::Tensor& w,
                 const torch::Tensor* b, double eps, bool ln) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  check_bf16(w, "weight");
  const int64_t H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && H <= 32768, "hidden size must be a multiple of 8 and <= 32768");
  TORCH_CHECK(w.numel() == H && out.sizes() == x.sizes(), "norm shape mismatch");
  if (res) {
    check_bf16(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape mismatch");
  }
  if (b) {
    check_bf16(*b, "bias");
    TORCH_CHECK(b->numel() == H, "bias shape mismatch");
  }
  const int rows = (int)(x.numel() / H);
  if (rows == 0) return;
  launch_norm(out.data_ptr(), x.data_ptr(), res ? res->data_ptr() : nullptr, w.data_ptr(), b ? b->data_ptr() : nullptr,
              rows, (int)H, (float)eps, res != nullptr, ln, cur_stream());
}

void rms_norm(torch::Tensor out, torch::Tensor x, torch::Tensor w, double eps) {
  norm_common(out, x, nullptr, w, nullptr, eps, false);
}
void fused_add_rms_norm(torch::Tensor out, torch::Tensor x, torch::Tensor res, torch::Tensor w, double eps) {
  norm_common(out, x, &res, w, nullptr, eps, false);
}
void layer_norm(torch::Tensor out, torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps) {
  norm_common(out, x, nullptr, w, &b, eps, true);
}
void fused_add_layer_norm(torch::Tensor out, torch::Tensor x, torch::Tensor res, torch::Tensor w, torch::Tensor b,
                          double eps) {
  norm_common(out, x, &res, w, &b, eps, true);
}

void check_caches(const torch::Tensor& kc, const torch::Tensor& vc, int64_t Hkv, int64_t D) {
  check_bf16(kc, "k_cache");
  check_bf16(vc, "v_cache");
  TORCH_CHECK(kc.dim() == 4 && vc.dim() == 4, "caches must be 4-D");
  TORCH_CHECK(kc.size(1) == Hkv && kc.size(3) == D, "k_cache must be [NB, Hkv, BS, D]");
  TORCH_CHECK(vc.size(0) == kc.size(0) && vc.size(1) == Hkv && vc.size(2) == D && vc.size(3) == kc.size(2),
              "v_cache must be [NB, Hkv, D, BS]");
}

void rope_and_cache(torch::Tensor q_out, torch::Tensor qkv, torch::Tensor positions, torch::Tensor cos_sin,
                    torch::Tensor k_cache, torch::Tensor v_cache, torch::Tensor slots, int64_t Hq, int64_t Hkv,
                    int64_t D) {
  check_bf16(q_out, "q_out");
  TORCH_CHECK(qkv.is_cuda() && qkv.scalar_type() == torch::kBFloat16 && qkv.stride(-1) == 1, "qkv must be bf16 rows");
  check_type(positions, torch::kInt64, "positions");
  check_type(slots, torch::kInt64, "slot_mapping");
  check_caches(k_cache, v_cache, Hkv, D);
  const int64_t T = qkv.size(0);
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv width mismatch");
  TORCH_CHECK(positions.numel() == T && slots.numel() == T && q_out.numel() == T * Hq * D, "token count mismatch");
  TORCH_CHECK(D % 8 == 0, "head_dim must be a multiple of 8");
  const bool rope = cos_sin.numel() > 0;
  if (rope) {
    check_type(cos_sin, torch::kFloat32, "cos_sin");
    TORCH_CHECK(cos_sin.size(1) == D, "cos_sin must be [max_pos, D]");
  }
  launch_rope_cache(q_out.data_ptr(), qkv.data_ptr(), positions.data_ptr<int64_t>(),
                    rope ? cos_sin.data_ptr<float>() : nullptr, k_cache.data_ptr(), v_cache.data_ptr(),
                    slots.data_ptr<int64_t>(), (int)T, (int)Hq, (int)Hkv, (int)D, (int)k_cache.size(2), qkv.stride(0),
                    rope, cur_stream());
}

int64_t paged_attention_decode(torch::Tensor out, torch::Tensor q, torch::Tensor k_cache, torch::Tensor v_cache,
                               torch::Tensor block_tables, torch::Tensor ctx_lens, double scale, int64_t num_splits,
                               torch::Tensor part_o, torch::Tensor part_ml, torch::Tensor counters,
                               c10::optional<torch::Tensor> groups, int64_t slot_stride, bool defer_combine,
                               c10::optional<torch::Tensor> plan, int64_t plan_stride) {
  check_bf16(out, "out");
  check_bf16(q, "q");
  TORCH_CHECK(q.dim() == 3, "q must be [B, Hq, D]");
  const int64_t B = q.size(0), Hq = q.size(1), D = q.size(2);
  check_caches(k_cache, v_cache, k_cache.size(1), D);
  TORCH_CHECK(k_cache.size(2) == 32, "decode kernel requires kv block_size == 32");
  check_type(block_tables, torch::kInt32, "block_tables");
  check_type(ctx_lens, torch::kInt32, "ctx_lens");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && ctx_lens.numel() >= B, "metadata shape");
  const int* gp = nullptr;
  int64_t stride = num_splits;
  if (groups.has_value() && groups->defined()) {
    check_type(*groups, torch::kInt32, "groups");
    TORCH_CHECK(groups->numel() >= 3 * B, "groups must be [B, 3] int32");
    TORCH_CHECK(slot_stride >= num_splits, "slot_stride must hold n * num_splits partials");
    gp = groups->data_ptr<int>();
    stride = slot_stride;
  }
  check_type(part_o, torch::kFloat32, "partial_o");
  check_type(part_ml, torch::kFloat32, "partial_ml");
  TORCH_CHECK(num_splits >= 1 && part_o.numel() >= B * Hq * stride * D && part_ml.numel() >= B * Hq * stride * 4,
              "split workspace too small");
  check_type(counters, torch::kInt32, "counters");
  TORCH_CHECK(counters.numel() >= B * k_cache.size(1), "split counters too small");
  const int* pp = nullptr;
  if (plan.has_value() && plan->defined()) {
    check_type(*plan, torch::kInt32, "plan");
    TORCH_CHECK(plan_stride > 8 && plan->numel() >= B * num_splits * plan_stride, "attention plan too small");
    pp = plan->data_ptr<int>();
  }
  int deferred = 0;
  const int rc = launch_paged_decode(out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                     block_tables.data_ptr<int>(), ctx_lens.data_ptr<int>(), part_o.data_ptr<float>(),
                                     part_ml.data_ptr<float>(), counters.data_ptr<int>(), (int)B, (int)Hq,
                                     (int)k_cache.size(1), (int)D,
                                     (int)block_tables.size(1), (float)scale, (int)num_splits, gp, (int)stride,
                                     cur_stream(), defer_combine ? 1 : 0, &deferred, pp, (int)plan_stride);
  TORCH_CHECK(rc == 0, "paged_attention_decode: unsupported configuration (rc=", rc, ")");
  return deferred;
}

// per-decode-step attention work plan (attention_decode.hip attn_plan_kernel)
void attn_plan(torch::Tensor plan, int64_t plan_stride, torch::Tensor block_tables, torch::Tensor ctx_lens,
               c10::optional<torch::Tensor> groups, int64_t B, int64_t Hq, int64_t Hkv, int64_t num_splits) {
  check_type(plan, torch::kInt32, "plan");
  check_type(block_tables, torch::kInt32, "block_tables");
  check_type(ctx_lens, torch::kInt32, "ctx_lens");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && ctx_lens.numel() >= B, "metadata shape");
  TORCH_CHECK(plan_stride > 8 && plan.numel() >= B * num_splits * plan_stride, "attention plan too small");
  const int* gp = nullptr;
  if (groups.has_value() && groups->defined()) {
    check_type(*groups, torch::kInt32, "groups");
    TORCH_CHECK(groups->numel() >= 3 * B, "groups must be [B, 3] int32");
    gp = groups->data_ptr<int>();
  }
  const int rc = launch_attn_plan(plan.data_ptr<int>(), (int)plan_stride, block_tables.data_ptr<int>(),
                                  ctx_lens.data_ptr<int>(), gp, (int)B, (int)Hq, (int)Hkv, (int)block_tables.size(1),
                                  (int)num_splits, cur_stream());
  TORCH_CHECK(rc == 0, "attn_plan: unsupported configuration (rc=", rc, ")");
}

void prefill_attention(torch::Tensor out, torch::Tensor q, torch::Tensor k_cache, torch::Tensor v_cache,
                       torch::Tensor block_tables, torch::Tensor cu_q, torch::Tensor start_pos, torch::Tensor tile_map,
                       double scale) {
  check_bf16(out, "out");
  check_bf16(q, "q");
  TORCH_CHECK(q.dim() == 3, "q must be [T, Hq, D]");
  const int64_t Hq = q.size(1), D = q.size(2);
  check_caches(k_cache, v_cache, k_cache.size(1), D);
  TORCH_CHECK(k_cache.size(2) == 32, "prefill kernel requires kv block_size == 32");
  check_type(block_tables, torch::kInt32, "block_tables");
  check_type(cu_q, torch::kInt32, "cu_q");
  check_type(start_pos, torch::kInt32, "start_pos");
  check_type(tile_map, torch::kInt32, "tile_map");
  TORCH_CHECK(block_tables.size(0) == cu_q.numel() - 1 && start_pos.numel() == cu_q.numel() - 1, "varlen metadata");
  TORCH_CHECK(tile_map.dim() == 2 && tile_map.size(1) == 2, "tile_map must be [n, 2]");
  const int rc = launch_prefill(out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                block_tables.data_ptr<int>(), cu_q.data_ptr<int>(), start_pos.data_ptr<int>(),
                                tile_map.data_ptr<int>(), (int)tile_map.size(0), (int)Hq, (int)k_cache.size(1), (int)D,
                                (int)block_tables.size(1), (float)scale, cur_stream());
  TORCH_CHECK(rc == 0, "prefill_attention: unsupported configuration (rc=", rc, ")");
}

void prefill_attention_split(torch::Tensor out, torch::Tensor q, torch::Tensor k_cache, torch::Tensor v_cache,
                             torch::Tensor block_tables, torch::Tensor cu_q, torch::Tensor start_pos,
                             torch::Tensor items, torch::Tensor cmap, torch::Tensor part_o, torch::Tensor part_ml,
                             int64_t n_parts, double scale) {
  check_bf16(out, "out");
  check_bf16(q, "q");
  TORCH_CHECK(q.dim() == 3, "q must be [T, Hq, D]");
  const int64_t Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(1);
  check_caches(k_cache, v_cache, Hkv, D);
  TORCH_CHECK(k_cache.size(2) == 32, "prefill kernel requires kv block_size == 32");
  TORCH_CHECK(prefill_split_supported((int)(Hq / Hkv), (int)D), "prefill_attention_split: needs D 128, G in {1,2,4,8}");
  check_type(block_tables, torch::kInt32, "block_tables");
  check_type(cu_q, torch::kInt32, "cu_q");
  check_type(start_pos, torch::kInt32, "start_pos");
  check_type(items, torch::kInt32, "items");
  check_type(cmap, torch::kInt32, "cmap");
  TORCH_CHECK(block_tables.size(0) == cu_q.numel() - 1 && start_pos.numel() == cu_q.numel() - 1, "varlen metadata");
  TORCH_CHECK(items.dim() == 2 && items.size(1) == 5 && items.is_contiguous(), "items must be [n, 5]");
  TORCH_CHECK(cmap.dim() == 2 && cmap.size(1) == 4 && cmap.is_contiguous(), "cmap must be [m, 4]");
  TORCH_CHECK(part_o.scalar_type() == torch::kFloat32 && part_ml.scalar_type() == torch::kFloat32 &&
                  part_o.is_contiguous() && part_ml.is_contiguous(), "partials must be contiguous fp32");
  TORCH_CHECK(part_o.numel() >= n_parts * Hkv * 8 * 32 * D && part_ml.numel() >= n_parts * Hkv * 8 * 32 * 2,
              "partial buffers too small");
  const int rc = launch_prefill_split(out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                      block_tables.data_ptr<int>(), cu_q.data_ptr<int>(), start_pos.data_ptr<int>(),
                                      items.data_ptr<int>(), (int)items.size(0), cmap.data_ptr<int>(),
                                      (int)cmap.size(0), part_o.data_ptr<float>(), part_ml.data_ptr<float>(), (int)Hq,
                                      (int)Hkv, (int)D, (int)block_tables.size(1), (float)scale, cur_stream());
  TORCH_CHECK(rc == 0, "prefill_attention_split: unsupported configuration (rc=", rc, ")");
}

void silu_and_mul(torch::Tensor out, torch::Tensor x) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  const int64_t I = x.size(-1) / 2;
  TORCH_CHECK(x.size(-1) % 16 == 0 && out.size(-1) == I && out.numel() * 2 == x.numel(), "silu_and_mul shape");
  launch_silu_mul(out.data_ptr(), x.data_ptr(), (int)(x.numel() / x.size(-1)), (int)I, cur_stream());
}

void gelu_tanh(torch::Tensor out, torch::Tensor x) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  TORCH_CHECK(x.numel() % 8 == 0 && out.numel() == x.numel(), "gelu shape");
  launch_gelu(out.data_ptr(), x.data_ptr(), x.numel(), cur_stream());
}

void sample(torch::Tensor out, torch::Tensor logits, torch::Tensor temperature, torch::Tensor top_p,
            torch::Tensor top_k, torch::Tensor seeds, torch::Tensor offsets, torch::Tensor ws) {
  check_type(out, torch::kInt64, "out");
  check_type(ws, torch::kFloat32, "sample workspace");
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits must be [B, V] row-major");
  const bool bf = logits.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == torch::kFloat32, "logits must be bf16 or fp32");
  const int64_t B = logits.size(0);
  check_type(temperature, torch::kFloat32, "temperature");
  check_type(top_p, torch::kFloat32, "top_p");
  check_type(top_k, torch::kInt32, "top_k");
  check_type(seeds, torch::kInt64, "seeds");
  check_type(offsets, torch::kInt64, "offsets");
  TORCH_CHECK(out.numel() >= B && temperature.numel() >= B && top_p.numel() >= B && top_k.numel() >= B &&
                  seeds.numel() >= B && offsets.numel() >= B,
              "sampling parameter vectors shorter than the batch");
  TORCH_CHECK(ws.numel() >= sample_workspace_floats((int)B), "sample workspace too small");
  const int rc = launch_sample(out.data_ptr<int64_t>(), logits.data_ptr(), bf, (int)B, (int)logits.size(1),
                               logits.stride(0), temperature.data_ptr<float>(), top_p.data_ptr<float>(),
                               top_k.data_ptr<int>(), seeds.data_ptr<int64_t>(), offsets.data_ptr<int64_t>(),
                               ws.data_ptr<float>(), cur_stream(), nullptr);
  TORCH_CHECK(rc == 0, "sample: rc=", rc);
}

// The captured decode step's sampler fused with decode_advance + next-step decode_prep (one launch).
// `offsets` is read as the sampler's RNG offsets AND rewritten with the next step's.
void sample_advance(torch::Tensor tok, torch::Tensor logits, torch::Tensor temperature, torch::Tensor top_p,
                    torch::Tensor top_k, torch::Tensor seeds, torch::Tensor offsets, torch::Tensor ws,
                    torch::Tensor out, torch::Tensor ids, torch::Tensor positions, torch::Tensor ctx_lens,
                    torch::Tensor step, torch::Tensor slots, torch::Tensor res, torch::Tensor block_tables,
                    torch::Tensor embed, int64_t block_size) {
  check_type(tok, torch::kInt64, "tok");
  check_type(ws, torch::kFloat32, "sample workspace");
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits must be [B, V] row-major");
  const bool bf = logits.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == torch::kFloat32, "logits must be bf16 or fp32");
  const int64_t B = logits.size(0);
  check_type(temperature, torch::kFloat32, "temperature");
  check_type(top_p, torch::kFloat32, "top_p");
  check_type(top_k, torch::kInt32, "top_k");
  check_type(seeds, torch::kInt64, "seeds");
  check_type(offsets, torch::kInt64, "offsets");
  check_type(out, torch::kInt64, "out");
  check_type(ids, torch::kInt64, "ids");
  check_type(positions, torch::kInt64, "positions");
  check_type(ctx_lens, torch::kInt32, "ctx_lens");
  check_type(step, torch::kInt64, "step");
  check_type(slots, torch::kInt64, "slots");
  check_type(block_tables, torch::kInt32, "block_tables");
  check_bf16(res, "res");
  check_bf16(embed, "embed");
  TORCH_CHECK(tok.numel() >= B && temperature.numel() >= B && top_p.numel() >= B && top_k.numel() >= B &&
                  seeds.numel() >= B && offsets.numel() >= B && ids.numel() == B && positions.numel() == B &&
                  ctx_lens.numel() == B && slots.numel() >= B && out.dim() == 2 && out.size(1) == B &&
                  block_tables.size(0) >= B && res.dim() == 2 && res.size(0) == B && embed.dim() == 2 &&
                  res.size(1) == embed.size(1) && block_size > 0,
              "sample_advance: shapes");
  TORCH_CHECK(ws.numel() >= sample_workspace_floats((int)B), "sample workspace too small");
  const int rc = launch_sample_advance(
      tok.data_ptr<int64_t>(), logits.data_ptr(), bf, (int)B, (int)logits.size(1), logits.stride(0),
      temperature.data_ptr<float>(), top_p.data_ptr<float>(), top_k.data_ptr<int>(), seeds.data_ptr<int64_t>(),
      offsets.data_ptr<int64_t>(), ws.data_ptr<float>(), out.data_ptr<int64_t>(), ids.data_ptr<int64_t>(),
      positions.data_ptr<int64_t>(), ctx_lens.data_ptr<int>(), step.data_ptr<int64_t>(), (int)out.size(0),
      slots.data_ptr<int64_t>(), res.data_ptr(), block_tables.data_ptr<int>(), embed.data_ptr(),
      (int)block_tables.size(1), (int)block_size, (int)embed.size(1), embed.size(0), cur_stream());
  TORCH_CHECK(rc == 0, "sample_advance: rc=", rc);
}
// Ws: fragment-shuffled weight [N_w, K] (N_w = 2N for SwiGLU); out [M, N] (unused for RESID).
// PRO_NORM_ADD (pro=2): x2 [M,K] is added to x before the norm; xout (optional) receives x + x2.
std::pair<const void*, void*> add_operands(const torch::Tensor& x, int64_t pro, const c10::optional<torch::Tensor>& x2,
                                           const c10::optional<torch::Tensor>& xout) {
  if (pro != 2) return {nullptr, nullptr};
  TORCH_CHECK(x2.has_value(), "pro=NORM_ADD needs x2");
  check_bf16(*x2, "x2");
  TORCH_CHECK(x2->sizes() == x.sizes(), "x2 must match x");
  void* xo = nullptr;
  if (xout.has_value()) {
    check_bf16(*xout, "xout");
    TORCH_CHECK(xout->sizes() == x.sizes(), "xout must match x");
    TORCH_CHECK(xout->data_ptr() != x.data_ptr() && xout->data_ptr() != x2->data_ptr(), "xout must not alias x / x2");
    xo = xout->data_ptr();
  }
  return {x2->data_ptr(), xo};
}

void skinny_gemm(torch::Tensor out, torch::Tensor x, torch::Tensor Ws, int64_t pro, int64_t epi,
                 c10::optional<torch::Tensor> res, double eps, c10::optional<torch::Tensor> x2,
                 c10::optional<torch::Tensor> xout, c10::optional<torch::Tensor> split_ws, int64_t split_mode) {
  check_bf16(x, "x");
  check_bf16(Ws, "Ws");
  TORCH_CHECK(x.dim() == 2 && Ws.dim() == 2 && x.size(1) == Ws.size(1), "skinny_gemm: x [M,K], Ws [N,K]");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 32, "skinny_gemm: 1 <= M <= 32");
  TORCH_CHECK(K % 32 == 0, "skinny_gemm: K must be a multiple of 32");
  int64_t N = Ws.size(0);
  if (epi == 2) {
    TORCH_CHECK(N % 32 == 0, "swiglu W must stack [gate; up]");
    N /= 2;
  }
  TORCH_CHECK(N % 16 == 0, "skinny_gemm: N must be a multiple of 16");
  void* rp = nullptr;
  int64_t ldo = N;
  if (epi == 1) {
    TORCH_CHECK(res.has_value(), "resid epilogue needs res");
    check_bf16(*res, "res");
    TORCH_CHECK(res->dim() == 2 && res->size(0) == M && res->size(1) == N, "resid epilogue shapes");
    rp = res->data_ptr();
  } else {
    check_bf16(out, "out");
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N, "out must be [M, N]");
    ldo = out.stride(0);
  }
  const auto addo = add_operands(x, pro, x2, xout);
  int* sw = nullptr;
  int64_t sw_n = 0;
  if (split_ws.has_value()) {   // split-K / CU-balanced launch workspace (counters zero between calls)
    TORCH_CHECK(split_ws->scalar_type() == torch::kInt32 && split_ws->is_contiguous() &&
                    split_ws->device() == x.device(), "split_ws: contiguous int32 on x's device");
    sw = split_ws->data_ptr<int>();
    sw_n = split_ws->numel();
  }
  const int rc = launch_skinny_gemm(epi == 1 ? nullptr : out.data_ptr(), x.data_ptr(), Ws.data_ptr(), rp, (int)M,
                                    (int)N, (int)K, (int)ldo, (float)eps, (int)pro, (int)epi, nullptr, addo.first,
                                    addo.second, cur_stream(), sw, sw_n, (int)split_mode);
  TORCH_CHECK(rc == 0, "skinny_gemm: unsupported configuration (rc=", rc, ")");
}

// qkv decode projection with the RoPE + paged-cache epilogue (Ws built with rope_heads = Hq + Hkv).
void skinny_gemm_rope(torch::Tensor q_out, torch::Tensor x, torch::Tensor Ws, int64_t pro, torch::Tensor positions,
                      torch::Tensor cos_sin, torch::Tensor k_cache, torch::Tensor v_cache, torch::Tensor slots,
                      int64_t Hq, int64_t Hkv, int64_t D, double eps, c10::optional<torch::Tensor> x2,
                      c10::optional<torch::Tensor> xout, c10::optional<torch::Tensor> split_ws,
                      int64_t split_mode, c10::optional<torch::Tensor> bias) {
  check_bf16(q_out, "q_out");
  check_bf16(x, "x");
  check_bf16(Ws, "Ws");
  TORCH_CHECK(x.dim() == 2 && Ws.dim() == 2 && x.size(1) == Ws.size(1), "skinny_gemm_rope: x [M,K], Ws [N,K]");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 32 && K % 32 == 0, "skinny_gemm_rope: 1 <= M <= 32, K % 32 == 0");
  TORCH_CHECK(Ws.size(0) == (Hq + 2 * Hkv) * D && D % 16 == 0, "skinny_gemm_rope: Ws must be [(Hq+2Hkv)*D, K]");
  TORCH_CHECK(q_out.numel() == M * Hq * D, "q_out must be [M, Hq, D]");
  check_type(positions, torch::kInt64, "positions");
  check_type(slots, torch::kInt64, "slots");
  check_type(cos_sin, torch::kFloat32, "cos_sin");
  TORCH_CHECK(positions.numel() >= M && slots.numel() >= M, "positions/slots must cover M rows");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D, "cos_sin must be [max_pos, D]");
  check_caches(k_cache, v_cache, Hkv, D);
  if (bias.has_value())   // fp32, already in the ROPE epilogue's column order (ops.rope_bias)
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->is_contiguous() && bias->numel() == Ws.size(0) &&
                    bias->device() == x.device(), "skinny_gemm_rope: bias must be contiguous fp32 [N] on x's device");
  const auto addo = add_operands(x, pro, x2, xout);
  int* sw = nullptr;
  int64_t sw_n = 0;
  if (split_ws.has_value()) {   // split-K / CU-balanced launch workspace (counters zero between calls)
    TORCH_CHECK(split_ws->scalar_type() == torch::kInt32 && split_ws->is_contiguous() &&
                    split_ws->device() == x.device(), "split_ws: contiguous int32 on x's device");
    sw = split_ws->data_ptr<int>();
    sw_n = split_ws->numel();
  }
  const int rc = launch_skinny_gemm_rope(q_out.data_ptr(), x.data_ptr(), Ws.data_ptr(), (int)M, (int)K, (int)pro,
                                         (float)eps, positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(),
                                         k_cache.data_ptr(), v_cache.data_ptr(), slots.data_ptr<int64_t>(), (int)Hq,
                                         (int)Hkv, (int)D, (int)k_cache.size(2), addo.first, addo.second,
                                         cur_stream(), sw, sw_n, (int)split_mode,
                                         bias.has_value() ? bias->data_ptr<float>() : nullptr);
  TORCH_CHECK(rc == 0, "skinny_gemm_rope: unsupported configuration (rc=", rc, ")");
}


// K9 one-shot all-reduce over IPC-mapped peer buffers (csrc/oneshot_ar.hip).
py::tuple py_oneshot_create(int64_t world, int64_t rank, int64_t cap_elems) {
  std::vector<char> h((size_t)oneshot_handle_bytes(), 0);
  const int id = oneshot_create((int)world, (int)rank, (int)cap_elems, h.data());
  TORCH_CHECK(id >= 0, "oneshot_create failed (rc=", id, ")");
  return py::make_tuple(id, py::bytes(h.data(), h.size()));
}
void py_oneshot_open(int64_t id, py::bytes all_handles, int64_t world) {
  const std::string hs = all_handles;
  TORCH_CHECK((int64_t)hs.size() == world * oneshot_handle_bytes(), "oneshot_open: need world x ",
              oneshot_handle_bytes(), " handle bytes");
  const int rc = oneshot_open((int)id, hs.data());
  TORCH_CHECK(rc == 0, "oneshot_open: hipIpcOpenMemHandle failed (rc=", rc, ")");
}
// res (optional): the residual form, res = bf16(res + bf16(sum over ranks of x)) in place, x kept.
void py_oneshot_allreduce(int64_t id, torch::Tensor x, c10::optional<torch::Tensor> res) {
  check_bf16(x, "oneshot_allreduce input");
  TORCH_CHECK(x.numel() % 8 == 0 && x.numel() <= oneshot_capacity((int)id), "oneshot_allreduce: size");
  void* rp = nullptr;
  if (res.has_value()) {
    check_bf16(*res, "oneshot_allreduce res");
    TORCH_CHECK(res->numel() == x.numel(), "oneshot_allreduce: res must match x");
    rp = res->data_ptr();
  }
  const int rc = oneshot_allreduce((int)id, x.data_ptr(), (int)x.numel(), rp, cur_stream());
  TORCH_CHECK(rc == 0, "oneshot_allreduce failed (rc=", rc, ")");
}
// One-shot all-gather along the last dim (C3 logits): out [rows, world * shard] from in [rows, shard].
void py_oneshot_allgather(int64_t id, torch::Tensor in, torch::Tensor out, int64_t world) {
  check_bf16(in, "oneshot_allgather in");
  check_bf16(out, "oneshot_allgather out");
  TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && out.size(0) == in.size(0) && out.size(1) == in.size(1) * world,
              "oneshot_allgather: in [rows, shard], out [rows, world * shard]");
  const int rc = oneshot_allgather((int)id, in.data_ptr(), out.data_ptr(), (int)in.size(0), (int)in.size(1),
                                   cur_stream());
  TORCH_CHECK(rc == 0, "oneshot_allgather: unsupported configuration (rc=", rc, ")");
}
// Row-parallel decode GEMM with the K9 exchange fused into its epilogue (EPI_AR).
// res (optional): the residual form — res [M,N] += the all-reduced product (bf16-rounded), in place.
void py_oneshot_gemm_ar(int64_t id, torch::Tensor out, torch::Tensor x, torch::Tensor Ws,
                        c10::optional<torch::Tensor> res) {
  check_bf16(out, "oneshot_gemm_ar out");
  check_bf16(x, "oneshot_gemm_ar x");
  check_bf16(Ws, "oneshot_gemm_ar Ws");
  TORCH_CHECK(x.dim() == 2 && Ws.dim() == 2 && x.size(1) == Ws.size(1), "oneshot_gemm_ar: x [M,K], Ws [N,K]");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == x.size(0) && out.size(1) == Ws.size(0), "oneshot_gemm_ar: out [M,N]");
  void* rp = nullptr;
  if (res.has_value()) {
    check_bf16(*res, "oneshot_gemm_ar res");
    TORCH_CHECK(res->dim() == 2 && res->size(0) == x.size(0) && res->size(1) == Ws.size(0),
                "oneshot_gemm_ar: res [M,N]");
    rp = res->data_ptr();
  }
  const int rc = oneshot_gemm_ar((int)id, out.data_ptr(), x.data_ptr(), Ws.data_ptr(), (int)x.size(0),
                                 (int)Ws.size(0), (int)x.size(1), rp, cur_stream());
  TORCH_CHECK(rc == 0, "oneshot_gemm_ar: unsupported configuration (rc=", rc, ")");
}

// Decode-step bookkeeping (csrc/decode_step.hip).
void decode_prep(torch::Tensor slots, torch::Tensor offsets, torch::Tensor res, torch::Tensor ids,
                 torch::Tensor positions, torch::Tensor block_tables, torch::Tensor embed, int64_t block_size) {
  check_type(slots, torch::kInt64, "slots");
  check_type(offsets, torch::kInt64, "offsets");
  check_type(ids, torch::kInt64, "ids");
  check_type(positions, torch::kInt64, "positions");
  check_type(block_tables, torch::kInt32, "block_tables");
  check_bf16(res, "res");
  check_bf16(embed, "embed");
  const int64_t B = ids.numel();
  TORCH_CHECK(slots.numel() >= B && offsets.numel() >= B && positions.numel() >= B && block_tables.size(0) >= B,
              "decode_prep: batch sizes");
  TORCH_CHECK(res.dim() == 2 && res.size(0) == B && embed.dim() == 2 && res.size(1) == embed.size(1),
              "decode_prep: res [B, H], embed [V, H]");
  const int rc = launch_decode_prep(slots.data_ptr<int64_t>(), offsets.data_ptr<int64_t>(), res.data_ptr(),
                                    ids.data_ptr<int64_t>(), positions.data_ptr<int64_t>(),
                                    block_tables.data_ptr<int>(), embed.data_ptr(), (int)B, (int)block_tables.size(1),
                                    (int)block_size, (int)embed.size(1), embed.size(0), cur_stream());
  TORCH_CHECK(rc == 0, "decode_prep: unsupported configuration (rc=", rc, ")");
}

void decode_advance(torch::Tensor out, torch::Tensor ids, torch::Tensor positions, torch::Tensor ctx_lens,
                    torch::Tensor step, torch::Tensor next, c10::optional<torch::Tensor> slots,
                    c10::optional<torch::Tensor> offsets, c10::optional<torch::Tensor> res,
                    c10::optional<torch::Tensor> block_tables, c10::optional<torch::Tensor> embed, int64_t block_size) {
  check_type(out, torch::kInt64, "out");
  check_type(ids, torch::kInt64, "ids");
  check_type(positions, torch::kInt64, "positions");
  check_type(ctx_lens, torch::kInt32, "ctx_lens");
  check_type(step, torch::kInt64, "step");
  check_type(next, torch::kInt64, "next");
  const int64_t B = ids.numel();
  TORCH_CHECK(out.dim() == 2 && out.size(1) == B && next.numel() == B && positions.numel() == B &&
                  ctx_lens.numel() == B,
              "decode_advance: shapes");
  int64_t* sp = nullptr;
  int64_t* op = nullptr;
  void* rp = nullptr;
  const int* btp = nullptr;
  const void* ep = nullptr;
  int maxb = 0, H = 0;
  int64_t V = 0;
  if (res.has_value() && res->defined()) {   // fused next-step prep (decode_prep semantics)
    TORCH_CHECK(slots.has_value() && offsets.has_value() && block_tables.has_value() && embed.has_value(),
                "decode_advance: prep needs slots, offsets, block_tables, embed");
    check_type(*slots, torch::kInt64, "slots");
    check_type(*offsets, torch::kInt64, "offsets");
    check_type(*block_tables, torch::kInt32, "block_tables");
    check_bf16(*res, "res");
    check_bf16(*embed, "embed");
    TORCH_CHECK(slots->numel() >= B && offsets->numel() >= B && block_tables->size(0) >= B && res->dim() == 2 &&
                    res->size(0) == B && embed->dim() == 2 && res->size(1) == embed->size(1) && block_size > 0,
                "decode_advance: prep shapes");
    sp = slots->data_ptr<int64_t>();
    op = offsets->data_ptr<int64_t>();
    rp = res->data_ptr();
    btp = block_tables->data_ptr<int>();
    ep = embed->data_ptr();
    maxb = (int)block_tables->size(1);
    H = (int)embed->size(1);
    V = embed->size(0);
  }
  const int rc = launch_decode_advance(out.data_ptr<int64_t>(), ids.data_ptr<int64_t>(), positions.data_ptr<int64_t>(),
                                       ctx_lens.data_ptr<int>(), step.data_ptr<int64_t>(), next.data_ptr<int64_t>(),
                                       (int)B, (int)out.size(0), sp, op, rp, btp, ep, maxb, (int)block_size, H, V,
                                       cur_stream());
  TORCH_CHECK(rc == 0, "decode_advance: unsupported configuration (rc=", rc, ")");
}

// Debug paging guard (csrc/decode_step.hip): err[0] |= violation code; capturable.
void paging_guard(torch::Tensor block_tables, torch::Tensor ctx_lens, c10::optional<torch::Tensor> positions,
                  c10::optional<torch::Tensor> slots, torch::Tensor err, int64_t num_blocks, int64_t block_size) {
  check_type(block_tables, torch::kInt32, "block_tables");
  check_type(ctx_lens, torch::kInt32, "ctx_lens");
  check_type(err, torch::kInt32, "err");
  const int64_t B = ctx_lens.numel();
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && block_tables.is_contiguous(),
              "paging_guard: block_tables [B, max_blocks]");
  const int64_t* pp = nullptr;
  const int64_t* sp = nullptr;
  if (positions && positions->defined()) {
    check_type(*positions, torch::kInt64, "positions");
    TORCH_CHECK(positions->numel() >= B, "paging_guard: positions");
    pp = positions->data_ptr<int64_t>();
  }
  if (slots && slots->defined()) {
    check_type(*slots, torch::kInt64, "slots");
    TORCH_CHECK(slots->numel() >= B, "paging_guard: slots");
    sp = slots->data_ptr<int64_t>();
  }
  const int rc = launch_paging_guard(block_tables.data_ptr<int>(), ctx_lens.data_ptr<int>(), pp, sp,
                                     err.data_ptr<int>(), (int)B, (int)block_tables.size(1), (int)num_blocks,
                                     (int)block_size, cur_stream());
  TORCH_CHECK(rc == 0, "paging_guard: rc=", rc);
}

void shuffle_weight(torch::Tensor Ws, torch::Tensor W, c10::optional<torch::Tensor> gamma, int64_t rope_heads,
                    int64_t head_dim, bool swiglu) {
  check_bf16(Ws, "Ws");
  check_bf16(W, "W");
  TORCH_CHECK(W.dim() == 2 && Ws.sizes() == W.sizes(), "shuffle_weight shapes");
  TORCH_CHECK(W.size(0) % 16 == 0 && W.size(1) % 32 == 0, "shuffle_weight: N%16, K%32");
  const void* gp = nullptr;
  if (gamma.has_value()) {
    check_bf16(*gamma, "gamma");
    TORCH_CHECK(gamma->numel() == W.size(1), "gamma must have K elements");
    gp = gamma->data_ptr();
  }
  const int rc = launch_shuffle_weight(Ws.data_ptr(), W.data_ptr(), gp, (int)W.size(0), (int)W.size(1),
                                       (int)(rope_heads * head_dim), (int)head_dim, swiglu ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "shuffle_weight: unsupported configuration (rc=", rc, ")");
}
void unshuffle_weight(torch::Tensor W, torch::Tensor Ws, int64_t rope_heads, int64_t head_dim, bool swiglu) {
  check_bf16(W, "W");
  check_bf16(Ws, "Ws");
  TORCH_CHECK(W.dim() == 2 && Ws.numel() == W.numel(), "unshuffle_weight shapes");
  const int rc = launch_unshuffle_weight(W.data_ptr(), Ws.data_ptr(), (int)W.size(0), (int)W.size(1),
                                         (int)(rope_heads * head_dim), (int)head_dim, swiglu ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "unshuffle_weight: unsupported configuration (rc=", rc, ")");
}
void kv_block_copy(torch::Tensor k, torch::Tensor v, torch::Tensor src, torch::Tensor dst) {
  check_bf16(k, "k_cache");
  check_bf16(v, "v_cache");
  TORCH_CHECK(k.dim() == 3 && k.sizes() == v.sizes(), "caches must be [L, NB, block_elems]");
  check_type(src, torch::kInt32, "src");
  check_type(dst, torch::kInt32, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "src/dst length");
  const int64_t nb = k.size(1);
  if (src.numel() == 0) return;
  // host-side validation before the launch: every id in range, no duplicate destination
  auto s = src.cpu(), d = dst.cpu();
  std::vector<char> seen(nb, 0);
  for (int64_t i = 0; i < s.numel(); ++i) {
    const int a = s.data_ptr<int>()[i], b = d.data_ptr<int>()[i];
    TORCH_CHECK(a >= 0 && a < nb && b >= 0 && b < nb, "kv_block_copy: block id out of range");
    TORCH_CHECK(!seen[b], "kv_block_copy: duplicate destination block");
    seen[b] = 1;
  }
  const int rc = launch_kv_block_copy(k.data_ptr(), v.data_ptr(), src.data_ptr<int>(), dst.data_ptr<int>(),
                                      (int)src.numel(), (int)k.size(0), (int)nb, k.size(2), cur_stream());
  TORCH_CHECK(rc == 0, "kv_block_copy: unsupported configuration (rc=", rc, ")");
}
}  // namespace

PYBIND11_MODULE(_C, m) {
  m.def("skinny_gemm", &skinny_gemm, "decode GEMM (M<=16), shuffled weights, fused norm / resid / swiglu",
        py::arg("out"), py::arg("x"), py::arg("Ws"), py::arg("pro"), py::arg("epi"), py::arg("res") = py::none(),
        py::arg("eps") = 1e-5, py::arg("x2") = py::none(), py::arg("xout") = py::none(),
        py::arg("split_ws") = py::none(), py::arg("split_mode") = 3);
  m.def("split_workspace_ints", &split_workspace_ints, "int32 words of a skinny_gemm split_ws for R split tiles");
  m.def("splitk_parts", [](int64_t T, int64_t ks, int64_t cus, int64_t ws_ints) {
    return splitk_parts((int)T, (int)ks, (int)cus, ws_ints);
  }, "split-K part count the launcher picks for T tiles x ks k-steps on `cus` CUs (0 = none)");
  m.def("shuffle_weight", &shuffle_weight, py::arg("Ws"), py::arg("W"), py::arg("gamma") = py::none(),
        py::arg("rope_heads") = 0, py::arg("head_dim") = 0, py::arg("swiglu") = false);
  m.def("kv_block_copy", &kv_block_copy, py::arg("k"), py::arg("v"), py::arg("src"), py::arg("dst"));
  m.def("unshuffle_weight", &unshuffle_weight, py::arg("W"), py::arg("Ws"), py::arg("rope_heads") = 0,
        py::arg("head_dim") = 0, py::arg("swiglu") = false);
  m.def("decode_prep", &decode_prep);
  m.def("oneshot_create", &py_oneshot_create, py::arg("world"), py::arg("rank"), py::arg("cap_elems"));
  m.def("oneshot_open", &py_oneshot_open, py::arg("id"), py::arg("all_handles"), py::arg("world"));
  m.def("oneshot_allreduce", &py_oneshot_allreduce, py::arg("id"), py::arg("x"), py::arg("res") = py::none());
  m.def("oneshot_gemm_ar", &py_oneshot_gemm_ar, py::arg("id"), py::arg("out"), py::arg("x"), py::arg("Ws"),
        py::arg("res") = py::none());
  m.def("oneshot_allgather", &py_oneshot_allgather, py::arg("id"), py::arg("in"), py::arg("out"), py::arg("world"));
  m.def("oneshot_gather_capacity", []() { return oneshot_gather_capacity(); });
  m.def("oneshot_capacity", [](int64_t id) { return oneshot_capacity((int)id); });
  m.def("oneshot_error", [](int64_t id) { return oneshot_error((int)id); });
  m.def("oneshot_clear_error", [](int64_t id) { return oneshot_clear_error((int)id); });
  m.def("oneshot_set_poll_limit", [](int64_t id, int64_t limit) { return oneshot_set_poll_limit((int)id, limit); });
  m.def("oneshot_set_ll", [](int64_t id, bool on) { return oneshot_set_ll((int)id, on ? 1 : 0); });
  m.def("sim_comm_spin", [](int64_t ticks, int64_t nb) {
    const int rc = sim_comm_spin((long long)ticks, (int)nb, cur_stream());
    TORCH_CHECK(rc == 0, "sim_comm_spin failed (rc=", rc, ")");
  });
  m.def("oneshot_epoch", [](int64_t id) { return (int64_t)oneshot_epoch((int)id); });
  m.def("oneshot_resync", [](int64_t id, int64_t epoch) { return oneshot_resync((int)id, (long long)epoch); });
  m.def("oneshot_destroy", [](int64_t id) { oneshot_destroy((int)id); });
  m.def("decode_advance", &decode_advance, py::arg("out"), py::arg("ids"), py::arg("positions"), py::arg("ctx_lens"),
        py::arg("step"), py::arg("next"), py::arg("slots") = py::none(), py::arg("offsets") = py::none(),
        py::arg("res") = py::none(), py::arg("block_tables") = py::none(), py::arg("embed") = py::none(),
        py::arg("block_size") = 0);
  m.def("paging_guard", &paging_guard, py::arg("block_tables"), py::arg("ctx_lens"), py::arg("positions"),
        py::arg("slots"), py::arg("err"), py::arg("num_blocks"), py::arg("block_size"));
  m.def("skinny_gemm_rope", &skinny_gemm_rope, "qkv decode GEMM with fused RoPE + paged K/V cache write",
        py::arg("q_out"), py::arg("x"), py::arg("Ws"), py::arg("pro"), py::arg("positions"), py::arg("cos_sin"),
        py::arg("k_cache"), py::arg("v_cache"), py::arg("slots"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"),
        py::arg("eps"), py::arg("x2") = py::none(), py::arg("xout") = py::none(),
        py::arg("split_ws") = py::none(), py::arg("split_mode") = 3, py::arg("bias") = py::none());
  m.doc() = "theroundtaible_amd CDNA4 (gfx950) HIP kernels";
  m.def("rms_norm", &rms_norm);
  m.def("fused_add_rms_norm", &fused_add_rms_norm);
  m.def("layer_norm", &layer_norm);
  m.def("fused_add_layer_norm", &fused_add_layer_norm);
  m.def("rope_and_cache", &rope_and_cache);
  m.def("paged_attention_decode", &paged_attention_decode, py::arg("out"), py::arg("q"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("block_tables"), py::arg("ctx_lens"), py::arg("scale"), py::arg("num_splits"),
        py::arg("part_o"), py::arg("part_ml"), py::arg("counters"), py::arg("groups") = py::none(),
        py::arg("slot_stride") = 0, py::arg("defer_combine") = false, py::arg("plan") = py::none(),
        py::arg("plan_stride") = 0);
  m.def("attn_plan", &attn_plan, py::arg("plan"), py::arg("plan_stride"), py::arg("block_tables"),
        py::arg("ctx_lens"), py::arg("groups"), py::arg("B"), py::arg("Hq"), py::arg("Hkv"), py::arg("num_splits"));
  m.def("prefill_rows_per_tile", &prefill_rows_per_tile, py::arg("G"), py::arg("D") = 128);
  m.def("prefill_attention", &prefill_attention);
  m.def("prefill_attention_split", &prefill_attention_split);
  m.def("prefill_split_supported", &prefill_split_supported, py::arg("G"), py::arg("D") = 128);
  m.def("silu_and_mul", &silu_and_mul);
  m.def("gelu_tanh", &gelu_tanh);
  m.def("sample", &sample);
  m.def("sample_advance", &sample_advance);
  m.def("sample_workspace_floats", &sample_workspace_floats);
  m.attr("arch") = "gfx950";
}
