// pybind11 bindings of the EXPERIMENT kernels kept out of the product extension (measured
// slower than the five-launch fused decode or never adopted; profiles/experiments/): the
// persistent decode layer, the loader-wave LDS-ring GEMM, the MALL prefetch and the split combine
// folded into the o-projection launch. Built on demand
// by tools/experiments/build_exp.py into tools/experiments/_exp*.so.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

int launch_decode_layer(void* res, void* q, void* a, void* g, const void* wqkv, const void* wo, const void* wgu,
                        const void* wd, const int64_t* positions, const float* cos_sin, void* k_cache, void* v_cache,
                        const int64_t* slots, const int* block_tables, const int* ctx_lens, float* part_o,
                        float* part_ml, int* split_counters, int* sync, int* err, long long* stamps, int M, int H,
                        int I, int Hq, int Hkv, int head_dim, int BS, int max_blocks, int num_splits, float eps,
                        float scale, hipStream_t stream);
int decode_layer_grid();
int launch_fused_mlp(void* res, void* g, const void* wgu, const void* wd, int* ws, int S, int* sync, int* err, int M,
                     int H, int I, float eps, int grid, int phases, hipStream_t stream);
int launch_ring_gemm(void* out, const void* x, const void* Ws, int M, int N, int K, int grid, int variant,
                     hipStream_t stream);
int launch_prefetch(const void* p, int64_t nbytes, int nwg, uint32_t* sink, hipStream_t stream);
int launch_combine_o(void* attn_out, const float* part_o, const float* part_ml, const int* groups, int stride,
                     int num_splits, int B, int Hq, int Hkv, int D, const void* Ws, void* res, int N, int* bar,
                     int* err, hipStream_t stream);

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
void check_caches(const torch::Tensor& k, const torch::Tensor& v, int64_t Hkv, int64_t D) {
  check_bf16(k, "k_cache");
  check_bf16(v, "v_cache");
  TORCH_CHECK(k.dim() == 4 && v.dim() == 4 && k.size(1) == Hkv && k.size(3) == D && v.size(1) == Hkv &&
                  v.size(2) == D && v.size(3) == k.size(2) && v.size(0) == k.size(0),
              "caches must be k [NB, Hkv, BS, D], v [NB, Hkv, D, BS]");
}

// EXPERIMENT: loader-wave + LDS-ring decode GEMM (csrc/ring_gemm.hip), microbenchmarks only.
void ring_gemm_exp(torch::Tensor out, torch::Tensor x, torch::Tensor Ws, int64_t grid, int64_t variant) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  check_bf16(Ws, "Ws");
  TORCH_CHECK(x.dim() == 2 && Ws.dim() == 2 && x.size(1) == Ws.size(1) && out.size(0) == x.size(0) &&
                  out.size(1) == Ws.size(0),
              "ring_gemm_exp: shapes");
  const int rc = launch_ring_gemm(out.data_ptr(), x.data_ptr(), Ws.data_ptr(), (int)x.size(0), (int)Ws.size(0),
                                  (int)x.size(1), (int)grid, (int)variant, cur_stream());
  TORCH_CHECK(rc == 0, "ring_gemm_exp: unsupported configuration (rc=", rc, ")");
}

// Persistent decode layer (csrc/decode_layer.hip): one launch = qkv -> attention -> o -> gate_up -> down.
void decode_layer(torch::Tensor res, torch::Tensor q, torch::Tensor a, torch::Tensor g, torch::Tensor wqkv,
                  torch::Tensor wo, torch::Tensor wgu, torch::Tensor wd, torch::Tensor positions, torch::Tensor cos_sin,
                  torch::Tensor k_cache, torch::Tensor v_cache, torch::Tensor slots, torch::Tensor block_tables,
                  torch::Tensor ctx_lens, torch::Tensor part_o, torch::Tensor part_ml, torch::Tensor split_counters,
                  torch::Tensor sync, torch::Tensor err, int64_t Hq, int64_t Hkv, int64_t num_splits, double eps,
                  double scale, c10::optional<torch::Tensor> stamps) {
  for (auto* t : {&res, &q, &a, &g, &wqkv, &wo, &wgu, &wd}) check_bf16(*t, "decode_layer operand");
  const int64_t M = res.size(0), H = res.size(1), I = g.size(1), D = q.size(-1);
  TORCH_CHECK(res.dim() == 2 && g.dim() == 2 && g.size(0) == M && a.numel() == M * Hq * D && q.numel() == M * Hq * D,
              "decode_layer: activation shapes");
  TORCH_CHECK(wqkv.size(0) == (Hq + 2 * Hkv) * D && wqkv.size(1) == H && wo.size(0) == H && wo.size(1) == Hq * D &&
                  wgu.size(0) == 2 * I && wgu.size(1) == H && wd.size(0) == H && wd.size(1) == I,
              "decode_layer: weight shapes");
  check_caches(k_cache, v_cache, Hkv, D);
  check_type(positions, torch::kInt64, "positions");
  check_type(slots, torch::kInt64, "slots");
  check_type(cos_sin, torch::kFloat32, "cos_sin");
  check_type(block_tables, torch::kInt32, "block_tables");
  check_type(ctx_lens, torch::kInt32, "ctx_lens");
  check_type(part_o, torch::kFloat32, "part_o");
  check_type(part_ml, torch::kFloat32, "part_ml");
  check_type(split_counters, torch::kInt32, "split_counters");
  check_type(sync, torch::kInt32, "sync");
  check_type(err, torch::kInt32, "err");
  TORCH_CHECK(positions.numel() >= M && slots.numel() >= M && ctx_lens.numel() >= M && block_tables.size(0) >= M,
              "decode_layer: metadata rows");
  TORCH_CHECK(part_o.numel() >= M * Hq * num_splits * D && part_ml.numel() >= M * Hq * num_splits * 4 &&
                  split_counters.numel() >= M * Hkv && sync.numel() >= 5 && err.numel() >= 1,
              "decode_layer: workspace too small");
  const int rc = launch_decode_layer(
      res.data_ptr(), q.data_ptr(), a.data_ptr(), g.data_ptr(), wqkv.data_ptr(), wo.data_ptr(), wgu.data_ptr(),
      wd.data_ptr(), positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(), k_cache.data_ptr(), v_cache.data_ptr(),
      slots.data_ptr<int64_t>(), block_tables.data_ptr<int>(), ctx_lens.data_ptr<int>(), part_o.data_ptr<float>(),
      part_ml.data_ptr<float>(), split_counters.data_ptr<int>(), sync.data_ptr<int>(), err.data_ptr<int>(),
      stamps.has_value() ? (long long*)stamps->data_ptr<int64_t>() : nullptr, (int)M,
      (int)H, (int)I, (int)Hq, (int)Hkv, (int)D, (int)k_cache.size(2), (int)block_tables.size(1), (int)num_splits,
      (float)eps, (float)scale, cur_stream());
  TORCH_CHECK(rc == 0, "decode_layer: unsupported configuration (rc=", rc, ")");
}

// Pull a tensor's bytes into the MALL ahead of its consumer (side-stream warm-up).
void prefetch(torch::Tensor t, int64_t nwg, torch::Tensor sink) {
  check_gpu(t, "t");
  check_type(sink, torch::kInt32, "sink");
  launch_prefetch(t.data_ptr(), t.numel() * t.element_size(), (int)nwg, (uint32_t*)sink.data_ptr(), cur_stream());
}

// K3 split combine + o-projection + residual in one launch (tools/experiments/combine_o.hip), after a
// paged_attention_decode call that returned 1 (combine deferred) with the same workspace.
void combine_o_gemm(torch::Tensor attn_out, torch::Tensor part_o, torch::Tensor part_ml,
                    c10::optional<torch::Tensor> groups, int64_t slot_stride, int64_t num_splits, int64_t Hkv,
                    torch::Tensor Ws, torch::Tensor res, torch::Tensor bar, torch::Tensor err) {
  check_bf16(attn_out, "attn_out");
  check_bf16(Ws, "Ws");
  check_bf16(res, "res");
  TORCH_CHECK(attn_out.dim() == 3, "attn_out must be [B, Hq, D]");
  const int64_t B = attn_out.size(0), Hq = attn_out.size(1), D = attn_out.size(2);
  TORCH_CHECK(Ws.dim() == 2 && Ws.size(1) == Hq * D && res.dim() == 2 && res.size(0) == B && res.size(1) == Ws.size(0),
              "combine_o_gemm: Ws [N, Hq*D], res [B, N]");
  check_type(part_o, torch::kFloat32, "partial_o");
  check_type(part_ml, torch::kFloat32, "partial_ml");
  check_type(bar, torch::kInt32, "bar");
  check_type(err, torch::kInt32, "err");
  TORCH_CHECK(bar.numel() >= 2 && err.numel() >= 1, "combine_o_gemm: bar [2], err [1]");
  const int* gp = nullptr;
  int64_t stride = num_splits;
  if (groups.has_value() && groups->defined()) {
    check_type(*groups, torch::kInt32, "groups");
    TORCH_CHECK(groups->numel() >= 3 * B && slot_stride >= num_splits, "groups / slot_stride");
    gp = groups->data_ptr<int>();
    stride = slot_stride;
  }
  TORCH_CHECK(part_o.numel() >= B * Hq * stride * D && part_ml.numel() >= B * Hq * stride * 4, "split workspace too small");
  const int rc = launch_combine_o(attn_out.data_ptr(), part_o.data_ptr<float>(), part_ml.data_ptr<float>(), gp,
                                  (int)stride, (int)num_splits, (int)B, (int)Hq, (int)Hkv, (int)D, Ws.data_ptr(),
                                  res.data_ptr(), (int)Ws.size(0), bar.data_ptr<int>(), err.data_ptr<int>(),
                                  cur_stream());
  TORCH_CHECK(rc == 0, "combine_o_gemm: unsupported configuration (rc=", rc, ")");
}

}  // namespace

PYBIND11_MODULE(_exp, m) {
  m.def("decode_layer", &decode_layer, py::arg("res"), py::arg("q"), py::arg("a"), py::arg("g"), py::arg("wqkv"),
        py::arg("wo"), py::arg("wgu"), py::arg("wd"), py::arg("positions"), py::arg("cos_sin"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("slots"), py::arg("block_tables"), py::arg("ctx_lens"), py::arg("part_o"),
        py::arg("part_ml"), py::arg("split_counters"), py::arg("sync"), py::arg("err"), py::arg("Hq"),
        py::arg("Hkv"), py::arg("num_splits"), py::arg("eps"), py::arg("scale"), py::arg("stamps") = py::none());
  m.def("decode_layer_grid", &decode_layer_grid);
  m.def("fused_mlp", [](torch::Tensor res, torch::Tensor g, torch::Tensor wgu, torch::Tensor wd, torch::Tensor ws,
                        int64_t S, torch::Tensor sync, torch::Tensor err, double eps, int64_t grid, int64_t phases) {
    check_bf16(res, "res");
    check_bf16(g, "g");
    check_bf16(wgu, "wgu");
    check_bf16(wd, "wd");
    check_type(ws, torch::kInt32, "ws");
    check_type(sync, torch::kInt32, "sync");
    check_type(err, torch::kInt32, "err");
    const int64_t M = res.size(0), H = res.size(1), I = g.size(1);
    TORCH_CHECK(g.size(0) == M && wgu.numel() == 2 * I * H && wd.numel() == H * I && sync.numel() >= ((phases & 16) ? 576 : 2) &&
                    grid > 0 && grid <= decode_layer_grid(),
                "fused_mlp: shapes / grid (must not exceed the CU count: every workgroup resident)");
    const int rc = launch_fused_mlp(res.data_ptr(), g.data_ptr(), wgu.data_ptr(), wd.data_ptr(), ws.data_ptr<int>(),
                                    (int)S, sync.data_ptr<int>(), err.data_ptr<int>(), (int)M, (int)H, (int)I,
                                    (float)eps, (int)grid, (int)phases, cur_stream());
    TORCH_CHECK(rc == 0, "fused_mlp: unsupported configuration (rc=", rc, ")");
  });
  m.def("ring_gemm_exp", &ring_gemm_exp, py::arg("out"), py::arg("x"), py::arg("Ws"), py::arg("grid") = 0,
        py::arg("variant") = 0);
  m.def("prefetch", &prefetch, py::arg("t"), py::arg("nwg"), py::arg("sink"));
  m.def("combine_o_gemm", &combine_o_gemm, py::arg("attn_out"), py::arg("part_o"), py::arg("part_ml"),
        py::arg("groups"), py::arg("slot_stride"), py::arg("num_splits"), py::arg("Hkv"), py::arg("Ws"),
        py::arg("res"), py::arg("bar"), py::arg("err"));
}
