// Probe: which XCD (HW_REG_XCC_ID) each workgroup of consecutive launches runs on. Do blocks
// b and b + 8 share an XCD, and does class b % 8 map to the SAME XCD in the next launch (the
// premise of an XCD-aware producer / consumer remap across a kernel boundary)?
//   hipcc --offload-arch=gfx950 -O2 tools/probes/xcc_probe.hip -o xcc_probe && ./xcc_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void record_xcc(int* out) {
  if (threadIdx.x == 0) {
    const unsigned id = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));   // HW_REG_XCC_ID[3:0]
    out[blockIdx.x] = (int)id;
  }
}

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    printf("%s: %s\n", what, hipGetErrorString(e));
    exit(1);
  }
}

int main() {
  // a decode-step-like sequence: 192 (attention), 384 (combine), 256 (o), 100 (odd), 192, 384
  const std::vector<int> grids = {192, 384, 256, 100, 192, 384, 1536, 192, 384};
  const int reps = 50;
  std::vector<int*> dev(grids.size());
  for (size_t k = 0; k < grids.size(); ++k) check(hipMalloc(&dev[k], grids[k] * reps * sizeof(int)), "malloc");
  hipStream_t s;
  check(hipStreamCreate(&s), "stream");
  for (int r = 0; r < reps; ++r)
    for (size_t k = 0; k < grids.size(); ++k)
      hipLaunchKernelGGL(record_xcc, dim3(grids[k]), dim3(64), 0, s, dev[k] + r * grids[k]);
  check(hipStreamSynchronize(s), "sync");
  int consistent_within = 0, total = 0, same_as_prev = 0, pairs = 0;
  std::vector<std::vector<int>> cls(grids.size() * reps, std::vector<int>(8, -1));
  for (int r = 0; r < reps; ++r)
    for (size_t k = 0; k < grids.size(); ++k) {
      std::vector<int> h(grids[k]);
      check(hipMemcpy(h.data(), dev[k] + r * grids[k], grids[k] * sizeof(int), hipMemcpyDeviceToHost), "copy");
      auto& c = cls[r * grids.size() + k];
      bool ok = true;
      for (int b = 0; b < grids[k]; ++b) {
        if (c[b % 8] < 0) c[b % 8] = h[b];
        ok = ok && c[b % 8] == h[b];
      }
      consistent_within += ok;
      ++total;
      if (r == 0 && k < 3) {
        printf("launch %zu (%d blocks) class->xcc:", k, grids[k]);
        for (int j = 0; j < 8; ++j) printf(" %d", c[j]);
        printf("\n");
      }
    }
  for (size_t i = 1; i < cls.size(); ++i) {
    same_as_prev += cls[i] == cls[i - 1];
    ++pairs;
  }
  // per transition type: after a launch of G blocks, is the next launch's mapping the same?
  for (size_t k = 0; k < grids.size(); ++k) {
    int same = 0, n = 0;
    for (int r = 0; r < reps; ++r) {
      const size_t i = r * grids.size() + k;
      if (i + 1 >= cls.size()) continue;
      same += cls[i + 1] == cls[i];
      ++n;
    }
    printf("after a %d-block launch: next launch's class->xcc mapping identical in %d / %d\n", grids[k], same, n);
  }
  printf("launches whose blocks b, b+8, ... share one XCD: %d / %d; consecutive launches with identical mapping: %d / %d\n",
         consistent_within, total, same_as_prev, pairs);
  return 0;
}
