// Probe: under ROC_GLOBAL_CU_MASK, do all blocks of a launch run, and on which XCDs / CUs?
//   ROC_GLOBAL_CU_MASK=0xffffffff ./cu_mask_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void record(int* out) {
  if (threadIdx.x == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));       // HW_REG_XCC_ID
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));        // HW_REG_HW_ID
    out[2 * blockIdx.x] = (int)xcc;
    out[2 * blockIdx.x + 1] = (int)hw;
  }
}

int main() {
  const int n = 1024;
  int* d;
  hipMalloc(&d, 2 * n * sizeof(int));
  hipMemset(d, 0xff, 2 * n * sizeof(int));
  hipLaunchKernelGGL(record, dim3(n), dim3(64), 0, 0, d);
  hipError_t e = hipDeviceSynchronize();
  std::vector<int> h(2 * n);
  hipMemcpy(h.data(), d, 2 * n * sizeof(int), hipMemcpyDeviceToHost);
  int ran = 0, xcc_count[8] = {0};
  std::vector<int> cus;
  for (int b = 0; b < n; ++b) {
    if (h[2 * b] < 0) continue;
    ++ran;
    if (h[2 * b] < 8) ++xcc_count[h[2 * b]];
    const int hw = h[2 * b + 1];
    const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    const int key = h[2 * b] * 1000 + se * 100 + sh * 16 + cu;
    bool seen = false;
    for (int k : cus) seen |= k == key;
    if (!seen) cus.push_back(key);
  }
  const char* m = getenv("ROC_GLOBAL_CU_MASK");
  printf("mask=%s status=%s blocks ran %d / %d, distinct CUs %zu, per XCC:", m ? m : "(none)", hipGetErrorString(e), ran,
         n, cus.size());
  for (int x = 0; x < 8; ++x) printf(" %d", xcc_count[x]);
  printf("\n");
  return 0;
}
