// CU-mask probe (diagnostic tool, not product): which CUs a CU-masked stream's workgroups land on,
// and whether two streams' kernels run concurrently.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <set>

__global__ void where(uint32_t* out, uint64_t spin) {
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {}
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2] = xcc & 0xF;
    out[blockIdx.x * 2 + 1] = hw;
  }
}

static void run(const char* name, const std::vector<uint32_t>& mask) {
  hipStream_t s;
  if (mask.empty()) hipStreamCreate(&s);
  else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) { printf("%s: mask refused\n", name); return; }
  const int n = 2048;
  uint32_t* d; hipMalloc(&d, n * 8);
  hipLaunchKernelGGL(where, dim3(n), dim3(64), 0, s, d, 2000ull);
  hipStreamSynchronize(s);
  std::vector<uint32_t> h(n * 2);
  hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
  std::set<uint32_t> cus; int per_xcc[16] = {0};
  for (int i = 0; i < n; ++i) {
    const uint32_t x = h[2 * i], hw = h[2 * i + 1];
    const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    cus.insert((x << 8) | (se << 5) | (sh << 4) | cu);
    per_xcc[x]++;
  }
  printf("%s: %zu distinct (xcc,se,sh,cu); blocks per xcc:", name, cus.size());
  for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
  printf("\n  cus:");
  int k = 0;
  for (uint32_t c : cus) { if (k++ < 40) printf(" %u.%u.%u.%u", c >> 8, (c >> 5) & 7, (c >> 4) & 1, c & 15); }
  printf("\n");
  hipFree(d); hipStreamDestroy(s);
}

int main() {
  run("nomask", {});
  std::vector<uint32_t> m(8, 0);
  m[0] = 0xFFFFFFFFu;  // bits 0..31
  run("bits0-31", m);
  std::fill(m.begin(), m.end(), 0); m[0] = 0x0000000Fu;
  run("bits0-3", m);
  std::fill(m.begin(), m.end(), 0); for (int i = 0; i < 8; ++i) m[i] = 0x1u;
  run("bit0 of each word", m);
  std::fill(m.begin(), m.end(), 0xFFFFFFFFu); m[0] = 0;
  run("all but bits0-31", m);
  return 0;
}
