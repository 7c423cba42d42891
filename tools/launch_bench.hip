// launch_bench.hip — host-side cost of the per-batch launch pattern (diagnostic, not engine code).
// Measures host wall time per iteration for: (a) 1 empty launch, (b) 2 launches on one stream,
// (c) 3 launches over prep/main streams with an event record + stream wait (the engine's
// per-batch pattern), and the GPU-side time of back-to-back small kernels.
// Build: hipcc -O3 --offload-arch=gfx950 tools/launch_bench.hip -o tools/launch_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

struct Args { unsigned* p; unsigned n; unsigned pad[30]; };  // ~128 B kernarg like the engine's

__global__ void k_small(Args a) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.n == 0xFFFFFFFFu) a.p[0] = 1;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev[8];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  Args a{};
  CK(hipMalloc(&a.p, 64));
  const int N = 20000;
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; ++i) {
        if (mode == 0) {
          hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s0, a);
        } else if (mode == 1) {
          hipLaunchKernelGGL(k_small, dim3(32), dim3(256), 0, s0, a);
          hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s0, a);
        } else if (mode == 2) {
          hipStream_t ps = (i & 1) ? s1 : s2;
          hipLaunchKernelGGL(k_small, dim3(32), dim3(256), 0, ps, a);
          hipLaunchKernelGGL(k_small, dim3(16), dim3(256), 0, ps, a);
          hipEventRecord(ev[i & 7], ps);
          hipStreamWaitEvent(s0, ev[i & 7], 0);
          hipLaunchKernelGGL(k_small, dim3(512), dim3(256), 0, s0, a);
          hipEventRecord(ev[(i + 4) & 7], s0);
        } else {
          hipStream_t ps = (i & 1) ? s1 : s2;
          hipLaunchKernelGGL(k_small, dim3(32), dim3(256), 0, ps, a);
          hipEventRecord(ev[i & 7], ps);
          hipStreamWaitEvent(s0, ev[i & 7], 0);
          hipLaunchKernelGGL(k_small, dim3(512), dim3(256), 0, s0, a);
        }
      }
      auto t1 = std::chrono::steady_clock::now();
      CK(hipDeviceSynchronize());
      auto t2 = std::chrono::steady_clock::now();
      double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
      double all = std::chrono::duration<double, std::micro>(t2 - t0).count() / N;
      if (rep) printf("mode %d: host %.2f us/iter, host+drain %.2f us/iter\n", mode, host, all);
    }
  }
  return 0;
}
