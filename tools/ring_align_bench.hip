// ring_align_bench.hip — what the ring-store pattern of pipeline stage 3 costs, by record alignment
// and processing order (diagnostic; not part of the engine). One launch = 65536 records x 128 B x 3
// replicas (config B's ring-store volume, 25.2 MB), 8 lanes per record, one 16-B store per lane
// per replica. Records go to 4096 partition rings (1 MiB each) with Zipf(1.1) load; every ring
// starts at a random phase of the record alignment (16, 64 or 128 B; 0 = one contiguous stream).
// Order: "input" = Zipf-random record order (today's stage 3), "sorted" = partition-major inside
// 1024-record tiles (consecutive records of a run are adjacent in the ring).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ring_align_bench tools/ring_align_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);      \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ __launch_bounds__(256) void ring_store(const uint2* __restrict__ rec, unsigned n, unsigned char* logs,
                                                  unsigned long long seg, unsigned long long rstride, int nt) {
  const unsigned g = blockIdx.x * 256u + threadIdx.x;
  const unsigned r = g >> 3, k = g & 7u;
  if (r >= n) return;
  const uint2 d = rec[r];  // {ring, byte position of the record in the ring}
  unsigned char* dst = logs + (unsigned long long)d.x * seg + ((d.y + 16ull * k) & (seg - 1));
  const u32x4 v = {g, r, k, 0x5A5A5A5Au};
  for (int q = 0; q < 3; ++q) {
    u32x4* a = reinterpret_cast<u32x4*>(dst + q * rstride);
    if (nt)
      __builtin_nontemporal_store(v, a);
    else
      *a = v;
  }
}

int main() {
  const unsigned P = 4096, N = 65536, T = 1024, NB = 16, ITER = 400;
  const unsigned long long seg = 1ull << 20, rstride = (unsigned long long)P * seg;
  unsigned char* logs = nullptr;
  CK(hipMalloc(&logs, 3 * rstride));
  CK(hipMemset(logs, 0, 3 * rstride));
  uint2* d_rec = nullptr;
  CK(hipMalloc(&d_rec, (size_t)NB * N * sizeof(uint2)));
  std::vector<double> w(P);
  for (unsigned k = 0; k < P; ++k) w[k] = std::pow(k + 1.0, -1.1);
  std::mt19937_64 rng(0x52495050);
  std::discrete_distribution<unsigned> zipf(w.begin(), w.end());
  std::vector<unsigned> perm(P);
  std::iota(perm.begin(), perm.end(), 0u);
  std::shuffle(perm.begin(), perm.end(), rng);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("%-6s %-7s %-3s %10s %8s\n", "align", "order", "nt", "us/launch", "TB/s");
  for (unsigned align : {0u, 16u, 64u, 128u})
    for (int sorted = 0; sorted < 2; ++sorted) {
      if (align == 0 && sorted) continue;
      std::vector<unsigned long long> cur(P);
      for (unsigned p = 0; p < P; ++p) cur[p] = align ? align * (rng() % (128 / align)) : 0;
      std::vector<uint2> h((size_t)NB * N);
      for (unsigned b = 0; b < NB; ++b) {
        if (align == 0) {  // reference: one contiguous stream over the rings
          for (unsigned s = 0; s < N; ++s) {
            const unsigned long long pos = ((unsigned long long)b * N + s) * 128;
            h[(size_t)b * N + s] = make_uint2((unsigned)(pos / seg) % P, (unsigned)(pos % seg));
          }
          continue;
        }
        std::vector<unsigned> ps(N), idx(N);
        for (unsigned i = 0; i < N; ++i) ps[i] = perm[zipf(rng)];
        std::iota(idx.begin(), idx.end(), 0u);
        for (unsigned t = 0; t < N; t += T)  // log order: partition-major inside each tile
          std::stable_sort(idx.begin() + t, idx.begin() + t + T, [&](unsigned a, unsigned c) { return ps[a] < ps[c]; });
        std::vector<uint2> byin(N);
        for (unsigned s = 0; s < N; ++s) {
          const unsigned i = idx[s], p = ps[i];
          byin[i] = make_uint2(p, (unsigned)(cur[p] & (seg - 1)));
          cur[p] += 128;
        }
        for (unsigned s = 0; s < N; ++s) h[(size_t)b * N + s] = sorted ? byin[idx[s]] : byin[s];
      }
      CK(hipMemcpy(d_rec, h.data(), h.size() * sizeof(uint2), hipMemcpyHostToDevice));
      for (int nt = 0; nt < 2; ++nt) {
        for (unsigned it = 0; it < 50; ++it)
          hipLaunchKernelGGL(ring_store, dim3(N * 8 / 256), dim3(256), 0, 0, d_rec + (size_t)(it % NB) * N, N, logs, seg, rstride, nt);
        CK(hipEventRecord(e0));
        for (unsigned it = 0; it < ITER; ++it)
          hipLaunchKernelGGL(ring_store, dim3(N * 8 / 256), dim3(256), 0, 0, d_rec + (size_t)(it % NB) * N, N, logs, seg, rstride, nt);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / ITER;
        std::printf("%-6u %-7s %-3d %10.2f %8.2f\n", align, align ? (sorted ? "sorted" : "input") : "stream", nt, us,
                    3.0 * N * 128 / us / 1e6);
      }
    }
  CK(hipFree(logs));
  CK(hipFree(d_rec));
  return 0;
}
