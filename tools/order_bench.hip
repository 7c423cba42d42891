// order_bench.hip — ring-store rate of one launch group's records (4 x 65536 records of 128 B,
// 3 replicas = 100.7 MB) by the ORDER stage 3 visits them (diagnostic; not part of the engine).
// Records go to 4096 partition rings (16 MiB each) with Zipf(1.1) load, 128-B aligned.
//   input  — input order (today's stage 3: 32 consecutive records per wave, random rings)
//   tile   — partition-major inside 1024-record tiles
//   group  — partition-major over the whole group: each partition's records of the group are one
//            contiguous run of its ring (what a destination-ordered apply would store)
//   stream — one contiguous stream (upper bound)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/order_bench tools/order_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

// 8 lanes per 128-B record, one 16-B store per lane per replica
__global__ __launch_bounds__(256) void ring_store(const uint2* __restrict__ rec, unsigned n, unsigned char* logs,
                                                  unsigned long long seg, unsigned long long rstride, int nt) {
  const unsigned g = blockIdx.x * 256u + threadIdx.x;
  const unsigned r = g >> 3, k = g & 7u;
  if (r >= n) return;
  const uint2 d = rec[r];
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

// the same stores plus a 128-B read per record from a separate random payload position (the
// gather a destination-ordered apply does), to see what scattered reads cost beside the stores
__global__ __launch_bounds__(256) void ring_copy(const uint2* __restrict__ rec, const unsigned* __restrict__ src,
                                                 const unsigned char* __restrict__ pay, unsigned n, unsigned char* logs,
                                                 unsigned long long seg, unsigned long long rstride) {
  const unsigned g = blockIdx.x * 256u + threadIdx.x;
  const unsigned r = g >> 3, k = g & 7u;
  if (r >= n) return;
  const uint2 d = rec[r];
  const u32x4 v = *reinterpret_cast<const u32x4*>(pay + 100ull * src[r] + 16ull * k - (100ull * src[r] & 15ull));
  unsigned char* dst = logs + (unsigned long long)d.x * seg + ((d.y + 16ull * k) & (seg - 1));
  for (int q = 0; q < 3; ++q) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + q * rstride));
}

int main() {
  const unsigned P = 4096, N = 4 * 65536, T = 1024, NB = 8, ITER = 200;
  const unsigned long long seg = 1ull << 24, rstride = (unsigned long long)P * seg;
  unsigned char* logs = nullptr;
  CK(hipMalloc(&logs, 3 * rstride));
  CK(hipMemset(logs, 0, 3 * rstride));
  uint2* d_rec = nullptr;
  unsigned* d_src = nullptr;
  unsigned char* d_pay = nullptr;
  CK(hipMalloc(&d_rec, (size_t)NB * N * sizeof(uint2)));
  CK(hipMalloc(&d_src, (size_t)NB * N * sizeof(unsigned)));
  CK(hipMalloc(&d_pay, (size_t)NB * N * 100 + 4096));
  CK(hipMemset(d_pay, 1, (size_t)NB * N * 100 + 4096));
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
  std::printf("%-7s %-5s %10s %8s\n", "order", "kind", "us/launch", "TB/s");
  const char* names[] = {"input", "tile", "group", "stream"};
  for (int order = 0; order < 4; ++order) {
    std::vector<unsigned long long> cur(P, 0);
    std::vector<uint2> h((size_t)NB * N);
    std::vector<unsigned> hs((size_t)NB * N);
    for (unsigned b = 0; b < NB; ++b) {
      std::vector<unsigned> ps(N), idx(N);
      for (unsigned i = 0; i < N; ++i) ps[i] = perm[zipf(rng)];
      std::iota(idx.begin(), idx.end(), 0u);
      // log order = partition-major over the group (stable): slots of each partition consecutive
      std::stable_sort(idx.begin(), idx.end(), [&](unsigned a, unsigned c) { return ps[a] < ps[c]; });
      std::vector<uint2> byin(N);
      for (unsigned s = 0; s < N; ++s) {
        const unsigned i = idx[s], p = ps[i];
        byin[i] = make_uint2(p, (unsigned)(cur[p] & (seg - 1)));
        cur[p] += 128;
      }
      std::vector<unsigned> vis(N);  // visiting order: vis[k] = input record visited k-th
      if (order == 0) std::iota(vis.begin(), vis.end(), 0u);
      if (order == 1) {
        std::iota(vis.begin(), vis.end(), 0u);
        for (unsigned t = 0; t < N; t += T)
          std::stable_sort(vis.begin() + t, vis.begin() + t + T, [&](unsigned a, unsigned c) { return ps[a] < ps[c]; });
      }
      if (order == 2) vis = idx;
      for (unsigned k = 0; k < N; ++k) {
        if (order == 3) {
          const unsigned long long pos = ((unsigned long long)b * N + k) * 128;
          h[(size_t)b * N + k] = make_uint2((unsigned)(pos / seg) % P, (unsigned)(pos % seg));
          hs[(size_t)b * N + k] = b * N + k;
        } else {
          h[(size_t)b * N + k] = byin[vis[k]];
          hs[(size_t)b * N + k] = b * N + vis[k];
        }
      }
    }
    CK(hipMemcpy(d_rec, h.data(), h.size() * sizeof(uint2), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_src, hs.data(), hs.size() * sizeof(unsigned), hipMemcpyHostToDevice));
    for (int kind = 0; kind < 3; ++kind) {
      auto launch = [&](unsigned it) {
        if (kind < 2)
          hipLaunchKernelGGL(ring_store, dim3(N * 8 / 256), dim3(256), 0, 0, d_rec + (size_t)(it % NB) * N, N, logs, seg,
                             rstride, kind);
        else
          hipLaunchKernelGGL(ring_copy, dim3(N * 8 / 256), dim3(256), 0, 0, d_rec + (size_t)(it % NB) * N,
                             d_src + (size_t)(it % NB) * N, d_pay, N, logs, seg, rstride);
      };
      for (unsigned it = 0; it < 20; ++it) launch(it);
      CK(hipEventRecord(e0));
      for (unsigned it = 0; it < ITER; ++it) launch(it);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / ITER;
      const char* kn[] = {"st", "st-nt", "copy"};
      const double bytes = 3.0 * N * 128 + (kind == 2 ? N * 128.0 : 0.0);
      std::printf("%-7s %-5s %10.2f %8.2f\n", names[order], kn[kind], us, bytes / us / 1e6);
    }
  }
  CK(hipFree(logs));
  CK(hipFree(d_rec));
  CK(hipFree(d_src));
  CK(hipFree(d_pay));
  return 0;
}
