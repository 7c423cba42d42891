// replica_bench.hip — store rate of RF replica copies by the spacing of the replica rings
// (diagnostic; not part of the engine). Config D's shape: 16384 records of 4 KB per launch, a wave
// per record (16-byte pieces, four per lane), each record to RF = 5 replica rings of one of 4096
// partitions (256 KiB rings, records appended in turn); replica r of a ring lies at
// base + r * rstride. rstride = the pool (a multiple of 2 MiB, as the engine lays it out) or the
// pool plus a stagger, which moves the replicas' copies of one offset onto other HBM channels.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/replica_bench tools/replica_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
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

constexpr unsigned kRec = 4096;        // record bytes
constexpr unsigned kN = 16384;         // records per launch
constexpr unsigned kP = 4096;          // partitions
constexpr unsigned long long kSeg = 256 << 10;  // ring bytes

// mode bit 0: a CRC-like fold of every piece through 16 LDS table lookups (slicing tables, 8 KB);
// the dynamic LDS size of the launch sets the residency (39 KB: four workgroups per CU, as the
// pipeline kernel); waves take records w, w + waves, ... (records per wave = n / waves)
__global__ __launch_bounds__(256) void replicate(const u32x4* __restrict__ src, const unsigned long long* __restrict__ dpos,
                                                 unsigned char* logs, unsigned long long rstride, int rf, unsigned n,
                                                 int mode, unsigned* sink) {
  extern __shared__ unsigned t8[];
  const unsigned lane = threadIdx.x & 63u, waves = gridDim.x * 4u;
  for (unsigned k = threadIdx.x; k < 2048; k += 256) t8[k] = k * 2654435761u;
  __syncthreads();
  unsigned acc = 0;
  for (unsigned w = (blockIdx.x * 256u + threadIdx.x) >> 6; w < n; w += waves) {
    const u32x4* s = src + (unsigned long long)w * (kRec / 16);
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = s[64 * u + lane];
    unsigned char* d = logs + dpos[w];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (mode & 1) {
        const unsigned x = v[u].x ^ acc, y = v[u].y, z = v[u].z, q = v[u].w;
        acc = t8[x & 255] ^ t8[256 + ((x >> 8) & 255)] ^ t8[512 + ((x >> 16) & 255)] ^ t8[768 + (x >> 24)] ^
              t8[1024 + (y & 255)] ^ t8[1280 + ((y >> 8) & 255)] ^ t8[1536 + ((y >> 16) & 255)] ^ t8[1792 + (y >> 24)] ^
              t8[z & 255] ^ t8[256 + ((z >> 8) & 255)] ^ t8[512 + ((z >> 16) & 255)] ^ t8[768 + (z >> 24)] ^
              t8[1024 + (q & 255)] ^ t8[1280 + ((q >> 8) & 255)] ^ t8[1536 + ((q >> 16) & 255)] ^ t8[1792 + (q >> 24)];
      }
      for (int r = 0; r < rf; ++r) {
        u32x4* a = reinterpret_cast<u32x4*>(d + r * rstride + 16ull * (64 * u + lane));
        if (mode & 4)
          *a = v[u];
        else
          __builtin_nontemporal_store(v[u], a);
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const int rf = 5;
  const unsigned long long pool = (unsigned long long)kP * kSeg;  // 1 GiB per replica
  std::vector<unsigned long long> staggers = {0};
  unsigned* sink = nullptr;
  CK(hipMalloc(&sink, 64));
  unsigned char* logs = nullptr;
  CK(hipMalloc(&logs, rf * (pool + (4ull << 20)) + (64ull << 20)));
  u32x4* src = nullptr;
  CK(hipMalloc(&src, (size_t)kN * kRec));
  CK(hipMemset(src, 1, (size_t)kN * kRec));
  unsigned long long* dpos = nullptr;
  CK(hipMalloc(&dpos, kN * 8ull));
  std::mt19937_64 g(7);
  std::vector<unsigned long long> used(kP, 0), h(kN);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // mode bit 1 (host): record starts at a 16-byte phase inside a 128-byte line (records of
  // 4096 + 16 bytes in the ring, as FORMAT.md lays them: a 16-byte header, payload padded to 16);
  // bit 2: plain stores instead of non-temporal ones
  struct Mode { int crc; unsigned lds, blocks; const char* name; };
  const Mode modes[] = {{0, 8192, kN / 4, "NT stores, 128-B aligned records"},
                        {2, 8192, kN / 4, "NT stores, records at 16-B phases"},
                        {4, 8192, kN / 4, "plain stores, 128-B aligned records"},
                        {6, 8192, kN / 4, "plain stores, records at 16-B phases"},
                        {7, 39 << 10, 2048, "plain, 16-B phases, CRC lookups, 2048 WGs looping"}};
  for (const Mode& md : modes)
  for (unsigned long long st : staggers) {
    const unsigned long long rstride = pool + st;
    float best = 1e9f;
    for (int it = 0; it < 20; ++it) {
      for (unsigned k = 0; k < kN; ++k) {  // uniform partitions, appended in turn (ring wraps)
        const unsigned p = (unsigned)(g() % kP);
        h[k] = (unsigned long long)p * kSeg + (used[p] % kSeg);
        used[p] += kRec + ((md.crc & 2) ? 16u : 0u);
      }
      CK(hipMemcpy(dpos, h.data(), kN * 8ull, hipMemcpyHostToDevice));
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(replicate, dim3(md.blocks), dim3(256), md.lds, 0, src, dpos, logs, rstride, rf, kN, md.crc, sink);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (it >= 3 && ms < best) best = ms;
    }
    const double wr = (double)kN * kRec * rf, rd = (double)kN * kRec;
    std::printf("%-50s: %.1f us, writes %.2f TB/s, reads+writes %.2f TB/s\n", md.name, best * 1e3,
                wr / best / 1e9, (wr + rd) / best / 1e9);
  }
  return 0;
}
