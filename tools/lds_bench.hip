// lds_bench.hip — microbenchmark of the append kernel's LDS-bound pieces on gfx950 (diagnostic;
// not part of the engine). One workgroup of 256 threads per CU (one wave per SIMD, as the append
// kernel runs), every wave holding a 64-record image of 100-byte payloads in LDS.
//   lat   : dependent ds_read_b32 chain, cycles per hop
//   crc0  : slicing-by-8, payload dwords read from LDS inside the chain (append v3)
//   crc1  : payload dwords preloaded into registers, table lookups only in the chain
//   crc2  : two interleaved chains (front / back half) merged by one GF(2) multiply
//   crc4  : four interleaved chains merged by three multiplies
// Build: hipcc -O3 --offload-arch=gfx950 tools/lds_bench.hip -o /tmp/lds_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;
constexpr u32 kPoly = 0x82F63B78u;
constexpr u32 kLen = 100;              // payload bytes per record
constexpr u32 kStride = 116;           // record bytes in the image (16 + align4(100))
constexpr u32 kImgDw = 64 * kStride / 4;

__device__ __forceinline__ u32 mulmod(u32 a, u32 b) {
  u32 p = 0;
#pragma unroll
  for (int k = 31; k >= 0; --k) {
    p ^= b & (0u - ((a >> k) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return p;
}

__device__ __forceinline__ u32 step8(const u32 (*t)[256], u32 c, u32 lo, u32 hi) {
  lo ^= c;
  return t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
         t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
}
__device__ __forceinline__ u32 step4(const u32 (*t)[256], u32 c, u32 w) {
  w ^= c;
  return t[3][w & 0xFF] ^ t[2][(w >> 8) & 0xFF] ^ t[1][(w >> 16) & 0xFF] ^ t[0][w >> 24];
}

struct Smem {
  u32 tab[8][256];
  u32 pow8[1024];  // x^(8n) mod P, n bytes of zeros
  u32 img[4][kImgDw];
};

template <int V>
__global__ __launch_bounds__(256) void bench_kernel(const u32* tables, const u32* pow8, const u32* data,
                                                    u32* out, u64* cycles, int iters) {
  __shared__ Smem S;
  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (u32 k = tid; k < 2048; k += 256) (&S.tab[0][0])[k] = tables[k];
  for (u32 k = tid; k < 1024; k += 256) S.pow8[k] = pow8[k];
  for (u32 k = lane; k < kImgDw; k += 64) S.img[w][k] = data[(blockIdx.x * 4 + w) * kImgDw + k];
  __syncthreads();
  const u32* rec = &S.img[w][lane * kStride / 4 + 4];
  u32 acc = 0;
  u64 t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
    if (V == 0) {  // pointer chase: next index from the previous load
      u32 idx = (lane * 37u + acc) & 2047u;
#pragma unroll 1
      for (int h = 0; h < 256; ++h) idx = (&S.tab[0][0])[idx] & 2047u;
      acc += idx;
    } else if (V == 1) {  // crc0: payload from LDS in the chain
      u32 c = 0xFFFFFFFFu ^ acc;
#pragma unroll 1
      for (u32 k = 0; k < kLen / 8; ++k) c = step8(S.tab, c, rec[2 * k], rec[2 * k + 1]);
      c = step4(S.tab, c, rec[kLen / 4 - 1]);
      acc = ~c;
    } else if (V == 2) {  // crc1: payload preloaded
      u32 d[kLen / 4];
#pragma unroll
      for (u32 k = 0; k < kLen / 4; ++k) d[k] = rec[k];
      u32 c = 0xFFFFFFFFu ^ acc;
#pragma unroll
      for (u32 k = 0; k < kLen / 8; ++k) c = step8(S.tab, c, d[2 * k], d[2 * k + 1]);
      c = step4(S.tab, c, d[kLen / 4 - 1]);
      acc = ~c;
    } else if (V == 3) {  // crc2: two chains, halves of 48 / 52 bytes
      u32 d[kLen / 4];
#pragma unroll
      for (u32 k = 0; k < kLen / 4; ++k) d[k] = rec[k];
      u32 ca = 0xFFFFFFFFu ^ acc, cb = 0;
#pragma unroll
      for (u32 k = 0; k < 6; ++k) {
        ca = step8(S.tab, ca, d[2 * k], d[2 * k + 1]);
        cb = step8(S.tab, cb, d[12 + 2 * k], d[12 + 2 * k + 1]);
      }
      cb = step4(S.tab, cb, d[24]);
      acc = ~(mulmod(S.pow8[52], ca) ^ cb);
    } else if (V == 4) {  // crc4: four chains of 24 / 24 / 24 / 28 bytes
      u32 d[kLen / 4];
#pragma unroll
      for (u32 k = 0; k < kLen / 4; ++k) d[k] = rec[k];
      u32 c0 = 0xFFFFFFFFu ^ acc, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
      for (u32 k = 0; k < 3; ++k) {
        c0 = step8(S.tab, c0, d[2 * k], d[2 * k + 1]);
        c1 = step8(S.tab, c1, d[6 + 2 * k], d[6 + 2 * k + 1]);
        c2 = step8(S.tab, c2, d[12 + 2 * k], d[12 + 2 * k + 1]);
        c3 = step8(S.tab, c3, d[18 + 2 * k], d[18 + 2 * k + 1]);
      }
      c3 = step4(S.tab, c3, d[24]);
      acc = ~(mulmod(S.pow8[76], c0) ^ mulmod(S.pow8[52], c1) ^ mulmod(S.pow8[28], c2) ^ c3);
    }
  }
  u64 t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 256 + tid] = acc;
  if (lane == 0) cycles[blockIdx.x * 4 + w] = t1 - t0;
}

static u32 crc_bitwise(const uint8_t* p, u32 n) {
  u32 c = 0xFFFFFFFFu;
  for (u32 i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
  }
  return ~c;
}

int main(int argc, char** argv) {
  int blocks = argc > 1 ? atoi(argv[1]) : 256;
  const int iters = 16;
  std::vector<u32> tab(2048), pw(1024);
  for (u32 b = 0; b < 256; ++b) {
    u32 c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
    tab[b] = c;
  }
  for (u32 t = 1; t < 8; ++t)
    for (u32 b = 0; b < 256; ++b) tab[t * 256 + b] = (tab[(t - 1) * 256 + b] >> 8) ^ tab[tab[(t - 1) * 256 + b] & 0xFF];
  // pow8[n] = x^(8n) mod P reflected: the register 0x80000000 (= x^0) after n zero bytes
  for (u32 n = 0; n < 1024; ++n) {
    u32 c = 0x80000000u;
    for (u32 i = 0; i < 8 * n; ++i) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
    pw[n] = c;
  }
  const size_t ndata = (size_t)blocks * 4 * kImgDw;
  std::vector<u32> data(ndata);
  u64 x = 88172645463325252ull;
  for (auto& v : data) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    v = (u32)x;
  }
  u32 *dt, *dp, *dd, *dout;
  u64* dcy;
  hipMalloc(&dt, 2048 * 4);
  hipMalloc(&dp, 1024 * 4);
  hipMalloc(&dd, ndata * 4);
  hipMalloc(&dout, (size_t)blocks * 256 * 4);
  hipMalloc(&dcy, (size_t)blocks * 4 * 8);
  hipMemcpy(dt, tab.data(), 2048 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dp, pw.data(), 1024 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dd, data.data(), ndata * 4, hipMemcpyHostToDevice);
  const char* names[] = {"lat(256 hops)", "crc0 lds-payload", "crc1 reg-payload", "crc2 two-chain", "crc4 four-chain"};
  std::vector<u32> out((size_t)blocks * 256);
  std::vector<u64> cy((size_t)blocks * 4);
  for (int v = 0; v < 5; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (v) {
        case 0: bench_kernel<0><<<blocks, 256>>>(dt, dp, dd, dout, dcy, iters); break;
        case 1: bench_kernel<1><<<blocks, 256>>>(dt, dp, dd, dout, dcy, iters); break;
        case 2: bench_kernel<2><<<blocks, 256>>>(dt, dp, dd, dout, dcy, iters); break;
        case 3: bench_kernel<3><<<blocks, 256>>>(dt, dp, dd, dout, dcy, iters); break;
        case 4: bench_kernel<4><<<blocks, 256>>>(dt, dp, dd, dout, dcy, iters); break;
      }
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    }
    hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(cy.data(), dcy, cy.size() * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (u64 c : cy) m += (double)c;
    m /= cy.size();
    // check crc variants: iteration chaining makes acc depend on earlier results; recompute on host
    int bad = 0;
    if (v >= 1) {
      for (int b = 0; b < blocks && b < 8; ++b)
        for (u32 t = 0; t < 256; ++t) {
          const u32 w = t >> 6, lane = t & 63;
          const uint8_t* rec = reinterpret_cast<const uint8_t*>(&data[((size_t)b * 4 + w) * kImgDw + lane * kStride / 4 + 4]);
          u32 acc = 0;
          for (int it = 0; it < iters; ++it) {
            // device computes crc with initial register 0xFFFFFFFF ^ acc
            u32 c = 0xFFFFFFFFu ^ acc;
            for (u32 i = 0; i < kLen; ++i) {
              c ^= rec[i];
              for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
            }
            acc = ~c;
          }
          bad += acc != out[(size_t)b * 256 + t];
        }
    }
    printf("%-18s blocks=%d  cycles/iter per wave: %.0f  (%.0f per hop/step)  mismatches=%d\n", names[v], blocks,
           m / iters, v == 0 ? m / iters / 256 : m / iters / 13, bad);
  }
  (void)crc_bitwise;
  return 0;
}
