// ringstore_bench.hip — the append kernel's image -> replica-ring store phase in isolation
// (diagnostic; not part of the engine). 256 workgroups x 4 waves, one 64-record tile per wave
// (config B: 100-B payloads, 116-B records), RF replicas. Records of a tile are grouped into runs
// of the same partition (run lengths drawn like a Zipf-sorted tile), each run contiguous in its
// partition's ring at a random tail. Variants:
//   0  map-driven dword stores, 8 chunks per batch (append v4)
//   1  record-per-lane dword stores (lane = record, loop over the record's dwords)
//   2  record-per-lane dwordx4 stores (16-B pieces, tail handled with dword stores)
//   3  map-driven, but per-dword destination precomputed into LDS before the loop
//   4  16-B aligned records (payload padded to 16: 128-B records), map per 16-B piece, dwordx4
// Reported: kernel time (hipEvent, 200 back-to-back launches) and per-wave phase cycles.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ringstore_bench.hip -o tools/ringstore_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32;
typedef uint64_t u64;

constexpr u32 kImgDw = 2048;

__device__ __forceinline__ u32 hash32(u32 x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

struct WaveSmem {
  u32 img[kImgDw];
  uint8_t map[kImgDw];
  u64 ra[64];
  u32 km[64];
  u32 dsto[kImgDw];  // variant 3: per-dword ring offset (low 32 bits relative to the partition ring)
};

template <int V>
__global__ __launch_bounds__(256) void ring_kernel(uint8_t* logs, u32 P, u64 seg, u32 RF, u32 iter, u64* cyc) {
  __shared__ WaveSmem S[4];
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6, gw = blockIdx.x * 4 + wv;
  WaveSmem& W = S[wv];
  const u32 L = 100, rs = V == 4 ? 128 : 116;
  // runs: record k belongs to run id = hash-driven breakpoints (about 1 in 3 records starts a run)
  const u32 h = hash32(gw * 64 + lane + iter * 131u);
  u32 head = (lane == 0 || (h & 3u) == 0) ? 1u : 0u;
  // run index per lane = inclusive count of heads
  u32 run = 0;
  {
    u64 hm = __ballot(head);
    run = __popcll(hm & ((2ull << lane) - 1)) - 1;
  }
  const u32 key = hash32(gw * 977u + run * 31u + iter) % P;
  // rank within run
  u64 hm = __ballot(head);
  const u32 run_start = 63 - __clzll(hm & ((2ull << lane) - 1));
  const u32 rank = lane - run_start;
  const u64 tail = ((u64)hash32(key + iter * 7u) * 116u) % (seg - 65536) / 16 * 16;
  const u64 pos = tail + (u64)rank * rs;  // ring position of this record
  const u32 ioff = lane * rs;
  const u64 segmask = seg - 1;  // seg is a power of two
  const u64 rstride = (u64)P * seg;
  for (u32 d = 0; d < rs / 4; ++d) {
    W.map[ioff / 4 + d] = (uint8_t)lane;
    W.img[ioff / 4 + d] = d * 0x01010101u + lane;
  }
  W.ra[lane] = pos - ioff;
  W.km[lane] = key | (((1u << RF) - 1u) << 24);
  const u32 ndw = 64 * rs / 4;
  __syncthreads();
  u64 t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (V == 4) {
    const u32 npc = ndw / 4;  // 16-B pieces
    for (u32 c0 = 0; c0 * 64 < npc; c0 += 4) {
      u32 k[4], km[4];
      u64 ra[4];
      uint4 v[4];
#pragma unroll
      for (u32 j = 0; j < 4; ++j) k[j] = W.map[((c0 + j) * 64 + lane) * 4 & (kImgDw - 1)];
#pragma unroll
      for (u32 j = 0; j < 4; ++j) {
        v[j] = *reinterpret_cast<const uint4*>(&W.img[(((c0 + j) * 64 + lane) * 4) & (kImgDw - 1)]);
        ra[j] = W.ra[k[j] & 63u];
        km[j] = W.km[k[j] & 63u];
      }
#pragma unroll
      for (u32 j = 0; j < 4; ++j) {
        const u32 q = (c0 + j) * 64 + lane;
        const u32 msk = q < npc ? km[j] >> 24 : 0u;
        if (msk) {
          const u64 lp = (ra[j] + 16ull * q) & segmask;
          uint8_t* dst = logs + (u64)(km[j] & 0xFFFFFFu) * seg + lp;
          for (u32 r = 0; r < RF; ++r)
            if (msk >> r & 1u) *reinterpret_cast<uint4*>(dst + r * rstride) = v[j];
        }
      }
    }
  } else if (V == 0 || V == 3) {
    if (V == 3) {
      for (u32 d = 0; d < rs / 4; ++d) W.dsto[ioff / 4 + d] = (u32)((pos + 4 * d) & segmask);
      __builtin_amdgcn_wave_barrier();
    }
    const u32 nchunks = (ndw + 63u) >> 6;
    for (u32 c0 = 0; c0 < nchunks; c0 += 8) {
      u32 k[8], v[8], km[8];
      u64 ra[8];
#pragma unroll
      for (u32 j = 0; j < 8; ++j) k[j] = W.map[(c0 + j) * 64 + lane];
#pragma unroll
      for (u32 j = 0; j < 8; ++j) {
        v[j] = W.img[(c0 + j) * 64 + lane];
        ra[j] = V == 3 ? (u64)W.dsto[(c0 + j) * 64 + lane] : W.ra[k[j] & 63u];
        km[j] = W.km[k[j] & 63u];
      }
#pragma unroll
      for (u32 j = 0; j < 8; ++j) {
        const u32 dw = (c0 + j) * 64 + lane;
        const u32 msk = dw < ndw ? km[j] >> 24 : 0u;
        if (msk) {
          const u64 lp = V == 3 ? ra[j] : ((ra[j] + 4ull * dw) & segmask);
          uint8_t* dst = logs + (u64)(km[j] & 0xFFFFFFu) * seg + lp;
          for (u32 r = 0; r < RF; ++r)
            if (msk >> r & 1u) *reinterpret_cast<u32*>(dst + r * rstride) = v[j];
        }
      }
    }
  } else if (V == 1) {
    uint8_t* base = logs + (u64)key * seg;
    for (u32 d = 0; d < rs / 4; ++d) {
      const u32 v = W.img[ioff / 4 + d];
      const u64 lp = (pos + 4 * d) & segmask;
      for (u32 r = 0; r < RF; ++r) *reinterpret_cast<u32*>(base + r * rstride + lp) = v;
    }
  } else {
    uint8_t* base = logs + (u64)key * seg;
    for (u32 q = 0; q < rs / 16; ++q) {
      uint4 v;
      v.x = W.img[ioff / 4 + 4 * q];
      v.y = W.img[ioff / 4 + 4 * q + 1];
      v.z = W.img[ioff / 4 + 4 * q + 2];
      v.w = W.img[ioff / 4 + 4 * q + 3];
      const u64 lp = (pos + 16 * q) & segmask;  // no wrap inside a piece in this bench
      for (u32 r = 0; r < RF; ++r) *reinterpret_cast<uint4*>(base + r * rstride + lp) = v;
    }
    for (u32 d = (rs / 16) * 4; d < rs / 4; ++d) {
      const u32 v = W.img[ioff / 4 + d];
      const u64 lp = (pos + 4 * d) & segmask;
      for (u32 r = 0; r < RF; ++r) *reinterpret_cast<u32*>(base + r * rstride + lp) = v;
    }
  }
  u64 t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (lane == 0) cyc[gw] = t1 - t0;
}

int main(int argc, char** argv) {
  const u32 P = argc > 1 ? atoi(argv[1]) : 4096;
  const u64 seg = (argc > 2 ? atoll(argv[2]) : 8) << 20;
  const u64 bytes = 3ull * P * seg;
  uint8_t* logs;
  if (hipMalloc(&logs, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(logs, 0, bytes);
  u64* cyc;
  hipMalloc(&cyc, 1024 * 8);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"map dword (v4)", "lane-record dword", "lane-record dwordx4", "map + precomputed dst",
                         "map dwordx4, 128-B recs"};
  for (int v = 0; v < 5; ++v)
    for (u32 RF = 1; RF <= 3; RF += 2) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        for (u32 it = 0; it < 200; ++it) {
          switch (v) {
            case 0: ring_kernel<0><<<256, 256>>>(logs, P, seg, RF, it, cyc); break;
            case 1: ring_kernel<1><<<256, 256>>>(logs, P, seg, RF, it, cyc); break;
            case 2: ring_kernel<2><<<256, 256>>>(logs, P, seg, RF, it, cyc); break;
            case 3: ring_kernel<3><<<256, 256>>>(logs, P, seg, RF, it, cyc); break;
            case 4: ring_kernel<4><<<256, 256>>>(logs, P, seg, RF, it, cyc); break;
          }
        }
        hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) { printf("kernel failed\n"); return 1; }
      }
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      u64 h[1024];
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double m = 0;
      for (u64 c : h) m += (double)c;
      printf("%-24s RF=%u: %.2f us/launch, store phase %.0f cycles/wave (mean)\n", names[v], RF, ms * 1000 / 200,
             m / 1024);
    }
  // empty-ish reference: launch cost
  return 0;
}
