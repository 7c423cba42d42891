// store_bench.hip — is the append kernel's ring-store phase bound by address translation?
// (diagnostic; not part of the engine)
//
// 1024 waves (256 workgroups x 4), each storing 29 chunks of 64 dwords = 64 records of 116 B, as
// the append kernel does for a config-B tile. Record k of wave w goes to partition hash(w, k) % P
// (skewed like Zipf: half of the records to 16 hot partitions), at that partition's ring tail.
// Layouts:
//   flat    : ring p at p * seg                    (engine ABI v1, FORMAT.md §2)
//   striped : 64 KiB block b of ring p at (b * P + p) * 64 KiB (concurrent tails share pages)
// Reported: mean kernel time over 20 launches (hipEvent), for RF = 1 and 3.
// Build: hipcc -O3 --offload-arch=gfx950 tools/store_bench.hip -o tools/store_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32;
typedef uint64_t u64;

__device__ __forceinline__ u32 hash32(u32 x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// mode 0: empty; 1: each wave's 7.4 KB tile contiguous at a random ring position; 2: scattered
// records (flat layout); 3: scattered 128-B aligned records (full lines)
__global__ __launch_bounds__(256) void mode_kernel(uint8_t* logs, u32 P, u64 seg, u32 RF, u32 iter, u32 mode) {
  const u32 lane = threadIdx.x & 63, wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 rstride = (u64)P * seg;
  if (mode == 0) return;
  for (u32 c = 0; c < 29; ++c) {
    const u32 dw = c * 64 + lane;
    const u32 k = dw / 29, rel = dw % 29;
    u64 a;
    if (mode == 1) {
      const u32 h = hash32(wv + iter * 7919u);
      a = (u64)(h % P) * seg + ((u64)(h >> 12) * 7424u) % (seg - 8192) / 4 * 4 + 4ull * dw;
    } else {
      const u32 h = hash32(wv * 64 + k + iter * 7919u);
      const u64 tail = ((u64)(h >> 8) * (mode == 3 ? 128u : 116u)) % (seg - 4096);
      a = (u64)(h % P) * seg + tail + 4ull * rel;
    }
    for (u32 r = 0; r < RF; ++r) *reinterpret_cast<u32*>(logs + r * rstride + a) = dw;
  }
}

template <bool kStriped>
__global__ __launch_bounds__(256) void store_kernel(uint8_t* logs, u32 P, u64 seg, u32 RF, u32 iter) {
  const u32 lane = threadIdx.x & 63, wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 rstride = (u64)P * seg;
  for (u32 c = 0; c < 29; ++c) {
    const u32 dw = c * 64 + lane;       // image dword
    const u32 k = dw / 29, rel = dw % 29;  // record, dword within record
    const u32 h = hash32(wv * 64 + k + iter * 7919u);
    const u32 p = (h & 1) ? (h >> 1) % 16u : (h >> 1) % P;
    // tail position: advances with the iteration; hot partitions deeper into their rings
    const u64 tail = ((u64)iter * 116u * ((h & 1) ? 256u : 4u) + (u64)(h % 1024u) * 116u) % (seg - 4096);
    const u64 off = tail + 4ull * rel;
    u64 a;
    if (kStriped) {
      const u64 B = 65536;
      a = ((off / B) * P + p) * B + (off % B);
    } else {
      a = (u64)p * seg + off;
    }
    for (u32 r = 0; r < RF; ++r) *reinterpret_cast<u32*>(logs + r * rstride + a) = dw;
  }
}

int main(int argc, char** argv) {
  const u32 P = argc > 1 ? atoi(argv[1]) : 4096;
  const u64 seg = (argc > 2 ? atoll(argv[2]) : 8) << 20;
  const u64 bytes = 3ull * P * seg;
  uint8_t* logs;
  if (hipMalloc(&logs, bytes) != hipSuccess) { printf("alloc %llu failed\n", (unsigned long long)bytes); return 1; }
  hipMemset(logs, 0, bytes);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int striped = 0; striped < 2; ++striped)
    for (u32 RF = 1; RF <= 3; RF += 2) {
      float tot = 0;
      for (u32 it = 0; it < 25; ++it) {
        hipEventRecord(e0);
        if (striped) store_kernel<true><<<256, 256>>>(logs, P, seg, RF, it);
        else store_kernel<false><<<256, 256>>>(logs, P, seg, RF, it);
        hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) { printf("kernel failed\n"); return 1; }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (it >= 5) tot += ms;
      }
      printf("P=%u seg=%lluMB footprint=%.1fGB %s RF=%u: %.2f us/launch\n", P, (unsigned long long)(seg >> 20),
             bytes / 1e9, striped ? "striped" : "flat   ", RF, tot / 20 * 1000);
    }
  const char* mn[] = {"empty", "contiguous tiles", "scattered 116B records", "scattered 128B-aligned"};
  for (u32 mode = 0; mode < 4; ++mode)
    for (u32 RF = 1; RF <= 3; RF += 2) {
      float tot = 0;
      for (u32 it = 0; it < 25; ++it) {
        hipEventRecord(e0);
        mode_kernel<<<256, 256>>>(logs, P, seg, RF, it, mode);
        hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) { printf("kernel failed\n"); return 1; }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (it >= 5) tot += ms;
      }
      printf("P=%u seg=%lluMB mode %-24s RF=%u: %.2f us/launch\n", P, (unsigned long long)(seg >> 20), mn[mode], RF,
             tot / 20 * 1000);
    }
  hipFree(logs);
  return 0;
}
