// device_common.hpp — gfx950 device helpers shared by the engine kernels.
//
//  * CRC32C (Castagnoli, reflected 0x82F63B78): slicing-by-8 tables resident in LDS, and the GF(2)
//    combine crc(A||B) = (crc(A) * x^(8|B|) mod P) ^ crc(B) used to merge per-lane partial CRCs.
//  * In-launch inter-workgroup hand-off: 8-byte {tag, value} granules written and polled with
//    relaxed agent-scope atomics (global `sc1` accesses; MI355X guide §6 Guideline 16, form R2),
//    every spin bounded and reported through an error word.
//  * wave64 / 256-thread block scans built on __shfl_up and one LDS word per wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rmq {

typedef uint32_t u32;
typedef uint64_t u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) u32 gu32;

constexpr u32 kCrcPoly = 0x82F63B78u;
constexpr u32 kSpinLimit = 1u << 22;  // polls before a hand-off is declared dead (~seconds)
constexpr u32 kErrSpinTimeout = 1u;

// Device constants: CRC tables and GF(2) shift constants, filled by the host at engine creation.
struct CrcConsts {
  u32 table[8][256];   // slicing-by-8: table[k][b] = CRC register after byte b then k zero bytes
  u32 shift_pow2[32];  // shift_pow2[j] = x^(8 * 2^j) mod P (reflected): "append 2^j zero bytes"
};

__device__ __forceinline__ u32 lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// ---------------------------------------------------------------------------------------------
// CRC32C
// ---------------------------------------------------------------------------------------------

// a * b mod P in the reflected representation (x^0 = 0x80000000). Branch-free, 32 steps.
__device__ __forceinline__ u32 gf2_mulmod(u32 a, u32 b) {
  u32 p = 0;
#pragma unroll
  for (int k = 31; k >= 0; --k) {
    p ^= b & (0u - ((a >> k) & 1u));
    b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
  }
  return p;
}

// crc(A||B) from crc(A), crc(B) and K = x^(8|B|) mod P.
__device__ __forceinline__ u32 crc_combine(u32 crc_a, u32 crc_b, u32 k_shift) {
  return gf2_mulmod(k_shift, crc_a) ^ crc_b;
}

// CRC register update over 4 bytes held in a little-endian dword (slicing-by-4 on table[0..3]).
__device__ __forceinline__ u32 crc_step4(const u32 (*t)[256], u32 c, u32 w) {
  w ^= c;
  return t[3][w & 0xFF] ^ t[2][(w >> 8) & 0xFF] ^ t[1][(w >> 16) & 0xFF] ^ t[0][w >> 24];
}

// CRC register update over 8 bytes (lo, hi little-endian dwords), slicing-by-8.
__device__ __forceinline__ u32 crc_step8(const u32 (*t)[256], u32 c, u32 lo, u32 hi) {
  lo ^= c;
  return t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
         t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
}

__device__ __forceinline__ u32 crc_step1(const u32 (*t)[256], u32 c, u32 byte) {
  return (c >> 8) ^ t[0][(c ^ byte) & 0xFF];
}

// Finalized CRC32C of `len` bytes held in LDS starting at a 4-byte aligned dword pointer.
__device__ __forceinline__ u32 crc32c_lds(const u32 (*t)[256], const u32* w, u32 len) {
  u32 c = 0xFFFFFFFFu;
  u32 n8 = len >> 3;
  for (u32 k = 0; k < n8; ++k) c = crc_step8(t, c, w[2 * k], w[2 * k + 1]);
  u32 rem = len & 7u, d = 2 * n8;
  if (rem >= 4) {
    c = crc_step4(t, c, w[d]);
    ++d;
    rem -= 4;
  }
  if (rem) {
    u32 last = w[d];
    for (u32 b = 0; b < rem; ++b) c = crc_step1(t, c, (last >> (8 * b)) & 0xFF);
  }
  return ~c;
}

// ---------------------------------------------------------------------------------------------
// Granule hand-off (data is the flag): {tag:32 | value:32}
// ---------------------------------------------------------------------------------------------

__device__ __forceinline__ void gran_store(u64* g, u32 tag, u32 value) {
  __hip_atomic_store((gu64*)g, ((u64)tag << 32) | value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 gran_load(const u64* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_sc1_u64(u64* p, u64 v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 load_sc1_u64(const u64* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Poll one granule until its tag equals `tag`; returns the value. Bounded spin.
__device__ __forceinline__ u32 gran_wait(const u64* g, u32 tag, u32* err) {
  for (u32 spins = 0;; ++spins) {
    u64 x = gran_load(g);
    if ((u32)(x >> 32) == tag) return (u32)x;
    if (spins >= kSpinLimit) {
      atomicOr(err, kErrSpinTimeout);
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// ---------------------------------------------------------------------------------------------
// Scans (256-thread blocks = 4 waves)
// ---------------------------------------------------------------------------------------------

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const u32 l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T o = __shfl_up(v, d, 64);
    if (l >= (u32)d) v += o;
  }
  return v;
}

// Block-wide exclusive scan for a block of NW waves. `sh` needs NW entries. Returns the
// exclusive prefix; *total gets the block sum. Contains two __syncthreads().
template <u32 NW, typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T* total) {
  const u32 l = lane_id(), w = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (l == 63) sh[w] = inc;
  __syncthreads();
  T base = 0, tot = 0;
#pragma unroll
  for (u32 k = 0; k < NW; ++k) {
    T s = sh[k];
    if (k < w) base += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// Segmented inclusive scan step helpers: pairs (flag, value). A set flag starts a new segment.
template <typename T>
__device__ __forceinline__ void wave_seg_incl_scan(u32& flag, T& v) {
  const u32 l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    u32 of = __shfl_up(flag, d, 64);
    T ov = __shfl_up(v, d, 64);
    if (l >= (u32)d) {
      if (!flag) v += ov;
      flag |= of;
    }
  }
}

}  // namespace rmq
