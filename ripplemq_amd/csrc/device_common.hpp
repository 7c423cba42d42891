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
constexpr u32 kRecAlign = 16;         // FORMAT.md §1: records padded to 16 bytes
constexpr u32 kCrcPow8 = 520;         // pow8[n] = x^(8n) mod P for n < kCrcPow8 (4-chain CRC merge)

// Device constants: CRC tables and GF(2) shift constants, filled by the host at engine creation.
struct CrcConsts {
  u32 table[8][256];   // slicing-by-8: table[k][b] = CRC register after byte b then k zero bytes
  u32 zshift[3][4][256];  // zshift[k][i][b] = (b << 8i) * x^(8 * 16 * 2^k): register shift past 16<<k zero bytes
  u32 shift_pow2[32];  // shift_pow2[j] = x^(8 * 2^j) mod P (reflected): "append 2^j zero bytes"
  u32 inv_pad[16];     // inv_pad[n] = x^(-8n) mod P: "remove n trailing zero bytes"
  u32 pow8[kCrcPow8];  // pow8[n] = x^(8n) mod P: "append n zero bytes"
};

// FORMAT.md §1 record size: 16-byte header + payload padded to kRecAlign.
__host__ __device__ __forceinline__ constexpr u32 record_bytes(u32 len) {
  return 16u + ((len + kRecAlign - 1u) & ~(kRecAlign - 1u));
}

typedef u32 u32x4 __attribute__((ext_vector_type(4)));

// 16-byte log store. RMQ_RING_NT=1: non-temporal (streams past L2, nothing left dirty for the
// end-of-kernel writeback); 0: default policy.
#ifndef RMQ_RING_NT
#define RMQ_RING_NT 1
#endif
__device__ __forceinline__ void store_log16(uint8_t* dst, uint4 v) {
#if RMQ_RING_NT
  const u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(dst));
#else
  *reinterpret_cast<uint4*>(dst) = v;
#endif
}

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

// Register shift past 16 << k zero bytes (k = 0, 1, 2) by a 4 x 256 table (linearity in the register).
__device__ __forceinline__ u32 crc_zshift(const u32 (*z)[256], u32 c) {
  return z[0][c & 0xFF] ^ z[1][(c >> 8) & 0xFF] ^ z[2][(c >> 16) & 0xFF] ^ z[3][c >> 24];
}

__device__ __forceinline__ u32 crc_step1(const u32 (*t)[256], u32 c, u32 byte) {
  return (c >> 8) ^ t[0][(c ^ byte) & 0xFF];
}

// CRC register after k in [0, 8] more bytes (lo = bytes 0..3, hi = bytes 4..7; bytes >= k
// ignored): c' = (c >> 8k) ^ XOR_{i<k} table[k-1-i][byte i of (c ^ data)], one round of lookups.
__device__ __forceinline__ u32 crc_stepn(const u32 (*t)[256], u32 c, u32 lo, u32 hi, u32 k) {
  const u32 x = lo ^ c;
  u32 r = k == 0 ? c : (k < 4 ? c >> (8 * k) : 0u);
#pragma unroll
  for (u32 i = 0; i < 8; ++i) {
    const u32 b = i < 4 ? (x >> (8 * i)) & 0xFF : (hi >> (8 * (i - 4))) & 0xFF;
    const u32 v = t[(k - 1 - i) & 7][b];
    r ^= i < k ? v : 0u;
  }
  return r;
}

// Finalized CRC32C of `len` bytes in LDS as four independent chains over contiguous quarters
// (8-byte blocks split as evenly as possible, the last chain also takes the 0..7 tail bytes),
// merged by linearity: reg(A||B) = reg(A) * x^(8|B|) ^ reg0(B). One wave per SIMD is LDS-latency
// bound; four chains keep four lookup rounds in flight (tools/lds_bench.hip: 2.5x over one chain
// reading its payload from LDS).
__device__ __forceinline__ u32 crc32c_lds4(const u32 (*t)[256], const u32* pow8, const u32* w, u32 len) {
  const u32 n8 = len >> 3, q = n8 >> 2, r = n8 & 3u;
  const u32 s1 = q + (r > 0), s2 = s1 + q + (r > 1), s3 = s2 + q + (r > 2);
  u32 c0 = 0xFFFFFFFFu, c1 = 0, c2 = 0, c3 = 0;
  for (u32 i = 0; i < s1; ++i) {
    const u32 i1 = s1 + i, i2 = s2 + i, i3 = s3 + i;
    const bool a1 = i1 < s2, a2 = i2 < s3, a3 = i3 < n8;
    const u32 j1 = a1 ? i1 : 0u, j2 = a2 ? i2 : 0u, j3 = a3 ? i3 : 0u;
    const u32 x0 = w[2 * i], y0 = w[2 * i + 1];
    const u32 x1 = w[2 * j1], y1 = w[2 * j1 + 1];
    const u32 x2 = w[2 * j2], y2 = w[2 * j2 + 1];
    const u32 x3 = w[2 * j3], y3 = w[2 * j3 + 1];
    c0 = crc_step8(t, c0, x0, y0);
    const u32 n1 = crc_step8(t, c1, x1, y1), n2 = crc_step8(t, c2, x2, y2), n3 = crc_step8(t, c3, x3, y3);
    c1 = a1 ? n1 : c1;
    c2 = a2 ? n2 : c2;
    c3 = a3 ? n3 : c3;
  }
  c3 = crc_stepn(t, c3, w[2 * n8], w[2 * n8 + 1], len & 7u);
  const u32 m = gf2_mulmod(pow8[len - 8 * s1], c0) ^ gf2_mulmod(pow8[len - 8 * s2], c1) ^
                gf2_mulmod(pow8[len - 8 * s3], c2);
  return ~(m ^ c3);
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
