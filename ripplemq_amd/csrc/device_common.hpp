// device_common.hpp — gfx950 device helpers shared by the engine kernels.
//
//  * CRC32C (Castagnoli, reflected 0x82F63B78): slicing-by-8 tables and 32-byte / 16-byte
//    zero-shift tables, copied into LDS by the kernels that checksum records (append, follower
//    ingest); a lane folds its 16-byte pieces by Horner's rule, reg(A || B) = reg(A) * x^(8|B|) ^ reg(B).
//  * wave64 scans built on __shfl_up and one LDS word per wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rmq {

typedef uint32_t u32;
typedef uint64_t u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) u32 gu32;

// Relaxed agent-scope (`sc1`) global accesses: an L2-coherent hand-off between workgroups of one
// launch without fences (MI355X_MICROARCH.md, inter-workgroup visibility, first table row).
__device__ __forceinline__ void store_sc1(u64* p, u64 v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 load_sc1(const u64* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr u32 kCrcPoly = 0x82F63B78u;
constexpr u32 kRecAlign = 16;         // FORMAT.md §1: records padded to 16 bytes

// Device constants: CRC tables and GF(2) shift constants, filled by the host at engine creation.
// table and zshift are adjacent so a kernel copies both into LDS as one run of 16-byte blocks.
struct CrcConsts {
  u32 table[8][256];      // slicing-by-8: table[k][b] = CRC register after byte b then k zero bytes
  u32 zshift[2][4][256];  // zshift[k][i][b] = (b << 8i) * x^(8 * 16 * 2^k): register shift past 16 << k zero bytes
  u32 zshift1k[4][256];   // register shift past 1024 zero bytes (a wave's round of 64 pieces)
  u32 inv_pad[16];        // inv_pad[n] = x^(-8n) mod P: "remove n trailing zero bytes"
  u32 sh16[64];           // sh16[e] = x^(8 * 16 * e) mod P: shift past e 16-byte pieces
  u32 inv_pad16[16];      // inv_pad16[n] = inv_pad[n] * x^16: the low half of a split pad removal
  u32 nib[16][32];        // the 16 tables of table and zshift in order by nibble: t[b] = nib[q][b & 15] ^ nib[q][16 + (b >> 4)]
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
// A payload block read once per launch (RMQ_PAYLOAD_NT: non-temporal).
#ifndef RMQ_PAYLOAD_NT
#define RMQ_PAYLOAD_NT 1
#endif
__device__ __forceinline__ uint4 load_payload16(const void* src) {
#if RMQ_PAYLOAD_NT
  const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
  return make_uint4(x[0], x[1], x[2], x[3]);
#else
  return *reinterpret_cast<const uint4*>(src);
#endif
}

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

// Half of gf2_mulmod(a, b) for a lane pair: lane 0 takes a's coefficients of x^0..x^15 (bits
// 31..16) against b, lane 1 those of x^16..x^31 (bits 15..0) against b * x^16; the product is the
// XOR of the two halves.
__device__ __forceinline__ u32 gf2_mulmod_half(u32 a16, u32 b) {
  u32 p = 0;
#pragma unroll
  for (int k = 15; k >= 0; --k) {
    p ^= b & (0u - ((a16 >> k) & 1u));
    b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
  }
  return p;
}

// CRC register update over 8 bytes (lo, hi little-endian dwords), slicing-by-8.
__device__ __forceinline__ u32 crc_step8(const u32 (*t)[256], u32 c, u32 lo, u32 hi) {
  lo ^= c;
  return t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
         t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
}

// Register shift past 16 << k zero bytes (k = 0, 1) by a 4 x 256 table (linearity in the register).
__device__ __forceinline__ u32 crc_zshift(const u32 (*z)[256], u32 c) {
  return z[0][c & 0xFF] ^ z[1][(c >> 8) & 0xFF] ^ z[2][(c >> 16) & 0xFF] ^ z[3][c >> 24];
}

// The 16 KB of table and zshift (sixteen 256-entry tables, contiguous at `tabs`) built in LDS from
// their 2 KB of nibble tables: every table is GF(2)-linear in its byte, so entry b is
// nib[q][b & 15] ^ nib[q][16 + (b >> 4)]. Copying the 16 KB from L2 was two of the ~4.8 L1->L2 read
// requests per record of the stage-3 launch (profiles/r06_stage3_counters.txt); the nibble tables
// are a quarter of one. `scratch`: 2 KB of LDS nothing else touches until the caller's next
// barrier. crc_nib_lds holds one workgroup barrier (every thread of the workgroup must call it).
template <u32 kThreads>
__device__ __forceinline__ void crc_nib_lds(const CrcConsts* crc, u32* scratch) {
  static_assert(sizeof(CrcConsts::nib) == 128 * 16 && kThreads >= 128, "one 16-byte block per thread");
  if (threadIdx.x < 128u)
    reinterpret_cast<uint4*>(scratch)[threadIdx.x] = reinterpret_cast<const uint4*>(&crc->nib[0][0])[threadIdx.x];
  __syncthreads();
}
template <u32 kThreads>
__device__ __forceinline__ void crc_expand_lds(u32* tabs, const u32* scratch) {
  for (u32 b = threadIdx.x; b < 256u; b += kThreads) {
#pragma unroll
    for (u32 q = 0; q < 16u; ++q) tabs[256u * q + b] = scratch[32u * q + (b & 15u)] ^ scratch[32u * q + 16u + (b >> 4)];
  }
}
// (both halves; the caller may issue loads between them)
template <u32 kThreads>
__device__ __forceinline__ void crc_tables_lds(const CrcConsts* crc, u32* tabs, u32* scratch) {
  crc_nib_lds<kThreads>(crc, scratch);
  crc_expand_lds<kThreads>(tabs, scratch);
}

// CRC register of one 16-byte piece (two slicing-by-8 steps from a zero register).
__device__ __forceinline__ u32 crc_piece16(const u32 (*t)[256], uint4 v) {
  return crc_step8(t, crc_step8(t, 0u, v.x, v.y), v.z, v.w);
}

// Value of the partner lane of a lane pair (lanes 2i, 2i + 1), one DPP move.
__device__ __forceinline__ u32 pair_swap(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
}

// ---------------------------------------------------------------------------------------------
// Scans
// ---------------------------------------------------------------------------------------------

// DPP moves (VALU cross-lane, no LDS round trip): lanes the row mask leaves out, and lanes whose
// source lies outside their row, read 0. 64-bit values move as two halves.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ u32 dpp_mov(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xf, true);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ u64 dpp_mov(u64 v) {
  return ((u64)dpp_mov<kCtrl, kRowMask>((u32)(v >> 32)) << 32) | dpp_mov<kCtrl, kRowMask>((u32)v);
}

// Lane l's value in every lane (l wave-uniform).
__device__ __forceinline__ u64 bcast_u64(u64 v, u32 l) {
  return ((u64)(u32)__builtin_amdgcn_readlane((int)(v >> 32), (int)l) << 32) |
         (u32)__builtin_amdgcn_readlane((int)(u32)v, (int)l);
}

// Inclusive wave64 scan (u32 / u64): Hillis-Steele inside each row of 16 lanes (row_shr 1, 2, 4,
// 8), then rows 1 / 3 take the last lane of rows 0 / 2 (row_bcast:15) and rows 2-3 the last lane of
// row 1 (row_bcast:31).
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  v += dpp_mov<0x111, 0xf>(v);
  v += dpp_mov<0x112, 0xf>(v);
  v += dpp_mov<0x114, 0xf>(v);
  v += dpp_mov<0x118, 0xf>(v);
  v += dpp_mov<0x142, 0xa>(v);
  v += dpp_mov<0x143, 0xc>(v);
  return v;
}

// XOR of every lane's value, in every lane (the same moves as a scan, then lane 63's value).
__device__ __forceinline__ u32 wave_xor_all(u32 v) {
  v ^= dpp_mov<0x111, 0xf>(v);
  v ^= dpp_mov<0x112, 0xf>(v);
  v ^= dpp_mov<0x114, 0xf>(v);
  v ^= dpp_mov<0x118, 0xf>(v);
  v ^= dpp_mov<0x142, 0xa>(v);
  v ^= dpp_mov<0x143, 0xc>(v);
  return (u32)__builtin_amdgcn_readlane((int)v, 63);
}

// Segmented inclusive scan of pairs (flag, value), a set flag starting a new segment; the same
// moves, each combining (f, v) with the pair before: v += v' unless f, f |= f'. flag ends as the
// OR of the flags up to the lane.
template <typename T>
__device__ __forceinline__ void seg_step_(u32& flag, T& v, u32 of, T ov) {
  if (!flag) v += ov;
  flag |= of;
}
template <typename T>
__device__ __forceinline__ void wave_seg_incl_scan(u32& flag, T& v) {
  seg_step_(flag, v, dpp_mov<0x111, 0xf>(flag), dpp_mov<0x111, 0xf>(v));
  seg_step_(flag, v, dpp_mov<0x112, 0xf>(flag), dpp_mov<0x112, 0xf>(v));
  seg_step_(flag, v, dpp_mov<0x114, 0xf>(flag), dpp_mov<0x114, 0xf>(v));
  seg_step_(flag, v, dpp_mov<0x118, 0xf>(flag), dpp_mov<0x118, 0xf>(v));
  seg_step_(flag, v, dpp_mov<0x142, 0xa>(flag), dpp_mov<0x142, 0xa>(v));
  seg_step_(flag, v, dpp_mov<0x143, 0xc>(flag), dpp_mov<0x143, 0xc>(v));
}

}  // namespace rmq
