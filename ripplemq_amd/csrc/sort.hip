// sort.hip — batch-local stable partition sort: the "segmented prefix-sum" front half of append.
//
// Reference semantics (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:64-69):
// the records of one partition are applied in batch order and get consecutive offsets. The append
// kernel consumes the batch reordered partition-major, *stably*, as 16-byte slot records
// {pidx, record index, payload length | bad-partition flag, payload offset}; this file makes them.
//
// LSD radix over the partition id, one launch per digit of <= 8 bits (1 launch for P <= 256,
// 2 for P <= 65536). One workgroup = one tile of 2048 keys; wave w owns the contiguous keys
// [base + 512w, +512) and reads them in 8 rounds of 64 lanes, so (wave, round, lane) is key order.
//  * in-tile stable rank: ballot-match the digit bits per 64-key round; a per-wave LDS counter per
//    digit carries ranks across rounds; the 4 waves are then prefixed per digit;
//  * cross-tile prefix and digit totals: every tile publishes its <= 256 counts as {epoch|count}
//    granules and reads every tile's counts back (tiles^2 * 2 KB; 2 MB at a 64k-record batch).
//    The loads of a poll are issued together (no serial look-back walk, which degenerates when
//    all tiles start at once);
//  * the first pass also sums {payload bytes, record bytes} per tile in input order and exchanges
//    those sums the same way: packed payload offsets and the batch record-byte total (ENOSPC).
// Tiles wait on each other, so all must be resident: <= 128 workgroups of 256 threads.
#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr u32 kST = kSortThreads;     // 256
constexpr u32 kSI = kSortItems;       // 8 keys per thread
constexpr u32 kSW = kST / 64;         // 4 waves
constexpr u32 kWK = kSortTile / kSW;  // keys per wave (512)

// Sum a column of {epoch|value} granules over all tiles and over tiles < `tile`. The loads of a
// sweep are issued 32 at a time before any is inspected (one round trip for <= 32 tiles); the
// sweep repeats until every tag matches (bounded).
__device__ __forceinline__ bool sweep_column(const u64* g, u32 stride, u32 tiles, u32 tile, u32 epoch,
                                             u32* before, u32* total) {
  for (u32 spins = 0; spins < kSpinLimit; ++spins) {
    u32 b = 0, t = 0;
    bool ok = true;
    for (u32 t0 = 0; t0 < tiles; t0 += 32) {
      u64 x[32];
#pragma unroll
      for (u32 i = 0; i < 32; ++i) x[i] = gran_load(g + (u64)(t0 + i < tiles ? t0 + i : 0) * stride);
#pragma unroll
      for (u32 i = 0; i < 32; ++i) {
        const bool in = t0 + i < tiles;
        ok &= !in || (u32)(x[i] >> 32) == epoch;
        const u32 c = in ? (u32)x[i] : 0u;
        t += c;
        b += t0 + i < tile ? c : 0u;
      }
    }
    if (ok) {
      *before = b;
      *total = t;
      return true;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}

// Payload-byte and record-byte sums of all tiles, by one whole wave: lane l holds tiles l and
// l + 64 (<= 128 tiles). The first poll's loads are issued by the caller early (`x`, `y`), so their
// latency overlaps the ranking; lanes re-poll only until every tag matches (bounded).
__device__ __forceinline__ bool sweep_lenrb_wave(const u64* g0, const u64* g1, u32 tiles, u32 tile, u32 epoch,
                                                 u32 lane, u64 (&x)[2], u64 (&y)[2], u32* pre_len,
                                                 u32* tot_len, u32* tot_rb) {
  for (u32 spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (u32 h = 0; h < 2; ++h) {
      const u32 t = lane + 64 * h;
      ok &= t >= tiles || ((u32)(x[h] >> 32) == epoch && (u32)(y[h] >> 32) == epoch);
    }
    if (__all(ok)) break;
    if (spins >= kSpinLimit) return false;
    __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (u32 h = 0; h < 2; ++h) {
      const u32 t = lane + 64 * h < tiles ? lane + 64 * h : 0;
      x[h] = gran_load(g0 + t);
      y[h] = gran_load(g1 + t);
    }
  }
  u32 pl = 0, tl = 0, tr = 0;
#pragma unroll
  for (u32 h = 0; h < 2; ++h) {
    const u32 t = lane + 64 * h;
    const u32 c0 = t < tiles ? (u32)x[h] : 0u, c1 = t < tiles ? (u32)y[h] : 0u;
    tl += c0;
    tr += c1;
    pl += t < tile ? c0 : 0u;
  }
  for (int d = 32; d >= 1; d >>= 1) {
    pl += __shfl_xor(pl, d, 64);
    tl += __shfl_xor(tl, d, 64);
    tr += __shfl_xor(tr, d, 64);
  }
  *pre_len = pl;
  *tot_len = tl;
  *tot_rb = tr;
  return true;
}

// Phase stamps for the diagnostic run (RMQ_STAMPS): never read by the kernel itself.
#define SORT_STAMP(i)                                                                 \
  do {                                                                                \
    if (a.stamps) {                                                                   \
      const u64 t_ = __builtin_amdgcn_s_memrealtime();                                \
      if (tid == 0) a.stamps[(u64)tile * 8 + (i)] = t_;                               \
    }                                                                                 \
  } while (0)

__global__ __launch_bounds__(kST) void sort_pass_kernel(SortPassArgs a) {
  __shared__ uint16_t s_wcnt[kSW][256];  // per-wave digit counters, then per-wave bases
  __shared__ u32 s_start[256];           // this tile's global position base per digit
  __shared__ u32 s_scan[kSW];
  __shared__ u64 s_wtot[kSW];
  __shared__ u32 s_pre_len;

  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const u32 tile = blockIdx.x, tiles = a.tiles, nd = a.ndig;
  const u32 base = tile * kSortTile + w * kWK;
  const u32 dmask = (1u << a.bits) - 1u;
  const u64 lt = (1ull << lane) - 1ull;

  SORT_STAMP(0);
  reinterpret_cast<u32*>(&s_wcnt[0][0])[tid] = 0;  // kSW * 256 u16 = 2 u32 per thread
  reinterpret_cast<u32*>(&s_wcnt[0][0])[tid + kST] = 0;

  u32 key[kSI], val[kSI], rnk[kSI], len_[kSI], so_[kSI];
  u32 bad = 0;  // bit k: record k of this thread names a partition >= P
#pragma unroll
  for (u32 k = 0; k < kSI; ++k) {
    const u32 j = base + k * 64u + lane;
    u32 kk = 0, v = 0, L = 0;
    if (j < a.n) {
      kk = a.keys_in[j];
      if (a.first) {
        if (kk >= a.P) bad |= 1u << k;
        kk = kk < a.P ? kk : a.P - 1;
        v = j;
        L = a.len[j];
      } else {
        v = a.vals_in[j];
      }
    }
    key[k] = kk;
    val[k] = v;
    len_[k] = L;
    so_[k] = 0;
  }

  if (a.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SORT_STAMP(1);
  // ---- first pass: input-order scan of {record bytes : payload bytes} inside the tile
  if (a.first) {
    u64 wcarry = 0;
#pragma unroll
    for (u32 k = 0; k < kSI; ++k) {
      const u32 j = base + k * 64u + lane;
      const u64 v = j < a.n ? ((u64)record_bytes(len_[k]) << 32) | len_[k] : 0ull;
      const u64 inc = wave_incl_scan(v);
      so_[k] = (u32)(wcarry + inc - v);
      wcarry += ((u64)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32) |
                __builtin_amdgcn_readlane((u32)inc, 63);
    }
    if (lane == 0) s_wtot[w] = wcarry;
    __syncthreads();
    u64 wpre = 0, tile_sum = 0;
#pragma unroll
    for (u32 ww = 0; ww < kSW; ++ww) {
      const u64 t = s_wtot[ww];
      wpre += ww < w ? t : 0ull;
      tile_sum += t;
    }
#pragma unroll
    for (u32 k = 0; k < kSI; ++k) so_[k] += (u32)wpre;
    if (tid == 0) {
      gran_store(&a.len_gran[tile], a.epoch, (u32)tile_sum);
      gran_store(&a.rb_gran[tile], a.epoch, (u32)(tile_sum >> 32));
    }
  }
  // first poll of every tile's {payload, record} byte sums: issued now, inspected after ranking
  u64 lx[2] = {0, 0}, ly[2] = {0, 0};
  if (a.first && w == 0) {
#pragma unroll
    for (u32 h = 0; h < 2; ++h) {
      const u32 t = lane + 64 * h < tiles ? lane + 64 * h : 0;
      lx[h] = gran_load(a.len_gran + t);
      ly[h] = gran_load(a.rb_gran + t);
    }
  }

  // ---- in-tile stable ranking per wave
  __syncthreads();
  SORT_STAMP(2);
#pragma unroll
  for (u32 k = 0; k < kSI; ++k) {
    const u32 j = base + k * 64u + lane;
    const bool valid = j < a.n;
    const u32 d = (key[k] >> a.shift) & dmask;
    u64 peers = __ballot(valid);
    for (u32 b = 0; b < a.bits; ++b) {
      const bool bit = (d >> b) & 1u;
      const u64 bb = __ballot(bit && valid);
      peers &= bit ? bb : ~bb;
    }
    const u64 below = peers & lt;
    rnk[k] = valid ? (u32)s_wcnt[w][d] + (u32)__popcll(below) : 0u;
    __builtin_amdgcn_wave_barrier();
    if (valid && below == 0) s_wcnt[w][d] = (uint16_t)(s_wcnt[w][d] + __popcll(peers));
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();

  SORT_STAMP(3);
  // ---- per digit: wave bases and the tile count, published as a granule
  u32 cnt = 0;
  if (tid < nd) {
#pragma unroll
    for (u32 ww = 0; ww < kSW; ++ww) {
      const u32 c = s_wcnt[ww][tid];
      s_wcnt[ww][tid] = (uint16_t)cnt;
      cnt += c;
    }
    gran_store(&a.hist_gran[(u64)tile * 256 + tid], a.epoch, cnt);
  }

  SORT_STAMP(4);
  // ---- all-to-all: counts of earlier tiles and digit totals (batched polls)
  u32 before = 0, total = 0;
  if (tid < nd && !sweep_column(a.hist_gran + tid, 256, tiles, tile, a.epoch, &before, &total))
    atomicOr(a.err, kErrSpinTimeout);
  if (a.first && w == 0) {  // the byte sums, by wave 0
    u32 lb = 0, ltot = 0, rtot = 0;
    if (!sweep_lenrb_wave(a.len_gran, a.rb_gran, tiles, tile, a.epoch, lane, lx, ly, &lb, &ltot, &rtot)) {
      if (lane == 0) atomicOr(a.err, kErrSpinTimeout);
    }
    if (lane == 0) {
      s_pre_len = lb;
      if (tile == tiles - 1) {
        a.batch_info[0] = rtot;  // record bytes of the batch
        a.batch_info[1] = ltot;  // payload bytes of the batch
      }
    }
  }
  SORT_STAMP(5);
  {
    u32 all_tot;
    const u32 dexcl = block_excl_scan<kSW>(tid < nd ? total : 0u, s_scan, &all_tot);
    if (tid < nd) s_start[tid] = dexcl + before;
  }
  __syncthreads();

  SORT_STAMP(6);
  // ---- scatter
  const u32 pre_len = a.first ? s_pre_len : 0u;
#pragma unroll
  for (u32 k = 0; k < kSI; ++k) {
    const u32 j = base + k * 64u + lane;
    if (j >= a.n) continue;
    const u32 d = (key[k] >> a.shift) & dmask;
    const u32 pos = s_start[d] + s_wcnt[w][d] + rnk[k];
    if (pos >= a.n) continue;  // only after a lost hand-off (err is set)
    if (a.last) {
      u32 L, so;
      bool b;
      if (a.first) {
        L = len_[k];
        so = a.payload_off ? (u32)a.payload_off[j] : pre_len + so_[k];
        b = (bad >> k) & 1u;
      } else {
        L = a.len[val[k]];
        so = a.payload_off ? (u32)a.payload_off[val[k]] : a.src_off[val[k]];
        b = a.pidx_raw[val[k]] >= a.P;
      }
      a.slots[pos] = make_uint4(key[k], val[k], b ? (L | 0x80000000u) : L, so);
    } else {
      a.keys_out[pos] = key[k];
      a.vals_out[pos] = val[k];
    }
  }
  if (a.first && !a.last && a.src_off) {
#pragma unroll
    for (u32 k = 0; k < kSI; ++k) {
      const u32 j = base + k * 64u + lane;
      if (j < a.n) a.src_off[j] = pre_len + so_[k];
    }
  }
  if (a.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SORT_STAMP(7);
}

void launch_sort_pass(const SortPassArgs& a, uint32_t tiles, hipStream_t s) {
  hipLaunchKernelGGL(sort_pass_kernel, dim3(tiles), dim3(kST), 0, s, a);
}

}  // namespace rmq
