// sort.hip — batch-local stable partition sort: the "segmented prefix-sum" front half of append.
//
// Reference semantics (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:64-69):
// the records of one partition are applied in batch order and get consecutive offsets. The append
// kernel consumes the batch reordered partition-major, *stably*, as 16-byte slot records
// {pidx, record index, payload length, payload offset}; this file produces them.
//
// One launch per 12-bit digit of the partition id (one launch for P <= 4096, two up to 2^24).
// One workgroup = one tile of 1024 keys; wave w owns the contiguous keys [base + 256w, +256) and
// reads them in rounds k of 64 (key j = base + 256w + 64k + lane), so (w, k, lane) is key order.
//  * in-tile stable rank: per wave, rounds of 64 keys are ballot-matched on the digit bits; a
//    per-wave LDS counter per digit carries ranks across rounds; waves are then prefixed per digit;
//  * cross-tile prefix: decoupled look-back per digit over {epoch | AGG/INCL | count} granules
//    (each thread owns 16 consecutive digits and walks them in lock-step, loads in flight together);
//  * global digit starts: every tile reads the LAST tile's inclusive prefix (= the digit totals)
//    once published — no histogram kernel and no memset between batches;
//  * the first pass also scans {payload bytes, record bytes} in input order with a one-value
//    look-back: packed payload offsets and the batch record-byte total (ENOSPC rule) for free.
// Every tile waits on predecessors and on the last tile, so all tiles must be resident together:
// the grid is capped at 256 workgroups of 256 threads (engine.cpp).
#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr u32 kST = kSortThreads;       // 256
constexpr u32 kSI = kSortItems;         // 4
constexpr u32 kSW = kST / 64;           // waves per tile
constexpr u32 kDPT = kMaxDigits / kST;  // digits owned per thread (16)
constexpr u32 kAgg = 1u, kIncl = 2u;

__global__ __launch_bounds__(kST) void sort_pass_kernel(SortPassArgs a) {
  __shared__ uint16_t s_wcnt[kSW][kMaxDigits];  // per-wave digit counters, then per-wave bases
  __shared__ u32 s_start[kMaxDigits];           // this tile's global position base per digit
  __shared__ u64 s_scan64[kSW];
  __shared__ u32 s_scan[kSW];
  __shared__ u64 s_pre_len;

  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const u32 tile = blockIdx.x, tiles = a.tiles, nd = a.ndig;
  const u32 base = tile * kSortTile;
  const u32 dmask = (1u << a.bits) - 1u;
  const u64 lt = (1ull << lane) - 1ull;
  const u32 d0 = tid * kDPT;  // first digit owned by this thread

  for (u32 k = tid; k < kSW * kMaxDigits / 2; k += kST) reinterpret_cast<u32*>(&s_wcnt[0][0])[k] = 0;

  u32 key[kSI], val[kSI], rnk[kSI], len_[kSI], so_[kSI];
  u32 bad = 0;  // bit k: record k of this thread names a partition >= P
#pragma unroll
  for (u32 k = 0; k < kSI; ++k) {
    const u32 j = base + w * 256u + k * 64u + lane;
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

  // ---- first pass: input-order scan of {record bytes : payload bytes}, one-value look-back
  if (a.first) {
    // wave-contiguous keys: scan per wave over its rounds, then prefix the 4 wave totals
    u64 wcarry = 0;
#pragma unroll
    for (u32 k = 0; k < kSI; ++k) {
      const u32 j = base + w * 256u + k * 64u + lane;
      const u64 v = j < a.n ? ((u64)(16u + ((len_[k] + 3u) & ~3u)) << 32) | len_[k] : 0ull;
      const u64 inc = wave_incl_scan(v);
      so_[k] = (u32)(wcarry + inc - v);
      wcarry += ((u64)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32) | __builtin_amdgcn_readlane((u32)inc, 63);
    }
    if (lane == 0) s_scan64[w] = wcarry;
    __syncthreads();
    u64 carry = 0, wpre = 0;
#pragma unroll
    for (u32 ww = 0; ww < kSW; ++ww) {
      const u64 t = s_scan64[ww];
      wpre += ww < w ? t : 0ull;
      carry += t;
    }
#pragma unroll
    for (u32 k = 0; k < kSI; ++k) so_[k] += (u32)wpre;
    if (tid == 0) {
      u64 pre = 0;
      if (tile == 0) {
        store_sc1_u64(&a.len_val[1], carry);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gran_store(&a.len_gran[0], a.epoch, kIncl);
      } else {
        store_sc1_u64(&a.len_val[2 * tile], carry);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gran_store(&a.len_gran[tile], a.epoch, kAgg);
        long t = (long)tile - 1;
        for (u32 spins = 0;;) {
          const u64 x = gran_load(&a.len_gran[t]);
          if ((u32)(x >> 32) == a.epoch) {
            if ((u32)x == kIncl) {
              pre += load_sc1_u64(&a.len_val[2 * t + 1]);
              break;
            }
            pre += load_sc1_u64(&a.len_val[2 * t]);
            --t;
            continue;
          }
          if (++spins >= kSpinLimit) {
            atomicOr(a.err, kErrSpinTimeout);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        store_sc1_u64(&a.len_val[2 * tile + 1], pre + carry);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gran_store(&a.len_gran[tile], a.epoch, kIncl);
      }
      s_pre_len = pre;
      if (tile == tiles - 1) {
        a.batch_info[0] = (pre + carry) >> 32;          // record bytes of the batch
        a.batch_info[1] = (u32)(pre + carry);           // payload bytes of the batch
      }
    }
  }

  // ---- in-tile stable ranking per wave (rounds k = 0..3 are in key order)
  __syncthreads();
#pragma unroll
  for (u32 k = 0; k < kSI; ++k) {
    const u32 j = base + w * 256u + k * 64u + lane;
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

  // ---- owned digits: wave bases, tile count; publish AGG (INCL on tile 0)
  u32 cnt[kDPT], pre[kDPT];
#pragma unroll
  for (u32 i = 0; i < kDPT; ++i) {
    const u32 d = d0 + i;
    u32 run = 0;
    if (d < nd) {
#pragma unroll
      for (u32 ww = 0; ww < kSW; ++ww) {
        const u32 c = s_wcnt[ww][d];
        s_wcnt[ww][d] = (uint16_t)run;
        run += c;
      }
      gran_store(&a.hist_gran[(u64)tile * nd + d], a.epoch, ((tile ? kAgg : kIncl) << 30) | run);
    }
    cnt[i] = run;
    pre[i] = 0;
  }

  // ---- decoupled look-back, the 16 owned digits in lock-step
  if (tile) {
    long t[kDPT];
    u32 live = 0;
#pragma unroll
    for (u32 i = 0; i < kDPT; ++i) {
      t[i] = (long)tile - 1;
      if (d0 + i < nd) live |= 1u << i;
    }
    for (u32 spins = 0; live;) {
      u64 x[kDPT];
#pragma unroll
      for (u32 i = 0; i < kDPT; ++i) x[i] = (live >> i & 1u) ? gran_load(&a.hist_gran[(u64)t[i] * nd + d0 + i]) : 0ull;
      bool progress = false;
#pragma unroll
      for (u32 i = 0; i < kDPT; ++i) {
        if (!(live >> i & 1u) || (u32)(x[i] >> 32) != a.epoch) continue;
        progress = true;
        pre[i] += ((u32)x[i]) & 0x3FFFFFFFu;
        if ((((u32)x[i]) >> 30) == kIncl)
          live &= ~(1u << i);
        else
          --t[i];
      }
      if (!progress) {
        if (++spins >= kSpinLimit) {
          atomicOr(a.err, kErrSpinTimeout);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
#pragma unroll
    for (u32 i = 0; i < kDPT; ++i)
      if (d0 + i < nd) gran_store(&a.hist_gran[(u64)tile * nd + d0 + i], a.epoch, (kIncl << 30) | (pre[i] + cnt[i]));
  }

  // ---- digit totals = the last tile's inclusive prefix; exclusive scan over digits
  u32 tot[kDPT];
  if (tile == tiles - 1) {
#pragma unroll
    for (u32 i = 0; i < kDPT; ++i) tot[i] = pre[i] + cnt[i];
  } else {
    for (u32 spins = 0;;) {
      bool all = true;
#pragma unroll
      for (u32 i = 0; i < kDPT; ++i) {
        tot[i] = 0;
        if (d0 + i >= nd) continue;
        const u64 x = gran_load(&a.hist_gran[(u64)(tiles - 1) * nd + d0 + i]);
        all &= (u32)(x >> 32) == a.epoch && (((u32)x) >> 30) == kIncl;
        tot[i] = ((u32)x) & 0x3FFFFFFFu;
      }
      if (all) break;
      if (++spins >= kSpinLimit) {
        atomicOr(a.err, kErrSpinTimeout);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  {
    u32 mine = 0;
#pragma unroll
    for (u32 i = 0; i < kDPT; ++i) mine += tot[i];
    u32 all_tot;
    u32 run = block_excl_scan<kSW>(mine, s_scan, &all_tot);
#pragma unroll
    for (u32 i = 0; i < kDPT; ++i) {
      if (d0 + i < nd) s_start[d0 + i] = run + pre[i];
      run += tot[i];
    }
  }
  __syncthreads();

  // ---- scatter
  const u32 pre_len = a.first ? (u32)s_pre_len : 0u;
#pragma unroll
  for (u32 k = 0; k < kSI; ++k) {
    const u32 j = base + w * 256u + k * 64u + lane;
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
      const u32 j = base + w * 256u + k * 64u + lane;
      if (j < a.n) a.src_off[j] = pre_len + so_[k];
    }
  }
}

void launch_sort_pass(const SortPassArgs& a, uint32_t tiles, hipStream_t s) {
  hipLaunchKernelGGL(sort_pass_kernel, dim3(tiles), dim3(kST), 0, s, a);
}

}  // namespace rmq
