// sort.hip — batch-local stable partition sort: the "segmented prefix-sum" front half of append.
//
// Reference semantics (PartitionStateMachine.java:64-69): records of one partition are applied in
// batch order and get consecutive offsets. The append kernel needs the batch reordered
// partition-major *stably*; this file provides one LSD radix pass per `bits`-wide digit of the
// partition id (1 pass for P <= 256, 2 for P <= 65536).
//
// One workgroup = one tile of 4096 keys (512 threads x 8, striped so that key j = q*512 + tid).
// Per tile: wave64 ballot matching ranks equal digits inside each 64-key round; an LDS table of
// per-(round, wave, digit) counts scanned per digit gives the stable in-tile rank and the tile
// histogram. Tiles exchange histograms in one launch through {epoch, count} granules (every
// tile reads every tile's 256 counts: tiles^2 * 2 KB, 512 KB at the 64k-record batch) — no
// separate histogram kernel, no scan kernel. Pass 0 also scans payload lengths in input order
// (packed payload offsets) and totals the batch's record bytes for the ENOSPC rule.
#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr u32 kW = kSortThreads / 64;  // waves per tile
constexpr u32 kQ = kSortItems;         // rounds per tile

__global__ __launch_bounds__(kSortThreads) void sort_pass_kernel(SortPassArgs a) {
  __shared__ uint16_t s_cnt[kQ][kW][256];
  __shared__ u32 s_base[256];
  __shared__ u32 s_scan[kW];
  __shared__ u32 s_scan2[kW];

  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const u32 tile = blockIdx.x, tiles = a.tiles;
  const u32 base = tile * kSortTile;
  const u32 dmask = (1u << a.bits) - 1u;

  {
    u32* z = reinterpret_cast<u32*>(&s_cnt[0][0][0]);
    for (u32 k = tid; k < kQ * kW * 256 / 2; k += kSortThreads) z[k] = 0;
  }
  if (a.first && tile == 0 && tid < 4) a.stats[tid] = 0;

  u32 key[kQ], val[kQ], rnk[kQ];
#pragma unroll
  for (u32 q = 0; q < kQ; ++q) {
    const u32 j = base + q * kSortThreads + tid;
    const bool valid = j < a.n;
    u32 k = 0, v = 0;
    if (valid) {
      k = a.keys_in[j];
      if (a.first) {
        k = k < a.P ? k : a.P - 1;
        v = j;
      } else {
        v = a.vals_in[j];
      }
    }
    key[q] = k;
    val[q] = v;
  }

  // pass 0: payload-length scan in input order (blocked layout: 8 consecutive records/thread)
  u32 len_run[kSortItems];
  u32 tile_len = 0, tile_rb = 0, len_excl = 0;
  if (a.first) {
    u32 s = 0, rb = 0;
#pragma unroll
    for (u32 k = 0; k < kSortItems; ++k) {
      const u32 j = base + tid * kSortItems + k;
      const u32 L = j < a.n ? a.len[j] : 0u;
      len_run[k] = s;
      s += L;
      rb += j < a.n ? 16u + ((L + 3u) & ~3u) : 0u;
    }
    len_excl = block_excl_scan<kW>(s, s_scan, &tile_len);
    u32 dummy = block_excl_scan<kW>(rb, s_scan2, &tile_rb);
    (void)dummy;
    if (tid == 0) {
      gran_store(&a.len_gran[tile], a.epoch, tile_len);
      gran_store(&a.rb_gran[tile], a.epoch, tile_rb);
    }
  }
  __syncthreads();

  // in-tile stable ranking: ballot-match equal digits per 64-key round
  const u64 lt_mask = (1ull << lane) - 1ull;
#pragma unroll
  for (u32 q = 0; q < kQ; ++q) {
    const u32 j = base + q * kSortThreads + tid;
    const bool valid = j < a.n;
    const u32 d = (key[q] >> a.shift) & dmask;
    u64 peers = __ballot(valid);
    for (u32 b = 0; b < a.bits; ++b) {
      const bool bit = (d >> b) & 1u;
      const u64 bb = __ballot(bit && valid);
      peers &= bit ? bb : ~bb;
    }
    const u64 below = peers & lt_mask;
    rnk[q] = __popcll(below);
    if (valid && below == 0) s_cnt[q][w][d] = (uint16_t)__popcll(peers);
  }
  __syncthreads();

  // per-digit exclusive scan over (round, wave) -> stable in-tile base; tile histogram
  if (tid < 256) {
    u32 run = 0;
#pragma unroll
    for (u32 q = 0; q < kQ; ++q)
#pragma unroll
      for (u32 ww = 0; ww < kW; ++ww) {
        const u32 c = s_cnt[q][ww][tid];
        s_cnt[q][ww][tid] = (uint16_t)run;
        run += c;
      }
    gran_store(&a.hist_gran[(u64)tile * 256 + tid], a.epoch, run);
  }

  // all-to-all: digit totals over all tiles and counts of the tiles before this one
  u32 before = 0, total = 0;
  if (tid < 256) {
    for (u32 spins = 0;; ++spins) {
      bool ok = true;
      before = 0;
      total = 0;
      for (u32 t = 0; t < tiles; ++t) {
        const u64 x = gran_load(&a.hist_gran[(u64)t * 256 + tid]);
        ok &= (u32)(x >> 32) == a.epoch;
        const u32 c = (u32)x;
        total += c;
        before += t < tile ? c : 0u;
      }
      if (ok) break;
      if (spins >= kSpinLimit) {
        atomicOr(a.err, kErrSpinTimeout);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  {
    u32 tot_all;
    const u32 dexcl = block_excl_scan<kW>(tid < 256 ? total : 0u, s_scan, &tot_all);
    if (tid < 256) s_base[tid] = dexcl + before;
  }

  // pass 0: packed payload offsets (prefix over earlier tiles) and the batch record-byte total
  if (a.first) {
    if (tid < 64) {
      u32 pre = 0;
      u64 rb_all = 0;
      for (u32 spins = 0;; ++spins) {
        bool ok = true;
        u32 p = 0;
        u64 r = 0;
        for (u32 t = lane; t < tiles; t += 64) {
          const u64 x = gran_load(&a.len_gran[t]);
          const u64 y = gran_load(&a.rb_gran[t]);
          ok &= (u32)(x >> 32) == a.epoch && (u32)(y >> 32) == a.epoch;
          p += t < tile ? (u32)x : 0u;
          r += (u32)y;
        }
        const bool all_ok = __all(ok);
        if (all_ok) {
          for (int d = 32; d >= 1; d >>= 1) {
            p += __shfl_xor(p, d, 64);
            r += __shfl_xor(r, d, 64);
          }
          pre = p;
          rb_all = r;
          break;
        }
        if (spins >= kSpinLimit) {
          if (lane == 0) atomicOr(a.err, kErrSpinTimeout);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (tid == 0) {
        s_scan2[0] = pre;
        if (tile == 0) a.batch_info[0] = rb_all;
      }
    }
    __syncthreads();
    if (a.src_off) {
      const u32 pre = s_scan2[0] + len_excl;
#pragma unroll
      for (u32 k = 0; k < kSortItems; ++k) {
        const u32 j = base + tid * kSortItems + k;
        if (j < a.n) a.src_off[j] = pre + len_run[k];
      }
    }
  }
  __syncthreads();

  // scatter to the stable global position
#pragma unroll
  for (u32 q = 0; q < kQ; ++q) {
    const u32 j = base + q * kSortThreads + tid;
    if (j < a.n) {
      const u32 d = (key[q] >> a.shift) & dmask;
      const u32 pos = s_base[d] + s_cnt[q][w][d] + rnk[q];
      if (pos < a.n) {  // always true for a consistent histogram; guards a lost hand-off
        a.keys_out[pos] = key[q];
        a.vals_out[pos] = val[q];
      }
    }
  }
}

void launch_sort_pass(const SortPassArgs& a, uint32_t tiles, hipStream_t s) {
  hipLaunchKernelGGL(sort_pass_kernel, dim3(tiles), dim3(kSortThreads), 0, s, a);
}

}  // namespace rmq
