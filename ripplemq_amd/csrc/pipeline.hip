// pipeline.hip — the append path as a four-stage software pipeline over GROUPS of batches: one
// launch ranks group g, scans group g-1, applies group g-2 and evaluates retention of group g-3,
// so no stage waits on another inside a launch.
//
// Reference semantics restated (file:line relative to the reference root):
//   PartitionStateMachine.onApply / handleMessageAppendRequest — messages.addAll(batch): record j of
//   an applied entry gets offset size_before + j, per partition, in apply order
//   (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:38-69);
//   MessageAppendRequestProcessor "Not leader" gate (.../processor/MessageAppendRequestProcessor.java:29-32);
//   jraft BallotBox quorum commit: commit = k-th largest matchIndex, k = RF/2 + 1,
//   when that entry is from the current term. Log bytes, index and retention: FORMAT.md.
//
// A group is up to kMaxGroup consecutive batches (engine.cpp forms them). Every batch keeps its own
// semantics: offsets in batch order, the no-space rule, its stats, retention after the batch.
// Stage 1 (group g, workgroup per 1024-record tile of one batch, no inter-workgroup traffic):
//   stable LDS radix sort of the tile by partition id (8-bit passes, ballot-match ranks), a
//   segmented scan of {1, record bytes/16} over the sorted tile, which gives every record its
//   count / byte rank inside its partition's run in the tile, and the tile aggregate of each
//   present partition, written sparsely into the column-major hist[p][tile]. Also the tile's
//   payload prefix and sums.
// Stage 2 (group g-1, 16 threads per partition column, contiguous column reads): the batch rule
//   for invalid payload ranges from the tile sums, then per batch an exclusive scan of hist[p][.]
//   over the batch's tiles -> excl[p][tile]; a (batch, partition) whose record bytes exceed
//   segment - interval takes no record (FORMAT.md §3: its cells are flagged kExclNoSpace and it
//   adds nothing to the prefix); the aggregate through each batch bcum[j][p] and totals[p]; clears
//   hist for reuse. Workgroup 0 also writes the payload base of every tile in its batch.
// Stage 3 (group g-2, wave per 32-record task): offset = log end + excl + rank, position likewise,
//   out offsets, sparse index, then the records' 16-byte pieces are spread over the lanes (a piece
//   whose ring slot a later piece of the same group overwrites is not stored, so no two stores of
//   one launch ever hit the same ring bytes): payload
//   loads as aligned 16-byte blocks, CRC32C of each piece from LDS tables (folded per lane by
//   Horner with a zero-byte shift table, XOR-reduced per record), 16-byte stores into every local replica ring
//   through an LDS image of the log. Partition threads (workgroups of their own, from the start of
//   the launch): the group's new log end, matchIndex, quorum commit and high watermark, into the
//   other state set, so no record ever reads a half-updated partition.
// Stage 4 (group g-3, the same partition threads): retention after each batch of the group, from
//   the sparse-index entries that stage 3 wrote one launch earlier (FORMAT.md §4).
//
// Launch k starts only after launch k-1 has finished (one stream), so every hand-off between
// stages crosses a kernel boundary. Launch k's first lane reports launch k-1 complete to the host.
#include <hip/hip_ext.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "partition_ops.hpp"


// This file is compiled twice (Makefile): as namespace rmq with RMQ_PIPE_THREADS=256 for the
// single-GPU kernel, and as namespace rmq_x with 512 threads and RMQ_PIPE_XR_TU for the kernel with
// a replication transport (its stage 3 also fills outboxes). The transport kernel keeps the
// 512-thread workgroups it was developed with: A/B runs over the in-process transport (2 ranks on
// one GPU) were inconclusive (the same kernel varied by +-8 % between runs).
#ifndef RMQ_PIPE_NS
#define RMQ_PIPE_NS rmq
#endif
namespace RMQ_PIPE_NS {
using namespace rmq;

constexpr u32 kPT = kPipeThreads;   // 512 (RMQ_PIPE_THREADS)
constexpr u32 kPW = kPT / 64;       // 8 waves
constexpr u32 kTR = kTileRecs;      // 1024
constexpr u32 kTI = kTR / kPT;      // 2 records per thread in stage 1
constexpr u32 kWR = kTR / kPW;      // 128 records per wave in stage 1
constexpr u32 kIB = kTileIdxBits;   // 10
constexpr u32 kFlagShift = 29;
constexpr u32 kRankMask = (1u << kFlagShift) - 1u;
// stage-1 flags (leadership is per partition, so it cannot change another partition's ranks:
// stage 3 checks it)
constexpr u32 kFlNoPart = 1u, kFlInvalid = 4u, kFlJunk = 7u;
constexpr u64 kOne40 = 1ull << 40;
constexpr u64 kCnt23 = (1ull << 23) - 1ull;  // count field of an excl value (bits 40..62)
constexpr u64 kExclNoSpace = 1ull << 63;     // excl flag: the cell's (batch, partition) is rejected
constexpr u32 kRejInvalid = 2u;

// Diagnostic phase stamps (RMQ_STAMPS): stamps[(workgroup * 8 + wave) * 8 + k], s_memrealtime
// (100 MHz). Never read by the kernel.
#define PIPE_STAMP_ROW(row, k)                                                                \
  do {                                                                                        \
    if (A.stamps) {                                                                           \
      const u64 t_ = __builtin_amdgcn_s_memrealtime();                                        \
      if ((threadIdx.x & 63) == 0)                                                            \
        A.stamps[((u64)(row) * kPW + (threadIdx.x >> 6)) * 8 + (k)] = t_;                    \
    }                                                                                         \
  } while (0)
#define PIPE_STAMP(k) PIPE_STAMP_ROW(blockIdx.x, k)

struct Stage1Smem {
  u32 items[2][kTR];   // key << 10 | position in tile (ping-pong between radix passes)
  u32 cnt[kPW][256];   // per-wave digit counters, then per-wave digit bases
  u32 dbase[256];      // digit totals, then digit bases
  u32 info[kTR];       // record bytes/16 | flags << 29, by input position in the tile
  u64 wsum[kPW][2];
  u64 wtail[kPW];
  u32 whead[kPW];
  u32 scan[kPW];
};

struct Stage3Smem {
  u32 t8[8][256];       // slicing-by-8 CRC32C tables
  u32 z[2][4][256];     // register shift past 16 and 32 zero bytes
  uint4 img[kPW][kTaskRecs][8];  // per wave: the task's records as laid out in the log (<= 128 B each)
  uint4 info[kPW][kTaskRecs];    // per wave: {pos lo, pos hi, p, lm | m << 8 | ok << 16 | dead << 24}
  union {
    // single-GPU kernel: the register shift past 1024 zero bytes of the large-record waves (the
    // kernel with a transport reads it from global memory, L1/L2-resident: with 256-thread
    // workgroups LDS has room for four per CU only without it)
    u32 zk[4][256];
    struct {
      u64 xdst[kPW][kTaskRecs][kMaxRemote];  // replication: each record's outbox address per remote slot
      u32 xn[kPW][kTaskRecs];                // and how many
    };
  };
};

constexpr size_t kSmemBytes = sizeof(Stage1Smem) > sizeof(Stage3Smem) ? sizeof(Stage1Smem) : sizeof(Stage3Smem);
static_assert(kSmemBytes >= kMaxTiles * sizeof(u64), "stage 2's tile bases fit the dynamic LDS");

__device__ __forceinline__ u64 wave_incl_scan_u64(u64 v) { return wave_incl_scan<u64>(v); }

__device__ __forceinline__ u32 record_rs16(u32 L) {  // (16 + align16(L)) / 16 without overflow
  return (L >> 4) + ((L & 15u) ? 1u : 0u) + 1u;
}

// Batch of a group tile / stage-3 task, and the tile after the last one of a tile's batch
// (kernel-argument lookups over <= kMaxGroup entries).
__device__ __forceinline__ u32 batch_of_tile(const PipeGroup& G, u32 t) {
  u32 j = 0;
#pragma unroll
  for (u32 k = 1; k < kMaxGroup; ++k) j += (k < G.nb && t >= G.tile0[k]) ? 1u : 0u;
  return j;
}
__device__ __forceinline__ u32 batch_of_task(const PipeGroup& G, u32 task) {
  u32 j = 0;
#pragma unroll
  for (u32 k = 1; k < kMaxGroup; ++k) j += (k < G.nb && task >= G.task0[k]) ? 1u : 0u;
  return j;
}
__device__ __forceinline__ u32 batch_end_tile(const PipeGroup& G, u32 t) {
  u32 e = G.tiles;
#pragma unroll
  for (int k = (int)kMaxGroup - 1; k >= 1; --k)
    if ((u32)k < G.nb && t < G.tile0[k]) e = G.tile0[k];
  return e;
}

// Records longer than kBigPieces payload pieces are stored by the whole wave, one after another
// (lane l takes pieces l, l + 64, ...; kBU pieces per lane in flight): the lane-pair path would
// keep its wave for m / 8 rounds while the other 31 pairs idle.
constexpr u32 kBigPieces = 64;
constexpr u32 kBU = 4;

__device__ __forceinline__ u64 readlane64(u64 v, u32 l) {
  return ((u64)(u32)__builtin_amdgcn_readlane((int)(v >> 32), (int)l) << 32) |
         (u32)__builtin_amdgcn_readlane((int)(u32)v, (int)l);
}
__device__ __forceinline__ u32 readlane32(u32 v, u32 l) { return (u32)__builtin_amdgcn_readlane((int)v, (int)l); }

// The rank of block b among the blocks [b0, b0 + n) (b inside it) when the blocks that share an XCD
// (b and b + 8 under round-robin placement; speed only, never correctness) take one contiguous run
// of ranks, XCD after XCD: neighbouring work items then share one L2.
__device__ __forceinline__ u32 xcd_rank(u32 b0, u32 n, u32 b) {
  const auto below = [](u32 m, u32 y) { return m > y ? (m - y + 7u) >> 3 : 0u; };  // k < m, k % 8 == y
  const u32 x = b & 7u;
  u32 r = below(b, x) - below(b0, x);
  for (u32 y = 0; y < x; ++y) r += below(b0 + n, y) - below(b0, y);
  return r;
}

// ------------------------------------------------------------------------------------------
// Stage 1: rank one tile
// ------------------------------------------------------------------------------------------
// A present (tile, partition) run's cell {count << 40 | bytes/16}: packed into the u32 column that
// stage 2 reads, or, for a run of more than kCellB16 16-byte units, kCellWide there and the value in
// the u64 cell at the same index.
__device__ __forceinline__ void put_cell(const PipeScratch& x, u64 at, u64 v) {
  const u64 b16 = v & kLow40;
  u32 c = ((u32)(v >> 40) << kCellCntShift) | (u32)b16;
  if (b16 > kCellB16) {
    x.hist[at] = v;
    c = kCellWide;
  }
  x.hist32[at] = c;
}

// srow: the stamp row of the tile (diagnostics): its dedicated stage-1 workgroup's, also when a
// stage-3 workgroup ranks it
__device__ __forceinline__ void stage1_tile(const PipeArgs& A, u32 t, Stage1Smem& S, u32 srow) {
  const PipeGroup& G = A.g1;
  const u32 jb = batch_of_tile(G, t);
  const PipeBatch& b = G.b[jb];
  const PipeScratch& x = A.s1;
  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const u32 base = (t - G.tile0[jb]) * kTR;  // first record of the tile inside its batch
  const u64 gbase = (u64)t * kTR;            // its slot in the group's per-record scratch
  const u32 P = A.st.P;
  const u64 lt = (1ull << lane) - 1ull;
  const u32 nin = b.n - base < kTR ? b.n - base : kTR;
  PIPE_STAMP_ROW(srow, 0);

  // ---- loads (input position q = 128w + 64r + lane)
  u32 item[kTI], lenv[kTI], fl[kTI];
  u32 pc[kTI];
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const u32 q = w * kWR + r * 64u + lane;
    const bool in = q < nin;
    const u32 p = in ? b.pidx[base + q] : 0u;
    lenv[r] = in ? b.len[base + q] : 0u;
    const bool bad = in && p >= P;
    pc[r] = (in && !bad) ? p : 0u;
    fl[r] = !in ? kFlJunk : bad ? kFlNoPart : 0u;
  }
  u64 inv_cnt = 0;
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const u32 q = w * kWR + r * 64u + lane;
    if (fl[r] != kFlJunk && b.poff) {  // explicit payload offsets: per-record range check
      const u64 o = b.poff[base + q];
      const u32 L = lenv[r];
      if (L && (o > b.payload_bytes || (u64)L > b.payload_bytes - o)) {
        inv_cnt += 1;
        if (fl[r] == 0u) fl[r] = kFlInvalid;
      }
    }
    const u32 rs16 = fl[r] == kFlJunk ? 0u : record_rs16(lenv[r]);
    S.info[q] = rs16 | (fl[r] << kFlagShift);
    item[r] = (pc[r] << kIB) | q;
    // records over 1 KB go to stage 3's large-record waves (kBigPieces)
    const bool bigr = fl[r] == 0u && lenv[r] > 16u * kBigPieces;
    const u64 bm = __ballot(bigr);
    if (bm) {
      u32 at = 0;
      if (lane == 0) at = atomicAdd(x.nbig, (u32)__popcll(bm));
      at = readlane32(at, 0) + (u32)__popcll(bm & lt);
      if (bigr) x.bigl[at] = (u32)(gbase + q);
    }
  }

  // ---- input-order scans: payload prefix per record, tile sums {payload, invalid ranges}
  {
    u64 carry = 0;
    u32 pre_r[kTI];
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) {
      const u64 v = lenv[r];
      const u64 inc = wave_incl_scan_u64(v);
      pre_r[r] = (u32)(carry + inc - v);
      carry += bcast_u64(inc, 63);
    }
    inv_cnt = bcast_u64(wave_incl_scan(inv_cnt), 63);  // (the wave's sum)
    if (lane == 0) {
      S.wsum[w][0] = carry;
      S.wsum[w][1] = inv_cnt;
    }
    __syncthreads();
    u64 wpre = 0;
#pragma unroll
    for (u32 ww = 0; ww < kPW; ++ww) wpre += ww < w ? S.wsum[ww][0] : 0ull;
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) {
      const u32 q = w * kWR + r * 64u + lane;
      if (q < nin) x.pre[gbase + q] = (u32)wpre + pre_r[r];
    }
    if (tid == 0) {
      u64 ps = 0, ic = 0;
      for (u32 ww = 0; ww < kPW; ++ww) {
        ps += S.wsum[ww][0];
        ic += S.wsum[ww][1];
      }
      x.tsum[(u64)t * 4 + 0] = ps;
      x.tsum[(u64)t * 4 + 1] = 0;
      x.tsum[(u64)t * 4 + 2] = ic;
      x.tsum[(u64)t * 4 + 3] = 0;
      // the batch's sums for stage 2's batch rule (one add per tile instead of a pass over the
      // tile sums in every stage-2 workgroup)
      if (ps) __hip_atomic_fetch_add(&x.bacc[jb * 2 + 0], ps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ic) __hip_atomic_fetch_add(&x.bacc[jb * 2 + 1], ic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  PIPE_STAMP_ROW(srow, 1);
  // ---- stable LDS radix sort of the tile by partition id, 8-bit digits
  u32 buf = 0;
  for (u32 pass = 0; pass < A.key_passes; ++pass) {
    const u32 sh = kIB + 8u * pass;
#pragma unroll
    for (u32 k = 0; k < 4; ++k) S.cnt[w][lane + 64u * k] = 0u;
    __builtin_amdgcn_wave_barrier();
    u32 rk[kTI];
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) {
      const u32 d = (item[r] >> sh) & 0xFFu;
      u64 peers = ~0ull;
#pragma unroll
      for (u32 bb = 0; bb < 8; ++bb) {
        const bool bit = (d >> bb) & 1u;
        const u64 m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      const u32 c = S.cnt[w][d];
      const u64 below = peers & lt;
      rk[r] = c + (u32)__popcll(below);
      __builtin_amdgcn_wave_barrier();
      if (below == 0ull) S.cnt[w][d] = c + (u32)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (tid < 256) {
      u32 run = 0;
#pragma unroll
      for (u32 ww = 0; ww < kPW; ++ww) {
        const u32 c = S.cnt[ww][tid];
        S.cnt[ww][tid] = run;
        run += c;
      }
      const u32 inc = wave_incl_scan(run);
      if (lane == 63) S.scan[w] = inc;
      S.dbase[tid] = inc - run;
    }
    __syncthreads();
    if (tid < 256) {
      u32 add = 0;
      for (u32 ww = 0; ww < w; ++ww) add += S.scan[ww];
      S.dbase[tid] += add;
    }
    __syncthreads();
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) {
      const u32 d = (item[r] >> sh) & 0xFFu;
      S.items[buf][S.dbase[d] + S.cnt[w][d] + rk[r]] = item[r];
    }
    __syncthreads();
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) item[r] = S.items[buf][w * kWR + r * 64u + lane];
    buf ^= 1u;
  }
  if (A.key_passes == 0) {  // single partition: input order is already sorted
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) S.items[buf][w * kWR + r * 64u + lane] = item[r];
    __syncthreads();
    buf ^= 1u;
  }
  const u32* sorted = S.items[buf ^ 1u];
  PIPE_STAMP_ROW(srow, 2);

  // ---- segmented scan of {1, rs16} over the sorted tile (segments = partitions)
  u64 val[kTI], inc[kTI];
  u32 hb[kTI];
  u64 carry = 0;
  u32 any_head = 0;
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const u32 s = w * kWR + r * 64u + lane;
    const u32 key = item[r] >> kIB, q = item[r] & (kTR - 1u);
    const u32 info = S.info[q];
    const u32 f = info >> kFlagShift;
    val[r] = f == 0u ? (kOne40 | (info & kRankMask)) : 0ull;
    const u32 pkey = s ? (sorted[s - 1] >> kIB) : 0xFFFFFFFFu;
    u32 head = pkey != key ? 1u : 0u;
    u64 v = val[r];
    wave_seg_incl_scan(head, v);
    if (!head) v += carry;
    carry = bcast_u64(v, 63);
    hb[r] = head | any_head;
    any_head |= __ballot(head) ? 1u : 0u;
    inc[r] = v;
  }
  if (lane == 63) {
    S.wtail[w] = carry;
    S.whead[w] = any_head;
  }
  __syncthreads();
  u64 cin = 0;
  for (int ww = (int)w - 1; ww >= 0; --ww) {
    cin += S.wtail[ww];
    if (S.whead[ww]) break;
  }
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const u32 s = w * kWR + r * 64u + lane;
    const u32 key = item[r] >> kIB, q = item[r] & (kTR - 1u);
    const u64 v = inc[r] + (hb[r] ? 0ull : cin);
    const u32 f = S.info[q] >> kFlagShift;
    if (q < nin) {
      const u64 ex = v - val[r];
      x.crank[gbase + q] = make_uint2((u32)(ex >> 40) | (f << kFlagShift), (u32)(ex & kLow40));
    }
    const u32 nkey = s + 1 < kTR ? (sorted[s + 1] >> kIB) : 0xFFFFFFFFu;
    if (nkey != key && (v >> 40)) put_cell(x, (u64)key * A.gt + t, v);
  }
  if (A.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PIPE_STAMP_ROW(srow, 3);
}

// ------------------------------------------------------------------------------------------
// Stage 1 without a sort (RMQ_RANK=1): wave-ordered partition counters in an LDS hash table
// ------------------------------------------------------------------------------------------
// A record's place inside its (tile, partition) run is the number (and record bytes) of the tile's
// earlier records of its partition. Each 64-record slot of a wave finds its peers (same partition)
// by ballots over the key bits, and the count / bytes of the peers below each lane by popcounts over
// ballots of the size bits; one leader per key then reads the partition's counter in the table (the
// tile's records of that partition in earlier slots) and adds the slot's own. The slots are served
// in input order (a wave's four in program order, the waves one after another), so the ranks are
// the stable ranks the sort gave, with no sort, no segmented scan and three barriers fewer.
constexpr u32 kHT = 2048;  // hash slots: at least twice the records of a tile
static_assert(kHT >= 2 * kTR, "hash table load factor");
struct Stage1HSmem {
  u32 key[kHT];     // partition + 1 (0: empty)
  u64 val[kHT];     // count << 40 | bytes/16 of the partition's records so far in the tile
  u64 wsum[kPW][2];
};
static_assert(sizeof(Stage1HSmem) <= kSmemBytes, "stage 1's hash table fits the launch's LDS");

__device__ __forceinline__ u32 wave_or_all(u32 v) {
  v |= dpp_mov<0x111, 0xf>(v);
  v |= dpp_mov<0x112, 0xf>(v);
  v |= dpp_mov<0x114, 0xf>(v);
  v |= dpp_mov<0x118, 0xf>(v);
  v |= dpp_mov<0x142, 0xa>(v);
  v |= dpp_mov<0x143, 0xc>(v);
  return (u32)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ void stage1_tile_hash(const PipeArgs& A, u32 t, Stage1HSmem& S, u32 srow) {
  const PipeGroup& G = A.g1;
  const u32 jb = batch_of_tile(G, t);
  const PipeBatch& b = G.b[jb];
  const PipeScratch& x = A.s1;
  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const u32 base = (t - G.tile0[jb]) * kTR;
  const u64 gbase = (u64)t * kTR;
  const u32 P = A.st.P;
  const u64 lt = (1ull << lane) - 1ull;
  const u32 nin = b.n - base < kTR ? b.n - base : kTR;
  PIPE_STAMP_ROW(srow, 0);
  for (u32 k = tid; k < kHT; k += kPT) S.key[k] = 0u;  // (ordered by the barrier of the scans below)

  // ---- loads (input position q = kWR w + 64 r + lane)
  u32 key[kTI], lenv[kTI], fl[kTI];
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const u32 q = w * kWR + r * 64u + lane;
    const bool in = q < nin;
    const u32 p = in ? b.pidx[base + q] : 0u;
    lenv[r] = in ? b.len[base + q] : 0u;
    const bool bad = in && p >= P;
    key[r] = (in && !bad) ? p : 0u;
    fl[r] = !in ? kFlJunk : bad ? kFlNoPart : 0u;
  }
  u64 inv_cnt = 0;
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const u32 q = w * kWR + r * 64u + lane;
    if (fl[r] != kFlJunk && b.poff) {  // explicit payload offsets: per-record range check
      const u64 o = b.poff[base + q];
      const u32 L = lenv[r];
      if (L && (o > b.payload_bytes || (u64)L > b.payload_bytes - o)) {
        inv_cnt += 1;
        if (fl[r] == 0u) fl[r] = kFlInvalid;
      }
    }
    const bool bigr = fl[r] == 0u && lenv[r] > 16u * kBigPieces;  // stage 3's large-record waves
    const u64 bm = __ballot(bigr);
    if (bm) {
      u32 at = 0;
      if (lane == 0) at = atomicAdd(x.nbig, (u32)__popcll(bm));
      at = readlane32(at, 0) + (u32)__popcll(bm & lt);
      if (bigr) x.bigl[at] = (u32)(gbase + q);
    }
  }
  // ---- input-order scans: payload prefix per record, tile sums {payload, invalid ranges}
  {
    u64 carry = 0;
    u32 pre_r[kTI];
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) {
      const u64 v = lenv[r];
      const u64 inc = wave_incl_scan_u64(v);
      pre_r[r] = (u32)(carry + inc - v);
      carry += bcast_u64(inc, 63);
    }
    inv_cnt = bcast_u64(wave_incl_scan(inv_cnt), 63);
    if (lane == 0) {
      S.wsum[w][0] = carry;
      S.wsum[w][1] = inv_cnt;
    }
    __syncthreads();
    u64 wpre = 0;
#pragma unroll
    for (u32 ww = 0; ww < kPW; ++ww) wpre += ww < w ? S.wsum[ww][0] : 0ull;
#pragma unroll
    for (u32 r = 0; r < kTI; ++r) {
      const u32 q = w * kWR + r * 64u + lane;
      if (q < nin) x.pre[gbase + q] = (u32)wpre + pre_r[r];
    }
    if (tid == 0) {
      u64 ps = 0, ic = 0;
      for (u32 ww = 0; ww < kPW; ++ww) {
        ps += S.wsum[ww][0];
        ic += S.wsum[ww][1];
      }
      x.tsum[(u64)t * 4 + 0] = ps;
      x.tsum[(u64)t * 4 + 1] = 0;
      x.tsum[(u64)t * 4 + 2] = ic;
      x.tsum[(u64)t * 4 + 3] = 0;
      if (ps) __hip_atomic_fetch_add(&x.bacc[jb * 2 + 0], ps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ic) __hip_atomic_fetch_add(&x.bacc[jb * 2 + 1], ic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  PIPE_STAMP_ROW(srow, 1);

  // ---- per slot, in registers: peers (same partition), the count and bytes/16 of the peers
  // below the lane, and the slot's total of the lane's partition
  u64 peers[kTI];
  u32 wr[kTI], wb[kTI];
  u64 stot[kTI];
  const u32 kbits = A.key_bits;
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const bool valid = fl[r] == 0u;
    u64 pm = __ballot(valid);
    for (u32 bb = 0; bb < kbits; ++bb) {
      const bool bit = (key[r] >> bb) & 1u;
      const u64 m = __ballot(bit);
      pm &= bit ? m : ~m;
    }
    pm = valid ? pm : 0ull;
    const u64 below = pm & lt;
    const u32 rs = valid ? record_rs16(lenv[r]) : 0u;
    const u32 orv = wave_or_all(rs);
    const u32 rbits = orv ? 32u - (u32)__builtin_clz(orv) : 0u;
    u32 bsum = 0, btot = 0;
    for (u32 bb = 0; bb < rbits; ++bb) {
      const u64 m = __ballot((rs >> bb) & 1u);
      bsum += (u32)__popcll(m & below) << bb;
      btot += (u32)__popcll(m & pm) << bb;
    }
    peers[r] = pm;
    wr[r] = (u32)__popcll(below);
    wb[r] = bsum;
    stot[r] = ((u64)__popcll(pm) << 40) | btot;
  }
  PIPE_STAMP_ROW(srow, 2);

  // ---- the partitions' counters, slot after slot in input order (wave after wave)
  u64 before[kTI];
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) before[r] = 0ull;
  for (u32 ww = 0; ww < kPW; ++ww) {
    if (w == ww) {
#pragma unroll
      for (u32 r = 0; r < kTI; ++r) {
        const u64 pm = peers[r];
        u64 c = 0;
        if (pm && !(pm & lt)) {  // the lowest lane of its partition in the slot
          const u32 kv = key[r] + 1u;
          u32 h = (kv * 2654435761u) >> (32u - 11u);
          for (;;) {
            const u32 k0 = S.key[h];
            if (k0 == kv) break;
            if (k0 == 0u) {
              const u32 old = atomicCAS(&S.key[h], 0u, kv);
              if (old == 0u) {
                S.val[h] = 0ull;
                break;
              }
              if (old == kv) break;
            }
            h = (h + 1u) & (kHT - 1u);
          }
          c = S.val[h];
          S.val[h] = c + stot[r];
        }
        const u32 ll = pm ? (u32)__builtin_ctzll(pm) : lane;  // the partition's leader in the slot
        const u32 lo = (u32)__shfl((int)(u32)c, (int)ll, 64), hi = (u32)__shfl((int)(u32)(c >> 32), (int)ll, 64);
        before[r] = ((u64)hi << 32) | lo;
      }
    }
    __syncthreads();
  }
  PIPE_STAMP_ROW(srow, 3);
#pragma unroll
  for (u32 r = 0; r < kTI; ++r) {
    const u32 q = w * kWR + r * 64u + lane;
    if (q < nin)
      x.crank[gbase + q] = make_uint2(((u32)(before[r] >> 40) + wr[r]) | (fl[r] << kFlagShift),
                                      (u32)(before[r] & kLow40) + wb[r]);
  }
  // ---- the tile's aggregate of every present partition (the sparse hist cells)
  for (u32 k = tid; k < kHT; k += kPT) {
    const u32 kv = S.key[k];
    if (kv) put_cell(x, (u64)(kv - 1u) * A.gt + t, S.val[k]);
  }
  if (A.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PIPE_STAMP_ROW(srow, 4);
}

// ------------------------------------------------------------------------------------------
// Stage 2: batch rules, column scans over the group's tiles, tile payload bases
// ------------------------------------------------------------------------------------------

// Block-wide inclusive scan of one u64 per thread (kPT threads); *total gets the block sum.
__device__ __forceinline__ u64 block_incl_scan_u64(u64 v, u64* s_w, u64* total) {
  const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const u64 inc = wave_incl_scan_u64(v);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  u64 pre = 0, tot = 0;
#pragma unroll
  for (u32 k = 0; k < kPW; ++k) {
    pre += k < w ? s_w[k] : 0ull;
    tot += s_w[k];
  }
  __syncthreads();
  *total = tot;
  return pre + inc;
}

// Catch-up decision of out entry e of the group being planned (FORMAT.md §9 v3), by the stage-2
// thread of its partition's column once the group's totals of p are known (`tot`). B = the leader's
// log end before the round: the state this launch's stage 3 reads (after the group two before)
// plus the totals of the group it applies (the group before), E = B + the round.
__device__ __forceinline__ void plan_decide(const PipeArgs& A, u32 p, u32 e, u64 tot) {
  const XPlanArgs& X = A.xp2;
  const DevState& st = A.st;
  const u64 t3 = A.g3.nb ? A.s3.totals[p] : 0ull;
  const u64 Boff = A.cur.leo[p] + (t3 >> 40), Bpos = A.cur.used[p] + 16ull * (t3 & kLow40);
  const u64 Epos = Bpos + 16ull * (tot & kLow40);
  const u64 S = 1ull << (st.ring[p] & 63ull);
  // index entries complete when the round is planned: up to C = B less the group before (whether
  // that group is applied by this launch or was by an earlier one: FORMAT.md §9)
  const u64 Cpos = A.g3.nb ? A.cur.used[p] : Bpos - 16ull * A.lastg[p];
  XDecision d;
  d.f_off = X.xnext[2 * e];
  d.f_pos = X.xnext[2 * e + 1];
  d.gap = 0;
  d.r_off = d.r_pos = 0;
  d.flags = 0;
  d.pad = 0;
  const u64 cu = X.xcu[e];
  u64 r1 = X.xreq[4 * e + 2], roff = X.xreq[4 * e], rpos = X.xreq[4 * e + 1];
  if (X.ackin && (X.ackin[2 * e] & kAckRefused)) {  // a refusal among this launch's acks
    r1 = X.acks_round + 1ull;
    roff = X.ackin[2 * e] & kAckLeoMask;
    rpos = X.ackin[2 * e + 1];
    if (X.acks_round >= cu) {
      d.flags |= kDecNewReq;
      d.r_off = roff;
      d.r_pos = rpos;
    }
  }
  if (r1 && r1 - 1ull >= cu) {
    d.f_off = roff;
    d.f_pos = rpos;
    d.flags |= kDecReq | kDecRow;
  }
  if (st.cdirty[p]) d.flags |= kDecRow;
  // the row version the entry carries if it carries a row (a general plan stores the final word)
  X.rowv[e] = (d.flags & kDecRow) ? st.cver[p] : 0ull;
  if (d.f_off >= Boff) {
    d.f_off = Boff;
    d.f_pos = Bpos;
  } else if (d.f_pos + S < Epos) {
    // the ring no longer holds [F, E) after the round: the follower's log restarts at the rebase
    // point R = E[m], m = ceil((E.pos - S) / I), when that entry is complete (else detached)
    const u32 ilog = st.interval_log2;
    const u64 m = (Epos - S + (1ull << ilog) - 1ull) >> ilog;
    if ((m << ilog) > Cpos) {
      d.flags |= kDecDetached;
    } else {
      const RingRef rg = ring_ref(st, p);
      const u64* ie = st.index + (rg.ibase + m % rg.icap) * 2;
      d.f_off = ie[0];
      d.f_pos = ie[1];
      d.flags |= kDecGapped | kDecRebase;
      d.gap = Bpos - d.f_pos;
    }
  } else {
    d.flags |= kDecGapped;
    d.gap = Bpos - d.f_pos;
  }
  store_sc1(&X.xdec[e].f_off, d.f_off);
  store_sc1(&X.xdec[e].f_pos, d.f_pos);
  store_sc1(&X.xdec[e].gap, d.gap);
  store_sc1(&X.xdec[e].r_off, d.r_off);
  store_sc1(&X.xdec[e].r_pos, d.r_pos);
  store_sc1(reinterpret_cast<u64*>(&X.xdec[e].flags), (u64)d.flags);
  u32 q = 0;
  for (u32 k = 1; k < X.world; ++k) q += e >= X.xo_start[k] ? 1u : 0u;
  if (d.flags & (kDecRow | kDecGapped))
    __hip_atomic_fetch_or(&X.dflag[q], d.flags & (kDecRow | kDecGapped), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (d.flags & kDecDetached) atomicAdd((unsigned long long*)&X.counters[1], 1ull);
  // the entry's words as the steady-state plan has them (its round's records from B, FORMAT.md §9):
  // directory words 0, 1 and 3 and the next expected follower log end; the plan adds word 2 (the
  // slots and pieces before the entry) and the placement. Stored through (sc1): a general plan of
  // the destination stores every one of these words later in this launch, and its stores win.
  u64* dw = reinterpret_cast<u64*>(X.outbox + (u64)q * X.dcap + kRegionHdr + (u64)kDirEntry * (e - X.xo_start[q]));
  store_sc1(&X.xtot[e], tot);
  store_sc1(dw, (tot >> 40) | ((tot & kLow40) << 32));
  store_sc1(dw + 1, Boff);
  store_sc1(dw + 3, st.term[p]);
  store_sc1(dw + 4, X.csnap[p]);  // the leader's commit as the launch started (FORMAT.md §9 v4)
  store_sc1(dw + 5, st.term[p]);  // (v5) the entry reaches the leader's term start: its term
  store_sc1(&X.xnext[2 * e], Boff + (tot >> 40));
  store_sc1(&X.xnext[2 * e + 1], Bpos + 16ull * (tot & kLow40));
}

// End of a partial catch-up (FORMAT.md §9): the largest sparse-index entry E[m] with
// F.pos < E[m].pos <= lim among the entries complete now (m I <= used); 0 if none.
__device__ __forceinline__ bool partial_end(const DevState& st, u32 p, u64 fpos, u64 lim, u64 used, u64* xoff, u64* xpos) {
  const RingRef rg = ring_ref(st, p);
  const u32 ilog = st.interval_log2;
  u64 lo = (fpos >> ilog) + 1ull, hi = min(lim, used) >> ilog;  // candidates m in [lo, hi]
  bool found = false;
  while (lo <= hi) {  // E[m].pos rises with m
    const u64 mid = lo + (hi - lo) / 2;
    const u64* ie = st.index + (rg.ibase + mid % rg.icap) * 2;
    const u64 ep = ie[1];
    if (ep <= lim) {
      if (ep > fpos) {
        *xoff = ie[0];
        *xpos = ep;
        found = true;
      }
      lo = mid + 1;
    } else {
      if (!mid) break;
      hi = mid - 1;
    }
  }
  return found;
}

// Inputs of out entry e (partition p) to the plan: the group's totals and the stage-2 verdict of
// the entry (sc1: written by other workgroups of this launch), the leader's log end before the
// round (the state this launch's stage 3 reads plus the group it applies) and the group before's
// bytes. Every load is issued whatever e is (e clamped into the destination's list, p a valid
// partition): a path without them would make the compiler's counted wait for the prefetched entry
// a wait for all memory operations. The caller ignores the values of an entry past the list, and
// selects t3 / lastg by A.g3.nb where it uses them.
struct PlanIn {
  u64 tot, f_off, f_pos, gap, t3, leo, used, lastg, term;
  u32 p, fl;
};
__device__ __forceinline__ PlanIn plan_in(const PipeArgs& A, u32 e, u32 p) {
  const XPlanArgs& X = A.xp2;
  PlanIn v;
  v.p = p;
  v.tot = load_sc1(&A.s2.totals[p]);
  v.f_off = load_sc1(&X.xdec[e].f_off);
  v.f_pos = load_sc1(&X.xdec[e].f_pos);
  v.gap = load_sc1(&X.xdec[e].gap);
  v.fl = (u32)load_sc1(reinterpret_cast<const u64*>(&X.xdec[e].flags));
  v.t3 = (A.g3.nb ? A.s3.totals : A.cur.used)[p];
  v.leo = A.cur.leo[p];
  v.used = A.cur.used[p];
  v.lastg = A.lastg[p];
  v.term = A.st.term[p];
  return v;
}

// Steady-state plan of one destination (FORMAT.md §9 v3): no entry has a consumer-offset row or a
// catch-up gap (the destination's dflag is clear), so each entry carries its round's records only,
// from the leader's log end B; the stage-2 workers already stored its directory words 0, 1, 3 and
// next expected follower end (plan_decide). What is left needs the exclusive prefix of the round
// totals over the destination's entries (scan A of the general plan: va = the totals word): word 2
// and the stage-3 placement. Row k = entries e0 + k kPT + tid (at most kFK rows), every row's
// totals loaded at once, one block scan per row (s_f: kPW words), the entries' data pieces kept in
// LDS until the destination's record count fixes the data section. Returns the destination's
// totals word (records << 40 | 16-byte units), as the general plan's run_a.
constexpr u32 kFK = 16;
static_assert(kSmemBytes >= kPW * sizeof(u64) + sizeof(u32) * kFK * kPT, "the steady plan's LDS");
static_assert(sizeof(XEntry) == 32 && offsetof(XEntry, k) == 24 && offsetof(XEntry, data_start16) == 28,
              "plan_steady stores XEntry words");
// (diagnostic, RMQ_STAMPS: event i of the first destination's steady plan in wave i / 3's slot 5 + i % 3)
#define PLAN_STAMP(i)                                                                      \
  do {                                                                                     \
    if (stamp && threadIdx.x == 0)                                                         \
      A.stamps[((u64)blockIdx.x * kPW + (i) / 3) * 8 + 5 + (i) % 3] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
__device__ __forceinline__ u64 plan_steady(const PipeArgs& A, u32 e0, u32 e1, u64 base, u64 tab, u64* s_f, bool stamp) {
  const XPlanArgs& X = A.xp2;
  const u32 tid = threadIdx.x;
  const u32 el = e1 - 1u;
  u32* s_dk = reinterpret_cast<u32*>(s_f + kPW);  // the entries' data pieces before them
  PLAN_STAMP(0);
  u64 tk[kFK];
#pragma unroll
  for (u32 k = 0; k < kFK; ++k) tk[k] = load_sc1(&X.xtot[min(e0 + k * kPT + tid, el)]);
  u64 run = 0;
#pragma unroll
  for (u32 k = 0; k < kFK; ++k) {
    const u32 e = e0 + k * kPT + tid;
    if (k * kPT > el - e0) break;  // (uniform)
    const u64 t = e <= el ? tk[k] : 0ull;
    u64 tot;
    const u64 x = run + block_incl_scan_u64(t, s_f, &tot) - t;
    run += tot;
    if (k == 0) PLAN_STAMP(1);
    const u64 t_ex = x >> 40, d_ex = x & kLow40;
    if (e <= el) {
      s_dk[e - e0] = (u32)d_ex;  // (a region is far below 64 GiB)
      const u64 dir = base + kRegionHdr + (u64)kDirEntry * (e - e0);
      reinterpret_cast<u64*>(X.outbox + dir)[2] = t_ex | (d_ex << 32);
      u64* xe = reinterpret_cast<u64*>(&X.xe[e]);
      xe[1] = tab + 8ull * t_ex;
      xe[2] = dir;
      xe[3] = (u64)(e - e0) | (d_ex << 32);
    }
  }
  PLAN_STAMP(2);
  const u64 data = tab + ((8ull * (run >> 40) + 15ull) & ~15ull);
  for (u32 i = tid; i <= el - e0; i += kPT) X.xe[e0 + i].data_abs = data + 16ull * s_dk[i];  // (own writes)
  if (stamp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PLAN_STAMP(3);
  }
  __syncthreads();  // s_f / s_dk free for the next destination
  return run;
}

// The group's outbox layout (FORMAT.md §9 v3), one workgroup: destination d's region sits at
// d * dcap of the outbox (the host sends [d * dcap, d * dcap + size)):
//   [header 64 B][directory n_d x 32 B][record table N_d x 8 B, padded to 16][records][rows]
// with the entries (led partition, remote slot) in the destination's list order. Per entry: the
// catch-up verdict (gap granted in list order out of the destination's reserve), its records
// (the gap, then the round's own), where stage 3 puts the round's records and table slots, the
// catch-up list for the stage-3 launch's copy waves, the consumer-offset row, the next expected
// follower log end.
__device__ __forceinline__ void stage2_plan(const PipeArgs& A, u64* s_f) {
  const XPlanArgs& X = A.xp2;
  const DevState& st = A.st;
  const u32 tid = threadIdx.x, C = X.C;
  const u64 dcap = X.dcap;
  __shared__ u64 s_w[kPW];
  __shared__ u64 s_cu[2];  // catch-up entries and items before this destination
  if (tid == 0) s_cu[0] = s_cu[1] = 0ull;
  __syncthreads();
  for (u32 dd = 0; dd < X.world; ++dd) {
    const u32 e0 = X.xo_start[dd], e1 = X.xo_start[dd + 1];
    if (e0 == e1) {
      if (tid == 0) X.sizes[2 * dd] = X.sizes[2 * dd + 1] = 0ull;
      continue;
    }
    const u32 df = __hip_atomic_load(&X.dflag[dd], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u64 n = e1 - e0, base = (u64)dd * dcap;
    const u64 tab = base + kRegionHdr + kDirEntry * n;
    const bool first_dd = dd == X.rank + 1u - (X.rank + 1u == X.world ? X.world : 0u);
    u64 run_a = 0, run_b = 0;
    if (!df && n <= (u64)kFK * kPT) {
      run_a = plan_steady(A, e0, e1, base, tab, s_f, A.stamps && first_dd);
      if (A.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (first_dd) PIPE_STAMP(2);
      if (first_dd) PIPE_STAMP(3);
    } else {
      if (tid == 0) atomicAdd((unsigned long long*)&X.counters[2], 1ull);  // (rmq_repl_stats.general_plans)
      // pass 1: record counts (for the table size) need the grants, which need the gap prefix. The
      // inputs of the thread's next entry are loaded while this one is planned (and the partition of
      // the one after), so an iteration waits on barriers and scans, not on memory.
      u64 gap_run = 0;
      const u32 el = e1 - 1u;  // entries past the list load the last one's inputs (ignored)
      PlanIn cur = plan_in(A, min(e0 + tid, el), X.xo_p[min(e0 + tid, el)]);
      u32 p_next = X.xo_p[min(e0 + kPT + tid, el)];
      const bool st_dd = A.stamps && first_dd;
      for (u32 c0 = e0; c0 < e1; c0 += kPT) {
        const u32 e = c0 + tid;
        const bool in = e < e1;
        // (diagnostic: wave w stamps iteration w's start, scan A and end in its slots 5..7)
        const bool st_it = st_dd && (c0 - e0) / kPT == (tid >> 6);
        if (st_it) PIPE_STAMP(5);
        const PlanIn nxt = plan_in(A, min(e + kPT, el), p_next);
        p_next = X.xo_p[min(e + 2 * kPT, el)];
        const u32 p = cur.p, fl = cur.fl;
        const u64 tot = cur.tot, f_off = cur.f_off, f_pos = cur.f_pos, gap = in ? cur.gap : 0ull;
        u64 gex = 0;
        if (df & kDecGapped) {
          u64 gt;
          gex = gap_run + block_incl_scan_u64(gap, s_w, &gt) - gap;
          gap_run += gt;
        }
        // the entry's verdict: normal / full catch-up / partial / stopped (round records only)
        const u64 rcnt = tot >> 40, rb16 = tot & kLow40;
        u64 cnt = rcnt, b16 = rb16, gcnt = 0, gb16 = 0, first = f_off;
        u64 nx_off = 0, nx_pos = 0;
        bool with_round = true, set_cu = false, cu_entry = false;
        bool below_ts = false;  // a partial catch-up ending below the leader's term start (v5 word: 0)
        const u64 t3 = A.g3.nb ? cur.t3 : 0ull;
        const u64 Boff = in ? cur.leo + (t3 >> 40) : 0ull;
        const u64 Bpos = in ? cur.used + 16ull * (t3 & kLow40) : 0ull;
        const u64 Cpos = !in ? 0ull : A.g3.nb ? cur.used : Bpos - 16ull * cur.lastg;  // as plan_decide
        if (in) {
          nx_off = Boff + rcnt;
          nx_pos = Bpos + 16ull * rb16;
          set_cu = (fl & kDecReq) && !(fl & (kDecGapped | kDecDetached));
          if (fl & kDecGapped) {
            if (gex + gap <= X.reserve) {
              gcnt = Boff - f_off;
              gb16 = gap >> 4;
              cnt += gcnt;
              b16 += gb16;
              set_cu = cu_entry = true;
            } else if (gex <= X.reserve) {  // the first entry past the reserve: a prefix of its gap
              u64 xo = 0, xp = 0;
              if (partial_end(st, p, f_pos, f_pos + (X.reserve - gex), Cpos, &xo, &xp)) {
                gcnt = cnt = xo - f_off;
                gb16 = b16 = (xp - f_pos) >> 4;
                with_round = false;
                below_ts = xo < st.term_start[p];
                nx_off = xo;
                nx_pos = xp;
                set_cu = cu_entry = true;
              }
            }
          }
          if (!cu_entry) first = Boff;  // the round's records from B (refused by a follower behind B)
        }
        const bool row = in && (((fl & kDecRow) != 0u) || cu_entry);
        const bool rebase = cu_entry && (fl & kDecRebase);  // granted: the follower's log restarts at F
        // scan A: table slots and data pieces before the entry
        const u64 va = in ? (cnt << 40) | b16 : 0ull;
        u64 ta;
        const u64 exa = run_a + block_incl_scan_u64(va, s_w, &ta) - va;
        run_a += ta;
        if (st_it) PIPE_STAMP(6);
        // scan B: rows, catch-up entries and their copy items before the entry
        u64 items = 0;
        if (cu_entry) {
          const u32 ilog = st.interval_log2;
          items = ((f_pos + 16ull * gb16 - 1ull) >> ilog) - (f_pos >> ilog) + 1ull;
        }
        const u64 vb = (row ? 1ull : 0ull) | (cu_entry ? 1ull << 20 : 0ull) | (items << 40);
        u64 exb = 0;
        if (df) {
          u64 tb;
          exb = run_b + block_incl_scan_u64(vb, s_w, &tb) - vb;
          run_b += tb;
        }
        if (in) {
          const u32 k = e - e0;
          const u64 t_ex = exa >> 40, d_ex = exa & kLow40;
          const u64 dir = base + kRegionHdr + (u64)kDirEntry * k;
          uint4* de = reinterpret_cast<uint4*>(X.outbox + dir);
          de[0] = make_uint4((u32)cnt, (u32)b16, (u32)first, (u32)(first >> 32));
          const u64 term = cur.term | (rebase ? kTermRebase : 0ull);
          de[1] = make_uint4((u32)t_ex, (u32)d_ex, (u32)term, (u32)(term >> 32));
          // (loaded here, not with the entry's prefetched inputs: two more live registers per
          // prefetched entry pushed the transport kernel into 3.5 KB of scratch per lane)
          const u64 lcm = X.csnap[p];
          const u64 ltm = below_ts ? 0ull : cur.term;  // (v5) the term of the entry's last entry, as counted
          de[2] = make_uint4((u32)lcm, (u32)(lcm >> 32), (u32)ltm, (u32)(ltm >> 32));
          XEntry xe;
          xe.data_abs = kNoRound;
          xe.tab_abs = 0;
          if (with_round) {
            xe.data_abs = 0;  // data section offset, fixed below once the table size is known
            xe.tab_abs = tab + 8ull * (t_ex + gcnt);
          }
          xe.dir_abs = dir;
          xe.k = k;
          xe.data_start16 = (u32)(d_ex + gb16);
          X.xe[e] = xe;
          if (cu_entry) {
            const u32 ci = (u32)(s_cu[0] + ((exb >> 20) & 0xFFFFFull));
            XCatch xc;
            xc.pos = f_pos;
            xc.first = f_off;
            xc.bytes = 16ull * gb16;
            xc.data_abs = 0;  // fixed below
            xc.tab_abs = tab + 8ull * t_ex;
            xc.k = k;
            xc.data_start16 = (u32)d_ex;
            xc.p = p;
            xc.items0 = (u32)(s_cu[1] + (exb >> 40));
            xc.pad = 0;
            X.xc[ci] = xc;
            atomicAdd((unsigned long long*)&X.counters[0], 1ull);
          }
            // catch-up state (FORMAT.md §9): next expected follower log end, last catch-up round; a
          // request that came with this launch's acks and was not served stays pending
          X.xnext[2 * e] = nx_off;
          X.xnext[2 * e + 1] = nx_pos;
          if (set_cu) X.xcu[e] = X.round;
          if ((fl & kDecNewReq) && !set_cu) {
            X.xreq[4 * e] = load_sc1(&X.xdec[e].r_off);
            X.xreq[4 * e + 1] = load_sc1(&X.xdec[e].r_pos);
            X.xreq[4 * e + 2] = X.acks_round + 1ull;
          }
        }
        // (row entries and the data section offset need the region totals: pass 2)
        if (in) {
          X.xdec[e].pad = (row ? 1u + (u32)(exb & 0xFFFFFull) : 0u) | (rebase ? kRowRebase : 0u);  // row index + 1
          X.rowv[e] = row ? st.cver[p] : 0ull;  // (the version of the row pass 2 writes)
        }
        if (st_it) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          PIPE_STAMP(7);
        }
        cur = nxt;  // (the scans' own barriers order every reuse of s_w)
      }
      if (dd == X.rank + 1u - (X.rank + 1u == X.world ? X.world : 0u)) PIPE_STAMP(2);  // first destination: pass 1
      const u64 N = run_a >> 40, B16 = run_a & kLow40;
      const u64 data = tab + ((8ull * N + 15ull) & ~15ull), rows = data + 16ull * B16;
      const u64 rowb = 16ull + 8ull * C;
      // pass 2: data offsets, rows (the entries' words of eight iterations loaded at once); a row's
      // partition has its consumer offsets sent: its change flag is cleared
      constexpr u32 kP2 = 8;
      for (u32 e8 = e0 + tid; e8 < e1; e8 += kP2 * kPT) {
        u64 da[kP2];
        u32 ds[kP2], pad[kP2];
#pragma unroll
        for (u32 k = 0; k < kP2; ++k) {
          const u32 e = e8 + k * kPT;
          da[k] = kNoRound;
          ds[k] = pad[k] = 0u;
          if (e < e1) {
            da[k] = X.xe[e].data_abs;
            ds[k] = X.xe[e].data_start16;
            pad[k] = X.xdec[e].pad;
          }
        }
#pragma unroll
        for (u32 k = 0; k < kP2; ++k) {
          const u32 e = e8 + k * kPT;
          if (e >= e1) continue;
          if (da[k] != kNoRound) X.xe[e].data_abs = data + 16ull * ds[k];
          const u32 ri = pad[k] & ~kRowRebase;
          if (ri) {
            const u32 p = X.xo_p[e];
            uint8_t* rw = X.outbox + rows + rowb * (ri - 1u);
            // a rebase entry's row carries the rebase point's position (FORMAT.md §9)
            const u64 rp = (pad[k] & kRowRebase) ? load_sc1(&X.xdec[e].f_pos) : 0ull;
            *reinterpret_cast<uint4*>(rw) = make_uint4(e - e0, 0u, (u32)rp, (u32)(rp >> 32));
            for (u32 c = 0; c < C; ++c) reinterpret_cast<u64*>(rw + 16)[c] = st.cons[(u64)p * C + c];
            st.cdirty[p] = 0u;
          }
        }
      }
      if (dd == X.rank + 1u - (X.rank + 1u == X.world ? X.world : 0u)) PIPE_STAMP(3);  // and pass 2
    }
    const u64 N = run_a >> 40, M = run_b & 0xFFFFFull;
    const u64 data = tab + ((8ull * N + 15ull) & ~15ull), rows = data + 16ull * (run_a & kLow40);
    const u64 rowb = 16ull + 8ull * C;
    if (tid == 0) {
      u32* h = reinterpret_cast<u32*>(X.outbox + base);
      h[0] = kXMagic;
      h[1] = (u32)n;
      h[2] = (u32)N;
      h[3] = X.rank;
      *reinterpret_cast<u64*>(h + 4) = X.keysum[dd];
      *reinterpret_cast<u64*>(h + 6) = data - base;
      *reinterpret_cast<u64*>(h + 8) = rows - base;
      h[10] = (u32)M;
      h[11] = C;
      *reinterpret_cast<u64*>(h + 12) = X.round;
      *reinterpret_cast<u64*>(h + 14) = 0ull;
      if (N & 1ull) *reinterpret_cast<u64*>(X.outbox + tab + 8ull * N) = 0ull;  // table padding
      X.sizes[2 * dd] = rows + rowb * M - base;  // the exchange swaps {region bytes, records} per peer
      X.sizes[2 * dd + 1] = N;
      X.dflag[dd] = 0u;
      s_cu[0] += (run_b >> 20) & 0xFFFFFull;
      s_cu[1] += run_b >> 40;
    }
    __syncthreads();
    // catch-up list entries of this destination: their data start
    for (u32 i = tid; i < (u32)((run_b >> 20) & 0xFFFFFull); i += kPT) {
      XCatch& xc = X.xc[(u32)s_cu[0] - (u32)((run_b >> 20) & 0xFFFFFull) + i];
      xc.data_abs = data + 16ull * xc.data_start16;
    }
    __syncthreads();
  }
  __syncthreads();
  if (tid == 0) {
    X.xc_n[0] = (u32)s_cu[0];
    X.xc_n[1] = (u32)s_cu[1];
    __hip_atomic_store(X.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next used six launches later
  }
}

// s_ex: kMaxTiles words of the launch's dynamic LDS (static arrays would add to every role's LDS)
constexpr u32 kCL = 256 / kScanLanes;  // stage 2: tiles per thread per column chunk (chunks of 256 tiles)
static_assert(kScanLanes == 8 || kScanLanes == 16 || kScanLanes == 32, "stage 2 lane groups: 8, 16 or 32 lanes");
static_assert(kCL % 4 == 0, "stage 2 loads four u32 cells at a time");

// A packed tile cell as stage 2 scans it: {count << 40 | bytes/16} of one (tile, partition) run.
__device__ __forceinline__ u64 cell_value(u32 c) {
  return ((u64)(c >> kCellCntShift) << 40) | (c & kCellB16);
}

// Tiles [t, t + kCL) of a hist column: 16-byte loads of four u32 cells, the column stride (gt) being
// a multiple of four. A cell past the group's T tiles inside the column is zero (stage 1 writes the
// present cells of tiles below T, stage 2 clears what it reads), and no load passes the column.
__device__ __forceinline__ void load_column_chunk(const u32* col, u32 t, u32 T, u32 (&h)[kCL]) {
#pragma unroll
  for (u32 k = 0; k < kCL; k += 4) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t + k < T) v = *reinterpret_cast<const uint4*>(col + t + k);
    h[k] = v.x;
    h[k + 1] = v.y;
    h[k + 2] = v.z;
    h[k + 3] = v.w;
  }
}

__device__ __forceinline__ void load_column_group(const PipeScratch& x, u32 cg, u32 P, u32 GT, u32 s, u32 T,
                                                  u32 (&h)[kScanCols][kCL]) {
#pragma unroll
  for (u32 c = 0; c < kScanCols; ++c) {
    const u32 p = cg * kScanCols + c;
    if (p < P) load_column_chunk(x.hist32 + (u64)p * GT, kCL * s, T, h[c]);
  }
}

// Inclusive scan inside aligned groups of kScanLanes lanes: DPP row moves inside each row of 16
// (a lane below the shift inside its group takes nothing), and for 32-lane groups rows 1 / 3 take
// the last lane of rows 0 / 2 (row_bcast:15; the half-waves never mix).
__device__ __forceinline__ u64 lane_group_incl_scan(u64 v) {
  const u32 ls = lane_id() & (kScanLanes - 1u);
  u64 t = dpp_mov<0x111, 0xf>(v);
  v += ls >= 1u ? t : 0ull;
  t = dpp_mov<0x112, 0xf>(v);
  v += ls >= 2u ? t : 0ull;
  t = dpp_mov<0x114, 0xf>(v);
  v += ls >= 4u ? t : 0ull;
  if (kScanLanes > 8) {
    t = dpp_mov<0x118, 0xf>(v);
    v += ls >= 8u ? t : 0ull;
  }
  if (kScanLanes > 16) v += dpp_mov<0x142, 0xa>(v);
  return v;
}
// The last lane of the caller's lane group (every lane of the group gets it).
__device__ __forceinline__ u64 lane_group_last(u64 v) {
  const int src = (int)(lane_id() | (kScanLanes - 1u));
  return ((u64)(u32)__shfl((int)(v >> 32), src, 64) << 32) | (u32)__shfl((int)(u32)v, src, 64);
}

// FORMAT.md §3: partition p takes no record of batch j (tiles [t0, t1)). The same threads that wrote
// the batch's cells flag them (program order), absent cells included (stage 3 never reads those).
__device__ __forceinline__ void flag_no_space(u64* ecol, u32 s, u32 t0, u32 t1) {
  for (u32 B = t0 - t0 % (kScanLanes * kCL); B < t1; B += kScanLanes * kCL)
#pragma unroll
    for (u32 k = 0; k < kCL; ++k) {
      const u32 t = B + kCL * s + k;
      if (t >= t0 && t < t1) ecol[t] = kExclNoSpace;
    }
}

// Column p's batch scans when some cell of the wave's columns is kCellWide (a tile run of more than
// kCellB16 16-byte units, i.e. records averaging over 32 KB) or the group spans more than one chunk
// of kScanLanes * kCL tiles: the same scans as stage2_column, the cells read from memory one by one.
// Returns the group aggregate over accepted cells.
__device__ __attribute__((noinline)) u64 stage2_column_general(const PipeArgs& A, u32 p, u32 s, u32 rm) {
  const PipeGroup& G = A.g2;
  const PipeScratch& x = A.s2;
  const u32 P = A.st.P, T = G.tiles, GT = A.gt;
  const u64 lim16 = ((1ull << (A.st.ring[p] & 63ull)) - (1ull << A.st.interval_log2)) >> 4;
  u32* const col = x.hist32 + (u64)p * GT;
  const u64* const wcol = x.hist + (u64)p * GT;
  u64* const ecol = x.excl + (u64)p * GT;
  u64 carry = 0, bsum = 0;
  u32 j = 0;
  for (u32 C = 0; C < T; C += kScanLanes * kCL) {
    const u32 ta = C + kCL * s;
    for (; j < G.nb && G.tile0[j] < C + kScanLanes * kCL; ++j) {
      const u32 t0 = G.tile0[j], t1 = G.tile0[j + 1];
      const bool binv = (rm >> j) & 1u;
      const u32 a = ta > t0 ? ta : t0, b = min(min(ta + kCL, t1), T);
      u64 loc = 0;
      for (u32 t = a; t < b; ++t) {
        const u32 c = col[t];
        if (c) loc += c == kCellWide ? wcol[t] : cell_value(c);
      }
      if (binv) loc = 0;
      const u64 inc = lane_group_incl_scan(loc);
      u64 run = carry + bsum + inc - loc;
      for (u32 t = a; t < b; ++t) {
        const u32 c = col[t];
        if (c) {
          if (!binv) ecol[t] = run;
          if (!binv) run += c == kCellWide ? wcol[t] : cell_value(c);
          col[t] = 0u;
        }
      }
      bsum += lane_group_last(inc);
      if (t1 > C + kScanLanes * kCL) break;
      if (!binv) {
        if ((bsum & kLow40) > lim16) flag_no_space(ecol, s, t0, t1);
        else carry += bsum;
      }
      bsum = 0;
      if (s == 0) x.bcum[(u64)j * P + p] = carry;
    }
  }
  return carry;
}

// Column p of the group: per batch, the exclusive scan of the column over the batch's tiles (thread
// s holding tiles [kCL s, kCL s + kCL) of the group's first kScanLanes * kCL tiles, h, already
// loaded), the batches scanned from those registers one after another.
__device__ __forceinline__ void stage2_column(const PipeArgs& A, u32 p, u32 s, u32 rm, u32 (&h)[kCL]) {
  const PipeGroup& G = A.g2;
  const PipeScratch& x = A.s2;
  const u32 P = A.st.P, T = G.tiles, GT = A.gt;
  bool wide = T > kScanLanes * kCL;
#pragma unroll
  for (u32 k = 0; k < kCL; ++k) wide |= h[k] == kCellWide;
  u64 carry = 0;
  u32 j = 0;
  if (__any(wide)) {
    carry = stage2_column_general(A, p, s, rm);
    j = G.nb;
  } else {
    // record bytes / 16 one batch may add to p: its ring less one index interval (FORMAT.md §3)
    const u64 lim16 = ((1ull << (A.st.ring[p] & 63ull)) - (1ull << A.st.interval_log2)) >> 4;
    u32* const col = x.hist32 + (u64)p * GT;
    u64* const ecol = x.excl + (u64)p * GT;
    const u32 ta = kCL * s;
    for (; j < G.nb && G.tile0[j] < T; ++j) {
      const u32 t0 = G.tile0[j], t1 = G.tile0[j + 1];
      const bool binv = (rm >> j) & 1u;  // invalid batch: its cells are cleared and count nothing
      // the lane's cells of the batch: k in [klo, khi)
      const u32 klo = t0 > ta ? min(t0 - ta, kCL) : 0u, khi = t1 > ta ? min(t1 - ta, kCL) : 0u;
      u32 lc = 0, lb = 0;  // their count, bytes / 16
#pragma unroll
      for (u32 k = 0; k < kCL; ++k) {
        const u32 c = (k >= klo && k < khi) ? h[k] : 0u;
        lc += c >> kCellCntShift;
        lb += c & kCellB16;
      }
      const u64 loc = binv ? 0ull : ((u64)lc << 40) | lb;
      const u64 inc = lane_group_incl_scan(loc);
      u64 run = carry + inc - loc;
#pragma unroll
      for (u32 k = 0; k < kCL; ++k) {
        if (k >= klo && k < khi && h[k]) {
          if (!binv) ecol[ta + k] = run;
          run += cell_value(h[k]);
          col[ta + k] = 0u;  // clear for the set's next group
        }
      }
      const u64 bsum = lane_group_last(inc);
      if (!binv) {
        if ((bsum & kLow40) > lim16) flag_no_space(ecol, s, t0, t1);
        else carry += bsum;
      }
      if (s == 0) x.bcum[(u64)j * P + p] = carry;
    }
  }
  for (; j < G.nb; ++j)  // batches without tiles at the group's end
    if (s == 0) x.bcum[(u64)j * P + p] = carry;
  if (s == 0) store_sc1(&x.totals[p], carry);  // sc1: the plan below reads it in this launch
  if (s == 0) {
    // stage 3 of the group (next launch) reads p's words in one 64-byte line: the log end before the
    // group = the state this launch's stage 3 reads plus the group it applies (what the next launch's
    // stage 3 reads as its state set: plan_decide's B), the totals, the ring, leadership and replicas
    const u64 t3 = A.g3.nb ? A.s3.totals[p] : 0ull;
    uint4* pk = reinterpret_cast<uint4*>(x.pk + (u64)p * 8);
    const u64 boff = A.cur.leo[p] + (t3 >> 40), bpos = A.cur.used[p] + 16ull * (t3 & kLow40);
    const u64 rd = A.st.ring[p];
    const u32 fl = A.st.is_leader[p] | (A.st.local_mask[p] << 8);
    pk[0] = make_uint4((u32)boff, (u32)(boff >> 32), (u32)bpos, (u32)(bpos >> 32));
    pk[1] = make_uint4((u32)carry, (u32)(carry >> 32), (u32)rd, (u32)(rd >> 32));
    pk[2] = make_uint4(fl, 0u, 0u, 0u);
  }
  if (A.xp2.n_out && s == 0 && A.st.is_leader[p]) {  // catch-up verdicts of p's out entries
    const u32 lm = A.st.local_mask[p];
    for (u32 r = 0; r < A.st.RF; ++r) {
      const u32 e = ((lm >> r) & 1u) ? ~0u : A.outidx[(u64)p * A.st.RF + r];
      if (e != ~0u) plan_decide(A, p, e, carry);
    }
  }
}

template <bool XR>
__device__ __forceinline__ void stage2(const PipeArgs& A, u32 wg, u64* s_ex) {
  const PipeGroup& G = A.g2;
  const PipeScratch& x = A.s2;
  const u32 P = A.st.P, T = G.tiles, GT = A.gt;
  const u32 tid = threadIdx.x;
  __shared__ u64 s_acc[kMaxGroup][2];
  __shared__ u64 s_w[kPW];
  __shared__ u32 s_rej;
  PIPE_STAMP(0);
  // kScanLanes consecutive threads (a column group) scan kScanCols adjacent partition columns
  // (contiguous in hist / excl): the first chunk of each is loaded up front, in flight while the
  // batch rule is worked out (a workgroup's lifetime is a few memory round trips, so fewer
  // workgroups with more loads each hold fewer of the launch's slots)
  const u32 s = tid % kScanLanes;
  const u32 ncg = (P + kScanCols - 1) / kScanCols;
  const u32 cstride = A.wg2 * (kPT / kScanLanes);
  u32 cg = (wg * kPT + tid) / kScanLanes;
  u32 h[kScanCols][kCL];
  if (cg < ncg) load_column_group(x, cg, P, GT, s, T, h);
  // ---- batch rule from stage 1's per-batch sums (every workgroup, since the scans skip invalid
  // batches)
  if (tid < kMaxGroup * 2) (&s_acc[0][0])[tid] = tid < G.nb * 2 ? x.bacc[tid] : 0ull;
  if (wg == 0) {  // payload offset of every tile's first record in the group (packed payloads)
    u64 carry = 0;
    for (u32 t0 = 0; t0 < T; t0 += kPT) {  // tiles t = tid, tid + kPT, ... (at most kMaxTiles)
      const u32 t = t0 + tid;
      const u64 pay = t < T ? x.tsum[(u64)t * 4 + 0] : 0ull;
      u64 tot;
      const u64 inc = block_incl_scan_u64(pay, s_w, &tot);
      if (t < T) s_ex[t] = carry + inc - pay;
      carry += tot;
    }
    __syncthreads();  // ... and inside its batch
    for (u32 t = tid; t < T; t += kPT) x.tile_base[t] = s_ex[t] - s_ex[G.tile0[batch_of_tile(G, t)]];
  }
  __syncthreads();
  if (tid == 0) {
    u32 rm = 0;
    for (u32 j = 0; j < G.nb; ++j) {
      const u64 ptot = s_acc[j][0], itot = s_acc[j][1];
      const u32 rej = (itot || (!G.b[j].poff && ptot > G.b[j].payload_bytes)) ? kRejInvalid : 0u;
      rm |= (rej ? 1u : 0u) << j;
      if (wg == 0) {
        x.binfo[j * 4 + 0] = rej;
        x.binfo[j * 4 + 1] = 0;
        x.binfo[j * 4 + 2] = ptot;
        x.binfo[j * 4 + 3] = 0;
      }
    }
    s_rej = rm;
  }
  __syncthreads();
  const u32 rm = s_rej;
  for (; cg < ncg; cg += cstride) {
#pragma unroll
    for (u32 c = 0; c < kScanCols; ++c)
      if (cg * kScanCols + c < P) stage2_column(A, cg * kScanCols + c, s, rm, h[c]);
    if (cg + cstride < ncg) load_column_group(x, cg + cstride, P, GT, s, T, h);
  }
  if (A.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PIPE_STAMP(1);
  if (XR && A.xp2.n_out) {
    // replication transport: the last stage-2 workgroup to finish lays out the group's outbox
    // (every storing wave drained, then one counter add per workgroup; the last adder reads the
    // sc1-stored totals with sc1 loads: MI355X_MICROARCH.md inter-workgroup visibility, row 1)
    __shared__ u32 s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      s_last = __hip_atomic_fetch_add(A.xp2.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == A.wg2 - 1u;
    __syncthreads();
    if (s_last) stage2_plan(A, s_ex);  // (s_ex: the tile bases are written)
  }
  if (A.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PIPE_STAMP(4);
}

// ------------------------------------------------------------------------------------------
// Stage 3: apply
// ------------------------------------------------------------------------------------------

// Bytes [s, s + nb) of b0 || b1 as 4 little-endian dwords, zero-padded past nb. 64-bit funnel
// shifts with two-way selects (no dynamically indexed array, which would go to scratch).
__device__ __forceinline__ uint4 extract_piece(uint4 b0, uint4 b1, u32 s, u32 nb) {
  const u64 q0 = ((u64)b0.y << 32) | b0.x, q1 = ((u64)b0.w << 32) | b0.z;
  const u64 q2 = ((u64)b1.y << 32) | b1.x, q3 = ((u64)b1.w << 32) | b1.z;
  const bool h = s >= 8u;
  const u64 a0 = h ? q1 : q0, a1 = h ? q2 : q1, a2 = h ? q3 : q2;
  const u32 sh = (s & 7u) * 8u;
  u64 lo = sh ? (a0 >> sh) | (a1 << (64u - sh)) : a0;
  u64 hi = sh ? (a1 >> sh) | (a2 << (64u - sh)) : a1;
  if (nb < 16u) {
    if (nb <= 8u) {
      hi = 0;
      lo = nb == 8u ? lo : lo & ((1ull << (8u * nb)) - 1ull);
    } else {
      hi &= (1ull << (8u * (nb - 8u))) - 1ull;
    }
  }
  return make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32));
}


// Stage 3 works on tasks of kTaskRecs = 32 records of one batch, one per lane pair. The pair loads
// the record's payload as aligned 16-byte blocks (lane j takes blocks j, j + 2, ...; 8 pieces =
// up to 9 blocks per round) and each lane builds its pieces (j, j + 2, j + 4, j + 6 of the round)
// from its own block and its partner's (DPP swap); lane 1 writes the header once the pair's CRC
// registers are XOR-reduced.
constexpr u32 kPR = 8;          // pieces per record per round
constexpr u32 kBL = 5;          // blocks per lane per round (9 blocks cover 8 misaligned pieces)

__device__ __forceinline__ uint4 pair_swap4(uint4 v) {
  return make_uint4(pair_swap(v.x), pair_swap(v.y), pair_swap(v.z), pair_swap(v.w));
}

struct TaskRec {  // round 1: the record (the same words in both lanes of its pair)
  u32 p, L;
  uint2 cr;
  u64 src;        // payload address
};

// Where a task's records live: its batch in the group and the first record's index in the batch
// (the task index is wave-uniform, so all of this stays in scalar registers).
struct TaskPos {
  u32 jb, i0;
};
__device__ __forceinline__ TaskPos task_pos(const PipeGroup& G, u32 task) {
  const u32 jb = batch_of_task(G, task);
  return TaskPos{jb, (task - G.task0[jb]) * kTaskRecs};
}
__device__ __forceinline__ u32 task_rec(const TaskPos& T) { return T.i0 + ((threadIdx.x & 63) >> 1); }

// Round 2: where the record goes and its first round of payload blocks (derived from the
// partition's state as soon as it arrives, so that only these words stay live).
constexpr u32 kLead = 1u << 31;     // TaskState::lm: this engine leads the partition
constexpr u32 kNoSpace = 1u << 30;  // TaskState::lm: the (batch, partition) cell is over its limit
struct TaskState {
  u64 pos, off;    // logical position and offset of the record
  u64 rdesc;       // the partition's ring descriptor (DevState::ring)
  u32 lm;          // local replica mask | kLead | kNoSpace
  u32 dead;        // leading pieces (0 = header) a later piece of the group overwrites
  u32 rel16, rk;   // replication: 16-byte units and records into the partition's group run
  uint4 blk[kBL];  // the lane's first round of payload blocks, or (staged) blk[0..3] = the task's span
  u32 nblk;        // staged: 16-byte blocks of the task's payload span from base `sbase` (wave-uniform;
  u64 sbase;       //   0: not staged)
};

// A task's records are packed back to back in the batch payload (no payload_off: one tile, so one
// contiguous span): the wave loads the span's 16-byte blocks with coalesced loads (lane l: blocks
// l, l + 64, ...; about 2 L1->L2 requests per 128-byte record instead of one per 32 bytes a lane
// pair loads), through its LDS image area, and each lane pair reads its record's blocks from there.
constexpr u32 kSpanPer = 4;  // blocks per lane: spans of up to 4 KB (32 records of <= 112 B take 3.6 KB)
#ifndef RMQ_SPAN_AUX
#define RMQ_SPAN_AUX 2  // the span loads' cache policy: nt (read once per launch, like load_payload16)
#endif

// Record i of batch jb of the group in stage 3 (every lane: its own record, or its pair's).
__device__ __forceinline__ TaskRec stage3_r1_at(const PipeArgs& A, u32 jb, u32 i) {
  const PipeGroup& G = A.g3;
  const PipeScratch& x = A.s3;
  const PipeBatch& b = G.b[jb];
  TaskRec r;
  r.p = 0u;
  r.L = 0u;
  r.cr = make_uint2(kFlJunk << kFlagShift, 0u);
  r.src = reinterpret_cast<u64>(b.payload);
  if (i < b.n) {
    const u64 gi = (u64)G.tile0[jb] * kTR + i;  // group record slot
    r.p = b.pidx[i];
    r.L = b.len[i];
    r.cr = x.crank[gi];
    r.src += b.poff ? b.poff[i] : x.tile_base[gi / kTR] + x.pre[gi];
  }
  return r;
}
__device__ __forceinline__ TaskRec stage3_r1(const PipeArgs& A, const TaskPos& T) { return stage3_r1_at(A, T.jb, task_rec(T)); }

__device__ __forceinline__ u32 batch_rej(const PipeArgs& A, u32 jb) { return (u32)A.s3.binfo[jb * 4]; }
__device__ __forceinline__ u32 batch_rej(const PipeArgs& A, const TaskPos& T) { return batch_rej(A, T.jb); }

__device__ __forceinline__ bool stage3_cand_at(const PipeArgs& A, u32 jb, u32 i, const TaskRec& R) {
  return i < A.g3.b[jb].n && (R.cr.x >> kFlagShift) == 0u && batch_rej(A, jb) == 0u;
}
__device__ __forceinline__ bool stage3_cand(const PipeArgs& A, const TaskPos& T, const TaskRec& R) {
  return stage3_cand_at(A, T.jb, task_rec(T), R);
}

// Aligned payload blocks of round c held by lane j: block 8c + j + 2q, q < kBL, loaded only if
// it holds a byte of the record (never touches a page without one).
__device__ __forceinline__ void round_blocks(const PipeArgs& A, const TaskRec& R, u32 c, bool live, uint4 (&blk)[kBL]) {
  const u32 j = threadIdx.x & 1u;
  const u64 a0 = R.src & ~15ull;
  const u64 lim = R.src + R.L;  // one past the last byte
#pragma unroll
  for (u32 q = 0; q < kBL; ++q) {
    const u64 blk_addr = a0 + 16ull * (kPR * c + j + 2u * q);
    blk[q] = make_uint4(0, 0, 0, 0);
    if (live && blk_addr < lim && !(A.debug & 4u)) blk[q] = load_payload16(reinterpret_cast<const void*>(blk_addr));
  }
}

// The words of record i's partition state that place it (one round of gathers; lanes without a
// candidate record load nothing).
struct RecWords {
  u64 ex, tot, leo, used, rdesc;
  u32 lead, lm;
};
__device__ __forceinline__ RecWords rec_words(const PipeArgs& A, u32 jb, u32 i, u32 p, bool cand) {
  const DevState& st = A.st;
  RecWords W;
  W.ex = W.tot = W.leo = W.used = 0ull;
  W.rdesc = 8ull;  // any valid descriptor (a 256-byte ring at 0) for lanes that store nothing
  W.lead = W.lm = 0u;
  if (cand) {
    const u32 t = A.g3.tile0[jb] + i / kTR;
    W.ex = A.s3.excl[(u64)p * A.gt + t];
    // the partition's words in one 64-byte line (stage 2 wrote them): three 16-byte loads
    const uint4* pk = reinterpret_cast<const uint4*>(A.s3.pk + (u64)p * 8);
    const uint4 a = pk[0], b = pk[1], c = pk[2];
    W.leo = ((u64)a.y << 32) | a.x;
    W.used = ((u64)a.w << 32) | a.z;
    W.tot = ((u64)b.y << 32) | b.x;
    W.rdesc = ((u64)b.w << 32) | b.z;
    W.lead = c.x & 0xFFu;
    W.lm = c.x >> 8;
    (void)st;
  }
  return W;
}

// Offset and position of a candidate record, its leading dead pieces (0 = header, k = payload
// piece k - 1 at pos + 16k: a piece whose ring slot a later piece of the same group overwrites,
// pos + 16k + seg < group end, is not stored) and its mask word (local replicas | kLead | kNoSpace).
__device__ __forceinline__ void rec_place(const RecWords& W, const TaskRec& R, u64& pos, u64& off, u32& dead,
                                          u32& lmo, u32& rk, u32& rel16) {
  rk = (u32)((W.ex >> 40) & kCnt23) + (R.cr.x & kRankMask);
  rel16 = (u32)(W.ex & kLow40) + R.cr.y;
  off = W.leo + rk;
  pos = W.used + 16ull * rel16;
  const u64 seg = 1ull << (W.rdesc & 63ull), gend = W.used + 16ull * (W.tot & kLow40);
  dead = gend > pos + seg ? (u32)min((gend - seg - pos) >> 4, (u64)((R.L + 15u) >> 4) + 1ull) : 0u;
  lmo = W.lm | (W.lead ? kLead : 0u) | ((W.ex & kExclNoSpace) ? kNoSpace : 0u);
}

__device__ __forceinline__ TaskState stage3_r2(const PipeArgs& A, const TaskPos& T, const TaskRec& R, bool cand,
                                               bool stage = false, RecWords* defer = nullptr) {
  TaskState S;
  S.pos = S.off = 0ull;
  S.lm = S.dead = S.rel16 = S.rk = 0u;
  S.nblk = 0u;
  S.sbase = 0ull;
  const RecWords W = rec_words(A, T.jb, task_rec(T), R.p, cand);
  S.rdesc = W.rdesc;
  // first round of payload blocks, speculatively (leadership is checked before any store): the
  // task's whole span by coalesced loads when it is packed and fits, else the lane pair's blocks
  const PipeBatch& b = A.g3.b[T.jb];
  if (stage && !b.poff && T.i0 < b.n && !(A.debug & 4u)) {
    const u32 last = 2u * (min(kTaskRecs, b.n - T.i0) - 1u);  // lane of the task's last record
    const u64 s0 = readlane64(R.src, 0) & ~15ull;
    const u64 e1 = readlane64(R.src, last) + readlane32(R.L, last);
    const u64 nb = (e1 - s0 + 15ull) >> 4;
    if (nb <= 64ull * kSpanPer) {
      S.nblk = (u32)nb;  // (s0, e1: read lanes, wave-uniform)
      S.sbase = s0;
    }
  }
  if (S.nblk) {
    // buffer loads through a descriptor of the span (bounds-checked: blocks past it read 0), one
    // 32-bit offset for all four (the span base is wave-uniform)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(S.sbase), 0, (int)(16u * S.nblk), 0x00020000);
    const u32 vo = 16u * (threadIdx.x & 63u);
#pragma unroll
    for (u32 u = 0; u < kSpanPer; ++u) {
      const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 1024u * u, 0, RMQ_SPAN_AUX);
      S.blk[u] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    S.blk[kBL - 1] = make_uint4(0, 0, 0, 0);
  } else {
    round_blocks(A, R, 0u, cand, S.blk);
  }
  if (defer)
    *defer = W;  // placed by the caller (rec_place) after work that does not wait for these loads
  else if (cand)
    rec_place(W, R, S.pos, S.off, S.dead, S.lm, S.rk, S.rel16);
  return S;
}

// CRC register of one 16-byte piece of the record (piece 0 carries the CRC init); the caller
// folds a lane's pieces by Horner's rule with the 32-byte zero-shift table.
__device__ __forceinline__ u32 piece_crc(const PipeArgs& A, const Stage3Smem& S, uint4 v, u32 jp) {
  if (jp == 0) v.x ^= 0xFFFFFFFFu;  // CRC init folded into the first payload dword
  return (A.debug & 2u) ? v.x : crc_piece16(S.t8, v);
}

// One record over 1 KB, by the whole wave (wave-uniform arguments): lane l takes payload pieces
// l, l + 64, ... (kBU per lane in flight, the block after each from the neighbour lane), folds
// them by Horner's rule with the 1 KB shift table, shifts its register past the pieces that follow
// its last one and the wave XOR-reduces; lane 0 writes the header. xdst: the record's outbox copies.
// Round k0 of a large record's payload blocks: kBU per lane (blocks 64 (k0 + u) + lane - ph of the
// record's 16-byte-aligned span, none below 0) and the block after the round for lane 63. ph: the
// destination phase (big_record).
__device__ __forceinline__ void big_round(u64 src, u32 L, u32 k0, u32 ph, uint4 (&b0)[kBU], uint4& tail) {
  const u32 lane = threadIdx.x & 63, sa = (u32)(src & 15u);
  const u64 a0 = src & ~15ull, lim = src + L;
#pragma unroll
  for (u32 u = 0; u < kBU; ++u) {
    const int jb = (int)(64u * (k0 + u) + lane) - (int)ph;
    const u64 ad = a0 + 16ll * jb;
    b0[u] = jb >= 0 && ad < lim ? load_payload16(reinterpret_cast<const void*>(ad)) : make_uint4(0, 0, 0, 0);
  }
  tail = make_uint4(0, 0, 0, 0);
  const u64 ad = a0 + 16ull * (64u * (k0 + kBU) - ph);
  if (sa && lane == 63u && ad < lim) tail = load_payload16(reinterpret_cast<const void*>(ad));
}

// The destination phase of a large record at ring position pos: its payload pieces start at piece
// (pos >> 4) + 1 of the ring; lane l takes payload piece 64 u + l - ph, so every store instruction
// covers whole 128-byte lines of the ring (at 16-byte phases, 1 KB stores measured 20 % slower:
// tools/replica_bench, 3.80 vs 4.71 TB/s).
__device__ __forceinline__ u32 big_phase(u64 pos) { return (u32)((pos >> 4) + 1ull) & 7u; }

// A large record's wave-uniform place (broadcast from the lane that resolved it).
struct BigRec {
  u64 src, pos, off, ring, segm;
  u64 x[kMaxRemote];
  u32 L, dead, lm, nx, ph, m;
};

// Round k0 of a large record, its blocks b0 / tail loaded: CRC fold into acc and the stores.
__device__ __forceinline__ void big_store_round(const PipeArgs& A, const Stage3Smem& S, const u32 (*zk)[256],
                                                const BigRec& R, u32 k0, const uint4 (&b0)[kBU], uint4 tail, u32& acc) {
  const u32 lane = threadIdx.x & 63, RF = A.st.RF;
  const u64 rstride = A.st.rstride;
  const u32 sa = (u32)(R.src & 15u);
  uint8_t* ring = reinterpret_cast<uint8_t*>(R.ring);
#pragma unroll
  for (u32 u = 0; u < kBU; ++u) {
    const u32 jp = 64u * (k0 + u) + lane - R.ph;  // (wraps below 0: then past m, skipped)
    uint4 b1;
    b1.x = (u32)__shfl_down((int)b0[u].x, 1, 64);
    b1.y = (u32)__shfl_down((int)b0[u].y, 1, 64);
    b1.z = (u32)__shfl_down((int)b0[u].z, 1, 64);
    b1.w = (u32)__shfl_down((int)b0[u].w, 1, 64);
    if (lane == 63u) {
      const u32 un = u + 1 < kBU ? u + 1 : u;  // unrolled: a constant
      b1 = u + 1 < kBU ? make_uint4(readlane32(b0[un].x, 0), readlane32(b0[un].y, 0), readlane32(b0[un].z, 0),
                                    readlane32(b0[un].w, 0))
                       : tail;
    }
    if (jp < R.m) {
      const u32 nb = R.L - 16u * jp < 16u ? R.L - 16u * jp : 16u;
      const uint4 v = extract_piece(b0[u], b1, sa, nb);
      acc = crc_zshift(zk, acc) ^ piece_crc(A, S, v, jp);
      uint8_t* dst = ring + ((R.pos + 16ull + 16ull * jp) & R.segm);
      if (jp + 1u >= R.dead)
        for (u32 r = 0; r < RF; ++r)
          if ((R.lm >> r) & 1u) store_log16(dst + r * rstride, v);
#pragma unroll
      for (u32 q = 0; q < kMaxRemote; ++q)
        if (q < R.nx) store_log16(reinterpret_cast<uint8_t*>(R.x[q]) + 16ull + 16ull * jp, v);
    }
  }
}

// After a large record's last round: lane l's pieces are l - ph (mod 64) apart by 64 and e pieces
// follow its last one, so its register is shifted past them; the wave XOR-reduces and lane 0
// writes the header.
__device__ __forceinline__ void big_close(const PipeArgs& A, const BigRec& R, u32 acc) {
  const u32 lane = threadIdx.x & 63, RF = A.st.RF;
  if (((lane + 64u - R.ph) & 63u) < R.m) {
    const u32 e = (R.m - 1u - lane + R.ph) & 63u;
    if (e) acc = gf2_mulmod(acc, A.crc->sh16[e]);
  }
  acc = wave_xor_all(acc);
  if (lane == 0) {
    const u32 pad = 16u * R.m - R.L;
    const u32 crc = ~(pad ? gf2_mulmod(A.crc->inv_pad[pad], acc) : acc);
    const uint4 h = make_uint4((u32)R.off, (u32)(R.off >> 32), R.L, crc);
    uint8_t* ring = reinterpret_cast<uint8_t*>(R.ring);
    if (R.dead == 0u)
      for (u32 r = 0; r < RF; ++r)
        if ((R.lm >> r) & 1u) store_log16(ring + (R.pos & R.segm) + r * A.st.rstride, h);
#pragma unroll
    for (u32 q = 0; q < kMaxRemote; ++q)
      if (q < R.nx) store_log16(reinterpret_cast<uint8_t*>(R.x[q]), h);
  }
}

// Large-record waves of the stage-3 launch: wave g of G takes entries g, g + G, ... of the group's
// list of records over 1 KB (stage 1), re-derives each record's place like stage3_r1/r2 and stores
// it with big_record. Their task waves leave these records to them (header and payload; the task
// wave still writes the out offset, index entries, record-table slots and statistics).
template <bool XR>
__device__ __forceinline__ void stage3_big_waves(const PipeArgs& A, Stage3Smem& S, u32 wg) {
  const PipeGroup& G = A.g3;
  const PipeScratch& x = A.s3;
  const DevState& st = A.st;
  const u32 nbig = __builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile const u32*>(x.nbig));
  if (!nbig) return;  // no table copy either
  {
    const uint4* src = reinterpret_cast<const uint4*>(&A.crc->table[0][0]);
    uint4* dst = reinterpret_cast<uint4*>(&S.t8[0][0]);
    for (u32 k = threadIdx.x; k < (sizeof(S.t8) + sizeof(S.z)) / 16u; k += kPT) dst[k] = src[k];
    if (!XR) {
      const uint4* zs = reinterpret_cast<const uint4*>(&A.crc->zshift1k[0][0]);
      uint4* zd = reinterpret_cast<uint4*>(&S.zk[0][0]);
      for (u32 k = threadIdx.x; k < sizeof(S.zk) / 16u; k += kPT) zd[k] = zs[k];
    }
  }
  __syncthreads();
  // the wave's records are e0, e0 + nw, ...: lane l resolves the place of the wave's record
  // b * 64 + l (every dependent lookup of 64 records at once: a chain of six loads each, which one
  // record at a time left the wave waiting ~10 us per record), then the wave stores them one after
  // the other
  const u32 nw = A.wgb * kPW, lane = threadIdx.x & 63u;
  const u32 e0 = __builtin_amdgcn_readfirstlane(wg * kPW + (threadIdx.x >> 6));
  for (u32 base = e0; base < nbig; base += 64u * nw) {
    const u32 e = base + lane * nw;
    bool ok = e < nbig;
    u64 src = 0, pos = 0, off = 0, ringb = 0, segm = 0;
    u32 L = 0, dead = 0, lm = 0, nx = 0;
    u64 xdst[kMaxRemote] = {};
    if (ok) {
      const u32 gi = x.bigl[e];
      const u32 t = gi / kTR, jb = batch_of_tile(G, t);
      const PipeBatch& b = G.b[jb];
      const u32 i = (t - G.tile0[jb]) * kTR + gi % kTR;
      const uint2 cr = x.crank[gi];
      ok = !(u32)A.s3.binfo[jb * 4] && (cr.x >> kFlagShift) == 0u;  // batch rejected / record refused
      const u32 p = b.pidx[i];
      L = b.len[i];
      src = reinterpret_cast<u64>(b.payload) + (b.poff ? b.poff[i] : x.tile_base[t] + x.pre[gi]);
      const u64 ex = ok ? x.excl[(u64)p * A.gt + t] : 0ull;
      ok = ok && st.is_leader[p] && !(ex & kExclNoSpace);
      if (ok) {
        const u64 tot = x.totals[p], leo = A.cur.leo[p], used = A.cur.used[p];
        const u32 rk = (u32)((ex >> 40) & kCnt23) + (cr.x & kRankMask);
        const u32 rel16 = (u32)(ex & kLow40) + cr.y;
        off = leo + rk;
        pos = used + 16ull * rel16;
        const RingRef rg = ring_ref(st.ring[p], st.interval_log2, st.icap_mul);
        const u64 gend = used + 16ull * (tot & kLow40);
        dead = gend > pos + rg.seg ? (u32)min((gend - rg.seg - pos) >> 4, (u64)((L + 15u) >> 4) + 1ull) : 0u;
        lm = (A.debug & 1u) ? 0u : st.local_mask[p];
        ringb = reinterpret_cast<u64>(st.logs + rg.base);
        segm = rg.seg - 1ull;
        if (XR) {
          const u32 lmx = st.local_mask[p];
          for (u32 r = 0; r < st.RF && nx < kMaxRemote; ++r) {
            if ((lmx >> r) & 1u) continue;
            const u32 oe = A.outidx[(u64)p * st.RF + r];
            if (oe == ~0u || A.xe3[oe].data_abs == kNoRound) continue;
            xdst[nx++] = reinterpret_cast<u64>(A.outbox3 + A.xe3[oe].data_abs + 16ull * rel16);
          }
        }
      }
    }
    // the wave's (record, round) units in order, each unit's payload loads issued before the unit
    // ahead of it is folded and stored: the next round of the same record, or the first round of
    // the next one (one load latency per round otherwise, behind the previous round's stores)
    u64 bm = __ballot(ok);
    if (!bm) continue;
    auto take = [&](u32 k) {
      BigRec R;
      R.src = bcast_u64(src, k);
      R.pos = bcast_u64(pos, k);
      R.off = bcast_u64(off, k);
      R.ring = bcast_u64(ringb, k);
      R.segm = bcast_u64(segm, k);
      R.L = readlane32(L, k);
      R.dead = readlane32(dead, k);
      R.lm = readlane32(lm, k);
      R.nx = XR ? readlane32(nx, k) : 0u;
#pragma unroll
      for (u32 q = 0; q < kMaxRemote; ++q) R.x[q] = XR ? bcast_u64(xdst[q], k) : 0ull;
      R.ph = big_phase(R.pos);
      R.m = (R.L + 15u) >> 4;
      return R;
    };
    u32 k = (u32)__builtin_ctzll(bm);
    bm &= bm - 1ull;
    BigRec cur = take(k);
    uint4 nb[kBU], ntail;
    big_round(cur.src, cur.L, 0u, cur.ph, nb, ntail);
    u32 k0 = 0, acc = 0;
    for (;;) {
      uint4 cb[kBU];
#pragma unroll
      for (u32 u = 0; u < kBU; ++u) cb[u] = nb[u];
      const uint4 ctail = ntail;
      const bool more = 64u * (k0 + kBU) < cur.m + cur.ph, last = !more && !bm;
      BigRec nxt = cur;
      if (more) {
        big_round(cur.src, cur.L, k0 + kBU, cur.ph, nb, ntail);
      } else if (bm) {
        nxt = take((u32)__builtin_ctzll(bm));
        bm &= bm - 1ull;
        big_round(nxt.src, nxt.L, 0u, nxt.ph, nb, ntail);
      }
      big_store_round(A, S, XR ? A.crc->zshift1k : S.zk, cur, k0, cb, ctail, acc);
      if (more) {
        k0 += kBU;
        continue;
      }
      big_close(A, cur, acc);
      if (last) break;
      cur = nxt;
      k0 = 0;
      acc = 0;
    }
  }
}

template <bool XR>
__device__ __forceinline__ void stage3_finish(const PipeArgs& A, const Stage3Smem& S, const TaskPos& T, const TaskRec& R,
                              const TaskState& Z, bool cand, uint4& stat_out) {
  const PipeBatch& b = A.g3.b[T.jb];
  const DevState& st = A.st;
  const u32 lane = threadIdx.x & 63, j = lane & 1u;
  const u32 RF = st.RF;
  const u32 i = task_rec(T);
  const bool in = i < b.n;
  const u32 p = R.p, L = R.L;
  const u32 fl = R.cr.x >> kFlagShift;
  const u32 rej = batch_rej(A, T);
  const bool ns = (Z.lm & kNoSpace) != 0u;  // the record's (batch, partition) is over its limit
  const bool lead = (Z.lm & kLead) != 0u;
  const u32 lm8 = Z.lm & 0xFFu;
  const bool ok = cand && lead && !ns;
  const u32 m = (L + 15u) >> 4;  // payload pieces
  const bool big = ok && m > kBigPieces;  // stored by the whole wave below
  const bool okp = ok && !big;           // stored by its lane pair
  const RingRef rg = ring_ref(Z.rdesc, st.interval_log2, st.icap_mul);
  const u64 segmask = rg.seg - 1ull;
  const u64 rstride = st.rstride;
  const u64 off = Z.off, pos = Z.pos;
  const u32 dead = Z.dead;
  uint8_t* const ring = st.logs + rg.base;
  const u32 lmw = (A.debug & 1u) ? 0u : lm8;
  const u32 sa = (u32)(R.src & 15u);
  u32 acc = 0;
  const u32 nr = okp ? (m + kPR - 1u) / kPR : 0u;
  // records of at most 7 pieces (112 payload bytes) go through an LDS image of the log so that
  // 8 consecutive lanes store each record's 128 bytes; longer ones are stored piecewise
  const bool img = __all(!okp || m <= 7u);
  const u32 w = threadIdx.x >> 6, r32 = lane >> 1;
  Stage3Smem& W = const_cast<Stage3Smem&>(S);
  // replication transport: every record also goes, whole, to the group's outbox once per remote
  // replica slot (FORMAT.md §9), with its record-table slot and, for the partition's first record
  // of the group, the directory's first offset
  constexpr bool xr = XR;
  if (xr) {
    if (j == 0) {
      u32 nx = 0;
      if (ok) {
        const u64 rel = 16ull * Z.rel16;  // bytes into the group
        const u64 rk = Z.rk;              // records into the group
        for (u32 r = 0; r < RF; ++r) {
          if ((lm8 >> r) & 1u) continue;
          const u32 e = A.outidx[(u64)p * RF + r];
          if (e == ~0u) continue;
          const XEntry x = A.xe3[e];
          if (x.data_abs == kNoRound) continue;  // a partial catch-up: the round's records wait
          W.xdst[w][r32][nx++] = reinterpret_cast<u64>(A.outbox3 + x.data_abs + rel);
          *reinterpret_cast<u64*>(A.outbox3 + x.tab_abs + 8ull * rk) =
              (u64)x.k | ((u64)(x.data_start16 + (u32)(rel >> 4)) << 32);
        }
      }
      W.xn[w][r32] = nx;
    }
    __builtin_amdgcn_wave_barrier();
  }
  uint4 blk[kBL];
#pragma unroll
  for (u32 q = 0; q < kBL; ++q) blk[q] = Z.blk[q];
  if (Z.nblk) {
    // the task's payload span through the wave's image area: every lane's blocks in, then each
    // lane pair's record blocks out (before any image write reuses the area)
    uint4* sg = &W.img[w][0][0];
    static_assert(sizeof(S.img[0]) >= 64u * kSpanPer * 16u, "a wave's image area holds the staged span");
#pragma unroll
    for (u32 u = 0; u < kSpanPer; ++u)
      if (lane + 64u * u < Z.nblk) sg[lane + 64u * u] = Z.blk[u];
    __builtin_amdgcn_wave_barrier();
    const u32 b0 = (u32)(((R.src & ~15ull) - Z.sbase) >> 4) + j;
#pragma unroll
    for (u32 q = 0; q < kBL; ++q) {
      const u32 k = b0 + 2u * q;
      blk[q] = k < Z.nblk ? sg[k] : make_uint4(0, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
  for (u32 c = 0; __any(c < nr); ++c) {
    if (c) round_blocks(A, R, c, c < nr, blk);
#pragma unroll
    for (u32 q = 0; q < 4; ++q) {
      // piece jp = blocks jp (own q-th) and jp + 1 (partner's q-th for lane 0, (q+1)-th for
      // lane 1): each lane offers what its partner needs, then one DPP swap
      const uint4 pb = pair_swap4(j ? blk[q] : blk[q + 1]);
      const u32 jp = kPR * c + j + 2u * q;
      if (c < nr && jp < m) {
        const u32 nb = L - 16u * jp < 16u ? L - 16u * jp : 16u;
        const uint4 v = extract_piece(blk[q], pb, sa, nb);
        // Horner over the lane's pieces (jp rises by 2 = 32 bytes): reg(.. || p) = reg(..) * x^256 ^ reg(p)
        acc = crc_zshift(S.z[1], acc) ^ piece_crc(A, S, v, jp);
        if (img) {
          const_cast<Stage3Smem&>(S).img[w][r32][jp + 1] = v;
        } else {
          uint8_t* dst = ring + ((pos + 16ull + 16ull * jp) & segmask);
          if (jp + 1u >= dead)
            for (u32 r = 0; r < RF; ++r)
              if ((lmw >> r) & 1u) store_log16(dst + r * rstride, v);
          if (xr)
            for (u32 q = 0; q < S.xn[w][r32]; ++q)
              store_log16(reinterpret_cast<uint8_t*>(S.xdst[w][r32][q]) + 16ull + 16ull * jp, v);
        }
      }
    }
  }
  // align the lane's register to the record end: its last piece is m-1 or m-2 (then 16 bytes short)
  if (okp && m > j && ((m - 1u - j) & 1u)) acc = crc_zshift(S.z[0], acc);
  acc ^= pair_swap(acc);

  // ---- header (lane 1), out offset (lane 0), sparse index (lane 1)
  // CRC32C = ~(register(M || pad zeros) * x^(-8 pad)); the pair splits the product by halves of
  // the register's coefficients
  u32 part = 0;
  if (okp && L) {
    const u32 pad = 16u * m - L;
    part = pad ? gf2_mulmod_half(j ? acc & 0xFFFFu : acc >> 16, j ? A.crc->inv_pad16[pad] : A.crc->inv_pad[pad])
               : (j ? 0u : acc);
  }
  part ^= pair_swap(part);
  uint4 h = make_uint4(0, 0, 0, 0);
  if (okp && j == 1) h = make_uint4((u32)off, (u32)(off >> 32), L, L ? ~part : 0u);
  if (img) {
    if (j == 1) W.img[w][r32][0] = h;
    // the 4-bit piece count is only meaningful for a stored record (ok implies m <= 7 here); a
    // rejected record may be long, and its count must not spill into the flag bits
    if (j == 0)
      W.info[w][r32] = make_uint4((u32)pos, (u32)(pos >> 32), (u32)(rg.base >> 8),
                                  okp ? lm8 | (m << 8) | (1u << 12) | (dead << 13) | ((u32)(Z.rdesc & 63ull) << 24) : 0u);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (u32 s4 = 0; s4 < kTaskRecs * 8u / 64u; ++s4) {
      const u32 idx = lane + 64u * s4, rr = idx >> 3, k = idx & 7u;
      const uint4 inf = W.info[w][rr];
      const u32 mr = (inf.w >> 8) & 0xFu;
      if (((inf.w >> 12) & 1u) && k <= mr) {
        const uint4 v = W.img[w][rr][k];
        if (k >= ((inf.w >> 13) & 0x1Fu)) {
          const u64 rpos = ((u64)inf.y << 32) | inf.x;
          const u64 rmask = (1ull << (inf.w >> 24)) - 1ull;
          uint8_t* dst = st.logs + ((u64)inf.z << 8) + ((rpos + 16ull * k) & rmask);
          const u32 lmr = (A.debug & 1u) ? 0u : (inf.w & 0xFFu);
          for (u32 r = 0; r < RF; ++r)
            if ((lmr >> r) & 1u) store_log16(dst + r * rstride, v);
        }
        if (xr)
          for (u32 q = 0; q < W.xn[w][rr]; ++q) store_log16(reinterpret_cast<uint8_t*>(W.xdst[w][rr][q]) + 16ull * k, v);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the image is rewritten by the wave's next task
  } else if (okp && j == 1) {
    uint8_t* dst = ring + (pos & segmask);
    if (dead == 0u)
      for (u32 r = 0; r < RF; ++r)
        if ((lm8 >> r) & 1u) store_log16(dst + r * rstride, h);
    if (xr)
      for (u32 q = 0; q < S.xn[w][r32]; ++q) store_log16(reinterpret_cast<uint8_t*>(S.xdst[w][r32][q]), h);
  }
  if (in && j == 0) b.out_offsets[i] = ok ? off : ~0ull;
  const u32 ilog = st.interval_log2;
  const u64 end = pos + 16ull * (1ull + m);
  if (ok && j == 1) {
    for (u64 mm = (pos >> ilog) + 1; (mm << ilog) <= end; ++mm) {
      u64* e = st.index + (rg.ibase + mm % rg.icap) * 2;
      e[0] = off + 1;
      e[1] = end;
    }
  }
  {
    const bool h0 = j == 0;
    const u32 n_in = (u32)__popcll(__ballot(h0 && in));
    const u32 n_app = (u32)__popcll(__ballot(h0 && ok));
    const u32 n_nl = (u32)__popcll(__ballot(h0 && cand && !lead));
    const u32 n_np = rej ? 0u : (u32)__popcll(__ballot(h0 && in && fl == kFlNoPart));
    const u32 n_inv = (rej & kRejInvalid) ? n_in : 0u;
    const u32 n_ns = (u32)__popcll(__ballot(h0 && cand && lead && ns));
    stat_out = make_uint4(n_app, n_nl, n_np, n_ns | (n_inv << 16));
  }
}

// Thread per partition: stage 3's state advance, retention of the group it applies, and stage 4.
// Everything these read is loaded first, in one round (speculatively: a partition this engine
// does not lead, or one without records, discards it), so the chain is that round, the index
// entries retention needs, and the stores.
//  * stage 3: the group's new log end, matchIndex, quorum commit and high watermark, into the next
//    state set. The commit rule is monotone in the log end, so evaluating it once after the group
//    equals evaluating it after each batch. A partition this engine does not lead keeps its state
//    outside the pipeline (its records are counted by stages 1/2, ranks being per partition, but
//    never applied; the host keeps both state sets equal for it); stage 2 leaves rejected
//    (batch, partition) cells out of totals.
//  * retention after each batch of the group applied by this launch, from index entries written
//    before it (an entry this launch writes ends the replay: a group that adds more than a ring
//    less one interval to the partition). Then a fetch ordered after the launch sees the log start
//    of the records it sees, and a drain needs no stage-4 launch unless a partition stopped early
//    (it writes the launch number into ret_late).
//  * stage 4: retention after each batch of the group applied one launch earlier, for the
//    partitions whose replay that launch stopped (rlate[p]; the batch aggregates are loaded only
//    for them, so the common case carries no stage-4 loads).
__device__ __forceinline__ void partition_threads(const PipeArgs& A, u32 p) {
  const DevState& st = A.st;
  const u32 RF = st.RF;
  const bool a3 = A.g3.nb != 0, a4 = A.g4.nb != 0;
  const bool lead = st.is_leader[p];
  const u64 tot3 = a3 ? A.s3.totals[p] : 0ull;
  const u64 leo0 = A.cur.leo[p], used0 = A.cur.used[p];
  const u32 lm = st.local_mask[p];
  u64 row[kMaxRF];
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) row[r] = r < RF ? st.match[(u64)p * RF + r] : 0ull;
  const u64 commit0 = st.commit[p], ts = st.term_start[p];
  const u64 soff0 = st.start_off[p], spos0 = st.start_pos[p];
  const u64 desc = st.ring[p];
  const u32 late4 = a4 ? A.rlate[p] : 0u;  // the launch before stopped p's retention early
  u64 bc3[kMaxGroup];
#pragma unroll
  for (u32 j = 0; j < kMaxGroup; ++j) bc3[j] = a3 && j < A.g3.nb ? A.s3.bcum[(u64)j * st.P + p] : 0ull;
  if (A.lastg && a3) A.lastg[p] = lead ? (tot3 & kLow40) : 0ull;  // the next plans' C (FORMAT.md §9)
  if (!lead) return;
  u64 cfin = commit0;  // the partition's commit at the end of this launch (st.csnap)
  // ---- stage 3: log end, matchIndex, commit (first: the match row is dead before retention)
  if (a3) {
    A.nxt.leo[p] = leo0 + (tot3 >> 40);
    A.nxt.used[p] = used0 + 16ull * (tot3 & kLow40);
  }
  const u64 tc = tot3 >> 40, leo = leo0 + tc;
  if (tc || A.ackin) {
    bool moved = tc != 0;
    if (tc) {
#pragma unroll
      for (u32 r = 0; r < kMaxRF; ++r)
        if (r < RF && ((lm >> r) & 1u)) {
          row[r] = leo;
          st.match[(u64)p * RF + r] = leo;
        }
    }
    // followers' acks of an earlier group (replication transport, FORMAT.md §9)
    if (A.ackin) {
      const u32 fl = apply_acks(st, p, A.outidx, A.ackin, leo, row, A.xreq, A.acks_round, A.ackrowv);
      moved |= (fl & kAckMatch) != 0u;
      if (fl & kAckRow) st.cq[p] = row_quorum(st, p);  // consumer-offset rows on a quorum (tickets)
    }
    if (moved) {
      const u64 c = quorum_commit(row, RF, commit0, ts);
      st.commit[p] = c;
      st.hw[p] = c;
      cfin = c;
    }
  }
  if (st.csnap) st.csnap[(A.launch_seq & 1ull) * st.P + p] = cfin;  // the next launch's plan carries it

  const RingRef rg = ring_ref(desc, st.interval_log2, st.icap_mul);
  u64 soff = soff0, spos = spos0;
  // ---- stage 4: retention of the group applied one launch earlier (cur: its final log end)
  if (late4) {
    u64 bc[kMaxGroup];
#pragma unroll
    for (u32 j = 0; j < kMaxGroup; ++j) bc[j] = j < A.g4.nb ? A.s4.bcum[(u64)j * st.P + p] : 0ull;
    retain_batches(st, rg, bc, A.g4.nb, false, used0, A.s4.totals[p], ~0ull, soff, spos);
  }
  // ---- retention of the group this launch applies (cur: the log end before it)
  bool late3 = false;
  if (tc) {
    late3 = !retain_batches(st, rg, bc3, A.g3.nb, true, used0, tot3, used0, soff, spos);
    if (late3 && A.ret_late) __hip_atomic_store(A.ret_late, A.launch_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (late3 || late4) A.rlate[p] = late3 ? 1u : 0u;
  if (soff != soff0 || spos != spos0) {
    st.start_off[p] = soff;
    st.start_pos[p] = spos;
  }
}

// Catch-up waves of the stage-3 launch (FORMAT.md §9 v3, replication transport): the gaps the
// plan granted, copied from this leader's ring into the outbox with their record-table slots. One
// item = one sparse-index interval [m I, (m + 1) I) of one gap: its first record is the gap's own
// (the first item) or E[m], the first record starting at or after m I; the wave copies the
// interval's bytes (a 16-byte piece per lane, 1 KiB per step) and walks the headers of the records
// that start in it. Round h-1's records are complete (the previous launch) and round h's stores
// into the ring land past the gap's end minus the ring size (the plan's condition), so nothing
// this reads changes under it.
__device__ __forceinline__ void stage3_catchup(const PipeArgs& A, u32 wg) {
  const u32 items = __builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile const u32*>(A.xc3_n + 1));
  const u32 ncu = __builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile const u32*>(A.xc3_n));
  if (!items) return;
  const DevState& st = A.st;
  const u32 lane = threadIdx.x & 63, ilog = st.interval_log2;
  for (u32 it = __builtin_amdgcn_readfirstlane(wg * kPW + (threadIdx.x >> 6)); it < items; it += A.wgc * kPW) {
    u32 lo = 0, hi = ncu;  // the catch-up entry holding item it: largest items0 <= it
    while (hi - lo > 1) {
      const u32 mid = (lo + hi) / 2;
      if (A.xc3[mid].items0 <= it) lo = mid; else hi = mid;
    }
    const XCatch c = A.xc3[lo];
    const u32 j = it - c.items0;
    const RingRef rg = ring_ref(st, c.p);
    const uint8_t* ring = st.logs + (u64)__builtin_ctz(st.local_mask[c.p]) * st.rstride + rg.base;
    const u64 mask = rg.seg - 1ull, end = c.pos + c.bytes;
    const u64 m = (c.pos >> ilog) + j;
    const u64 w0 = j ? m << ilog : c.pos, w1 = min(end, (m + 1ull) << ilog);
    // the first record starting in the window
    u64 roff = c.first, rpos = c.pos;
    if (j) {
      const u64* ie = st.index + (rg.ibase + m % rg.icap) * 2;
      roff = ie[0];
      rpos = ie[1];
    }
    for (u64 sub = w0 & ~1023ull; sub < w1; sub += 1024) {
      const u64 q = sub + 16ull * lane;
      uint4 v = make_uint4(0, 0, 0, 0);
      const bool mine = q >= w0 && q < w1;
      if (mine) {
        v = *reinterpret_cast<const uint4*>(ring + (q & mask));
        store_log16(A.outbox3 + c.data_abs + (q - c.pos), v);
      }
      // walk the headers that start in [max(sub, w0), min(sub + 1 KiB, w1)): lane (pos - sub) / 16
      while (rpos < min(sub + 1024ull, w1)) {
        const u32 L = (u32)__shfl((int)v.z, (int)((rpos - sub) >> 4), 64);
        if (lane == 0)
          *reinterpret_cast<u64*>(A.outbox3 + c.tab_abs + 8ull * (roff - c.first)) =
              (u64)c.k | ((u64)(c.data_start16 + (u32)((rpos - c.pos) >> 4)) << 32);
        rpos += 16ull + ((L + 15ull) & ~15ull);
        ++roff;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Stage 3 in two roles (RMQ_S3_ROLES, single-GPU kernel): loader waves and a storer wave
// ------------------------------------------------------------------------------------------
// On gfx950 `vmcnt` counts stores as well as loads, and a wave's slot is held until its stores are
// acknowledged (s_endpgm waits for them): a wave that loads, checksums and stores its task keeps its
// slot through the store latency, and a wave that loops over tasks waits for the previous task's
// stores before the next task's loads return. Here a workgroup takes a contiguous run of tasks and
// splits the work by wave: kS3Loaders loader waves load each task's record words, partition line and
// payload, compute the CRCs and build the task's log image in an LDS buffer, with no global stores
// (so each loader prefetches its next task's record words while it checksums the current one, and
// no load ever waits behind a store); the storer wave takes the images in task order and issues only
// stores: ring pieces, out offsets, sparse-index entries and statistics. It never waits on vmcnt.
// The hand-off is a ring of kS3Bufs LDS buffers with one sequence word each: a loader publishes task
// i in buffer i % kS3Bufs as 2i + 1 once its image writes have completed (lgkmcnt(0)); the storer
// reads the buffer into registers and releases it as 2i + 2. Every wait is for a smaller task index,
// so the smallest unfinished task always progresses (no deadlock), and every wave ends when its
// share of the run is done.
#ifndef RMQ_S3_LOADERS
#define RMQ_S3_LOADERS 3
#endif
constexpr u32 kS3Loaders = RMQ_S3_LOADERS;
constexpr u32 kS3Storers = kPW > kS3Loaders ? kPW - kS3Loaders : 1u;
constexpr u32 kS3Bufs = 4;
struct Stage3RSmem {
  u32 t8[8][256];
  u32 z[2][4][256];
  uint4 img[kS3Bufs][kTaskRecs][8];   // the task's records as laid out in the log (<= 128 B each)
  uint4 info[kS3Bufs][kTaskRecs][2];  // {pos, off}, {ring descriptor, flags, payload pieces}
  uint4 stat[kS3Bufs];                // the task's statistics
  u32 seq[kS3Bufs];                   // 2i + 1: task i published; 2i + 2: task i taken
};
static_assert(sizeof(Stage3RSmem) <= kSmemBytes, "the role-split stage 3 fits the launch's LDS");
// info flags
constexpr u32 kRfImg = 8u;            // bits 8..11: payload pieces the storer stores from the image
constexpr u32 kRfSt = 1u << 12;       // the storer stores the header (and the image's pieces)
constexpr u32 kRfDead = 13u;          // bits 13..17: leading dead pieces (0 = header), clipped at 31
constexpr u32 kRfOk = 1u << 18;       // appended: out offset = off, index entries
constexpr u32 kRfIn = 1u << 19;       // a record of the batch: an out offset is written

__device__ __forceinline__ u32 lds_seq(const u32* s) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// Wait until the sequence word reaches v (LDS only: no vmcnt wait), then order later LDS accesses
// after it. The wait is bounded (about a second): a broken hand-off ends in wrong results that the
// parity tests catch, never in waves that do not finish.
__device__ __forceinline__ void lds_wait_seq(const u32* s, u32 v) {
  for (u32 k = 0; lds_seq(s) < v && k < (1u << 24); ++k) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}
// Every LDS write (and read) of this wave has completed, then the sequence word is set.
__device__ __forceinline__ void lds_post_seq(u32* s, u32 v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(s, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Loader: the task's CRCs and log image into buffer bi (stage3_finish without the stores; records of
// 8-64 payload pieces, which do not fit the image, store their payload pieces here themselves).
__device__ __forceinline__ void stage3_build(const PipeArgs& A, Stage3RSmem& S, const TaskPos& T, const TaskRec& R,
                                             const TaskState& Z, bool cand, u32 bi) {
  const PipeBatch& b = A.g3.b[T.jb];
  const DevState& st = A.st;
  const u32 lane = threadIdx.x & 63, j = lane & 1u, r32 = lane >> 1;
  const u32 RF = st.RF;
  const u32 i = task_rec(T);
  const bool in = i < b.n;
  const u32 L = R.L;
  const u32 fl = R.cr.x >> kFlagShift;
  const u32 rej = batch_rej(A, T);
  const bool ns = (Z.lm & kNoSpace) != 0u;
  const bool lead = (Z.lm & kLead) != 0u;
  const u32 lm8 = Z.lm & 0xFFu;
  const bool ok = cand && lead && !ns;
  const u32 m = (L + 15u) >> 4;
  const bool big = ok && m > kBigPieces;  // the large-record waves store it
  const bool okp = ok && !big;
  const RingRef rg = ring_ref(Z.rdesc, st.interval_log2, st.icap_mul);
  const u64 segmask = rg.seg - 1ull;
  const u64 pos = Z.pos;
  uint8_t* const ring = st.logs + rg.base;
  const u32 lmw = (A.debug & 1u) ? 0u : lm8;
  const u32 sa = (u32)(R.src & 15u);
  const u32 nr = okp ? (m + kPR - 1u) / kPR : 0u;
  const bool img = __all(!okp || m <= 7u);
  u32 acc = 0;
  uint4 blk[kBL];
#pragma unroll
  for (u32 q = 0; q < kBL; ++q) blk[q] = Z.blk[q];
  for (u32 c = 0; __any(c < nr); ++c) {
    if (c) round_blocks(A, R, c, c < nr, blk);
#pragma unroll
    for (u32 q = 0; q < 4; ++q) {
      const uint4 pb = pair_swap4(j ? blk[q] : blk[q + 1]);
      const u32 jp = kPR * c + j + 2u * q;
      if (c < nr && jp < m) {
        const u32 nb = L - 16u * jp < 16u ? L - 16u * jp : 16u;
        uint4 v = extract_piece(blk[q], pb, sa, nb);
        uint4 vc = v;
        if (jp == 0) vc.x ^= 0xFFFFFFFFu;
        acc = crc_zshift(S.z[1], acc) ^ ((A.debug & 2u) ? vc.x : crc_piece16(S.t8, vc));
        if (img) {
          S.img[bi][r32][jp + 1] = v;
        } else {
          uint8_t* dst = ring + ((pos + 16ull + 16ull * jp) & segmask);
          if (jp + 1u >= Z.dead)
            for (u32 r = 0; r < RF; ++r)
              if ((lmw >> r) & 1u) store_log16(dst + r * st.rstride, v);
        }
      }
    }
  }
  if (okp && m > j && ((m - 1u - j) & 1u)) acc = crc_zshift(S.z[0], acc);
  acc ^= pair_swap(acc);
  u32 part = 0;
  if (okp && L) {
    const u32 pad = 16u * m - L;
    part = pad ? gf2_mulmod_half(j ? acc & 0xFFFFu : acc >> 16, j ? A.crc->inv_pad16[pad] : A.crc->inv_pad[pad])
               : (j ? 0u : acc);
  }
  part ^= pair_swap(part);
  if (j == 1) {
    S.img[bi][r32][0] = okp ? make_uint4((u32)Z.off, (u32)(Z.off >> 32), L, L ? ~part : 0u) : make_uint4(0, 0, 0, 0);
  } else {
    const u32 f = (okp ? (lmw | ((img ? m : 0u) << kRfImg) | kRfSt) : 0u) | (min(Z.dead, 31u) << kRfDead) |
                  (ok ? kRfOk : 0u) | (in ? kRfIn : 0u);
    S.info[bi][r32][0] = make_uint4((u32)pos, (u32)(pos >> 32), (u32)Z.off, (u32)(Z.off >> 32));
    S.info[bi][r32][1] = make_uint4((u32)Z.rdesc, (u32)(Z.rdesc >> 32), f, m);
  }
  const bool h0 = j == 0;
  const u32 n_in = (u32)__popcll(__ballot(h0 && in));
  const u32 n_app = (u32)__popcll(__ballot(h0 && ok));
  const u32 n_nl = (u32)__popcll(__ballot(h0 && cand && !lead));
  const u32 n_np = rej ? 0u : (u32)__popcll(__ballot(h0 && in && fl == kFlNoPart));
  const u32 n_inv = (rej & kRejInvalid) ? n_in : 0u;
  const u32 n_ns = (u32)__popcll(__ballot(h0 && cand && lead && ns));
  if (lane == 0) S.stat[bi] = make_uint4(n_app, n_nl, n_np, n_ns | (n_inv << 16));
}

// Storer: task `task` from buffer bi (published as sequence ti): everything into registers, the
// buffer released, then the stores.
__device__ __forceinline__ void stage3_store(const PipeArgs& A, Stage3RSmem& S, u32 task, u32 bi, u32 ti) {
  const PipeGroup& G = A.g3;
  const DevState& st = A.st;
  const u32 lane = threadIdx.x & 63;
  const TaskPos T = task_pos(G, task);
  const PipeBatch& b = G.b[T.jb];
  constexpr u32 kS4 = kTaskRecs * 8u / 64u;  // (record, piece) slots per lane
  uint4 v[kS4], i0[kS4], i1[kS4];
#pragma unroll
  for (u32 s4 = 0; s4 < kS4; ++s4) {
    const u32 idx = lane + 64u * s4, rr = idx >> 3, k = idx & 7u;
    v[s4] = S.img[bi][rr][k];
    i0[s4] = S.info[bi][rr][0];
    i1[s4] = S.info[bi][rr][1];
  }
  const u32 rr = lane & (kTaskRecs - 1u);  // lanes 0..31: record lane's out offset and index entries
  const uint4 r0 = S.info[bi][rr][0], r1 = S.info[bi][rr][1];
  const uint4 so = S.stat[bi];
  lds_post_seq(&S.seq[bi], 2u * ti + 2u);
  const u64 rstride = st.rstride;
#pragma unroll
  for (u32 s4 = 0; s4 < kS4; ++s4) {
    const u32 k = (lane + 64u * s4) & 7u;
    const u32 f = i1[s4].z;
    if ((f & kRfSt) && k <= ((f >> kRfImg) & 0xFu) && k >= ((f >> kRfDead) & 31u)) {
      const u64 rpos = ((u64)i0[s4].y << 32) | i0[s4].x;
      const RingRef rg = ring_ref(((u64)i1[s4].y << 32) | i1[s4].x, st.interval_log2, st.icap_mul);
      uint8_t* dst = st.logs + rg.base + ((rpos + 16ull * k) & (rg.seg - 1ull));
      for (u32 r = 0; r < st.RF; ++r)
        if ((f >> r) & 1u) store_log16(dst + r * rstride, v[s4]);
    }
  }
  if (lane < kTaskRecs) {
    const u32 f = r1.z;
    const u64 off = ((u64)r0.w << 32) | r0.z;
    if (f & kRfIn) b.out_offsets[T.i0 + lane] = (f & kRfOk) ? off : ~0ull;
    if (f & kRfOk) {
      const u32 ilog = st.interval_log2;
      const u64 pos = ((u64)r0.y << 32) | r0.x;
      const u64 end = pos + 16ull * (1ull + r1.w);
      const RingRef rg = ring_ref(((u64)r1.y << 32) | r1.x, ilog, st.icap_mul);
      for (u64 mm = (pos >> ilog) + 1; (mm << ilog) <= end; ++mm) {
        u64* e = st.index + (rg.ibase + mm % rg.icap) * 2;
        e[0] = off + 1;
        e[1] = end;
      }
    }
  }
  if (lane == 0) G.stats[T.jb][task - G.task0[T.jb]] = so;
}

// The CRC tables into LDS by the loader waves: every 16-byte block loaded before any is written
// (one load round trip instead of one per block a thread copies).
__device__ __forceinline__ void roles_tables(const PipeArgs& A, Stage3RSmem& S) {
  static_assert(offsetof(CrcConsts, zshift) == sizeof(A.crc->table), "table and zshift adjacent");
  constexpr u32 kN = (sizeof(S.t8) + sizeof(S.z)) / 16u, kT = kS3Loaders * 64u, kPer = (kN + kT - 1u) / kT;
  const uint4* src = reinterpret_cast<const uint4*>(&A.crc->table[0][0]);
  uint4* dst = reinterpret_cast<uint4*>(&S.t8[0][0]);
  uint4 v[kPer];
#pragma unroll
  for (u32 q = 0; q < kPer; ++q) v[q] = src[min(threadIdx.x + q * kT, kN - 1u)];  // (unconditional: registers)
#pragma unroll
  for (u32 q = 0; q < kPer; ++q)
    if (threadIdx.x + q * kT < kN) dst[threadIdx.x + q * kT] = v[q];
}

// A workgroup's run of tasks [slot * tasks / wg3, (slot + 1) * tasks / wg3) in two roles.
__device__ __forceinline__ void stage3_roles(const PipeArgs& A, Stage3RSmem& S, u32 slot) {
  const PipeGroup& G = A.g3;
  const u32 tasks = G.task0[G.nb];
  const u32 t0 = (u32)((u64)slot * tasks / A.wg3), n = (u32)((u64)(slot + 1u) * tasks / A.wg3) - t0;
  const u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  PIPE_STAMP(0);
  if (w < kS3Loaders && w < n) {
    // the first task's record words are in flight while the tables fill LDS
    u32 i = w;
    TaskPos T = task_pos(G, t0 + i);
    TaskRec R = stage3_r1(A, T);
    if (!(A.debug & 8u)) roles_tables(A, S);
    bool cand = stage3_cand(A, T, R);
    TaskState Z = stage3_r2(A, T, R, cand);
    if (threadIdx.x < kS3Bufs) S.seq[threadIdx.x] = 0u;
    __syncthreads();
    PIPE_STAMP(1);
    u64 waited = 0, tw = 0;  // (stamps: time spent waiting for a free buffer, for its loads)
    for (;;) {
      const u32 in_ = i + kS3Loaders;
      const bool more = in_ < n;  // (wave-uniform)
      TaskPos Tn = T;
      TaskRec Rn = R;
      if (more) {  // the next task's record words, issued before this task's stores... of which there are none
        Tn = task_pos(G, t0 + in_);
        Rn = stage3_r1(A, Tn);
      }
      const u32 bi = i % kS3Bufs;
      if (A.stamps) tw = __builtin_amdgcn_s_memrealtime();
      if (i >= kS3Bufs) lds_wait_seq(&S.seq[bi], 2u * (i - kS3Bufs) + 2u);
      if (A.stamps) {
        waited += __builtin_amdgcn_s_memrealtime() - tw;
        if (i == w) PIPE_STAMP(2);
      }
      stage3_build(A, S, T, R, Z, cand, bi);
      lds_post_seq(&S.seq[bi], 2u * i + 1u);
      if (!more) break;
      i = in_;
      T = Tn;
      R = Rn;
      cand = stage3_cand(A, T, R);
      Z = stage3_r2(A, T, R, cand);
    }
    if (A.stamps) {
      PIPE_STAMP(3);
      if ((threadIdx.x & 63) == 0) A.stamps[((u64)blockIdx.x * kPW + w) * 8 + 4] = waited;
    }
    return;
  }
  if (w < kS3Loaders) {  // a loader without a task: the tables and the barrier only
    if (!(A.debug & 8u)) roles_tables(A, S);
    if (threadIdx.x < kS3Bufs) S.seq[threadIdx.x] = 0u;
    __syncthreads();
    return;
  }
  __syncthreads();
  PIPE_STAMP(1);
  u64 waited = 0;  // (stamps: time spent waiting for a published image)
  for (u32 i = w - kS3Loaders; i < n; i += kS3Storers) {
    const u32 bi = i % kS3Bufs;
    const u64 tw = A.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
    lds_wait_seq(&S.seq[bi], 2u * i + 1u);
    if (A.stamps) {
      waited += __builtin_amdgcn_s_memrealtime() - tw;
      if (i == w - kS3Loaders) PIPE_STAMP(2);
    }
    stage3_store(A, S, t0 + i, bi, i);
  }
  if (A.stamps) {
    PIPE_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PIPE_STAMP(5);
    if ((threadIdx.x & 63) == 0) A.stamps[((u64)blockIdx.x * kPW + w) * 8 + 4] = waited;
  }
}

#ifndef RMQ_PIPE_WAVES_PER_SIMD
#define RMQ_PIPE_WAVES_PER_SIMD 4  // <= 128 VGPRs, no spills: 2 resident workgroups per CU
#endif
// Stage 1 of the launch's group, tile by tile: a static share (tiles wg, wg + wg1, ...) or, with
// RMQ_STEAL, tiles taken from the group's counter (s1.nbig[1]) by the dedicated stage-1 workgroups
// and by stage-3 workgroups that ran out of tasks, so ranking starts as soon as stage 3 frees a
// slot instead of when the dispatcher reaches the stage-1 workgroups.
__device__ __forceinline__ void stage1_tiles(const PipeArgs& A, char* smem, u32 wg, bool take) {
  __shared__ u32 s_t;
  // (RMQ_S1_XCD: the tiles of one XCD's workgroups contiguous, so the 32 tiles whose cells share a
  // 128-byte line of a partition's hist32 column are written through one L2)
  const u32 t0 = !take && A.s1_xcd ? xcd_rank(A.s3_lead, A.wg1, A.s3_lead + wg) : wg;
  for (u32 t = t0;;) {
    if (take) {
      if (threadIdx.x == 0) s_t = __hip_atomic_fetch_add(A.s1.nbig + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      t = s_t;
    }
    if (t >= A.g1.tiles) break;
    const u32 srow = A.s3_lead + t % A.wg1;
    if (A.rank_mode)
      stage1_tile_hash(A, t, *reinterpret_cast<Stage1HSmem*>(smem), srow);
    else
      stage1_tile(A, t, *reinterpret_cast<Stage1Smem*>(smem), srow);
    __syncthreads();  // the tile's LDS (and s_t) are reused by the next one
    if (!take) t += A.wg1;
  }
}

// XR: a replication transport is attached (stage 3 also fills the group's outbox); a separate
// instantiation so the single-GPU kernel keeps its register budget.
template <bool XR>
__global__ __launch_bounds__(kPT, RMQ_PIPE_WAVES_PER_SIMD) void pipeline_kernel(PipeArgs args) {
  // The arguments are read in place from the kernarg segment: with the by-value parameter, a select
  // between two of its fields (batch lookups) made the compiler copy all 3.4 KB of it into scratch
  // in every lane of the transport kernel (6x slower launches, round 4)
  (void)args;
  const PipeArgs& A = *(const PipeArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if (blockIdx.x == 0 && threadIdx.x == 0 && A.done_word)
    __hip_atomic_store(A.done_word, A.launch_seq - 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  u32 wg = blockIdx.x;
  // roles along blockIdx.x: [s3_lead stage-3 workgroups | stage 1 | stage 2 | partition threads |
  // the other stage-3 workgroups | large records] (dispatch order)
  if (wg >= A.wg1 + A.wg2 + A.wgp + A.wg3) {
    const u32 b = wg - (A.wg1 + A.wg2 + A.wgp + A.wg3);
    if (XR && b >= A.wgb)
      stage3_catchup(A, b - A.wgb);
    else
      stage3_big_waves<XR>(A, *reinterpret_cast<Stage3Smem*>(smem_raw), b);
    return;
  }
  bool s3 = false;
  {
    const u32 other = A.wg1 + A.wg2 + A.wgp;
    if (wg < A.s3_lead) {
      s3 = true;
    } else if (wg < A.s3_lead + other) {
      wg -= A.s3_lead;
    } else {
      s3 = true;
      wg -= other;
    }
  }
  if (!s3) {
    if ((A.debug & 16u) && wg < A.wg1 + A.wg2) return;
    // the ranking / scan / partition chains are latency-bound: their waves first at the issue
    // arbiter, stage 3's fill the rest (RMQ_PRIO)
    if (A.prio) __builtin_amdgcn_s_setprio(3);
    if (wg < A.wg1) {  // a workgroup ranks tiles wg, wg + wg1, ... (RMQ_S1_WGS < tiles: fewer slots held)
      stage1_tiles(A, smem_raw, wg, A.steal != 0u);
      return;
    }
    wg -= A.wg1;
    if (wg < A.wg2) {
      stage2<XR>(A, wg, reinterpret_cast<u64*>(smem_raw));
      return;
    }
    wg -= A.wg2;
    // partition threads: stage 3's state advance and stage 4's retention
    PIPE_STAMP(0);
    if (wg == 0 && A.g4.nb) {  // the set's next group starts its list, tile counter and batch sums
      if (threadIdx.x < 4) A.s4.nbig[threadIdx.x] = 0u;
      if (threadIdx.x < kMaxGroup * 2) A.s4.bacc[threadIdx.x] = 0ull;
    }
    for (u32 p = wg * kPT + threadIdx.x; p < A.st.P; p += A.wgp * kPT) partition_threads(A, p);
    if (A.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PIPE_STAMP(6);
    return;
  }
  Stage3Smem& S = *reinterpret_cast<Stage3Smem*>(smem_raw);
  const PipeGroup& G = A.g3;
  const u32 tasks = G.task0[G.nb];
  const u32 lane = threadIdx.x & 63;
  // the task index is wave-uniform: keep it (and the batch lookups) in scalar registers
  // (RMQ_S3_XCD: the stage-3 workgroups of one XCD take one contiguous range of slots, so records
  // next to each other in a batch, and in their partitions' rings, are stored through one L2)
  // (stage 3 first: its blocks are [0, wg3); last: [other, other + wg3))
  const u32 slot = A.s3_xcd ? xcd_rank(A.s3_lead ? 0u : A.wg1 + A.wg2 + A.wgp, A.wg3, blockIdx.x) : wg;
  if (!XR && A.s3_roles) {
    stage3_roles(A, *reinterpret_cast<Stage3RSmem*>(smem_raw), slot);
    return;
  }
  u32 task = __builtin_amdgcn_readfirstlane(slot * kPW + (threadIdx.x >> 6));
  PIPE_STAMP(0);
  if (!XR && A.s3_pair) {
    // two tasks per wave (task and task + wg3 waves; the engine sizes wg3 so every task has its
    // place), each load round issued for both before either is waited for: a wave spends most of
    // its life waiting on its dependent loads (record -> partition state and payload), so two
    // chains in flight per wave halve the waves and overlap their waits
    const u32 tb = task + A.wg3 * kPW;
    const bool ha = task < tasks, hb = tb < tasks;  // (wave-uniform)
    const TaskPos Ta = task_pos(G, ha ? task : 0u), Tb = task_pos(G, hb ? tb : 0u);
    const TaskRec Ra = stage3_r1(A, Ta), Rb = stage3_r1(A, Tb);
    if (!(A.debug & 8u)) crc_tables_lds<kPT>(A.crc, &S.t8[0][0], reinterpret_cast<u32*>(&S.img[0][0][0]));
    const bool ca = ha && stage3_cand(A, Ta, Ra), cb = hb && stage3_cand(A, Tb, Rb);
    const TaskState Za = stage3_r2(A, Ta, Ra, ca);
    const TaskState Zb = stage3_r2(A, Tb, Rb, cb);
    __syncthreads();
    uint4 so;
    if (ha) {
      stage3_finish<XR>(A, S, Ta, Ra, Za, ca, so);
      if (lane == 0) G.stats[Ta.jb][task - G.task0[Ta.jb]] = so;
    }
    if (hb) {
      stage3_finish<XR>(A, S, Tb, Rb, Zb, cb, so);
      if (lane == 0) G.stats[Tb.jb][tb - G.task0[Tb.jb]] = so;
    }
    return;
  }
  // first task: its record and state/payload loads are in flight while the CRC tables fill LDS
  TaskPos T = task_pos(G, task < tasks ? task : 0u);
  TaskRec R = stage3_r1(A, T);
  // the slicing and zero-shift tables (contiguous in Stage3Smem) from their nibble tables, through
  // the image area (first written after the barrier below); the expansion runs while the record's
  // state and payload loads are in flight
  static_assert(offsetof(Stage3Smem, z) == sizeof(S.t8), "t8 and z adjacent in LDS");
  if (!(A.debug & 8u)) crc_nib_lds<kPT>(A.crc, reinterpret_cast<u32*>(&S.img[0][0][0]));
  bool cand = task < tasks && stage3_cand(A, T, R);
  RecWords W0;
  TaskState Z = stage3_r2(A, T, R, cand, A.s3_stage != 0u, &W0);
  if (!(A.debug & 8u)) crc_expand_lds<kPT>(&S.t8[0][0], reinterpret_cast<const u32*>(&S.img[0][0][0]));
  if (cand) rec_place(W0, R, Z.pos, Z.off, Z.dead, Z.lm, Z.rk, Z.rel16);
  __syncthreads();
  PIPE_STAMP(1);
  while (task < tasks) {
    uint4 so;
    PIPE_STAMP(2);
    stage3_finish<XR>(A, S, T, R, Z, cand, so);
    if (lane == 0) G.stats[T.jb][task - G.task0[T.jb]] = so;
    PIPE_STAMP(3);
    task += A.wg3 * kPW;
    if (task < tasks) {
      T = task_pos(G, task);
      R = stage3_r1(A, T);
      cand = stage3_cand(A, T, R);
      Z = stage3_r2(A, T, R, cand, A.s3_stage != 0u);
    }
  }
  if (A.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PIPE_STAMP(6);
  if (A.steal && A.g1.nb && !(A.debug & 16u)) {  // out of tasks: rank tiles of the launch's group
    __syncthreads();  // every wave is done with the stage-3 LDS
    stage1_tiles(A, smem_raw, 0, true);
  }
}

#ifdef RMQ_PIPE_XR_TU
// the kernel with a replication transport (engine.cpp sizes its roles for kPipeThreadsXR)
void launch_pipeline_xr(const PipeArgs& a, hipStream_t s, hipEvent_t start) {
  const u32 grid = a.wg1 + a.wg2 + a.wgp + a.wg3 + a.wgb + a.wgc;
  hipExtLaunchKernelGGL(pipeline_kernel<true>, dim3(grid), dim3(kPT), kSmemBytes, s, start, nullptr, 0, a);
}
#else
uint32_t pipeline_wgs_per_cu(uint32_t threads) { return RMQ_PIPE_WAVES_PER_SIMD * 4u / (threads / 64u); }

void launch_pipeline(const PipeArgs& a, hipStream_t s, hipEvent_t start) {
  const u32 grid = a.wg1 + a.wg2 + a.wgp + a.wg3 + a.wgb + a.wgc;
  if (!grid) {
    if (start) (void)hipEventRecord(start, s);
    return;
  }
  if (a.outidx)
    rmq_x::launch_pipeline_xr(a, s, start);
  else
    hipExtLaunchKernelGGL(pipeline_kernel<false>, dim3(grid), dim3(kPT), kSmemBytes, s, start, nullptr, 0, a);
}
#endif

}  // namespace RMQ_PIPE_NS
