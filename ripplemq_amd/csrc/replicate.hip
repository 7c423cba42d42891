// replicate.hip — the follower side of a replica-log round (FORMAT.md §9).
//
// Reference: jraft replicates every partition log to its RF-1 followers with AppendEntries; a
// follower appends the entries after checking that they continue its log (Raft log matching) and
// acknowledges the index it now holds, which the leader's BallotBox turns into the commit index
// (PartitionRaftServer.java:82-93 configures the group; MessageAppendRequestProcessor.java:59 is
// the Node.apply that starts it). Here a round carries one launch group of the leader's appends
// for every partition the two ranks share, as one region of the exchange:
//   ingest_prepare (thread per entry): the log end the entry continues — the follower's own, or,
//     when the round's first offset lies inside the follower's retained log below its end, that
//     offset and its position (the follower truncates its log to the leader's: Raft's follower
//     deletes the entries that conflict with the leader's; the position comes from the sparse
//     index and a walk over the follower's record headers). An entry whose leader term is older
//     than the follower's is refused (a stale leader);
//   ingest_records (wave per 32 records, a lane pair per record, like the append's stage 3):
//     checks the record continues the follower's log (first offset == follower log end, header
//     offset == first offset + rank), recomputes its CRC32C from the payload pieces (slicing-by-8
//     and zero-shift tables in LDS, Horner fold per lane, the pad removed by x^(-8 pad)) against
//     the header's, and stores the record into the follower's replica ring at the same logical
//     position the leader used (pieces a later piece of the round overwrites are not stored), plus
//     the sparse-index entries;
//   ingest_finish (thread per entry): moves the follower partition's log end (both state sets:
//     the append pipeline never touches a partition it does not lead), adopts a newer leader term,
//     evaluates retention once per round (FORMAT.md §4 rule) and writes the ack (the follower's
//     log end, 0 when the entry does not continue it) for the leader.
// A refused entry (CRC, log mismatch or stale term) leaves the follower's log end where it was.
#include "device_common.hpp"
#include "kernels.hpp"
#include "partition_ops.hpp"

namespace rmq {

constexpr u32 kIT = 512;           // threads per ingest workgroup
constexpr u32 kIW = kIT / 64;      // waves = tasks per workgroup
constexpr u32 kIR = 32;            // records per task
constexpr u32 kBigIngest = 64;     // records over this many 16-byte pieces: the whole wave

struct RegionView {
  const uint8_t* base;
  u32 n_entries, n_records;
  u64 data_off;
};

__device__ __forceinline__ RegionView region_of(const IngestArgs& A, u32 src) {
  RegionView v;
  v.base = A.inbox + A.region[src];
  const u32* h = reinterpret_cast<const u32*>(v.base);
  v.n_entries = h[1];
  v.n_records = h[2];
  v.data_off = *reinterpret_cast<const u64*>(h + 6);
  return v;
}

__device__ __forceinline__ u32 source_of_task(const IngestArgs& A, u32 task) {
  u32 q = 0;
  for (u32 k = 1; k < A.world; ++k) q += task >= A.task0[k] ? 1u : 0u;
  return q;
}

// Directory entry k of a region: {count, bytes / 16, first offset} and the leader's term.
struct DirView {
  u32 count, bytes16, tstart, dstart16;
  u64 first, term;
};
__device__ __forceinline__ DirView dir_of(const RegionView& R, u32 k) {
  const uint4* de = reinterpret_cast<const uint4*>(R.base + kRegionHdr + (u64)kDirEntry * k);
  const uint4 d0 = de[0], d1 = de[1];
  DirView d;
  d.count = d0.x;
  d.bytes16 = d0.y;
  d.first = ((u64)d0.w << 32) | d0.z;
  d.tstart = d1.x;
  d.dstart16 = d1.y;
  d.term = ((u64)d1.w << 32) | d1.z;
  return d;
}

__device__ __forceinline__ u32 source_of_entry(const IngestArgs& A, u32 e) {
  u32 src = 0;
  for (u32 q = 1; q < A.world; ++q) src += e >= A.xi_start[q] ? 1u : 0u;
  return src;
}

// Logical position of offset t (start_off <= t <= leo) in the follower's log of partition p, read
// from replica slot `slot`: the largest live index entry at or below t, then the record headers
// (FORMAT.md §5 lookup).
__device__ u64 follower_pos(const DevState& st, u32 p, u32 slot, u64 t) {
  const RingRef rg = ring_ref(st, p);
  const u32 ilog = st.interval_log2;
  u64 off = st.start_off[p], pos = st.start_pos[p];
  u64 lo = (pos + (1ull << ilog) - 1) >> ilog, hi = (st.used[p] >> ilog) + 1;  // live m in [lo, hi)
  while (lo < hi) {
    const u64 mid = lo + (hi - lo) / 2;
    const u64* ie = st.index + (rg.ibase + mid % rg.icap) * 2;
    if (ie[0] <= t) {
      if (ie[0] >= off) {
        off = ie[0];
        pos = ie[1];
      }
      lo = mid + 1;
    } else {
      hi = mid;
    }
  }
  const uint8_t* ring = st.logs + (u64)slot * st.rstride + rg.base;
  for (; off < t; ++off) {
    const u32 L = *reinterpret_cast<const u32*>(ring + ((pos + 8ull) & (rg.seg - 1ull)));
    pos += 16ull + ((L + 15ull) & ~15ull);
  }
  return pos;
}

__global__ void ingest_prepare_kernel(IngestArgs A) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= A.n_in) return;
  const u32 src = source_of_entry(A, e), k = e - A.xi_start[src];
  const DevState& st = A.st;
  const u32 p = A.xi_p[e];
  u64 leo = st.leo[p], used = st.used[p];
  A.bad[e] = 0u;  // this round's verdict starts clean (the finish kernel only reads it)
  if (A.rbytes[src]) {
    const RegionView R = region_of(A, src);
    if (R.n_entries == A.xi_start[src + 1] - A.xi_start[src]) {
      const DirView d = dir_of(R, k);
      if (d.term < st.term[p]) {
        A.bad[e] = 4u;  // a stale leader
      } else if (d.first < leo && d.first >= st.start_off[p]) {
        used = follower_pos(st, p, A.xi_slot[e], d.first);  // the leader's log wins: truncate
        leo = d.first;
      }
    }
  }
  A.base[2 * e] = leo;
  A.base[2 * e + 1] = used;
}

__global__ __launch_bounds__(kIT) void ingest_records_kernel(IngestArgs A) {
  __shared__ __attribute__((aligned(16))) u32 t8[8][256];
  __shared__ __attribute__((aligned(16))) u32 z[2][4][256];
  __shared__ __attribute__((aligned(16))) u32 zk[4][256];  // 1 KB shift: records over 1 KB, by the wave
  {
    static_assert(offsetof(CrcConsts, zshift) == sizeof(A.crc->table), "table and zshift adjacent");
    static_assert(offsetof(CrcConsts, zshift1k) == offsetof(CrcConsts, zshift) + sizeof(A.crc->zshift), "zshift1k next");
    const uint4* src = reinterpret_cast<const uint4*>(&A.crc->table[0][0]);
    uint4* d0 = reinterpret_cast<uint4*>(&t8[0][0]);
    uint4* d1 = reinterpret_cast<uint4*>(&z[0][0][0]);
    uint4* d2 = reinterpret_cast<uint4*>(&zk[0][0]);
    for (u32 k = threadIdx.x; k < sizeof(t8) / 16; k += kIT) d0[k] = src[k];
    for (u32 k = threadIdx.x; k < sizeof(z) / 16; k += kIT) d1[k] = src[sizeof(t8) / 16 + k];
    for (u32 k = threadIdx.x; k < sizeof(zk) / 16; k += kIT) d2[k] = src[(sizeof(t8) + sizeof(z)) / 16 + k];
  }
  __syncthreads();
  const u32 task = __builtin_amdgcn_readfirstlane(blockIdx.x * kIW + (threadIdx.x >> 6));
  if (task >= A.task0[A.world]) return;
  const u32 src = source_of_task(A, task);
  if (!A.rbytes[src]) return;
  const RegionView R = region_of(A, src);
  if (R.n_entries != A.xi_start[src + 1] - A.xi_start[src]) return;  // malformed (finish counts it)
  const u32 lane = threadIdx.x & 63, j = lane & 1u;
  const u32 i = (task - A.task0[src]) * kIR + (lane >> 1);
  const bool in = i < R.n_records;
  const DevState& st = A.st;
  u32 p = 0, L = 0, m = 0, e = 0;
  u64 pos = 0, gend = 0, off = 0;
  bool ok = false, owner = false;
  const uint8_t* rec = R.base;
  uint4 hdr = make_uint4(0, 0, 0, 0);
  if (in) {
    const u64 tab = *reinterpret_cast<const u64*>(R.base + kRegionHdr + (u64)kDirEntry * R.n_entries + 8ull * i);
    const u32 k = min((u32)tab, R.n_entries - 1u), d16 = (u32)(tab >> 32);  // ok below requires k == tab
    const DirView d = dir_of(R, k);
    const u32 bytes16 = d.bytes16, tstart = d.tstart, dstart16 = d.dstart16;
    const u64 first = d.first;
    e = A.xi_start[src] + k;
    p = A.xi_p[e];
    owner = k == 0 || A.xi_p[e - 1] != p;  // two local slots of one partition: the first owns the state
    const u64 leo = A.base[2 * e], used = A.base[2 * e + 1];  // after a truncation: the leader's first offset
    rec = R.base + R.data_off + 16ull * d16;
    hdr = *reinterpret_cast<const uint4*>(rec);
    off = ((u64)hdr.y << 32) | hdr.x;
    L = hdr.z;
    m = (L + 15u) >> 4;
    const u64 rel = 16ull * (d16 - dstart16);
    pos = used + rel;
    gend = used + 16ull * bytes16;
    ok = k == (u32)tab && first == leo && off == first + (i - tstart) && d16 >= dstart16 &&
         rel + 16ull * (1ull + m) <= 16ull * bytes16 && !(A.bad[e] & 4u);
    if (!ok && j == 1) atomicOr(&A.bad[e], 2u);  // does not continue the follower's log
  }
  // CRC32C of the payload from its 16-byte pieces (zero-padded in the log): lane j folds pieces
  // j, j + 2, ... by Horner's rule with the 32-byte zero-shift table; records over 1 KB are done
  // by the whole wave below
  const bool big = ok && m > kBigIngest;
  const u32 mm = ok && !big ? m : 0u;
  u32 acc = 0;
  const RingRef rg = ring_ref(st, p);  // p = 0 for lanes without a record (nothing is stored)
  uint8_t* const ring = st.logs + (u64)(in ? A.xi_slot[e] : 0u) * st.rstride + rg.base;
  const u64 segmask = rg.seg - 1ull;
  for (u32 c = 0; __any(c < (mm + 1u) / 2u); ++c) {
    const u32 jp = 2u * c + j;
    if (jp < mm) {
      uint4 v = *reinterpret_cast<const uint4*>(rec + 16ull + 16ull * jp);
      const u64 x = pos + 16ull + 16ull * jp;
      if (x + rg.seg >= gend) store_log16(ring + (x & segmask), v);
      if (jp == 0) v.x ^= 0xFFFFFFFFu;
      acc = crc_zshift(z[1], acc) ^ crc_piece16(t8, v);
    }
  }
  if (ok && mm > j && ((mm - 1u - j) & 1u)) acc = crc_zshift(z[0], acc);
  acc ^= pair_swap(acc);
  // records over 1 KB, one at a time by the wave: lane l takes pieces l, l + 64, ... (Horner with
  // the 1 KB shift), shifts past the pieces after its last one, XOR-reduce; the record's lane 1
  // gets the register
  for (u64 bm = __ballot(j == 0 && big); bm; bm &= bm - 1ull) {
    const u32 sl = (u32)__builtin_ctzll(bm);
    const u64 brec = ((u64)(u32)__builtin_amdgcn_readlane((int)(reinterpret_cast<u64>(rec) >> 32), (int)sl) << 32) |
                     (u32)__builtin_amdgcn_readlane((int)(u32)reinterpret_cast<u64>(rec), (int)sl);
    const u64 bpos = ((u64)(u32)__builtin_amdgcn_readlane((int)(pos >> 32), (int)sl) << 32) |
                     (u32)__builtin_amdgcn_readlane((int)(u32)pos, (int)sl);
    const u64 bgend = ((u64)(u32)__builtin_amdgcn_readlane((int)(gend >> 32), (int)sl) << 32) |
                      (u32)__builtin_amdgcn_readlane((int)(u32)gend, (int)sl);
    const u64 bring = ((u64)(u32)__builtin_amdgcn_readlane((int)(reinterpret_cast<u64>(ring) >> 32), (int)sl) << 32) |
                      (u32)__builtin_amdgcn_readlane((int)(u32)reinterpret_cast<u64>(ring), (int)sl);
    const u32 bm16 = ((u32)__builtin_amdgcn_readlane((int)L, (int)sl) + 15u) >> 4;
    const u64 bseg = ((u64)(u32)__builtin_amdgcn_readlane((int)(rg.seg >> 32), (int)sl) << 32) |
                     (u32)__builtin_amdgcn_readlane((int)(u32)rg.seg, (int)sl);
    u32 bacc = 0;
    for (u32 k0 = 0; 64u * k0 < bm16; k0 += 4u) {
      uint4 v[4];
#pragma unroll
      for (u32 u = 0; u < 4u; ++u) {
        const u32 jp = 64u * (k0 + u) + lane;
        v[u] = jp < bm16 ? *reinterpret_cast<const uint4*>(brec + 16ull + 16ull * jp) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (u32 u = 0; u < 4u; ++u) {
        const u32 jp = 64u * (k0 + u) + lane;
        if (jp < bm16) {
          const u64 x = bpos + 16ull + 16ull * jp;
          if (x + bseg >= bgend) store_log16(reinterpret_cast<uint8_t*>(bring) + (x & (bseg - 1ull)), v[u]);
          uint4 w = v[u];
          if (jp == 0) w.x ^= 0xFFFFFFFFu;
          bacc = crc_zshift(zk, bacc) ^ crc_piece16(t8, w);
        }
      }
    }
    if (lane < bm16) {
      const u32 eb = (bm16 - 1u - lane) & 63u;
      if (eb) bacc = gf2_mulmod(bacc, A.crc->sh16[eb]);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) bacc ^= (u32)__shfl_xor((int)bacc, d, 64);
    if (lane == sl + 1u) acc = bacc;
  }
  if (ok && j == 1) {
    u32 crc = 0;
    if (L) {
      const u32 pad = 16u * m - L;
      crc = ~(pad ? gf2_mulmod(A.crc->inv_pad[pad], acc) : acc);
    }
    ok = crc == hdr.w;
    if (ok) {
      if (pos + rg.seg >= gend) store_log16(ring + (pos & segmask), hdr);
      if (owner) {  // sparse index: every multiple of the interval the record crosses names the next record
        const u32 ilog = st.interval_log2;
        const u64 end = pos + 16ull * (1ull + m);
        for (u64 q = (pos >> ilog) + 1; (q << ilog) <= end; ++q) {
          u64* ie = st.index + (rg.ibase + q % rg.icap) * 2;
          ie[0] = off + 1;
          ie[1] = end;
        }
      }
    } else {
      atomicOr(&A.bad[e], 1u);  // CRC32C differs from the header's
    }
  }
  const u32 n_ok = (u32)__popcll(__ballot(in && ok && j == 1));
  if (lane == 0 && n_ok) atomicAdd((unsigned long long*)&A.counters[0], (unsigned long long)n_ok);
}

__global__ void ingest_finish_kernel(IngestArgs A) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= A.n_in) return;
  const u32 src = source_of_entry(A, e);
  const DevState& st = A.st;
  const u32 p = A.xi_p[e], k = e - A.xi_start[src];
  const bool owner = k == 0 || A.xi_p[e - 1] != p;
  u64 ack = st.leo[p];  // no region from this leader: nothing new
  const bool whole = A.rbytes[src] && region_of(A, src).n_entries == A.xi_start[src + 1] - A.xi_start[src];
  if (A.rbytes[src] && !whole) {
    ack = 0;
    if (k == 0) atomicAdd((unsigned long long*)&A.counters[2], 1ull);
  } else if (A.rbytes[src]) {
    const DirView d = dir_of(region_of(A, src), k);
    // two local slots of one partition (adjacent entries of the same source): the owner keeps the
    // partition's state, so a refusal of either is a refusal of both (no slot acks records the
    // follower's log end does not hold)
    u32 bad = A.bad[e];
    for (u32 q = e; q > A.xi_start[src] && A.xi_p[q - 1] == p; --q) bad |= A.bad[q - 1] ? 8u : 0u;
    for (u32 q = e + 1; q < A.xi_start[src + 1] && A.xi_p[q] == p; ++q) bad |= A.bad[q] ? 8u : 0u;
    const u64 bleo = A.base[2 * e], bused = A.base[2 * e + 1];
    if (bad) {
      ack = 0;  // no new information (match only moves up)
      if (bad & 7u) atomicAdd((unsigned long long*)&A.counters[(bad & 6u) ? 2 : 1], 1ull);
    } else {
      // the entry continues the log at bleo (or does not: a follower behind the leader acks 0)
      const bool cont = d.first == bleo;
      ack = d.count ? d.first + d.count : (cont ? bleo : 0ull);
      if (owner) {
        if (d.term > st.term[p]) st.term[p] = d.term;
        const u64 nleo = d.count ? ack : bleo, nused = bused + 16ull * d.bytes16;
        for (u32 s = 0; s < 2; ++s) {
          A.sets[s].leo[p] = nleo;
          A.sets[s].used[p] = nused;
        }
        if (d.count) {
          // retention once per round (FORMAT.md §4 rule on the follower's log)
          const RingRef rg = ring_ref(st, p);
          if (nused - st.start_pos[p] > rg.seg) {
            const u64 ms = (nused - rg.seg + (1ull << st.interval_log2) - 1) >> st.interval_log2;
            const u64* ie = st.index + (rg.ibase + ms % rg.icap) * 2;
            st.start_off[p] = ie[0];
            st.start_pos[p] = ie[1];
          }
          atomicAdd((unsigned long long*)&A.counters[3], 16ull * d.bytes16);
        }
      }
    }
  }
  A.ackout[e] = ack;
}

// Acks of one round applied after the pipeline has drained (thread per partition).
__global__ void ack_apply_kernel(AckApplyArgs a) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  const DevState& st = a.st;
  if (p >= st.P || !st.is_leader[p]) return;
  u64 row[kMaxRF];
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) row[r] = r < st.RF ? st.match[(u64)p * st.RF + r] : 0ull;
  if (apply_acks(st, p, a.outidx, a.ackin, st.leo[p], row)) {
    const u64 c = quorum_commit(row, st.RF, st.commit[p], st.term_start[p]);
    st.commit[p] = c;
    st.hw[p] = c;
  }
}

void launch_ingest(const IngestArgs& a, uint32_t tasks, hipStream_t s) {
  if (a.n_in) hipLaunchKernelGGL(ingest_prepare_kernel, dim3((a.n_in + 255) / 256), dim3(256), 0, s, a);
  if (tasks) hipLaunchKernelGGL(ingest_records_kernel, dim3((tasks + kIW - 1) / kIW), dim3(kIT), 0, s, a);
  if (a.n_in) hipLaunchKernelGGL(ingest_finish_kernel, dim3((a.n_in + 255) / 256), dim3(256), 0, s, a);
}

void launch_ack_apply(const AckApplyArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ack_apply_kernel, dim3((a.st.P + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace rmq
