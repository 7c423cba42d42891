// replicate.hip — the follower side of a replica-log round (FORMAT.md §9 v3).
//
// Reference: jraft replicates every partition log to its RF-1 followers with AppendEntries; a
// follower appends the entries after checking that they continue its log (Raft log matching) and
// acknowledges the index it now holds, which the leader's BallotBox turns into the commit index
// (PartitionRaftServer.java:82-93 configures the group; MessageAppendRequestProcessor.java:59 is
// the Node.apply that starts it); consumer-offset commits are log entries too, applied on every
// replica (ConsumerOffsetUpdateRequestProcessor.java:59-60, PartitionStateMachine.java:48-49). Here
// a round carries one launch group of the leader's appends (and any catch-up gap) for every
// partition the two ranks share, as one region of the exchange, plus the changed consumer-offset
// rows. Three launches, in order on the exchange stream (finish and copy share the last one: both
// only read verify's verdicts):
//   ingest_prepare (thread per entry): the log end the entry continues — the follower's own, or,
//     when the entry's first offset lies inside the follower's retained log below its end, that
//     offset and its position (truncation: the leader's log wins; the position from the sparse
//     index and the record headers). A stale leader term or a missed round (no region) refuses it;
//   ingest_verify (wave per 64 records, a lane per record, records over 1 KB by the whole wave;
//     RMQ_VERIFY_LANE=0: 32 records, a lane pair each): the record continues the entry (header
//     offset = first + rank, inside the entry's bytes) and its CRC32C from the 16-byte payload
//     pieces (slicing-by-8 tables in LDS, the pad removed by x^(-8 pad)) equals the header's; sparse-index
//     entries past the follower's live log (slots no live entry uses). Nothing else is written;
//   ingest_finish (thread per entry): the verdict — a refusal of either of two local slots of one
//     partition refuses both — then for an accepted entry the follower's log end (both state sets:
//     the append pipeline never touches a partition it does not lead), a newer term, the index
//     entries a truncation re-covers, retention once per round (FORMAT.md §4 rule) and the
//     consumer-offset row; every entry acks {log end | status, position};
//   ingest_copy (wave per 16 KiB of an entry): the accepted entries' record bytes, whole
//     16-byte pieces, into the follower's replica ring at the leader's logical positions (pieces a
//     later piece of the round overwrites are not stored). A refused entry writes nothing.
#include "device_common.hpp"
#include "kernels.hpp"
#include "partition_ops.hpp"


namespace rmq {

constexpr u32 kIT = 512;           // threads per verify workgroup
constexpr u32 kIW = kIT / 64;      // waves = tasks per workgroup
#ifndef RMQ_VERIFY_LANE
#define RMQ_VERIFY_LANE 1
#endif
// verify: a lane per record (a task = 64 records: one resident generation of waves for a round of
// 2 x 262,144 records) or a lane pair per record (RMQ_VERIFY_LANE=0: 32 records per task)
constexpr u32 kIR = RMQ_VERIFY_LANE ? 64 : 32;  // records per task
#ifndef RMQ_VSPEC
#define RMQ_VSPEC (RMQ_VERIFY_LANE ? 4 : 2)  // (more spills at 8 waves per SIMD)
#endif
#ifndef RMQ_VERIFY_WAVES
#define RMQ_VERIFY_WAVES 8
#endif
constexpr u32 kVSpec = RMQ_VSPEC;    // pieces per lane loaded with the table slot (0..4)
static_assert(kVSpec <= 4, "at most four speculative pieces per lane");
#ifndef RMQ_ENTRY_THREADS
#define RMQ_ENTRY_THREADS 256
#endif
// threads per prepare / finish workgroup (a thread per entry; one-wave workgroups, spreading a
// round's entries over more CUs, measured the same: 1.554 vs 1.550 G in the rehearsal, round 4)
constexpr u32 kEntryT = RMQ_ENTRY_THREADS;
static_assert(kEntryT % 64 == 0, "whole waves (finish sums its counters per wave)");
constexpr u32 kBigIngest = 64;     // records over this many 16-byte pieces: the whole wave
constexpr u32 kCT = 64;            // threads per copy workgroup (one wave: many items resident per CU)

struct RegionView {
  const uint8_t* base;
  u32 n_entries, n_records, M, C;
  u64 data_off, rows_off;
  bool sane;
};

// The region of source src in this round's inbox (FORMAT.md §9 header), checked against the
// entry list both sides derive from the placement (count and key sum) and against its own size:
// the sections lie where the format puts them, inside the region. A region failing this is
// unreadable (every entry refused, like a missed round).
__device__ __forceinline__ RegionView region_of(const IngestArgs& A, u32 src) {
  RegionView v;
  v.base = A.inbox + A.region[src];
  const u64 size = A.rbytes[src];
  v.sane = size >= kRegionHdr;
  const u32* h = reinterpret_cast<const u32*>(v.base);
  v.n_entries = v.sane ? h[1] : 0u;
  v.n_records = v.sane ? h[2] : 0u;
  v.data_off = v.sane ? *reinterpret_cast<const u64*>(h + 6) : 0ull;
  v.rows_off = v.sane ? *reinterpret_cast<const u64*>(h + 8) : 0ull;
  v.M = v.sane ? h[10] : 0u;
  v.C = v.sane ? h[11] : 0u;
  if (v.sane) {
    const u64 tab = kRegionHdr + (u64)kDirEntry * v.n_entries, rowb = 16ull + 8ull * A.C;
    v.sane = h[0] == kXMagic && v.n_entries == A.xi_start[src + 1] - A.xi_start[src] && h[3] == src &&
             *reinterpret_cast<const u64*>(h + 4) == A.keysum_in[src] && v.C == A.C &&
             v.data_off == tab + ((8ull * v.n_records + 15ull) & ~15ull) && v.rows_off >= v.data_off &&
             v.rows_off <= size && !((v.rows_off - v.data_off) & 15ull) && v.M <= v.n_entries &&
             (size - v.rows_off) / rowb >= v.M;
  }
  return v;
}

__device__ __forceinline__ u32 source_of_task(const IngestArgs& A, u32 task) {
  u32 q = 0;
  for (u32 k = 1; k < A.world; ++k) q += task >= A.task0[k] ? 1u : 0u;
  return q;
}

// Directory entry k of a region: {count, bytes / 16, first offset}, the leader's term and whether
// the entry restarts the follower's log (a rebase, FORMAT.md §9: flag in the term's top bit).
struct DirView {
  u32 count, bytes16, tstart, dstart16;
  u64 first, term, commit;
  u64 lterm;  // (v5) the term of the entry's last entry the follower may count (0: older, unknown)
  bool rebase;
};
__device__ __forceinline__ DirView dir_of(const RegionView& R, u32 k) {
  const uint4* de = reinterpret_cast<const uint4*>(R.base + kRegionHdr + (u64)kDirEntry * k);
  const uint4 d0 = de[0], d1 = de[1], d2 = de[2];
  DirView d;
  d.count = d0.x;
  d.bytes16 = d0.y;
  d.first = ((u64)d0.w << 32) | d0.z;
  d.tstart = d1.x;
  d.dstart16 = d1.y;
  d.term = ((u64)d1.w << 32) | d1.z;
  d.commit = ((u64)d2.y << 32) | d2.x;  // the leader's commit (v4)
  d.lterm = ((u64)d2.w << 32) | d2.z;   // (v5)
  d.rebase = (d.term & kTermRebase) != 0ull;
  d.term &= ~kTermRebase;
  return d;
}

// The consumer-offset row of entry k (rows ascend by entry), or null.
__device__ __forceinline__ const uint8_t* row_of(const RegionView& R, u32 C, u32 k) {
  const u64 rowb = 16ull + 8ull * C;
  u32 lo = 0, hi = R.M;
  while (lo < hi) {
    const u32 mid = (lo + hi) / 2;
    const u32 rk = *reinterpret_cast<const u32*>(R.base + R.rows_off + rowb * mid);
    if (rk < k) lo = mid + 1; else hi = mid;
  }
  if (lo < R.M && *reinterpret_cast<const u32*>(R.base + R.rows_off + rowb * lo) == k)
    return R.base + R.rows_off + rowb * lo;
  return nullptr;
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

constexpr u32 kBadCrc = 1u, kBadLog = 2u, kBadStale = 4u, kBadMissed = 8u;
constexpr u32 kBadUnread = 16u;  // (with kBadLog) the region's header is unreadable: nothing heard from the leader

// A structural fault of source src's region this round (FORMAT.md §9: directory entries that do
// not tile the table and data sections, a table slot outside its entry, rows out of order): every
// entry of the region is refused.
__device__ __forceinline__ void mark_insane(const IngestArgs& A, u32 src) {
  __hip_atomic_fetch_or(&A.insane[src], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void ingest_prepare_kernel(IngestArgs A) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = e < A.n_in;
  // the next round's counters (the round before used them; its kernels ran before this one)
  static_assert(1 + kMaxWorld <= kEntryT, "one workgroup clears them");
  if (blockIdx.x == 0 && threadIdx.x < 1 + kMaxWorld) A.n_items_next[threadIdx.x] = 0u;
  u32 nc = 0;  // copy work items of the entry
  if (in) {
    const u32 src = source_of_entry(A, e), k = e - A.xi_start[src];
    const DevState& st = A.st;
    const u32 p = A.xi_p[e];
    u64 leo = st.leo[p], used = st.used[p];
    u32 bad = 0;
    if (!A.rbytes[src]) {
      bad = kBadMissed;  // the leader sent nothing this round (it failed before replicating)
    } else {
      const RegionView R = region_of(A, src);
      if (!R.sane) {
        bad = kBadLog | kBadUnread;
      } else {
        const DirView d = dir_of(R, k);
        // the entry's slice of the table and of the data section ends where the next entry's
        // starts (the last: at the section ends), the first starts at 0; rows ascend by entry
        const bool last = k + 1u == R.n_entries;
        const DirView dn = dir_of(R, last ? k : k + 1u);
        const u64 t_end = last ? (u64)R.n_records : (u64)dn.tstart;
        const u64 d_end = last ? (R.rows_off - R.data_off) >> 4 : (u64)dn.dstart16;
        bool tiled = (u64)d.tstart + d.count == t_end && (u64)d.dstart16 + d.bytes16 == d_end;
        if (k == 0) tiled = tiled && d.tstart == 0u && d.dstart16 == 0u;
        if (k < R.M) {
          const u64 rowb = 16ull + 8ull * A.C;
          const u32 rk = *reinterpret_cast<const u32*>(R.base + R.rows_off + rowb * k);
          const u32 pk = k ? *reinterpret_cast<const u32*>(R.base + R.rows_off + rowb * (k - 1u)) : 0u;
          tiled = tiled && rk < R.n_entries && (k == 0 || pk < rk);
        }
        if (!tiled) mark_insane(A, src);
        if (d.term < st.term[p]) {
          bad = kBadStale;  // a stale leader
        } else if (d.rebase) {  // the log restarts at the entry's first record (its row: the position)
          const uint8_t* row = row_of(R, A.C, k);
          if (row) {
            leo = d.first;
            used = *reinterpret_cast<const u64*>(row + 8);
          } else {
            bad = kBadLog;  // malformed: a rebase entry always carries its row
          }
        } else if (d.first < leo && d.first >= st.start_off[p]) {
          used = follower_pos(st, p, A.xi_slot[e], d.first);  // the leader's log wins: truncate
          leo = d.first;
        }
        if (!bad && d.first != leo) bad = kBadLog;  // does not continue the follower's log
        if (!bad && !d.count && d.bytes16) bad = kBadCrc;  // bytes without records
        // copy items only for an entry whose bytes tile the data section (so the items of a round
        // stay within the host's bound: one per 16 KiB of received bytes plus one per entry)
        if (!bad && tiled) {
          nc = (u32)((16ull * d.bytes16 + kCopyChunk - 1) / kCopyChunk);
          // the copy's addresses, so its workgroups start their data loads after two lookups
          const RingRef rg = ring_ref(st, p);
          u64* cd = A.cdesc + 4ull * e;
          cd[0] = reinterpret_cast<u64>(R.base + R.data_off + 16ull * d.dstart16);
          cd[1] = reinterpret_cast<u64>(st.logs + (u64)A.xi_slot[e] * st.rstride + rg.base);
          cd[2] = used;
          cd[3] = (16ull * d.bytes16) << 6 | (u64)(63 - __builtin_clzll(rg.seg));
        }
      }
    }
    A.bad[e] = bad;
    A.base[2 * e] = leo;
    A.base[2 * e + 1] = used;
  }
  // the items' slots (their order does not matter): one counter add per wave; slots past the
  // capacity are not written (only a corrupted region can ask for them: finish refuses the round)
  const u32 inc = wave_incl_scan(nc);
  const u32 tot = (u32)__builtin_amdgcn_readlane((int)inc, 63);
  u32 at = 0;
  if (lane_id() == 0 && tot) at = atomicAdd(A.n_items, tot);
  at = (u32)__builtin_amdgcn_readlane((int)at, 0);
  // the wave writes its items together (an entry of many chunks would otherwise keep one lane
  // busy): item i belongs to the lane whose inclusive count first exceeds i (all lanes take part
  // in every shuffle)
  for (u32 b = 0; b < tot; b += 64) {
    const u32 i = b + lane_id();
    u32 lo = 0;
#pragma unroll
    for (u32 step = 32; step; step >>= 1) {
      const u32 v = (u32)__shfl((int)inc, (int)(lo + step - 1u), 64);
      if (v <= i) lo += step;
    }
    const u32 own_inc = (u32)__shfl((int)inc, (int)lo, 64), own_nc = (u32)__shfl((int)nc, (int)lo, 64);
    const u32 own_e = (u32)__shfl((int)e, (int)lo, 64);
    if (i < tot && at + i < A.items_cap) {
      A.items[2 * (at + i)] = own_e;
      A.items[2 * (at + i) + 1] = i - (own_inc - own_nc);
    }
  }
}

// One task (32 records of one source region) of the verify kernel, by one wave.
__device__ __forceinline__ void verify_task(const IngestArgs& A, const u32 (*t8)[256], const u32 (*z32)[256], u32 task) {
  const u32 src = source_of_task(A, task);
  if (!A.rbytes[src]) return;
  const RegionView R = region_of(A, src);
  if (!R.sane) return;  // every entry refused (prepare)
  const u32 lane = threadIdx.x & 63, j = lane & 1u;
  const u32 i = (task - A.task0[src]) * kIR + (lane >> 1);
  const bool in = i < R.n_records;
  const DevState& st = A.st;
  u32 p = 0, L = 0, m = 0, e = 0;
  u64 pos = 0, off = 0;
  bool ok = false, owner = false, reb = false;
  const uint8_t* rec = R.base;
  uint4 hdr = make_uint4(0, 0, 0, 0);
  // the header and this lane's first four pieces are loaded with the directory entry, from the
  // table slot alone (inside the data section; used only once the checks below pass): one round
  // trip instead of three (directory, then header, then payload)
  uint4 sp0 = make_uint4(0, 0, 0, 0), sp1 = sp0, sp2 = sp0, sp3 = sp0;
  if (in) {
    const u64* tabp = reinterpret_cast<const u64*>(R.base + kRegionHdr + (u64)kDirEntry * R.n_entries) + i;
    const u64 tab = tabp[0];
    const u64 tabn = i + 1u < R.n_records ? tabp[1] : 0ull;  // the next slot (the record after, if any)
    const u32 k = min((u32)tab, R.n_entries - 1u), d16 = (u32)(tab >> 32);  // ok below requires k == tab
    rec = R.base + R.data_off + 16ull * d16;
    const u64 dsz16 = (R.rows_off - R.data_off) >> 4;  // pieces in the data section
    uint4 sh = make_uint4(0, 0, 0, 0);
    if ((u64)d16 + 1ull <= dsz16) sh = *reinterpret_cast<const uint4*>(rec);
    if (kVSpec > 0 && (u64)d16 + 2ull + j <= dsz16) sp0 = *reinterpret_cast<const uint4*>(rec + 16ull + 16ull * j);
    if (kVSpec > 1 && (u64)d16 + 4ull + j <= dsz16) sp1 = *reinterpret_cast<const uint4*>(rec + 48ull + 16ull * j);
    if (kVSpec > 2 && (u64)d16 + 6ull + j <= dsz16) sp2 = *reinterpret_cast<const uint4*>(rec + 80ull + 16ull * j);
    if (kVSpec > 3 && (u64)d16 + 8ull + j <= dsz16) sp3 = *reinterpret_cast<const uint4*>(rec + 112ull + 16ull * j);
    const DirView d = dir_of(R, k);
    // structure: the slot lies in the range of the entry it names (prepare checked that the ranges
    // tile the table)
    const bool named = k == (u32)tab && i >= d.tstart && (u64)i < (u64)d.tstart + d.count;
    if (!named && j == 1) mark_insane(A, src);
    e = A.xi_start[src] + k;
    p = A.xi_p[e];
    owner = k == 0 || A.xi_p[e - 1] != p;  // two local slots of one partition: the first owns the state
    reb = d.rebase;
    const u64 used = A.base[2 * e + 1];   // after a truncation: at the leader's first offset
    const u64 rel = 16ull * (u64)(d16 - d.dstart16);
    if (k == (u32)tab && d16 >= d.dstart16 && (u64)d16 + 1ull <= dsz16) {
      hdr = sh;
      off = ((u64)hdr.y << 32) | hdr.x;
      L = hdr.z;
      m = (L + 15u) >> 4;
    }
    pos = used + rel;
    // the record continues the entry (its directory verdict is prepare's): its offset, inside the
    // entry's bytes (which lie inside the data section), the first at the entry's start, each one
    // where the one before ends and the last at the entry's end (FORMAT.md §9)
    const u64 rend16 = (u64)d16 + 1ull + m;
    const bool last = (u64)i + 1ull == (u64)d.tstart + d.count;
    const bool chained = (i != d.tstart || d16 == d.dstart16) &&
                         (last ? rend16 == (u64)d.dstart16 + d.bytes16 : (u64)(u32)(tabn >> 32) == rend16);
    ok = named && d16 >= d.dstart16 && (u64)d.dstart16 + d.bytes16 <= (R.rows_off - R.data_off) >> 4 &&
         off == d.first + (i - d.tstart) && rel + 16ull * (1ull + m) <= 16ull * d.bytes16 && chained &&
         A.bad[e] == 0u;
    if (!ok && j == 1 && A.bad[e] == 0u) atomicOr(&A.bad[e], kBadCrc);  // the record's content is wrong
  }
  // CRC32C of the payload from its 16-byte pieces (zero-padded in the log): lane j folds pieces
  // j, j + 2, ... by Horner's rule with the 32-byte zero-shift table; records over 1 KB are done
  // by the whole wave below
  const bool big = ok && m > kBigIngest;
  const u32 mm = ok && !big ? m : 0u;
  u32 acc = 0;
  {  // pieces j, j + 2, ...: the speculative loads (inside the record once ok)
    const uint4 sv[4] = {sp0, sp1, sp2, sp3};
#pragma unroll
    for (u32 u = 0; u < kVSpec; ++u) {
      const u32 jp = 2u * u + j;
      if (jp < mm) {
        uint4 w = sv[u];
        if (jp == 0) w.x ^= 0xFFFFFFFFu;
        acc = crc_zshift(z32, acc) ^ crc_piece16(t8, w);
      }
    }
  }
  for (u32 c = kVSpec; __any(c < (mm + 1u) / 2u); c += 4) {
    uint4 v[4];
#pragma unroll
    for (u32 u = 0; u < 4; ++u) {  // four pieces in flight per lane
      const u32 jp = 2u * (c + u) + j;
      v[u] = jp < mm ? *reinterpret_cast<const uint4*>(rec + 16ull + 16ull * jp) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (u32 u = 0; u < 4; ++u) {
      const u32 jp = 2u * (c + u) + j;
      if (jp < mm) {
        uint4 w = v[u];
        if (jp == 0) w.x ^= 0xFFFFFFFFu;
        acc = crc_zshift(z32, acc) ^ crc_piece16(t8, w);
      }
    }
  }
  // the lane whose last piece is one short of the record's end: shift past those 16 bytes
  if (ok && mm > j && ((mm - 1u - j) & 1u)) acc = gf2_mulmod(acc, A.crc->sh16[1]);
  acc ^= pair_swap(acc);
  // records over 1 KB, one at a time by the wave: lane l takes pieces l, l + 64, ... (Horner with
  // the 1 KB shift), shifts past the pieces after its last one, XOR-reduce; the record's lane 1
  // gets the register
  for (u64 bm = __ballot(j == 0 && big); bm; bm &= bm - 1ull) {
    const u32 sl = (u32)__builtin_ctzll(bm);
    const u64 brec = ((u64)(u32)__builtin_amdgcn_readlane((int)(reinterpret_cast<u64>(rec) >> 32), (int)sl) << 32) |
                     (u32)__builtin_amdgcn_readlane((int)(u32)reinterpret_cast<u64>(rec), (int)sl);
    const u32 bm16 = ((u32)__builtin_amdgcn_readlane((int)L, (int)sl) + 15u) >> 4;
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
          uint4 w = v[u];
          if (jp == 0) w.x ^= 0xFFFFFFFFu;
          bacc = crc_zshift(A.crc->zshift1k, bacc) ^ crc_piece16(t8, w);  // (L1/L2-resident)
        }
      }
    }
    if (lane < bm16) {
      const u32 eb = (bm16 - 1u - lane) & 63u;
      if (eb) bacc = gf2_mulmod(bacc, A.crc->sh16[eb]);
    }
    bacc = wave_xor_all(bacc);
    if (lane == sl + 1u) acc = bacc;
  }
  if (ok && j == 1) {
    u32 crc = 0;
    if (L) {
      const u32 pad = 16u * m - L;
      crc = ~(pad ? gf2_mulmod(A.crc->inv_pad[pad], acc) : acc);
    }
    // the zero padding after the payload (FORMAT.md §1) is part of the record
    if (m && (L & 15u)) {
      const uint4 t = *reinterpret_cast<const uint4*>(rec + 16ull * m);  // the last piece
      const u32 nb = L & 15u;
      const u32 w4[4] = {t.x, t.y, t.z, t.w};
      for (u32 b = nb; b < 16u; ++b)
        if ((w4[b >> 2] >> (8u * (b & 3u))) & 0xFFu) crc = ~hdr.w;
    }
    if (crc == hdr.w) {
      // (a rebase entry's index entries are written by finish, once the entry is accepted: its
      // positions lie past the live log but may share index slots with it)
      if (owner && !reb) {
        // sparse index past the follower's live log: every interval multiple the record crosses
        const u32 ilog = st.interval_log2;
        const RingRef rg = ring_ref(st, p);
        const u64 end = pos + 16ull * (1ull + m), live = st.used[p] >> ilog;
        for (u64 q = (pos >> ilog) + 1; (q << ilog) <= end; ++q) {
          if (q <= live) continue;  // inside the live log (a truncation): finish writes it if accepted
          u64* ie = st.index + (rg.ibase + q % rg.icap) * 2;
          ie[0] = off + 1;
          ie[1] = end;
        }
      }
    } else {
      atomicOr(&A.bad[e], kBadCrc);  // CRC32C differs from the header's
    }
  }
}

// Whether the bytes of a record's last 16-byte piece past its payload (L bytes) are zero.
__device__ __forceinline__ bool pad_zero(const uint4 t, u32 L) {
  const u32 nb = L & 15u;  // payload bytes in the last piece (0: it is all payload)
  u32 z = 0;
  const u32 w4[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (u32 i = 0; i < 4; ++i) {
    const u32 lo = 4u * i;  // the word's first byte
    const u32 keep = nb <= lo ? 0u : nb >= lo + 4u ? 0xFFFFFFFFu : (1u << (8u * (nb - lo))) - 1u;
    z |= w4[i] & ~keep;
  }
  return nb == 0u || z == 0u;
}

// One task (64 records of one source region) of the verify kernel, by one wave: a lane per record.
// The lane runs the CRC32C register through the record's payload pieces in order (slicing-by-8 from
// LDS, two steps per 16-byte piece, no zero-shift tables); records over 1 KB by the whole wave.
__device__ __forceinline__ void verify_task_lane(const IngestArgs& A, const u32 (*t8)[256], u32 task) {
  const u32 src = source_of_task(A, task);
  if (!A.rbytes[src]) return;
  const RegionView R = region_of(A, src);
  if (!R.sane) return;  // every entry refused (prepare)
  const u32 lane = threadIdx.x & 63;
  const u32 i = (task - A.task0[src]) * kIR + lane;
  const bool in = i < R.n_records;
  const DevState& st = A.st;
  u32 p = 0, L = 0, m = 0, e = 0;
  u64 pos = 0, off = 0;
  u64 p_used = 0, p_ring = 0;  // the partition's live log end and ring word (the index writes below)
  bool ok = false, owner = false, reb = false;
  const uint8_t* rec = R.base;
  uint4 hdr = make_uint4(0, 0, 0, 0);
  // the header and the first kVSpec pieces are loaded with the directory entry, from the table slot
  // alone (inside the data section; used only once the checks below pass)
  uint4 sp0 = make_uint4(0, 0, 0, 0), sp1 = sp0, sp2 = sp0, sp3 = sp0;
  if (in) {
    const u64* tabp = reinterpret_cast<const u64*>(R.base + kRegionHdr + (u64)kDirEntry * R.n_entries) + i;
    const u64 tab = tabp[0];
    const u64 tabn = i + 1u < R.n_records ? tabp[1] : 0ull;  // the next slot (the record after, if any)
    const u32 k = min((u32)tab, R.n_entries - 1u), d16 = (u32)(tab >> 32);  // ok below requires k == tab
    rec = R.base + R.data_off + 16ull * d16;
    const u64 dsz16 = (R.rows_off - R.data_off) >> 4;  // pieces in the data section
    uint4 sh = make_uint4(0, 0, 0, 0);
    if ((u64)d16 + 1ull <= dsz16) sh = *reinterpret_cast<const uint4*>(rec);
    if (kVSpec > 0 && (u64)d16 + 2ull <= dsz16) sp0 = *reinterpret_cast<const uint4*>(rec + 16ull);
    if (kVSpec > 1 && (u64)d16 + 3ull <= dsz16) sp1 = *reinterpret_cast<const uint4*>(rec + 32ull);
    if (kVSpec > 2 && (u64)d16 + 4ull <= dsz16) sp2 = *reinterpret_cast<const uint4*>(rec + 48ull);
    if (kVSpec > 3 && (u64)d16 + 5ull <= dsz16) sp3 = *reinterpret_cast<const uint4*>(rec + 64ull);
    const DirView d = dir_of(R, k);
    // structure: the slot lies in the range of the entry it names (prepare checked that the ranges
    // tile the table)
    const bool named = k == (u32)tab && i >= d.tstart && (u64)i < (u64)d.tstart + d.count;
    if (!named) mark_insane(A, src);
    e = A.xi_start[src] + k;
    p = A.xi_p[e];
    owner = k == 0 || A.xi_p[e - 1] != p;  // two local slots of one partition: the first owns the state
    reb = d.rebase;
    const u64 used = A.base[2 * e + 1];   // after a truncation: at the leader's first offset
    const u64 rel = 16ull * (u64)(d16 - d.dstart16);
    if (k == (u32)tab && d16 >= d.dstart16 && (u64)d16 + 1ull <= dsz16) {
      hdr = sh;
      off = ((u64)hdr.y << 32) | hdr.x;
      L = hdr.z;
      m = (L + 15u) >> 4;
    }
    pos = used + rel;
    // the record continues the entry (its directory verdict is prepare's): its offset, inside the
    // entry's bytes (which lie inside the data section), the first at the entry's start, each one
    // where the one before ends and the last at the entry's end (FORMAT.md §9)
    const u64 rend16 = (u64)d16 + 1ull + m;
    const bool last = (u64)i + 1ull == (u64)d.tstart + d.count;
    const bool chained = (i != d.tstart || d16 == d.dstart16) &&
                         (last ? rend16 == (u64)d.dstart16 + d.bytes16 : (u64)(u32)(tabn >> 32) == rend16);
    ok = named && d16 >= d.dstart16 && (u64)d.dstart16 + d.bytes16 <= (R.rows_off - R.data_off) >> 4 &&
         off == d.first + (i - d.tstart) && rel + 16ull * (1ull + m) <= 16ull * d.bytes16 && chained &&
         A.bad[e] == 0u;
    if (!ok && A.bad[e] == 0u) atomicOr(&A.bad[e], kBadCrc);  // the record's content is wrong
    // loaded now (in flight with the payload loads below) rather than after the CRC
    if (ok && owner && !reb) {
      p_used = st.used[p];
      p_ring = st.ring[p];
    }
  }
  const bool big = ok && m > kBigIngest;
  const u32 mm = ok && !big ? m : 0u;
  // the CRC register over the payload pieces in order (zero-padded in the log), from ~0
  u32 acc = 0xFFFFFFFFu;
  bool padz = true;  // the zero padding after the payload in the record's last piece (small records)
  {
    const uint4 sv[4] = {sp0, sp1, sp2, sp3};
#pragma unroll
    for (u32 u = 0; u < kVSpec; ++u)
      if (u < mm) {
        acc = crc_step8(t8, crc_step8(t8, acc, sv[u].x, sv[u].y), sv[u].z, sv[u].w);
        if (u + 1u == mm) padz = pad_zero(sv[u], L);
      }
  }
  for (u32 c = kVSpec; __any(c < mm); c += 4) {
    uint4 v[4];
#pragma unroll
    for (u32 u = 0; u < 4; ++u)  // four pieces in flight per lane
      v[u] = c + u < mm ? *reinterpret_cast<const uint4*>(rec + 16ull + 16ull * (c + u)) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (u32 u = 0; u < 4; ++u)
      if (c + u < mm) {
        acc = crc_step8(t8, crc_step8(t8, acc, v[u].x, v[u].y), v[u].z, v[u].w);
        if (c + u + 1u == mm) padz = pad_zero(v[u], L);
      }
  }
  // records over 1 KB, one at a time by the wave: lane l takes pieces l, l + 64, ... (Horner with
  // the 1 KB shift), shifts past the pieces after its last one, XOR-reduce; the record's lane gets
  // the register
  for (u64 bm = __ballot(big); bm; bm &= bm - 1ull) {
    const u32 sl = (u32)__builtin_ctzll(bm);
    const u64 brec = ((u64)(u32)__builtin_amdgcn_readlane((int)(reinterpret_cast<u64>(rec) >> 32), (int)sl) << 32) |
                     (u32)__builtin_amdgcn_readlane((int)(u32)reinterpret_cast<u64>(rec), (int)sl);
    const u32 bm16 = ((u32)__builtin_amdgcn_readlane((int)L, (int)sl) + 15u) >> 4;
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
          uint4 w = v[u];
          if (jp == 0) w.x ^= 0xFFFFFFFFu;
          bacc = crc_zshift(A.crc->zshift1k, bacc) ^ crc_piece16(t8, w);  // (L1/L2-resident)
        }
      }
    }
    if (lane < bm16) {
      const u32 eb = (bm16 - 1u - lane) & 63u;
      if (eb) bacc = gf2_mulmod(bacc, A.crc->sh16[eb]);
    }
    bacc = wave_xor_all(bacc);
    if (lane == sl) acc = bacc;
  }
  if (ok) {
    u32 crc = 0;
    if (L) {
      const u32 pad = 16u * m - L;
      crc = ~(pad ? gf2_mulmod(A.crc->inv_pad[pad], acc) : acc);
    }
    // the zero padding after the payload (FORMAT.md §1) is part of the record
    // (a large record's last piece is read again: the wave folded its pieces)
    if (big && m) padz = pad_zero(*reinterpret_cast<const uint4*>(rec + 16ull * m), L);
    if (!padz) crc = ~hdr.w;
    if (crc == hdr.w) {
      // (a rebase entry's index entries are written by finish, once the entry is accepted: its
      // positions lie past the live log but may share index slots with it)
      if (owner && !reb) {
        // sparse index past the follower's live log: every interval multiple the record crosses
        const u32 ilog = st.interval_log2;
        const RingRef rg = ring_ref(p_ring, ilog, st.icap_mul);
        const u64 end = pos + 16ull * (1ull + m), live = p_used >> ilog;
        for (u64 q = (pos >> ilog) + 1; (q << ilog) <= end; ++q) {
          if (q <= live) continue;  // inside the live log (a truncation): finish writes it if accepted
          u64* ie = st.index + (rg.ibase + q % rg.icap) * 2;
          ie[0] = off + 1;
          ie[1] = end;
        }
      }
    } else {
      atomicOr(&A.bad[e], kBadCrc);  // CRC32C differs from the header's
    }
  }
}

// A grid of at most a few workgroups per CU: each copies the CRC tables into LDS once and its waves
// take tasks w, w + waves, ... (the tables were 20 KB per 32 records' worth of workgroup before;
// the 16-byte shift is a multiply, the 1 KB one of large records is read from global memory).
__global__ __launch_bounds__(kIT, RMQ_VERIFY_WAVES) void ingest_verify_kernel(IngestArgs A) {
  __shared__ __attribute__((aligned(16))) u32 t8[8][256];
  __shared__ __attribute__((aligned(16))) u32 z32[4][256];  // register shift past 32 zero bytes
  {
    static_assert(offsetof(CrcConsts, zshift) == sizeof(A.crc->table), "table and zshift adjacent");
    const uint4* src = reinterpret_cast<const uint4*>(&A.crc->table[0][0]);
    const uint4* zs = reinterpret_cast<const uint4*>(&A.crc->zshift[1][0][0]);
    uint4* d0 = reinterpret_cast<uint4*>(&t8[0][0]);
    uint4* d1 = reinterpret_cast<uint4*>(&z32[0][0]);
    for (u32 k = threadIdx.x; k < sizeof(t8) / 16; k += kIT) d0[k] = src[k];
    if (!RMQ_VERIFY_LANE)  // (a lane per record needs no zero-shift table)
      for (u32 k = threadIdx.x; k < sizeof(z32) / 16; k += kIT) d1[k] = zs[k];
  }
  __syncthreads();
  const u32 tasks = A.task0[A.world], stride = gridDim.x * kIW;
  for (u32 task = __builtin_amdgcn_readfirstlane(blockIdx.x * kIW + (threadIdx.x >> 6)); task < tasks; task += stride) {
    if (RMQ_VERIFY_LANE)
      verify_task_lane(A, t8, task);
    else
      verify_task(A, t8, z32, task);
  }
}

// The verdict and state of entry e (thread per entry); its records and bytes ingested are added
// to n_rec / n_bytes (the kernel sums them over the wave: one atomic per wave, not per entry).
// The verdict on entry e once verify has run: its own refusal bits (a structurally broken region
// refuses all its entries; so does a round whose copy items overflowed: only corrupted regions ask
// for more than the host's bound, and no entry may be accepted with bytes left uncopied), and those
// of the partition's other local slot (adjacent entries of the same source: a refusal of either
// refuses both). Finish and the copy each derive it.
struct Verdict {
  u32 own, bad;
};
__device__ __forceinline__ Verdict entry_verdict(const IngestArgs& A, u32 e, u32 src, u32 p) {
  const bool broken = __hip_atomic_load(&A.insane[src], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                      *A.n_items > A.items_grid;
  Verdict v;
  v.own = A.bad[e] | (broken ? kBadCrc : 0u);
  v.bad = v.own;
  for (u32 q = e; q > A.xi_start[src] && A.xi_p[q - 1] == p; --q) v.bad |= A.bad[q - 1];
  for (u32 q = e + 1; q < A.xi_start[src + 1] && A.xi_p[q] == p; ++q) v.bad |= A.bad[q];
  return v;
}

__device__ __forceinline__ void finish_entry(const IngestArgs& A, u32 e, u64& n_rec, u64& n_bytes) {
  const u32 src = source_of_entry(A, e);
  const DevState& st = A.st;
  const u32 p = A.xi_p[e], k = e - A.xi_start[src];
  const bool owner = k == 0 || A.xi_p[e - 1] != p;
  const Verdict vd = entry_verdict(A, e, src, p);
  const u32 own = vd.own, bad = vd.bad;
  if (own) atomicAdd((unsigned long long*)&A.counters[(own & kBadCrc) && !(own & ~kBadCrc) ? 1 : 2], 1ull);
  A.acc[e] = bad ? 0u : 1u;
  // an entry of the current term from a leader whose region arrived: the leader is alive (the
  // election timer restarts), whatever the verdict on its records
  if (owner && !(A.bad[e] & (kBadMissed | kBadUnread | kBadStale))) st.heard[p] = A.stamp;
  if (bad) {
    A.ackout[2 * e] = st.leo[p] | kAckRefused;
    A.ackout[2 * e + 1] = st.used[p];
    return;
  }
  const RegionView R = region_of(A, src);
  const DirView d = dir_of(R, k);
  const u64 bused = A.base[2 * e + 1];
  const u64 nleo = d.first + d.count, nused = bused + 16ull * d.bytes16;
  if (owner) {
    const u32 ilog = st.interval_log2;
    const u64 old_used = st.used[p];
    if (d.term > st.term[p]) st.term[p] = d.term;
    // the entry's last entry term; 0: older than the leader's term start, unknown here, so the log
    // ends in a term below the leader's (the vote's bound, never 0: a replica whose log ends in
    // term-t entries must not grant a candidate of an older last term)
    st.lterm[p] = d.lterm ? d.lterm : kLtermBound | (d.term ? d.term - 1ull : 0ull);
    st.mterm[p] = d.term;   // the log matches the term-d.term leader's through the entry's end
    u64 spos = st.start_pos[p];
    if (d.rebase) {
      // the log restarts at the entry's first record: its start, and every index entry of the
      // records (E[m] of a start on an interval multiple is that record, as in the leader's index)
      const RingRef rg = ring_ref(st, p);
      const uint8_t* data = R.base + R.data_off + 16ull * d.dstart16;
      st.start_off[p] = d.first;
      st.start_pos[p] = spos = bused;
      if (!(bused & ((1ull << ilog) - 1ull))) {
        u64* ie = st.index + (rg.ibase + (bused >> ilog) % rg.icap) * 2;
        ie[0] = d.first;
        ie[1] = bused;
      }
      u64 pos = bused;
      for (u32 r = 0; r < d.count; ++r) {
        const u32 L = *reinterpret_cast<const u32*>(data + (pos - bused) + 8);
        const u64 end = pos + 16ull + ((L + 15ull) & ~15ull);
        for (u64 q = (pos >> ilog) + 1; (q << ilog) <= end; ++q) {
          u64* ie = st.index + (rg.ibase + q % rg.icap) * 2;
          ie[0] = d.first + r + 1;
          ie[1] = end;
        }
        pos = end;
      }
    } else if (bused < old_used && d.count) {
      // a truncation: the index slots inside the old live log name the new log's records
      const RingRef rg = ring_ref(st, p);
      const uint8_t* data = R.base + R.data_off + 16ull * d.dstart16;
      const u64 live = old_used >> ilog;
      u64 pos = bused;
      for (u32 r = 0; r < d.count && (pos >> ilog) < live; ++r) {
        const u32 L = *reinterpret_cast<const u32*>(data + (pos - bused) + 8);
        const u64 end = pos + 16ull + ((L + 15ull) & ~15ull);
        for (u64 q = (pos >> ilog) + 1; (q << ilog) <= end && q <= live; ++q) {
          u64* ie = st.index + (rg.ibase + q % rg.icap) * 2;
          ie[0] = d.first + r + 1;
          ie[1] = end;
        }
        pos = end;
      }
    }
    for (u32 s = 0; s < 2; ++s) {
      A.sets[s].leo[p] = nleo;
      A.sets[s].used[p] = nused;
    }
    learn_commit(st, p, d.commit, nleo);  // the leader's commit the entry carries (Raft leaderCommit)
    if (d.count) {
      // retention once per round (FORMAT.md §4 rule on the follower's log)
      const RingRef rg = ring_ref(st, p);
      if (nused - spos > rg.seg) {
        const u64 ms = (nused - rg.seg + (1ull << ilog) - 1) >> ilog;
        const u64* ie = st.index + (rg.ibase + ms % rg.icap) * 2;
        st.start_off[p] = ie[0];
        st.start_pos[p] = ie[1];
      }
      n_bytes += 16ull * d.bytes16;
    }
    if (R.M) {  // the partition's consumer-offset row, if the round carries one (rows ascend by entry)
      const u64 rowb = 16ull + 8ull * A.C;
      u32 lo = 0, hi = R.M;
      while (lo < hi) {
        const u32 mid = (lo + hi) / 2;
        const u32 rk = *reinterpret_cast<const u32*>(R.base + R.rows_off + rowb * mid);
        if (rk < k) lo = mid + 1; else hi = mid;
      }
      if (lo < R.M && *reinterpret_cast<const u32*>(R.base + R.rows_off + rowb * lo) == k) {
        const u64* row = reinterpret_cast<const u64*>(R.base + R.rows_off + rowb * lo + 16);
        for (u32 c = 0; c < A.C; ++c) st.cons[(u64)p * A.C + c] = row[c];
      }
    }
  }
  n_rec += d.count;
  A.ackout[2 * e] = nleo;
  A.ackout[2 * e + 1] = nused;
}

__device__ __forceinline__ void finish_block(const IngestArgs& A, u32 e) {
  u64 n_rec = 0, n_bytes = 0;
  if (e < A.n_in) finish_entry(A, e, n_rec, n_bytes);
  // every lane of the wave is back here (blockDim is a multiple of 64)
  for (int o = 32; o; o >>= 1) {
    n_rec += __shfl_xor(n_rec, o, 64);
    n_bytes += __shfl_xor(n_bytes, o, 64);
  }
  if ((threadIdx.x & 63u) == 0) {
    if (n_rec) atomicAdd((unsigned long long*)&A.counters[0], (unsigned long long)n_rec);
    if (n_bytes) atomicAdd((unsigned long long*)&A.counters[3], (unsigned long long)n_bytes);
  }
}

// Accepted entries' record bytes into the follower's replica rings: workgroup per work item
// {entry, 16 KiB chunk of its data}, 16-byte pieces, four in flight per thread. A work item is a
// chain of dependent lookups before its first data load, so items are one wave each: up to 32 per
// CU in flight.
__device__ __forceinline__ void copy_item(const IngestArgs& A, u32 it) {
  if (it >= *A.n_items) return;
  const u32 e = A.items[2 * it], c = A.items[2 * it + 1];
  // the verdict (derived here, as finish derives it beside this copy) and the entry's descriptor
  // (prepare), loaded together
  const u64* cd = A.cdesc + 4ull * e;
  const u64 d0 = cd[0], d1 = cd[1], bused = cd[2], d3 = cd[3];
  const u32 src = source_of_entry(A, e);
  if (entry_verdict(A, e, src, A.xi_p[e]).bad) return;
  const uint8_t* data = reinterpret_cast<const uint8_t*>(d0);
  uint8_t* const ring = reinterpret_cast<uint8_t*>(d1);
  const u64 seg = 1ull << (d3 & 63ull), segmask = seg - 1ull;
  const u64 bytes = d3 >> 6, gend = bused + bytes;
  const u64 b0 = (u64)c * kCopyChunk, b1 = min(bytes, b0 + kCopyChunk);
  // lane l takes piece l - ph of each 1 KB step, so every store instruction covers whole 128-byte
  // lines of the ring (the leader's positions are at any 16-byte phase; such 1 KB stores measured
  // 20 % slower, tools/replica_bench)
  const u64 ph = ((bused + b0) >> 4) & 7ull;
  for (u64 q0 = b0 + 16ull * threadIdx.x; q0 < b1 + 16ull * ph; q0 += 16ull * kCT * 4) {
    uint4 v[4];
#pragma unroll
    for (u32 u = 0; u < 4; ++u) {
      const u64 q = q0 + 16ull * kCT * u - 16ull * ph;  // (below b0: wraps past b1, skipped)
      v[u] = q >= b0 && q < b1 ? *reinterpret_cast<const uint4*>(data + q) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (u32 u = 0; u < 4; ++u) {
      const u64 q = q0 + 16ull * kCT * u - 16ull * ph;
      const u64 x = bused + q;
      if (q >= b0 && q < b1 && x + seg >= gend) store_log16(ring + (x & segmask), v[u]);
    }
  }
}

// Finish and copy in one launch (both only read verify's verdicts): one-wave workgroups, the
// first fin_blocks finish entries (a thread each), the rest copy one work item each. The copy no
// longer waits for finish to end (one kernel less in each round's ingest chain).
__global__ __launch_bounds__(kCT) void ingest_finish_copy_kernel(IngestArgs A, u32 fin_blocks) {
  static_assert(kCT == 64, "one-wave workgroups (finish sums its counters per wave)");
  if (blockIdx.x < fin_blocks)
    finish_block(A, blockIdx.x * kCT + threadIdx.x);
  else
    copy_item(A, blockIdx.x - fin_blocks);
}

// Acks of one round applied after the pipeline has drained (thread per partition).
__global__ void ack_apply_kernel(AckApplyArgs a) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  const DevState& st = a.st;
  if (p >= st.P || !st.is_leader[p]) return;
  u64 row[kMaxRF];
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) row[r] = r < st.RF ? st.match[(u64)p * st.RF + r] : 0ull;
  const u32 fl = apply_acks(st, p, a.outidx, a.ackin, st.leo[p], row, a.xreq, a.acks_round, a.rowv);
  if (fl & kAckRow) st.cq[p] = row_quorum(st, p);
  if (fl & kAckMatch) {
    const u64 c = quorum_commit(row, st.RF, st.commit[p], st.term_start[p]);
    st.commit[p] = c;
    st.hw[p] = c;
    if (st.csnap) st.csnap[(u64)st.csnap_slot * st.P + p] = c;
  }
}

// Commit notices (FORMAT.md §9 v4), exchanged by a drain after its rounds' acks: the leader's
// {commit, term} per out entry, and a follower learning it (a notice of an older term is ignored;
// a newer term is adopted, as any Raft message of a newer term makes a replica do).
__global__ void notice_fill_kernel(NoticeArgs a) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n_out) return;
  const u32 p = a.xo_p[e];
  a.out[2 * e] = a.st.commit[p];
  a.out[2 * e + 1] = a.st.term[p];
}

__global__ void notice_apply_kernel(NoticeArgs a) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n_in) return;
  const DevState& st = a.st;
  const u32 p = a.xi_p[e];
  const u64 c = a.in[2 * e], t = a.in[2 * e + 1];
  if (t < st.term[p]) return;  // an older term's (or a lost notice, term 0)
  if (t > st.term[p]) st.term[p] = t;
  st.heard[p] = a.stamp;
  // the commit moves over this log only if it was matched in the notice's term; the leader's commit
  // is learned either way (rmq_become_leader's RMQ_ESTALE). (Two slots of one partition: the same
  // values.)
  if (st.mterm[p] == t) learn_commit(st, p, c, a.sets[0].leo[p]);
  else if (c > st.lcommit[p]) st.lcommit[p] = c;
}

void launch_notice_fill(const NoticeArgs& a, hipStream_t s) {
  if (a.n_out) hipLaunchKernelGGL(notice_fill_kernel, dim3((a.n_out + 255) / 256), dim3(256), 0, s, a);
}

void launch_notice_apply(const NoticeArgs& a, hipStream_t s) {
  if (a.n_in) hipLaunchKernelGGL(notice_apply_kernel, dim3((a.n_in + 255) / 256), dim3(256), 0, s, a);
}

// resident verify workgroups per CU at the kernel's launch bounds (the default verify grid)
uint32_t verify_wgs_per_cu() { return RMQ_VERIFY_WAVES * 4u / kIW; }
uint32_t verify_records_per_task() { return kIR; }

void launch_ingest(const IngestArgs& a, uint32_t tasks, uint32_t items_bound, uint32_t verify_wgs, hipStream_t s) {
  if (a.n_in) hipLaunchKernelGGL(ingest_prepare_kernel, dim3((a.n_in + kEntryT - 1) / kEntryT), dim3(kEntryT), 0, s, a);
  if (tasks)
    hipLaunchKernelGGL(ingest_verify_kernel, dim3(std::min<uint32_t>((tasks + kIW - 1) / kIW, verify_wgs)), dim3(kIT), 0, s, a);
  const u32 fin = (a.n_in + kCT - 1) / kCT;
  if (fin + items_bound) hipLaunchKernelGGL(ingest_finish_copy_kernel, dim3(fin + items_bound), dim3(kCT), 0, s, a, fin);
}

// Fault injection (rmq_fault_corrupt): one byte of a region flipped before it is sent.
__global__ void flip_kernel(uint8_t* region, uint64_t size, int64_t at) {
  const u64 rows = *reinterpret_cast<const u64*>(region + 32);  // end of the data section
  const int64_t pos = at < 0 ? (int64_t)rows + at : at;
  if (pos >= 0 && (u64)pos < size) region[pos] ^= 0x5Au;
}

void launch_flip(uint8_t* region, uint64_t size, int64_t at, hipStream_t s) {
  hipLaunchKernelGGL(flip_kernel, dim3(1), dim3(1), 0, s, region, size, at);
}

void launch_ack_apply(const AckApplyArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ack_apply_kernel, dim3((a.st.P + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace rmq
