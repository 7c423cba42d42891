// partition_ops.hpp — per-partition state transitions shared by the append and control kernels.
#pragma once
#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr u64 kLow40 = (1ull << 40) - 1ull;  // bytes/16 field of a {count << 40 | bytes/16} aggregate


// Raft quorum commit (jraft BallotBox semantics; restated from the Raft paper since
// jraft-core 1.3.15 is not in the container): N = k-th largest matchIndex of the partition's
// replica row, k = RF/2 + 1 (the median for odd RF), held in registers and ordered by a
// compare-exchange network; commit advances to N only if N > commit and N >= term_start: the
// leader's term starts with a virtual entry at term_start (jraft appends a configuration entry
// when a leader starts, [jraft]), which a replica holds once it holds the log up to term_start in
// the new term (its match is reset to 0 at leader start and only moves by acks of that term); a
// quorum holding it commits every earlier-term record before it (Raft's current-term rule, FORMAT.md
// §6). hw (consumer-visible end) = commit.
// k-th largest of a replica row, k = RF/2 + 1 (compare-exchange network in registers).
__device__ __forceinline__ u64 quorum_value(const u64 (&row)[kMaxRF], u32 RF) {
  u64 m[kMaxRF];
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) m[r] = r < RF ? row[r] : 0ull;
#pragma unroll
  for (u32 i = 1; i < kMaxRF; ++i)
#pragma unroll
    for (u32 j = i; j > 0; --j) {  // compare-exchange network, descending
      const u64 a = m[j - 1], b = m[j];
      m[j - 1] = a > b ? a : b;
      m[j] = a > b ? b : a;
    }
  const u32 k = RF / 2 + 1;
  u64 N = 0;
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) N = (r == k - 1) ? m[r] : N;
  return N;
}

__device__ __forceinline__ u64 quorum_commit(const u64 (&row)[kMaxRF], u32 RF, u64 commit, u64 term_start) {
  const u64 N = quorum_value(row, RF);
  return (N > commit && N >= term_start) ? N : commit;
}

// The newest consumer-offset row version a quorum of partition p's replicas holds (FORMAT.md §8):
// co-located slots hold the leader's own (cver), a remote slot what its follower acknowledged.
__device__ __forceinline__ u64 row_quorum(const DevState& st, u32 p) {
  u64 v[kMaxRF];
  const u64 own = st.cver[p];
  const u32 lm = st.local_mask[p];
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) {
    u64 x = 0;
    if (r < st.RF) {
      if ((lm >> r) & 1u) {
        x = own;
      } else if (st.outidx && st.eackv) {
        const u32 e = st.outidx[(u64)p * st.RF + r];
        x = e == ~0u ? 0ull : st.eackv[e];
      }
    }
    v[r] = x;
  }
  return quorum_value(v, st.RF);
}

// Remote replica acks of one replication round (FORMAT.md §9 v3, [n_out][2] {log end | status << 62,
// log end position}) into the partition's matchIndex row: an accepted ack moves match = max(match,
// min(ack, log end)) for its slot; a refused one becomes a catch-up request {offset, position,
// round + 1} when xreq is given (no plan reads these acks itself). An accepted ack also acknowledges
// the consumer-offset row version the round carried to that follower (rowv, 0: none).
// Returns bit 0: a match moved, bit 1: an acknowledged row version moved.
constexpr u32 kAckMatch = 1u, kAckRow = 2u;
__device__ __forceinline__ u32 apply_acks(const DevState& st, u32 p, const u32* outidx, const u64* ackin, u64 leo,
                                          u64 (&row)[kMaxRF], u64* xreq, u64 acks_round, const u64* rowv) {
  u32 moved = 0;
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) {
    if (r >= st.RF) continue;
    const u32 e = outidx[(u64)p * st.RF + r];
    if (e == ~0u) continue;
    const u64 a0 = ackin[2 * e];
    if (a0 & kAckRefused) {
      if (xreq) {
        xreq[4 * e] = a0 & kAckLeoMask;
        xreq[4 * e + 1] = ackin[2 * e + 1];
        xreq[4 * e + 2] = acks_round + 1ull;
      }
      continue;
    }
    const u64 a = a0 < leo ? a0 : leo;
    if (a > row[r]) {
      row[r] = a;
      st.match[(u64)p * st.RF + r] = a;
      moved |= kAckMatch;
    }
    if (rowv && st.eackv) {
      const u64 v = rowv[e];
      if (v > st.eackv[e]) {
        st.eackv[e] = v;
        moved |= kAckRow;
      }
    }
  }
  return moved;
}

__device__ __forceinline__ void commit_rule(const DevState& st, u32 p) {
  u64 row[kMaxRF];
#pragma unroll
  for (u32 r = 0; r < kMaxRF; ++r) row[r] = r < st.RF ? st.match[(u64)p * st.RF + r] : 0ull;
  const u64 c = quorum_commit(row, st.RF, st.commit[p], st.term_start[p]);
  st.commit[p] = c;
  st.hw[p] = c;
  if (st.csnap) st.csnap[(u64)st.csnap_slot * st.P + p] = c;  // (the next plan's carried commit)
}

// A follower learns its leader's commit (FORMAT.md §9 v4: a round entry it accepted, or a commit
// notice): leader_commit = the newest, and its own commit = the part of its log below it (never
// past its log end: a replica whose log ends below the leader's commit lacks committed records).
__device__ __forceinline__ void learn_commit(const DevState& st, u32 p, u64 lc, u64 leo) {
  const u64 l = st.lcommit[p] > lc ? st.lcommit[p] : lc;
  st.lcommit[p] = l;
  u64 c = st.commit[p];
  const u64 k = l < leo ? l : leo;
  c = c > k ? c : k;
  c = c < leo ? c : leo;
  st.commit[p] = c;
  st.hw[p] = c;
}

// Retention after each batch of a group (FORMAT.md §4), batch by batch: after batch j the start
// moves to index entry ceil((fin_j - seg) / I) when fin_j - start > seg, fin_j = the log end after
// batch j: used0 + 16 (bc_j bytes) when used0 is the log end before the group (pre), else
// used0 - 16 (tot - bc_j bytes) (used0 after it); bc = the group's aggregates through each batch
// (a batch that appended nothing of p cannot move it). The start only grows, so a batch with
// fin_j - start0 <= seg never moves it: the positions of the others' entries are loaded together,
// the batches replayed in order in registers, and the offset of the last entry taken loaded after
// (the same index entry: one cache line). An entry at or past position `lim` may be written by
// the running launch: it is not read, the replay stops at its batch and the function returns
// false (the next launch's stage 4 finishes the group; replaying applied batches moves nothing).
__device__ __forceinline__ bool retain_batches(const DevState& st, const RingRef& rg, const u64 (&bc)[kMaxGroup], u32 nb,
                                               bool pre, u64 used0, u64 tot, u64 lim, u64& soff, u64& spos) {
  const u32 ilog = st.interval_log2;
  u64 ep[kMaxGroup];
  u32 cand = 0, late = 0;  // bit j: batch j may move the start / its entry is not readable yet
  u64 prev = 0;
#pragma unroll
  for (u32 j = 0; j < kMaxGroup; ++j) {
    ep[j] = 0ull;
    const bool app = j < nb && (bc[j] >> 40) != (prev >> 40);
    const u64 fin = pre ? used0 + 16ull * (bc[j] & kLow40) : used0 - 16ull * ((tot - bc[j]) & kLow40);
    if (app && fin - spos > rg.seg) {
      const u64 ms = (fin - rg.seg + (1ull << ilog) - 1) >> ilog;
      cand |= 1u << j;
      if ((ms << ilog) > lim) late |= 1u << j;
      else ep[j] = st.index[(rg.ibase + ms % rg.icap) * 2 + 1];
    }
    prev = j < nb ? bc[j] : prev;
  }
  bool done = true;
  int last = -1;
  u64 sp = spos;
#pragma unroll
  for (u32 j = 0; j < kMaxGroup; ++j) {
    const u64 fin = pre ? used0 + 16ull * (bc[j] & kLow40) : used0 - 16ull * ((tot - bc[j]) & kLow40);
    if (done && ((cand >> j) & 1u) && fin - sp > rg.seg) {
      if ((late >> j) & 1u) {
        done = false;
      } else {
        sp = ep[j];
        last = (int)j;
      }
    }
  }
  if (last >= 0) {
    u64 ms = 0;
#pragma unroll
    for (u32 j = 0; j < kMaxGroup; ++j)
      if ((int)j == last) {
        const u64 fin = pre ? used0 + 16ull * (bc[j] & kLow40) : used0 - 16ull * ((tot - bc[j]) & kLow40);
        ms = (fin - rg.seg + (1ull << ilog) - 1) >> ilog;
      }
    soff = st.index[(rg.ibase + ms % rg.icap) * 2];
    spos = sp;
  }
  return done;
}

}  // namespace rmq
