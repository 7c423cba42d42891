// control.hip — small per-partition kernels around the append path:
//   * quorum commit over all partitions (after external acks),
//   * external replica acks (matchIndex = max(matchIndex, ack)),
//   * leader start (term_start = log end; Raft matchIndex reset for remote replicas),
//   * consumer-offset commits (PartitionStateMachine.handleConsumerOffsetUpdateRequest,
//     mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:71-77): last writer wins;
//     the host keeps the last item per (partition, consumer), so this is a plain scatter;
//   * ring moves (rmq_set_segments): a partition's retained log and index entries into a new ring.
#include "device_common.hpp"
#include "kernels.hpp"
#include <algorithm>
#include "partition_ops.hpp"

namespace rmq {

__global__ void commit_all_kernel(DevState st) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < st.P) commit_rule(st, p);
}

__global__ void ack_kernel(AckArgs a) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  // a follower cannot have persisted past the leader's log end: clamp (Raft matchIndex <= lastLogIndex)
  const u64 leo = a.st.leo[a.pidx[i]];
  const u64 m = a.match[i] < leo ? a.match[i] : leo;
  atomicMax((unsigned long long*)&a.st.match[(u64)a.pidx[i] * a.st.RF + a.slot[i]], (unsigned long long)m);
}

// Leader start (Raft's leader initialisation, FORMAT.md §6): term_start = log end (the virtual
// leader-start entry), local matchIndex = log end, remote 0; the commit rule runs at once (a quorum
// of local replicas holds the leader-start entry already); the consumer-offset row goes to every
// follower with the next round (the new leader's table replaces theirs).
__global__ void become_leader_kernel(DevState st, u32 only) {
  const u32 p = only == 0xFFFFFFFFu ? blockIdx.x * blockDim.x + threadIdx.x : only;
  if (p >= st.P || (only != 0xFFFFFFFFu && (blockIdx.x | threadIdx.x))) return;
  const u64 leo = st.leo[p];
  st.term_start[p] = leo;
  st.lterm[p] = st.mterm[p] = st.term[p];  // its leader-start entry (the host wrote the new term)
  const u32 lm = st.local_mask[p];
  for (u32 r = 0; r < st.RF; ++r) {
    st.match[(u64)p * st.RF + r] = (lm >> r & 1u) ? leo : 0ull;
    // the followers acknowledge the new leader's rows afresh (tickets of the new term)
    if (st.outidx && st.eackv && !(lm >> r & 1u)) {
      const u32 e = st.outidx[(u64)p * st.RF + r];
      if (e != ~0u) st.eackv[e] = 0ull;
    }
  }
  commit_rule(st, p);
  st.cdirty[p] = 1u;
  st.cq[p] = row_quorum(st, p);
}

__global__ void consumer_apply_kernel(ConsumerCommitArgs a) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const u32 p = a.pidx[i];
  a.st.cons[(u64)p * a.st.C + a.consumer[i]] = a.offset[i];
  a.st.cdirty[p] = 1u;  // the row travels with the next replication round (FORMAT.md §9)
  // the row's new version (every item of p writes the same words); co-located replicas hold it now
  a.st.cver[p] = a.ver[i];
  a.st.cq[p] = row_quorum(a.st, p);
}

// Every partition's row quorum afresh (after a placement change reset the followers' row acks).
__global__ void row_quorum_all_kernel(DevState st) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < st.P) st.cq[p] = row_quorum(st, p);
}

static inline dim3 grid_for(u32 n, u32 b) { return dim3((n + b - 1) / b ? (n + b - 1) / b : 1); }

// rmq_get_partition_states: the state words of partitions [first, first + n) gathered into one
// page-locked host area in a single pass (field-major: 11 fields, then the match rows), instead of a
// DMA per field (12 serialized copies measured 0.86 ms for 4,096 partitions).
__global__ void state_gather_kernel(DevState st, uint64_t* out, u32 first, u32 n, u32 RF) {
  const u64* const src[11] = {st.leo, st.used, st.start_off, st.start_pos, st.commit, st.hw, st.term,
                              st.term_start, st.lcommit, st.lterm, st.heard};
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
#pragma unroll
    for (u32 f = 0; f < 11; ++f) out[(u64)f * n + i] = src[f][first + i];
    for (u32 r = 0; r < RF; ++r) out[11ull * n + (u64)i * RF + r] = st.match[(u64)(first + i) * RF + r];
  }
}

void launch_state_gather(const DevState& st, uint64_t* out, uint32_t first, uint32_t n, uint32_t RF, hipStream_t s) {
  hipLaunchKernelGGL(state_gather_kernel, dim3(std::min<uint32_t>((n + 255) / 256, 1024u)), dim3(256), 0, s, st, out,
                     first, n, RF);
}

void launch_row_quorum_all(const DevState& st, hipStream_t s) {
  hipLaunchKernelGGL(row_quorum_all_kernel, grid_for(st.P, 256), dim3(256), 0, s, st);
}

// Retention of the last applied group for the partitions whose replay its own launch stopped early
// (rlate[p]: the group added more than a ring less an interval to p, so the index entries retention
// needed were being written by that launch; pipeline.hip partition_threads): issued by the host
// before a fetch or a state read that follows that launch, so they see the log start the oracle has
// after the group's last batch (FORMAT.md §4) rather than the next launch's stage 4 doing it. The
// flag is cleared, so that stage 4 finds nothing left.
__global__ void late_retention_kernel(LateArgs a) {
  const DevState& st = a.st;
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= st.P || !a.rlate[p] || !st.is_leader[p]) return;
  u64 bc[kMaxGroup];
#pragma unroll
  for (u32 j = 0; j < kMaxGroup; ++j) bc[j] = j < a.nb ? a.bcum[(u64)j * st.P + p] : 0ull;
  const RingRef rg = ring_ref(st, p);
  u64 soff = st.start_off[p], spos = st.start_pos[p];
  retain_batches(st, rg, bc, a.nb, false, st.used[p], a.totals[p], ~0ull, soff, spos);
  st.start_off[p] = soff;
  st.start_pos[p] = spos;
  a.rlate[p] = 0u;
}
void launch_late_retention(const LateArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(late_retention_kernel, grid_for(a.st.P, 256), dim3(256), 0, s, a);
}

void launch_commit_all(const DevState& st, hipStream_t s) {
  hipLaunchKernelGGL(commit_all_kernel, grid_for(st.P, 256), dim3(256), 0, s, st);
}
void launch_ack(const AckArgs& a, hipStream_t s) {
  if (!a.n) return;
  hipLaunchKernelGGL(ack_kernel, grid_for(a.n, 256), dim3(256), 0, s, a);
  launch_commit_all(a.st, s);
}
void launch_become_leader(const DevState& st, uint32_t pidx, hipStream_t s) {
  if (pidx == 0xFFFFFFFFu)
    hipLaunchKernelGGL(become_leader_kernel, grid_for(st.P, 256), dim3(256), 0, s, st, pidx);
  else
    hipLaunchKernelGGL(become_leader_kernel, dim3(1), dim3(64), 0, s, st, pidx);
}
void launch_consumer_commit(const ConsumerCommitArgs& a, hipStream_t s) {
  if (!a.n) return;
  hipLaunchKernelGGL(consumer_apply_kernel, grid_for(a.n, 256), dim3(256), 0, s, a);
}

// A move in chunks: workgroup c of a moved partition owns bytes [c K, (c + 1) K) of the new ring
// of every replica slot (K = kMigrateChunk, or the whole ring when smaller) and the same share of
// its index ring. Each 16-byte piece gets its logical position's bytes if that position is
// retained ([spos, used) is at most one new ring long), zero otherwise; each index slot gets entry
// m (the retained m with m mod icap = slot) or zero. Old and new blocks are disjoint (both
// allocated while moving). The first chunk writes the partition's new descriptor and log start on
// the device (a host copy into these arrays could leave other XCDs' L2 holding the old lines).
__global__ __launch_bounds__(256) void migrate_kernel(DevState st, const MigrateItem* items, u32 n) {
  u32 lo = 0, hi = n;  // the item whose chunks hold blockIdx.x: largest chunk0 <= blockIdx.x
  while (hi - lo > 1) {
    const u32 mid = (lo + hi) / 2;
    if (items[mid].chunk0 <= blockIdx.x) lo = mid; else hi = mid;
  }
  const MigrateItem it = items[lo];
  const u32 c = blockIdx.x - it.chunk0;
  if (c == 0 && threadIdx.x == 0) {
    st.ring[it.p] = it.new_desc;
    st.start_pos[it.p] = it.spos;
    st.start_off[it.p] = it.soff;
  }
  const RingRef o = ring_ref(it.old_desc, st.interval_log2, st.icap_mul);
  const RingRef nw = ring_ref(it.new_desc, st.interval_log2, st.icap_mul);
  const u64 keep = it.used - it.spos, nmask = nw.seg - 1ull, omask = o.seg - 1ull;
  const u64 s0 = it.spos & nmask;
  const u64 K = nw.seg < kMigrateChunk ? nw.seg : kMigrateChunk;
  const u64 q0 = (c * K) >> 4, q1 = ((c + 1ull) * K) >> 4;
  for (u32 r = 0; r < st.RF; ++r) {
    const uint8_t* src = st.logs + (u64)r * st.rstride + o.base;
    uint8_t* dst = st.logs + (u64)r * st.rstride + nw.base;
    for (u64 q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
      const u64 d = ((16ull * q - s0) & nmask);  // bytes after spos, if retained
      uint4 v = make_uint4(0, 0, 0, 0);
      if (d < keep) v = *reinterpret_cast<const uint4*>(src + ((it.spos + d) & omask));
      store_log16(dst + 16ull * q, v);  // the pipeline's ring-store flavour (non-temporal)
    }
  }
  const u32 ilog = st.interval_log2;
  const u64 m0 = (it.spos + (1ull << ilog) - 1) >> ilog, m1 = it.used >> ilog;
  const u64 nch = nw.seg / K, i0 = nw.icap * c / nch, i1 = nw.icap * (c + 1ull) / nch;
  for (u64 q = i0 + threadIdx.x; q < i1; q += blockDim.x) {
    const u64 m = m0 + ((q + nw.icap - m0 % nw.icap) % nw.icap);
    u64 e0 = 0, e1 = 0;
    if (m <= m1) {
      const u64* oe = st.index + (o.ibase + m % o.icap) * 2;
      e0 = oe[0];
      e1 = oe[1];
    }
    u64* ne = st.index + (nw.ibase + q) * 2;
    ne[0] = e0;
    ne[1] = e1;
  }
}

void launch_migrate(const DevState& st, const MigrateItem* items, uint32_t n, uint32_t chunks, hipStream_t s) {
  if (n) hipLaunchKernelGGL(migrate_kernel, dim3(chunks), dim3(256), 0, s, st, items, n);
}

}  // namespace rmq
