// fetch.hip — batched consumer fetch: PartitionStateMachine.handleBatchRead
// (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:85-110), served directly from
// committed state like MessageBatchReadRequestProcessor.java:39 (no read-index).
//
//  one launch, a wave per request (fetch_kernel): resolve the slice [off, min(off + max, hw)) and
//  its byte range (a 32-ary search of the sparse offset index, FORMAT.md §5, then the record headers
//  of the 1 KiB after the entry found, loaded at once and walked in registers); place it in the
//  output by a decoupled look-back scan of the requests' bytes (ENOSPC marking: every request's
//  bytes count, served or not, FORMAT.md §7); gather it with 16-byte loads and stores. Records and
//  output positions are 16-byte aligned (FORMAT.md §1), so no piece straddles a record, the ring
//  end or an output boundary.
//
// The kernel runs on the engine's fetch stream, after the last pipeline launch the host had
// issued and before the next one (engine.cpp orders the two streams with events), so the committed
// state they read is stable and the append pipeline is never flushed for a fetch.
#include <hip/hip_ext.h>

#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr int kOk = 0, kNotLeader = -1, kNoPart = -2, kInval = -3, kNoSpc = -4, kOffset = -6;
constexpr u32 kFW = 4;  // waves per workgroup (resolve, gather)

struct PartView {
  u64 leo, used, start_off, start_pos;
  RingRef rg;           // the partition's ring and index ring
  const uint8_t* ring;  // lowest local replica ring of the partition
};

// Logical byte positions of records t0 (lanes 0..31) and t1 (lanes 32..63), start_off <= t <= leo,
// found together (wave-uniform arguments; the half-wave of each record returns its position).
__device__ u64 record_pos2(const DevState& st, u32 p, const PartView& v, u64 t0, u64 t1) {
  const u32 lane = lane_id(), h = lane >> 5, hl = lane & 31u;
  const u64 t = h ? t1 : t0;
  const u32 ilog = st.interval_log2;
  const u64 I = 1ull << ilog;
  const u64* E = st.index + v.rg.ibase * 2;
  // per half: largest m in [lo, hi] with E[m].offset <= t (E rises with m), 32 probes per round;
  // none: the log start
  u64 c_off = v.start_off, c_pos = v.start_pos;
  long lo = (long)((v.start_pos + I - 1) >> ilog), hi = (long)(v.used >> ilog);
  bool open = t < v.leo && lo <= hi;
  while (__any(open)) {
    const long span = hi - lo + 1;
    const long step = (span + 31) / 32;
    const long m = lo + (long)hl * step;
    bool le = false;
    u64 eo = 0, ep = 0;
    if (open && m <= hi) {
      const u64* e = E + ((u64)m % v.rg.icap) * 2;
      eo = e[0];
      ep = e[1];
      le = eo <= t;
    }
    const u32 bal = (u32)(__ballot(le) >> (32u * h));  // this half's probes
    const u32 last = bal ? 31u - (u32)__builtin_clz(bal) : 0u;
    const u64 so = __shfl(eo, (int)(32u * h + last), 64), sp = __shfl(ep, (int)(32u * h + last), 64);
    if (open) {
      if (!bal) {
        open = false;  // every probe past t: the answer precedes this round's range
      } else {
        c_off = so;
        c_pos = sp;
        if (step == 1) {
          open = false;
        } else {
          lo = lo + (long)last * step + 1;  // the answer is that probe or one of the next step - 1
          hi = min(hi, lo + step - 2);
          open = lo <= hi;
        }
      }
    }
  }
  if (t >= v.leo) return v.used;
  // walk the headers of the records in [c_off, t): they start in the interval after c_pos, so one
  // 1 KiB window of 16-byte pieces holds them all (two pieces per lane of the half)
  const u64 mask = v.rg.seg - 1;
  const u32 Lw0 = *reinterpret_cast<const u32*>(v.ring + ((c_pos + 32ull * hl + 8ull) & mask));
  const u32 Lw1 = *reinterpret_cast<const u32*>(v.ring + ((c_pos + 32ull * hl + 24ull) & mask));
  u64 k = t - c_off;
  u32 cur = 0;  // window piece of the current record
  while (__any(k > 0)) {
    const u32 src = 32u * h + (cur >> 1);
    const u32 a0 = (u32)__shfl((int)Lw0, (int)src, 64), a1 = (u32)__shfl((int)Lw1, (int)src, 64);
    if (k > 0) {
      cur += record_bytes((cur & 1u) ? a1 : a0) >> 4;
      --k;
    }
  }
  return c_pos + 16ull * cur;
}

// Fetch status words of the look-back scan: [epoch 24 | flag 2 | bytes 38] per workgroup. The
// epoch names the fetch call (engine.cpp clears the words when it wraps), so no word of an earlier
// call is ever taken for this one's.
constexpr u32 kFlagAgg = 1u, kFlagIncl = 2u;
constexpr u64 kVal38 = (1ull << 38) - 1ull;
constexpr u32 kLB = 16;  // look-back words per lane and round
__device__ __forceinline__ u64 sat38(u64 v) { return v > kVal38 ? kVal38 : v; }

// One launch per fetch call, a wave per request, kFW requests per workgroup:
//  1. resolve: consumer offset, slice [off, min(off + max, hw)), status, byte range (record_pos2);
//  2. place: the workgroup's byte sum; its exclusive prefix over all earlier requests by a
//     decoupled look-back over the workgroups' status words (virtual workgroup ids from a ticket, so
//     every workgroup waited on has started and never waits on a later one); the output position
//     of a request is that prefix plus the bytes of the workgroup's earlier requests. Every
//     request's bytes count, served or not (FORMAT.md §7); one that ends past out_cap is ENOSPC;
//  3. gather: 16-byte loads from the lowest local replica ring, four in flight per lane, 16-byte
//     stores to the output.
// Prefixes saturate at 2^38 - 1 bytes (256 GiB, above any output buffer): past it every request
// with bytes is ENOSPC either way.
__global__ __launch_bounds__(64 * kFW) void fetch_kernel(FetchArgs a) {
  __shared__ u64 s_nb[kFW];
  __shared__ u64 s_pre;
  __shared__ u32 s_vid;
  const u32 lane = lane_id(), wv = threadIdx.x >> 6;
  if (threadIdx.x == 0)
    s_vid = (u32)(__hip_atomic_fetch_add(a.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.ticket_base);
  __syncthreads();
  const u32 vid = s_vid;
  const u32 r = vid * kFW + wv;
  const DevState& st = a.st;
  int status = kOk;
  u64 start = 0, count = 0, bytes = 0, pos0 = 0, ring_off = 0, rdesc = 0;
  if (r < a.n) {
    const u32 p = a.req[4 * r], c = a.req[4 * r + 1], mx = a.req[4 * r + 2];
    if (p >= st.P) {
      status = kNoPart;
    } else if (!st.is_leader[p]) {
      status = kNotLeader;
    } else if (c >= st.C) {
      status = kInval;
    } else {
      const u64 off = st.cons[(u64)p * st.C + c];
      start = off;
      u64 lim = off + mx;
      if (lim < off) lim = ~0ull;
      const u64 hw = st.hw[p];
      const u64 end = lim < hw ? lim : hw;
      if (off < end) {
        PartView v;
        v.leo = st.leo[p];
        v.used = st.used[p];
        v.start_off = st.start_off[p];
        v.start_pos = st.start_pos[p];
        if (off < v.start_off) {
          status = kOffset;
        } else {
          const u32 lm = st.local_mask[p];
          const u32 r0 = lm ? (u32)__ffs(lm) - 1u : 0u;
          rdesc = st.ring[p];
          v.rg = ring_ref(st, p);
          ring_off = (u64)r0 * st.rstride + v.rg.base;
          v.ring = st.logs + ring_off;
          const u64 pp = record_pos2(st, p, v, off, end);
          pos0 = __shfl(pp, 0, 64);
          bytes = __shfl(pp, 32, 64) - pos0;
          count = end - off;
        }
      }
    }
  }
  if (lane == 0) s_nb[wv] = bytes;
  __syncthreads();
  if (wv == 0) {
    u64 agg = 0;
#pragma unroll
    for (u32 k = 0; k < kFW; ++k) agg += s_nb[k];
    agg = sat38(agg);
    const u64 tag = (u64)a.epoch << 40;
    u64* const flags = a.flags;
    u64 pre = 0;
    if (vid == 0) {
      if (lane == 0) __hip_atomic_store(&flags[0], tag | ((u64)kFlagIncl << 38) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&flags[vid], tag | ((u64)kFlagAgg << 38) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // look back over the kLB x 64 workgroups before `top`, nearest first: lane l reads the words
      // of workgroups top - 1 - (kLB l + i), i < kLB (one round covers 1024 workgroups, so the
      // look-back of any workgroup takes few rounds however slowly inclusive words spread)
      long top = (long)vid;
      while (true) {
        u64 sum = 0;
        u32 first = kLB, ready_pre = 1u, ready_all = 1u;
#pragma unroll
        for (u32 i = 0; i < kLB; ++i) {
          const long q = top - 1 - (long)(kLB * lane + i);
          u64 w = tag | ((u64)kFlagIncl << 38);  // before the first workgroup: an inclusive 0
          if (q >= 0) w = __hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const u32 fl = (w >> 40) == a.epoch ? (u32)(w >> 38) & 3u : 0u;
          if (first == kLB) {  // still before this lane's nearest inclusive word
            if (!fl) ready_pre = 0u;
            sum += w & kVal38;
            if (fl == kFlagIncl) first = i;
          }
          if (!fl) ready_all = 0u;
        }
        const u64 has = __ballot(first < kLB);
        const u32 k = has ? (u32)__builtin_ctzll(has) : 64u;  // lane holding the nearest inclusive word
        // every word up to that one must be written (lanes before k: all of theirs; lane k: its prefix)
        const bool ok = lane < k ? ready_all != 0u : (lane == k ? ready_pre != 0u : true);
        if (!__all(ok)) {
          __builtin_amdgcn_s_sleep(2);
          continue;
        }
        u64 v = lane <= k ? sum : 0ull;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        pre = sat38(pre + v);
        if (k < 64u) break;
        top -= 64 * (long)kLB;
      }
      if (lane == 0) __hip_atomic_store(&flags[vid], tag | ((u64)kFlagIncl << 38) | sat38(pre + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_pre = pre;
      if (vid == a.nwg - 1) a.res[4ull * a.n] = sat38(pre + agg);  // bytes needed
    }
  }
  __syncthreads();
  if (r >= a.n) return;
  u64 pos = s_pre;
  for (u32 k = 0; k < wv; ++k) pos += s_nb[k];
  pos = sat38(pos);
  const bool served = bytes && pos + bytes <= a.out_cap;
  if (lane == 0) {
    const bool nospc = bytes && !served;
    a.res[4 * r + 0] = start;
    a.res[4 * r + 1] = pos;
    a.res[4 * r + 2] = nospc ? 0ull : (count | (bytes << 32));
    a.res[4 * r + 3] = (u64)(uint32_t)(nospc ? kNoSpc : status);
  }
  if (!served) return;
  const uint8_t* ring = st.logs + ring_off;
  const u64 mask = (1ull << (rdesc & 63ull)) - 1ull;
  uint8_t* out = a.out + pos;
  const u64 pieces = bytes >> 4;
  u64 q = lane;
  for (; q + 192 < pieces; q += 256) {  // four 16-byte pieces in flight per lane
    uint4 v[4];
#pragma unroll
    for (u32 u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * (q + 64 * u)) & mask));
#pragma unroll
    for (u32 u = 0; u < 4; ++u) *reinterpret_cast<uint4*>(out + 16ull * (q + 64 * u)) = v[u];
  }
  for (; q < pieces; q += 64)
    *reinterpret_cast<uint4*>(out + 16ull * q) = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * q) & mask));
}

u32 fetch_workgroups(u32 n) { return (n + kFW - 1) / kFW; }

// e0 / e1: events the dispatch itself records at the kernel's start and end (profiling), or null
void launch_fetch(const FetchArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  if (!a.n) return;
  hipExtLaunchKernelGGL(fetch_kernel, dim3(a.nwg), dim3(64 * kFW), 0, s, e0, e1, 0, a);
}

}  // namespace rmq
