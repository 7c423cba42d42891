// fetch.hip — batched consumer fetch: PartitionStateMachine.handleBatchRead
// (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:85-110), served directly from
// committed state like MessageBatchReadRequestProcessor.java:39 (no read-index).
//
//  resolve (wave per request): off = consumerOffsets.getOrDefault(id, 0); end = min(off + max, hw);
//          byte range of records [off, end): a 64-ary search of the sparse offset index (FORMAT.md
//          §5: E[m] = first record starting at or after m*I; 64 probes per round, one round per
//          factor 64 of index entries), then the record headers of the 1 KiB after the entry found
//          are loaded at once (a lane per 16 bytes) and walked in registers;
//  place   (one workgroup): exclusive scan of the requests' bytes -> compact output positions
//          (into the result rows' out_pos), ENOSPC marking (every request's bytes count, served or
//          not: FORMAT.md §7);
//  gather  (wave per request): 16-byte loads from the lowest local replica ring, four in flight per
//          lane, 16-byte stores to the output. Records and output positions are 16-byte aligned
//          (FORMAT.md §1), so no piece straddles a record, the ring end or an output boundary.
//
// The three kernels run on the engine's fetch stream, after the last pipeline launch the host had
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

__global__ __launch_bounds__(64 * kFW) void fetch_resolve_kernel(FetchArgs a) {
  const u32 r = __builtin_amdgcn_readfirstlane(blockIdx.x * kFW + (threadIdx.x >> 6));
  if (r >= a.n) return;
  const DevState& st = a.st;
  const u32 p = a.req[4 * r], c = a.req[4 * r + 1], mx = a.req[4 * r + 2];
  int status = kOk;
  u64 start = 0, count = 0, bytes = 0, pos0 = 0, ring_off = 0;
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
  if (lane_id() == 0) {
    a.res[4 * r + 0] = start;
    a.res[4 * r + 2] = count | (bytes << 32);
    a.res[4 * r + 3] = (u64)(uint32_t)status;
    a.aux[2 * r + 0] = pos0;
    a.aux[2 * r + 1] = (ring_off << 6) | (st.ring[p < st.P ? p : 0] & 63ull);  // ring | log2(ring bytes)
    a.cpre[r] = (u32)bytes;
  }
}

// One workgroup: output positions = exclusive scan of the requests' bytes in request order; each
// thread scans 16 consecutive requests per pass (16-byte loads of the byte counts, 16-byte stores of
// the compact positions: one load round per 16384 requests).
__global__ __launch_bounds__(1024) void fetch_place_kernel(FetchArgs a) {
  __shared__ u64 sh[16];
  constexpr u32 kPer = 16;
  const u32 tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  u64 carry = 0;
  for (u32 b = 0; b < a.n; b += 1024 * kPer) {
    const u32 r0 = b + tid * kPer;
    u32 nb[kPer];
    if (r0 + kPer <= a.n) {
      const uint4* src = reinterpret_cast<const uint4*>(a.cpre + r0);
#pragma unroll
      for (u32 k = 0; k < kPer / 4; ++k) {
        const uint4 v = src[k];
        nb[4 * k] = v.x;
        nb[4 * k + 1] = v.y;
        nb[4 * k + 2] = v.z;
        nb[4 * k + 3] = v.w;
      }
    } else {
#pragma unroll
      for (u32 k = 0; k < kPer; ++k) nb[k] = r0 + k < a.n ? a.cpre[r0 + k] : 0u;
    }
    u64 loc = 0;
#pragma unroll
    for (u32 k = 0; k < kPer; ++k) loc += nb[k];
    const u64 inc = wave_incl_scan(loc);
    if (l == 63) sh[w] = inc;
    __syncthreads();
    u64 cur = carry + inc - loc, tot = 0;
#pragma unroll
    for (u32 k = 0; k < 16; ++k) {
      cur += k < w ? sh[k] : 0ull;
      tot += sh[k];
    }
    u64 pos[kPer];
#pragma unroll
    for (u32 k = 0; k < kPer; ++k) {
      pos[k] = cur;
      if (nb[k] && cur + nb[k] > a.out_cap && r0 + k < a.n) {  // does not fit: not served (rare)
        a.res[4 * (r0 + k) + 2] = 0;
        a.res[4 * (r0 + k) + 3] = (u64)(uint32_t)kNoSpc;
      }
      cur += nb[k];
    }
#pragma unroll
    for (u32 k = 0; k < kPer; ++k)
      if (r0 + k < a.n) a.res[4 * (r0 + k) + 1] = pos[k];  // out_pos (one result copy to the host)
    carry += tot;
    __syncthreads();
  }
  if (tid == 0) a.res[4ull * a.n] = carry;  // bytes needed
}

__global__ __launch_bounds__(64 * kFW) void fetch_gather_kernel(FetchArgs a) {
  const DevState& st = a.st;
  const u32 lane = lane_id();
  const u32 nw = gridDim.x * kFW;
  for (u32 r = __builtin_amdgcn_readfirstlane(blockIdx.x * kFW + (threadIdx.x >> 6)); r < a.n; r += nw) {
    const u64 nb = a.res[4 * r + 2] >> 32;  // 0 for requests not served
    if (!nb) continue;
    const u64 pos0 = a.aux[2 * r + 0];
    const uint8_t* ring = st.logs + (a.aux[2 * r + 1] >> 6);
    const u64 mask = (1ull << (a.aux[2 * r + 1] & 63ull)) - 1ull;
    uint8_t* out = a.out + a.res[4 * r + 1];
    const u64 pieces = nb >> 4;
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
}

// ev[6]: start / end events of the three kernels, recorded by the dispatches themselves
// (profiling: kernel time without the host's launch gaps), or null
void launch_fetch(const FetchArgs& a, hipStream_t s, const hipEvent_t* ev) {
  if (!a.n) return;
  const hipEvent_t* e = ev;
  hipExtLaunchKernelGGL(fetch_resolve_kernel, dim3((a.n + kFW - 1) / kFW), dim3(64 * kFW), 0, s, e ? e[0] : nullptr,
                        e ? e[1] : nullptr, 0, a);
  hipExtLaunchKernelGGL(fetch_place_kernel, dim3(1), dim3(1024), 0, s, e ? e[2] : nullptr, e ? e[3] : nullptr, 0, a);
  hipExtLaunchKernelGGL(fetch_gather_kernel, dim3(std::min<u32>((a.n + kFW - 1) / kFW, a.gather_wgs)), dim3(64 * kFW), 0,
                        s, e ? e[4] : nullptr, e ? e[5] : nullptr, 0, a);
}

}  // namespace rmq
