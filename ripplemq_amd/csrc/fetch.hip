// fetch.hip — batched consumer fetch: PartitionStateMachine.handleBatchRead
// (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:85-110), served directly from
// committed state like MessageBatchReadRequestProcessor.java:39 (no read-index).
//
//  resolve (lane per request): off = consumerOffsets.getOrDefault(id, 0); end = min(off + max, hw);
//          byte range of records [off, end) by binary search of the sparse offset index
//          (FORMAT.md §5: E[m] = first record starting at or after m*I) plus a short header walk;
//  place   (one workgroup): exclusive scans of request bytes -> output positions (ENOSPC marking)
//          and of request 1 KiB chunks -> the gather's work list;
//  gather  (wave per 1 KiB chunk of one request, grid-stride): 16-byte loads from the leader ring
//          and 16-byte stores to the output. Records and output positions are 16-byte aligned
//          (FORMAT.md §1), so no piece straddles a record, the ring end or an output boundary.
//
// The three kernels run on the engine's fetch stream, after the last pipeline launch the host had
// issued and before the next one (engine.cpp orders the two streams with events), so the committed
// state they read is stable and the append pipeline is never flushed for a fetch.
#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr int kOk = 0, kNotLeader = -1, kNoPart = -2, kInval = -3, kNoSpc = -4, kOffset = -6;
constexpr u32 kChunkLog2 = 10;  // gather chunk: 1 KiB = 64 lanes x 16 B

struct PartView {
  u64 leo, used, start_off, start_pos;
  const uint8_t* ring;  // lowest local replica ring of the partition
};

// Logical byte position of record t, start_off <= t <= leo.
__device__ u64 record_pos(const DevState& st, u32 p, const PartView& v, u64 t) {
  if (t == v.leo) return v.used;
  const u32 ilog = st.interval_log2;
  const u64 I = 1ull << ilog;
  u64 c_off = v.start_off, c_pos = v.start_pos;
  long lo = (long)((v.start_pos + I - 1) >> ilog), hi = (long)(v.used >> ilog);
  const u64* E = st.index + (u64)p * st.icap * 2;
  while (lo <= hi) {  // largest m with E[m].offset <= t
    const long mid = lo + ((hi - lo) >> 1);
    const u64* e = E + ((u64)mid % st.icap) * 2;
    const u64 eo = e[0];
    if (eo <= t) {
      c_off = eo;
      c_pos = e[1];
      lo = mid + 1;
    } else {
      hi = mid - 1;
    }
  }
  const u64 mask = st.seg - 1;
  for (u32 guard = 0; c_off < t && guard < (1u << 20); ++guard) {  // at most ~I / 16 records
    const u32 L = *reinterpret_cast<const u32*>(v.ring + ((c_pos + 8) & mask));
    c_pos += record_bytes(L);
    ++c_off;
  }
  return c_pos;
}

__global__ void fetch_resolve_kernel(FetchArgs a) {
  const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
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
        ring_off = ((u64)r0 * st.P + p) * st.seg;
        v.ring = st.logs + ring_off;
        pos0 = record_pos(st, p, v, off);
        bytes = record_pos(st, p, v, end) - pos0;
        count = end - off;
      }
    }
  }
  a.res[4 * r + 0] = start;
  a.res[4 * r + 2] = count | (bytes << 32);
  a.res[4 * r + 3] = (u64)(uint32_t)status;
  a.aux[2 * r + 0] = pos0;
  a.aux[2 * r + 1] = ring_off;
}

__global__ __launch_bounds__(1024) void fetch_place_kernel(FetchArgs a) {
  __shared__ u64 sh[16];
  __shared__ u64 shc[16];
  const u32 tid = threadIdx.x, T = blockDim.x, l = tid & 63, w = tid >> 6;
  const u32 per = (a.n + T - 1) / T;
  const u32 b = tid * per, e = b + per < a.n ? b + per : a.n;
  u64 local = 0;
  for (u32 r = b; r < e; ++r) local += a.res[4 * r + 2] >> 32;
  // output positions: every request's bytes count, served or not (FORMAT.md §7)
  const u64 inc = wave_incl_scan(local);
  if (l == 63) sh[w] = inc;
  __syncthreads();
  u64 cur = inc - local, tot = 0;
  for (u32 k = 0; k < 16; ++k) {
    cur += k < w ? sh[k] : 0ull;
    tot += sh[k];
  }
  u64 lch = 0;
  for (u32 r = b; r < e; ++r) {
    const u64 cb = a.res[4 * r + 2];
    const u64 nb = cb >> 32;
    a.res[4 * r + 1] = cur;
    if (nb && cur + nb > a.out_cap) {
      a.res[4 * r + 2] = 0;
      a.res[4 * r + 3] = (u64)(uint32_t)kNoSpc;
    } else {
      lch += (nb + (1ull << kChunkLog2) - 1) >> kChunkLog2;
    }
    cur += nb;
  }
  // gather work list: chunks of the requests that are served
  const u64 cinc = wave_incl_scan(lch);
  if (l == 63) shc[w] = cinc;
  __syncthreads();
  u64 ccur = cinc - lch, ctot = 0;
  for (u32 k = 0; k < 16; ++k) {
    ccur += k < w ? shc[k] : 0ull;
    ctot += shc[k];
  }
  for (u32 r = b; r < e; ++r) {
    a.cpre[r] = (u32)ccur;
    const u64 nb = a.res[4 * r + 2] >> 32;
    ccur += (nb + (1ull << kChunkLog2) - 1) >> kChunkLog2;
  }
  if (tid == 0) {
    a.cpre[a.n] = (u32)ctot;
    a.total[0] = tot;
    a.total[1] = ctot;
  }
}

__global__ __launch_bounds__(256) void fetch_gather_kernel(FetchArgs a) {
  const DevState& st = a.st;
  const u64 mask = st.seg - 1;
  const u32 lane = threadIdx.x & 63;
  const u32 nw = gridDim.x * (blockDim.x >> 6);
  const u32 chunks = (u32)a.total[1];
  for (u32 c = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); c < chunks;
       c += nw) {
    // request of chunk c: the last r with cpre[r] <= c (requests without chunks are skipped)
    u32 lo = 0, hi = a.n;  // cpre[lo] <= c < cpre[hi]
    while (hi - lo > 1) {
      const u32 mid = (lo + hi) >> 1;
      if (a.cpre[mid] <= c) lo = mid; else hi = mid;
    }
    const u32 r = lo;
    const u64 nb = a.res[4 * r + 2] >> 32;
    const u64 pos0 = a.aux[2 * r + 0];
    const uint8_t* ring = st.logs + a.aux[2 * r + 1];
    uint8_t* out = a.out + a.res[4 * r + 1];
    const u64 piece = ((u64)(c - a.cpre[r]) << (kChunkLog2 - 4)) + lane;
    if (16ull * piece < nb) {
      const uint4 v = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * piece) & mask));
      *reinterpret_cast<uint4*>(out + 16ull * piece) = v;
    }
  }
}

void launch_fetch(const FetchArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1, hipEvent_t g0,
                  hipEvent_t g1) {
  if (!a.n) return;
  if (e0) hipEventRecord(e0, s);
  hipLaunchKernelGGL(fetch_resolve_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
  hipLaunchKernelGGL(fetch_place_kernel, dim3(1), dim3(1024), 0, s, a);
  if (e1) hipEventRecord(e1, s);
  if (g0) hipEventRecord(g0, s);
  hipLaunchKernelGGL(fetch_gather_kernel, dim3(a.gather_wgs), dim3(256), 0, s, a);
  if (g1) hipEventRecord(g1, s);
}

}  // namespace rmq
