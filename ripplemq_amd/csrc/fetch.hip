// fetch.hip — batched consumer fetch: PartitionStateMachine.handleBatchRead
// (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:85-110), served directly from
// committed state like MessageBatchReadRequestProcessor.java:39 (no read-index).
//
//  resolve (lane per request): off = consumerOffsets.getOrDefault(id, 0); end = min(off + max, hw);
//          byte range of records [off, end) by binary search of the sparse offset index
//          (FORMAT.md §5: E[m] = first record starting at or after m*I) plus a short header walk;
//  place   (one workgroup): exclusive scan of request bytes -> output positions, ENOSPC marking;
//  gather  (workgroup per request): dword copy out of the leader ring, contiguous on both sides.
#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr int kOk = 0, kNotLeader = -1, kNoPart = -2, kInval = -3, kNoSpc = -4, kOffset = -6;

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
  u64 start = 0, count = 0, bytes = 0, pos0 = 0;
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
        v.ring = st.logs + ((u64)r0 * st.P + p) * st.seg;
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
  a.aux[2 * r + 1] = p;
}

__global__ __launch_bounds__(1024) void fetch_place_kernel(FetchArgs a) {
  __shared__ u64 sh[16];
  const u32 tid = threadIdx.x, T = blockDim.x;
  const u32 per = (a.n + T - 1) / T;
  const u32 b = tid * per, e = b + per < a.n ? b + per : a.n;
  u64 local = 0;
  for (u32 r = b; r < e; ++r) local += a.res[4 * r + 2] >> 32;
  u64 tot;
  u64 cur = block_excl_scan<16>(local, sh, &tot);
  for (u32 r = b; r < e; ++r) {
    const u64 cb = a.res[4 * r + 2];
    const u64 nb = cb >> 32;
    a.res[4 * r + 1] = cur;
    if (nb && cur + nb > a.out_cap) {
      a.res[4 * r + 2] = 0;
      a.res[4 * r + 3] = (u64)(uint32_t)kNoSpc;
    }
    cur += nb;
  }
  if (tid == 0) a.total[0] = tot;
}

__global__ __launch_bounds__(256) void fetch_gather_kernel(FetchArgs a) {
  const DevState& st = a.st;
  const u64 mask = st.seg - 1;
  for (u32 r = blockIdx.x; r < a.n; r += gridDim.x) {
    const u64 nb = a.res[4 * r + 2] >> 32;
    if (!nb) continue;
    const u32 p = (u32)a.aux[2 * r + 1];
    const u64 pos0 = a.aux[2 * r + 0];
    const u64 op = a.res[4 * r + 1];
    const u32 lm = st.local_mask[p];
    const u32 r0 = lm ? (u32)__ffs(lm) - 1u : 0u;
    const uint8_t* ring = st.logs + ((u64)r0 * st.P + p) * st.seg;
    u32* out = reinterpret_cast<u32*>(a.out + op);
    const u64 ndw = nb >> 2;
    for (u64 d = threadIdx.x; d < ndw; d += blockDim.x)
      out[d] = *reinterpret_cast<const u32*>(ring + ((pos0 + 4 * d) & mask));
  }
}

void launch_fetch(const FetchArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1, hipEvent_t g0,
                  hipEvent_t g1) {
  if (!a.n) return;
  if (e0) hipEventRecord(e0, s);
  hipLaunchKernelGGL(fetch_resolve_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
  if (e1) hipEventRecord(e1, s);
  hipLaunchKernelGGL(fetch_place_kernel, dim3(1), dim3(1024), 0, s, a);
  if (g0) hipEventRecord(g0, s);
  const u32 grid = a.n < 8192 ? a.n : 8192;
  hipLaunchKernelGGL(fetch_gather_kernel, dim3(grid), dim3(256), 0, s, a);
  if (g1) hipEventRecord(g1, s);
}

}  // namespace rmq
