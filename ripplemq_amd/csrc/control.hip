// control.hip — small per-partition kernels around the append path:
//   * quorum commit over all partitions (after external acks),
//   * external replica acks (matchIndex = max(matchIndex, ack)),
//   * leader start (term_start = log end; Raft matchIndex reset for remote replicas),
//   * consumer-offset commits (PartitionStateMachine.handleConsumerOffsetUpdateRequest,
//     mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:71-77): last writer wins;
//     the host keeps the last item per (partition, consumer), so this is a plain scatter.
#include "device_common.hpp"
#include "kernels.hpp"
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

__global__ void become_leader_kernel(DevState st, u32 only) {
  const u32 p = only == 0xFFFFFFFFu ? blockIdx.x * blockDim.x + threadIdx.x : only;
  if (p >= st.P || (only != 0xFFFFFFFFu && (blockIdx.x | threadIdx.x))) return;
  const u64 leo = st.leo[p];
  st.term_start[p] = leo;
  const u32 lm = st.local_mask[p];
  for (u32 r = 0; r < st.RF; ++r) st.match[(u64)p * st.RF + r] = (lm >> r & 1u) ? leo : 0ull;
}

__global__ void consumer_apply_kernel(ConsumerCommitArgs a) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) a.st.cons[(u64)a.pidx[i] * a.st.C + a.consumer[i]] = a.offset[i];
}

static inline dim3 grid_for(u32 n, u32 b) { return dim3((n + b - 1) / b ? (n + b - 1) / b : 1); }

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

}  // namespace rmq
