// transport.hpp — how replica-log rounds move between engines.
//
// The engine only ever needs one collective shape: a grouped point-to-point exchange in which
// every rank sends a byte range to each peer and receives one from each peer, sizes known on both
// sides beforehand (they travel in an earlier exchange of 8-byte words). Two implementations:
//   * RcclTransport — ncclSend/ncclRecv inside one ncclGroupStart/End on the engine's exchange
//     stream: RCCL over xGMI, one process per GPU (the reference's jraft AppendEntries RPCs between
//     brokers, PartitionRaftServer.java:82-93, MessageAppendRequestProcessor.java:59);
//   * LocalTransport — engines of one process (any devices, the same one included) exchange by
//     device-to-device copies ordered with events; each rank's engine is driven by its own host
//     thread, and a host barrier stands in for the collective. It checks that the sizes every pair
//     announced agree and fails instead of hanging (tests on a single GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <mutex>
#include <vector>

namespace rmq {

class Transport {
 public:
  virtual ~Transport() {}
  virtual uint32_t world() const = 0;
  virtual uint32_t rank() const = 0;
  // For every peer q != rank(): send sbytes[q] bytes at sbuf[q] to q and receive rbytes[q] bytes
  // from q into rbuf[q], ordered on stream s. Zero-byte transfers are skipped (both sides know the
  // sizes). Every rank must make the same sequence of calls. Returns 0 or a negative RMQ_ status.
  virtual int exchange(void* const* sbuf, const uint64_t* sbytes, void* const* rbuf, const uint64_t* rbytes,
                       hipStream_t s) = 0;
};

// In-process rendezvous of `world` engines (one host thread per rank).
struct LocalHub {
  explicit LocalHub(uint32_t w);
  ~LocalHub();
  // Host barrier over the world; false on timeout (a rank stopped calling: the test has a bug).
  bool barrier();
  uint32_t world;
  std::mutex mu;
  std::condition_variable cv;
  uint32_t arrived = 0;
  uint64_t generation = 0;
  // posted by each rank for the current exchange
  std::vector<void*> sbuf;        // [src][dst]
  std::vector<uint64_t> sbytes;   // [src][dst]
  std::vector<uint64_t> rbytes;   // [dst][src]
  std::vector<int> device;        // [rank]
  std::vector<hipEvent_t> posted;  // [rank] sends ready
  std::vector<hipEvent_t> copied;  // [rank] its receives done (the senders' buffers are free again)
};

Transport* make_local_transport(LocalHub* hub, uint32_t rank, int device);
// comm_id: NCCL_UNIQUE_ID_BYTES from rmq_rccl_unique_id on one rank, shared by the application.
// Collective over the world (every rank calls it). Returns nullptr on failure.
Transport* make_rccl_transport(const uint8_t* comm_id, uint32_t world, uint32_t rank);
int rccl_unique_id(uint8_t* out);  // 0 or negative status

}  // namespace rmq
