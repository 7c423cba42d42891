// transport.cpp — RCCL and in-process implementations of rmq::Transport (transport.hpp).
#include "transport.hpp"

#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#include "../../include/ripplemq_engine.h"

namespace rmq {

namespace {

constexpr auto kBarrierTimeout = std::chrono::seconds(120);

class RcclTransport : public Transport {
 public:
  RcclTransport(ncclComm_t c, uint32_t w, uint32_t r) : comm_(c), world_(w), rank_(r) {}
  ~RcclTransport() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  uint32_t world() const override { return world_; }
  uint32_t rank() const override { return rank_; }
  int exchange(void* const* sbuf, const uint64_t* sbytes, void* const* rbuf, const uint64_t* rbytes,
               hipStream_t s) override {
    if (ncclGroupStart() != ncclSuccess) return RMQ_EDEVICE;
    ncclResult_t r = ncclSuccess;
    for (uint32_t q = 0; q < world_ && r == ncclSuccess; ++q) {
      if (q == rank_) continue;
      if (sbytes[q]) r = ncclSend(sbuf[q], sbytes[q], ncclUint8, (int)q, comm_, s);
      if (r == ncclSuccess && rbytes[q]) r = ncclRecv(rbuf[q], rbytes[q], ncclUint8, (int)q, comm_, s);
    }
    const ncclResult_t e = ncclGroupEnd();
    if (r != ncclSuccess || e != ncclSuccess) {
      std::fprintf(stderr, "ripplemq: RCCL exchange failed: %s\n", ncclGetErrorString(r != ncclSuccess ? r : e));
      return RMQ_EDEVICE;
    }
    return RMQ_OK;
  }

 private:
  ncclComm_t comm_;
  uint32_t world_, rank_;
};

class LocalTransport : public Transport {
 public:
  LocalTransport(LocalHub* h, uint32_t r, int dev) : hub_(h), rank_(r), device_(dev) {}
  uint32_t world() const override { return hub_->world; }
  uint32_t rank() const override { return rank_; }
  int exchange(void* const* sbuf, const uint64_t* sbytes, void* const* rbuf, const uint64_t* rbytes,
               hipStream_t s) override {
    LocalHub& h = *hub_;
    const uint32_t W = h.world, me = rank_;
    // 1. post: our send ranges and the sizes we expect, sends ready once stream s reaches here
    if (hipEventRecord(h.posted[me], s) != hipSuccess) return RMQ_EDEVICE;
    {
      std::lock_guard<std::mutex> g(h.mu);
      for (uint32_t q = 0; q < W; ++q) {
        h.sbuf[(size_t)me * W + q] = sbuf[q];
        h.sbytes[(size_t)me * W + q] = q == me ? 0 : sbytes[q];
        h.rbytes[(size_t)me * W + q] = q == me ? 0 : rbytes[q];
      }
      h.device[me] = device_;
    }
    if (!h.barrier()) return RMQ_EDEVICE;
    // 2. every rank sees every posted size: a mismatch anywhere fails the exchange on all ranks
    //    (no shared flag to reset), then copy from every peer's send range once its stream posted it
    bool bad = false;
    for (uint32_t q = 0; q < W; ++q)
      for (uint32_t t = 0; t < W; ++t)
        if (q != t && h.sbytes[(size_t)q * W + t] != h.rbytes[(size_t)t * W + q]) {
          if (t == me)
            std::fprintf(stderr, "ripplemq: local exchange size mismatch %u->%u: sent %llu, expected %llu\n", q, me,
                         (unsigned long long)h.sbytes[(size_t)q * W + me],
                         (unsigned long long)h.rbytes[(size_t)me * W + q]);
          bad = true;
        }
    for (uint32_t q = 0; q < W && !bad; ++q) {
      const uint64_t n = q == me ? 0 : h.rbytes[(size_t)me * W + q];
      if (!n) continue;
      if (hipStreamWaitEvent(s, h.posted[q], 0) != hipSuccess) return RMQ_EDEVICE;
      if (hipMemcpyPeerAsync(rbuf[q], device_, h.sbuf[(size_t)q * W + me], h.device[q], n, s) != hipSuccess)
        return RMQ_EDEVICE;
    }
    if (hipEventRecord(h.copied[me], s) != hipSuccess) return RMQ_EDEVICE;
    // every rank has read the posted table and recorded its copies: a rank may post the next
    // exchange from here (it records `posted` again, never `copied` before the next barrier)
    if (!h.barrier()) return RMQ_EDEVICE;
    // 3. our send buffers may be rewritten only after every receiver's copies
    for (uint32_t q = 0; q < W; ++q)
      if (q != me && h.sbytes[(size_t)me * W + q] && hipStreamWaitEvent(s, h.copied[q], 0) != hipSuccess)
        return RMQ_EDEVICE;
    return bad ? RMQ_EINVAL : RMQ_OK;
  }

 private:
  LocalHub* hub_;
  uint32_t rank_;
  int device_;
};

}  // namespace

LocalHub::LocalHub(uint32_t w) : world(w) {
  sbuf.assign((size_t)w * w, nullptr);
  sbytes.assign((size_t)w * w, 0);
  rbytes.assign((size_t)w * w, 0);
  device.assign(w, 0);
  posted.assign(w, nullptr);
  copied.assign(w, nullptr);
  for (uint32_t r = 0; r < w; ++r) {
    hipEventCreateWithFlags(&posted[r], hipEventDisableTiming);
    hipEventCreateWithFlags(&copied[r], hipEventDisableTiming);
  }
}

LocalHub::~LocalHub() {
  for (hipEvent_t e : posted)
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : copied)
    if (e) hipEventDestroy(e);
}

bool LocalHub::barrier() {
  std::unique_lock<std::mutex> g(mu);
  const uint64_t gen = generation;
  if (++arrived == world) {
    arrived = 0;
    ++generation;
    cv.notify_all();
    return true;
  }
  return cv.wait_for(g, kBarrierTimeout, [&] { return generation != gen; });
}

Transport* make_local_transport(LocalHub* hub, uint32_t rank, int device) {
  return new LocalTransport(hub, rank, device);
}

Transport* make_rccl_transport(const uint8_t* comm_id, uint32_t world, uint32_t rank) {
  ncclUniqueId id;
  std::memcpy(id.internal, comm_id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, (int)world, id, (int)rank);
  if (r != ncclSuccess) {
    std::fprintf(stderr, "ripplemq: ncclCommInitRank failed: %s\n", ncclGetErrorString(r));
    return nullptr;
  }
  return new RcclTransport(c, world, rank);
}

int rccl_unique_id(uint8_t* out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return RMQ_EDEVICE;
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return RMQ_OK;
}

}  // namespace rmq
