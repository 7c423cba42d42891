// replication.cpp — replica-log rounds between engines over a Transport (FORMAT.md §9).
//
// Reference: each partition is a jraft group whose leader replicates its log to RF-1 followers
// with AppendEntries and commits on a quorum of acks (BallotBox) — configured in
// PartitionRaftServer.java:82-93 (peers of the group), started by node.apply at
// MessageAppendRequestProcessor.java:59; replicas are spread over brokers by
// PartitionAssigner.java:25-94. Here one engine per GPU leads some partitions and follows others
// (rmq_set_placement); every launch group of appends is one round:
//
//   launch k+1 (stage 2 of group g): the last stage-2 workgroup plans g's outbox (pipeline.hip);
//       after it, the exchange stream swaps {region bytes, records} with every peer;
//   launch k+2 (stage 3 of g): records also go, once per remote slot, into g's outbox;
//   after launch k+3 is issued: the host reads g's sizes (exchanged one launch earlier) and posts
//       on the exchange stream, behind launch k+2: the grouped send/recv of the regions, the
//       follower ingest (CRC32C check, ring + index writes, log end, retention; replicate.hip) and
//       the grouped send/recv of the acks (follower log ends);
//   launch k+5 (three launches after g's stage 3): waits for g's exchange and applies the acks to
//       the matchIndex rows in its partition threads, then the quorum commit rule; the plan of the
//       group that launch scans reads the same acks for its catch-up verdicts (FORMAT.md §9 v3:
//       a refused entry's next round starts at the follower's log end, the gap re-sent from the
//       leader's ring by the catch-up waves of the stage-3 launch).
//
// Every rank makes the same calls in the same order (rounds are collective, like the launches
// that drive them): with a transport attached, launch groups close only when full, and control
// calls that flush (rmq_sync, placement, leadership) are collective. At a drain the remaining
// rounds are exchanged and their acks applied by a separate kernel.
#include <chrono>
#include <numeric>

#include "engine_internal.hpp"

namespace rmq {

namespace {

template <typename T>
int upload(T** d, const std::vector<T>& h) {
  if (*d) hipFree(*d);
  *d = nullptr;
  int rc = dalloc(d, h.size());
  if (rc || h.empty()) return rc;
  HIP_TRY(hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return RMQ_OK;
}

struct Entry {
  uint64_t key;
  uint32_t slot, p;
  bool operator<(const Entry& o) const { return key != o.key ? key < o.key : slot < o.slot; }
};

uint64_t entry_hash(uint64_t key, uint32_t slot) { return key * RMQ_MAX_RF + slot; }

void free_set_buffers(Replication* r) {
  for (XchgSet& x : r->sets) {
    void* bufs[] = {x.outbox, x.inbox, x.xe, x.xc, x.xc_n, x.sizes, x.ackout, x.ackin, x.rowv};
    for (void* p : bufs)
      if (p) hipFree(p);
    x.outbox = x.inbox = nullptr;
    x.xe = nullptr;
    x.xc = nullptr;
    x.xc_n = nullptr;
    x.sizes = x.ackout = x.ackin = x.rowv = nullptr;
  }
}

}  // namespace

// The leader's catch-up state of every out entry starts over (FORMAT.md §9: placement and leader
// start): next = the leader's log end, no request, no catch-up round. Engine drained.
int reset_catchup(rmq_engine* e) {
  Replication* r = e->repl;
  const size_t n = r->xo_p.size();
  if (!n) return RMQ_OK;
  const uint32_t P = e->cfg.num_partitions;
  std::vector<uint64_t> leo(P), used(P), nx(2 * n);
  HIP_TRY(hipMemcpy(leo.data(), e->st.leo, P * 8ull, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(used.data(), e->st.used, P * 8ull, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < n; ++k) {
    nx[2 * k] = leo[r->xo_p[k]];
    nx[2 * k + 1] = used[r->xo_p[k]];
  }
  HIP_TRY(hipMemcpy(r->d_xnext, nx.data(), nx.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(r->d_xreq, 0, n * 32));
  HIP_TRY(hipMemset(r->d_xcu, 0, n * 8));
  return RMQ_OK;
}

namespace {

// Post the {region bytes, records} swap of the group in set s (after its stage-2 launch). drop: the
// leader sends no region this round; lost: bit q, the region to q is lost (rmq_fault_isolate).
int post_sizes(rmq_engine* e, uint32_t s, bool drop, uint32_t lost) {
  Replication* r = e->repl;
  XchgSet& x = r->sets[s];
  const uint32_t W = r->world;
  void* sb[kMaxWorld];
  void* rb[kMaxWorld];
  uint64_t n16[kMaxWorld];
  for (uint32_t q = 0; q < W; ++q) {
    sb[q] = x.sizes + 2 * q;
    rb[q] = x.sizes + 2 * W + 2 * q;
    n16[q] = q == r->rank ? 0 : 16;
  }
  HIP_TRY(hipStreamWaitEvent(r->xchg_s, x.ev_s2, 0));
  if (drop) HIP_TRY(hipMemsetAsync(x.sizes, 0, 2ull * W * 8, r->xchg_s));  // no region to anyone
  for (uint32_t q = 0; q < W && !drop; ++q)
    if ((lost >> q) & 1u) HIP_TRY(hipMemsetAsync(x.sizes + 2 * q, 0, 16, r->xchg_s));
  int rc = r->xport->exchange(sb, n16, rb, n16, r->xchg_s);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(x.h_sizes, x.sizes, 4ull * W * 8, hipMemcpyDeviceToHost, r->xchg_s));
  HIP_TRY(hipEventRecord(x.ev_sz, r->xchg_s));
  return RMQ_OK;
}

// Post the round of the group in set s (applied already): regions, follower ingest, acks.
int post_round(rmq_engine* e, uint32_t s) {
  Replication* r = e->repl;
  XchgSet& x = r->sets[s];
  const uint32_t W = r->world, me = r->rank;
  // RCCL's grouped send/recv take host-side byte counts: the sizes were swapped one launch earlier,
  // so this normally finds them landed; a wait is counted (rmq_repl_stats.host_waits)
  if (hipEventQuery(x.ev_sz) == hipErrorNotReady) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = event_wait(x.ev_sz);
    if (rc) return rc;
    r->host_waits++;
    r->host_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  }
  const uint64_t* hs = x.h_sizes;  // [q]: {send bytes, send records}, then [W + q]: {recv bytes, recv records}
  void* sb[kMaxWorld];
  void* rb[kMaxWorld];
  uint64_t sn[kMaxWorld], rn[kMaxWorld];
  IngestArgs a{};
  uint64_t ro = 0, smax = 0;
  uint32_t tasks = 0;
  const uint64_t kvr = verify_records_per_task();
  for (uint32_t q = 0; q < W; ++q) {
    sn[q] = q == me ? 0 : hs[2 * q];
    rn[q] = q == me ? 0 : hs[2 * W + 2 * q];
    sb[q] = x.outbox + (uint64_t)q * r->dcap;
    rb[q] = x.inbox + ro;
    a.region[q] = ro;
    a.rbytes[q] = rn[q];
    a.task0[q] = tasks;
    tasks += (uint32_t)((rn[q] ? hs[2 * W + 2 * q + 1] : 0) + kvr - 1) / kvr;
    smax = std::max(smax, sn[q]);
    ro += (rn[q] + 15) & ~15ull;
  }
  a.task0[W] = tasks;
  if (smax > r->dcap || ro > r->in_cap) {
    std::fprintf(stderr, "ripplemq: replication round exceeds its buffers (%llu/%llu out, %llu/%llu in)\n",
                 (unsigned long long)smax, (unsigned long long)r->dcap, (unsigned long long)ro,
                 (unsigned long long)r->in_cap);
    return RMQ_EDEVICE;
  }
  // copy work items: at most one per 16 KiB of received region bytes plus one per entry
  const uint32_t items = (uint32_t)std::min<uint64_t>(r->items_cap, ro / kCopyChunk + W + r->xi_p.size());
  HIP_TRY(hipStreamWaitEvent(r->xchg_s, x.ev_s3, 0));
  for (uint32_t q = 0; q < W; ++q)  // rmq_fault_corrupt
    if (r->flip[q] && sn[q]) {
      launch_flip(static_cast<uint8_t*>(sb[q]), sn[q], r->flip_at[q], r->xchg_s);
      r->flip[q] = false;
    }
  int rc = r->xport->exchange(sb, sn, rb, rn, r->xchg_s);
  if (rc) return rc;
  a.st = e->st;
  a.sets[0] = e->sets[0];
  a.sets[1] = e->sets[1];
  a.inbox = x.inbox;
  a.xi_p = r->d_xi_p;
  a.xi_slot = r->d_xi_slot;
  a.xi_start = r->d_xi_start;
  a.world = W;
  a.rank = me;
  a.n_in = (uint32_t)r->xi_p.size();
  a.C = e->cfg.max_consumers;
  a.bad = r->d_bad;
  a.acc = r->d_acc;
  a.base = r->d_base;
  a.cdesc = r->d_cdesc;
  a.ackout = x.ackout;
  a.items = r->d_items;
  {
    constexpr uint32_t NW = 1 + kMaxWorld;
    uint32_t* cur = r->d_nitems + (r->nitems_par ? NW : 0u);
    a.n_items = cur;
    a.insane = cur + 1;
    a.n_items_next = r->d_nitems + (r->nitems_par ? 0u : NW);
  }
  a.keysum_in = r->d_keysum_in;
  a.items_cap = (uint32_t)r->items_cap;
  a.items_grid = items;
  a.crc = e->d_crc;
  a.counters = r->d_counters;
  a.stamp = x.round + 1ull;  // (rmq_leader_silent's clock: rounds ingested)
  if (a.stamp > r->stamp) r->stamp = a.stamp;
  r->stamp_time[a.stamp % 64] = std::chrono::steady_clock::now();
  launch_ingest(a, tasks, items, e->verify_wgs, r->xchg_s);
  if (a.n_in) r->nitems_par ^= 1u;  // (prepare ran: it cleared the other half)
  HIP_TRY(hipGetLastError());
  // acks: {log end | status, position} of every in entry back to its leader, fixed sizes both ways
  for (uint32_t q = 0; q < W; ++q) {
    sn[q] = q == me ? 0 : 16ull * (r->xi_start[q + 1] - r->xi_start[q]);
    rn[q] = q == me ? 0 : 16ull * (r->xo_start[q + 1] - r->xo_start[q]);
    sb[q] = x.ackout + 2ull * r->xi_start[q];
    rb[q] = x.ackin + 2ull * r->xo_start[q];
  }
  rc = r->xport->exchange(sb, sn, rb, rn, r->xchg_s);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(x.ev_x, r->xchg_s));
  r->rounds++;
  for (uint32_t q = 0; q < W; ++q) r->bytes_sent += q == me ? 0 : hs[2 * q];
  r->bytes_recv += ro;
  r->last_set = s;
  r->acking.push_back(s);
  return RMQ_OK;
}

}  // namespace

int repl_attach(rmq_engine* e, Transport* t) {
  if (e->repl) return RMQ_EINVAL;
  if (t->world() > kMaxWorld || t->rank() != e->cfg.rank || t->world() <= e->cfg.rank) return RMQ_EINVAL;
  // groups must close by count alone so every rank forms the same rounds
  if (e->group_max * e->max_tiles > kMaxTiles) return RMQ_EINVAL;
  Replication* r = new (std::nothrow) Replication();
  if (!r) return RMQ_ENOMEM;
  r->xport = t;
  r->world = t->world();
  r->rank = t->rank();
  e->repl = r;
  HIP_TRY(hipStreamCreateWithFlags(&r->xchg_s, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&r->ev_notice, hipEventDisableTiming));
  for (XchgSet& x : r->sets) {
    HIP_TRY(hipEventCreateWithFlags(&x.ev_s2, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&x.ev_s3, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&x.ev_sz, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&x.ev_x, hipEventDisableTiming));
    int rc = dalloc(&x.count, 1);
    if (rc) return rc;
    HIP_TRY(hipHostMalloc((void**)&x.h_sizes, 4ull * kMaxWorld * 8, 0));
  }
  int rc = dalloc(&r->d_counters, 7);
  if (!rc) rc = dalloc(&r->d_lastg, e->cfg.num_partitions);
  if (!rc && !e->st.csnap) rc = dalloc(&e->st.csnap, 2ull * e->cfg.num_partitions);
  if (rc) return rc;
  {
    // both slots start at the current commits (the first plan reads the slot of the launch before)
    for (uint32_t k = 0; k < 2; ++k)
      HIP_TRY(hipMemcpy(e->st.csnap + (size_t)k * e->cfg.num_partitions, e->st.commit,
                        e->cfg.num_partitions * 8ull, hipMemcpyDeviceToDevice));
  }
  return repl_set_lists(e);
}

void repl_free(rmq_engine* e) {
  Replication* r = e->repl;
  if (!r) return;
  if (r->xchg_s) hipStreamSynchronize(r->xchg_s);
  free_set_buffers(r);
  for (XchgSet& x : r->sets) {
    hipEvent_t evs[] = {x.ev_s2, x.ev_s3, x.ev_sz, x.ev_x};
    for (hipEvent_t v : evs)
      if (v) hipEventDestroy(v);
    if (x.count) hipFree(x.count);
    if (x.h_sizes) hipHostFree(x.h_sizes);
  }
  void* bufs[] = {r->d_xo_p, r->d_xo_slot, r->d_xo_start, r->d_keysum, r->d_keysum_in, r->d_outidx, r->d_xi_p, r->d_xi_slot,
                  r->d_xi_start, r->d_bad, r->d_acc, r->d_base, r->d_cdesc, r->d_items, r->d_nitems, r->d_counters,
                  r->d_xnext, r->d_xreq, r->d_xcu, r->d_xdec, r->d_xtot, r->d_dflag, r->d_lastg,
                  r->d_nout, r->d_nin, r->d_eackv};
  for (void* p : bufs)
    if (p) hipFree(p);
  e->st.outidx = nullptr;
  e->st.eackv = nullptr;
  if (r->ev_notice) hipEventDestroy(r->ev_notice);
  if (r->xchg_s) hipStreamDestroy(r->xchg_s);
  delete r->xport;
  delete r;
  e->repl = nullptr;
}

// Out / in lists from the placement, the collective consistency check, and the round buffers.
// Called with the engine drained, by every rank.
int repl_set_lists(rmq_engine* e) {
  Replication* r = e->repl;
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor, W = r->world, me = r->rank;
  std::vector<std::vector<Entry>> out(W), in(W);
  int bad = RMQ_OK;
  for (uint32_t p = 0; p < P; ++p) {
    const uint32_t* rk = &e->ranks[(size_t)p * RF];
    const uint32_t lead = rk[e->leader_slot[p]];
    uint32_t remote = 0;
    for (uint32_t s = 0; s < RF; ++s) {
      if (rk[s] >= W) bad = RMQ_EINVAL;
      else if (lead == me && rk[s] != me) {
        out[rk[s]].push_back({e->key[p], s, p});
        ++remote;
      } else if (lead != me && rk[s] == me && lead < W) {
        in[lead].push_back({e->key[p], s, p});
      }
    }
    if (remote > kMaxRemote) bad = RMQ_EINVAL;
  }
  r->xo_p.clear();
  r->xo_slot.clear();
  r->xi_p.clear();
  r->xi_slot.clear();
  r->xo_start.assign(W + 1, 0);
  r->xi_start.assign(W + 1, 0);
  r->keysum.assign(W, 0);
  std::vector<uint64_t> keysum_in(W, 0);
  std::vector<uint32_t> outidx((size_t)P * RF, ~0u);
  for (uint32_t q = 0; q < W; ++q) {
    std::sort(out[q].begin(), out[q].end());
    std::sort(in[q].begin(), in[q].end());
    r->xo_start[q] = (uint32_t)r->xo_p.size();
    for (const Entry& x : out[q]) {
      outidx[(size_t)x.p * RF + x.slot] = (uint32_t)r->xo_p.size();
      r->xo_p.push_back(x.p);
      r->xo_slot.push_back(x.slot);
      r->keysum[q] += entry_hash(x.key, x.slot);
    }
    r->xi_start[q] = (uint32_t)r->xi_p.size();
    for (const Entry& x : in[q]) {
      r->xi_p.push_back(x.p);
      r->xi_slot.push_back(x.slot);
      keysum_in[q] += entry_hash(x.key, x.slot);
    }
  }
  r->xo_start[W] = (uint32_t)r->xo_p.size();
  r->xi_start[W] = (uint32_t)r->xi_p.size();
  // handshake: what I send to q must be what q expects from me, and every rank learns whether all
  // pairs agree (two exchanges, so no rank starts rounds that another refuses)
  {
    std::vector<uint64_t> h(8ull * W, 0);  // [q]: send {entries, keysum}; [W + q]: recv; [2W..] verdicts
    for (uint32_t q = 0; q < W; ++q) {
      h[2 * q] = r->xo_start[q + 1] - r->xo_start[q];
      h[2 * q + 1] = r->keysum[q];
    }
    uint64_t* d = nullptr;
    int rc = dalloc(&d, h.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    void* sb[kMaxWorld];
    void* rb[kMaxWorld];
    uint64_t n[kMaxWorld];
    for (uint32_t q = 0; q < W; ++q) {
      sb[q] = d + 2 * q;
      rb[q] = d + 2 * W + 2 * q;
      n[q] = q == me ? 0 : 16;
    }
    rc = r->xport->exchange(sb, n, rb, n, r->xchg_s);
    if (!rc) rc = hip_fail(hipStreamSynchronize(r->xchg_s));
    if (!rc) rc = hip_fail(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    uint64_t verdict = bad ? 1 : 0;
    for (uint32_t q = 0; q < W && !rc; ++q)
      if (q != me && (h[2 * W + 2 * q] != r->xi_start[q + 1] - r->xi_start[q] || h[2 * W + 2 * q + 1] != keysum_in[q]))
        verdict = 1;
    for (uint32_t q = 0; q < W; ++q) h[4 * W + q] = verdict;
    if (!rc) rc = hip_fail(hipMemcpy(d + 4 * W, h.data() + 4 * W, 8ull * W, hipMemcpyHostToDevice));
    for (uint32_t q = 0; q < W; ++q) {
      sb[q] = d + 4 * W + q;
      rb[q] = d + 5 * W + q;
      n[q] = q == me ? 0 : 8;
    }
    if (!rc) rc = r->xport->exchange(sb, n, rb, n, r->xchg_s);
    if (!rc) rc = hip_fail(hipStreamSynchronize(r->xchg_s));
    if (!rc) rc = hip_fail(hipMemcpy(h.data() + 5 * W, d + 5 * W, 8ull * W, hipMemcpyDeviceToHost));
    hipFree(d);
    if (rc) return rc;
    for (uint32_t q = 0; q < W; ++q) verdict |= q != me ? h[5 * W + q] : 0;
    if (verdict) {
      std::fprintf(stderr, "ripplemq: replica placement differs between ranks (rank %u)\n", me);
      return RMQ_EINVAL;
    }
  }
  int rc = upload(&r->d_xo_p, r->xo_p);
  if (!rc) rc = upload(&r->d_xo_slot, r->xo_slot);
  if (!rc) rc = upload(&r->d_xo_start, r->xo_start);
  if (!rc) rc = upload(&r->d_keysum, r->keysum);
  if (!rc) rc = upload(&r->d_keysum_in, keysum_in);
  if (!rc) rc = upload(&r->d_outidx, outidx);
  if (!rc) rc = upload(&r->d_xi_p, r->xi_p);
  if (!rc) rc = upload(&r->d_xi_slot, r->xi_slot);
  if (!rc) rc = upload(&r->d_xi_start, r->xi_start);
  const size_t n_in = std::max<size_t>(1, r->xi_p.size()), n_out = std::max<size_t>(1, r->xo_p.size());
  if (!rc) rc = upload(&r->d_bad, std::vector<uint32_t>(n_in, 0u));
  if (!rc) rc = upload(&r->d_acc, std::vector<uint32_t>(n_in, 0u));
  if (!rc) rc = upload(&r->d_base, std::vector<uint64_t>(2 * n_in, 0ull));
  if (!rc) rc = upload(&r->d_cdesc, std::vector<uint64_t>(4 * n_in, 0ull));
  if (!rc) rc = upload(&r->d_xnext, std::vector<uint64_t>(2 * n_out, 0ull));
  if (!rc) rc = upload(&r->d_xreq, std::vector<uint64_t>(4 * n_out, 0ull));
  if (!rc) rc = upload(&r->d_xcu, std::vector<uint64_t>(n_out, 0ull));
  if (!rc) rc = upload(&r->d_dflag, std::vector<uint32_t>(W, 0u));
  if (!rc) rc = upload(&r->d_nout, std::vector<uint64_t>(2 * n_out, 0ull));
  if (!rc) rc = upload(&r->d_nin, std::vector<uint64_t>(2 * n_in, 0ull));
  if (r->d_xdec) hipFree(r->d_xdec);
  if (r->d_xtot) hipFree(r->d_xtot);
  r->d_xdec = nullptr;
  r->d_xtot = nullptr;
  if (!rc) rc = dalloc(&r->d_xdec, n_out);
  if (!rc) rc = dalloc(&r->d_xtot, n_out);
  if (rc) return rc;
  // round buffers (FORMAT.md §9 bounds): a record is at most 31 + L bytes in the log, sent once per
  // remote slot, plus an 8-byte table slot; the catch-up reserve of a destination is one such
  // round bound (ro_catchup_reserve in the oracle); per region a header, a directory, table padding
  // and the consumer-offset rows
  const uint64_t G = e->group_max, NR = e->cfg.max_batch_records, MB = e->cfg.max_batch_bytes;
  const uint64_t rec = G * (39ull * NR + MB), C = e->cfg.max_consumers;
  uint32_t max_remote = 0;
  for (uint32_t p = 0; p < P; ++p) {
    uint32_t k = 0;
    for (uint32_t s = 0; s < RF; ++s) k += outidx[(size_t)p * RF + s] != ~0u;
    max_remote = std::max(max_remote, k);
  }
  const uint64_t per_entry = kDirEntry + 16 + 8 * C;
  r->reserve = rec;
  r->dcap = ((uint64_t)max_remote * rec + r->reserve + kRegionHdr + 16 + per_entry * n_out + 255) & ~255ull;
  r->out_cap = (uint64_t)W * r->dcap;
  r->in_cap = (uint64_t)(W - 1) * ((uint64_t)(RF - 1) * rec + r->reserve + kRegionHdr + 32) + per_entry * n_in;
  r->items_cap = r->in_cap / kCopyChunk + W + n_in;
  if (r->d_items) hipFree(r->d_items);
  if (r->d_nitems) hipFree(r->d_nitems);
  r->d_items = nullptr;
  r->d_nitems = nullptr;
  rc = dalloc(&r->d_items, 2 * r->items_cap);
  if (!rc) rc = dalloc(&r->d_nitems, 2 * (1 + kMaxWorld));  // both halves zero
  r->nitems_par = 0;
  if (rc) return rc;
  free_set_buffers(r);
  for (XchgSet& x : r->sets) {
    rc = dalloc(&x.outbox, r->out_cap);
    if (!rc) rc = dalloc(&x.inbox, r->in_cap);
    if (!rc) rc = dalloc(&x.xe, n_out);
    if (!rc) rc = dalloc(&x.xc, n_out);
    if (!rc) rc = dalloc(&x.xc_n, 2);
    if (!rc) rc = dalloc(&x.sizes, 4ull * W);
    if (!rc) rc = dalloc(&x.ackout, 2 * n_in);
    if (!rc) rc = dalloc(&x.ackin, 2 * n_out);
    if (!rc) rc = dalloc(&x.rowv, n_out);
    if (rc) return rc;
  }
  // consumer-offset rows: the followers acknowledge them afresh under the new lists (the rows of
  // every led partition with committed offsets go out with the next round) and every partition's
  // row quorum is recomputed (pending offset tickets wait for those rounds' acks)
  if (r->d_eackv) hipFree(r->d_eackv);
  r->d_eackv = nullptr;
  rc = dalloc(&r->d_eackv, n_out);
  if (rc) return rc;
  e->st.outidx = r->d_outidx;
  e->st.eackv = r->d_eackv;
  {
    std::vector<uint32_t> dirty(P, 0u);
    bool any = false;
    for (uint32_t p = 0; p < P; ++p)
      if (e->is_leader[p] && e->cver[p]) dirty[p] = 1u, any = true;
    if (any) {
      std::vector<uint32_t> cur(P);
      HIP_TRY(hipMemcpy(cur.data(), e->st.cdirty, P * 4ull, hipMemcpyDeviceToHost));
      for (uint32_t p = 0; p < P; ++p) dirty[p] |= cur[p];
      HIP_TRY(hipMemcpy(e->st.cdirty, dirty.data(), P * 4ull, hipMemcpyHostToDevice));
    }
  }
  launch_row_quorum_all(e->st, e->main_s);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->main_s));
  return reset_catchup(e);
}

void repl_pipe_args(rmq_engine* e, PipeArgs& a, const GroupFlight* s2, const GroupFlight* s3) {
  Replication* r = e->repl;
  if (!r) return;
  a.lastg = r->d_lastg;               // kept by every launch that applies a group
  // every rank numbers every round (the follower side stamps its ingest with it), also one that
  // leads nothing with a remote replica
  if (s2) r->sets[s2->set].round = r->planned++;
  if (r->xo_p.empty()) return;        // nothing led here has a remote replica
  a.outidx = r->d_outidx;
  if (s2) {
    XchgSet& x = r->sets[s2->set];
    a.xp2.xo_p = r->d_xo_p;
    a.xp2.xo_slot = r->d_xo_slot;
    a.xp2.xo_start = r->d_xo_start;
    a.xp2.keysum = r->d_keysum;
    a.xp2.world = r->world;
    a.xp2.rank = r->rank;
    a.xp2.n_out = (uint32_t)r->xo_p.size();
    a.xp2.C = e->cfg.max_consumers;
    a.xp2.count = x.count;
    a.xp2.xe = x.xe;
    a.xp2.outbox = x.outbox;
    a.xp2.sizes = x.sizes;
    a.xp2.round = x.round;
    a.xp2.reserve = r->reserve;
    a.xp2.xnext = r->d_xnext;
    a.xp2.xreq = r->d_xreq;
    a.xp2.xcu = r->d_xcu;
    a.xp2.xdec = r->d_xdec;
    a.xp2.xtot = r->d_xtot;
    a.xp2.dflag = r->d_dflag;
  // the commit the round carries: the slot of the launch before this one (launch_seq not yet advanced)
  a.xp2.csnap = e->st.csnap + (size_t)(e->launch_seq & 1ull) * e->cfg.num_partitions;
    a.xp2.dirty = e->st.cdirty;
    a.xp2.rowv = x.rowv;
    a.xp2.xc = x.xc;
    a.xp2.xc_n = x.xc_n;
    a.xp2.counters = r->d_counters + 4;
    a.xp2.dcap = r->dcap;
  }
  if (s3) {
    XchgSet& x = r->sets[s3->set];
    a.xe3 = x.xe;
    a.outbox3 = x.outbox;
    a.xc3 = x.xc;
    a.xc3_n = x.xc_n;
    a.wgc = 2u * e->cu_count / (kPipeThreadsXR / 64u);  // two catch-up waves per CU (most rounds: none)
  }
}

// Before issuing launch launch_seq + 1: the acks of the group applied three launches earlier.
int repl_before_launch(rmq_engine* e, PipeArgs& a) {
  Replication* r = e->repl;
  if (!r || r->acking.empty()) return RMQ_OK;
  const uint32_t s = r->acking.front();
  if (r->sets[s].applied_launch + 3 > e->launch_seq + 1) return RMQ_OK;
  HIP_TRY(hipStreamWaitEvent(e->main_s, r->sets[s].ev_x, 0));
  if (!r->xo_p.empty()) {
    a.ackin = r->sets[s].ackin;
    a.ackrowv = r->sets[s].rowv;
    a.acks_round = r->sets[s].round;
    if (a.xp2.n_out) {  // the plan of this launch turns refusals into catch-up verdicts itself
      a.xp2.ackin = a.ackin;
      a.xp2.acks_round = a.acks_round;
    } else {  // no plan reads these acks: the partition threads keep the requests
      a.xreq = r->d_xreq;
    }
  }
  r->acking.pop_front();
  return RMQ_OK;
}

// After launch launch_seq: post the size swap of its stage-2 group and the rounds of the groups
// applied by earlier launches.
int repl_after_launch(rmq_engine* e, const GroupFlight* s2, const GroupFlight* s3) {
  Replication* r = e->repl;
  if (!r) return RMQ_OK;
  // the rounds of groups applied by earlier launches first: on the exchange stream they then wait
  // only for their own apply launch, not behind the size swap of this launch's group (which waits
  // for this whole launch)
  while (!r->sized.empty() && r->sets[r->sized.front()].applied_launch < e->launch_seq) {
    int rc = post_round(e, r->sized.front());
    if (rc) return rc;
    r->sized.pop_front();
  }
  if (s2) {
    HIP_TRY(hipEventRecord(r->sets[s2->set].ev_s2, e->main_s));
    const bool drop = r->drop_n && s2->b[0].ticket >= r->drop_from;
    if (drop) r->drop_n--;
    uint32_t lost = 0;
    for (uint32_t q = 0; q < r->world; ++q)
      if (r->iso_n[q] && s2->b[0].ticket >= r->iso_from[q]) {
        lost |= 1u << q;
        r->iso_n[q]--;
      }
    int rc = post_sizes(e, s2->set, drop, lost);
    if (rc) return rc;
  }
  if (s3) {
    XchgSet& x = r->sets[s3->set];
    HIP_TRY(hipEventRecord(x.ev_s3, e->main_s));
    x.applied_launch = e->launch_seq;
    r->sized.push_back(s3->set);
  }
  return RMQ_OK;
}

// Commit notices (FORMAT.md §9 v4, the heartbeat of a drain): every leader sends each follower its
// {commit, term} per entry of their list after the drain's acks are in; the followers learn it.
// Collective like the rounds before it (every rank drains the same rounds).
int post_notices(rmq_engine* e) {
  Replication* r = e->repl;
  const uint32_t W = r->world, me = r->rank;
  NoticeArgs a{};
  a.st = e->st;
  a.sets[0] = e->sets[0];
  a.sets[1] = e->sets[1];
  a.xo_p = r->d_xo_p;
  a.out = r->d_nout;
  a.xi_p = r->d_xi_p;
  a.in = r->d_nin;
  a.n_out = (uint32_t)r->xo_p.size();
  a.n_in = (uint32_t)r->xi_p.size();
  a.stamp = r->stamp;
  launch_notice_fill(a, e->main_s);  // after the acks applied on the pipeline stream
  HIP_TRY(hipGetLastError());
  for (uint32_t q = 0; q < W; ++q)  // rmq_fault_cut: these notices are lost (term 0: ignored)
    if (((r->cut_notice >> q) & 1u) && r->xo_start[q + 1] > r->xo_start[q])
      HIP_TRY(hipMemsetAsync(r->d_nout + 2ull * r->xo_start[q], 0, 16ull * (r->xo_start[q + 1] - r->xo_start[q]), e->main_s));
  r->cut_notice = 0;
  HIP_TRY(hipEventRecord(r->ev_notice, e->main_s));
  HIP_TRY(hipStreamWaitEvent(r->xchg_s, r->ev_notice, 0));
  void* sb[kMaxWorld];
  void* rb[kMaxWorld];
  uint64_t sn[kMaxWorld], rn[kMaxWorld];
  for (uint32_t q = 0; q < W; ++q) {
    sn[q] = q == me ? 0 : 16ull * (r->xo_start[q + 1] - r->xo_start[q]);
    rn[q] = q == me ? 0 : 16ull * (r->xi_start[q + 1] - r->xi_start[q]);
    sb[q] = r->d_nout + 2ull * r->xo_start[q];
    rb[q] = r->d_nin + 2ull * r->xi_start[q];
  }
  int rc = r->xport->exchange(sb, sn, rb, rn, r->xchg_s);
  if (rc) return rc;
  launch_notice_apply(a, r->xchg_s);
  HIP_TRY(hipGetLastError());
  // the pipeline stream sees the followers' new commits before anything issued after the drain
  HIP_TRY(hipEventRecord(r->ev_notice, r->xchg_s));
  HIP_TRY(hipStreamWaitEvent(e->main_s, r->ev_notice, 0));
  return RMQ_OK;
}

// After the pipeline is flushed: post the remaining rounds, apply their acks, and (if any round
// was in flight) exchange the commit notices.
int repl_drain(rmq_engine* e) {
  Replication* r = e->repl;
  if (!r) return RMQ_OK;
  const bool rounds = !r->sized.empty() || !r->acking.empty();
  while (!r->sized.empty()) {
    int rc = post_round(e, r->sized.front());
    if (rc) return rc;
    r->sized.pop_front();
  }
  while (!r->acking.empty()) {
    XchgSet& x = r->sets[r->acking.front()];
    HIP_TRY(hipStreamWaitEvent(e->main_s, x.ev_x, 0));
    if (!r->xo_p.empty()) {
      AckApplyArgs a{};
      a.st = e->st;
      a.outidx = r->d_outidx;
      a.ackin = x.ackin;
      a.rowv = x.rowv;
      a.xreq = r->d_xreq;
      a.acks_round = x.round;
      launch_ack_apply(a, e->main_s);
      HIP_TRY(hipGetLastError());
    }
    r->acking.pop_front();
  }
  if (rounds) {
    int rc = post_notices(e);
    if (rc) return rc;
  }
  HIP_TRY(hipStreamSynchronize(r->xchg_s));
  return RMQ_OK;
}

}  // namespace rmq
