// engine.cpp — host side of the C-ABI (include/ripplemq_engine.h).
//
// Owns all device memory of one engine (one HIP device): per-(replica, partition) ring segments,
// the sparse offset index, per-partition Raft state and consumer offsets. Appended batches are
// collected into groups of up to cfg.pipeline_depth; each full group issues exactly ONE kernel
// launch (pipeline.hip) that ranks it (stage 1), scans the group before (stage 2), applies the one
// before that (stage 3) and evaluates the retention of the one before that (stage 4). A batch is
// therefore applied two launches after its group's own; rmq_poll_commit / rmq_sync / any control
// call close the forming group and flush the pipeline with up to three more launches that carry
// only the later stages. No host synchronisation and no HIP events sit on the
// append path: launch k reports launch k-1 complete through a host-visible word, and the tail is
// read with hipStreamQuery. Control-plane calls (leadership, replicas, acks, consumer offsets,
// fetch) flush and drain first and run synchronously: they are rare next to the append stream.
#include <chrono>

#include "engine_internal.hpp"

using namespace rmq;

namespace rmq {

uint32_t host_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int k = 31; k >= 0; --k) {
    if ((a >> k) & 1u) p ^= b;
    b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
  }
  return p;
}

// Inverse of a in GF(2)[x] mod P (reflected), by Gaussian elimination of y -> y * a.
uint32_t host_inverse(uint32_t a) {
  uint32_t col[32];
  for (int k = 0; k < 32; ++k) col[k] = host_mulmod(1u << k, a);  // image of basis vector bit k
  // solve sum_k y_k col[k] = one (x^0 = 0x80000000): rows = output bits
  uint32_t rows[32];  // rows[b]: bit k = bit b of col[k]; bit 32 handled separately
  uint32_t rhs = 0;
  for (int bb = 0; bb < 32; ++bb) {
    rows[bb] = 0;
    for (int k = 0; k < 32; ++k) rows[bb] |= ((col[k] >> bb) & 1u) << k;
    rhs |= ((0x80000000u >> bb) & 1u) << bb;
  }
  int r = 0;
  int piv[32];
  for (int k = 0; k < 32 && r < 32; ++k) {
    int sel = -1;
    for (int bb = r; bb < 32; ++bb)
      if ((rows[bb] >> k) & 1u) { sel = bb; break; }
    if (sel < 0) continue;
    std::swap(rows[sel], rows[r]);
    const uint32_t t = (rhs >> sel) & 1u, u = (rhs >> r) & 1u;
    rhs = (rhs & ~((1u << sel) | (1u << r))) | (u << sel) | (t << r);
    for (int bb = 0; bb < 32; ++bb)
      if (bb != r && ((rows[bb] >> k) & 1u)) {
        rows[bb] ^= rows[r];
        rhs ^= ((rhs >> r) & 1u) << bb;
      }
    piv[r] = k;
    ++r;
  }
  uint32_t y = 0;
  for (int q = 0; q < r; ++q)
    if ((rhs >> q) & 1u) y |= 1u << piv[q];
  return y;
}

void build_crc_consts(CrcConsts* c) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t x = b;
    for (int k = 0; k < 8; ++k) x = (x >> 1) ^ (kCrcPoly & (0u - (x & 1u)));
    c->table[0][b] = x;
  }
  for (uint32_t t = 1; t < 8; ++t)
    for (uint32_t b = 0; b < 256; ++b)
      c->table[t][b] = (c->table[t - 1][b] >> 8) ^ c->table[0][c->table[t - 1][b] & 0xFF];
  uint32_t x2n[40];
  x2n[0] = 0x40000000u;  // x^1 in the reflected representation
  for (int k = 1; k < 40; ++k) x2n[k] = host_mulmod(x2n[k - 1], x2n[k - 1]);
  for (uint32_t k = 0; k < 2; ++k)  // shift past 16 << k zero bytes = multiply by x^(2^(7+k))
    for (uint32_t i = 0; i < 4; ++i)
      for (uint32_t b = 0; b < 256; ++b) c->zshift[k][i][b] = host_mulmod(b << (8 * i), x2n[7 + k]);
  for (uint32_t i = 0; i < 4; ++i)  // 1024 bytes = 2^13 bits
    for (uint32_t b = 0; b < 256; ++b) c->zshift1k[i][b] = host_mulmod(b << (8 * i), x2n[13]);
  uint32_t x128e = 0x80000000u;  // x^(128 e), e = 0..63
  for (uint32_t e = 0; e < 64; ++e) {
    c->sh16[e] = x128e;
    x128e = host_mulmod(x128e, x2n[7]);
  }
  uint32_t x8n = 0x80000000u;  // x^(8n), n = 0..15
  for (uint32_t n = 0; n < 16; ++n) {
    c->inv_pad[n] = n ? host_inverse(x8n) : 0x80000000u;
    c->inv_pad16[n] = host_mulmod(c->inv_pad[n], x2n[4]);
    x8n = host_mulmod(x8n, x2n[3]);
  }
  // nibble tables of the sixteen LDS tables of stage 3 (table[0..7], then zshift[0][0..3],
  // zshift[1][0..3], as laid out in LDS): each is GF(2)-linear in its byte
  for (uint32_t q = 0; q < 16; ++q) {
    const uint32_t* t = q < 8 ? c->table[q] : c->zshift[(q - 8) / 4][(q - 8) % 4];
    for (uint32_t n = 0; n < 16; ++n) {
      c->nib[q][n] = t[n];
      c->nib[q][16 + n] = t[n << 4];
    }
  }
}

bool is_pow2(uint64_t v) { return v && !(v & (v - 1)); }

uint32_t ilog2(uint64_t v) {
  uint32_t r = 0;
  while ((1ull << r) < v) ++r;
  return r;
}

// A fault of earlier work on the pipeline stream (kernels report nothing else: every rejection is
// a per-record status). Asynchronous errors are sticky, so a query sees them without a copy.
int check_err(rmq_engine* e) {
  const hipError_t q = hipStreamQuery(e->main_s);
  return q == hipSuccess || q == hipErrorNotReady ? RMQ_OK : hip_fail(q);
}

int fetch_flush(rmq_engine* e);
// The engine lock of every call: held-back asynchronous fetches go to the pipeline stream first, so
// whatever the call issues is ordered after them (their contract); a launch error stays sticky on the
// stream and surfaces at the next check.
struct EngineLock {
  std::lock_guard<std::mutex> g;
  explicit EngineLock(rmq_engine* e) : g(e->mu) {
    if (!e->fpend.empty() && hipSetDevice(e->device) == hipSuccess) (void)fetch_flush(e);
  }
};

// Wait for everything issued on stream s. A blocking hipStreamSynchronize returns ~10 us after the
// last kernel ends (interrupt wake-up); a sync sits on the producer's path (rmq_sync, a poll that
// needs commit indices), so poll the stream for up to 20 ms first, then block.
// Wait for an event the same way: a blocking hipEventSynchronize now and then woke milliseconds
// late (8 ms stalls in one synchronous fetch of ten, round 4), so spin on queries first.
int event_wait(hipEvent_t ev) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return RMQ_OK;
    if (q != hipErrorNotReady) return hip_fail(q);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
  }
  HIP_TRY(hipEventSynchronize(ev));
  return RMQ_OK;
}

int stream_wait(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return RMQ_OK;
    if (q != hipErrorNotReady) return hip_fail(q);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
  }
  HIP_TRY(hipStreamSynchronize(s));
  return RMQ_OK;
}

hipEvent_t pool_event(rmq_engine* e) {
  if (!e->ev_pool.empty()) {
    hipEvent_t ev = e->ev_pool.back();
    e->ev_pool.pop_back();
    return ev;
  }
  hipEvent_t ev = nullptr;
  if (hipEventCreate(&ev) != hipSuccess) return nullptr;
  return ev;
}

PipeGroup make_group(const rmq_engine* e, const GroupFlight& g) {
  PipeGroup G{};
  uint32_t tile = 0, task = 0;
  for (uint32_t j = 0; j < kMaxGroup; ++j) {
    G.tile0[j] = tile;
    G.task0[j] = task;
    if (j < g.nb) {
      const InFlight& f = g.b[j];
      G.b[j] = f.b;
      G.stats[j] = e->d_stats + (size_t)(f.ticket % kStatsRing) * e->max_tasks;
      tile += f.b.tiles;
      task += (f.b.n + kTaskRecs - 1) / kTaskRecs;
    }
  }
  G.tile0[kMaxGroup] = tile;
  G.task0[kMaxGroup] = task;
  G.nb = g.nb;
  G.tiles = tile;
  return G;
}

// One pipeline launch: stage 1 on group s1, 2 on s2, 3 on s3, 4 on s4 (each may be null).
int launch_stages(rmq_engine* e, const GroupFlight* s1, const GroupFlight* s2, const GroupFlight* s3,
                  const GroupFlight* s4) {
  PipeArgs a{};
  const uint32_t P = e->cfg.num_partitions;
  const StateSet cur = e->sets[e->applied & 1u], nxt = e->sets[(e->applied + 1) & 1u];
  a.st = e->st;
  a.cur = cur;
  a.nxt = nxt;
  a.key_passes = e->key_passes;
  a.key_bits = e->key_bits;
  a.rank_mode = e->rank_mode;
  a.steal = e->steal;
  a.prio = e->prio;
  a.gt = e->max_group_tiles;
  a.crc = e->d_crc;
  a.done_word = e->done_dev;
  a.ret_late = e->done_dev + 1;
  a.rlate = e->d_rlate;
  a.debug = e->debug;
  if (s1) {
    a.g1 = make_group(e, *s1);
    a.s1 = e->scratch[s1->set];
    if (e->set_reset & (1u << s1->set)) {  // a drain skipped the stage 4 that resets the set's list and sums
      HIP_TRY(hipMemsetAsync(a.s1.bacc, 0, kMaxGroup * 2 * sizeof(uint64_t), e->main_s));
      HIP_TRY(hipMemsetAsync(a.s1.nbig, 0, 4 * sizeof(uint32_t), e->main_s));
      e->set_reset &= ~(1u << s1->set);
    }
    a.wg1 = e->s1_wgs ? std::min<uint32_t>(s1->tiles, e->s1_wgs) : s1->tiles;
    a.s1_xcd = e->s1_xcd;
  }
  if (s2) {
    a.g2 = make_group(e, *s2);
    a.s2 = e->scratch[s2->set];
  }
  repl_pipe_args(e, a, s2, s3);
  // the kernel with a transport (outboxes) runs 512-thread workgroups, the single-GPU one 256
  const uint32_t PT = a.outidx ? kPipeThreadsXR : kPipeThreads;
  if (s2) {
    const uint32_t groups = (P + kScanCols - 1) / kScanCols;
    a.wg2 = std::max<uint32_t>(1u, std::min<uint32_t>((groups * kScanLanes + PT - 1) / PT, 2u * e->cu_count));
    if (e->s2_wgs) a.wg2 = std::min(a.wg2, e->s2_wgs);
  }
  {
    int rc = repl_before_launch(e, a);  // followers' acks of the group applied three launches ago
    if (rc) return rc;
  }
  // partition threads: the group applied, retention, acks; with a transport in every launch (they
  // also record each led partition's commit at the launch's end, which the next plan carries)
  if (s3 || s4 || a.ackin || e->repl) a.wgp = (P + PT - 1) / PT;
  if (s4) {
    a.g4 = make_group(e, *s4);
    a.s4 = e->scratch[s4->set];
  }
  if (s3) {
    a.g3 = make_group(e, *s3);
    a.s3 = e->scratch[s3->set];
    const uint32_t wpb = PT / 64;
    const uint32_t want = std::max<uint32_t>(1u, (s3->tasks + wpb - 1) / wpb);
    // default: one wave per task (the workgroups past the resident slots start as stage-1/2
    // workgroups retire); RMQ_WG3_ALL=0 fills only the slots next to the other roles (resident
    // workgroups per CU from the kernel's launch bounds) and the task waves loop over the rest
    const bool split = e->split && !a.outidx;  // (the apply launch holds no stage-1/2 workgroups)
    const uint32_t slots = pipeline_wgs_per_cu(PT) * e->cu_count, busy = (split ? 0u : a.wg1 + a.wg2) + a.wgp;
    const uint32_t room = slots > busy + e->cu_count ? slots - busy : e->cu_count;
    a.wg3 = e->wg3_all ? want : std::min<uint32_t>(want, room);
    if (e->s3_pair && !a.outidx) {  // two tasks per wave: every task has its place (no loop)
      a.s3_pair = 1;
      a.wg3 = std::max<uint32_t>(1u, (s3->tasks + 2 * wpb - 1) / (2 * wpb));
    }
    if (e->s3_roles && !a.outidx && !e->split) {  // loader / storer waves: a run of tasks per workgroup
      a.s3_roles = 1;
      a.s3_pair = 0;
      a.wg3 = std::max<uint32_t>(1u, std::min<uint32_t>(s3->tasks, e->s3_roles * e->cu_count));
    }
    a.wgb = e->big_wgs ? e->big_wgs : 32u * e->cu_count / (PT / 64u);  // 32 large-record waves per CU
    // dispatch order: s3_lead stage-3 workgroups, then ranking, scans and partition threads, then
    // the rest of stage 3. Round 6 default: all of stage 3 last, so the ranking and scan chains
    // start with the launch instead of in its tail, when the first stage-3 workgroups retire
    // (42.5-43.3 vs 43.7-44.0 us per launch, 20-step 34.4-34.7 vs 35.6-35.8, profiles/r06_dispatch_order.txt;
    // round 2's +2.8 % for stage 3 first no longer holds); RMQ_S3_FIRST=1 all first, RMQ_S3_LEAD=<n> n first
    a.s3_lead = e->s3_lead ? std::min<uint32_t>(a.wg3, e->s3_lead) : e->s3_first ? a.wg3 : 0u;
    // (with every stage-3 workgroup first or every one last: one contiguous range of blocks)
    a.s3_xcd = e->s3_xcd && (a.s3_lead == a.wg3 || a.s3_lead == 0u) && !a.s3_pair ? 1u : 0u;
    a.s3_stage = e->s3_stage;
  }
  a.launch_seq = ++e->launch_seq;
  e->st.csnap_slot = (uint32_t)(a.launch_seq & 1ull);  // control kernels after this launch write its slot
  if (e->d_stamps && a.launch_seq == e->stamps_at) {
    a.stamps = e->d_stamps;
    e->stamps_wg[0] = a.wg1;
    e->stamps_wg[1] = a.wg2;
    e->stamps_wg[2] = a.wgp;
    e->stamps_wg[3] = a.wg3;
    e->stamps_wg[4] = a.s3_lead;
  }
  hipEvent_t ev_start = nullptr;
  if (e->profile && !e->prof_ended) {
    if (!e->prof_started) {
      ev_start = e->prof_t0;  // recorded by the launch itself (no separate hipEventRecord call)
      e->prof_started = true;
    }
    e->prof_launches++;
    if (s3) e->prof_batches += s3->nb;
  }
  if (e->trace)  // RMQ_TRACE: the roles of every launch (diagnostics only)
    std::fprintf(stderr, "rmq launch %llu: s1 %u batches %u wgs | s2 %u batches %u wgs | parts %u wgs | s3 %u batches %u wgs + %u big | s4 %u batches\n",
                 (unsigned long long)a.launch_seq, a.g1.nb, a.wg1, a.g2.nb, a.wg2, a.wgp, a.g3.nb, a.wg3, a.wgb, a.g4.nb);
  if (e->split && !a.outidx) {
    // two launches side by side: ranking on rank_s, apply on main_s (rmq_engine::split)
    PipeArgs ra = a, aa = a;
    ra.wgp = ra.wg3 = ra.wgb = ra.wgc = ra.s3_lead = 0;
    ra.done_word = nullptr;
    aa.wg1 = aa.wg2 = 0;
    if (ra.wg1 + ra.wg2) {
      HIP_TRY(hipEventRecord(e->ev_pre_rank, e->main_s));  // apply L - 1 and the control work before it
      HIP_TRY(hipStreamWaitEvent(e->rank_s, e->ev_pre_rank, 0));
      launch_pipeline(ra, e->rank_s, ev_start);
      HIP_TRY(hipGetLastError());
      ev_start = nullptr;
      if (e->split == 2) {  // (timing experiment: the two launches one after the other)
        HIP_TRY(hipEventRecord(e->ev_rank[a.launch_seq & 1u], e->rank_s));
        e->rank_seq = a.launch_seq;
      }
    }
    if (aa.wgp + aa.wg3 + aa.wgb + aa.wgc) {
      if (e->rank_seq) {  // the scans of the group it applies (the last rank launch before this one)
        HIP_TRY(hipStreamWaitEvent(e->main_s, e->ev_rank[e->rank_seq & 1u], 0));
        e->rank_seq = 0;
      }
      launch_pipeline(aa, e->main_s, ev_start);
      HIP_TRY(hipGetLastError());
    }
    if (ra.wg1 + ra.wg2) {
      HIP_TRY(hipEventRecord(e->ev_rank[a.launch_seq & 1u], e->rank_s));
      e->rank_seq = a.launch_seq;
    }
  } else {
    launch_pipeline(a, e->main_s, ev_start);
    HIP_TRY(hipGetLastError());
  }
  if (s3) {
    e->applied++;
    e->st.leo = nxt.leo;
    e->st.used = nxt.used;
    for (uint32_t j = 0; j < s3->nb; ++j) {
      const InFlight& f = s3->b[j];
      if (f.host_out && f.b.n)
        HIP_TRY(hipMemcpyAsync(f.host_out, f.b.out_offsets, f.b.n * 8ull, hipMemcpyDeviceToHost, e->main_s));
    }
    // this launch also completes the empty tickets up to the next group's first one
    const GroupFlight* next = s2 ? s2 : s1;
    const uint64_t hi = next ? next->b[0].ticket - 1 : e->last_ticket;
    e->marks.emplace_back(hi, e->launch_seq);
  }
  return repl_after_launch(e, s2, s3);
}

// One launch: ranks the group being formed (if any) and advances the groups ahead of it.
int close_group(rmq_engine* e) {
  const GroupFlight* s1 = e->forming.nb ? &e->forming : nullptr;
  // bounded run-ahead (RMQ_AHEAD launches queued at most, no transport): a fetch or an offset
  // commit is ordered after the launches issued before it, so an unbounded queue would make its
  // latency grow with how far the host runs ahead (device batches are never waited for otherwise).
  // Launch L's first lane reports L - 1 complete (done word).
  if (e->max_ahead && !e->repl) {
    const uint64_t need = e->launch_seq + 1 > e->max_ahead ? e->launch_seq + 1 - e->max_ahead : 0;
    // poll the done word (host memory); the stream itself only now and then (a faulted launch
    // never moves the word: its sticky error ends the wait)
    for (uint32_t spin = 1; need > __atomic_load_n(e->done_host, __ATOMIC_ACQUIRE); ++spin) {
      if ((spin & 1023u) == 0) {
        const hipError_t q = hipStreamQuery(e->main_s);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) return hip_fail(q);
      }
      __builtin_ia32_pause();
    }
  }
  int rc = launch_stages(e, s1, e->has1 ? &e->g1 : nullptr, e->has2 ? &e->g2 : nullptr,
                         e->has3 ? &e->g3 : nullptr);
  if (rc) return rc;
  e->has3 = e->has2;
  e->g3 = e->g2;
  if (e->has3) e->g3_seq = e->launch_seq;  // the launch that applied it
  e->has2 = e->has1;
  e->g2 = e->g1;
  e->has1 = s1 != nullptr;
  if (s1) e->g1 = e->forming;
  e->forming = GroupFlight{};
  return RMQ_OK;
}

// Push everything through stage 3 (at most three launches). The stage-3 launch of a group applies
// its retention too unless a partition's group outgrew the entries written before it
// (pipeline.hip partition_threads): drain() then adds the stage-4 launch. With a transport a flush
// is collective and every rank makes the same launches: stage 4 always.
int flush(rmq_engine* e) {
  while (e->forming.nb || e->has1 || e->has2 || (e->has3 && e->repl)) {
    int rc = close_group(e);
    if (rc) return rc;
  }
  return RMQ_OK;
}

void collect_done(rmq_engine* e);

int drain(rmq_engine* e) {
  int rc = flush(e);
  if (!rc) rc = repl_drain(e);  // the remaining replication rounds and their acks
  if (rc) return rc;
  if (e->profile && e->prof_started && !e->prof_ended) {
    HIP_TRY(hipEventRecord(e->prof_t1, e->main_s));
    e->prof_ended = true;
  }
  rc = stream_wait(e->main_s);
  if (rc) return rc;
  if (e->has3) {  // the last group's retention: finished by its own launch unless ret_late names it
    if (__atomic_load_n(e->done_host + 1, __ATOMIC_ACQUIRE) >= e->g3_seq) {
      rc = close_group(e);  // stage 4 alone
      if (rc) return rc;
      if (e->profile && e->prof_ended) HIP_TRY(hipEventRecord(e->prof_t1, e->main_s));
      rc = stream_wait(e->main_s);
      if (rc) return rc;
    } else {
      e->set_reset |= 1u << e->g3.set;  // its stage 4 would reset the set's list and sums
    }
    e->has3 = false;
  }
  collect_done(e);
  return RMQ_OK;
}

// The last applied group's retention, where its own launch stopped early (late_retention_kernel),
// before a fetch or a state read ordered after that launch; once per applied group.
int late_retention(rmq_engine* e) {
  if (!e->has3 || e->late_done == e->g3_seq) return RMQ_OK;
  LateArgs a{};
  a.st = e->st;
  a.bcum = e->scratch[e->g3.set].bcum;
  a.totals = e->scratch[e->g3.set].totals;
  a.rlate = e->d_rlate;
  a.nb = e->g3.nb;
  launch_late_retention(a, e->main_s);
  HIP_TRY(hipGetLastError());
  e->late_done = e->g3_seq;
  return RMQ_OK;
}

// The asynchronous fetches held back (fetch_issue) as ONE resolve + gather pair (kFetchBatch tickets
// at most), each ticket's completion event after it. Called (under mu) by the next fetch that cannot
// join them, by every other call that takes the engine lock (EngineLock: whatever it issues on the
// pipeline stream stays ordered after the fetches issued before it), and by a poll of a held ticket.
int fetch_flush(rmq_engine* e) {
  if (e->fpend.empty()) return RMQ_OK;
  int rc = late_retention(e);
  if (rc) return rc;
  FetchArgs t[kFetchBatch];
  uint32_t nt = 0;
  for (uint32_t i : e->fpend) t[nt++] = e->fslot[i].args;
  launch_fetch_batch(t, nt, e->main_s);
  HIP_TRY(hipGetLastError());
  for (uint32_t i : e->fpend) {
    HIP_TRY(hipEventRecord(e->fslot[i].ev, e->main_s));
    e->fslot[i].pending = false;
  }
  e->fpend.clear();
  return RMQ_OK;
}

// Wait for everything issued on the pipeline stream, without flushing batches that are still
// forming or in the pipeline's earlier stages (reads of committed state, consumer commits).
int quiesce(rmq_engine* e) {
  int rc0 = late_retention(e);
  if (rc0) return rc0;
  int rc = stream_wait(e->main_s);
  if (rc) return rc;
  collect_done(e);
  return RMQ_OK;
}

// Drain, or with a replication transport (where a flush is collective: rmq_sync) just wait for
// what is issued: device memory management and profiling calls.
int settle(rmq_engine* e) { return e->repl ? quiesce(e) : drain(e); }

// Has the launch with sequence number L completed?
bool launch_done(rmq_engine* e, uint64_t L) {
  if (L <= __atomic_load_n(e->done_host, __ATOMIC_ACQUIRE)) return true;
  return hipStreamQuery(e->main_s) == hipSuccess;
}

// Completed launches: the tickets they complete, and those host batches' out offsets from their
// pinned slots into the callers' buffers.
void collect_done(rmq_engine* e) {
  while (!e->marks.empty() && launch_done(e, e->marks.front().second)) {
    e->done_ticket = std::max(e->done_ticket, e->marks.front().first);
    e->marks.pop_front();
  }
  for (Staging& sg : e->staging)
    if (sg.user_out && sg.ticket <= e->done_ticket) {
      std::memcpy(sg.user_out, sg.h_out, (size_t)sg.out_n * 8);
      sg.user_out = nullptr;
    }
}

// Ticket completion: 1 complete, 0 applied by a launch still running, -1 not applied yet.
int ticket_state(rmq_engine* e, uint64_t t) {
  collect_done(e);
  if (t <= e->done_ticket) return 1;
  if (!e->marks.empty() && t <= e->marks.back().first) return 0;
  return -1;
}

// Block until ticket t (issued) is applied and complete.
int wait_ticket(rmq_engine* e, uint64_t t) {
  int s = ticket_state(e, t);
  if (s < 0) {
    if (e->repl) return RMQ_PENDING;  // a flush is collective with a transport: rmq_sync on every rank
    int rc = flush(e);
    if (rc) return rc;
    s = ticket_state(e, t);
  }
  if (s == 0) {  // wait for the launch that completes t, not for everything queued behind it
    uint64_t L = e->launch_seq;
    for (const auto& m : e->marks)
      if (m.first >= t) {
        L = m.second;
        break;
      }
    // the done word only moves while launches succeed: a faulted stream (sticky error) ends the wait
    while (L > __atomic_load_n(e->done_host, __ATOMIC_ACQUIRE)) {
      const hipError_t q = hipStreamQuery(e->main_s);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) return hip_fail(q);
      std::this_thread::yield();
    }
    ticket_state(e, t);
  }
  return RMQ_OK;
}

// The pipeline advances the double-buffered log end only for partitions this engine leads; before
// a partition changes role, both state sets must hold its current log end (engine drained).
int equalize_state_sets(rmq_engine* e) {
  const StateSet other = e->sets[(e->applied + 1) & 1u];
  const size_t bytes = (size_t)e->cfg.num_partitions * 8;
  HIP_TRY(hipMemcpy(other.leo, e->st.leo, bytes, hipMemcpyDeviceToDevice));
  HIP_TRY(hipMemcpy(other.used, e->st.used, bytes, hipMemcpyDeviceToDevice));
  return RMQ_OK;
}

int ensure_ctl(rmq_engine* e, uint32_t n) {
  if (n <= e->ctl_cap) return RMQ_OK;
  hipFree(e->d_ctl32);
  hipFree(e->d_ctl64);
  e->ctl_cap = 0;
  uint32_t cap = std::max<uint32_t>(n, 1024);
  int rc = dalloc(&e->d_ctl32, (size_t)cap * 2);
  if (rc) return rc;
  rc = dalloc(&e->d_ctl64, (size_t)cap);
  if (rc) return rc;
  e->ctl_cap = cap;
  return RMQ_OK;
}

void dump_stamps(rmq_engine* e) {
  const uint32_t nwg = e->stamps_wg[0] + e->stamps_wg[1] + e->stamps_wg[2] + e->stamps_wg[3];
  if (!e->stamps_path || !e->d_stamps || !nwg) return;
  // the launch's layout: waves per workgroup of its variant, roles in dispatch order
  const uint32_t wpg = (e->repl ? kPipeThreadsXR : kPipeThreads) / 64u;
  std::vector<uint64_t> h((size_t)nwg * wpg * 8);
  if (hipMemcpy(h.data(), e->d_stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  FILE* f = std::fopen(e->stamps_path, "w");
  if (!f) return;
  std::fprintf(f, "wg,wave,stage,t0,t1,t2,t3,t4,t5,t6,t7\n");
  const uint32_t w1 = e->stamps_wg[0], w2 = e->stamps_wg[1], wp = e->stamps_wg[2];
  for (uint32_t g = 0; g < nwg; ++g) {
    const uint32_t ld = e->stamps_wg[4];  // stage-3 workgroups before the other roles
    const int stage = g < ld ? 3 : g < ld + w1 ? 1 : g < ld + w1 + w2 ? 2 : g < ld + w1 + w2 + wp ? 4 : 3;  // 4: partitions
    for (uint32_t w = 0; w < wpg; ++w) {
      std::fprintf(f, "%u,%u,%d", g, w, stage);
      for (int k = 0; k < 8; ++k) std::fprintf(f, ",%llu", (unsigned long long)h[((size_t)g * wpg + w) * 8 + k]);
      std::fprintf(f, "\n");
    }
  }
  std::fclose(f);
}

void free_engine(rmq_engine* e) {
  if (!e) return;
  hipSetDevice(e->device);
  if (e->main_s) {
    // every submitted batch is applied before the memory goes away; with a replication transport
    // a flush is collective, so the application must have called rmq_sync on every rank
    (void)fetch_flush(e);
    if (!e->repl) flush(e);
    hipStreamSynchronize(e->main_s);
    if (e->rank_s) hipStreamSynchronize(e->rank_s);
    dump_stamps(e);
  }
  repl_free(e);
  DevState& s = e->st;
  std::vector<void*> bufs = {s.start_off, s.start_pos, s.commit, s.hw, s.term_start, s.term, s.match, s.is_leader,
                             s.local_mask, s.index, s.logs, s.ring, s.cons, s.pcache, s.rcur, s.cdirty, s.lcommit, s.csnap, s.cver, s.cq,
                             s.lterm, s.mterm, s.heard, e->d_crc,
                             e->d_stats, e->d_ctl32, e->d_ctl64, e->d_stamps, e->d_rlate};
  if (e->state_stage) hipHostFree(e->state_stage);
  for (rmq_engine::FetchSlot& f : e->fslot) {
    void* fs[] = {f.d_req, f.d_res, f.d_aux, f.d_cpre, f.d_csum, f.d_out};
    for (void* p : fs) bufs.push_back(p);
    if (f.h_req) hipHostFree(f.h_req);
    if (f.h_res) hipHostFree(f.h_res);
    if (f.ev) hipEventDestroy(f.ev);
    if (f.ev_copy) hipEventDestroy(f.ev_copy);
    if (f.ev_in) hipEventDestroy(f.ev_in);
    if (f.ev_k) hipEventDestroy(f.ev_k);
  }
  for (const StateSet& z : e->sets) {
    bufs.push_back(z.leo);
    bufs.push_back(z.used);
  }
  for (const PipeScratch& x : e->scratch) {
    void* xs[] = {x.hist32, x.hist, x.excl, x.totals, x.pk, x.bcum, x.crank, x.pre, x.tsum, x.tile_base, x.binfo, x.bacc, x.nbig, x.bigl};
    for (void* p : xs) bufs.push_back(p);
  }
  delete e->copy_pool;
  for (const Staging& sg : e->staging) {
    bufs.push_back(sg.d_blk);
    bufs.push_back(sg.d_out);
    if (sg.h_blk) hipHostFree(sg.h_blk);
    if (sg.h_out) hipHostFree(sg.h_out);
    if (sg.ev_in) hipEventDestroy(sg.ev_in);
  }
  for (void* p : bufs)
    if (p) hipFree(p);
  if (e->done_host) hipHostFree(e->done_host);
  if (e->fetch_need_host) hipHostFree(e->fetch_need_host);
  for (auto& cs : e->cslot) {
    if (cs.h) hipHostFree(cs.h);
    if (cs.d) hipFree(cs.d);
    if (cs.ev) hipEventDestroy(cs.ev);
  }
  if (e->ev_main) hipEventDestroy(e->ev_main);
  for (hipEvent_t ev : e->ev_rank)
    if (ev) hipEventDestroy(ev);
  if (e->ev_pre_rank) hipEventDestroy(e->ev_pre_rank);
  if (e->rank_s) hipStreamDestroy(e->rank_s);
  if (e->fetch_out_s) hipStreamDestroy(e->fetch_out_s);
  if (e->copy_s) hipStreamDestroy(e->copy_s);
  for (auto& v : e->prof)
    for (EvPair& p : v) {
      if (p.a) hipEventDestroy(p.a);
      if (p.b) hipEventDestroy(p.b);
    }
  for (hipEvent_t ev : e->ev_pool) hipEventDestroy(ev);
  if (e->prof_t0) hipEventDestroy(e->prof_t0);
  if (e->prof_t1) hipEventDestroy(e->prof_t1);
  if (e->main_s) hipStreamDestroy(e->main_s);
  delete e;
}

int validate_cfg(const rmq_config* c) {
  if (!c) return RMQ_EINVAL;
  if (c->num_partitions == 0 || c->num_partitions > kMaxPartitions) return RMQ_EINVAL;
  if (c->replication_factor == 0 || c->replication_factor > RMQ_MAX_RF) return RMQ_EINVAL;
  if (!is_pow2(c->index_interval) || c->index_interval < 64 || c->index_interval > (1u << 20))
    return RMQ_EINVAL;
  if (!is_pow2(c->segment_bytes) || c->segment_bytes < 4ull * c->index_interval) return RMQ_EINVAL;
  if (c->max_consumers == 0) return RMQ_EINVAL;
  if (c->max_batch_records == 0 || c->max_batch_records > kMaxBatchRecords) return RMQ_EINVAL;
  if (c->max_batch_bytes >= (1ull << 32)) return RMQ_EINVAL;
  if (c->pipeline_depth > kMaxGroup) return RMQ_EINVAL;
  const uint64_t g = c->pipeline_depth ? c->pipeline_depth : 2u;
  const uint64_t pool = c->pool_bytes ? c->pool_bytes : (uint64_t)c->num_partitions * c->segment_bytes;
  if (pool < (uint64_t)c->num_partitions * c->segment_bytes || pool % c->index_interval) return RMQ_EINVAL;
  if ((2 * g + 2) * (pool / c->index_interval) >= (1ull << 40)) return RMQ_EINVAL;
  return RMQ_OK;
}

}  // namespace rmq

extern "C" {

uint32_t rmq_abi_version(void) { return RMQ_ABI_VERSION; }

int rmq_host_alloc(rmq_engine* e, uint64_t bytes, void** out) {
  if (!e || !out || !bytes) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  *out = nullptr;
  if (hipHostMalloc(out, bytes, 0) != hipSuccess) return RMQ_ENOMEM;
  return RMQ_OK;
}

int rmq_host_free(rmq_engine* e, void* p) {  // e may be NULL (after rmq_destroy)
  (void)e;
  if (p && hipHostFree(p) != hipSuccess) return RMQ_EDEVICE;
  return RMQ_OK;
}

int rmq_host_register(rmq_engine* e, void* p, uint64_t bytes) {
  if (!e || !p || !bytes) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterDefault));
  return RMQ_OK;
}

int rmq_host_unregister(rmq_engine* e, void* p) {
  if (!e || !p) return RMQ_EINVAL;
  HIP_TRY(hipHostUnregister(p));
  return RMQ_OK;
}

const char* rmq_strerror(int s) {
  switch (s) {
    case RMQ_OK: return "ok";
    case RMQ_PENDING: return "pending";
    case RMQ_ENOTLEADER: return "Not leader";
    case RMQ_ENOPART: return "unknown partition";
    case RMQ_EINVAL: return "invalid argument";
    case RMQ_ENOSPC: return "no space";
    case RMQ_EDEVICE: return "device error";
    case RMQ_EOFFSET: return "offset out of range";
    case RMQ_ENOMEM: return "out of memory";
    case RMQ_ESTALE: return "replica lags the committed log";
    case RMQ_ETERM: return "term already led or voted for another candidate";
    default: return "unknown status";
  }
}

void rmq_config_default(rmq_config* c, uint32_t P, uint32_t RF) {
  if (!c) return;
  std::memset(c, 0, sizeof *c);
  c->num_partitions = P;
  c->replication_factor = RF;
  c->segment_bytes = 1ull << 20;
  c->index_interval = 1024;
  c->max_consumers = 8;
  c->max_batch_records = 65536;
  c->pipeline_depth = 2;
  c->max_batch_bytes = 64ull << 20;
  c->device = 0;
  c->rank = 0;
}

int rmq_create(const rmq_config* cfg, rmq_engine** out) {
  if (!out) return RMQ_EINVAL;
  *out = nullptr;
  int rc = validate_cfg(cfg);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || cfg->device < 0 || cfg->device >= ndev)
    return RMQ_EDEVICE;
  rmq_engine* e = new (std::nothrow) rmq_engine();
  if (!e) return RMQ_ENOMEM;
  e->cfg = *cfg;
  if (!e->cfg.pipeline_depth) e->cfg.pipeline_depth = 2;
  e->device = cfg->device;
  e->stamps_path = std::getenv("RMQ_STAMPS");
  if (const char* v = std::getenv("RMQ_TRACE")) e->trace = std::atoi(v) != 0;
  if (const char* v = std::getenv("RMQ_DEBUG")) e->debug = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_WG3_ALL")) e->wg3_all = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S1_WGS")) e->s1_wgs = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S2_WGS")) e->s2_wgs = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S3_FIRST")) e->s3_first = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_PRIO")) e->prio = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S3_LEAD")) e->s3_lead = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_RANK")) e->rank_mode = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_STEAL")) e->steal = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_AHEAD")) e->max_ahead = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_STAMPS_AT")) e->stamps_at = std::strtoull(v, nullptr, 10);
  if (const char* v = std::getenv("RMQ_SPLIT")) e->split = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S3_PAIR")) e->s3_pair = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S3_ROLES")) e->s3_roles = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S3_STAGE")) e->s3_stage = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_FETCH_COALESCE")) e->fetch_coalesce = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S3_XCD")) e->s3_xcd = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_S1_XCD")) e->s1_xcd = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_RANK_CUS")) e->rank_cus = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_FETCH_DMA")) e->fetch_dma = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RMQ_FETCH_DMA_IN")) e->fetch_dma_in = (uint32_t)std::atoi(v);
  if (e->stamps_path || e->steal) e->split = 0;  // (phase stamps and stealing read one launch's roles)
#define CREATE_TRY(x)      \
  do {                     \
    int _r = (x);          \
    if (_r) {              \
      free_engine(e);      \
      return _r;           \
    }                      \
  } while (0)
#define CREATE_HIP(x) CREATE_TRY(hip_fail(x))
  CREATE_HIP(hipSetDevice(e->device));
  hipDeviceProp_t prop;
  CREATE_HIP(hipGetDeviceProperties(&prop, e->device));
  e->cu_count = (uint32_t)prop.multiProcessorCount;
  e->verify_wgs = verify_wgs_per_cu() * e->cu_count;
  if (const char* v = std::getenv("RMQ_VERIFY_WGS")) e->verify_wgs = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("RMQ_BIG_WGS")) e->big_wgs = (uint32_t)std::atoi(v);
  std::snprintf(e->dev_name, sizeof e->dev_name, "%s (%s)", prop.name, prop.gcnArchName);
  if (e->split && e->rank_cus && e->rank_cus < e->cu_count) {
    // CU masks (bit i = the i-th CU in the runtime's numbering): the rank stream takes the first
    // rank_cus bits, the pipeline stream the rest
    std::vector<uint32_t> mr((e->cu_count + 31) / 32, 0u), mm(mr.size(), 0u);
    for (uint32_t i = 0; i < e->cu_count; ++i) (i < e->rank_cus ? mr : mm)[i / 32] |= 1u << (i % 32);
    CREATE_HIP(hipExtStreamCreateWithCUMask(&e->main_s, (uint32_t)mm.size(), mm.data()));
    CREATE_HIP(hipExtStreamCreateWithCUMask(&e->rank_s, (uint32_t)mr.size(), mr.data()));
  } else {
    CREATE_HIP(hipStreamCreateWithFlags(&e->main_s, hipStreamNonBlocking));
    if (e->split) CREATE_HIP(hipStreamCreateWithFlags(&e->rank_s, hipStreamNonBlocking));
  }
  if (e->split) {
    for (hipEvent_t& ev : e->ev_rank) CREATE_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CREATE_HIP(hipEventCreateWithFlags(&e->ev_pre_rank, hipEventDisableTiming));
  }
  CREATE_HIP(hipStreamCreateWithFlags(&e->fetch_out_s, hipStreamNonBlocking));
  preload_fetch_kernels();
  CREATE_HIP(hipStreamCreateWithFlags(&e->copy_s, hipStreamNonBlocking));
  CREATE_HIP(hipEventCreateWithFlags(&e->ev_main, hipEventDisableTiming));
  for (rmq_engine::FetchSlot& f : e->fslot) {
    CREATE_HIP(hipEventCreateWithFlags(&f.ev, hipEventDisableTiming));
    CREATE_HIP(hipEventCreateWithFlags(&f.ev_copy, hipEventDisableTiming));
    CREATE_HIP(hipEventCreateWithFlags(&f.ev_in, hipEventDisableTiming));
    CREATE_HIP(hipEventCreateWithFlags(&f.ev_k, hipEventDisableTiming));
  }

  const uint32_t P = cfg->num_partitions, RF = cfg->replication_factor, C = cfg->max_consumers;
  DevState& s = e->st;
  s.P = P;
  s.RF = RF;
  s.C = C;
  s.interval_log2 = ilog2(cfg->index_interval);
  e->group_max = std::min<uint32_t>(kMaxGroup, e->cfg.pipeline_depth);
  // stage 4 reads a group's index entries while stage 3 of the group two later writes new ones
  // (each batch adds at most ring - interval bytes to a partition): 2G + 1 rings' worth of entries
  // (+2) keep every entry stage 4 may read from being overwritten in time; (2G + 2) per interval
  // of ring covers that for every ring of at least 4 intervals
  s.icap_mul = 2u * e->group_max + 2u;
  s.rstride = cfg->pool_bytes ? cfg->pool_bytes : (uint64_t)P * cfg->segment_bytes;
  e->pool.size = s.rstride;
  e->ring.assign(P, 0);
  for (uint32_t p = 0; p < P; ++p) {  // every partition starts with a segment_bytes ring
    uint64_t off = 0;
    const uint32_t lg = ilog2(cfg->segment_bytes);
    if (!e->pool.alloc(lg, &off)) {
      free_engine(e);
      return RMQ_EINVAL;
    }
    e->ring[p] = off | lg;
  }
  for (StateSet& z : e->sets) {
    CREATE_TRY(dalloc(&z.leo, P));
    CREATE_TRY(dalloc(&z.used, P));
  }
  s.leo = e->sets[0].leo;
  s.used = e->sets[0].used;
  CREATE_TRY(dalloc(&s.start_off, P));
  CREATE_TRY(dalloc(&s.start_pos, P));
  CREATE_TRY(dalloc(&s.commit, P));
  CREATE_TRY(dalloc(&s.hw, P));
  CREATE_TRY(dalloc(&s.term_start, P));
  CREATE_TRY(dalloc(&s.term, P));
  CREATE_TRY(dalloc(&s.match, (size_t)P * RF));
  CREATE_TRY(dalloc(&s.is_leader, P));
  CREATE_TRY(dalloc(&s.local_mask, P));
  CREATE_TRY(dalloc(&s.index, (size_t)(s.rstride >> s.interval_log2) * s.icap_mul * 2));
  CREATE_TRY(dalloc(&s.logs, (size_t)RF * s.rstride));
  CREATE_TRY(dalloc(&s.ring, P));
  CREATE_HIP(hipMemcpy(s.ring, e->ring.data(), (size_t)P * 8, hipMemcpyHostToDevice));
  CREATE_TRY(dalloc(&s.cons, (size_t)P * C));
  CREATE_TRY(dalloc(&s.pcache, (size_t)P * C * 2));
  CREATE_TRY(dalloc(&s.rcur, (size_t)P));  // (dalloc zero-fills: every replica cursor at offset 0)
  CREATE_HIP(hipMemset(s.pcache, 0xFF, (size_t)P * C * 16));  // every entry empty
  CREATE_TRY(dalloc(&s.cdirty, P));
  CREATE_TRY(dalloc(&s.lcommit, P));
  CREATE_TRY(dalloc(&s.lterm, P));
  CREATE_TRY(dalloc(&s.mterm, P));
  CREATE_TRY(dalloc(&s.heard, P));
  CREATE_TRY(dalloc(&s.cver, P));
  CREATE_TRY(dalloc(&s.cq, P));
  e->cver.assign(P, 0ull);
  CREATE_TRY(dalloc(&e->d_rlate, P));
  e->max_tiles = (cfg->max_batch_records + kTileRecs - 1) / kTileRecs;
  e->max_tasks = (cfg->max_batch_records + kTaskRecs - 1) / kTaskRecs;
  CREATE_TRY(dalloc(&e->d_stats, (size_t)kStatsRing * e->max_tasks));
  // a multiple of four: stage 2 reads u32 hist columns with 16-byte loads
  e->max_group_tiles = (std::min<uint32_t>(kMaxTiles, e->group_max * e->max_tiles) + 3u) & ~3u;
  for (PipeScratch& x : e->scratch) {
    const size_t GT = e->max_group_tiles, TP = GT * P;
    CREATE_TRY(dalloc(&x.hist32, TP));
    CREATE_TRY(dalloc(&x.hist, TP));
    CREATE_TRY(dalloc(&x.excl, TP));
    CREATE_TRY(dalloc(&x.totals, P));
    CREATE_TRY(dalloc(&x.pk, (size_t)P * 8));
    CREATE_TRY(dalloc(&x.bcum, (size_t)kMaxGroup * P));
    CREATE_TRY(dalloc(&x.crank, GT * kTileRecs));
    CREATE_TRY(dalloc(&x.pre, GT * kTileRecs));
    CREATE_TRY(dalloc(&x.tsum, GT * 4));
    CREATE_TRY(dalloc(&x.tile_base, GT));
    CREATE_TRY(dalloc(&x.binfo, (size_t)kMaxGroup * 4));
    CREATE_TRY(dalloc(&x.bacc, (size_t)kMaxGroup * 2));
    CREATE_TRY(dalloc(&x.nbig, 4));
    CREATE_TRY(dalloc(&x.bigl, GT * kTileRecs));
  }
  if (e->stamps_path) CREATE_TRY(dalloc(&e->d_stamps, (size_t)(2u * e->cu_count + kMaxTiles + (P + kPipeThreads - 1) / kPipeThreads +
                                                       kMaxTiles * kTileRecs / (kTaskRecs * kPipeThreads / 64)) * 64));
  CREATE_HIP(hipHostMalloc((void**)&e->fetch_need_host, 8 * rmq_engine::kFetchSlots, hipHostMallocCoherent | hipHostMallocMapped));
  for (uint32_t k = 0; k < rmq_engine::kFetchSlots; ++k) {
    e->fslot[k].need = e->fetch_need_host + k;
    *e->fslot[k].need = 0;
    CREATE_HIP(hipHostGetDevicePointer((void**)&e->fslot[k].need_dev, e->fslot[k].need, 0));
  }
  CREATE_HIP(hipHostMalloc((void**)&e->done_host, 64, hipHostMallocCoherent | hipHostMallocMapped));
  e->done_host[0] = e->done_host[1] = 0;
  CREATE_HIP(hipHostGetDevicePointer((void**)&e->done_dev, e->done_host, 0));
  {
    CrcConsts h;
    build_crc_consts(&h);
    CREATE_TRY(dalloc(&e->d_crc, 1));
    CREATE_HIP(hipMemcpy(e->d_crc, &h, sizeof h, hipMemcpyHostToDevice));
  }
  {
    std::vector<uint32_t> ones(P, 1u), mask(P, (1u << RF) - 1u);
    CREATE_HIP(hipMemcpy(s.is_leader, ones.data(), P * 4ull, hipMemcpyHostToDevice));
    CREATE_HIP(hipMemcpy(s.local_mask, mask.data(), P * 4ull, hipMemcpyHostToDevice));
  }
  e->is_leader.assign(P, 1u);
  e->leader_slot.assign(P, 0u);
  e->ranks.assign((size_t)P * RF, cfg->rank);
  e->term.assign(P, 1ull);
  CREATE_HIP(hipMemcpy(s.term, e->term.data(), P * 8ull, hipMemcpyHostToDevice));
  // every partition is led here from term 1 (its leader-start entry, its own vote)
  CREATE_HIP(hipMemcpy(s.lterm, e->term.data(), P * 8ull, hipMemcpyHostToDevice));
  CREATE_HIP(hipMemcpy(s.mterm, e->term.data(), P * 8ull, hipMemcpyHostToDevice));
  e->vterm.assign(P, 1ull);
  e->vfor.assign(P, cfg->rank);
  e->vled.assign(P, 1u);
  e->key.resize(P);
  for (uint32_t p = 0; p < P; ++p) e->key[p] = p;
  e->ticket_n.assign(kStatsRing, 0u);
  {
    uint32_t bits = 0;
    while ((1u << bits) < P) ++bits;  // keys in [0, P)
    e->key_passes = bits == 0 ? 0u : bits <= 8 ? 1u : 2u;
    e->key_bits = bits;
  }
  e->staging.resize(4u * e->group_max + 1u);  // batches of the forming group and of three in flight
  CREATE_HIP(hipDeviceSynchronize());
  *out = e;
  return RMQ_OK;
#undef CREATE_TRY
#undef CREATE_HIP
}

void rmq_destroy(rmq_engine* e) { free_engine(e); }

namespace {

// Placement of n partitions (engine locked). With a replication transport this is collective:
// every rank recomputes its out / in lists and checks them against its peers'.
int set_placement(rmq_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* key, const uint32_t* ranks,
                  const uint32_t* leader_slot) {
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  if (n && (!pidx || !ranks || !leader_slot)) return RMQ_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    if (pidx[i] >= P) return RMQ_ENOPART;
    if (leader_slot[i] >= RF) return RMQ_EINVAL;
  }
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (!rc) rc = equalize_state_sets(e);
  if (rc) return rc;
  std::vector<uint32_t> mask(P);
  std::vector<uint32_t> demoted;  // partitions this engine stops leading
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t p = pidx[i];
    for (uint32_t r = 0; r < RF; ++r) e->ranks[(size_t)p * RF + r] = ranks[(size_t)i * RF + r];
    e->leader_slot[p] = leader_slot[i];
    const uint32_t lead = ranks[(size_t)i * RF + leader_slot[i]] == e->cfg.rank;
    if (e->is_leader[p] && !lead) demoted.push_back(p);
    // a placement keeps or ends this replica's leadership; it never starts one: a replica the
    // placement names leader leads once rmq_become_leader passes Raft's checks
    e->is_leader[p] = lead && e->is_leader[p];
    if (key) e->key[p] = key[i];
  }
  if (!demoted.empty()) {  // a former leader knows its own commit as the leader's (FORMAT.md §9 v4)
    std::vector<uint64_t> c(P), lc(P);
    HIP_TRY(hipMemcpy(c.data(), e->st.commit, P * 8ull, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(lc.data(), e->st.lcommit, P * 8ull, hipMemcpyDeviceToHost));
    for (uint32_t p : demoted) lc[p] = std::max(lc[p], c[p]);
    HIP_TRY(hipMemcpy(e->st.lcommit, lc.data(), P * 8ull, hipMemcpyHostToDevice));
  }
  for (uint32_t p = 0; p < P; ++p) {
    mask[p] = 0;
    for (uint32_t r = 0; r < RF; ++r) mask[p] |= (e->ranks[(size_t)p * RF + r] == e->cfg.rank ? 1u : 0u) << r;
  }
  HIP_TRY(hipMemcpy(e->st.is_leader, e->is_leader.data(), P * 4ull, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->st.local_mask, mask.data(), P * 4ull, hipMemcpyHostToDevice));
  if (n) {  // the election timer of every placed partition restarts
    std::vector<uint64_t> hd(P);
    HIP_TRY(hipMemcpy(hd.data(), e->st.heard, P * 8ull, hipMemcpyDeviceToHost));
    const uint64_t cur = e->repl ? e->repl->stamp : 0ull;
    for (uint32_t i = 0; i < n; ++i) hd[pidx[i]] = cur;
    HIP_TRY(hipMemcpy(e->st.heard, hd.data(), P * 8ull, hipMemcpyHostToDevice));
    e->place_time = std::chrono::steady_clock::now();
  }
  return e->repl ? repl_set_lists(e) : RMQ_OK;
}

}  // namespace

int rmq_set_replicas(rmq_engine* e, uint32_t pidx, const uint32_t* ranks, uint32_t rf, uint32_t leader_slot) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (pidx >= e->cfg.num_partitions) return RMQ_ENOPART;
  if (!ranks || rf != e->cfg.replication_factor || leader_slot >= rf) return RMQ_EINVAL;
  return set_placement(e, 1, &pidx, nullptr, ranks, &leader_slot);
}

int rmq_set_placement(rmq_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* key, const uint32_t* ranks,
                      const uint32_t* leader_slot) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  return set_placement(e, n, pidx, key, ranks, leader_slot);
}

int rmq_become_leader(rmq_engine* e, uint32_t pidx, uint64_t term) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  if (pidx != RMQ_ALL_PARTITIONS && pidx >= P) return RMQ_ENOPART;
  const uint32_t lo = pidx == RMQ_ALL_PARTITIONS ? 0 : pidx, hi = pidx == RMQ_ALL_PARTITIONS ? P : pidx + 1;
  for (uint32_t p = lo; p < hi; ++p) {  // validate everything before changing anything
    bool local = false;
    for (uint32_t r = 0; r < RF; ++r) local |= e->ranks[(size_t)p * RF + r] == e->cfg.rank;
    if (!local) return RMQ_EINVAL;
    // with a transport the placement (collective) names the leader; this starts its term
    if (e->repl && e->ranks[(size_t)p * RF + e->leader_slot[p]] != e->cfg.rank) return RMQ_EINVAL;
  }
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (!rc) rc = equalize_state_sets(e);
  if (rc) return rc;
  // a follower adopts newer leader terms from replication rounds (FORMAT.md §9): the device holds
  // the current terms
  HIP_TRY(hipMemcpy(&e->term[lo], e->st.term + lo, (size_t)(hi - lo) * 8, hipMemcpyDeviceToHost));
  for (uint32_t p = lo; p < hi; ++p) {
    if (term < e->term[p]) return RMQ_EINVAL;
    // one leader per term: not a term this replica led, nor one it gave its vote to another candidate
    if (e->vterm[p] == term && (e->vled[p] || e->vfor[p] != e->cfg.rank)) return RMQ_ETERM;
  }
  {
    // Raft's vote restriction, as far as this replica can tell: it may not lead a partition whose
    // leader committed records its log does not verifiably hold (leader_commit from rounds and
    // commit notices; verified: the whole log when it was matched in the current term, else the
    // replica's own commit)
    const size_t m = hi - lo;
    std::vector<uint64_t> leo(m), lc(m), mt(m), cm(m);
    HIP_TRY(hipMemcpy(leo.data(), e->st.leo + lo, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(lc.data(), e->st.lcommit + lo, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(mt.data(), e->st.mterm + lo, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(cm.data(), e->st.commit + lo, m * 8, hipMemcpyDeviceToHost));
    for (uint32_t p = lo; p < hi; ++p) {
      const size_t i = p - lo;
      const uint64_t verified = mt[i] == e->term[p] ? leo[i] : cm[i];
      if (verified < lc[i]) return RMQ_ESTALE;  // (a partition always led here: lc = 0)
    }
  }
  for (uint32_t p = lo; p < hi; ++p) {
    uint32_t slot = e->leader_slot[p];
    if (!e->repl) {
      slot = 0;
      while (e->ranks[(size_t)p * RF + slot] != e->cfg.rank) ++slot;
    }
    e->leader_slot[p] = slot;
    e->is_leader[p] = 1;
    e->term[p] = term;
    e->vterm[p] = term;  // a leader's vote is its own
    e->vfor[p] = e->cfg.rank;
    e->vled[p] = 1;
  }
  HIP_TRY(hipMemcpy(e->st.is_leader + lo, &e->is_leader[lo], (size_t)(hi - lo) * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->st.term + lo, &e->term[lo], (size_t)(hi - lo) * 8, hipMemcpyHostToDevice));
  launch_become_leader(e->st, pidx, e->main_s);
  HIP_TRY(hipGetLastError());
  rc = drain(e);
  // Raft's leader start: nextIndex of every follower = the leader's last index + 1
  if (!rc && e->repl) rc = reset_catchup(e);
  return rc;
}

// Before a vote reads a partition's term and log: without a transport every batch submitted is
// applied first (drain); with one, a flush would be collective (rmq_sync), so only what is issued is
// waited for: the pipeline stream and the rounds' ingest on the exchange stream.
static int vote_settle(rmq_engine* e) {
  if (!e->repl) return drain(e);
  int rc = quiesce(e);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(e->repl->xchg_s));
  return RMQ_OK;
}

int rmq_vote(rmq_engine* e, uint32_t pidx, uint64_t term, uint32_t candidate, uint64_t cand_last_log_term,
             uint64_t cand_log_end, uint32_t* granted) {
  if (!e || !granted) return RMQ_EINVAL;
  *granted = 0;
  EngineLock g(e);
  if (pidx >= e->cfg.num_partitions) return RMQ_ENOPART;
  HIP_TRY(hipSetDevice(e->device));
  int rc = vote_settle(e);
  if (rc) return rc;
  // with a transport nothing is flushed (a flush is collective): a leader of pidx whose groups in
  // flight may still add its records answers RMQ_PENDING and changes nothing (a delayed RequestVote)
  if (e->repl && e->is_leader[pidx] && (e->forming.nb || e->has1 || e->has2)) return RMQ_PENDING;
  uint64_t cur = 0, lterm = 0, leo = 0;
  HIP_TRY(hipMemcpy(&cur, e->st.term + pidx, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&lterm, e->st.lterm + pidx, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&leo, e->st.leo + pidx, 8, hipMemcpyDeviceToHost));
  lterm &= ~kLtermBound;  // an unknown last log term: its upper bound (a stricter vote)
  if (term < cur) return RMQ_OK;  // a candidate of an older term
  if (term > cur) {  // Raft: a newer term is adopted; a leader steps down
    e->term[pidx] = term;
    HIP_TRY(hipMemcpy(e->st.term + pidx, &term, 8, hipMemcpyHostToDevice));
    if (e->is_leader[pidx]) {
      rc = equalize_state_sets(e);
      if (rc) return rc;
      uint64_t c = 0, lc = 0;
      HIP_TRY(hipMemcpy(&c, e->st.commit + pidx, 8, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(&lc, e->st.lcommit + pidx, 8, hipMemcpyDeviceToHost));
      if (c > lc) HIP_TRY(hipMemcpy(e->st.lcommit + pidx, &c, 8, hipMemcpyHostToDevice));  // (FORMAT.md §9 v4)
      e->is_leader[pidx] = 0;
      const uint32_t z = 0;
      HIP_TRY(hipMemcpy(e->st.is_leader + pidx, &z, 4, hipMemcpyHostToDevice));
    }
  }
  const bool up = cand_last_log_term > lterm || (cand_last_log_term == lterm && cand_log_end >= leo);
  const bool free_vote = e->vterm[pidx] != term || (!e->vled[pidx] && e->vfor[pidx] == candidate);
  if (up && free_vote) {
    e->vterm[pidx] = term;
    e->vfor[pidx] = candidate;
    e->vled[pidx] = 0;
    *granted = 1;
  }
  return RMQ_OK;
}

int rmq_set_vote(rmq_engine* e, uint32_t pidx, uint64_t term, uint32_t voted_for) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (pidx >= e->cfg.num_partitions) return RMQ_ENOPART;
  HIP_TRY(hipSetDevice(e->device));
  int rc = vote_settle(e);
  if (rc) return rc;
  uint64_t cur = 0;
  HIP_TRY(hipMemcpy(&cur, e->st.term + pidx, 8, hipMemcpyDeviceToHost));
  if (term > cur) {
    e->term[pidx] = term;
    HIP_TRY(hipMemcpy(e->st.term + pidx, &term, 8, hipMemcpyHostToDevice));
  }
  e->vterm[pidx] = term;
  e->vfor[pidx] = voted_for;
  e->vled[pidx] = 0;
  return RMQ_OK;
}

int rmq_leader_silent(rmq_engine* e, uint32_t silent_rounds, uint32_t timeout_ms, uint32_t* out_pidx, uint32_t cap,
                      uint32_t* n) {
  if (!e || !n || (cap && !out_pidx)) return RMQ_EINVAL;
  *n = 0;
  EngineLock g(e);
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  HIP_TRY(hipSetDevice(e->device));
  if (e->repl) HIP_TRY(hipStreamSynchronize(e->repl->xchg_s));  // (the rounds' ingest writes the words)
  std::vector<uint64_t> hd(P);
  HIP_TRY(hipMemcpy(hd.data(), e->st.heard, P * 8ull, hipMemcpyDeviceToHost));
  const uint64_t cur = e->repl ? e->repl->stamp : 0ull;
  const auto now = std::chrono::steady_clock::now();
  uint32_t k = 0;
  for (uint32_t p = 0; p < P; ++p) {
    if (e->is_leader[p]) continue;
    bool local = false;
    for (uint32_t r = 0; r < RF; ++r) local |= e->ranks[(size_t)p * RF + r] == e->cfg.rank;
    if (!local || hd[p] + silent_rounds > cur) continue;
    // wall time since the leader was last heard (the round's posting, or the placement)
    auto at = e->place_time;
    if (e->repl && hd[p] && cur - hd[p] < 64) at = std::max(at, e->repl->stamp_time[hd[p] % 64]);
    if (std::chrono::duration_cast<std::chrono::milliseconds>(now - at).count() < (long long)timeout_ms) continue;
    if (k < cap) out_pidx[k] = p;
    ++k;
  }
  *n = k;
  return RMQ_OK;
}

int rmq_set_segments(rmq_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* seg) {
  if (!e) return RMQ_EINVAL;
  if (!n) return RMQ_OK;
  if (!pidx || !seg) return RMQ_EINVAL;
  std::lock_guard<std::mutex> fg(e->fetch_mu);  // no fetch reads a ring while it moves
  EngineLock g(e);
  const uint32_t P = e->cfg.num_partitions, ilog = e->st.interval_log2;
  std::vector<uint8_t> seen(P, 0);
  for (uint32_t i = 0; i < n; ++i) {
    if (pidx[i] >= P) return RMQ_ENOPART;
    if (seen[pidx[i]]++ || !is_pow2(seg[i]) || seg[i] < 4ull * e->cfg.index_interval || seg[i] > e->st.rstride)
      return RMQ_EINVAL;
  }
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  // (fetches run on the pipeline stream: the drain waited for them too)
  // new rings first, all or nothing
  std::vector<MigrateItem> items;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t p = pidx[i], lg = ilog2(seg[i]);
    if ((e->ring[p] & 63ull) == lg) continue;
    uint64_t off = 0;
    if (!e->pool.alloc(lg, &off)) {
      for (const MigrateItem& it : items) e->pool.release((uint32_t)(it.new_desc & 63ull), it.new_desc & ~63ull);
      return RMQ_ENOMEM;
    }
    MigrateItem it{};
    it.p = p;
    it.old_desc = e->ring[p];
    it.new_desc = off | lg;
    items.push_back(it);
  }
  if (items.empty()) return RMQ_OK;
  // retained range of every moved partition; a shrinking ring first applies retention at its new
  // size (FORMAT.md §4: start = the first record at or after used - S', from the index)
  std::vector<uint64_t> spos(P), soff(P), used(P);
  HIP_TRY(hipMemcpy(spos.data(), e->st.start_pos, (size_t)P * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(soff.data(), e->st.start_off, (size_t)P * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(used.data(), e->st.used, (size_t)P * 8, hipMemcpyDeviceToHost));
  for (MigrateItem& it : items) {
    const uint64_t S1 = 1ull << (it.new_desc & 63ull);
    const uint32_t p = it.p;
    if (used[p] - spos[p] > S1) {
      const uint64_t m = (used[p] - S1 + (1ull << ilog) - 1) >> ilog;
      const RingRef o = ring_ref(it.old_desc, ilog, e->st.icap_mul);
      uint64_t ent[2];
      HIP_TRY(hipMemcpy(ent, e->st.index + (o.ibase + m % o.icap) * 2, 16, hipMemcpyDeviceToHost));
      soff[p] = ent[0];
      spos[p] = ent[1];
    }
    it.spos = spos[p];
    it.soff = soff[p];
    it.used = used[p];
  }
  uint32_t chunks = 0;  // workgroups of each move: its new ring in kMigrateChunk pieces
  for (MigrateItem& it : items) {
    it.chunk0 = chunks;
    const uint64_t S1 = 1ull << (it.new_desc & 63ull);
    chunks += (uint32_t)((S1 + kMigrateChunk - 1) / kMigrateChunk);
  }
  MigrateItem* d_items = nullptr;
  rc = dalloc(&d_items, items.size());
  if (!rc) {
    HIP_TRY(hipMemcpy(d_items, items.data(), items.size() * sizeof(MigrateItem), hipMemcpyHostToDevice));
    launch_migrate(e->st, d_items, (uint32_t)items.size(), chunks, e->main_s);
    if (hipGetLastError() != hipSuccess) rc = RMQ_EDEVICE;
  }
  if (!rc) {
    for (const MigrateItem& it : items) {
      e->ring[it.p] = it.new_desc;
      e->pool.release((uint32_t)(it.old_desc & 63ull), it.old_desc & ~63ull);
    }
    HIP_TRY(hipStreamSynchronize(e->main_s));
    rc = check_err(e);
  } else {
    for (const MigrateItem& it : items) e->pool.release((uint32_t)(it.new_desc & 63ull), it.new_desc & ~63ull);
  }
  if (d_items) hipFree(d_items);
  return rc;
}

int rmq_append(rmq_engine* e, const rmq_batch* b, uint64_t* out_offsets, uint64_t* ticket) {
  if (!e || !b || !ticket) return RMQ_EINVAL;
  EngineLock g(e);
  const uint32_t n = b->n;
  if (n > e->cfg.max_batch_records) return RMQ_ENOSPC;
  if (b->payload_bytes > e->cfg.max_batch_bytes) return RMQ_ENOSPC;
  if (b->mem != RMQ_MEM_HOST && b->mem != RMQ_MEM_DEVICE && b->mem != RMQ_MEM_PINNED) return RMQ_EINVAL;
  if (n && (!b->pidx || !b->len || !out_offsets)) return RMQ_EINVAL;
  if (b->payload_bytes && !b->payload) return RMQ_EINVAL;
  if (b->mem == RMQ_MEM_DEVICE && (reinterpret_cast<uintptr_t>(b->payload) & 3u)) return RMQ_EINVAL;
  if (b->mem == RMQ_MEM_HOST) {  // host batches: validate payload ranges like the oracle (EINVAL)
    uint64_t run = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint64_t off = b->payload_off ? b->payload_off[i] : run;
      run += b->len[i];
      if (b->len[i] && (off > b->payload_bytes || b->len[i] > b->payload_bytes - off)) return RMQ_EINVAL;
    }
  }
  HIP_TRY(hipSetDevice(e->device));

  // the ticket is taken only once nothing below can fail short of a device error: the staging
  // slot's wait and the first host batch's allocations come first (with a transport a used-up
  // ticket without a queued batch would leave this rank's groups out of step with its peers')
  const uint64_t t = e->last_ticket + 1;
  // an empty batch still takes its place in a launch group (0 tiles, 0 tasks): every rank of a
  // replication transport forms the same groups from the same number of calls
  InFlight f;
  f.ticket = t;
  f.b.pidx = b->pidx;
  f.b.len = b->len;
  f.b.poff = b->payload_off;
  f.b.payload = b->payload;
  f.b.payload_bytes = b->payload_bytes;
  f.b.out_offsets = out_offsets;
  f.b.n = n;
  f.b.tiles = (n + kTileRecs - 1) / kTileRecs;
  if (b->mem != RMQ_MEM_DEVICE && n) {
    const bool pinned = b->mem == RMQ_MEM_PINNED;
    Staging& sg = e->staging[t % e->staging.size()];
    if (sg.ticket) {  // the batch that used this staging slot must be complete
      int rc = wait_ticket(e, sg.ticket);
      if (rc) return rc;
      collect_done(e);
    }
    const uint64_t NB = e->cfg.max_batch_records, cap = 32ull * NB + e->cfg.max_batch_bytes + 64;
    if (!sg.d_blk)  // the first host batch sets up every slot (allocation synchronizes the device)
      for (Staging& z : e->staging) {
        int rc = dalloc(&z.d_blk, cap);
        if (!rc) rc = dalloc(&z.d_out, NB);
        if (rc) return rc;
        HIP_TRY(hipHostMalloc((void**)&z.h_blk, cap, 0));
        HIP_TRY(hipHostMalloc((void**)&z.h_out, NB * 8, 0));
        HIP_TRY(hipEventCreateWithFlags(&z.ev_in, hipEventDisableTiming));
      }
    const uint64_t o_len = (4ull * n + 15) & ~15ull, o_poff = o_len + ((4ull * n + 15) & ~15ull);
    const uint64_t o_pay = o_poff + (b->payload_off ? (8ull * n + 15) & ~15ull : 0ull);
    if (pinned) {
      // caller-pinned sections: one DMA each straight into the device slot, no host copy
      sg.ticket = t;
      HIP_TRY(hipMemcpyAsync(sg.d_blk, b->pidx, 4ull * n, hipMemcpyHostToDevice, e->copy_s));
      HIP_TRY(hipMemcpyAsync(sg.d_blk + o_len, b->len, 4ull * n, hipMemcpyHostToDevice, e->copy_s));
      if (b->payload_off)
        HIP_TRY(hipMemcpyAsync(sg.d_blk + o_poff, b->payload_off, 8ull * n, hipMemcpyHostToDevice, e->copy_s));
      if (b->payload_bytes)
        HIP_TRY(hipMemcpyAsync(sg.d_blk + o_pay, b->payload, b->payload_bytes, hipMemcpyHostToDevice, e->copy_s));
    } else {
      if (!e->copy_pool) {
        // RMQ_COPY_THREADS: packing threads besides the caller's (default min(7, cores / 2))
        const char* env = std::getenv("RMQ_COPY_THREADS");
        const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
        unsigned k = env ? (unsigned)std::atoi(env) : std::min(7u, hc / 2u);
        e->copy_pool = new (std::nothrow) CopyPool(std::min(k, 64u));
        if (!e->copy_pool) return RMQ_ENOMEM;
      }
      std::vector<CopyPool::Seg> segs = {{sg.h_blk, reinterpret_cast<const uint8_t*>(b->pidx), 4ull * n},
                                         {sg.h_blk + o_len, reinterpret_cast<const uint8_t*>(b->len), 4ull * n}};
      if (b->payload_off) segs.push_back({sg.h_blk + o_poff, reinterpret_cast<const uint8_t*>(b->payload_off), 8ull * n});
      if (b->payload_bytes) segs.push_back({sg.h_blk + o_pay, b->payload, b->payload_bytes});
      sg.ticket = t;
      e->copy_pool->run(segs, 512u << 10);
      HIP_TRY(hipMemcpyAsync(sg.d_blk, sg.h_blk, o_pay + b->payload_bytes, hipMemcpyHostToDevice, e->copy_s));
    }
    HIP_TRY(hipEventRecord(sg.ev_in, e->copy_s));
    HIP_TRY(hipStreamWaitEvent(e->main_s, sg.ev_in, 0));  // before the group's first launch
    if (e->rank_s) HIP_TRY(hipStreamWaitEvent(e->rank_s, sg.ev_in, 0));  // (its ranking, split launches)
    f.b.pidx = reinterpret_cast<const uint32_t*>(sg.d_blk);
    f.b.len = reinterpret_cast<const uint32_t*>(sg.d_blk + o_len);
    f.b.poff = b->payload_off ? reinterpret_cast<const uint64_t*>(sg.d_blk + o_poff) : nullptr;
    f.b.payload = sg.d_blk + o_pay;
    f.b.out_offsets = sg.d_out;
    f.host_out = pinned ? out_offsets : sg.h_out;  // pinned: the DMA writes the caller's array
    sg.user_out = pinned ? nullptr : out_offsets;
    sg.out_n = n;
  }
  e->last_ticket = t;
  *ticket = t;
  e->ticket_n[t % kStatsRing] = n;
  if (e->forming.nb && e->forming.tiles + f.b.tiles > e->max_group_tiles) {  // (never with a transport)
    int rc = close_group(e);
    if (rc) return rc;
  }
  GroupFlight& fg = e->forming;
  if (!fg.nb) fg.set = (uint32_t)(e->groups++ % kSets);
  fg.b[fg.nb++] = f;
  fg.tiles += f.b.tiles;
  fg.tasks += (n + kTaskRecs - 1) / kTaskRecs;
  return fg.nb >= e->group_max ? close_group(e) : RMQ_OK;
}

int rmq_ack(rmq_engine* e, const uint32_t* pidx, const uint32_t* slot, const uint64_t* match, uint32_t n) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (!n) return RMQ_OK;
  if (!pidx || !slot || !match) return RMQ_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    if (pidx[i] >= e->cfg.num_partitions) return RMQ_ENOPART;
    if (slot[i] >= e->cfg.replication_factor) return RMQ_EINVAL;
  }
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  rc = ensure_ctl(e, n);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(e->d_ctl32, pidx, n * 4ull, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_ctl32 + e->ctl_cap, slot, n * 4ull, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_ctl64, match, n * 8ull, hipMemcpyHostToDevice));
  AckArgs a{};
  a.st = e->st;
  a.pidx = e->d_ctl32;
  a.slot = e->d_ctl32 + e->ctl_cap;
  a.match = e->d_ctl64;
  a.n = n;
  launch_ack(a, e->main_s);
  HIP_TRY(hipGetLastError());
  return drain(e);
}

// A consumer-offset ticket (RMQ_TICKET_OFFSETS): are its partitions' rows on a quorum?
int poll_offsets(rmq_engine* e, uint64_t ticket) {
  auto it = std::find_if(e->off_tickets.begin(), e->off_tickets.end(),
                         [ticket](const auto& x) { return x.first == ticket; });
  if (it == e->off_tickets.end()) return RMQ_EINVAL;  // unknown, or resolved already
  int rc = quiesce(e);  // the commit kernels and the ack folds issued so far (no flush)
  if (rc) return rc;
  const size_t P = e->cfg.num_partitions;
  std::vector<uint64_t> cq(P);
  HIP_TRY(hipMemcpy(cq.data(), e->st.cq, P * 8, hipMemcpyDeviceToHost));
  bool done = true, lost = false;
  for (const auto& pv : it->second) {
    if (cq[pv.first] >= pv.second) continue;
    done = false;
    if (!e->is_leader[pv.first]) lost = true;  // leadership moved before its row reached a quorum
  }
  if (!done && !lost) return RMQ_PENDING;
  e->off_tickets.erase(it);
  return done ? RMQ_OK : RMQ_ENOTLEADER;
}

int rmq_poll_commit(rmq_engine* e, uint64_t ticket, uint64_t* commit_out, uint64_t* hw_out) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (ticket & RMQ_TICKET_OFFSETS) {
    HIP_TRY(hipSetDevice(e->device));
    return poll_offsets(e, ticket);
  }
  if (ticket > e->last_ticket) return RMQ_EINVAL;  // never issued
  HIP_TRY(hipSetDevice(e->device));
  if (ticket) {
    int s = ticket_state(e, ticket);
    if (s < 0 && !e->repl) {
      int rc = flush(e);  // a poll pushes the batch through the remaining stages
      if (rc) return rc;
      s = ticket_state(e, ticket);
    }
    if (s <= 0) return RMQ_PENDING;
  }
  int rc = check_err(e);
  if (rc) return rc;
  const size_t P = e->cfg.num_partitions;
  if (commit_out || hw_out) {
    rc = e->repl ? quiesce(e) : drain(e);  // snapshot after everything submitted (applied, with a transport)
    if (rc) return rc;
    if (commit_out) HIP_TRY(hipMemcpy(commit_out, e->st.commit, P * 8, hipMemcpyDeviceToHost));
    if (hw_out) HIP_TRY(hipMemcpy(hw_out, e->st.hw, P * 8, hipMemcpyDeviceToHost));
  }
  return RMQ_OK;
}

int rmq_ticket_stats(rmq_engine* e, uint64_t ticket, rmq_append_stats* out) {
  if (!e || !out) return RMQ_EINVAL;
  EngineLock g(e);
  if (!ticket || ticket > e->last_ticket || e->last_ticket - ticket >= kStatsRing) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = wait_ticket(e, ticket);
  if (rc) return rc;  // RMQ_PENDING with a transport until an rmq_sync applied the ticket
  const uint32_t n = e->ticket_n[ticket % kStatsRing];
  const uint32_t tasks = (n + kTaskRecs - 1) / kTaskRecs;
  std::vector<uint4> ts(tasks ? tasks : 1);
  if (tasks)
    HIP_TRY(hipMemcpy(ts.data(), e->d_stats + (size_t)(ticket % kStatsRing) * e->max_tasks,
                      tasks * sizeof(uint4), hipMemcpyDeviceToHost));
  std::memset(out, 0, sizeof *out);
  out->records = n;
  for (uint32_t k = 0; k < tasks; ++k) {
    out->appended += ts[k].x;
    out->rejected_not_leader += ts[k].y;
    out->rejected_no_partition += ts[k].z;
    out->rejected_no_space += ts[k].w & 0xFFFFu;
    out->rejected_invalid += ts[k].w >> 16;
  }
  return check_err(e);
}

int rmq_sync(rmq_engine* e) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  HIP_TRY(hipSetDevice(e->device));
  return drain(e);
}

int rmq_set_replica_cursor(rmq_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* offset) {
  if (!e || (n && (!pidx || !offset))) return RMQ_EINVAL;
  EngineLock g(e);
  const uint32_t P = e->cfg.num_partitions;
  for (uint32_t i = 0; i < n; ++i)
    if (pidx[i] >= P) return RMQ_ENOPART;
  if (!n) return RMQ_OK;
  HIP_TRY(hipSetDevice(e->device));
  int rc = quiesce(e);  // (fetches on the pipeline stream read and commit the cursors)
  if (rc) return rc;
  std::vector<uint64_t> cur(P);
  HIP_TRY(hipMemcpy(cur.data(), e->st.rcur, P * 8ull, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < n; ++i) cur[pidx[i]] = offset[i];
  HIP_TRY(hipMemcpy(e->st.rcur, cur.data(), P * 8ull, hipMemcpyHostToDevice));
  return RMQ_OK;
}

int rmq_commit_consumer_offset(rmq_engine* e, const uint32_t* pidx, const uint32_t* consumer,
                               const uint64_t* offset, uint32_t n, int32_t* status, uint64_t* ticket) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (ticket) *ticket = 0;
  if (!n) return RMQ_OK;
  if (!pidx || !consumer || !offset) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  // no flush and no wait for the pipeline (it never reads the table): the items go to the device
  // with one copy on the pipeline stream, behind the launches issued so far, from a staging slot
  // whose previous use has completed; a fetch or read-back issued later sees them
  rmq_engine::CommitSlot& cs = e->cslot[e->cslot_next];
  e->cslot_next = (e->cslot_next + 1) % rmq_engine::kCommitSlots;
  if (cs.used) {
    const int rc = event_wait(cs.ev);
    if (rc) return rc;
  }
  cs.used = false;
  if (n > cs.cap) {
    if (cs.h) hipHostFree(cs.h);
    if (cs.d) hipFree(cs.d);
    cs.h = cs.d = nullptr;
    cs.cap = 0;
    const uint32_t cap = std::max<uint32_t>(n, 4096);
    HIP_TRY(hipHostMalloc((void**)&cs.h, 24ull * cap, 0));
    int rc = dalloc(&cs.d, 24ull * cap);
    if (rc) return rc;
    if (!cs.ev) HIP_TRY(hipEventCreateWithFlags(&cs.ev, hipEventDisableTiming));
    cs.cap = cap;
  }
  // ONE pass from the last item back, straight into the staging slot: the per-item checks, last
  // writer wins (PartitionStateMachine.java:71-77: only the last item per (partition, consumer) is
  // kept, so the device scatter has no two writers to one slot; a generation stamp per slot instead
  // of a hash set), and the new row version of every partition the call commits to (one per call)
  // with the ticket's (partition, version) pairs. The kept items end up at [k, n) in call order.
  const size_t slots = (size_t)e->cfg.num_partitions * e->cfg.max_consumers;
  if (e->lww_stamp.size() != slots) {
    e->lww_stamp.assign(slots, 0u);
    e->lww_gen = 0;
  }
  if (++e->lww_gen == 0) {  // wrapped: stale stamps could alias the new generation
    std::fill(e->lww_stamp.begin(), e->lww_stamp.end(), 0u);
    e->lww_gen = 1;
  }
  if (e->cstamp.size() != e->cfg.num_partitions) {
    e->cstamp.assign(e->cfg.num_partitions, 0u);
    e->cstamp_gen = 0;
  }
  if (++e->cstamp_gen == 0) {
    std::fill(e->cstamp.begin(), e->cstamp.end(), 0u);
    e->cstamp_gen = 1;
  }
  const uint32_t gen = e->lww_gen, cgen = e->cstamp_gen, C = e->cfg.max_consumers;
  uint32_t* const hp = reinterpret_cast<uint32_t*>(cs.h);
  uint32_t* const hc = reinterpret_cast<uint32_t*>(cs.h + 4ull * cs.cap);
  uint64_t* const ho = reinterpret_cast<uint64_t*>(cs.h + 8ull * cs.cap);
  uint64_t* const hv = reinterpret_cast<uint64_t*>(cs.h + 16ull * cs.cap);
  std::vector<std::pair<uint32_t, uint64_t>> tv;
  int rc_all = RMQ_OK;
  uint32_t k = n;
  for (uint32_t i = n; i-- > 0;) {
    const uint32_t p = pidx[i], c = consumer[i];
    int st = RMQ_OK;
    if (p >= e->cfg.num_partitions)
      st = RMQ_ENOPART;
    else if (!e->is_leader[p])
      st = RMQ_ENOTLEADER;
    else if (c >= C)
      st = RMQ_EINVAL;
    if (status) status[i] = st;
    if (st) {
      rc_all = st;  // scanning back, the last one set is the first failing item in call order
      continue;
    }
    uint32_t& sl = e->lww_stamp[(size_t)p * C + c];
    if (sl == gen) continue;  // a later item of the call wins
    sl = gen;
    if (e->cstamp[p] != cgen) {  // the partition's first kept item
      e->cstamp[p] = cgen;
      tv.emplace_back(p, ++e->cver[p]);
    }
    --k;
    hp[k] = p;
    hc[k] = c;
    ho[k] = offset[i];
    hv[k] = e->cver[p];
  }
  const uint32_t m = n - k;
  if (!m) return rc_all;
  HIP_TRY(hipMemcpyAsync(cs.d, cs.h, 24ull * cs.cap, hipMemcpyHostToDevice, e->main_s));
  ConsumerCommitArgs a{};
  a.st = e->st;
  a.pidx = reinterpret_cast<const uint32_t*>(cs.d) + k;
  a.consumer = reinterpret_cast<const uint32_t*>(cs.d + 4ull * cs.cap) + k;
  a.offset = reinterpret_cast<const uint64_t*>(cs.d + 8ull * cs.cap) + k;
  a.ver = reinterpret_cast<const uint64_t*>(cs.d + 16ull * cs.cap) + k;
  a.n = m;
  launch_consumer_commit(a, e->main_s);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(cs.ev, e->main_s));
  cs.used = true;
  if (ticket) {
    *ticket = RMQ_TICKET_OFFSETS | ++e->off_ticket_seq;
    e->off_tickets.emplace_back(*ticket, std::move(tv));
    while (e->off_tickets.size() > rmq_engine::kMaxOffsetTickets) e->off_tickets.pop_front();  // never polled
  }
  const int rc = check_err(e);
  return rc ? rc : rc_all;
}

namespace {

// Scratch of a fetch slot for n requests and, for a host output, out_cap bytes of device staging.
// Plain hipMalloc (no zeroing, no device synchronisation: a slot first used while the pipeline
// runs must not wait for it; every word a fetch reads is written by it first).
int fetch_alloc(void** p, size_t bytes) {
  *p = nullptr;
  HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 16)));
  return RMQ_OK;
}

int fetch_slot_reserve(rmq_engine::FetchSlot& f, uint32_t n, uint64_t stage, hipStream_t s) {
  if (n > f.cap) {
    void* ds[] = {f.d_req, f.d_res, f.d_aux, f.d_cpre, f.d_csum};
    for (void* p : ds)
      if (p) hipFree(p);
    if (f.h_req) hipHostFree(f.h_req);
    if (f.h_res) hipHostFree(f.h_res);
    f.d_req = f.d_cpre = f.h_req = nullptr;
    f.d_res = f.d_aux = f.d_csum = f.h_res = nullptr;
    f.cap = 0;
    const uint32_t cap = std::max<uint32_t>(n, 1024);
    int rc = fetch_alloc((void**)&f.d_req, (size_t)cap * 16);
    if (!rc) rc = fetch_alloc((void**)&f.d_res, ((size_t)cap * 4 + 2) * 8);
    if (!rc) rc = fetch_alloc((void**)&f.d_aux, (size_t)cap * 16);
    if (!rc) rc = fetch_alloc((void**)&f.d_cpre, ((size_t)cap + 4) * 4);
    const uint32_t lines = cap / kFetchChunk + 2;
    if (!rc) rc = fetch_alloc((void**)&f.d_csum, 2ull * lines * kCsumStride * 8);
    if (rc) return rc;
    // both halves start zeroed (stream-ordered before the slot's first fetch)
    HIP_TRY(hipMemsetAsync(f.d_csum, 0, 2ull * lines * kCsumStride * 8, s));
    f.csum_lines = lines;
    f.csum_par = 0;
    HIP_TRY(hipHostMalloc((void**)&f.h_req, (size_t)cap * 16, 0));
    HIP_TRY(hipHostMalloc((void**)&f.h_res, ((size_t)cap * 4 + 2) * 8, 0));  // res, bytes needed
    f.cap = cap;
  }
  if (stage > f.out_alloc) {
    if (f.d_out) hipFree(f.d_out);
    f.d_out = nullptr;
    f.out_alloc = 0;
    const int rc = fetch_alloc((void**)&f.d_out, stage);
    if (rc) return rc;
    f.out_alloc = stage;
  }
  return RMQ_OK;
}

// Advance the fetch in slot f (fetch_mu held): RMQ_PENDING while its kernels or host copies run
// (wait: block instead); else its result, with the caller's res (and host output) filled and the
// slot idle again.
int fetch_slot_step(rmq_engine* e, rmq_engine::FetchSlot& f, bool wait, uint64_t* bytes_used) {
  if (f.phase == 1) {
    std::lock_guard<std::mutex> g(e->mu);  // a held-back ticket is launched (with the others held) when polled
    if (f.pending) {
      const int rc = fetch_flush(e);
      if (rc) return rc;
    }
  }
  if (f.phase == 1) {
    if (wait) {
      const int rc = event_wait(f.ev);
      if (rc) return rc;
    } else {
      const hipError_t q = hipEventQuery(f.ev);
      if (q == hipErrorNotReady) return RMQ_PENDING;
      HIP_TRY(q);
    }
    // the device writes rmq_fetch_res rows (status zero-extended into its reserved word)
    static_assert(sizeof(rmq_fetch_res) == 32, "result rows are four words");
    if (!f.rows_pinned) std::memcpy(f.res, f.h_res, (size_t)f.n * 32);  // (pinned: written in place)
    // some request did not fit iff the bytes needed exceed the output (requests are placed in
    // order: the one holding byte out_cap is cut), so no pass over the rows
    f.rc = __atomic_load_n(f.need, __ATOMIC_ACQUIRE) > f.out_cap ? RMQ_ENOSPC : RMQ_OK;
    f.phase = 2;
    if (f.mem == RMQ_MEM_HOST && f.out_cap) {
      // copy back the byte runs of the served requests only: the regions of requests that did not
      // fit stay untouched in the caller's buffer, as with a device buffer the gather writes itself
      uint64_t lo = 0, hi = 0;
      for (uint32_t r = 0; r <= f.n; ++r) {
        const bool served = r < f.n && f.res[r].status == RMQ_OK && f.res[r].bytes;
        if (served && f.res[r].out_pos == hi && hi > lo) {
          hi += f.res[r].bytes;
          continue;
        }
        if (hi > lo) HIP_TRY(hipMemcpyAsync(f.out + lo, f.d_out + lo, hi - lo, hipMemcpyDeviceToHost, e->fetch_out_s));
        lo = hi = served ? f.res[r].out_pos : 0;
        if (served) hi += f.res[r].bytes;
      }
      HIP_TRY(hipEventRecord(f.ev_copy, e->fetch_out_s));
    } else {
      f.phase = 3;  // nothing to copy
    }
  }
  if (f.phase == 2) {
    if (wait) {
      const int rc = event_wait(f.ev_copy);
      if (rc) return rc;
    } else {
      const hipError_t q = hipEventQuery(f.ev_copy);
      if (q == hipErrorNotReady) return RMQ_PENDING;
      HIP_TRY(q);
    }
  }
  if (bytes_used) *bytes_used = __atomic_load_n(f.need, __ATOMIC_ACQUIRE);
  f.phase = 0;
  f.ticket = 0;
  return f.rc;
}

}  // namespace

namespace {
// Issue a fetch into the next slot: its kernels on the pipeline stream, an event after them.
int fetch_issue(rmq_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint32_t mem, uint8_t* out,
                uint64_t out_cap, rmq_fetch_res* res, uint64_t* ticket, bool sync) {
  if (!e || !ticket) return RMQ_EINVAL;
  bool rows_pinned = (mem & RMQ_FETCH_PINNED_ROWS) != 0;
  const bool rows_dev = (mem & RMQ_FETCH_DEVICE_ROWS) != 0;
  mem &= ~(RMQ_FETCH_PINNED_ROWS | RMQ_FETCH_DEVICE_ROWS);
  if (rows_dev && (rows_pinned || mem != RMQ_MEM_DEVICE)) return RMQ_EINVAL;  // (output on the device too)
  if ((n && (!reqs || !res)) || (mem != RMQ_MEM_HOST && mem != RMQ_MEM_DEVICE)) return RMQ_EINVAL;
  if (out_cap && !out) return RMQ_EINVAL;
  if (mem == RMQ_MEM_DEVICE && (reinterpret_cast<uintptr_t>(out) & 15u)) return RMQ_EINVAL;
  std::lock_guard<std::mutex> fg(e->fetch_mu);
  HIP_TRY(hipSetDevice(e->device));
  rmq_engine::FetchSlot& f = e->fslot[e->fslot_next];
  if (f.ticket) {  // every slot taken: complete the oldest into its caller's arrays, keep its result
    uint64_t used = 0;
    const uint64_t old = f.ticket;
    const int rc = fetch_slot_step(e, f, true, &used);
    if (rc < 0 && rc != RMQ_ENOSPC) return rc;
    e->fetch_done.push_back({old, (uint64_t)(int64_t)rc, used});
  }
  // RMQ_FETCH_COMMIT: known flags only, one committing request per (partition, consumer)
  bool any = false, replica = false;
  if (!rows_dev) {  // (device rows: never read here; their flags are ignored)
    // the OR of every row's flags word (the high half of its second 8-byte word), four rows per
    // step with no early exit: 16,384 rows in a few us instead of a branch per row
    static_assert(sizeof(rmq_fetch_req) == 16 && offsetof(rmq_fetch_req, flags) == 12, "request rows are four words");
    typedef uint64_t __attribute__((__may_alias__)) u64a;
    const u64a* w = reinterpret_cast<const u64a*>(reqs);
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint32_t r = 0;
    for (; r + 4 <= n; r += 4) {
      a0 |= w[2 * r + 1];
      a1 |= w[2 * r + 3];
      a2 |= w[2 * r + 5];
      a3 |= w[2 * r + 7];
    }
    for (; r < n; ++r) a0 |= w[2 * r + 1];
    const uint32_t fl = (uint32_t)((a0 | a1 | a2 | a3) >> 32);
    if (fl & ~(RMQ_FETCH_COMMIT | RMQ_FETCH_REPLICA)) return RMQ_EINVAL;
    any = (fl & RMQ_FETCH_COMMIT) != 0;
    replica = (fl & RMQ_FETCH_REPLICA) != 0;
    if (any) {
      const size_t slots = (size_t)e->cfg.num_partitions * e->cfg.max_consumers;
      if (e->fetch_stamp.size() != slots) {
        e->fetch_stamp.assign(slots, 0u);
        e->fetch_stamp_rep.assign(e->cfg.num_partitions, 0u);
        e->fetch_gen = 0;
      }
      if (++e->fetch_gen == 0) {
        std::fill(e->fetch_stamp.begin(), e->fetch_stamp.end(), 0u);
        std::fill(e->fetch_stamp_rep.begin(), e->fetch_stamp_rep.end(), 0u);
        e->fetch_gen = 1;
      }
      for (uint32_t r = 0; r < n; ++r) {
        const rmq_fetch_req& q = reqs[r];
        if (!(q.flags & RMQ_FETCH_COMMIT) || q.pidx >= e->cfg.num_partitions || q.consumer >= e->cfg.max_consumers)
          continue;
        // a replica read commits the partition's replica cursor: one per partition (any consumer key)
        uint32_t& sl = (q.flags & RMQ_FETCH_REPLICA) ? e->fetch_stamp_rep[q.pidx]
                                                     : e->fetch_stamp[(size_t)q.pidx * e->cfg.max_consumers + q.consumer];
        if (sl == e->fetch_gen) return RMQ_EINVAL;
        sl = e->fetch_gen;
      }
    }
  }
  const uint64_t tk = ++e->fetch_seq;
  if (!n) {  // nothing to fetch: complete at once
    e->fetch_done.push_back({tk, (uint64_t)(int64_t)RMQ_OK, 0});
    while (e->fetch_done.size() > 256) e->fetch_done.pop_front();
    *ticket = tk;
    return RMQ_OK;
  }
  int rc = fetch_slot_reserve(f, n, mem == RMQ_MEM_HOST ? out_cap : 0, e->main_s);
  if (rc) return rc;
  uint8_t* d_out = mem == RMQ_MEM_HOST ? (out_cap ? f.d_out : nullptr) : out;
  // Host rows are page-locked: the caller's own (RMQ_FETCH_PINNED_ROWS, if the runtime maps them),
  // else the slot's staging rows. The kernels read and write them in place across PCIe (no copy
  // either way: the lowest latency for one call), or (RMQ_FETCH_DMA, asynchronous calls by
  // default) the request rows go to the slot's device rows by DMA on the copy stream and the
  // result rows come back by DMA on the result stream, so the kernels touch device memory only
  // and a burst's copies overlap the other fetches' kernels.
  void* d_rq = nullptr;
  void* d_rs = nullptr;
  if (rows_dev) {
    d_rq = const_cast<rmq_fetch_req*>(reqs);
    d_rs = res;
  } else if (rows_pinned && (hipHostGetDevicePointer(&d_rq, const_cast<rmq_fetch_req*>(reqs), 0) != hipSuccess ||
                      hipHostGetDevicePointer(&d_rs, res, 0) != hipSuccess)) {
    (void)hipGetLastError();
    rows_pinned = false;  // not mapped: staged like ordinary rows
  }
  if (!rows_pinned && !rows_dev) {
    std::memcpy(f.h_req, reqs, (size_t)n * sizeof(rmq_fetch_req));
    d_rq = f.h_req;
    d_rs = f.h_res;
  }
  const bool dma = !rows_dev && (e->fetch_dma >= 2 || (e->fetch_dma == 1 && !sync));
  void* h_rs = rows_pinned ? static_cast<void*>(res) : static_cast<void*>(f.h_res);  // (DMA) result rows' host copy
  const bool dma_in = dma && e->fetch_dma_in;
  if (dma_in) {
    HIP_TRY(hipMemcpyAsync(f.d_req, rows_pinned ? static_cast<const void*>(reqs) : static_cast<const void*>(f.h_req),
                           (size_t)n * sizeof(rmq_fetch_req), hipMemcpyHostToDevice, e->copy_s));
    HIP_TRY(hipEventRecord(f.ev_in, e->copy_s));
    d_rq = f.d_req;
  }
  if (dma) d_rs = f.d_res;  // (the gather reads a request's resolve words, then writes its final row there)
  {
    // Order against the append pipeline without flushing it: on the pipeline's stream, after the
    // last launch issued so far and before the next, so no ring bytes or log starts it reads change
    // under it.
    std::lock_guard<std::mutex> g(e->mu);  // (not EngineLock: this decides about the held-back fetches)
    // an asynchronous fetch that commits nothing waits to go with the next ones (up to kFetchBatch
    // tickets in one resolve + gather pair: the requests of different tickets never depend on one
    // another); anything else launches the held ones first, then itself
    const bool hold = !sync && !any && !dma && !e->profile && e->fetch_coalesce > 1;
    if (!hold) {
      rc = fetch_flush(e);
      if (rc) return rc;
    }
    if (dma_in) HIP_TRY(hipStreamWaitEvent(e->main_s, f.ev_in, 0));
    if (!hold) {
      rc = late_retention(e);  // (the log starts the fetch reads: every batch applied so far retained)
      if (rc) return rc;
    }
    FetchArgs a{};
    a.st = e->st;
    a.req = static_cast<const uint32_t*>(d_rq);
    a.req_dev = f.d_req;
    a.res = f.d_res;
    a.res_host = static_cast<uint64_t*>(d_rs);
    a.aux = f.d_aux;
    a.cpre = f.d_cpre;
    a.csum_lines = f.csum_lines;
    a.out = d_out;
    a.out_cap = out_cap;
    a.need_host = f.need_dev;
    a.n = n;
    a.commits = any ? 1u : 0u;
    a.replica = replica ? 1u : 0u;
    if (hold) {
      const size_t half = (size_t)f.csum_lines * kCsumStride;
      a.csum = f.d_csum + half * f.csum_par;
      a.csum_next = f.d_csum + half * (f.csum_par ^ 1u);
      f.csum_par ^= 1u;
      f.args = a;
      f.pending = true;
      e->fpend.push_back(e->fslot_next);
      if (e->fpend.size() >= std::min<uint32_t>(kFetchBatch, e->fetch_coalesce)) {
        rc = fetch_flush(e);
        if (rc) return rc;
      }
    }
    hipEvent_t ev[4] = {}, r0 = nullptr, r1 = nullptr;
    // (profiling replays a fetch's kernels back to back; a committing fetch runs once: each run
    // would commit again and the next would read from the committed offset)
    const uint32_t runs = hold ? 0u : e->profile && !any ? e->fetch_replay : 1u;
    // (a committing fetch records no dispatch spans: the events the kernels' own dispatches record
    // were measured to hold the second kernel ~10 us behind the first, which its one run would carry)
    const bool spans = e->profile && !any;
    if (e->profile) {  // kernel 3: the first run's dispatch spans; 4: every run
      if (spans) {
        for (hipEvent_t& x : ev) x = pool_event(e);
        for (int k = 0; k < 2; ++k) e->prof[3].push_back({ev[2 * k], ev[2 * k + 1]});
      }
      r0 = pool_event(e);
      r1 = pool_event(e);
      e->prof[4].push_back({r0, r1});
      e->prof_fetch_runs += runs;
      HIP_TRY(hipEventRecord(r0, e->main_s));
    }
    for (uint32_t k = 0; k < runs; ++k) {
      const size_t half = (size_t)f.csum_lines * kCsumStride;
      a.csum = f.d_csum + half * f.csum_par;
      a.csum_next = f.d_csum + half * (f.csum_par ^ 1u);
      f.csum_par ^= 1u;
      launch_fetch(a, e->main_s, spans && k == 0 ? ev : nullptr);
      HIP_TRY(hipGetLastError());
    }
    if (e->profile) HIP_TRY(hipEventRecord(r1, e->main_s));
    if (hold) {
      // (the completion event: recorded when fetch_flush launches the kernels)
    } else if (dma) {  // the result rows to the host behind the kernels, off the pipeline stream
      HIP_TRY(hipEventRecord(f.ev_k, e->main_s));
      HIP_TRY(hipStreamWaitEvent(e->fetch_out_s, f.ev_k, 0));
      HIP_TRY(hipMemcpyAsync(h_rs, f.d_res, (size_t)n * sizeof(rmq_fetch_res), hipMemcpyDeviceToHost, e->fetch_out_s));
      HIP_TRY(hipEventRecord(f.ev, e->fetch_out_s));
    } else {
      HIP_TRY(hipEventRecord(f.ev, e->main_s));  // kernels done: result rows and bytes needed in place
    }
  }
  f.rows_pinned = rows_pinned || rows_dev;  // (no copy of the rows at completion)
  f.ticket = tk;
  f.phase = 1;
  f.rc = RMQ_OK;
  f.n = n;
  f.mem = mem;
  f.out = out;
  f.out_cap = out_cap;
  f.res = res;
  e->fslot_next = (e->fslot_next + 1) % rmq_engine::kFetchSlots;
  while (e->fetch_done.size() > 256) e->fetch_done.pop_front();
  *ticket = tk;
  return RMQ_OK;
}

}  // namespace

int rmq_fetch_async(rmq_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint32_t mem, uint8_t* out,
                    uint64_t out_cap, rmq_fetch_res* res, uint64_t* ticket) {
  return fetch_issue(e, reqs, n, mem, out, out_cap, res, ticket, false);
}

int rmq_fetch_poll(rmq_engine* e, uint64_t ticket, uint32_t wait, uint64_t* bytes_used) {
  if (!e || !ticket) return RMQ_EINVAL;
  std::lock_guard<std::mutex> fg(e->fetch_mu);
  if (bytes_used) *bytes_used = 0;
  for (rmq_engine::FetchSlot& f : e->fslot)
    if (f.ticket == ticket) {
      HIP_TRY(hipSetDevice(e->device));
      return fetch_slot_step(e, f, wait != 0, bytes_used);
    }
  for (auto it = e->fetch_done.begin(); it != e->fetch_done.end(); ++it)
    if ((*it)[0] == ticket) {
      const int rc = (int)(int64_t)(*it)[1];
      if (bytes_used) *bytes_used = (*it)[2];
      e->fetch_done.erase(it);
      return rc;
    }
  return RMQ_EINVAL;
}

int rmq_fetch(rmq_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint32_t mem, uint8_t* out,
              uint64_t out_cap, rmq_fetch_res* res, uint64_t* bytes_used) {
  if (bytes_used) *bytes_used = 0;
  if (!e) return RMQ_EINVAL;
  if (!n) return RMQ_OK;
  uint64_t t = 0;
  const int rc = fetch_issue(e, reqs, n, mem, out, out_cap, res, &t, true);
  if (rc) return rc;
  return rmq_fetch_poll(e, t, 1, bytes_used);
}

int rmq_get_partition_state(rmq_engine* e, uint32_t p, rmq_partition_state* o) {
  if (!e || !o) return RMQ_EINVAL;
  EngineLock g(e);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  HIP_TRY(hipSetDevice(e->device));
  int rc = quiesce(e);
  if (rc) return rc;
  const DevState& s = e->st;
  const uint32_t RF = e->cfg.replication_factor;
  std::memset(o, 0, sizeof *o);
  HIP_TRY(hipMemcpy(&o->log_end_offset, s.leo + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->log_end_pos, s.used + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->log_start_offset, s.start_off + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->log_start_pos, s.start_pos + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->commit, s.commit + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->high_watermark, s.hw + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->term_start, s.term_start + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(o->match, s.match + (size_t)p * RF, RF * 8ull, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->term, s.term + p, 8, hipMemcpyDeviceToHost));
  for (uint32_t r = 0; r < RF; ++r) o->replica_rank[r] = e->ranks[(size_t)p * RF + r];
  o->leader_slot = e->leader_slot[p];
  o->is_leader = e->is_leader[p];
  o->segment_bytes = 1ull << (e->ring[p] & 63ull);
  if (o->is_leader) o->leader_commit = o->commit;
  else HIP_TRY(hipMemcpy(&o->leader_commit, s.lcommit + p, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&o->last_log_term, s.lterm + p, 8, hipMemcpyDeviceToHost));
  if (o->last_log_term & kLtermBound) o->last_log_term = 0;  // unknown: a candidate claims none
  HIP_TRY(hipMemcpy(&o->heard_round, s.heard + p, 8, hipMemcpyDeviceToHost));
  o->voted_term = e->vterm[p];
  o->voted_for = e->vfor[p];
  o->led = e->vled[p];
  return RMQ_OK;
}

int rmq_get_partition_states(rmq_engine* e, uint32_t first, uint32_t n, rmq_partition_state* o) {
  if (!e || (n && !o)) return RMQ_EINVAL;
  EngineLock g(e);
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  if (first > P || n > P - first) return RMQ_ENOPART;
  if (!n) return RMQ_OK;
  HIP_TRY(hipSetDevice(e->device));
  int rc = quiesce(e);
  if (rc) return rc;
  const DevState& s = e->st;
  uint64_t* const src[] = {s.leo, s.used, s.start_off, s.start_pos, s.commit, s.hw, s.term, s.term_start, s.lcommit,
                           s.lterm, s.heard};
  constexpr int NF = sizeof src / sizeof src[0];
  // every field gathered by one kernel into a page-locked staging area, one wait (12 synchronous
  // copies into pageable vectors took 0.86 ms for 4,096 partitions)
  const size_t words = (size_t)P * (NF + RF);
  if (e->state_stage_words < words) {
    if (e->state_stage) hipHostFree(e->state_stage);
    e->state_stage = nullptr;
    e->state_stage_words = 0;
    HIP_TRY(hipHostMalloc((void**)&e->state_stage, words * 8, 0));
    e->state_stage_words = words;
  }
  uint64_t* const v = e->state_stage;
  uint64_t* const m = v + (size_t)n * NF;
  static_assert(NF == 11, "state_gather_kernel's fields");
  (void)src;
  launch_state_gather(s, v, first, n, RF, e->main_s);  // (page-locked: the kernel writes it in place)
  HIP_TRY(hipGetLastError());
  rc = stream_wait(e->main_s);
  if (rc) return rc;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t p = first + i;
    rmq_partition_state& x = o[i];
    std::memset(&x, 0, sizeof x);
    x.log_end_offset = v[i];
    x.log_end_pos = v[(size_t)n + i];
    x.log_start_offset = v[2ull * n + i];
    x.log_start_pos = v[3ull * n + i];
    x.commit = v[4ull * n + i];
    x.high_watermark = v[5ull * n + i];
    x.term = v[6ull * n + i];
    x.term_start = v[7ull * n + i];
    for (uint32_t r = 0; r < RF; ++r) {
      x.match[r] = m[(size_t)i * RF + r];
      x.replica_rank[r] = e->ranks[(size_t)p * RF + r];
    }
    x.leader_slot = e->leader_slot[p];
    x.is_leader = e->is_leader[p];
    x.segment_bytes = 1ull << (e->ring[p] & 63ull);
    x.leader_commit = x.is_leader ? x.commit : v[8ull * n + i];
    x.last_log_term = (v[9ull * n + i] & kLtermBound) ? 0ull : v[9ull * n + i];
    x.heard_round = v[10ull * n + i];
    x.voted_term = e->vterm[p];
    x.voted_for = e->vfor[p];
    x.led = e->vled[p];
  }
  return RMQ_OK;
}

int rmq_read_segment(rmq_engine* e, uint32_t replica, uint32_t p, uint64_t ring_off, uint64_t len, uint8_t* out) {
  if (!e || (len && !out)) return RMQ_EINVAL;
  EngineLock g(e);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  const RingRef rg = ring_ref(e->ring[p], e->st.interval_log2, e->st.icap_mul);
  if (replica >= e->cfg.replication_factor || ring_off > rg.seg || len > rg.seg - ring_off) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = quiesce(e);
  if (rc) return rc;
  if (len)
    HIP_TRY(hipMemcpy(out, e->st.logs + (uint64_t)replica * e->st.rstride + rg.base + ring_off, len,
                      hipMemcpyDeviceToHost));
  return RMQ_OK;
}

int rmq_read_index(rmq_engine* e, uint32_t p, uint64_t m_first, uint64_t count, uint64_t* out) {
  if (!e || (count && !out)) return RMQ_EINVAL;
  EngineLock g(e);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  const RingRef rg = ring_ref(e->ring[p], e->st.interval_log2, e->st.icap_mul);
  const uint32_t icap = rg.icap;
  if (count > icap) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = quiesce(e);
  if (rc) return rc;
  std::vector<uint64_t> ring((size_t)icap * 2);
  HIP_TRY(hipMemcpy(ring.data(), e->st.index + rg.ibase * 2, ring.size() * 8, hipMemcpyDeviceToHost));
  for (uint64_t k = 0; k < count; ++k) {
    const uint64_t sl = (m_first + k) % icap;
    out[2 * k] = ring[2 * sl];
    out[2 * k + 1] = ring[2 * sl + 1];
  }
  return RMQ_OK;
}

int rmq_read_consumer_offsets(rmq_engine* e, uint32_t p, uint64_t* out) {
  if (!e || !out) return RMQ_EINVAL;
  EngineLock g(e);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  HIP_TRY(hipSetDevice(e->device));
  int rc = quiesce(e);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(out, e->st.cons + (size_t)p * e->cfg.max_consumers, e->cfg.max_consumers * 8ull,
                    hipMemcpyDeviceToHost));
  return RMQ_OK;
}

int rmq_read_consumer_table(rmq_engine* e, uint32_t first, uint32_t n, uint64_t* out) {
  if (!e || (n && !out)) return RMQ_EINVAL;
  EngineLock g(e);
  if (first > e->cfg.num_partitions || n > e->cfg.num_partitions - first) return RMQ_ENOPART;
  if (!n) return RMQ_OK;
  HIP_TRY(hipSetDevice(e->device));
  int rc = quiesce(e);
  if (rc) return rc;
  const size_t C = e->cfg.max_consumers;
  HIP_TRY(hipMemcpy(out, e->st.cons + (size_t)first * C, (size_t)n * C * 8, hipMemcpyDeviceToHost));
  return RMQ_OK;
}

int rmq_device_alloc(rmq_engine* e, uint64_t bytes, void** out) {
  if (!e || !out) return RMQ_EINVAL;
  EngineLock g(e);
  HIP_TRY(hipSetDevice(e->device));
  *out = nullptr;
  HIP_TRY(hipMalloc(out, bytes ? bytes : 1));
  return RMQ_OK;
}

int rmq_device_free(rmq_engine* e, void* p) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  HIP_TRY(hipSetDevice(e->device));
  int rc = settle(e);
  if (rc) return rc;
  if (p) HIP_TRY(hipFree(p));
  return RMQ_OK;
}

int rmq_memcpy(rmq_engine* e, void* dst, const void* src, uint64_t bytes, int kind) {
  if (!e || (bytes && (!dst || !src))) return RMQ_EINVAL;
  EngineLock g(e);
  HIP_TRY(hipSetDevice(e->device));
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                        : kind == 1 ? hipMemcpyDeviceToHost
                                    : hipMemcpyDeviceToDevice;
  int rc = settle(e);
  if (rc) return rc;
  if (bytes) HIP_TRY(hipMemcpy(dst, src, bytes, k));
  return RMQ_OK;
}

int rmq_profile_enable(rmq_engine* e, int enable) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  HIP_TRY(hipSetDevice(e->device));
  int rc = settle(e);
  if (rc) return rc;
  for (auto& v : e->prof) {
    for (EvPair& p : v) {
      e->ev_pool.push_back(p.a);
      e->ev_pool.push_back(p.b);
    }
    v.clear();
  }
  e->profile = enable > 0 ? 1u : 0u;
  e->fetch_replay = enable > 1 ? (uint32_t)enable : 1u;
  e->prof_launches = e->prof_batches = e->prof_fetch_runs = 0;
  e->prof_started = e->prof_ended = false;
  if (e->profile && !e->prof_t0) {
    HIP_TRY(hipEventCreate(&e->prof_t0));
    HIP_TRY(hipEventCreate(&e->prof_t1));
  }
  return RMQ_OK;
}

int rmq_profile_query(rmq_engine* e, int kernel, uint64_t* launches, double* total_ms) {
  if (!e || kernel < 0 || kernel > 4) return RMQ_EINVAL;
  EngineLock g(e);
  HIP_TRY(hipSetDevice(e->device));
  int rc = settle(e);
  if (rc) return rc;
  if (kernel <= 1) {  // 0: pipeline launches in the region, 1: batches applied in it
    float ms = 0;
    if (e->prof_ended) HIP_TRY(hipEventElapsedTime(&ms, e->prof_t0, e->prof_t1));
    if (launches) *launches = e->prof_ended ? (kernel ? e->prof_batches : e->prof_launches) : 0;
    if (total_ms) *total_ms = ms;
    return RMQ_OK;
  }
  double tot = 0;
  for (const EvPair& p : e->prof[kernel]) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
    tot += ms;
  }
  if (launches) *launches = kernel == 4 ? e->prof_fetch_runs : e->prof[kernel].size();
  if (total_ms) *total_ms = tot;
  return RMQ_OK;
}

int rmq_device_info(rmq_engine* e, char* name, uint32_t name_cap, uint32_t* cu_count) {
  if (!e) return RMQ_EINVAL;
  if (name && name_cap) std::snprintf(name, name_cap, "%s", e->dev_name);
  if (cu_count) *cu_count = e->cu_count;
  return RMQ_OK;
}

int rmq_rccl_unique_id(uint8_t* out) {
  if (!out) return RMQ_EINVAL;
  return rccl_unique_id(out);
}

int rmq_attach_rccl(rmq_engine* e, const uint8_t* comm_id, uint32_t world) {
  if (!e || !comm_id || world < 2 || world > kMaxWorld) return RMQ_EINVAL;
  EngineLock g(e);
  if (e->repl) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  Transport* t = make_rccl_transport(comm_id, world, e->cfg.rank);
  if (!t) return RMQ_EDEVICE;
  rc = repl_attach(e, t);
  if (rc && !e->repl) delete t;
  return rc;
}

struct rmq_local_hub {
  rmq::LocalHub hub;
  explicit rmq_local_hub(uint32_t w) : hub(w) {}
};

int rmq_local_hub_create(uint32_t world, rmq_local_hub** out) {
  if (!out || world < 2 || world > kMaxWorld) return RMQ_EINVAL;
  *out = new (std::nothrow) rmq_local_hub(world);
  return *out ? RMQ_OK : RMQ_ENOMEM;
}

void rmq_local_hub_destroy(rmq_local_hub* h) { delete h; }

int rmq_attach_local(rmq_engine* e, rmq_local_hub* h) {
  if (!e || !h) return RMQ_EINVAL;
  EngineLock g(e);
  if (e->repl) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  Transport* t = make_local_transport(&h->hub, e->cfg.rank, e->device);
  rc = repl_attach(e, t);
  if (rc && !e->repl) delete t;
  return rc;
}

int rmq_replication_stats(rmq_engine* e, rmq_repl_stats* out) {
  if (!e || !out) return RMQ_EINVAL;
  EngineLock g(e);
  std::memset(out, 0, sizeof *out);
  if (!e->repl) return RMQ_OK;
  const Replication* r = e->repl;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(r->xchg_s));
  uint64_t c[7];
  HIP_TRY(hipMemcpy(c, r->d_counters, sizeof c, hipMemcpyDeviceToHost));
  out->world = r->world;
  out->rank = r->rank;
  out->out_entries = (uint32_t)r->xo_p.size();
  out->in_entries = (uint32_t)r->xi_p.size();
  out->rounds = r->rounds;
  out->bytes_sent = r->bytes_sent;
  out->bytes_received = r->bytes_recv;
  out->records_ingested = c[0];
  out->refused_crc = c[1];
  out->refused_log = c[2];
  out->bytes_ingested = c[3];
  out->catchup_entries = c[4];
  out->detached_plans = c[5];
  out->general_plans = c[6];
  out->host_waits = r->host_waits;
  out->host_wait_ns = r->host_wait_ns;
  return RMQ_OK;
}

int rmq_fault_drop_rounds(rmq_engine* e, uint32_t n) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (!e->repl) return RMQ_EINVAL;
  e->repl->drop_from = e->last_ticket + 1;
  e->repl->drop_n = n;
  return RMQ_OK;
}

int rmq_fault_cut(rmq_engine* e, uint32_t dst, uint32_t n) {
  int rc = rmq_fault_isolate(e, dst, n);
  if (rc) return rc;
  EngineLock g(e);
  e->repl->cut_notice |= 1u << dst;
  return RMQ_OK;
}

int rmq_fault_isolate(rmq_engine* e, uint32_t dst, uint32_t n) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (!e->repl || dst >= e->repl->world || dst == e->repl->rank) return RMQ_EINVAL;
  e->repl->iso_from[dst] = e->last_ticket + 1;
  e->repl->iso_n[dst] = n;
  return RMQ_OK;
}

int rmq_fault_corrupt(rmq_engine* e, uint32_t dst, int64_t at) {
  if (!e) return RMQ_EINVAL;
  EngineLock g(e);
  if (!e->repl || dst >= e->repl->world || dst == e->repl->rank) return RMQ_EINVAL;
  e->repl->flip[dst] = true;
  e->repl->flip_at[dst] = at;
  return RMQ_OK;
}

int rmq_read_outbox(rmq_engine* e, uint32_t dst, uint8_t* out, uint64_t cap, uint64_t* size) {
  if (!e || !size) return RMQ_EINVAL;
  EngineLock g(e);
  *size = 0;
  Replication* r = e->repl;
  if (!r || dst >= r->world) return RMQ_EINVAL;
  if (r->last_set == ~0u) return RMQ_OK;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(r->xchg_s));
  const XchgSet& x = r->sets[r->last_set];
  const uint64_t off = (uint64_t)dst * r->dcap;  // region d at d * dcap of the outbox
  const uint64_t n = dst == r->rank ? 0 : x.h_sizes[2 * dst];
  *size = n;
  if (!out) return RMQ_OK;
  if (n > cap) return RMQ_ENOSPC;
  if (n) HIP_TRY(hipMemcpy(out, x.outbox + off, n, hipMemcpyDeviceToHost));
  return RMQ_OK;
}

}  // extern "C"
