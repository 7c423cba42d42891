// engine_internal.hpp — the engine object shared by the host-side translation units
// (engine.cpp: C-ABI, append pipeline, fetch, control; replication.cpp: replica-log rounds).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <chrono>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ripplemq_engine.h"
#include "device_common.hpp"
#include "kernels.hpp"
#include "transport.hpp"

using namespace rmq;

namespace rmq {

constexpr uint32_t kStatsRing = 64;                                // tickets whose stats stay readable
constexpr uint32_t kMaxBatchRecords = kMaxTiles * kTileRecs;       // 524288
// pipeline scratch sets: a group's set lives from its stage 1 (launch k) to the application of its
// followers' acks (launch k + 5 with a replication transport), so six sets rotate
constexpr uint32_t kSets = 6;

struct EvPair {
  hipEvent_t a = nullptr, b = nullptr;
};

// Device staging of host-memory batches.
// Host threads that pack a host batch into its pinned staging slot: one memcpy split into chunks
// that the workers and the submitting thread take in turn (a single thread fills pinned memory at
// ~7 GB/s, a quarter of what the DMA behind it moves).
class CopyPool {
 public:
  struct Seg {
    uint8_t* d;
    const uint8_t* s;
    size_t n;
  };
  explicit CopyPool(unsigned workers) {
    for (unsigned i = 0; i < workers; ++i) th_.emplace_back([this] { work(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  // Copy every segment (chunked), using the workers and the calling thread; returns when done.
  void run(const std::vector<Seg>& segs, size_t chunk) {
    chunks_.clear();
    for (const Seg& g : segs)
      for (size_t o = 0; o < g.n; o += chunk) chunks_.push_back({g.d + o, g.s + o, std::min(chunk, g.n - o)});
    if (th_.empty() || chunks_.size() < 2) {
      for (const Seg& c : chunks_) std::memcpy(c.d, c.s, c.n);
      return;
    }
    next_.store(0);
    left_.store(chunks_.size());
    {
      std::lock_guard<std::mutex> g(m_);
      ++gen_;
    }
    cv_.notify_all();
    take();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return left_.load() == 0; });
  }
  unsigned workers() const { return (unsigned)th_.size(); }

 private:
  void take() {
    for (size_t i; (i = next_.fetch_add(1)) < chunks_.size();) {
      std::memcpy(chunks_[i].d, chunks_[i].s, chunks_[i].n);
      if (left_.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> g(m_);
        done_.notify_all();
      }
    }
  }
  void work() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      take();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::vector<Seg> chunks_;
  std::atomic<size_t> next_{0}, left_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// A host batch's slot: the caller's arrays are packed into pinned memory (pidx | len | payload_off |
// payload, 16-byte aligned sections) and cross PCIe as one DMA on the copy stream, which the
// pipeline stream waits for; the out offsets come back into pinned memory and reach the caller's
// buffer when the ticket is seen complete.
struct Staging {
  uint8_t* h_blk = nullptr;    // pinned, packed batch
  uint8_t* d_blk = nullptr;    // device copy
  uint64_t* h_out = nullptr;   // pinned out offsets
  uint64_t* d_out = nullptr;
  hipEvent_t ev_in = nullptr;  // the DMA of the batch is done
  uint64_t ticket = 0;         // last ticket that used it
  uint64_t* user_out = nullptr;  // caller's out_offsets, pending copy-out
  uint32_t out_n = 0;
};

// A batch inside the launch pipeline.
struct InFlight {
  uint64_t ticket = 0;
  PipeBatch b{};
  uint64_t* host_out = nullptr;  // host batches: caller's out_offsets
};

// A group of consecutive batches moving through the pipeline together (one launch per stage).
struct GroupFlight {
  uint32_t nb = 0, tiles = 0, tasks = 0;
  uint32_t set = 0;              // scratch set = group number % kSets
  InFlight b[kMaxGroup];
};

// Replica-log rounds over a transport (replication.cpp, FORMAT.md §9): per scratch set, the
// group's outbox and inbox and the exchange's events.
struct XchgSet {
  uint8_t* outbox = nullptr;   // region for destination d at d * dcap
  uint8_t* inbox = nullptr;    // received regions packed in source order
  XEntry* xe = nullptr;        // [n_out]
  XCatch* xc = nullptr;        // [n_out] catch-up list (plan -> stage-3 catch-up waves)
  uint32_t* xc_n = nullptr;    // [2]
  uint64_t* sizes = nullptr;   // device [4 * world]: send sizes (plan), receive sizes (exchange)
  uint64_t* h_sizes = nullptr; // pinned copy
  uint64_t* ackout = nullptr;  // [n_in][2]
  uint64_t* ackin = nullptr;   // [n_out][2]
  uint64_t* rowv = nullptr;    // [n_out] consumer-offset row version each entry of the round carries
  uint32_t* count = nullptr;   // stage-2 arrival counter
  hipEvent_t ev_s2 = nullptr, ev_s3 = nullptr, ev_sz = nullptr, ev_x = nullptr;
  uint64_t applied_launch = 0; // launch that ran the group's stage 3
  uint64_t round = 0;          // the group's round number (FORMAT.md §9)
};

struct Replication {
  Transport* xport = nullptr;
  uint32_t world = 1, rank = 0;
  hipStream_t xchg_s = nullptr;
  // out list: (led partition, remote slot) grouped by destination, ascending (key, slot);
  // in list: (followed partition, local slot) grouped by source, same order on both sides
  std::vector<uint32_t> xo_p, xo_slot, xo_start, xi_p, xi_slot, xi_start;
  std::vector<uint64_t> keysum;  // [world] of the out lists
  uint32_t* d_xo_p = nullptr;
  uint32_t* d_xo_start = nullptr;
  uint64_t* d_keysum = nullptr;
  uint64_t* d_keysum_in = nullptr;  // [world] key sums of the in lists (the follower's side)
  uint32_t* d_outidx = nullptr;  // [P][RF]
  uint32_t* d_xi_p = nullptr;
  uint32_t* d_xi_slot = nullptr;
  uint32_t* d_xi_start = nullptr;
  uint32_t* d_xo_slot = nullptr;  // [n_out]
  uint32_t* d_bad = nullptr;     // [n_in]
  uint32_t* d_acc = nullptr;     // [n_in]
  uint64_t* d_base = nullptr;    // [n_in][2] IngestArgs::base
  uint64_t* d_cdesc = nullptr;   // [n_in][4] IngestArgs::cdesc
  uint32_t* d_items = nullptr;   // [items_cap][2] follower copy work items
  uint32_t* d_nitems = nullptr;  // [2][1 + kMaxWorld]: copy items allocated, structural flag per source;
                                 // rounds alternate halves, each round's prepare clears the other
  uint32_t nitems_par = 0;
  uint64_t* d_counters = nullptr;  // [7]: follower [0..4) (IngestArgs), leader [4..7) (XPlanArgs)
  uint64_t* d_lastg = nullptr;     // [P] record bytes / 16 of the last group applied (PipeArgs::lastg)
  // leader catch-up state per out entry (FORMAT.md §9 v3)
  uint64_t* d_xnext = nullptr;   // [n_out][2]
  uint64_t* d_xreq = nullptr;    // [n_out][4]
  uint64_t* d_xcu = nullptr;     // [n_out]
  XDecision* d_xdec = nullptr;   // [n_out]
  uint64_t* d_xtot = nullptr;    // [n_out]
  uint32_t* d_dflag = nullptr;   // [world]
  uint64_t* d_nout = nullptr;    // [n_out][2] commit notices sent {commit, term} (FORMAT.md §9 v4)
  uint64_t* d_nin = nullptr;     // [n_in][2] commit notices received
  uint64_t* d_eackv = nullptr;   // [n_out] row version each follower acknowledged (offset tickets)
  hipEvent_t ev_notice = nullptr;
  uint64_t dcap = 0;             // outbox bytes per destination
  uint64_t reserve = 0;          // catch-up bytes per destination
  uint64_t items_cap = 0;
  uint64_t planned = 0;          // rounds planned (the next plan's round number)
  uint64_t out_cap = 0, in_cap = 0;
  XchgSet sets[kSets];
  std::deque<uint32_t> sized;    // sets whose size exchange is posted, data exchange not yet
  std::deque<uint32_t> acking;   // sets whose data exchange is posted, acks not yet applied
  uint64_t rounds = 0, bytes_sent = 0, bytes_recv = 0;
  uint64_t host_waits = 0, host_wait_ns = 0;  // post_round found the sizes not landed yet
  uint32_t last_set = ~0u;       // set of the last posted round (rmq_read_outbox)
  // fault injection (rmq_fault_drop_rounds): the rounds of the next `drop_n` groups whose first
  // ticket is at least `drop_from` send empty regions
  uint64_t drop_from = 0;
  uint32_t drop_n = 0;
  // rmq_fault_isolate: the next iso_n[q] rounds (groups from ticket iso_from[q] on) to q are lost
  uint64_t iso_from[kMaxWorld] = {};
  uint32_t iso_n[kMaxWorld] = {};
  uint32_t cut_notice = 0;      // rmq_fault_cut: bit q, the next drain's commit notices to q are lost
  uint64_t stamp = 0;           // round stamp: the last round posted for ingest, + 1 (heard words)
  std::chrono::steady_clock::time_point stamp_time[64];  // when stamp s was posted, at [s % 64]
  // rmq_fault_corrupt: the next round to destination q flips the byte at flip_at[q]
  bool flip[kMaxWorld] = {};
  int64_t flip_at[kMaxWorld] = {};
};

}  // namespace rmq

namespace rmq {
// Ring space of the pool (FORMAT.md §2): power-of-two blocks aligned to their size, free lists per
// size class, blocks split from larger free ones or cut from the unused tail; no coalescing.
struct SegPool {
  uint64_t size = 0, bump = 0;
  std::vector<uint64_t> free[64];
  void give(uint64_t off, uint64_t end) {  // [off, end) into the free lists as aligned blocks
    while (off < end) {
      uint32_t lg = off ? (uint32_t)__builtin_ctzll(off) : 63u;
      while ((1ull << lg) > end - off) --lg;
      free[lg].push_back(off);
      off += 1ull << lg;
    }
  }
  bool alloc(uint32_t lg, uint64_t* off) {
    for (uint32_t k = lg; k < 64; ++k) {
      if (free[k].empty()) continue;
      const uint64_t o = free[k].back();
      free[k].pop_back();
      for (uint32_t q = k; q > lg; --q) free[q - 1].push_back(o + (1ull << (q - 1)));  // split
      *off = o;
      return true;
    }
    const uint64_t a = (bump + (1ull << lg) - 1) & ~((1ull << lg) - 1);
    if (a + (1ull << lg) > size) return false;
    give(bump, a);
    bump = a + (1ull << lg);
    *off = a;
    return true;
  }
  void release(uint32_t lg, uint64_t off) { free[lg].push_back(off); }
};
}  // namespace rmq

struct rmq_engine {
  rmq_config cfg{};
  std::mutex mu;
  int device = 0;
  uint32_t cu_count = 0;
  uint32_t verify_wgs = 0;  // follower verify grid (RMQ_VERIFY_WGS; default 4 workgroups per CU)
  char dev_name[256] = {0};
  hipStream_t main_s = nullptr;
  DevState st{};            // leo/used point at sets[applied & 1]
  StateSet sets[2]{};
  uint64_t applied = 0;     // stage-3 launches issued
  CrcConsts* d_crc = nullptr;
  uint32_t* d_rlate = nullptr;  // [P] partitions whose retention of the applied group stopped early
  uint4* d_stats = nullptr;  // [kStatsRing][max tasks]
  rmq::SegPool pool;         // ring space of each replica region
  std::vector<uint64_t> ring;  // [P] host copy of DevState::ring
  uint32_t max_tasks = 0;
  uint32_t max_tiles = 0;
  uint32_t key_passes = 0;
  uint32_t key_bits = 0;
  uint32_t rank_mode = 0;  // RMQ_RANK: stage 1 by the LDS radix sort (0) or by hash counters (1;
                           // 4.86 vs 5.14 G msgs/s at config B, profiles/r04c_*)
  uint32_t max_ahead = 0;  // RMQ_AHEAD: pipeline launches queued at most (0: unbounded; a bound of
                           // 4 or 8 cost 4-6 % at config B, profiles/r04i_*: bound it in the app)
  uint32_t steal = 0;      // RMQ_STEAL=1: stage-3 workgroups take stage-1 tiles when out of tasks
  uint32_t prio = 1;  // RMQ_PRIO (round 6 default 1; 0 off): stage-1/2 and partition waves at s_setprio 3
                           // (5.20 -> 4.00 G msgs/s: stage 2 and the second half of stage 3 start later)
  PipeScratch scratch[kSets]{};
  std::vector<Staging> staging;
  CopyPool* copy_pool = nullptr;  // host batches (created with the first one)
  uint32_t big_wgs = 0;           // stage-3 workgroups for records over 1 KB (RMQ_BIG_WGS; 0: 32 waves per CU)
  // pipeline: the group being formed, then groups ranked (need stage 2), scanned (need stage 3)
  // and applied (need stage 4)
  GroupFlight forming, g1, g2, g3;
  bool has1 = false, has2 = false, has3 = false;
  uint64_t g3_seq = 0;
  uint32_t set_reset = 0;  // scratch sets whose large-record list and batch sums the next stage 1 zeroes  // the launch that applied g3 (its retention is late if done_host[1] >= it)
  uint32_t group_max = 2;       // batches per group (cfg.pipeline_depth)
  uint32_t max_group_tiles = 0;
  uint64_t groups = 0;          // groups formed
  uint64_t launch_seq = 0;
  uint64_t* done_host = nullptr;     // pinned: [0] launch k-1 complete, written by launch k;
                                     // [1] the last launch whose retention stopped early
  uint64_t* done_dev = nullptr;
  uint64_t last_ticket = 0;
  std::vector<uint32_t> ticket_n;        // [kStatsRing] records of each recent ticket (stats)
  // completion: tickets are applied in order, launch after launch. marks = {hi, L}: every ticket
  // <= hi not covered by an earlier mark is applied by launch L (empty tickets count with the
  // non-empty one before them); every ticket <= done_ticket is complete.
  std::deque<std::pair<uint64_t, uint64_t>> marks;
  uint64_t done_ticket = 0;
  // host mirrors of control state
  std::vector<uint32_t> is_leader, leader_slot, ranks;  // ranks [P][RF]
  std::vector<uint64_t> term;
  // votes (Raft's votedFor per term, raft_meta): the term of the last vote, the candidate, and whether
  // this replica led that term (rmq_become_leader succeeded in it)
  std::vector<uint64_t> vterm;
  std::vector<uint32_t> vfor, vled;
  std::chrono::steady_clock::time_point place_time = std::chrono::steady_clock::now();  // last placement
  // fetch: its own stream and scratch, serialised by fetch_mu (engine state under mu only while
  // the fetch is ordered against the pipeline stream)
  std::mutex fetch_mu;
  hipStream_t fetch_out_s = nullptr;  // fetch results (and host outputs) -> host, after the kernels:
                                      // a fetch's result copy overlaps the next fetch's kernels
  hipStream_t copy_s = nullptr;  // host batches and fetch requests: pinned -> device DMA
  hipEvent_t ev_main = nullptr;
  bool trace = false;           // RMQ_TRACE: print every launch's roles to stderr
  // fetches in flight (rmq_fetch_async), each with its own scratch: a fetch is ordered after the
  // launches issued before it and before the ones issued after it; the host only waits in
  // rmq_fetch_poll (or when every slot is taken: the oldest is completed into its caller's arrays
  // and its result kept for its poll)
  struct FetchSlot {
    uint32_t* d_req = nullptr;
    uint64_t* d_res = nullptr;
    uint64_t* d_aux = nullptr;
    uint32_t* d_cpre = nullptr;
    uint64_t* d_csum = nullptr;   // two halves of csum_lines lines: a fetch adds into one, its gather
                                  // zeroes the other for the next fetch of the slot (same stream)
    uint32_t csum_lines = 0;
    uint32_t csum_par = 0;
    uint32_t* h_req = nullptr;   // pinned
    uint64_t* h_res = nullptr;   // pinned [cap][4] + {bytes needed, 0}
    uint32_t cap = 0;
    uint8_t* d_out = nullptr;    // device staging of a host output
    uint64_t out_alloc = 0;
    hipEvent_t ev = nullptr;     // its kernels done (result rows and bytes needed in place)
    hipEvent_t ev_copy = nullptr;  // host output copies done
    hipEvent_t ev_in = nullptr;    // (DMA rows) request rows on the device
    hipEvent_t ev_k = nullptr;     // (DMA rows) kernels done: the result rows' copy may start
    bool rows_pinned = false;      // the caller's rows read / written in place (pinned or device rows)
    uint64_t* need = nullptr;      // bytes needed: a word of fetch_need_host (the gather stores it)
    uint64_t* need_dev = nullptr;  // its device address
    // the fetch in flight: ticket 0 = idle; phase 1: kernels, 2: host output copies
    uint64_t ticket = 0;
    int phase = 0;
    int rc = 0;
    uint32_t n = 0, mem = 0;
    uint8_t* out = nullptr;
    uint64_t out_cap = 0;
    rmq_fetch_res* res = nullptr;
    bool pending = false;  // its kernels held back to go with the next asynchronous fetches (fetch_flush)
    FetchArgs args{};      //   and their arguments
  };
  static constexpr uint32_t kFetchSlots = 4;
  FetchSlot fslot[kFetchSlots];
  uint32_t fslot_next = 0;
  uint64_t* fetch_need_host = nullptr;  // [kFetchSlots] coherent pinned words (FetchSlot::need)
  uint64_t fetch_seq = 0;        // tickets
  std::vector<uint32_t> fetch_stamp;  // RMQ_FETCH_COMMIT duplicate check ([P][C] generation stamps)
  std::vector<uint32_t> fetch_stamp_rep;  // the same for replica reads ([P]: one replica cursor each)
  uint32_t fetch_gen = 0;
  std::deque<std::array<uint64_t, 3>> fetch_done;  // {ticket, rc, bytes used} completed, not yet polled
  // consumer-offset commits: staging slots (pinned items -> device by one copy on the pipeline
  // stream), so a commit is ordered with the append stream without waiting for it
  struct CommitSlot {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    uint32_t cap = 0;
    hipEvent_t ev = nullptr;
    bool used = false;
  };
  // a slot is reused once the commit that last used it has run on the pipeline stream, which may
  // queue a few launches ahead of it (RMQ_AHEAD): enough slots that a commit rarely waits
  static constexpr uint32_t kCommitSlots = 16;
  CommitSlot cslot[kCommitSlots];
  uint32_t cslot_next = 0;
  std::vector<uint32_t> lww_stamp;  // [P * C] generation of the last commit item seen per slot
  uint32_t lww_gen = 0;
  // consumer-offset tickets (rmq_commit_consumer_offset): the row version of every partition (host
  // mirror of DevState::cver) and, per pending ticket, the (partition, version) pairs it waits for
  std::vector<uint64_t> cver;
  std::vector<uint32_t> cstamp;  // [P] generation of the last call that bumped the version
  uint32_t cstamp_gen = 0;
  uint64_t off_ticket_seq = 0;
  std::deque<std::pair<uint64_t, std::vector<std::pair<uint32_t, uint64_t>>>> off_tickets;
  static constexpr size_t kMaxOffsetTickets = 256;   // the newest unpolled ones are kept
  // ack scratch
  uint32_t* d_ctl32 = nullptr;
  uint64_t* d_ctl64 = nullptr;
  uint32_t ctl_cap = 0;
  // profiling: pipeline launches are timed as one region (event before the first launch after
  // enable, event at the next drain) so no per-launch events sit between kernels; fetch kernels
  // keep per-launch event pairs (prof[3], prof[4])
  uint32_t profile = 0;
  uint32_t fetch_replay = 1;     // rmq_profile_enable(k >= 2): each fetch's kernels run k times
  uint64_t prof_fetch_runs = 0;
  uint64_t prof_launches = 0, prof_batches = 0;
  hipEvent_t prof_t0 = nullptr, prof_t1 = nullptr;
  bool prof_started = false, prof_ended = false;
  std::vector<EvPair> prof[5];
  std::vector<hipEvent_t> ev_pool;
  // diagnostics: RMQ_STAMPS=<csv> records per-wave phase stamps of launch RMQ_STAMPS_AT (default 100)
  const char* stamps_path = nullptr;
  uint64_t stamps_at = 100;
  uint64_t* d_stamps = nullptr;
  uint32_t stamps_wg[5] = {0, 0, 0, 0, 0};  // roles of the stamped launch: s1, s2, parts, s3, s3 lead
  // one stage-3 wave per task: the workgroups beyond the resident slots dispatch as stage-1/2
  // workgroups retire (RMQ_WG3_ALL=0: only as many as fit next to them, looping over tasks)
  uint32_t wg3_all = 1;
  uint32_t s1_wgs = 0;    // RMQ_S1_WGS: stage-1 workgroups per launch (0: one per tile; fewer loop over tiles)
  uint32_t s2_wgs = 0;    // RMQ_S2_WGS: cap on stage-2 workgroups (0: one thread group per column)
  uint32_t s3_first = 0;  // RMQ_S3_FIRST=1: stage-3 workgroups first in dispatch order (round 6 default: last, -2.5 %)
  uint32_t s3_lead = 0;   // stage-3 workgroups before the other roles (RMQ_S3_LEAD; 0: all of them)
  uint32_t debug = 0;  // RMQ_DEBUG (timing experiments only; results are invalid when set)
  // Split launches (single-GPU kernel, no transport): each pipeline step is two launches of the
  // pipeline kernel that run side by side, the ranking roles (stage 1 of group g, stage 2 of g - 1)
  // on rank_s and the apply roles (stage 3 of g - 2, partition threads, stage 4) on main_s. Rank
  // launch L waits for everything main_s issued before it (apply L - 1 resets the set stage 1 of L
  // reuses); apply launch L waits for rank launch L - 1 (the scans of the group it applies).
  // RMQ_SPLIT=1 (2: the two launches one after the other, timing only); 0 default: one launch per
  // step with every role (the split measured slower: 60 vs 49 us per step).
  uint32_t split = 0;
  uint32_t rank_cus = 0;        // RMQ_RANK_CUS=n: rank_s runs on n CUs and main_s on the others
  uint64_t* state_stage = nullptr;  // page-locked staging of rmq_get_partition_states
  size_t state_stage_words = 0;
  uint32_t s3_pair = 0;         // RMQ_S3_PAIR=1: stage-3 waves take two tasks each (single-GPU kernel)
  uint64_t late_done = 0;       // the applied group (by launch) whose late retention ran (late_retention)
  std::vector<uint32_t> fpend;  // slots of asynchronous fetches whose kernels wait for fetch_flush (under mu)
  uint32_t fetch_coalesce = kFetchBatch;  // RMQ_FETCH_COALESCE: asynchronous fetches launched together (1: none)
  uint32_t s3_stage = 1;        // RMQ_S3_STAGE (default 1): stage-3 payload spans by coalesced loads through LDS
  uint32_t s3_roles = 0;        // RMQ_S3_ROLES=k: stage 3 in loader / storer waves, k workgroups per CU (single-GPU kernel)
  uint32_t s3_xcd = 1;          // RMQ_S3_XCD (default 1): stage-3 tasks in contiguous ranges per XCD
                                //   (blockIdx % 8); round 5: 5.51-5.58 vs 5.43-5.51 G, 3 pairs, r05X8
  uint32_t s1_xcd = 0;          // RMQ_S1_XCD=1: stage-1 tiles in contiguous ranges per XCD
  // RMQ_FETCH_DMA: host request / result rows of a fetch moved by DMA (request rows on copy_s before
  // the kernels, result rows on fetch_out_s after them) instead of read and written in place by
  // the kernels across PCIe: 0 never (default), 1 for rmq_fetch_async, 2 for every fetch. Measured
  // (round 5, tools/exp_dma.sh): the kernels gain 4-11 us but each fetch's copies and cross-stream
  // waits add ~100 us (max = 10 bursts 3.3 -> 1.1 G records/s), so in place stays the default
  uint32_t fetch_dma = 0;
  uint32_t fetch_dma_in = 1;    // RMQ_FETCH_DMA_IN=0: with DMA, the request rows still read in place
  hipStream_t rank_s = nullptr;
  hipEvent_t ev_rank[2] = {nullptr, nullptr};  // rank launch L recorded in slot L & 1
  hipEvent_t ev_pre_rank = nullptr;            // main_s before a rank launch
  uint64_t rank_seq = 0;        // the last launch that had a rank launch (0: none)
  std::vector<uint64_t> key;  // [P] placement key of each partition (FORMAT.md §9 list order)
  rmq::Replication* repl = nullptr;  // replication transport attached (collective mode)
};

namespace rmq {

inline int hip_fail(hipError_t e) {
  if (e == hipSuccess) return RMQ_OK;
  std::fprintf(stderr, "ripplemq: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
  return e == hipErrorOutOfMemory ? RMQ_ENOMEM : RMQ_EDEVICE;
}

#define HIP_TRY(x)                      \
  do {                                  \
    hipError_t _e = (x);                \
    if (_e != hipSuccess) return hip_fail(_e); \
  } while (0)

template <typename T>
int dalloc(T** p, size_t count) {
  *p = nullptr;
  if (!count) count = 1;
  HIP_TRY(hipMalloc((void**)p, count * sizeof(T)));
  // The null stream does not order with the engine's non-blocking streams: finish the zeroing
  // before any engine stream can touch the buffer (a lazily allocated staging buffer would
  // otherwise be zeroed after its first H2D copy).
  HIP_TRY(hipMemset(*p, 0, count * sizeof(T)));
  HIP_TRY(hipDeviceSynchronize());
  return RMQ_OK;
}

// engine.cpp
int flush(rmq_engine* e);
int drain(rmq_engine* e);
int quiesce(rmq_engine* e);
int check_err(rmq_engine* e);
int event_wait(hipEvent_t ev);  // spin on queries (20 ms), then block
// replication.cpp
int repl_attach(rmq_engine* e, Transport* t);
void repl_free(rmq_engine* e);
int repl_set_lists(rmq_engine* e);
void repl_pipe_args(rmq_engine* e, PipeArgs& a, const GroupFlight* s2, const GroupFlight* s3);
int repl_before_launch(rmq_engine* e, PipeArgs& a);
int repl_after_launch(rmq_engine* e, const GroupFlight* s2, const GroupFlight* s3);
int repl_drain(rmq_engine* e);
int reset_catchup(rmq_engine* e);

}  // namespace rmq
