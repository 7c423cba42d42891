// kernels.hpp — launch interface between the host engine (engine.cpp) and the gfx950 kernels.
// Plain structs of device pointers; no torch types, no host STL.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rmq {

#ifndef RMQ_PIPE_THREADS
#define RMQ_PIPE_THREADS 256
#endif
constexpr uint32_t kPipeThreadsXR = 512;  // threads per workgroup of the kernel with a transport
constexpr uint32_t kPipeThreads = RMQ_PIPE_THREADS;  // threads per workgroup, every role of the pipeline launch (4 resident per CU)
#ifndef RMQ_TILE_BITS
#define RMQ_TILE_BITS 10
#endif
constexpr uint32_t kTileIdxBits = RMQ_TILE_BITS;       // log2(kTileRecs)
constexpr uint32_t kTileRecs = 1u << kTileIdxBits;     // records per ranking tile (stage 1)
constexpr uint32_t kMaxTiles = 512;      // tiles per group (stage 2 keeps their payload bases in LDS)
#ifndef RMQ_SCAN_LANES
#define RMQ_SCAN_LANES 16
#endif
constexpr uint32_t kScanLanes = RMQ_SCAN_LANES;  // stage 2: threads per partition column (8, 16 or 32)
// Stage 1 -> 2 tile cells (hist32): count of the (tile, partition) run in the high bits, its record
// bytes / 16 in the low kCellCntShift bits; kCellWide marks a run too large for that (its value is in
// the u64 hist cell at the same index). A count never reaches the field's all-ones value.
constexpr uint32_t kCellCntShift = kTileRecs <= 1024u ? 21u : 20u;
constexpr uint32_t kCellB16 = (1u << kCellCntShift) - 1u;
constexpr uint32_t kCellWide = ~0u;
static_assert((kTileRecs >> (32u - kCellCntShift)) == 0u, "a tile's count fits its cell field below all-ones");
#ifndef RMQ_SCAN_COLS
#define RMQ_SCAN_COLS 1
#endif
constexpr uint32_t kScanCols = RMQ_SCAN_COLS;  // stage 2: adjacent columns per thread group
constexpr uint32_t kTaskRecs = 32;       // records per apply task (one wave, 2 lanes per record)
constexpr uint32_t kMaxGroup = 8;        // batches per pipeline group (cfg.pipeline_depth)
constexpr uint32_t kMaxPartitions = 1u << 16;  // 16-bit partition keys (two 8-bit LDS radix passes)
constexpr uint32_t kMaxRF = 8;
constexpr uint32_t kMaxWorld = 16;       // ranks of a replication transport
constexpr uint32_t kMaxRemote = 4;       // remote replica slots per partition with a transport (RF <= 5)
constexpr uint32_t kXMagic = 0x34514D52u;  // "RMQ4": replica-log round region v4 (FORMAT.md §9)
constexpr uint32_t kRegionHdr = 64;      // region header bytes
constexpr uint32_t kDirEntry = 48;       // directory entry bytes (v4: + the leader's commit)
constexpr uint64_t kAckRefused = 1ull << 62;  // ack status bit (FORMAT.md §9 acks)
constexpr uint64_t kAckLeoMask = kAckRefused - 1ull;
constexpr uint64_t kNoRound = ~0ull;     // XEntry::data_abs: the entry carries no round records
constexpr uint64_t kTermRebase = 1ull << 63;  // directory term flag: the entry restarts the follower's log
                                              // at its first record (position in the entry's row)

struct CrcConsts;

// Where one out entry (a led partition's remote replica slot) of a group lands in the group's
// outbox (FORMAT.md §9), written by stage 2's plan, read by stage 3. 32 bytes.
struct XEntry {
  uint64_t data_abs;      // outbox byte offset of the entry's first ROUND record (after a catch-up
                          //   gap), or kNoRound: the entry carries none (partial catch-up)
  uint64_t tab_abs;       // outbox byte offset of that record's record-table slot
  uint64_t dir_abs;       // outbox byte offset of the entry's directory entry
  uint32_t k;             // entry index inside its destination's list
  uint32_t data_start16;  // that record's position inside the region's data section, / 16
};

// A catch-up entry of a round (FORMAT.md §9): the gap [first, first + count) of the leader's log,
// bytes [pos, pos + bytes), copied from the leader's ring into the outbox by the stage-3 launch's
// catch-up waves, one item per sparse-index interval the gap touches. 64 bytes.
struct XCatch {
  uint64_t pos;           // leader log position of the gap's first record (the follower's log end)
  uint64_t first;         // its offset
  uint64_t bytes;         // gap bytes
  uint64_t data_abs;      // outbox byte offset of the entry's first record
  uint64_t tab_abs;       // outbox byte offset of its record-table slot
  uint32_t k;             // entry index inside its destination's list
  uint32_t data_start16;  // the entry's first record inside the region's data section, / 16
  uint32_t p;             // led partition
  uint32_t items0;        // first copy item of the entry (prefix over the list)
  uint64_t pad;
};

// Per out entry, what the stage-2 workers of a group decide before the plan lays out the outbox:
// the follower log end F the entry would start at, the gap bytes before the round's records, kind.
struct XDecision {
  uint64_t f_off, f_pos;  // F (the leader's log end B before the round when not gapped)
  uint64_t gap;           // B.pos - F.pos for a gapped entry, 0 otherwise
  uint64_t r_off, r_pos;  // a catch-up request that arrived with this launch's acks (kDecNewReq)
  uint32_t flags;         // kDec*
  uint32_t pad;
};
constexpr uint32_t kDecReq = 1u, kDecRow = 2u, kDecDetached = 4u, kDecGapped = 8u, kDecNewReq = 16u;
constexpr uint32_t kDecRebase = 32u;     // the gap starts at the leader's rebase point, not at the follower
constexpr uint32_t kRowRebase = 1u << 31;  // XDecision::pad: the planned entry is a granted rebase

// Leader side of a replication round: the layout plan of one group's outbox (stage 2 of the group,
// computed by the last stage-2 workgroup of the launch) and the catch-up state it advances.
struct XPlanArgs {
  const uint32_t* xo_p;      // [n_out] led partition of each out entry, grouped by destination
  const uint32_t* xo_slot;   // [n_out] its replica slot
  const uint32_t* xo_start;  // [world + 1]
  const uint64_t* keysum;    // [world] FORMAT.md §9 key sum of each destination's entry list
  uint32_t world, rank, n_out, C;
  uint32_t* count;           // arrival counter of the launch's stage-2 workgroups (reset by the plan)
  XEntry* xe;                // [n_out]
  uint8_t* outbox;
  uint64_t* sizes;           // [world][2] {region bytes, records} per destination (0: nothing to send)
  // catch-up and consumer-offset rows (FORMAT.md §9 v3)
  uint64_t round;            // this group's round number
  uint64_t reserve;          // catch-up bytes per destination
  uint64_t* xnext;           // [n_out][2] leader's expectation of the follower log end {offset, pos}
  uint64_t* xreq;            // [n_out][4] pending catch-up request {offset, pos, round + 1 (0 none), 0}
  uint64_t* xcu;             // [n_out] round of the last catch-up plan
  XDecision* xdec;           // [n_out] stage-2 workers -> plan
  uint64_t* xtot;            // [n_out] the group's totals word of the entry's partition (workers -> plan)
  uint32_t* dflag;           // [world] kDecRow | kDecGapped of any entry to that destination
  const uint64_t* csnap;     // [P] the leader's commit when the launch started (the previous launch's slot)
  const uint64_t* ackin;     // acks applied in this launch, [n_out][2], or null
  uint64_t acks_round;       // the round they answer
  uint32_t* dirty;           // [P] consumer offsets changed since the last round (cleared by the plan)
  uint64_t* rowv;            // [n_out] this round: the row version each entry carries (0: no row)
  XCatch* xc;                // [n_out] catch-up list of the group
  uint32_t* xc_n;            // [2] {catch-up entries, copy items}
  uint64_t* counters;        // [3] leader: catch-up entries planned, detached entry plans, general plans
  uint64_t dcap;             // outbox bytes per destination: region d at d * dcap
};

// Per-partition device state (SoA, [P] unless noted). Owned by the engine.
struct DevState {
  // leo / used point at the CURRENT state set (see StateSet)
  uint64_t* leo;         // log end offset (next offset)
  uint64_t* used;        // log end byte position (logical)
  uint64_t* start_off;   // retained log start (pipeline stage 4 updates it in place)
  uint64_t* start_pos;
  uint64_t* commit;
  uint64_t* hw;
  uint64_t* term_start;
  uint64_t* term;        // current term of the partition known here (leader: its own; follower: the
                         // newest leader term a round carried, FORMAT.md §9)
  uint64_t* match;       // [P][RF]
  uint32_t* is_leader;   // 0/1
  uint32_t* local_mask;  // bit r set: replica slot r is stored on this device
  uint64_t* index;       // sparse offset index {offset, pos}: partition p's ring of entries at RingRef.ibase
  uint8_t* logs;         // [RF][pool] replica regions; partition p's ring at RingRef.base in each
  uint64_t* ring;        // [P] ring descriptor: byte offset in the pool | log2(ring bytes) (bits 0..5)
  uint64_t* cons;        // [P][C] consumer offsets
  uint64_t* pcache;      // [P][C][2] fetch position cache {offset, its ring byte position}: the end
                         //   of each consumer's last served slice (fetch.hip); an entry is always a
                         //   true pair (committed records never move), offset ~0 = empty
  uint32_t* cdirty;      // [P] consumer offsets changed since the last replication round (FORMAT §9)
  uint64_t* rcur;        // [P] replica cursor: where an RMQ_FETCH_REPLICA read starts (local, not replicated)
  uint64_t* lcommit;     // [P] follower: the newest leader commit learned (rounds, commit notices;
                         //   FORMAT.md §9); a leader's own is `commit`
  uint64_t* csnap;       // [2][P] leader commit at the end of launch L, in slot L & 1 (partition threads
                         //   of every transport launch, and the control kernels after it): the plan of
                         //   launch L + 1 carries it in its directory (one value per round, whatever
                         //   that launch's partition threads fold in meanwhile)
  uint32_t csnap_slot;   // the slot of the last launch issued (control kernels write it)
  // consumer-offset rows on a quorum (rmq_commit_consumer_offset tickets, FORMAT.md §8)
  // leader election: Raft's lastLogTerm, the term this log was last verified in
  // against its leader's, and the round stamp of the last entry or notice heard from the leader
  uint64_t* lterm;       // [P] last log term; kLtermBound | t: unknown, at most t (a partial catch-up)
  uint64_t* mterm;       // [P]
  uint64_t* heard;       // [P]
  uint64_t* cver;        // [P] leader: version of the partition's row (one per commit call touching it)
  uint64_t* cq;          // [P] leader: the newest row version a quorum of its replicas holds
  const uint32_t* outidx;  // [P][RF] out entry of (partition, remote slot), ~0: none (transport), or null
  uint64_t* eackv;       // [n_out] newest row version the entry's follower acknowledged, or null
  uint64_t rstride;      // bytes per replica region (the pool)
  uint32_t P, RF, C;
  uint32_t icap_mul;     // index entries per interval of ring (2 * group + 2)
  uint32_t interval_log2;
  uint32_t pad;
};

// Where partition p's ring and index live (FORMAT.md §2, §5). A ring of S bytes sits at a multiple
// of S inside each replica region; its index ring holds icap_mul * S / I entries at a proportional
// offset of the index pool, so rings and index rings never overlap.
// DevState::lterm of a follower whose last entry's term is unknown (a partial catch-up that ended below
// its leader's term start, FORMAT.md §9 v5): the flag and an upper bound, the leader's term - 1. A vote
// compares against the bound (stricter: only liveness can suffer), a candidate claims 0 (never more
// than it has).
constexpr uint64_t kLtermBound = 1ull << 63;

struct RingRef {
  uint64_t base;   // byte offset of the ring inside a replica region
  uint64_t seg;    // ring bytes (power of two)
  uint64_t ibase;  // first index entry of the partition
  uint32_t icap;   // index ring entries
};

__host__ __device__ __forceinline__ RingRef ring_ref(uint64_t desc, uint32_t interval_log2, uint32_t icap_mul) {
  RingRef r;
  r.seg = 1ull << (desc & 63ull);
  r.base = desc & ~63ull;
  r.ibase = (r.base >> interval_log2) * icap_mul;
  r.icap = icap_mul * (uint32_t)(r.seg >> interval_log2);
  return r;
}
__host__ __device__ __forceinline__ RingRef ring_ref(const DevState& st, uint32_t p) {
  return ring_ref(st.ring[p], st.interval_log2, st.icap_mul);
}

// Double-buffered per-partition log end: the apply of group #a reads set a&1 and writes set
// (a+1)&1, so records can read their partition's group-start state while its new one is written.
struct StateSet {
  uint64_t* leo;
  uint64_t* used;
};

// One append batch as the pipeline sees it (device pointers).
struct PipeBatch {
  const uint32_t* pidx;
  const uint32_t* len;
  const uint64_t* poff;        // caller payload offsets, or nullptr (packed)
  const uint8_t* payload;
  uint64_t payload_bytes;
  uint64_t* out_offsets;       // input order
  uint32_t n;
  uint32_t tiles;              // ceil(n / kTileRecs)
};

// A group of up to kMaxGroup consecutive batches moving through the pipeline together. Batch j
// owns the group tiles [tile0[j], tile0[j+1]) and the stage-3 tasks [task0[j], task0[j+1]).
struct PipeGroup {
  PipeBatch b[kMaxGroup];
  uint4* stats[kMaxGroup];        // per batch: [tasks] {appended, not leader, unknown partition,
                                  //   no space | invalid << 16}
  uint32_t tile0[kMaxGroup + 1];
  uint32_t task0[kMaxGroup + 1];
  uint32_t nb;                    // batches (0: the stage is absent from the launch)
  uint32_t tiles;                 // tile0[nb]
};

// Group-local scratch of one pipeline set (four sets rotate: a group is ranked in launch k,
// scanned in k+1, applied in k+2 and its retention evaluated in k+3).
struct PipeScratch {
  uint32_t* hist32;     // [P][gt] tile cell (kCellCntShift packing, kCellWide); 0 = absent (stage 2 clears)
  uint64_t* hist;       // [P][gt] tile aggregate {count << 40 | bytes/16} of a kCellWide cell only
  uint64_t* excl;       // [P][gt] exclusive prefix over the group's accepted cells (bit 63: the
                        //   cell's (batch, partition) is rejected for space, FORMAT.md §3)
  uint64_t* totals;     // [P] group aggregate over accepted cells
  uint64_t* pk;         // [P][8] what stage 3 reads of partition p for the group, in one 64-byte line
                        //   (stage 2 writes it): {log end offset, position before the group, totals,
                        //   ring descriptor, is_leader | local_mask << 8, 0, 0, 0}
  uint64_t* bcum;       // [kMaxGroup][P] aggregate through batch j (accepted cells)
  uint2* crank;         // [tiles * kTileRecs] {rank in tile run | flags << 29, bytes/16 before it in the run}
  uint32_t* pre;        // [tiles * kTileRecs] payload bytes before the record inside its tile
  uint64_t* tsum;       // [tiles][4] {payload bytes, record bytes, invalid records, 0}
  uint64_t* tile_base;  // [tiles] payload offset of the tile's first record inside its batch
  uint64_t* binfo;      // [kMaxGroup][4] per batch {reject flags (2 invalid payload ranges), 0, payload bytes, 0}
  uint64_t* bacc;       // [kMaxGroup][2] per batch {payload bytes, invalid records} (stage 1 adds,
                        //   stage 2 reads, stage 4 resets)
  uint32_t* nbig;       // [4] {records over 1 KB in the group (stage 1 appends), tiles taken by
                        //   stage-1 workgroups, 0, 0} (stage 4 resets)
  uint32_t* bigl;       // [tiles * kTileRecs] their group record slots, in no particular order
};

// The single per-group launch: stage 1 (rank the tiles of group k), stage 2 (column scans of
// group k-1), stage 3 (apply group k-2) and stage 4 (retention of group k-3). Any may be absent.
struct PipeArgs {
  DevState st;
  StateSet cur, nxt;       // stage 3: read cur, write nxt; stage 4: cur = log end after its group
  PipeGroup g1, g2, g3, g4;
  PipeScratch s1, s2, s3, s4;
  uint32_t wg1, wg2, wgp, wg3;  // workgroups per role, in this order along blockIdx.x
  uint32_t wgb;                 // stage 3's large-record workgroups (last along blockIdx.x)
  uint32_t key_passes;     // 1 (P <= 256) or 2
  uint32_t key_bits;       // bits of the largest partition id (P - 1)
  uint32_t rank_mode;      // stage 1: 0 LDS radix sort + segmented scan, 1 wave-ordered hash counters
  uint32_t gt;             // tiles per hist / excl column (group tile capacity)
  uint32_t s3_lead;        // stage-3 workgroups placed before the other roles along blockIdx.x
  uint32_t s3_pair;        // stage-3 waves take two tasks each, their loads interleaved (task, task + wg3 waves)
  uint32_t s3_roles;       // stage 3 in loader / storer waves (RMQ_S3_ROLES): each workgroup a run of tasks
  uint32_t s3_stage;       // stage 3 loads a packed task's payload span by coalesced loads through LDS (RMQ_S3_STAGE)
  uint32_t s3_xcd;         // stage-3 task order by XCD: the workgroups sharing an XCD take one contiguous task range
  uint32_t s1_xcd;         // stage-1 tile order by XCD (the same for the ranking workgroups)
  uint32_t debug;         // diagnostic only (RMQ_DEBUG, results invalid): 1 no payload ring
                           // stores, 2 no CRC lookups, 4 no payload loads, 8 no CRC tables,
                           // 16 skip stages 1-2, 32 no leader / mask / totals gathers in stage 3
  // replication transport attached (else all null / n_out = 0)
  XPlanArgs xp2;           // stage 2's group: outbox plan
  const uint32_t* outidx;  // [P][RF] out entry of (partition, slot), ~0: local or no entry
  const XEntry* xe3;       // stage 3's group: entry placement
  uint8_t* outbox3;        // stage 3's group: its outbox
  const uint64_t* ackin;   // acks of an earlier group, by out entry [n_out][2] (partition threads), or null
  const uint64_t* ackrowv; // the row versions that group's round carried [n_out]
  uint64_t acks_round;     // the round they answer
  uint64_t* xreq;          // catch-up requests (partition threads write them when no plan runs)
  const XCatch* xc3;       // stage 3's group: its catch-up list and counts (catch-up waves)
  const uint32_t* xc3_n;
  uint32_t wgc;            // catch-up workgroups (last along blockIdx.x)
  const CrcConsts* crc;
  uint64_t* done_word;     // host-visible: sequence number of the previous launch (written at start)
  uint64_t* lastg;         // replication: [P] record bytes / 16 of the last group applied (a plan's C)
  uint32_t* rlate;         // [P] 1: the partition's retention of the group applied stopped early
  uint64_t* ret_late;      // host-visible: written with launch_seq when a partition's retention of
                           // the group applied stops early (its stage 4 in the next launch finishes it)
  uint64_t launch_seq;
  uint32_t steal;          // stage-3 workgroups rank stage-1 tiles once out of tasks (RMQ_STEAL)
  uint32_t prio;           // stage-1/2 and partition waves at raised issue priority (RMQ_PRIO)
  uint64_t* stamps;        // diagnostic only (RMQ_STAMPS): [workgroup][wave][8] s_memrealtime, or null
};

struct FetchArgs {
  DevState st;
  const uint32_t* req;       // [n][4] {pidx, consumer, max, flags}: page-locked host rows (read once)
  uint32_t* req_dev;         // [n][4] the resolve's device copy of them (the gather reads it)
  uint64_t* res;             // [n][4] {start_offset, out_pos, count|bytes<<32, status}, then {bytes needed}
                             //   (device: resolve -> gather)
  uint64_t* res_host;        // [n][4] the final result rows, written by the gather into page-locked
                             //   host memory (no copy node)
  uint64_t* aux;             // [n][2] {source byte position, ring byte offset in logs}
  uint32_t* cpre;            // [n + 1] bytes of each request (resolve -> gather), 16-byte aligned
  uint64_t* csum;            // [n / kFetchChunk + 1][kCsumStride] bytes of each chunk of kFetchChunk
                             //   requests (one 128-byte line per chunk: the adds of different
                             //   chunks never meet in one L2 line)
                             //   (resolve adds; zeroed by the previous fetch of the slot)
  uint64_t* csum_next;       // the slot's other chunk-sum half, which the gather zeroes for the next
                             //   fetch (word 0 of csum_lines lines; no memset between the fetches)
  uint8_t* out;              // 16-byte aligned
  uint64_t out_cap;
  uint64_t* need_host;       // host-visible word (coherent pinned): bytes needed, written by the
                             //   gather with a system-scope store (no copy node for it)
  uint32_t n;
  uint32_t csum_lines;
  uint32_t commits;          // the host checked read-and-commit requests in the call (else flags ignored)
  uint32_t replica;          // the host checked RMQ_FETCH_REPLICA requests in the call (else flags ignored)
};
constexpr uint32_t kFetchChunk = 256;  // requests per chunk sum (placement)
// Up to kFetchBatch asynchronous fetches (tickets) are launched as one resolve + gather pair: ticket k
// owns the kernels' workgroups [wg0, wg0 + its own count) (no workgroup straddles two tickets), and
// reads its own arguments, rows, scratch and output.
constexpr uint32_t kFetchBatch = 4;
struct FetchBatch {
  FetchArgs t[kFetchBatch];
  uint32_t rwg0[kFetchBatch + 1];  // first resolve workgroup of each ticket (then the total)
  uint32_t gwg0[kFetchBatch + 1];  // first gather workgroup of each ticket
  uint32_t nt;
};
constexpr uint32_t kFetchReplica = 2u;  // rmq_fetch_req.flags RMQ_FETCH_REPLICA
constexpr uint32_t kCsumStride = 16;   // u64 words per chunk sum (128 bytes)



struct ConsumerCommitArgs {  // one item per (partition, consumer): the host resolved last-writer-wins
  DevState st;
  const uint32_t* pidx;
  const uint32_t* consumer;
  const uint64_t* offset;
  const uint64_t* ver;     // the partition's new row version (the same for every item of a partition)
  uint32_t n;
  uint32_t pad;
};

// The last applied group's retention for partitions whose replay its launch stopped early
// (late_retention_kernel): the group's batch aggregates and totals, and the per-partition flags.
struct LateArgs {
  DevState st;
  const uint64_t* bcum;  // [kMaxGroup][P] the group's aggregate through each batch
  const uint64_t* totals;
  uint32_t* rlate;
  uint32_t nb;
};

struct AckArgs {
  DevState st;
  const uint32_t* pidx;
  const uint32_t* slot;
  const uint64_t* match;
  uint32_t n;
};

// Follower side of a replication round: ingest every source's region of one inbox.
struct IngestArgs {
  DevState st;
  StateSet sets[2];          // follower partitions keep both sets equal
  const uint8_t* inbox;
  uint64_t region[kMaxWorld];     // inbox byte offset of each source's region
  uint64_t rbytes[kMaxWorld];     // its size (0: nothing from that source)
  uint32_t task0[kMaxWorld + 1];  // prefix of the per-source task bounds (32 records per task)
  const uint32_t* xi_p;      // [n_in] local partition of each in entry, grouped by source
  const uint32_t* xi_slot;   // [n_in] local replica slot
  const uint32_t* xi_start;  // [world + 1]
  uint32_t world, rank, n_in, C;
  uint32_t* bad;             // [n_in] entry refused this round: bit 0 CRC, 1 log mismatch, 2 stale
                             //   term, 3 missed round (prepare sets it, verify adds to it)
  uint32_t* acc;             // [n_in] 1: accepted (finish -> copy)
  uint64_t* base;            // [n_in][2] {log end offset, log end position} the entry continues:
                             // the follower's, or the leader's first offset after a truncation
  uint64_t* ackout;          // [n_in][2] follower log end after the round | status (FORMAT.md §9)
  uint64_t* cdesc;           // [n_in][4] copy descriptor of an entry with copy items (prepare ->
                             //   copy): {data address, ring address, log end position it continues,
                             //   bytes << 6 | log2(ring bytes)}
  uint32_t* items;           // [cap][2] copy work items {entry, chunk of kCopyChunk bytes} (prepare)
  uint32_t* n_items;         // [1] items allocated this round (prepare adds; zero at the start)
  uint32_t* insane;          // [kMaxWorld] a structural fault of that source's region (prepare and
                             //   verify set it; zero at the start)
  uint32_t* n_items_next;    // the next round's n_items and insane words: prepare clears them (no
                             //   memset node between the rounds)
  const uint64_t* keysum_in; // [world] FORMAT.md §9 key sum of each source's entry list (this side's)
  uint32_t items_cap;        // slots of `items`
  uint32_t items_grid;       // copy workgroups launched: items past it are never copied
  const CrcConsts* crc;
  uint64_t* counters;        // [4] records ingested, entries refused (CRC), refused (log mismatch), bytes
  uint64_t stamp;            // the round's stamp (its number + 1): heard words of the entries from a live leader
};
constexpr uint64_t kCopyChunk = 16ull << 10;  // follower copy: region bytes per workgroup

// Commit notices (FORMAT.md §9, a drain's heartbeat): the leader's {commit, term} per out entry,
// and the follower's application per in entry.
struct NoticeArgs {
  DevState st;
  StateSet sets[2];
  const uint32_t* xo_p;      // [n_out]
  uint64_t* out;             // [n_out][2] {commit, term}
  const uint32_t* xi_p;      // [n_in]
  const uint64_t* in;        // [n_in][2]
  uint32_t n_out, n_in;
  uint64_t stamp;            // the drain's round stamp (heard words)
};

// Acks of one round applied outside the pipeline (drain): thread per partition.
struct AckApplyArgs {
  DevState st;
  const uint32_t* outidx;
  const uint64_t* ackin;     // [n_out][2]
  const uint64_t* rowv;      // [n_out] the row versions that round carried
  uint64_t* xreq;            // refused acks become catch-up requests
  uint64_t acks_round;
};

// One partition's ring moving to a new block of the pool (rmq_set_segments): the retained log
// [spos, used) of every replica slot and its index entries are copied; the new block is zeroed first.
struct MigrateItem {
  uint32_t p;
  uint32_t chunk0;              // first workgroup of the move (prefix of kMigrateChunk pieces)
  uint64_t old_desc, new_desc;  // DevState::ring descriptors
  uint64_t spos, used;          // retained log [spos, used) after the move
  uint64_t soff;                // offset of the record at spos
};

// launchers (defined in the .hip files)
// start: an event the dispatch records as the kernel starts (profiling), or null
void launch_pipeline(const PipeArgs& a, hipStream_t s, hipEvent_t start = nullptr);
uint32_t pipeline_wgs_per_cu(uint32_t threads);  // resident workgroups per CU of that size
void launch_commit_all(const DevState& st, hipStream_t s);
void launch_ack(const AckArgs& a, hipStream_t s);
void launch_late_retention(const LateArgs& a, hipStream_t s);
void launch_become_leader(const DevState& st, uint32_t pidx, hipStream_t s);
void launch_fetch(const FetchArgs& a, hipStream_t s, const hipEvent_t* ev4);
void launch_fetch_batch(const FetchArgs* t, uint32_t nt, hipStream_t s);  // nt <= kFetchBatch tickets, one pair
void preload_fetch_kernels();

void launch_consumer_commit(const ConsumerCommitArgs& a, hipStream_t s);
void launch_row_quorum_all(const DevState& st, hipStream_t s);
void launch_state_gather(const DevState& st, uint64_t* out, uint32_t first, uint32_t n, uint32_t RF, hipStream_t s);
void launch_ingest(const IngestArgs& a, uint32_t tasks, uint32_t items_bound, uint32_t verify_wgs, hipStream_t s);
uint32_t verify_wgs_per_cu();
uint32_t verify_records_per_task();  // the host sizes the verify tasks with it
constexpr uint64_t kMigrateChunk = 256ull << 10;  // new-ring bytes per workgroup of a move
// chunks = total workgroups (sum over the items of ceil(new ring bytes / kMigrateChunk))
void launch_migrate(const DevState& st, const MigrateItem* items, uint32_t n, uint32_t chunks, hipStream_t s);
void launch_ack_apply(const AckApplyArgs& a, hipStream_t s);
void launch_notice_fill(const NoticeArgs& a, hipStream_t s);   // leader: {commit, term} per out entry
void launch_notice_apply(const NoticeArgs& a, hipStream_t s);  // follower: learn the leader's commit
void launch_flip(uint8_t* region, uint64_t size, int64_t at, hipStream_t s);  // rmq_fault_corrupt

}  // namespace rmq

namespace rmq_x {
// pipeline.hip compiled for a replication transport (512-thread workgroups)
void launch_pipeline_xr(const rmq::PipeArgs& a, hipStream_t s, hipEvent_t start);
}  // namespace rmq_x
