/*
 * ripplemq_engine.h — C-ABI of the MI355X-native Partition-Raft engine.
 *
 * This is the drop-in boundary for RippleMQ's partition data path.
 * The Java broker keeps its RPC processors; each processor replaces the call it makes into
 * the per-partition jraft group with a call into this library (JNI stub: INTEGRATION.md).
 *
 * Reference interface each entry point replaces (paths relative to the reference root):
 *
 *   rmq_append                  <- Node.apply(new Task(ByteBuffer, done)) for a MessageAppendRequest,
 *                                  mq-broker/src/main/java/metadata/raft/request/processor/
 *                                  MessageAppendRequestProcessor.java:52-59, applied by
 *                                  PartitionStateMachine.onApply/handleMessageAppendRequest
 *                                  (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:38-69)
 *   rmq_poll_commit             <- the PartitionClosure completion (request/PartitionClosure.java:32-36)
 *                                  that turns Status into MessageAppendResponse{success,errorMsg}
 *                                  (MessageAppendRequestProcessor.java:39-48); jraft BallotBox commit
 *   rmq_ack                     <- follower AppendEntries success -> BallotBox.commitAt  [jraft, SURVEY §3.4]
 *   rmq_commit_consumer_offset  <- Node.apply for a ConsumerOffsetUpdateRequest
 *                                  (ConsumerOffsetUpdateRequestProcessor.java:38-60) applied by
 *                                  PartitionStateMachine.handleConsumerOffsetUpdateRequest (:71-77)
 *   rmq_fetch                   <- PartitionStateMachine.handleBatchRead (:85-110) called from
 *                                  MessageBatchReadRequestProcessor.java:39 (direct read, no read-index)
 *   rmq_become_leader           <- PartitionStateMachine.onLeaderStart(term) (:121-126)
 *   rmq_vote / rmq_leader_silent <- jraft's RequestVote and election timer of each partition group
 *                                  (PartitionRaftServer.setupRaft: electionTimeoutMs 1000, raft_meta
 *                                  term/votedFor, PartitionRaftServer.java:85,89)  [jraft]
 *   rmq_set_replicas            <- PartitionRaftServer.setupRaft initial Configuration(peers)
 *                                  (mq-broker/src/main/java/metadata/raft/PartitionRaftServer.java:82-86)
 *   rmq_create / rmq_destroy    <- PartitionManager.startPartition / PartitionRaftServer.shutdown
 *                                  (PartitionManager.java:166-176, PartitionRaftServer.java:100-108)
 *   rmq_set_segments            <- no reference counterpart (its logs never evict, PartitionStateMachine.java
 *                                  :26,66): per-partition retention size inside a shared HBM pool
 *   rmq_set_placement           <- PartitionManager.handleTopicListChange starting the groups this broker
 *                                  hosts with their peers (PartitionManager.java:111-176), as placed by
 *                                  PartitionAssigner.assignPartitions (PartitionAssigner.java:25-94)
 *   rmq_attach_rccl /           <- the shared RpcServer/BoltRpcClient pair jraft replicates over
 *   rmq_attach_local               (PartitionRaftServer.java:93): AppendEntries to the followers and
 *                                  their acks, here grouped RCCL send/recv of replica-log rounds
 *                                  (FORMAT.md §9) between the engines of one node
 *
 * Only dense partition indices (pidx) cross this boundary; the Java side keeps the
 * "topic-partitionId" -> pidx map (PartitionManager.java:121,196-198).
 *
 * Threading: one submitter thread per engine for rmq_append / rmq_ack /
 * rmq_commit_consumer_offset / rmq_become_leader / rmq_set_replicas. rmq_fetch, rmq_poll_commit
 * and the read-back calls may be called from any thread (they serialize on an internal lock).
 * Completion is by polling tickets; the library never calls back into the host.
 *
 * Replication transport (multi-GPU): after rmq_attach_rccl / rmq_attach_local the
 * engines of the world replicate every launch group of appends to the followers named by the
 * placement and commit on quorum. Rounds are collective, like the launches that drive them: every
 * rank must make the same sequence of rmq_append calls (empty batches count) and of the calls that
 * flush the pipeline (rmq_sync, rmq_set_placement, rmq_set_replicas, rmq_become_leader, rmq_ack);
 * rmq_poll_commit / rmq_ticket_stats never flush then: they answer RMQ_PENDING until later launch
 * groups (further rmq_append calls on every rank, empty batches included: ripplemq_amd/pacer.py) or
 * an rmq_sync on every rank pushed the ticket through its stages; rmq_sync before rmq_destroy.
 *
 * Log byte format, offset index and retention are defined in FORMAT.md.
 */
#ifndef RIPPLEMQ_ENGINE_H
#define RIPPLEMQ_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMQ_ABI_VERSION 10u
#define RMQ_MAX_RF 8u
#define RMQ_ALL_PARTITIONS 0xFFFFFFFFu
#define RMQ_OFFSET_NONE 0xFFFFFFFFFFFFFFFFull /* out_offsets value of a rejected record */
#define RMQ_RECORD_HEADER_BYTES 16u
#define RMQ_RECORD_ALIGN 16u /* records start and end on 16-byte boundaries (FORMAT.md §1) */
#define RMQ_TICKET_OFFSETS 0x8000000000000000ull /* tickets of rmq_commit_consumer_offset carry this bit */

/* Status codes. Negative = error; RMQ_PENDING is a non-error poll result. */
enum {
  RMQ_OK = 0,
  RMQ_PENDING = 1,
  RMQ_ENOTLEADER = -1, /* "Not leader" reply of the reference processors */
  RMQ_ENOPART = -2,    /* unknown pidx (reference: NPE at MessageAppendRequestProcessor.java:29) */
  RMQ_EINVAL = -3,
  RMQ_ENOSPC = -4,     /* batch larger than configured capacity / fetch output buffer too small */
  RMQ_EDEVICE = -5,    /* HIP runtime error or no HIP device */
  RMQ_EOFFSET = -6,    /* fetch offset below the retained log start (evicted by retention) */
  RMQ_ENOMEM = -7,
  RMQ_ESTALE = -8,     /* rmq_become_leader: this replica lacks records its partition's leader
                          committed (Raft's vote restriction: it may not lead) */
  RMQ_ETERM = -9       /* rmq_become_leader: the term already has a leader here (this replica led it,
                          or voted for another candidate in it: Raft's one vote per term) */
};
#define RMQ_NO_VOTE 0xFFFFFFFFu /* rmq_partition_state.voted_for: no vote in voted_term */

/* Memory kind of caller buffers.
   RMQ_MEM_HOST: pageable host memory (rmq_append packs it into a pinned staging slot with host
     threads, then one DMA; payload ranges are checked on the host: RMQ_EINVAL).
   RMQ_MEM_DEVICE: device memory (rmq_device_alloc).
   RMQ_MEM_PINNED (rmq_append only): page-locked host memory (rmq_host_alloc, or pages registered
     with rmq_host_register): every section goes to the device by its own DMA on the engine's copy
     stream, with no host copy; out_offsets must be page-locked too and is written by a DMA. The
     caller keeps all of them unchanged until the ticket completes (like device batches), and
     payload ranges are checked on the device like device batches (rejected_invalid). */
enum { RMQ_MEM_HOST = 0, RMQ_MEM_DEVICE = 1, RMQ_MEM_PINNED = 2 };

typedef struct rmq_config {
  uint32_t num_partitions;     /* P: dense pidx in [0, P), P <= 65536 per engine */
  uint32_t replication_factor; /* RF in [1, RMQ_MAX_RF]; quorum = RF/2 + 1 */
  uint64_t segment_bytes;      /* ring bytes per (replica, partition) log; multiple of index_interval */
  uint32_t index_interval;     /* sparse offset-index interval in bytes; power of two in [64, 1<<20] */
  uint32_t max_consumers;      /* consumer-offset table width per partition (dense consumer ids) */
  uint32_t max_batch_records;  /* capacity of one rmq_append call */
  uint32_t pipeline_depth;     /* batches applied per pipeline launch group, 1..8; 0 -> default 2 */
  uint64_t max_batch_bytes;    /* payload bytes of one rmq_append call */
  int32_t device;              /* HIP device ordinal */
  uint32_t rank;               /* replica rank of this engine (placement in rmq_set_replicas) */
  uint64_t pool_bytes;         /* ring bytes per replica shared by all partitions (FORMAT.md §2);
                                  0 -> num_partitions * segment_bytes. Every partition starts with a
                                  segment_bytes ring; rmq_set_segments resizes them inside the pool */
} rmq_config;

/* One append batch: records of many partitions, interleaved, in apply order (SoA). */
typedef struct rmq_batch {
  uint32_t n;                  /* number of records */
  uint32_t mem;                /* RMQ_MEM_HOST, RMQ_MEM_DEVICE or RMQ_MEM_PINNED for every pointer below */
  const uint32_t* pidx;        /* [n] partition of each record */
  const uint32_t* len;         /* [n] payload length of each record */
  const uint64_t* payload_off; /* [n] byte offset of each payload in `payload`, or NULL = packed
                                  (payload_off[i] = sum of len[j], j < i) */
  const uint8_t* payload;      /* payload bytes */
  uint64_t payload_bytes;      /* readable bytes at `payload` */
} rmq_batch;

typedef struct rmq_fetch_req {
  uint32_t pidx;
  uint32_t consumer;           /* dense consumer id in [0, max_consumers) */
  uint32_t max_records;        /* reference: MessageBatchReadRequest.maxMessages */
  uint32_t flags;              /* RMQ_FETCH_COMMIT, or 0 */
} rmq_fetch_req;
/* rmq_fetch_req.flags: once the request is served (RMQ_OK, its records in the output) or answered
   RMQ_EOFFSET, commit the consumer's next offset — start_offset + count (the first retained offset
   for RMQ_EOFFSET) — as rmq_commit_consumer_offset would (no ticket; with a transport the row
   travels with the next round). The consumer client's read-then-commit
   (ConsumerClientImpl.java:61-117) in one device pass. At most one committing request per
   (partition, consumer) in a call (RMQ_EINVAL otherwise). */
#define RMQ_FETCH_COMMIT 1u
/* rmq_fetch_req.flags (ABI 10): read this engine's own replica of pidx, whether it leads the
   partition or follows it: the slice starts at the partition's replica cursor (rmq_set_replica_cursor;
   the consumer field only keys the position cache and must be < max_consumers) and ends at the
   replica's commit (its high_watermark: on a follower the part of its log below the leader commit
   it learned). With RMQ_FETCH_COMMIT the replica cursor moves to start_offset + count (local to this
   engine, never replicated; one committing replica request per partition in a call). This is how a
   replica's durable tier reads its own log: jraft keeps the whole log on every node
   (PartitionRaftServer.java:53,88-90), so a follower persists what it holds, not only a leader. */
#define RMQ_FETCH_REPLICA 2u

typedef struct rmq_fetch_res {
  uint64_t start_offset;       /* reference: MessageBatchReadResponse.offset (the consumer offset);
                                  RMQ_EOFFSET: the first retained offset, where the consumer can resume */
  uint64_t out_pos;            /* byte position of this request's records in the output buffer */
  uint32_t count;              /* records returned (reference: messages.size()) */
  uint32_t bytes;              /* bytes of the returned records (FORMAT.md record layout) */
  int32_t status;              /* RMQ_OK, RMQ_ENOTLEADER, RMQ_ENOPART, RMQ_EINVAL, RMQ_EOFFSET, RMQ_ENOSPC */
  uint32_t reserved;
} rmq_fetch_res;

typedef struct rmq_partition_state {
  uint64_t log_end_offset;     /* next offset to assign (reference: messages.size() on the leader) */
  uint64_t log_end_pos;        /* logical byte position of the log end */
  uint64_t log_start_offset;   /* first retained offset */
  uint64_t log_start_pos;      /* logical byte position of log_start_offset */
  uint64_t commit;             /* quorum commit (count of committed records) */
  uint64_t high_watermark;     /* consumer-visible end (== commit) */
  uint64_t term;
  uint64_t term_start;         /* log_end_offset at rmq_become_leader */
  uint64_t match[RMQ_MAX_RF];  /* per replica slot: records known persisted */
  uint32_t replica_rank[RMQ_MAX_RF];
  uint32_t leader_slot;
  uint32_t is_leader;
  uint64_t segment_bytes;      /* ring bytes of this partition (retention keeps at most this much) */
  uint64_t leader_commit;      /* the newest commit index of the partition's leader this replica knows
                                  (the Raft leaderCommit of the rounds and commit notices it received,
                                  FORMAT.md §9); on the leader its own commit. A replica whose log
                                  ends below it lacks committed records (rmq_become_leader: RMQ_ESTALE) */
  /* ABI 8: leader election (PartitionRaftServer.java:85,89) */
  uint64_t last_log_term;      /* Raft's lastLogTerm: the newest term whose leader-start entry this
                                  replica's log holds (its own term once it leads; on a follower the
                                  term of the last round entry it accepted that reached its leader's
                                  term start; 0 = unknown, after a catch-up that ended below its
                                  leader's term start: rmq_vote then compares against an upper bound,
                                  the leader's term - 1, while a candidacy claims 0) */
  uint64_t voted_term;         /* the term of this replica's last vote (raft_meta votedFor's term) */
  uint32_t voted_for;          /* the rank it voted for in voted_term (RMQ_NO_VOTE: none) */
  uint32_t led;                /* 1: this replica led voted_term (rmq_become_leader succeeded in it) */
  uint64_t heard_round;        /* the round stamp at which this replica last heard its partition's
                                  leader (a round entry or a commit notice of the current term);
                                  rmq_leader_silent compares it with the engine's round count */
} rmq_partition_state;

typedef struct rmq_append_stats {
  uint32_t records;            /* records submitted */
  uint32_t appended;           /* records given offsets */
  uint32_t rejected_not_leader;
  uint32_t rejected_no_partition;
  uint32_t rejected_no_space;  /* records of partitions whose record bytes in this batch exceed
                                  segment - interval (FORMAT.md §3: the partition takes none) */
  uint32_t rejected_invalid;   /* device batches only: whole batch rejected, a payload range lies
                                  outside payload_bytes (host batches get RMQ_EINVAL instead) */
} rmq_append_stats;

typedef struct rmq_repl_stats {
  uint32_t world, rank;
  uint32_t out_entries;        /* (led partition, remote slot) pairs this engine sends rounds for */
  uint32_t in_entries;         /* (followed partition, local slot) pairs it receives rounds for */
  uint64_t rounds;             /* replication rounds posted (one per launch group) */
  uint64_t bytes_sent;         /* round regions sent (FORMAT.md §9), all peers */
  uint64_t bytes_received;
  uint64_t records_ingested;   /* follower records whose CRC32C and log position checked out */
  uint64_t refused_crc;        /* follower entries refused: a record's CRC32C / header / bounds is wrong */
  uint64_t refused_log;        /* follower entries refused: do not continue the follower's log, stale
                                  leader term, or the round missed (no region from the leader) */
  uint64_t bytes_ingested;
  uint64_t catchup_entries;    /* leader: entries that re-sent a follower's gap (FORMAT.md §9 catch-up) */
  uint64_t detached_plans;     /* leader: entry plans whose follower lies beyond the ring and no rebase point was complete (FORMAT.md §9) */
  uint64_t general_plans;      /* leader: destination plans by the general path (a consumer-offset row or
                                  a catch-up gap among the entries, or over 4,096 entries); the
                                  steady-state plan covers the rest. A diagnostic of the round's cost */
  uint64_t host_waits;         /* rounds whose {bytes, records} swap had not landed when the host
                                  posted the round (RCCL's send/recv take host-side byte counts) */
  uint64_t host_wait_ns;       /* host time spent in those waits */
} rmq_repl_stats;

typedef struct rmq_engine rmq_engine;
typedef struct rmq_local_hub rmq_local_hub;

uint32_t rmq_abi_version(void);
const char* rmq_strerror(int status);
/* Fills a config with the defaults documented in DESIGN.md for P partitions and RF replicas. */
void rmq_config_default(rmq_config* cfg, uint32_t num_partitions, uint32_t replication_factor);

int rmq_create(const rmq_config* cfg, rmq_engine** out);
void rmq_destroy(rmq_engine* e);

/* Replica placement of one partition (reference: the Configuration(peers) of its raft group).
   replica_ranks[slot] = rank holding that replica; leader_slot names the leader replica.
   The engine leads pidx iff replica_ranks[leader_slot] == cfg.rank. rf must equal cfg RF. */
int rmq_set_replicas(rmq_engine* e, uint32_t pidx, const uint32_t* replica_ranks, uint32_t rf,
                     uint32_t leader_slot);
/* Placement of n partitions at once (one drain): for partition pidx[i], replica_ranks[i * RF + slot]
   and leader_slot[i] as in rmq_set_replicas, and key[i] (nullable: keys unchanged, default pidx) a
   cluster-wide id of the partition (its groupId) that orders replication lists identically on
   every rank (FORMAT.md §9). With a transport attached this is collective and checks every pair of
   ranks agrees on what they replicate to each other (RMQ_EINVAL on every rank if not). */
int rmq_set_placement(rmq_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* key,
                      const uint32_t* replica_ranks, const uint32_t* leader_slot);

/* Ring sizes of n partitions (reference: per-topic log retention; the reference keeps every
   message in memory, PartitionStateMachine.java:26,66): segment_bytes[i] (power of two, at least
   4 * index_interval) for partition pidx[i], allocated from the engine's pool. A shrinking ring
   first applies retention at the new size (FORMAT.md §4 rule); the retained records, their bytes in
   every local replica and their index entries keep their offsets and logical positions. All or
   nothing: RMQ_ENOMEM (nothing changed) if the pool cannot hold the new rings. Drains first (with a
   transport attached: collective, like rmq_sync). */
int rmq_set_segments(rmq_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* segment_bytes);

/* New leader term for pidx (or RMQ_ALL_PARTITIONS): term_start = log_end_offset, so only
   entries appended in this term can advance the commit (Raft current-term rule). */
int rmq_become_leader(rmq_engine* e, uint32_t pidx, uint64_t term);
/* Raft RequestVote on this replica (jraft's election, PartitionRaftServer.java:85; the vote persists
   in raft_meta, :89): a request of an older term is denied; a newer term is adopted first (a leader
   of pidx steps down: it stops accepting appends, offset commits and fetches); the vote is granted
   when this replica has not voted for another candidate in `term` and the candidate's log is at least
   as up to date, (cand_last_log_term, cand_log_end) >= (last_log_term, log_end_offset) in that order.
   *granted = 1 records the vote (voted_term = term, voted_for = candidate). A candidate votes for
   itself through this call too, then rmq_become_leader(pidx, term) once a quorum granted.
   Without a transport the batches submitted are applied first. With one nothing is flushed (a flush
   is collective): the call waits for what is issued only, and a replica that leads pidx with launch
   groups still in flight answers RMQ_PENDING with nothing changed (the request is delayed: send it
   again after the next rmq_sync). */
int rmq_vote(rmq_engine* e, uint32_t pidx, uint64_t term, uint32_t candidate, uint64_t cand_last_log_term,
             uint64_t cand_log_end, uint32_t* granted);
/* Replay of a persisted vote (raft_meta): voted_term / voted_for of pidx, and the term if newer. */
int rmq_set_vote(rmq_engine* e, uint32_t pidx, uint64_t term, uint32_t voted_for);
/* Partitions this replica follows whose leader has been silent (jraft's election timeout, 1000 ms,
   PartitionRaftServer.java:85): no round entry or commit notice of the current term from the leader
   in the last `silent_rounds` rounds (heard_round + silent_rounds <= the engine's round count) AND
   none for at least timeout_ms of wall time. out_pidx gets at most cap of them in ascending order,
   *n = how many there are. A placement change restarts every partition's timer. */
int rmq_leader_silent(rmq_engine* e, uint32_t silent_rounds, uint32_t timeout_ms, uint32_t* out_pidx,
                      uint32_t cap, uint32_t* n);

/* Append one batch. Assigns offsets (stable per partition, in batch order), writes the records
   with CRC32C into every local replica log, advances the offset index, the quorum commit and
   the high watermark. Asynchronous: returns a ticket; caller buffers must stay valid until
   rmq_poll_commit(ticket) returns RMQ_OK. out_offsets (same memory kind as the batch) gets the
   offset of each record, or RMQ_OFFSET_NONE if it was rejected (unknown pidx / not leader / no
   space). A partition whose record bytes in this batch (sum of 16 + align16(len)) exceed
   segment_bytes - index_interval takes none of the batch's records (rmq_ticket_stats reports them
   as rejected_no_space); the batch's other partitions are unaffected.
   Batches are collected into launch groups of up to cfg.pipeline_depth: the call that fills a
   group issues one kernel launch that ranks it and advances the three groups submitted before
   it (scan, apply, retention); every batch keeps its own semantics. A batch is applied by the
   second launch after its group's own, or when rmq_poll_commit / rmq_ticket_stats / rmq_sync /
   any control call closes the forming group and flushes the pipeline. */
int rmq_append(rmq_engine* e, const rmq_batch* batch, uint64_t* out_offsets, uint64_t* ticket);

/* External replica acks (followers on other ranks): match[slot] = max(match[slot],
   min(value, log_end_offset)),
   then the quorum commit rule is re-evaluated for those partitions. Host arrays of n. */
int rmq_ack(rmq_engine* e, const uint32_t* pidx, const uint32_t* replica_slot,
            const uint64_t* match, uint32_t n);

/* Append tickets: RMQ_OK if every operation up to `ticket` completed (then commit/hw snapshots of all
   P partitions are copied to the optional host arrays), RMQ_PENDING if not yet.
   Consumer-offset tickets (RMQ_TICKET_OFFSETS set, from rmq_commit_consumer_offset): RMQ_OK once the
   consumer-offset row of every partition the call committed to, as of that call or newer, is held
   by a quorum of the partition's replicas (co-located replicas hold it once applied; a remote one
   once it accepted a round carrying it, FORMAT.md §8) — the reference's PartitionClosure answering a
   ConsumerOffsetUpdateRequest after the Raft commit (ConsumerOffsetUpdateRequestProcessor.java:40-49,
   60, PartitionClosure.java:32-36); RMQ_PENDING until then; RMQ_ENOTLEADER if this engine stopped
   leading one of those partitions first (the commit may be lost, like a jraft closure failed by a
   leader change). A resolved offset ticket is forgotten (a second poll: RMQ_EINVAL). Never flushes. */
int rmq_poll_commit(rmq_engine* e, uint64_t ticket, uint64_t* commit_out, uint64_t* hw_out);
int rmq_ticket_stats(rmq_engine* e, uint64_t ticket, rmq_append_stats* out);
int rmq_sync(rmq_engine* e);

/* Consumer-offset commits, applied in array order: last writer wins, no bounds or monotonic
   check (PartitionStateMachine.java:71-77). status (nullable, host, [n]) reports per item (not
   leader, unknown partition, bad consumer id). The items reach the device table in order with the
   append stream (one copy on the pipeline stream, no wait for the pipeline): a later rmq_fetch or
   read-back sees them. With a replication transport the partition's row travels to every follower
   with the next round (FORMAT.md §8, §9). ticket (nullable) gets a consumer-offset ticket
   (RMQ_TICKET_OFFSETS set) that rmq_poll_commit resolves once the accepted items are on a quorum;
   0 if no item was accepted. The engine keeps the 256 newest unpolled offset tickets: an older
   one polls as RMQ_EINVAL. */
int rmq_commit_consumer_offset(rmq_engine* e, const uint32_t* pidx, const uint32_t* consumer,
                               const uint64_t* offset, uint32_t n, int32_t* status, uint64_t* ticket);
/* ABI 10: the replica cursors of n partitions (where RMQ_FETCH_REPLICA reads start): a durable
   tier's end after it reopens its files. Local to this engine (no round carries it); ordered with
   the pipeline stream like a consumer-offset commit. */
int rmq_set_replica_cursor(rmq_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* offset);

/* Batched consumer fetch: for each request, off = committed consumer offset (default 0),
   returns records [off, min(off + max, high_watermark)) (PartitionStateMachine.java:85-110).
   Records are copied in FORMAT.md layout, request after request, into `out` (mem kind `mem`).
   reqs/res are host arrays. Synchronous. Returns RMQ_OK, or RMQ_ENOSPC if some request did not
   fit in out_cap (those get count 0, status RMQ_ENOSPC). */
int rmq_fetch(rmq_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint32_t mem, uint8_t* out,
              uint64_t out_cap, rmq_fetch_res* res, uint64_t* bytes_used);
/* rmq_fetch without blocking the host (ABI 6). The fetch is ordered after every launch and call
   issued before it and before the ones issued after it, exactly like rmq_fetch, and returns at once
   with a fetch ticket; reqs are copied before the call returns. res (and out with RMQ_MEM_HOST)
   must stay valid until rmq_fetch_poll returns something other than RMQ_PENDING. Four fetches can
   be in flight: a fifth first completes the oldest into its caller's arrays (its poll then returns
   at once). MessageBatchReadRequestProcessor.java:36-42 answers each read from its own closure;
   this is the batched, pipelined form of that call.
   mem | RMQ_FETCH_PINNED_ROWS (ABI 7; rmq_fetch too): reqs and res are page-locked host memory
   (rmq_host_alloc or rmq_host_register): the fetch kernels read the request rows and write the
   result rows there themselves, with no copy (rows the runtime cannot map are staged like ordinary
   ones). The caller then keeps reqs unchanged until the ticket completes (as with pinned batches);
   res is written before the poll that returns the result.
   mem | RMQ_FETCH_DEVICE_ROWS (ABI 9; rmq_fetch too): reqs and res are device memory (a broker whose
   requests arrive on the GPU): no transfer at all. The host never sees these requests, so their
   flags word must be 0 (RMQ_FETCH_COMMIT needs host rows: the call checks them) and is ignored. */
#define RMQ_FETCH_PINNED_ROWS 0x100u
#define RMQ_FETCH_DEVICE_ROWS 0x200u
int rmq_fetch_async(rmq_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint32_t mem, uint8_t* out,
                    uint64_t out_cap, rmq_fetch_res* res, uint64_t* ticket);
/* Completion of an rmq_fetch_async ticket: RMQ_PENDING while it runs (wait != 0: block instead), else
   what rmq_fetch would have returned (RMQ_OK / RMQ_ENOSPC) with res, out and *bytes_used filled. A
   ticket is answered once; an unknown or already answered ticket gets RMQ_EINVAL. */
int rmq_fetch_poll(rmq_engine* e, uint64_t ticket, uint32_t wait, uint64_t* bytes_used);

/* ---- replication transport (FORMAT.md §9) ---- */
/* 128-byte communicator id: one rank creates it, the application hands it to every rank. */
int rmq_rccl_unique_id(uint8_t* out /* 128 bytes */);
/* RCCL over xGMI between the world's engines, one per GPU and process; rank = cfg.rank. Collective. */
int rmq_attach_rccl(rmq_engine* e, const uint8_t* comm_id, uint32_t world);
/* In-process transport: engines of one process exchange by device copies; each rank's engine must
   be driven by its own host thread (the hub's barriers stand in for the collective). */
int rmq_local_hub_create(uint32_t world, rmq_local_hub** out);
void rmq_local_hub_destroy(rmq_local_hub* hub);
int rmq_attach_local(rmq_engine* e, rmq_local_hub* hub);
int rmq_replication_stats(rmq_engine* e, rmq_repl_stats* out);
/* Region bytes of the last posted round for destination rank dst (FORMAT.md §9): *size gets its
   length; copied to out if out != NULL and cap suffices (tests, tools). */
int rmq_read_outbox(rmq_engine* e, uint32_t dst, uint8_t* out, uint64_t cap, uint64_t* size);
/* Fault injection (tests): the rounds of the next n launch groups this engine forms from batches
   appended after the call send empty regions, as if the leader failed before replicating them
   (its own log keeps the records; followers neither see nor ack them). Not collective. */
int rmq_fault_drop_rounds(rmq_engine* e, uint32_t n);
/* Fault injection (tests): the regions of the next n rounds this engine sends to rank dst are lost
   (launch groups formed from batches appended after the call), as a failed link to dst would lose
   them: dst misses those rounds (every entry refused); its other peers and the commit notices of a
   drain still reach it. Not collective. */
int rmq_fault_isolate(rmq_engine* e, uint32_t dst, uint32_t n);
/* Fault injection (tests): as rmq_fault_isolate, and the commit notices of the next drain to dst are
   lost as well: a network partition between this leader and dst (dst's rmq_leader_silent reports the
   partitions this engine leads toward it). Not collective. */
int rmq_fault_cut(rmq_engine* e, uint32_t dst, uint32_t n);
/* Fault injection (tests): the next round this engine sends to rank dst has the byte at `at` of its
   region XORed with 0x5A (at < 0: counted back from the end of the region's data section, i.e. a
   payload byte of its last record), as a link or memory corruption would; the follower refuses the
   entry it hits and the leader's catch-up re-sends it (FORMAT.md §9). Not collective. */
int rmq_fault_corrupt(rmq_engine* e, uint32_t dst, int64_t at);

/* ---- read-back (tests, tools) ---- */
int rmq_get_partition_state(rmq_engine* e, uint32_t pidx, rmq_partition_state* out);
/* The states of partitions [first, first + n) at once (one device copy per field). */
int rmq_get_partition_states(rmq_engine* e, uint32_t first, uint32_t n, rmq_partition_state* out);
/* Raw ring bytes [ring_off, ring_off + len) of replica slot `replica` of pidx. */
int rmq_read_segment(rmq_engine* e, uint32_t replica, uint32_t pidx, uint64_t ring_off,
                     uint64_t len, uint8_t* out);
/* Offset-index entries m in [m_first, m_first + count): out[2k] = offset, out[2k+1] = pos. */
int rmq_read_index(rmq_engine* e, uint32_t pidx, uint64_t m_first, uint64_t count, uint64_t* out);
int rmq_read_consumer_offsets(rmq_engine* e, uint32_t pidx, uint64_t* out /* max_consumers */);
/* The consumer-offset rows of partitions [first, first + n): out[n][max_consumers]. */
int rmq_read_consumer_table(rmq_engine* e, uint32_t first, uint32_t n, uint64_t* out);

/* ---- host utilities ---- */
/* FORMAT.md §1 records laid back to back in host memory (segment files of a durable tier, fetch
   output): walks them from buf[0], expecting header offsets first, first + 1, ..., and stops at the
   first record that is out of sequence or cut short, or (flags & RMQ_SCAN_CHECK) whose CRC32C or
   zero padding is wrong, or after max_records. *count / *bytes = the whole records before that;
   pos_out (nullable, max_records + 1 slots) gets each one's byte position and then the end. Needs no
   engine (or GPU). */
#define RMQ_SCAN_CHECK 1u
int rmq_scan_records(const uint8_t* buf, uint64_t len, uint64_t first, uint64_t max_records, uint32_t flags,
                     uint64_t* pos_out, uint64_t* count, uint64_t* bytes);
/* Durable-tier spill (ripplemq_amd/tier.py; jraft's per-group log, PartitionRaftServer.java:53,88-90):
   run i = buf[buf_pos[i], buf_pos[i] + bytes[i]), count[i] back-to-back FORMAT.md §1 records with
   header offsets first[i], first[i] + 1, ... (as one rmq_fetch returns a partition's slice), is
   appended to the open file descriptor fd[i]; pos_out gets, run after run, each record's position
   inside its run and then the run's end (count[i] + 1 words per run). Runs are checked first
   (RMQ_EINVAL, nothing written); the writes go over `threads` threads (0: up to 8); fsync_each != 0
   fsyncs every file. RMQ_EDEVICE on an I/O error (errno set). Needs no engine (or GPU). */
int rmq_tier_append(uint32_t n, const int32_t* fd, const uint64_t* first, const uint64_t* count,
                    const uint64_t* buf_pos, const uint64_t* bytes, const uint8_t* buf, uint64_t* pos_out,
                    uint32_t threads, int fsync_each);

/* ---- device buffers and timing (bench / tests keep inputs resident in HBM) ---- */
int rmq_device_alloc(rmq_engine* e, uint64_t bytes, void** out);
int rmq_device_free(rmq_engine* e, void* p);
int rmq_memcpy(rmq_engine* e, void* dst, const void* src, uint64_t bytes, int kind /*0 h2d,1 d2h,2 d2d*/);
/* Page-locked host memory for RMQ_MEM_PINNED batches (reference side: the JNI layer's direct
   ByteBuffers): allocate, or register / unregister existing pages. */
int rmq_host_alloc(rmq_engine* e, uint64_t bytes, void** out);
int rmq_host_free(rmq_engine* e, void* p);  /* e may be NULL (buffers outliving the engine) */
int rmq_host_register(rmq_engine* e, void* p, uint64_t bytes);
int rmq_host_unregister(rmq_engine* e, void* p);
/* Kernel timing with HIP events on the engine's stream (enable != 0 turns it on and resets it).
   kernels 0 and 1: the pipeline launches from the first one after enable up to the next drain
   (sync, control call, read-back) timed as ONE region (no events between launches): total_ms =
   region time; launches = pipeline launches in it (kernel 0) or batches they applied (kernel 1).
   kernel 3: rmq_fetch, the summed dispatch-recorded spans of its kernels; 4: rmq_fetch, an event
   before its first kernel to one after its last (the request copy before and the result copy after
   outside), launches = kernel executions. enable = k >= 2 also runs every fetch's kernels k times
   back to back (idempotent: the same results), so kernel 4 / launches is a kernel time that no
   copy or host gap inflates and a rocprofv3 trace shows the kernels back to back; a fetch with an
   RMQ_FETCH_COMMIT request runs once (each run would commit). 2: unused. */
int rmq_profile_enable(rmq_engine* e, int enable);
int rmq_profile_query(rmq_engine* e, int kernel, uint64_t* launches, double* total_ms);
/* Device name / CU count for reports. */
int rmq_device_info(rmq_engine* e, char* name, uint32_t name_cap, uint32_t* cu_count);

#ifdef __cplusplus
}
#endif
#endif /* RIPPLEMQ_ENGINE_H */
