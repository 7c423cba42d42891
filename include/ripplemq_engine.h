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
 *   rmq_set_replicas            <- PartitionRaftServer.setupRaft initial Configuration(peers)
 *                                  (mq-broker/src/main/java/metadata/raft/PartitionRaftServer.java:82-86)
 *   rmq_create / rmq_destroy    <- PartitionManager.startPartition / PartitionRaftServer.shutdown
 *                                  (PartitionManager.java:166-176, PartitionRaftServer.java:100-108)
 *
 * Only dense partition indices (pidx) cross this boundary; the Java side keeps the
 * "topic-partitionId" -> pidx map (PartitionManager.java:121,196-198).
 *
 * Threading: one submitter thread per engine for rmq_append / rmq_ack /
 * rmq_commit_consumer_offset / rmq_become_leader / rmq_set_replicas. rmq_fetch, rmq_poll_commit
 * and the read-back calls may be called from any thread (they serialize on an internal lock).
 * Completion is by polling tickets; the library never calls back into the host.
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

#define RMQ_ABI_VERSION 1u
#define RMQ_MAX_RF 8u
#define RMQ_ALL_PARTITIONS 0xFFFFFFFFu
#define RMQ_OFFSET_NONE 0xFFFFFFFFFFFFFFFFull /* out_offsets value of a rejected record */
#define RMQ_RECORD_HEADER_BYTES 16u
#define RMQ_RECORD_ALIGN 16u /* records start and end on 16-byte boundaries (FORMAT.md §1) */

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
  RMQ_ENOMEM = -7
};

/* Memory kind of caller buffers. */
enum { RMQ_MEM_HOST = 0, RMQ_MEM_DEVICE = 1 };

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
} rmq_config;

/* One append batch: records of many partitions, interleaved, in apply order (SoA). */
typedef struct rmq_batch {
  uint32_t n;                  /* number of records */
  uint32_t mem;                /* RMQ_MEM_HOST or RMQ_MEM_DEVICE for every pointer below */
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
  uint32_t reserved;
} rmq_fetch_req;

typedef struct rmq_fetch_res {
  uint64_t start_offset;       /* reference: MessageBatchReadResponse.offset (the consumer offset) */
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

typedef struct rmq_engine rmq_engine;

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
/* New leader term for pidx (or RMQ_ALL_PARTITIONS): term_start = log_end_offset, so only
   entries appended in this term can advance the commit (Raft current-term rule). */
int rmq_become_leader(rmq_engine* e, uint32_t pidx, uint64_t term);

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

/* RMQ_OK if every operation up to `ticket` completed (then commit/hw snapshots of all P
   partitions are copied to the optional host arrays), RMQ_PENDING if not yet. */
int rmq_poll_commit(rmq_engine* e, uint64_t ticket, uint64_t* commit_out, uint64_t* hw_out);
int rmq_ticket_stats(rmq_engine* e, uint64_t ticket, rmq_append_stats* out);
int rmq_sync(rmq_engine* e);

/* Consumer-offset commits, applied in array order: last writer wins, no bounds or monotonic
   check (PartitionStateMachine.java:71-77). status (nullable, host, [n]) reports per item. */
int rmq_commit_consumer_offset(rmq_engine* e, const uint32_t* pidx, const uint32_t* consumer,
                               const uint64_t* offset, uint32_t n, int32_t* status);

/* Batched consumer fetch: for each request, off = committed consumer offset (default 0),
   returns records [off, min(off + max, high_watermark)) (PartitionStateMachine.java:85-110).
   Records are copied in FORMAT.md layout, request after request, into `out` (mem kind `mem`).
   reqs/res are host arrays. Synchronous. Returns RMQ_OK, or RMQ_ENOSPC if some request did not
   fit in out_cap (those get count 0, status RMQ_ENOSPC). */
int rmq_fetch(rmq_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint32_t mem, uint8_t* out,
              uint64_t out_cap, rmq_fetch_res* res, uint64_t* bytes_used);

/* ---- read-back (tests, tools) ---- */
int rmq_get_partition_state(rmq_engine* e, uint32_t pidx, rmq_partition_state* out);
/* Raw ring bytes [ring_off, ring_off + len) of replica slot `replica` of pidx. */
int rmq_read_segment(rmq_engine* e, uint32_t replica, uint32_t pidx, uint64_t ring_off,
                     uint64_t len, uint8_t* out);
/* Offset-index entries m in [m_first, m_first + count): out[2k] = offset, out[2k+1] = pos. */
int rmq_read_index(rmq_engine* e, uint32_t pidx, uint64_t m_first, uint64_t count, uint64_t* out);
int rmq_read_consumer_offsets(rmq_engine* e, uint32_t pidx, uint64_t* out /* max_consumers */);

/* ---- device buffers and timing (bench / tests keep inputs resident in HBM) ---- */
int rmq_device_alloc(rmq_engine* e, uint64_t bytes, void** out);
int rmq_device_free(rmq_engine* e, void* p);
int rmq_memcpy(rmq_engine* e, void* dst, const void* src, uint64_t bytes, int kind /*0 h2d,1 d2h,2 d2d*/);
/* Kernel timing with HIP events on the engine's stream (enable != 0 turns it on and resets it).
   kernels 0 and 1: the pipeline launches from the first one after enable up to the next drain
   (sync, control call, read-back) timed as ONE region (no events between launches): total_ms =
   region time; launches = pipeline launches in it (kernel 0) or batches they applied (kernel 1).
   kernels 3 / 4: fetch-resolve / fetch-gather, one event pair per launch. 2: unused. */
int rmq_profile_enable(rmq_engine* e, int enable);
int rmq_profile_query(rmq_engine* e, int kernel, uint64_t* launches, double* total_ms);
/* Device name / CU count for reports. */
int rmq_device_info(rmq_engine* e, char* name, uint32_t name_cap, uint32_t* cu_count);

#ifdef __cplusplus
}
#endif
#endif /* RIPPLEMQ_ENGINE_H */
