/*
 * ripple_oracle.h — CPU restatement of RippleMQ's partition state machine (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle for the MI355X engine. It is NOT part of the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker
 * (or as the timed CPU baseline). The engine library never links or calls it.
 *
 * It restates, record by record in apply order, what the reference computes:
 *   - PartitionStateMachine.handleMessageAppendRequest: messages.addAll(batch), so the record j of
 *     an applied entry gets offset size_before + j  (mq-broker/src/main/java/metadata/raft/
 *     PartitionStateMachine.java:64-69; apply loop :38-62);
 *   - handleConsumerOffsetUpdateRequest: consumerOffsets.put(id, off), last writer wins (:71-77);
 *   - handleBatchRead: off = getOrDefault(id, 0); messages[off, min(off + max, size)) (:85-110);
 *   - the "Not leader" gate of the three processors (MessageAppendRequestProcessor.java:29-32,
 *     MessageBatchReadRequestProcessor.java:29-33, ConsumerOffsetUpdateRequestProcessor.java:31-35),
 *     as a documented divergence: the engine rejects instead of continuing;
 *   - the Raft quorum-commit rule that jraft's BallotBox implements (third-party
 *     com.alipay.sofa:jraft-core:1.3.15, not present in the container — restated from the Raft
 *     paper: commit = max(commit, k-th largest matchIndex, k = RF/2+1) gated on the current term).
 * plus the build-defined byte format of FORMAT.md (record header, CRC32C, ring segments, sparse
 * offset index, size retention), which has no reference counterpart.
 *
 * Parity pins: CRC32C against the RFC 3720 §B.4 known-answer vectors; offsets / fetch slices /
 * consumer offsets against a literal Python restatement of PartitionStateMachine.java
 * (tests/refmodel.py); commit indices vs jraft are UNPINNED (no JVM, no jraft jar here).
 */
#ifndef RIPPLE_ORACLE_H
#define RIPPLE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/ripplemq_engine.h" /* shared result structs only */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ro_engine ro_engine;

uint32_t ro_crc32c_bitwise(const uint8_t* p, size_t n); /* definitional, 1 bit per step */
uint32_t ro_crc32c(const uint8_t* p, size_t n);         /* table (or SSE4.2) implementation */
int ro_crc32c_hw_available(void);

ro_engine* ro_create(const rmq_config* cfg);
void ro_destroy(ro_engine* e);
int ro_set_replicas(ro_engine* e, uint32_t pidx, const uint32_t* ranks, uint32_t rf, uint32_t leader_slot);
int ro_become_leader(ro_engine* e, uint32_t pidx, uint64_t term);
int ro_append(ro_engine* e, uint32_t n, const uint32_t* pidx, const uint32_t* len,
              const uint64_t* payload_off, const uint8_t* payload, uint64_t payload_bytes,
              uint64_t* out_offsets, rmq_append_stats* stats);
/* Partition-sharded ro_append over nb batches (the CPU baseline's multi-core leg):
   thread t of `threads` applies, batch after batch, the records of the partitions p with
   p % threads == t. Same results as ro_append per batch; *batches_done = batches applied before
   the first error. pin != 0 pins thread t to the t-th CPU this process may run on. */
int ro_append_sharded(ro_engine* e, uint32_t nb, const rmq_batch* batches, uint64_t* const* out_offsets,
                      rmq_append_stats* stats, uint32_t threads, int pin, uint32_t* batches_done);
/* First touch of ring bytes [0, min(segment, bytes[p])) of every local replica of every partition
   (untimed setup, so a timed run does not pay page faults the device rings never see). */
int ro_reserve(ro_engine* e, const uint64_t* bytes);
int ro_set_segments(ro_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* seg);
int ro_ack(ro_engine* e, const uint32_t* pidx, const uint32_t* slot, const uint64_t* match, uint32_t n);
int ro_commit_consumer_offset(ro_engine* e, const uint32_t* pidx, const uint32_t* consumer,
                              const uint64_t* offset, uint32_t n, int32_t* status);
int ro_set_replica_cursor(ro_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* offset);
int ro_fetch(ro_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint8_t* out, uint64_t out_cap,
             rmq_fetch_res* res, uint64_t* bytes_used);

int ro_get_partition_state(ro_engine* e, uint32_t pidx, rmq_partition_state* out);
int ro_get_partition_states(ro_engine* e, uint32_t first, uint32_t n, rmq_partition_state* out);
int ro_read_segment(ro_engine* e, uint32_t replica, uint32_t pidx, uint64_t ring_off, uint64_t len,
                    uint8_t* out);
int ro_read_index(ro_engine* e, uint32_t pidx, uint64_t m_first, uint64_t count, uint64_t* out);
int ro_read_consumer_offsets(ro_engine* e, uint32_t pidx, uint64_t* out);
/* Logical position of record `offset` (dense, for cross-checking the sparse index). */
int ro_record_pos(ro_engine* e, uint32_t pidx, uint64_t offset, uint64_t* pos);

/* Replication rounds (FORMAT.md §9 v3): world > 1 makes the leader keep each round's
   records; the caller closes a round after the batches the engine groups into one launch group.
   ro_round_region plans without changing state (it may be called twice per destination: size, then
   bytes); ro_end_round applies the plan's per-entry state (catch-up next / round, consumer-offset
   rows sent) and starts the next round. Acks are 2 words per entry: {log end offset | status << 62,
   log end position}; ro_apply_acks takes the round number they answer (ro_round_no before the
   round's ro_end_round). */
int ro_set_world(ro_engine* e, uint32_t world);
int ro_set_key(ro_engine* e, uint32_t pidx, uint64_t key);
int ro_round_region(ro_engine* e, uint32_t dst, uint8_t* out, uint64_t cap, uint64_t* size);
void ro_end_round(ro_engine* e);
uint64_t ro_round_no(ro_engine* e);
int ro_ingest(ro_engine* e, uint32_t src, const uint8_t* region, uint64_t size, uint64_t* acks);
int ro_apply_acks(ro_engine* e, uint32_t dst, const uint64_t* acks, uint32_t n_acks, uint64_t round);
uint32_t ro_pair_entries(ro_engine* e, uint32_t src, uint32_t dst);
/* Commit notices (a drain's heartbeat, FORMAT.md §9 v4): 2 words per entry of the pair {commit, term}. */
int ro_commit_notice(ro_engine* e, uint32_t dst, uint64_t* out);
int ro_apply_notice(ro_engine* e, uint32_t src, const uint64_t* in, uint32_t n);
/* Consumer-offset rows on a quorum (offset tickets, FORMAT.md §8): partition p's row version and the
   newest version a quorum of its replicas holds. */
int ro_offset_quorum(ro_engine* e, uint32_t p, uint64_t* cver, uint64_t* cq);
/* [0] records ingested, [1] entries refused (CRC), [2] refused (log / term / missed round),
   [3] bytes ingested, [4] catch-up entries sent, [5] detached entry plans (gap beyond the ring) */
void ro_counters(ro_engine* e, uint64_t* out /* [6] */);
/* Leader election (rmq_vote, rmq_set_vote, rmq_leader_silent without its wall-clock part). */
int ro_vote(ro_engine* e, uint32_t pidx, uint64_t term, uint32_t candidate, uint64_t cand_last_log_term,
            uint64_t cand_log_end, uint32_t* granted);
int ro_set_vote(ro_engine* e, uint32_t pidx, uint64_t term, uint32_t voted_for);
int ro_leader_silent(ro_engine* e, uint32_t silent_rounds, uint32_t* out_pidx, uint32_t cap, uint32_t* n);
/* Catch-up reserve per destination (FORMAT.md §9): pipeline_depth x (39 max_batch_records +
   max_batch_bytes) bytes. */
uint64_t ro_catchup_reserve(const rmq_config* cfg);

#ifdef __cplusplus
}
#endif
#endif
