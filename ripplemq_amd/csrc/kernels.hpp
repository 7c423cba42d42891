// kernels.hpp — launch interface between the host engine (engine.cpp) and the gfx950 kernels.
// Plain structs of device pointers; no torch types, no host STL.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rmq {

constexpr uint32_t kPipeThreads = 512;   // 8 waves per workgroup, every role of the pipeline launch
constexpr uint32_t kTileRecs = 1024;     // records per ranking tile (stage 1)
constexpr uint32_t kTileIdxBits = 10;    // log2(kTileRecs)
constexpr uint32_t kMaxTiles = 256;      // max_batch_records <= kMaxTiles * kTileRecs
constexpr uint32_t kScanLanes = 8;       // stage 2: threads per partition column
constexpr uint32_t kTaskRecs = 32;       // records per apply task (one wave, 2 lanes per record)
constexpr uint32_t kMaxPartitions = 1u << 16;  // 16-bit partition keys (two 8-bit LDS radix passes)
constexpr uint32_t kMaxRF = 8;

struct CrcConsts;

// Per-partition device state (SoA, [P] unless noted). Owned by the engine.
struct DevState {
  // leo / used / start_off / start_pos point at the CURRENT state set (see StateSet)
  uint64_t* leo;         // log end offset (next offset)
  uint64_t* used;        // log end byte position (logical)
  uint64_t* start_off;   // retained log start
  uint64_t* start_pos;
  uint64_t* commit;
  uint64_t* hw;
  uint64_t* term_start;
  uint64_t* match;       // [P][RF]
  uint32_t* is_leader;   // 0/1
  uint32_t* local_mask;  // bit r set: replica slot r is stored on this device
  uint64_t* index;       // [P][icap][2] sparse offset index {offset, pos}
  uint8_t* logs;         // [RF][P][seg] ring segments
  uint64_t* cons;        // [P][C] consumer offsets
  uint32_t P, RF, C;
  uint32_t icap;         // index ring entries per partition
  uint64_t seg;          // ring bytes (power of two)
  uint32_t interval_log2;
  uint32_t pad;
};

// Double-buffered per-partition log-position state: apply #a reads set a&1 and writes set (a+1)&1,
// so records can read their partition's batch-start state while its new state is being written.
struct StateSet {
  uint64_t* leo;
  uint64_t* used;
  uint64_t* start_off;
  uint64_t* start_pos;
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

// Batch-local scratch of one pipeline set (three sets rotate: a batch is ranked in launch k,
// scanned in launch k+1 and applied in launch k+2).
struct PipeScratch {
  uint64_t* hist;       // [tiles][P] tile aggregate {count << 40 | bytes/16}; 0 = absent (stage 2 clears)
  uint64_t* excl;       // [tiles][P] exclusive prefix of the aggregates over tiles (present entries only)
  uint64_t* totals;     // [P] batch aggregate per partition
  uint2* crank;         // [n] {rank in tile run | flags << 29, bytes/16 before it in the tile run}
  uint32_t* pre;        // [n] payload bytes before the record inside its tile (packed payloads)
  uint64_t* tsum;       // [tiles][4] {payload bytes, record bytes, invalid records, 0}
  uint64_t* tile_base;  // [tiles] payload offset of the tile's first record (packed payloads)
  uint64_t* binfo;      // [4] {reject flags (1 no space, 2 invalid), record bytes, payload bytes, 0}
};

// The single per-batch launch: stage 1 (rank tiles of batch k), stage 2 (column scans of batch
// k-1), stage 3 (apply batch k-2). Any stage may be absent (count 0).
struct PipeArgs {
  DevState st;
  StateSet cur, nxt;    // stage 3: read cur, write nxt
  PipeBatch b1, b2, b3;
  PipeScratch s1, s2, s3;
  uint32_t wg1, wg2, wg3;  // workgroups per stage, in this order along blockIdx.x
  uint32_t key_passes;     // 1 (P <= 256) or 2
  uint64_t nospace_limit;  // segment - interval
  const CrcConsts* crc;
  uint4* stats3;           // [tasks] {appended, not leader, unknown partition, no space | invalid << 16}
  uint64_t* done_word;     // host-visible: sequence number of the previous launch (written at start)
  uint64_t launch_seq;
  uint32_t debug;          // diagnostic only (RMQ_DEBUG, results invalid): 1 no payload ring
                           // stores, 2 no CRC lookups, 4 no payload loads
  uint32_t pad0;
  uint64_t* stamps;        // diagnostic only (RMQ_STAMPS): [workgroup][wave][8] s_memrealtime, or null
};

struct FetchArgs {
  DevState st;
  const uint32_t* req;       // [n][4] {pidx, consumer, max, reserved}
  uint64_t* res;             // [n][4] {start_offset, out_pos, count|bytes<<32, status}
  uint64_t* aux;             // [n][2] {source byte position, pidx}
  uint8_t* out;
  uint64_t out_cap;
  uint32_t n;
  uint32_t pad;
  uint64_t* total;           // [1] bytes needed
};

struct ConsumerCommitArgs {
  DevState st;
  const uint32_t* pidx;
  const uint32_t* consumer;
  const uint64_t* offset;
  uint64_t* winner;          // [P*C] {epoch:32 | item+1:32}, monotone across calls
  uint32_t n;
  uint32_t epoch;
};

struct AckArgs {
  DevState st;
  const uint32_t* pidx;
  const uint32_t* slot;
  const uint64_t* match;
  uint32_t n;
};

// launchers (defined in the .hip files)
void launch_pipeline(const PipeArgs& a, hipStream_t s);
uint32_t pipeline_lds_bytes();
uint32_t pipeline_wgs_per_cu();
void launch_commit_all(const DevState& st, hipStream_t s);
void launch_ack(const AckArgs& a, hipStream_t s);
void launch_become_leader(const DevState& st, uint32_t pidx, hipStream_t s);
void launch_fetch(const FetchArgs& a, hipStream_t s, hipEvent_t ev_resolve0, hipEvent_t ev_resolve1,
                  hipEvent_t ev_gather0, hipEvent_t ev_gather1);
void launch_consumer_commit(const ConsumerCommitArgs& a, hipStream_t s);

}  // namespace rmq
