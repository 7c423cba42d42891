// kernels.hpp — launch interface between the host engine (engine.cpp) and the gfx950 kernels.
// Plain structs of device pointers; no torch types, no host STL.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rmq {

constexpr uint32_t kSortThreads = 256;
constexpr uint32_t kSortItems = 8;
constexpr uint32_t kSortDigitBits = 8;                     // <= 256 buckets per radix pass
constexpr uint32_t kSortTile = kSortThreads * kSortItems;  // keys per sort tile
constexpr uint32_t kAppendThreads = 256;                    // 4 waves; one 64-slot tile per wave
constexpr uint32_t kAppendTile = 64;
constexpr uint32_t kAppendImageBytes = 8192;                // LDS record image per wave
constexpr uint32_t kMaxRF = 8;

struct CrcConsts;

// Per-partition device state (SoA, [P] unless noted). Owned by the engine.
struct DevState {
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

// One stable sort pass over the partition ids of a batch (see sort.hip).
struct SortPassArgs {
  const uint32_t* keys_in;      // first pass: raw pidx of the input batch
  const uint32_t* pidx_raw;     // raw pidx of the input batch (last pass of a multi-pass sort)
  const uint32_t* vals_in;      // later passes: record indices
  uint32_t* keys_out;           // intermediate passes
  uint32_t* vals_out;
  uint4* slots;                 // last pass: {pidx, record, len, payload offset} per slot
  const uint32_t* len;          // record payload lengths (input order)
  const uint64_t* payload_off;  // caller payload offsets, or nullptr (packed)
  uint32_t* src_off;            // packed payload offsets written by the first pass of a multi-pass sort
  uint64_t* batch_info;         // first pass: [0] record bytes, [1] payload bytes of the batch
  uint64_t* hist_gran;          // [tiles][256] tile digit counts {epoch | count}
  uint64_t* len_gran;           // [tiles] tile payload bytes {epoch | bytes}
  uint64_t* rb_gran;            // [tiles] tile record bytes {epoch | bytes}
  uint32_t n, tiles;
  uint32_t shift, bits, ndig;   // digit = (key >> shift) & ((1 << bits) - 1), ndig digits used
  uint32_t P;
  uint32_t first, last;
  uint32_t epoch;
  uint32_t* err;
  uint64_t* stamps;             // diagnostic build only: [tiles][8] s_memrealtime per phase, or null
};

struct AppendArgs {
  DevState st;
  const uint4* slots;        // sorted slot records {pidx, record, len | bad-partition flag, payload off}
  const uint8_t* payload;
  uint64_t payload_bytes;
  uint64_t* out_offsets;     // input order
  const uint64_t* batch_info;
  uint4* tile_stats;         // [tiles] {appended, not leader, unknown partition, no space}
  uint64_t* lb_cnt;          // [tiles] look-back granules {epoch<<2|status : record count}
  uint64_t* lb_bytes;        // [tiles] look-back granules {epoch<<2|status : record bytes}
  uint32_t n;
  uint32_t tiles;            // 64-slot tiles
  uint32_t epoch;
  uint32_t nospace_limit_lo, nospace_limit_hi;  // segment - interval (u64 split)
  const CrcConsts* crc;
  uint32_t* err;
  uint32_t spin_limit;
  uint32_t debug;            // diagnostics (RMQ_DEBUG_FLAGS): bit 2 no ring stores, bit 3 replica 0 only
  uint64_t* stamps;          // diagnostic build only: [tiles][8] s_memrealtime per phase, or null
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
void launch_sort_pass(const SortPassArgs& a, uint32_t tiles, hipStream_t s);
void launch_append(const AppendArgs& a, uint32_t grid, hipStream_t s);
void launch_commit_all(const DevState& st, hipStream_t s);
void launch_ack(const AckArgs& a, hipStream_t s);
void launch_become_leader(const DevState& st, uint32_t pidx, hipStream_t s);
void launch_fetch(const FetchArgs& a, hipStream_t s, hipEvent_t ev_resolve0, hipEvent_t ev_resolve1,
                  hipEvent_t ev_gather0, hipEvent_t ev_gather1);
void launch_consumer_commit(const ConsumerCommitArgs& a, hipStream_t s);
int append_blocks_per_cu();
int append_waves_per_block();

}  // namespace rmq
