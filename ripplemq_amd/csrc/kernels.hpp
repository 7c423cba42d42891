// kernels.hpp — launch interface between the host engine (engine.cpp) and the gfx950 kernels.
// Plain structs of device pointers; no torch types, no host STL.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rmq {

constexpr uint32_t kSortThreads = 512;
constexpr uint32_t kSortItems = 8;
constexpr uint32_t kSortTile = kSortThreads * kSortItems;  // keys per sort tile
constexpr uint32_t kAppendThreads = 256;                    // = slots per append tile
constexpr uint32_t kAppendImageBytes = 32768;               // LDS image budget per tile
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

// One append batch after the sort: slot s (sorted order) holds record vals[s] of partition keys[s].
struct SortPassArgs {
  const uint32_t* keys_in;   // pass 0: raw pidx of the input batch
  const uint32_t* vals_in;   // pass 0: nullptr (identity)
  uint32_t* keys_out;
  uint32_t* vals_out;
  uint32_t n;
  uint32_t shift, bits;      // digit = (key >> shift) & ((1 << bits) - 1)
  uint32_t P;                // pass 0 clamps key = min(pidx, P-1)
  uint32_t first;            // 1 on pass 0
  uint32_t epoch;
  uint64_t* hist_gran;       // [tiles][256]
  uint32_t tiles;
  uint64_t* len_gran;        // [tiles] payload bytes per tile (pass 0)
  uint64_t* rb_gran;         // [tiles] record bytes per tile (pass 0)
  const uint32_t* len;       // pass 0: record payload lengths
  uint32_t* src_off;         // pass 0: packed payload offsets out (nullptr if caller gave payload_off)
  uint64_t* batch_info;      // pass 0: [0] total record bytes
  uint32_t* stats;           // pass 0: zeroed stats slot [4]
  uint32_t* err;
};

struct AppendArgs {
  DevState st;
  const uint32_t* skeys;     // sorted keys [n]
  const uint32_t* svals;     // sorted record indices [n]
  const uint32_t* pidx;      // input order
  const uint32_t* len;
  const uint32_t* src_off32; // packed payload offsets (or nullptr)
  const uint64_t* src_off64; // caller payload offsets (or nullptr)
  const uint8_t* payload;
  uint64_t payload_bytes;
  uint64_t* out_offsets;     // input order
  const uint64_t* batch_info;
  uint32_t* stats;           // [4] appended, not_leader, no_partition, no_space
  uint64_t* lb_status;       // [tiles] look-back granules
  uint64_t* lb_abs;          // [tiles][2] absolute {offset, pos} at tile end (INCLUSIVE)
  uint64_t* tile_counter;    // monotonic dynamic tile ticket
  uint64_t tile_base;        // value of *tile_counter at launch
  uint32_t n;
  uint32_t tiles;
  uint32_t epoch;
  uint32_t nospace_limit_lo, nospace_limit_hi;  // segment - interval (u64 split)
  const CrcConsts* crc;
  uint32_t* err;
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

}  // namespace rmq
