// engine.cpp — host side of the C-ABI (include/ripplemq_engine.h).
//
// Owns all device memory of one engine (one HIP device): per-(replica, partition) ring segments,
// the sparse offset index, per-partition Raft state and consumer offsets. Orchestrates, per
// append batch, the batch-local partition sort on a prep stream and the fused append kernel on
// the main stream, with `pipeline_depth` batches in flight so the sort of batch k+1 overlaps the
// append of batch k. Control-plane calls (leadership, replicas, acks, consumer offsets, fetch)
// drain both streams first and run synchronously: they are rare next to the append stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/ripplemq_engine.h"
#include "device_common.hpp"
#include "kernels.hpp"

using namespace rmq;

namespace {

constexpr uint32_t kStatsRing = 64;                               // tickets whose stats stay readable
constexpr uint32_t kMaxSortTiles = 128;                           // all sort tiles must be co-resident
constexpr uint32_t kMaxBatchRecords = kMaxSortTiles * kSortTile;  // 262144

struct EvPair {
  hipEvent_t a = nullptr, b = nullptr;
};

struct Slot {
  uint32_t* d_pidx = nullptr;  // staging for host batches
  uint32_t* d_len = nullptr;
  uint64_t* d_poff = nullptr;
  uint8_t* d_payload = nullptr;
  uint64_t* d_out = nullptr;
  uint32_t* keys[2] = {nullptr, nullptr};  // intermediate radix passes (P > 4096 only)
  uint32_t* vals[2] = {nullptr, nullptr};
  uint32_t* src_off = nullptr;             // packed payload offsets (multi-pass only)
  uint4* slots = nullptr;                  // sorted slot records for the append kernel
  uint64_t* batch_info = nullptr;
  uint64_t* hist_gran = nullptr;           // sort tile histograms [tiles][256]
  uint64_t* len_gran = nullptr;
  uint64_t* rb_gran = nullptr;
  hipEvent_t prep_done = nullptr, append_done = nullptr;
  uint64_t ticket = 0;
  bool used = false;
};

}  // namespace

struct rmq_engine {
  rmq_config cfg{};
  std::mutex mu;
  int device = 0;
  uint32_t cu_count = 0;
  char dev_name[256] = {0};
  hipStream_t main_s = nullptr;
  hipStream_t prep[2] = {nullptr, nullptr};  // batch sorts alternate between two prep streams
  DevState st{};
  CrcConsts* d_crc = nullptr;
  uint64_t* d_winner = nullptr;
  uint32_t* d_err = nullptr;
  uint4* d_tile_stats = nullptr;  // [kStatsRing][max append tiles]
  uint32_t max_app_tiles = 0;
  uint64_t* d_lb_cnt = nullptr;
  uint64_t* d_lb_bytes = nullptr;
  uint32_t epoch = 0;
  std::vector<Slot> slots;
  uint64_t last_ticket = 0;
  std::vector<uint32_t> ticket_n;  // [kStatsRing]
  // host mirrors of control state
  std::vector<uint32_t> is_leader, leader_slot, ranks;  // ranks [P][RF]
  std::vector<uint64_t> term;
  // sort plan
  uint32_t passes = 1, pass_shift[3] = {0, 0, 0}, pass_bits[3] = {1, 0, 0}, pass_ndig[3] = {1, 0, 0};
  // fetch scratch
  uint32_t* d_req = nullptr;
  uint64_t* d_res = nullptr;
  uint64_t* d_aux = nullptr;
  uint64_t* d_total = nullptr;
  uint32_t fetch_cap = 0;
  uint8_t* d_fetch_out = nullptr;
  uint64_t fetch_out_cap = 0;
  // consumer-commit / ack scratch
  uint32_t* d_ctl32 = nullptr;
  uint64_t* d_ctl64 = nullptr;
  uint32_t ctl_cap = 0;
  // RMQ_DEBUG_SKIP bit 0: skip the sort launch, bit 1: skip the append launch, bit 2: run each
  // batch's sort after the previous append (no overlap; to time the kernels alone)
  uint32_t debug_skip = 0;
  uint32_t debug_flags = 0;   // RMQ_DEBUG_FLAGS -> AppendArgs.debug
  uint32_t spin_limit = 1u << 22;
  hipEvent_t last_append_done = nullptr;
  uint64_t* d_stamps = nullptr;     // RMQ_STAMPS=<csv path>: append phase stamps of the last batch
  uint64_t* d_sort_stamps = nullptr;  // [pass][tiles][8] sort phase stamps of the last batch
  uint32_t sort_stamps_tiles = 0, sort_stamps_passes = 0;
  const char* stamps_path = nullptr;
  uint32_t stamps_tiles = 0;
  // profiling
  bool profile = false;
  std::vector<EvPair> prof[5];
  std::vector<hipEvent_t> ev_pool;
};

namespace {

int hip_fail(hipError_t e) {
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

uint32_t host_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int k = 31; k >= 0; --k) {
    if ((a >> k) & 1u) p ^= b;
    b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
  }
  return p;
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
  for (int j = 0; j < 32; ++j) c->shift_pow2[j] = x2n[j + 3];  // x^(8 * 2^j)
  c->pow8[0] = 0x80000000u;                                     // x^0
  for (uint32_t n = 1; n < kCrcPow8; ++n) c->pow8[n] = host_mulmod(c->pow8[n - 1], x2n[3]);
}

bool is_pow2(uint64_t v) { return v && !(v & (v - 1)); }

uint32_t ilog2(uint64_t v) {
  uint32_t r = 0;
  while ((1ull << r) < v) ++r;
  return r;
}

int check_err(rmq_engine* e) {
  uint32_t err = 0;
  HIP_TRY(hipMemcpy(&err, e->d_err, 4, hipMemcpyDeviceToHost));
  if (err) {
    std::fprintf(stderr, "ripplemq: device hand-off timeout (err=%u)\n", err);
    return RMQ_EDEVICE;
  }
  return RMQ_OK;
}

int drain(rmq_engine* e) {
  HIP_TRY(hipStreamSynchronize(e->prep[0]));
  HIP_TRY(hipStreamSynchronize(e->prep[1]));
  HIP_TRY(hipStreamSynchronize(e->main_s));
  return check_err(e);
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
  if (!e->stamps_path || !e->d_stamps || !e->stamps_tiles) return;
  std::vector<uint64_t> h((size_t)e->stamps_tiles * 8);
  if (hipMemcpy(h.data(), e->d_stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  FILE* f = std::fopen(e->stamps_path, "w");
  if (!f) return;
  std::fprintf(f, "tile,t0,t1,t2,t3,t4,t5,t6,t7\n");
  for (uint32_t t = 0; t < e->stamps_tiles; ++t) {
    std::fprintf(f, "%u", t);
    for (int k = 0; k < 8; ++k) std::fprintf(f, ",%llu", (unsigned long long)h[(size_t)t * 8 + k]);
    std::fprintf(f, "\n");
  }
  std::fclose(f);
  if (!e->d_sort_stamps || !e->sort_stamps_tiles) return;
  std::vector<uint64_t> g((size_t)3 * kMaxSortTiles * 8);
  if (hipMemcpy(g.data(), e->d_sort_stamps, g.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  std::string sp = std::string(e->stamps_path) + ".sort.csv";
  f = std::fopen(sp.c_str(), "w");
  if (!f) return;
  std::fprintf(f, "pass,tile,t0,t1,t2,t3,t4,t5,t6,t7\n");
  for (uint32_t k = 0; k < e->sort_stamps_passes; ++k)
    for (uint32_t t = 0; t < e->sort_stamps_tiles; ++t) {
      std::fprintf(f, "%u,%u", k, t);
      for (int q = 0; q < 8; ++q)
        std::fprintf(f, ",%llu", (unsigned long long)g[((size_t)k * kMaxSortTiles + t) * 8 + q]);
      std::fprintf(f, "\n");
    }
  std::fclose(f);
}

void free_engine(rmq_engine* e) {
  if (!e) return;
  hipSetDevice(e->device);
  if (e->main_s) hipStreamSynchronize(e->main_s);
  for (hipStream_t ps : e->prep)
    if (ps) hipStreamSynchronize(ps);
  dump_stamps(e);
  for (hipStream_t ps : e->prep)
    if (ps) hipStreamSynchronize(ps);
  DevState& s = e->st;
  void* bufs[] = {s.leo, s.used, s.start_off, s.start_pos, s.commit, s.hw, s.term_start, s.match,
                  s.is_leader, s.local_mask, s.index, s.logs, s.cons, e->d_crc, e->d_winner,
                  e->d_err, e->d_tile_stats,
                  e->d_lb_cnt, e->d_lb_bytes, e->d_req, e->d_res, e->d_aux,
                  e->d_total, e->d_fetch_out, e->d_ctl32, e->d_ctl64, e->d_stamps, e->d_sort_stamps};
  for (void* b : bufs)
    if (b) hipFree(b);
  for (Slot& sl : e->slots) {
    void* sb[] = {sl.d_pidx, sl.d_len, sl.d_poff, sl.d_payload, sl.d_out, sl.keys[0], sl.keys[1],
                  sl.vals[0], sl.vals[1], sl.src_off, sl.slots, sl.batch_info, sl.hist_gran,
                  sl.len_gran, sl.rb_gran};
    for (void* b : sb)
      if (b) hipFree(b);
    if (sl.prep_done) hipEventDestroy(sl.prep_done);
    if (sl.append_done) hipEventDestroy(sl.append_done);
  }
  for (auto& v : e->prof)
    for (EvPair& p : v) {
      if (p.a) hipEventDestroy(p.a);
      if (p.b) hipEventDestroy(p.b);
    }
  for (hipEvent_t ev : e->ev_pool) hipEventDestroy(ev);
  if (e->main_s) hipStreamDestroy(e->main_s);
  for (hipStream_t ps : e->prep)
    if (ps) hipStreamDestroy(ps);
  delete e;
}

int validate_cfg(const rmq_config* c) {
  if (!c) return RMQ_EINVAL;
  if (c->num_partitions == 0 || c->num_partitions > (1u << 24)) return RMQ_EINVAL;
  if (c->replication_factor == 0 || c->replication_factor > RMQ_MAX_RF) return RMQ_EINVAL;
  if (!is_pow2(c->index_interval) || c->index_interval < 64 || c->index_interval > (1u << 20))
    return RMQ_EINVAL;
  if (!is_pow2(c->segment_bytes) || c->segment_bytes < 4ull * c->index_interval) return RMQ_EINVAL;
  if (c->max_consumers == 0) return RMQ_EINVAL;
  if (c->max_batch_records == 0 || c->max_batch_records > kMaxBatchRecords) return RMQ_EINVAL;
  if (c->max_batch_bytes >= (1ull << 32)) return RMQ_EINVAL;
  return RMQ_OK;
}

}  // namespace

extern "C" {

uint32_t rmq_abi_version(void) { return RMQ_ABI_VERSION; }

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
  c->pipeline_depth = 3;
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
  if (!e->cfg.pipeline_depth) e->cfg.pipeline_depth = 3;
  if (const char* dbg = std::getenv("RMQ_DEBUG_SKIP")) e->debug_skip = (uint32_t)std::atoi(dbg);
  if (const char* dbg = std::getenv("RMQ_DEBUG_FLAGS")) e->debug_flags = (uint32_t)std::atoi(dbg);
  if (const char* dbg = std::getenv("RMQ_SPIN_LIMIT")) e->spin_limit = (uint32_t)std::atoi(dbg);
  e->stamps_path = std::getenv("RMQ_STAMPS");
  e->device = cfg->device;
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
  std::snprintf(e->dev_name, sizeof e->dev_name, "%s (%s)", prop.name, prop.gcnArchName);
  CREATE_HIP(hipStreamCreateWithFlags(&e->main_s, hipStreamNonBlocking));
  CREATE_HIP(hipStreamCreateWithFlags(&e->prep[0], hipStreamNonBlocking));
  CREATE_HIP(hipStreamCreateWithFlags(&e->prep[1], hipStreamNonBlocking));

  const uint32_t P = cfg->num_partitions, RF = cfg->replication_factor, C = cfg->max_consumers;
  DevState& s = e->st;
  s.P = P;
  s.RF = RF;
  s.C = C;
  s.seg = cfg->segment_bytes;
  s.interval_log2 = ilog2(cfg->index_interval);
  s.icap = (uint32_t)(cfg->segment_bytes / cfg->index_interval + 2);
  CREATE_TRY(dalloc(&s.leo, P));
  CREATE_TRY(dalloc(&s.used, P));
  CREATE_TRY(dalloc(&s.start_off, P));
  CREATE_TRY(dalloc(&s.start_pos, P));
  CREATE_TRY(dalloc(&s.commit, P));
  CREATE_TRY(dalloc(&s.hw, P));
  CREATE_TRY(dalloc(&s.term_start, P));
  CREATE_TRY(dalloc(&s.match, (size_t)P * RF));
  CREATE_TRY(dalloc(&s.is_leader, P));
  CREATE_TRY(dalloc(&s.local_mask, P));
  CREATE_TRY(dalloc(&s.index, (size_t)P * s.icap * 2));
  CREATE_TRY(dalloc(&s.logs, (size_t)RF * P * s.seg));
  CREATE_TRY(dalloc(&s.cons, (size_t)P * C));
  CREATE_TRY(dalloc(&e->d_winner, (size_t)P * C));
  CREATE_TRY(dalloc(&e->d_err, 1));
  const uint32_t max_sort_tiles = (cfg->max_batch_records + kSortTile - 1) / kSortTile;
  e->max_app_tiles = (cfg->max_batch_records + kAppendTile - 1) / kAppendTile;
  CREATE_TRY(dalloc(&e->d_tile_stats, (size_t)kStatsRing * e->max_app_tiles));
  CREATE_TRY(dalloc(&e->d_lb_cnt, e->max_app_tiles));
  CREATE_TRY(dalloc(&e->d_lb_bytes, e->max_app_tiles));
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
  e->ticket_n.assign(kStatsRing, 0u);

  // radix plan: <= 8-bit digits of the partition id (one pass for P <= 256)
  uint32_t bits = ilog2((uint64_t)P);  // keys in [0, P-1]
  if (bits == 0) bits = 1;
  e->passes = (bits + kSortDigitBits - 1) / kSortDigitBits;
  const uint32_t dw = (bits + e->passes - 1) / e->passes;
  for (uint32_t k = 0; k < e->passes; ++k) {
    e->pass_shift[k] = k * dw;
    e->pass_bits[k] = std::min(dw, bits - k * dw);
    e->pass_ndig[k] = k + 1 == e->passes ? ((P - 1) >> e->pass_shift[k]) + 1 : 1u << e->pass_bits[k];
  }

  const uint32_t D = e->cfg.pipeline_depth;
  e->slots.resize(D);
  const uint32_t NB = cfg->max_batch_records;
  for (Slot& sl : e->slots) {
    if (e->passes > 1) {
      CREATE_TRY(dalloc(&sl.keys[0], NB));
      CREATE_TRY(dalloc(&sl.vals[0], NB));
      CREATE_TRY(dalloc(&sl.src_off, NB));
    }
    CREATE_TRY(dalloc(&sl.slots, NB));
    CREATE_TRY(dalloc(&sl.batch_info, 4));
    CREATE_TRY(dalloc(&sl.hist_gran, (size_t)max_sort_tiles * 256));
    CREATE_TRY(dalloc(&sl.len_gran, max_sort_tiles));
    CREATE_TRY(dalloc(&sl.rb_gran, max_sort_tiles));
    CREATE_HIP(hipEventCreateWithFlags(&sl.prep_done, hipEventDisableTiming));
    CREATE_HIP(hipEventCreateWithFlags(&sl.append_done, hipEventDisableTiming));
  }
  CREATE_HIP(hipDeviceSynchronize());
  *out = e;
  return RMQ_OK;
#undef CREATE_TRY
#undef CREATE_HIP
}

void rmq_destroy(rmq_engine* e) { free_engine(e); }

int rmq_set_replicas(rmq_engine* e, uint32_t pidx, const uint32_t* ranks, uint32_t rf, uint32_t leader_slot) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (pidx >= e->cfg.num_partitions) return RMQ_ENOPART;
  const uint32_t RF = e->cfg.replication_factor;
  if (!ranks || rf != RF || leader_slot >= rf) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  uint32_t mask = 0;
  for (uint32_t r = 0; r < RF; ++r) {
    e->ranks[(size_t)pidx * RF + r] = ranks[r];
    if (ranks[r] == e->cfg.rank) mask |= 1u << r;
  }
  e->leader_slot[pidx] = leader_slot;
  e->is_leader[pidx] = ranks[leader_slot] == e->cfg.rank;
  HIP_TRY(hipMemcpy(e->st.is_leader + pidx, &e->is_leader[pidx], 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->st.local_mask + pidx, &mask, 4, hipMemcpyHostToDevice));
  return RMQ_OK;
}

int rmq_become_leader(rmq_engine* e, uint32_t pidx, uint64_t term) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  if (pidx != RMQ_ALL_PARTITIONS && pidx >= P) return RMQ_ENOPART;
  const uint32_t lo = pidx == RMQ_ALL_PARTITIONS ? 0 : pidx, hi = pidx == RMQ_ALL_PARTITIONS ? P : pidx + 1;
  for (uint32_t p = lo; p < hi; ++p) {  // validate everything before changing anything
    if (term < e->term[p]) return RMQ_EINVAL;
    bool local = false;
    for (uint32_t r = 0; r < RF; ++r) local |= e->ranks[(size_t)p * RF + r] == e->cfg.rank;
    if (!local) return RMQ_EINVAL;
  }
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  for (uint32_t p = lo; p < hi; ++p) {
    uint32_t slot = 0;
    while (e->ranks[(size_t)p * RF + slot] != e->cfg.rank) ++slot;
    e->leader_slot[p] = slot;
    e->is_leader[p] = 1;
    e->term[p] = term;
  }
  HIP_TRY(hipMemcpy(e->st.is_leader + lo, &e->is_leader[lo], (size_t)(hi - lo) * 4, hipMemcpyHostToDevice));
  launch_become_leader(e->st, pidx, e->main_s);
  HIP_TRY(hipGetLastError());
  return drain(e);
}

int rmq_append(rmq_engine* e, const rmq_batch* b, uint64_t* out_offsets, uint64_t* ticket) {
  if (!e || !b || !ticket) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  const uint32_t n = b->n;
  if (n > e->cfg.max_batch_records) return RMQ_ENOSPC;
  if (b->payload_bytes > e->cfg.max_batch_bytes) return RMQ_ENOSPC;
  if (b->mem != RMQ_MEM_HOST && b->mem != RMQ_MEM_DEVICE) return RMQ_EINVAL;
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

  const uint64_t t = ++e->last_ticket;
  *ticket = t;
  e->ticket_n[t % kStatsRing] = n;
  Slot& sl = e->slots[t % e->slots.size()];
  hipStream_t prep_s = e->prep[t & 1];
  if (sl.used) {
    HIP_TRY(hipEventSynchronize(sl.append_done));  // scratch of ticket t - depth is free again
  }
  sl.used = true;
  sl.ticket = t;
  if (n == 0) {
    HIP_TRY(hipEventRecord(sl.append_done, e->main_s));
    return RMQ_OK;
  }

  const uint32_t* pidx = b->pidx;
  const uint32_t* len = b->len;
  const uint64_t* poff = b->payload_off;
  const uint8_t* payload = b->payload;
  uint64_t* d_out = out_offsets;
  if (b->mem == RMQ_MEM_HOST) {
    const uint32_t NB = e->cfg.max_batch_records;
    if (!sl.d_pidx) {
      int rc = dalloc(&sl.d_pidx, NB);
      if (!rc) rc = dalloc(&sl.d_len, NB);
      if (!rc) rc = dalloc(&sl.d_poff, NB);
      if (!rc) rc = dalloc(&sl.d_out, NB);
      if (!rc) rc = dalloc(&sl.d_payload, e->cfg.max_batch_bytes + 8);
      if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(sl.d_pidx, pidx, n * 4ull, hipMemcpyHostToDevice, prep_s));
    HIP_TRY(hipMemcpyAsync(sl.d_len, len, n * 4ull, hipMemcpyHostToDevice, prep_s));
    if (poff) HIP_TRY(hipMemcpyAsync(sl.d_poff, poff, n * 8ull, hipMemcpyHostToDevice, prep_s));
    if (b->payload_bytes)
      HIP_TRY(hipMemcpyAsync(sl.d_payload, payload, b->payload_bytes, hipMemcpyHostToDevice, prep_s));
    pidx = sl.d_pidx;
    len = sl.d_len;
    poff = poff ? sl.d_poff : nullptr;
    payload = sl.d_payload;
    d_out = sl.d_out;
  }

  if ((e->debug_skip & 4u) && e->last_append_done)
    HIP_TRY(hipStreamWaitEvent(prep_s, e->last_append_done, 0));
  // ---- prep stream: stable partition-major sort of the batch into slot records
  const uint32_t sort_tiles = (n + kSortTile - 1) / kSortTile;
  hipEvent_t ps0 = nullptr, ps1 = nullptr;
  if (e->profile) {
    ps0 = pool_event(e);
    ps1 = pool_event(e);
    HIP_TRY(hipEventRecord(ps0, prep_s));
  }
  const uint32_t* kin = pidx;
  const uint32_t* vin = nullptr;
  for (uint32_t k = 0; k < e->passes; ++k) {
    SortPassArgs a{};
    a.keys_in = kin;
    a.pidx_raw = pidx;
    a.vals_in = vin;
    a.keys_out = sl.keys[0];
    a.vals_out = sl.vals[0];
    a.slots = sl.slots;
    a.len = len;
    a.payload_off = poff;
    a.src_off = poff ? nullptr : sl.src_off;
    a.batch_info = sl.batch_info;
    a.hist_gran = sl.hist_gran;
    a.len_gran = sl.len_gran;
    a.rb_gran = sl.rb_gran;
    a.n = n;
    a.tiles = sort_tiles;
    a.shift = e->pass_shift[k];
    a.bits = e->pass_bits[k];
    a.ndig = e->pass_ndig[k];
    a.P = e->cfg.num_partitions;
    a.first = k == 0;
    a.last = k + 1 == e->passes;
    a.epoch = ++e->epoch;
    a.err = e->d_err;
    if (e->stamps_path) {
      if (!e->d_sort_stamps) {
        int rc = dalloc(&e->d_sort_stamps, (size_t)3 * kMaxSortTiles * 8);
        if (rc) return rc;
      }
      a.stamps = e->d_sort_stamps + (size_t)k * kMaxSortTiles * 8;
      e->sort_stamps_tiles = sort_tiles;
      e->sort_stamps_passes = e->passes;
    }
    if (!(e->debug_skip & 1u)) launch_sort_pass(a, sort_tiles, prep_s);
    kin = sl.keys[0];
    vin = sl.vals[0];
  }
  HIP_TRY(hipGetLastError());
  if (e->profile) {
    HIP_TRY(hipEventRecord(ps1, prep_s));
    e->prof[1].push_back({ps0, ps1});
  }
  HIP_TRY(hipEventRecord(sl.prep_done, prep_s));

  // ---- main stream: fused append
  HIP_TRY(hipStreamWaitEvent(e->main_s, sl.prep_done, 0));
  AppendArgs a{};
  a.st = e->st;
  a.slots = sl.slots;
  a.payload = payload;
  a.payload_bytes = b->payload_bytes;
  a.out_offsets = d_out;
  a.batch_info = sl.batch_info;
  a.tile_stats = e->d_tile_stats + (size_t)(t % kStatsRing) * e->max_app_tiles;
  a.lb_cnt = e->d_lb_cnt;
  a.lb_bytes = e->d_lb_bytes;
  a.n = n;
  a.tiles = (n + kAppendTile - 1) / kAppendTile;
  a.epoch = ++e->epoch;
  const uint64_t lim = e->cfg.segment_bytes - e->cfg.index_interval;
  a.nospace_limit_lo = (uint32_t)lim;
  a.nospace_limit_hi = (uint32_t)(lim >> 32);
  a.crc = e->d_crc;
  a.err = e->d_err;
  a.spin_limit = e->spin_limit;
  a.debug = e->debug_flags;
  if (e->stamps_path) {
    if (!e->d_stamps) {
      int rc = dalloc(&e->d_stamps, (size_t)e->max_app_tiles * 8);
      if (rc) return rc;
    }
    a.stamps = e->d_stamps;
    e->stamps_tiles = a.tiles;
  }
  const uint32_t wpb = (uint32_t)append_waves_per_block();
  const uint32_t grid = std::min<uint32_t>((a.tiles + wpb - 1) / wpb, e->cu_count * (uint32_t)append_blocks_per_cu());
  hipEvent_t pa0 = nullptr, pa1 = nullptr;
  if (e->profile) {
    pa0 = pool_event(e);
    pa1 = pool_event(e);
    HIP_TRY(hipEventRecord(pa0, e->main_s));
  }
  if (!(e->debug_skip & 2u)) launch_append(a, grid, e->main_s);
  HIP_TRY(hipGetLastError());
  if (e->profile) {
    HIP_TRY(hipEventRecord(pa1, e->main_s));
    e->prof[0].push_back({pa0, pa1});
  }
  if (b->mem == RMQ_MEM_HOST)
    HIP_TRY(hipMemcpyAsync(out_offsets, d_out, n * 8ull, hipMemcpyDeviceToHost, e->main_s));
  HIP_TRY(hipEventRecord(sl.append_done, e->main_s));
  e->last_append_done = sl.append_done;
  return RMQ_OK;
}

int rmq_ack(rmq_engine* e, const uint32_t* pidx, const uint32_t* slot, const uint64_t* match, uint32_t n) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
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

int rmq_poll_commit(rmq_engine* e, uint64_t ticket, uint64_t* commit_out, uint64_t* hw_out) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (ticket > e->last_ticket) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  if (ticket) {
    Slot& sl = e->slots[ticket % e->slots.size()];
    if (sl.ticket == ticket) {
      hipError_t q = hipEventQuery(sl.append_done);
      if (q == hipErrorNotReady) return RMQ_PENDING;
      if (q != hipSuccess) return hip_fail(q);
    }
  }
  int rc = check_err(e);
  if (rc) return rc;
  const size_t P = e->cfg.num_partitions;
  if (commit_out || hw_out) {
    HIP_TRY(hipStreamSynchronize(e->main_s));  // snapshot after everything submitted so far
    if (commit_out) HIP_TRY(hipMemcpy(commit_out, e->st.commit, P * 8, hipMemcpyDeviceToHost));
    if (hw_out) HIP_TRY(hipMemcpy(hw_out, e->st.hw, P * 8, hipMemcpyDeviceToHost));
  }
  return RMQ_OK;
}

int rmq_ticket_stats(rmq_engine* e, uint64_t ticket, rmq_append_stats* out) {
  if (!e || !out) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (!ticket || ticket > e->last_ticket || e->last_ticket - ticket >= kStatsRing) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  Slot& sl = e->slots[ticket % e->slots.size()];
  if (sl.ticket == ticket) HIP_TRY(hipEventSynchronize(sl.append_done));
  const uint32_t n = e->ticket_n[ticket % kStatsRing];
  const uint32_t tiles = (n + kAppendTile - 1) / kAppendTile;
  std::vector<uint4> ts(tiles ? tiles : 1);
  if (tiles)
    HIP_TRY(hipMemcpy(ts.data(), e->d_tile_stats + (size_t)(ticket % kStatsRing) * e->max_app_tiles,
                      tiles * sizeof(uint4), hipMemcpyDeviceToHost));
  std::memset(out, 0, sizeof *out);
  out->records = n;
  for (uint32_t k = 0; k < tiles; ++k) {
    out->appended += ts[k].x;
    out->rejected_not_leader += ts[k].y;
    out->rejected_no_partition += ts[k].z;
    out->rejected_no_space += ts[k].w;
  }
  return check_err(e);
}

int rmq_sync(rmq_engine* e) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  return drain(e);
}

int rmq_commit_consumer_offset(rmq_engine* e, const uint32_t* pidx, const uint32_t* consumer,
                               const uint64_t* offset, uint32_t n, int32_t* status) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (!n) return RMQ_OK;
  if (!pidx || !consumer || !offset) return RMQ_EINVAL;
  std::vector<uint32_t> vp, vc;
  std::vector<uint64_t> vo;
  int rc_all = RMQ_OK;
  for (uint32_t i = 0; i < n; ++i) {
    int st = RMQ_OK;
    if (pidx[i] >= e->cfg.num_partitions)
      st = RMQ_ENOPART;
    else if (!e->is_leader[pidx[i]])
      st = RMQ_ENOTLEADER;
    else if (consumer[i] >= e->cfg.max_consumers)
      st = RMQ_EINVAL;
    if (status) status[i] = st;
    if (st) {
      if (!rc_all) rc_all = st;
      continue;
    }
    vp.push_back(pidx[i]);
    vc.push_back(consumer[i]);
    vo.push_back(offset[i]);
  }
  if (vp.empty()) return rc_all;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  const uint32_t m = (uint32_t)vp.size();
  rc = ensure_ctl(e, m);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(e->d_ctl32, vp.data(), m * 4ull, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_ctl32 + e->ctl_cap, vc.data(), m * 4ull, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_ctl64, vo.data(), m * 8ull, hipMemcpyHostToDevice));
  ConsumerCommitArgs a{};
  a.st = e->st;
  a.pidx = e->d_ctl32;
  a.consumer = e->d_ctl32 + e->ctl_cap;
  a.offset = e->d_ctl64;
  a.winner = e->d_winner;
  a.n = m;
  a.epoch = ++e->epoch;
  launch_consumer_commit(a, e->main_s);
  HIP_TRY(hipGetLastError());
  rc = drain(e);
  return rc ? rc : rc_all;
}

int rmq_fetch(rmq_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint32_t mem, uint8_t* out,
              uint64_t out_cap, rmq_fetch_res* res, uint64_t* bytes_used) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (bytes_used) *bytes_used = 0;
  if (!n) return RMQ_OK;
  if (!reqs || !res || (mem != RMQ_MEM_HOST && mem != RMQ_MEM_DEVICE)) return RMQ_EINVAL;
  if (out_cap && !out) return RMQ_EINVAL;
  if (mem == RMQ_MEM_DEVICE && (reinterpret_cast<uintptr_t>(out) & 3u)) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  if (n > e->fetch_cap) {
    hipFree(e->d_req);
    hipFree(e->d_res);
    hipFree(e->d_aux);
    e->fetch_cap = 0;
    const uint32_t cap = std::max<uint32_t>(n, 1024);
    rc = dalloc(&e->d_req, (size_t)cap * 4);
    if (!rc) rc = dalloc(&e->d_res, (size_t)cap * 4);
    if (!rc) rc = dalloc(&e->d_aux, (size_t)cap * 2);
    if (!rc && !e->d_total) rc = dalloc(&e->d_total, 1);
    if (rc) return rc;
    e->fetch_cap = cap;
  }
  uint8_t* d_out = out;
  if (mem == RMQ_MEM_HOST && out_cap) {
    if (out_cap > e->fetch_out_cap) {
      hipFree(e->d_fetch_out);
      e->d_fetch_out = nullptr;
      e->fetch_out_cap = 0;
      rc = dalloc(&e->d_fetch_out, out_cap);
      if (rc) return rc;
      e->fetch_out_cap = out_cap;
    }
    d_out = e->d_fetch_out;
  }
  HIP_TRY(hipMemcpy(e->d_req, reqs, (size_t)n * sizeof(rmq_fetch_req), hipMemcpyHostToDevice));
  FetchArgs a{};
  a.st = e->st;
  a.req = e->d_req;
  a.res = e->d_res;
  a.aux = e->d_aux;
  a.out = d_out;
  a.out_cap = out_cap;
  a.n = n;
  a.total = e->d_total;
  hipEvent_t r0 = nullptr, r1 = nullptr, g0 = nullptr, g1 = nullptr;
  if (e->profile) {
    r0 = pool_event(e);
    r1 = pool_event(e);
    g0 = pool_event(e);
    g1 = pool_event(e);
  }
  launch_fetch(a, e->main_s, r0, r1, g0, g1);
  HIP_TRY(hipGetLastError());
  if (e->profile) {
    e->prof[3].push_back({r0, r1});
    e->prof[4].push_back({g0, g1});
  }
  rc = drain(e);
  if (rc) return rc;
  std::vector<uint64_t> hres((size_t)n * 4);
  uint64_t total = 0;
  HIP_TRY(hipMemcpy(hres.data(), e->d_res, hres.size() * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&total, e->d_total, 8, hipMemcpyDeviceToHost));
  int rc_all = RMQ_OK;
  for (uint32_t r = 0; r < n; ++r) {
    rmq_fetch_res& x = res[r];
    std::memset(&x, 0, sizeof x);
    x.start_offset = hres[4 * r + 0];
    x.out_pos = hres[4 * r + 1];
    x.count = (uint32_t)hres[4 * r + 2];
    x.bytes = (uint32_t)(hres[4 * r + 2] >> 32);
    x.status = (int32_t)(uint32_t)hres[4 * r + 3];
    if (x.status == RMQ_ENOSPC) rc_all = RMQ_ENOSPC;
  }
  if (mem == RMQ_MEM_HOST && out_cap) {
    const uint64_t nb = std::min(total, out_cap);
    if (nb) HIP_TRY(hipMemcpy(out, d_out, nb, hipMemcpyDeviceToHost));
  }
  if (bytes_used) *bytes_used = total;
  return rc_all;
}

int rmq_get_partition_state(rmq_engine* e, uint32_t p, rmq_partition_state* o) {
  if (!e || !o) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
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
  o->term = e->term[p];
  for (uint32_t r = 0; r < RF; ++r) o->replica_rank[r] = e->ranks[(size_t)p * RF + r];
  o->leader_slot = e->leader_slot[p];
  o->is_leader = e->is_leader[p];
  return RMQ_OK;
}

int rmq_read_segment(rmq_engine* e, uint32_t replica, uint32_t p, uint64_t ring_off, uint64_t len, uint8_t* out) {
  if (!e || (len && !out)) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  const uint64_t S = e->cfg.segment_bytes;
  if (replica >= e->cfg.replication_factor || ring_off > S || len > S - ring_off) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  if (len)
    HIP_TRY(hipMemcpy(out, e->st.logs + ((uint64_t)replica * e->cfg.num_partitions + p) * S + ring_off,
                      len, hipMemcpyDeviceToHost));
  return RMQ_OK;
}

int rmq_read_index(rmq_engine* e, uint32_t p, uint64_t m_first, uint64_t count, uint64_t* out) {
  if (!e || (count && !out)) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  const uint32_t icap = e->st.icap;
  if (count > icap) return RMQ_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  std::vector<uint64_t> ring((size_t)icap * 2);
  HIP_TRY(hipMemcpy(ring.data(), e->st.index + (size_t)p * icap * 2, ring.size() * 8, hipMemcpyDeviceToHost));
  for (uint64_t k = 0; k < count; ++k) {
    const uint64_t sl = (m_first + k) % icap;
    out[2 * k] = ring[2 * sl];
    out[2 * k + 1] = ring[2 * sl + 1];
  }
  return RMQ_OK;
}

int rmq_read_consumer_offsets(rmq_engine* e, uint32_t p, uint64_t* out) {
  if (!e || !out) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(out, e->st.cons + (size_t)p * e->cfg.max_consumers, e->cfg.max_consumers * 8ull,
                    hipMemcpyDeviceToHost));
  return RMQ_OK;
}

int rmq_device_alloc(rmq_engine* e, uint64_t bytes, void** out) {
  if (!e || !out) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  *out = nullptr;
  HIP_TRY(hipMalloc(out, bytes ? bytes : 1));
  return RMQ_OK;
}

int rmq_device_free(rmq_engine* e, void* p) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  if (p) HIP_TRY(hipFree(p));
  return RMQ_OK;
}

int rmq_memcpy(rmq_engine* e, void* dst, const void* src, uint64_t bytes, int kind) {
  if (!e || (bytes && (!dst || !src))) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                        : kind == 1 ? hipMemcpyDeviceToHost
                                    : hipMemcpyDeviceToDevice;
  int rc = drain(e);
  if (rc) return rc;
  if (bytes) HIP_TRY(hipMemcpy(dst, src, bytes, k));
  return RMQ_OK;
}

int rmq_profile_enable(rmq_engine* e, int enable) {
  if (!e) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  for (auto& v : e->prof) {
    for (EvPair& p : v) {
      e->ev_pool.push_back(p.a);
      e->ev_pool.push_back(p.b);
    }
    v.clear();
  }
  e->profile = enable != 0;
  return RMQ_OK;
}

int rmq_profile_query(rmq_engine* e, int kernel, uint64_t* launches, double* total_ms) {
  if (!e || kernel < 0 || kernel > 4) return RMQ_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  int rc = drain(e);
  if (rc) return rc;
  double tot = 0;
  for (const EvPair& p : e->prof[kernel]) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
    tot += ms;
  }
  if (launches) *launches = e->prof[kernel].size();
  if (total_ms) *total_ms = tot;
  return RMQ_OK;
}

int rmq_device_info(rmq_engine* e, char* name, uint32_t name_cap, uint32_t* cu_count) {
  if (!e) return RMQ_EINVAL;
  if (name && name_cap) std::snprintf(name, name_cap, "%s", e->dev_name);
  if (cu_count) *cu_count = e->cu_count;
  return RMQ_OK;
}

}  // extern "C"
