// segscan.cpp — host-side walk of FORMAT.md §1 records laid back to back (segment files of the
// durable tier, ripplemq_amd/tier.py; fetch output buffers). The reference keeps every message in
// its `messages` list and jraft persists the log under the partition's data path
// (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:26,64-69,
// PartitionRaftServer.java:53,88-90); the tier restores that below the HBM rings, and reopening a
// segment file after a crash must find where its whole records end. This was a Python loop over
// the headers (tier.py round 3); it is one pass over the bytes here, with the CRC32C of every
// payload checked by the SSE4.2 crc32 instruction when asked.
#include <algorithm>
#include <cstdint>
#include <cstring>

#include "../../include/ripplemq_engine.h"

namespace {

uint32_t crc_table[8][256];
bool crc_ready = false;

void crc_init() {
  if (crc_ready) return;
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    crc_table[0][b] = c;
  }
  for (uint32_t t = 1; t < 8; ++t)
    for (uint32_t b = 0; b < 256; ++b) crc_table[t][b] = (crc_table[t - 1][b] >> 8) ^ crc_table[0][crc_table[t - 1][b] & 0xFF];
  crc_ready = true;
}

uint32_t crc_sw(const uint8_t* p, uint64_t n) {
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = crc_table[7][lo & 0xFF] ^ crc_table[6][(lo >> 8) & 0xFF] ^ crc_table[5][(lo >> 16) & 0xFF] ^
        crc_table[4][lo >> 24] ^ crc_table[3][hi & 0xFF] ^ crc_table[2][(hi >> 8) & 0xFF] ^
        crc_table[1][(hi >> 16) & 0xFF] ^ crc_table[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ crc_table[0][(c ^ *p++) & 0xFF];
  return c ^ 0xFFFFFFFFu;
}

__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, uint64_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32 ^ 0xFFFFFFFFu;
}

}  // namespace

extern "C" int rmq_scan_records(const uint8_t* buf, uint64_t len, uint64_t first, uint64_t max_records,
                                uint32_t flags, uint64_t* pos_out, uint64_t* count, uint64_t* bytes) {
  if ((len && !buf) || !count || !bytes) return RMQ_EINVAL;
  const bool check = (flags & RMQ_SCAN_CHECK) != 0;
  const bool hw = __builtin_cpu_supports("sse4.2");
  if (check && !hw) crc_init();
  uint64_t pos = 0, k = 0;
  while (k < max_records && pos + 16 <= len) {
    uint64_t off;
    uint32_t L, crc;
    std::memcpy(&off, buf + pos, 8);
    std::memcpy(&L, buf + pos + 8, 4);
    std::memcpy(&crc, buf + pos + 12, 4);
    const uint64_t rs = 16ull + ((L + 15ull) & ~15ull);
    if (off != first + k || rs > len - pos) break;  // out of sequence, or cut short
    if (check) {
      const uint8_t* pl = buf + pos + 16;
      if ((hw ? crc_hw(pl, L) : crc_sw(pl, L)) != crc) break;
      bool pad_zero = true;  // the zero padding is part of the record (FORMAT.md §1)
      for (uint64_t z = L; z < rs - 16; ++z) pad_zero &= pl[z] == 0;
      if (!pad_zero) break;
    }
    if (pos_out) pos_out[k] = pos;
    pos += rs;
    ++k;
  }
  if (pos_out) pos_out[k] = pos;
  *count = k;
  *bytes = pos;
  return RMQ_OK;
}

// ------------------------------------------------------------------------------------------
// Durable-tier spill (ripplemq_amd/tier.py): the record runs of many partitions, as one rmq_fetch
// returned them, appended to the partitions' open segment files in one call (the per-partition
// Python loop of round 4 ran at 0.26 GB/s). jraft persists each partition group's log under its
// data path (PartitionRaftServer.java:53,88-90); the reference never drops a message
// (PartitionStateMachine.java:26).
// ------------------------------------------------------------------------------------------
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <thread>
#include <vector>

extern "C" int rmq_tier_append(uint32_t n, const int32_t* fd, const uint64_t* first, const uint64_t* count,
                               const uint64_t* buf_pos, const uint64_t* bytes, const uint8_t* buf,
                               uint64_t* pos_out, uint32_t threads, int fsync_each) {
  if (!n) return RMQ_OK;
  if (!fd || !first || !count || !buf_pos || !bytes || !buf || !pos_out) return RMQ_EINVAL;
  // each run's first slot in pos_out
  std::vector<uint64_t> at(n);
  for (uint32_t i = 0, a = 0; i < n; ++i) {
    at[i] = a;
    a += count[i] + 1;
  }
  // on a few threads: every run's check (header offsets first, first + 1, ..., exactly count records
  // filling exactly its bytes), then — none failed — every run's write (independent files)
  std::atomic<uint32_t> next{0};
  std::atomic<int> err{0};
  auto check = [&]() {
    for (uint32_t i; (i = next.fetch_add(1)) < n && !err.load();) {
      const uint8_t* b = buf + buf_pos[i];
      uint64_t pos = 0, k = 0;
      for (; k < count[i] && pos + 16 <= bytes[i]; ++k) {
        uint64_t off;
        uint32_t L;
        std::memcpy(&off, b + pos, 8);
        std::memcpy(&L, b + pos + 8, 4);
        const uint64_t rs = 16ull + ((L + 15ull) & ~15ull);
        if (off != first[i] + k || rs > bytes[i] - pos) break;
        pos_out[at[i] + k] = pos;
        pos += rs;
      }
      if (k != count[i] || pos != bytes[i]) {
        err.store(-1);
        return;
      }
      pos_out[at[i] + k] = pos;
    }
  };
  auto write_run = [&](uint32_t i) {
    const uint8_t* b = buf + buf_pos[i];
    uint64_t left = bytes[i];
    while (left) {
      const ssize_t w = ::write(fd[i], b, left);
      if (w < 0) {
        if (errno == EINTR) continue;
        err.store(errno ? errno : EIO);
        return;
      }
      b += w;
      left -= (uint64_t)w;
    }
    if (fsync_each && ::fsync(fd[i]) != 0) err.store(errno ? errno : EIO);
  };
  const uint32_t t = std::max<uint32_t>(1u, std::min<uint32_t>(threads ? threads : 8u, (n + 7) / 8));
  // one set of threads for both phases, meeting between them (thread start-up is tens of us each)
  std::atomic<uint32_t> arrived{0}, next_w{0};
  auto both = [&]() {
    check();
    arrived.fetch_add(1);
    while (arrived.load() < t) std::this_thread::yield();
    if (err.load()) return;
    for (uint32_t i; (i = next_w.fetch_add(1)) < n && !err.load();) write_run(i);
  };
  std::vector<std::thread> pool;
  for (uint32_t k = 1; k < t; ++k) pool.emplace_back(both);
  both();
  for (std::thread& th : pool) th.join();
  if (err.load() < 0) return RMQ_EINVAL;
  if (err.load()) {
    errno = err.load();
    return RMQ_EDEVICE;  // an I/O error (errno set)
  }
  return RMQ_OK;
}
