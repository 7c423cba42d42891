// fetch.hip — batched consumer fetch: PartitionStateMachine.handleBatchRead
// (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:85-110), served directly from
// committed state like MessageBatchReadRequestProcessor.java:39 (no read-index).
//
//  resolve (half-wave per request, two per wave: 16,384 requests are 8,192 waves, about one round
//          of the chip's resident waves): off = consumerOffsets.getOrDefault(id, 0); end = min(off + max, hw);
//          byte range of records [off, end): both ends found together, a quarter-wave each, by a
//          16-ary search of the sparse offset index (FORMAT.md §5: E[m] = first record starting at
//          or after m*I; 16 probes per round, one round per factor 16 of index entries), then the
//          record headers of the 512 B after the entry found are loaded at once (two 16-byte pieces
//          per lane of the quarter) and walked in registers;
//          each workgroup adds its requests' bytes to the sum of their chunk of 256 requests;
//  gather  (workgroup per 16 requests, a wave per 4): the output position of its first request from
//          the chunk sums before it and the byte counts of its chunk before it (at most 64 + 255
//          values, L2-resident), an exclusive scan over its 16 requests -> compact output positions
//          (into the result rows' out_pos), ENOSPC marking (every request's bytes count, served or
//          not: FORMAT.md §7); then each wave copies its 4 requests one after the other (the
//          requests' ring words loaded before the placement barrier), 16-byte loads from the
//          lowest local replica ring, four in flight per lane, 16-byte stores to the output. Records and output positions are 16-byte aligned
//          (FORMAT.md §1), so no piece straddles a record, the ring end or an output boundary.
//          (Round 2 placed with a single 1024-thread workgroup between the two: 12.6 us of the
//          max = 10 fetch of 16,384 requests with the rest of the GPU idle.)
//
// The kernels (resolve, gather; the chunk sums a slot's previous gather cleared) run on the
// pipeline stream itself, after the last pipeline launch the host had issued and before the next
// one, so the committed state they read is stable and the append pipeline is never flushed for a
// fetch.
#include <hip/hip_ext.h>

#include <type_traits>

#include "device_common.hpp"
#include "kernels.hpp"

namespace rmq {

constexpr int kOk = 0, kNotLeader = -1, kNoPart = -2, kInval = -3, kNoSpc = -4, kOffset = -6;
constexpr u32 kFW = 4;  // waves per workgroup (gather)
#ifndef RMQ_RESOLVE_WAVES
#define RMQ_RESOLVE_WAVES 8  // round 5 (rows read by one load per workgroup): 8 vs 4 waves, max = 10
                             // 24.8-25.3 vs 25.1-25.5 us, consumer loop 36.0 vs 36.9-37.6 us; 16: max = 10 27 us
#endif
constexpr u32 kRW = RMQ_RESOLVE_WAVES;  // waves per resolve workgroup

struct PartView {
  u64 leo, used, start_off, start_pos;
  RingRef rg;           // the partition's ring and index ring
  const uint8_t* ring;  // lowest local replica ring of the partition
};

// A wave resolves two requests (lanes 0..31 and 32..63), and each request's two ends are found
// together by a quarter-wave each: kQL lanes per searched position.
constexpr u32 kQL = 16;
constexpr u64 kWalkMax = 32;  // longest slice walked from a cached position
constexpr u32 kRPW = 2;  // requests per resolve wave

// Logical byte position of record t (start_off <= t <= leo) in the lane's view, found by the kQL
// lanes of its quarter (t, v, act quarter-uniform; an inactive quarter loads nothing and gets 0).
// The largest index entry at or before t: E[m] = first record starting at or after m I rises with
// m, so a kQL-ary search over the live entries (round 0 probes the kQL entries around the
// interpolated position of t: records of one size give it exactly), then the record headers after
// that entry, read as windows of 2 kQL 16-byte pieces (two per lane) and walked in registers; the
// window the interpolation puts t in is loaded with the first probe round and used when the entry
// found lies inside it.
#ifndef RMQ_FETCH_PPL
#define RMQ_FETCH_PPL 2
#endif
// header-window pieces per lane: 2 (512 B windows); 4 (1 KB: the whole 1 KB interval in one window)
// measured slower, 28.1-29.1 vs 26.5-26.8 us per max = 10 fetch (more loads, 6 waves per SIMD)
constexpr u32 kPPL = RMQ_FETCH_PPL;
static_assert(kPPL == 2 || kPPL == 4, "two or four pieces per lane");

// The length words of window pieces kPPL*hl .. kPPL*hl + kPPL-1 (16-byte pieces from byte wb).
struct WinWords {
  u32 w[4];
};
__device__ __forceinline__ WinWords load_window(const uint8_t* ring, u64 wb, u32 hl, u64 mask) {
  WinWords x{};
#pragma unroll
  for (u32 k = 0; k < kPPL; ++k)
    x.w[k] = *reinterpret_cast<const u32*>(ring + ((wb + 16ull * (kPPL * hl + k) + 8ull) & mask));
  return x;
}

// hit: the position cache holds the position of record h_off <= t (h_pos): no index search, the
// walk starts there.
__device__ __forceinline__ u64 record_posq(const DevState& st, const PartView& v, u64 t, bool act, bool hit,
                                           u64 h_off, u64 h_pos) {
  const u32 lane = lane_id(), h = lane / kQL, hl = lane % kQL;
  constexpr u32 kWin = kPPL * kQL;  // pieces per header window
  const u32 ilog = st.interval_log2;
  const u64 I = 1ull << ilog;
  const u64* E = st.index + v.rg.ibase * 2;
  u64 c_off = v.start_off, c_pos = v.start_pos;
  long lo = (long)((v.start_pos + I - 1) >> ilog), hi = (long)(v.used >> ilog);
  bool open = act && t < v.leo && lo <= hi;
  long ws = lo, step = 1;
  const u64 mask = v.rg.seg - 1;
  u64 sw = ~0ull;  // speculative header window
  if (act && hit) {
    open = false;
    c_off = h_off;
    c_pos = h_pos;
    sw = h_pos & ~15ull;
  } else if (open) {
    const double f = (double)(t - v.start_off) / (double)(v.leo - v.start_off);
    const u64 gpos = v.start_pos + (u64)(f * (double)(v.used - v.start_pos));
    const long me = (long)(gpos >> ilog);
    ws = max(lo, min(me - (long)(kQL / 2 - 1), hi - (long)(kQL - 1)));
    sw = max((u64)me << ilog, v.start_pos) & ~15ull;
  } else if (act && t < v.leo) {
    sw = v.start_pos;  // no index entry past the start: the walk starts at the log start
  }
  WinWords Sw{};
  if (sw != ~0ull) Sw = load_window(v.ring, sw, hl, mask);
  constexpr u32 kQMask = (1u << kQL) - 1u;
  for (bool first = true; __any(open); first = false) {
    if (!first) {
      ws = lo;
      step = (hi - lo + (long)kQL) / (long)kQL;
    }
    const long we = min(hi, ws + (long)(kQL - 1) * step);  // last probe of the round
    const long m = ws + (long)hl * step;
    bool le = false;
    u64 eo = 0, ep = 0;
    if (open && m <= we) {
      const u64* e = E + ((u64)m % v.rg.icap) * 2;
      eo = e[0];
      ep = e[1];
      le = eo <= t;
    }
    const u32 bal = (u32)(__ballot(le) >> (kQL * h)) & kQMask;  // this quarter's probes
    const u32 last = bal ? 31u - (u32)__builtin_clz(bal) : 0u;
    const u64 so = __shfl(eo, (int)(kQL * h + last), 64), sp = __shfl(ep, (int)(kQL * h + last), 64);
    if (open) {
      if (!bal) {  // every probe past t: the answer precedes this round's first probe
        hi = ws - 1;
        open = lo <= hi;
      } else {
        c_off = so;
        c_pos = sp;
        const long mk = ws + (long)last * step;  // a probe at or before t
        if (step == 1 && (mk < we || we == hi)) {
          open = false;  // the next entry is past t (or there is none)
        } else {
          lo = mk + 1;  // the answer is that probe or a later entry, up to the next probe
          if (step > 1 && mk < we) hi = min(hi, mk + step - 1);
          open = lo <= hi;
        }
      }
    }
  }
  if (!act) return 0;
  if (t >= v.leo) return v.used;
  u64 wb = sw;
  WinWords Lw = Sw;
  u32 cur = (u32)((c_pos - sw) >> 4);  // window piece of the current record
  if (sw == ~0ull || c_pos < sw || c_pos >= sw + 16ull * kWin) {
    wb = c_pos;
    cur = 0;
    Lw = load_window(v.ring, wb, hl, mask);
  }
  u64 k = t - c_off;
  while (__any(k > 0)) {
    const bool mv = k > 0 && cur >= kWin;  // quarter-uniform: the quarter walked off its window
    if (__any(mv)) {
      if (mv) {
        wb += 16ull * cur;
        cur = 0;
        Lw = load_window(v.ring, wb, hl, mask);
      }
    }
    const u32 src = kQL * h + (cur / kPPL);
    u32 a = 0;
#pragma unroll
    for (u32 q = 0; q < kPPL; ++q) {
      const u32 x = (u32)__shfl((int)Lw.w[q], (int)(src & 63u), 64);
      a = (cur % kPPL) == q ? x : a;
    }
    if (k > 0) {
      cur += record_bytes(a) >> 4;
      --k;
    }
  }
  return wb + 16ull * cur;
}

// Request r, resolved by one half-wave (half-uniform results): status, start offset, count,
// bytes, the source position and the ring word {ring byte offset in logs << 6 | log2(ring bytes)}.
struct Resolved {
  u64 start, count, bytes, pos0, ring;
  int status;
};

__device__ __forceinline__ Resolved resolve_request(const FetchArgs& a, const uint4 rq, bool live) {
  const DevState& st = a.st;
  const u32 p = rq.x, c = rq.y, mx = rq.z;
  int status = kOk;
  u64 start = 0, count = 0, end = 0, ring_off = 0;
  // every word of the partition in one round, the leader flag included (a request refused by the
  // checks below, or with an empty slice, leaves them unused)
  const bool okp = live && p < st.P;
  const u32 pp = okp ? p : 0u, cc = c < st.C ? c : 0u;
  const u32 lead = okp ? st.is_leader[pp] : 0u;
  // RMQ_FETCH_REPLICA: this engine's own replica, from its replica cursor, leader or follower
  const bool rep = a.replica && (rq.w & kFetchReplica);
  const u64 off = okp ? (rep ? st.rcur[pp] : st.cons[(u64)pp * st.C + cc]) : 0ull;
  const u64 hw = okp ? st.hw[pp] : 0ull;
  PartView v;
  v.leo = okp ? st.leo[pp] : 0ull;
  v.used = okp ? st.used[pp] : 0ull;
  v.start_off = okp ? st.start_off[pp] : 0ull;
  v.start_pos = okp ? st.start_pos[pp] : 0ull;
  const u32 lm = okp ? st.local_mask[pp] : 0u;
  const u64 desc = okp ? st.ring[pp] : 0ull;
  const ulonglong2 ce = okp ? *reinterpret_cast<const ulonglong2*>(st.pcache + ((u64)pp * st.C + cc) * 2)
                            : make_ulonglong2(~0ull, 0ull);
  const u64 h_off = ce.x, h_pos = ce.y;
  v.rg = ring_ref(desc, st.interval_log2, st.icap_mul);
  v.ring = st.logs;
  bool need = false;  // the slice is not empty: both its ends are searched
  if (!live) {
  } else if (p >= st.P) {
    status = kNoPart;
  } else if (!lead && !rep) {
    status = kNotLeader;
  } else if (c >= st.C) {
    status = kInval;
  } else {
    start = off;
    u64 lim = off + mx;
    if (lim < off) lim = ~0ull;
    end = lim < hw ? lim : hw;
    if (off < end) {
      if (off < v.start_off) {
        status = kOffset;
        start = v.start_off;  // where the consumer can resume (FORMAT.md §7)
      } else {
        const u32 r0 = lm ? (u32)__ffs(lm) - 1u : 0u;
        ring_off = (u64)r0 * st.rstride + v.rg.base;
        v.ring = st.logs + ring_off;
        count = end - off;
        need = true;
      }
    }
  }
  // quarter 0 of the half: the slice's first record, quarter 1: one past its last
  const u32 hb = lane_id() & 32u;
  // the position cache (the record after this consumer's last served slice): a consumer reading on
  // from there skips the index search, and walks from the cached position (a short slice only:
  // a long one takes the search, which skips most of it)
  const bool hit = need && h_off == off && h_pos >= v.start_pos && h_pos < v.used && count <= kWalkMax;
  const u64 pq = record_posq(st, v, (lane_id() & 16u) ? end : off, need, hit, off, h_pos);
  const u64 pos0 = __shfl(pq, (int)hb, 64), pend = __shfl(pq, (int)(hb + 16u), 64);
  return Resolved{start, count, need ? pend - pos0 : 0ull, pos0, (ring_off << 6) | (desc & 63ull), status};
}

// The ticket of workgroup b (wg0: first workgroup of each ticket) and b's index inside it; the
// arguments are read in place from the kernarg segment (an indexed by-value copy could go to scratch).
// kMulti false: a launch of one ticket (every synchronous fetch, every fetch that commits): its
// arguments at fixed kernarg offsets, as before batches existed.
template <bool kMulti>
__device__ __forceinline__ const FetchArgs& ticket_of(const u32* wg0, u32& b) {
  if (!kMulti) return *(const FetchArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const FetchBatch& B = *(const FetchBatch*)__builtin_amdgcn_kernarg_segment_ptr();
  u32 k = 0;
#pragma unroll
  for (u32 i = 1; i < kFetchBatch; ++i) k += (i < B.nt && b >= wg0[i]) ? 1u : 0u;
  b -= wg0[k];
  return B.t[k];
}

template <bool kMulti>
using FetchKArgs = typename std::conditional<kMulti, FetchBatch, FetchArgs>::type;  // (t[0] first in both)
static_assert(offsetof(FetchBatch, t) == 0, "a batch's first ticket at the kernarg base");

template <bool kMulti>
__global__ __launch_bounds__(64 * kRW) void fetch_resolve_kernel(FetchKArgs<kMulti> batch) {
  (void)batch;
  const FetchBatch& B = *(const FetchBatch*)__builtin_amdgcn_kernarg_segment_ptr();
  u32 bid = blockIdx.x;
  const FetchArgs& a = ticket_of<kMulti>(B.rwg0, bid);
  const u32 lane = lane_id(), w = threadIdx.x >> 6;
  const u32 r = (bid * kRW + w) * kRPW + (lane >> 5);
  const bool live = r < a.n;  // (no early return: the workgroup meets at barriers below)
  // the workgroup's request rows, read once by one load of consecutive 16-byte rows (host rows:
  // one PCIe read of 128 bytes instead of a 16-byte read per request), through LDS; the device
  // copy for the gather and the position cache
  __shared__ uint4 s_rq[kRW * kRPW];
  {
    const u32 r0 = bid * kRW * kRPW + threadIdx.x;
    if (threadIdx.x < kRW * kRPW && r0 < a.n) {
      const uint4 x = *reinterpret_cast<const uint4*>(a.req + 4ull * r0);
      s_rq[threadIdx.x] = x;
      if (a.req != a.req_dev) *reinterpret_cast<uint4*>(a.req_dev + 4ull * r0) = x;
    }
  }
  __syncthreads();
  const Resolved q = resolve_request(a, live ? s_rq[w * kRPW + (lane >> 5)] : make_uint4(0, 0, 0, 0), live);
  __shared__ u64 s_b[kRW];
  const u64 b2 = bcast_u64(q.bytes, 0) + bcast_u64(q.bytes, 32);  // the wave's two requests
  if (lane == 0) s_b[w] = b2;
  if (live && (lane & 31u) == 0) {
    // the position cache's next entry for this consumer: the record after the slice (a served
    // request's partition and consumer are in range; reloaded here rather than held through the
    // resolve, which would take 8 more VGPRs)
    if (q.status == kOk && q.count) {
      // one 16-byte store: requests of one (partition, consumer) in one call (allowed when none
      // commits) each write a true {offset, position} pair, and a pair is never torn between two
      u64* ce = a.st.pcache + ((u64)a.req_dev[4 * r] * a.st.C + a.req_dev[4 * r + 1]) * 2;
      *reinterpret_cast<ulonglong2*>(ce) = make_ulonglong2(q.start + q.count, q.pos0 + q.bytes);
    }
    a.res[4 * r + 0] = q.start;
    a.res[4 * r + 2] = q.count | (q.bytes << 32);
    a.res[4 * r + 3] = (u64)(uint32_t)q.status;
    a.aux[2 * r + 0] = q.pos0;
    a.aux[2 * r + 1] = q.ring;
    a.cpre[r] = (u32)q.bytes;
  }
  // one add per workgroup (its kRW * kRPW requests share a chunk) into the chunk's own L2 line
  static_assert(kFetchChunk % (kRW * kRPW) == 0, "a resolve workgroup never straddles a chunk");
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 b = 0;
    for (u32 k = 0; k < kRW; ++k) b += s_b[k];
    if (b) atomicAdd((unsigned long long*)&a.csum[(u64)(bid * kRW * kRPW / kFetchChunk) * kCsumStride], (unsigned long long)b);
  }
}

// Lane src's value (src per lane).
__device__ __forceinline__ u64 shfl_u64(u64 v, int src) {
  return ((u64)(u32)__shfl((int)(v >> 32), src, 64) << 32) | (u32)__shfl((int)(u32)v, src, 64);
}

constexpr u32 kGQ = 4;          // requests per gather wave
constexpr u32 kGR = kFW * kGQ;  // requests per gather workgroup

// Placement + gather: workgroup per kGR consecutive requests. Two rounds of loads: the wave's
// request words with the placement sums, then (requests of at most 128 pieces) the records' pieces,
// issued before the placement barriers; only the stores wait for the output positions.
template <bool kMulti>
__global__ __launch_bounds__(64 * kFW) void fetch_gather_kernel(FetchKArgs<kMulti> batch) {
  (void)batch;
  const FetchBatch& B = *(const FetchBatch*)__builtin_amdgcn_kernarg_segment_ptr();
  u32 bid = blockIdx.x;
  const FetchArgs& a = ticket_of<kMulti>(B.gwg0, bid);
  const u32 nwg = (a.n + kGR - 1) / kGR;  // the ticket's gather workgroups
  __shared__ u64 s_red[kFW];
  __shared__ u64 s_pos[kGR];
  const DevState& st = a.st;
  const u32 tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const u32 r0 = bid * kGR, c0 = r0 / kFetchChunk;
  // the wave's kGQ requests (lanes 0..kGQ-1 read one each)
  const u32 rq = r0 + w * kGQ + (lane < kGQ ? lane : 0u);
  const bool qv = lane < kGQ && rq < a.n;
  const u64 q_pos = qv ? a.aux[2 * rq + 0] : 0ull, q_ring = qv ? a.aux[2 * rq + 1] : 0ull;
  const u64 q_nb = qv ? a.cpre[rq] : 0ull;
  // the next fetch's chunk sums (its resolve runs after this kernel on the same stream)
  for (u32 k = bid * 64 * kFW + tid; k < a.csum_lines; k += nwg * 64 * kFW) a.csum_next[(u64)k * kCsumStride] = 0;
  // bytes of every request before r0: the chunk sums before its chunk, then its chunk's requests
  u64 v = 0;
  for (u32 k = tid; k < c0; k += 64 * kFW) v += a.csum[(u64)k * kCsumStride];
  for (u32 k = c0 * kFetchChunk + tid; k < r0; k += 64 * kFW) v += a.cpre[k];
  const u32 rr = r0 + tid;
  const u64 nb = tid < kGR && rr < a.n ? a.cpre[rr] : 0ull;
  // requests of at most 128 pieces each (max = 10 of short records): all four copied with one round
  // of loads (two pieces per lane and request), loaded now, stored once placed (named registers:
  // a local array here went to scratch)
  bool small = true;
#pragma unroll
  for (u32 q = 0; q < kGQ; ++q) small = small && (bcast_u64(q_nb, q) >> 4) <= 128u;
#define RMQ_GQ_LOAD(q, x0, x1)                                                                        \
  uint4 x0 = make_uint4(0, 0, 0, 0), x1 = x0;                                                        \
  if (small) {                                                                                        \
    const u64 nbr = bcast_u64(q_nb, q);                                                               \
    const u64 pos0 = bcast_u64(q_pos, q), rw = bcast_u64(q_ring, q);                                  \
    const uint8_t* ring = st.logs + (rw >> 6);                                                        \
    const u64 mask = (1ull << (rw & 63ull)) - 1ull;                                                   \
    if (lane < (nbr >> 4)) x0 = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * lane) & mask)); \
    if (lane + 64u < (nbr >> 4)) x1 = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * (lane + 64u)) & mask)); \
  }
  static_assert(kGQ == 4, "four requests per gather wave");
  RMQ_GQ_LOAD(0, a0, a1)
  RMQ_GQ_LOAD(1, b0, b1)
  RMQ_GQ_LOAD(2, c0_, c1_)
  RMQ_GQ_LOAD(3, d0, d1)
#undef RMQ_GQ_LOAD
  v = bcast_u64(wave_incl_scan(v), 63);  // the wave's sum
  if (lane == 0) s_red[w] = v;
  // this workgroup's requests: exclusive scan of their bytes
  const u64 inc = wave_incl_scan(nb);  // kGR <= 64: one wave holds them all
  __syncthreads();
  const u64 base = s_red[0] + s_red[1] + s_red[2] + s_red[3];
  u64 f0 = 0, f1 = 0, f2 = 0, f3 = 0;  // the final row of request rr (tid < kGR)
  if (tid < kGR && rr < a.n) {
    const u64 pos = base + inc - nb;
    s_pos[tid] = pos;
    u64 w0 = a.res[4 * rr], w2 = a.res[4 * rr + 2], w3 = a.res[4 * rr + 3];  // the resolve's words
    const bool nospc = nb && pos + nb > a.out_cap;
    const int s0 = (int)(uint32_t)w3;
    if (nospc) {  // does not fit: not served (rare); its bytes still count
      w2 = 0;
      w3 = (u64)(uint32_t)kNoSpc;
    }
    f0 = w0;
    f1 = pos;
    f2 = w2;
    f3 = w3;
    if (rr + 1 == a.n)  // bytes needed
      __hip_atomic_store(a.need_host, pos + nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // RMQ_FETCH_COMMIT: the consumer's next offset once its records are in the output (or the
    // first retained offset after RMQ_EOFFSET); every request's offset was read by the resolve
    // kernel before (the host refuses two committing requests for one consumer in a call)
    if (a.commits && (a.req_dev[4 * rr + 3] & 1u)) {
      if (!nospc && (s0 == kOk || s0 == kOffset)) {
        const u32 p = a.req_dev[4 * rr], c = a.req_dev[4 * rr + 1];
        const u64 nx = w0 + (s0 == kOk ? (u64)(uint32_t)w2 : 0ull);
        if (a.replica && (a.req_dev[4 * rr + 3] & kFetchReplica)) {
          a.st.rcur[p] = nx;  // the replica cursor (local: no round carries it)
        } else {
          a.st.cons[(u64)p * a.st.C + c] = nx;
          a.st.cdirty[p] = 1u;  // (with a transport the row travels with the next round)
        }
      }
    }
  }
  if (w == 0) {
    // the final rows into the caller's page-locked rows (or the slot's staging rows): lane j
    // stores half j & 1 of row r0 + j / 2, so one store covers the workgroup's rows contiguously
    // (host rows: whole PCIe writes, not 16-byte pieces at a 32-byte stride)
    static_assert(2 * kGR <= 64, "one wave holds the workgroup's rows");
    const int src = (int)(lane >> 1);
    const u64 x0 = shfl_u64(f0, src), x1 = shfl_u64(f1, src), x2 = shfl_u64(f2, src), x3 = shfl_u64(f3, src);
    if (lane < 2 * kGR && r0 + (lane >> 1) < a.n)
      *reinterpret_cast<ulonglong2*>(a.res_host + 4ull * r0 + 2ull * lane) =
          (lane & 1u) ? make_ulonglong2(x2, x3) : make_ulonglong2(x0, x1);
  }
  __syncthreads();
  // the wave's requests one after the other (one stream of 16-byte pieces per wave: four requests
  // side by side, a quarter-wave or an interleaved run each, measured 1.7x slower at max = 1024)
  const u64 q_out = lane < kGQ ? s_pos[(w * kGQ + lane) & (kGR - 1u)] : 0ull;
  if (small) {
#define RMQ_GQ_STORE(q, x0, x1)                                                                       \
  {                                                                                                   \
    const u64 nbr = bcast_u64(q_nb, q), po = bcast_u64(q_out, q);                                     \
    const bool sv = nbr && po + nbr <= a.out_cap;  /* served (loaded speculatively either way) */   \
    if (sv && lane < (nbr >> 4)) *reinterpret_cast<uint4*>(a.out + po + 16ull * lane) = x0;         \
    if (sv && lane + 64u < (nbr >> 4)) *reinterpret_cast<uint4*>(a.out + po + 16ull * (lane + 64u)) = x1; \
  }
    RMQ_GQ_STORE(0, a0, a1)
    RMQ_GQ_STORE(1, b0, b1)
    RMQ_GQ_STORE(2, c0_, c1_)
    RMQ_GQ_STORE(3, d0, d1)
#undef RMQ_GQ_STORE
    return;
  }
  for (u32 q = 0; q < kGQ; ++q) {
    const u64 nbr = bcast_u64(q_nb, q), pos0_out = bcast_u64(q_out, q);
    if (!nbr || pos0_out + nbr > a.out_cap) continue;  // nothing, past the end, or not served
    const u64 pos0 = bcast_u64(q_pos, q), rw = bcast_u64(q_ring, q);
    const uint8_t* ring = st.logs + (rw >> 6);
    const u64 mask = (1ull << (rw & 63ull)) - 1ull;
    uint8_t* out = a.out + pos0_out;
    const u64 pieces = nbr >> 4;
    u64 p = lane;
    for (; p + 192 < pieces; p += 256) {  // four 16-byte pieces in flight per lane
      const uint4 x0 = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * p) & mask));
      const uint4 x1 = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * (p + 64)) & mask));
      const uint4 x2 = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * (p + 128)) & mask));
      const uint4 x3 = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * (p + 192)) & mask));
      *reinterpret_cast<uint4*>(out + 16ull * p) = x0;
      *reinterpret_cast<uint4*>(out + 16ull * (p + 64)) = x1;
      *reinterpret_cast<uint4*>(out + 16ull * (p + 128)) = x2;
      *reinterpret_cast<uint4*>(out + 16ull * (p + 192)) = x3;
    }
    for (; p < pieces; p += 64)
      *reinterpret_cast<uint4*>(out + 16ull * p) = *reinterpret_cast<const uint4*>(ring + ((pos0 + 16ull * p) & mask));
  }
}

// ev[4]: start / end events of the two kernels, recorded by the dispatches themselves
// (profiling: kernel time without the host's launch gaps), or null
// Load the fetch kernels' code at engine creation (a process's first launch of a kernel otherwise
// loads it: ~20 ms inside the first rmq_fetch, profiles/r03q_prof).
void preload_fetch_kernels() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&fetch_resolve_kernel<false>));
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&fetch_gather_kernel<false>));
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&fetch_resolve_kernel<true>));
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&fetch_gather_kernel<true>));
}

static void launch_batch(const FetchBatch& b, hipStream_t s, const hipEvent_t* e) {
  if (!b.rwg0[b.nt]) return;
  if (b.nt == 1) {  // one ticket: the 4x smaller kernarg, fixed offsets
    hipExtLaunchKernelGGL(fetch_resolve_kernel<false>, dim3(b.rwg0[1]), dim3(64 * kRW), 0, s, e ? e[0] : nullptr,
                          e ? e[1] : nullptr, 0, b.t[0]);
    hipExtLaunchKernelGGL(fetch_gather_kernel<false>, dim3(b.gwg0[1]), dim3(64 * kFW), 0, s, e ? e[2] : nullptr,
                          e ? e[3] : nullptr, 0, b.t[0]);
    return;
  }
  hipExtLaunchKernelGGL(fetch_resolve_kernel<true>, dim3(b.rwg0[b.nt]), dim3(64 * kRW), 0, s, e ? e[0] : nullptr,
                        e ? e[1] : nullptr, 0, b);
  hipExtLaunchKernelGGL(fetch_gather_kernel<true>, dim3(b.gwg0[b.nt]), dim3(64 * kFW), 0, s, e ? e[2] : nullptr,
                        e ? e[3] : nullptr, 0, b);
}

void launch_fetch_batch(const FetchArgs* t, uint32_t nt, hipStream_t s) {
  FetchBatch b{};
  b.nt = nt;
  for (uint32_t k = 0; k < nt; ++k) {
    b.t[k] = t[k];
    b.rwg0[k + 1] = b.rwg0[k] + (t[k].n + kRW * kRPW - 1) / (kRW * kRPW);
    b.gwg0[k + 1] = b.gwg0[k] + (t[k].n + kGR - 1) / kGR;
  }
  launch_batch(b, s, nullptr);
}

void launch_fetch(const FetchArgs& a, hipStream_t s, const hipEvent_t* ev) {
  if (!a.n) return;
  FetchBatch b{};
  b.nt = 1;
  b.t[0] = a;
  b.rwg0[1] = (a.n + kRW * kRPW - 1) / (kRW * kRPW);
  b.gwg0[1] = (a.n + kGR - 1) / kGR;
  launch_batch(b, s, ev);
}

}  // namespace rmq
