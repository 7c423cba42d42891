// append.hip — the fused append kernel: per-partition offsets, CRC32C, replica-log scatter,
// sparse offset index, quorum commit and retention, in one launch per batch.
//
// Reference semantics restated here (file:line relative to the reference root):
//   PartitionStateMachine.onApply / handleMessageAppendRequest — messages.addAll(batch): record j
//   of the applied batch gets offset size_before + j, per partition, in apply order
//   (mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:38-69);
//   MessageAppendRequestProcessor "Not leader" gate (.../processor/MessageAppendRequestProcessor.java:29-32);
//   jraft BallotBox quorum commit: commit = max(commit, k-th largest matchIndex,
//   k = RF/2+1) when that entry is from the current term.
//
// Input: the sort's slot records {pidx, record, len, payload offset} in stable partition-major
// order. One WAVE = one tile of 64 slots (no workgroup barriers on the hot loop); waves take
// tiles from a monotonic ticket, so every tile a wave waits on has already started.
//
// Per tile:
//  1. wave segmented scan of (record count, record bytes) keyed by partition -> rank and byte
//     offset of each record inside its partition run;
//  2. the head of each run reads the partition's log end from state; a run continued from
//     earlier tiles gets its absolute base from a decoupled look-back over {epoch|status|count}
//     granules (64-tile window per probe);
//  3. the records are laid out in an LDS image exactly as in the log (FORMAT.md: u64 offset |
//     u32 len | u32 crc32c | payload | pad to 4); payload dwords arrive by LDS-DMA
//     (global_load_lds_dword, one wave-instruction per 256 image bytes, all in flight at once);
//  4. CRC32C from LDS, slicing-by-8 tables in LDS, one lane per record (a whole wave with GF(2)
//     shift-combine for payloads over 512 B);
//  5. the image streams to every local replica ring: dword stores contiguous across lanes inside
//     a run; the lane that ends a run finalizes the partition (log end, matchIndex, quorum commit,
//     high watermark, retention).
// Tiles whose records overflow the wave's LDS image, or with unaligned payloads, take a
// wave-per-record path with register staging.
#include "device_common.hpp"
#include "kernels.hpp"
#include "partition_ops.hpp"

namespace rmq {

constexpr u32 kWaves = kAppendThreads / 64;        // waves per workgroup
constexpr u32 kImgDw = kAppendImageBytes / 4;      // image dwords per wave
constexpr u32 kLongCrc = 512;                      // payloads above this: whole-wave CRC
constexpr u32 kStAgg = 1u, kStIncl = 2u;  // look-back granule tag = epoch << 2 | status
constexpr u32 kBadPart = 0x80000000u;              // slot len flag: pidx >= P

constexpr u32 kDmaChunks = kImgDw / 64;             // LDS-DMA wave-instructions per tile

struct alignas(16) WaveSmem {
  u32 img[kImgDw];
  uint8_t map[kImgDw];
  u64 pos[64];
  u64 ra[64];   // pos - imgoff: ring position of image byte 0 as seen by the record's dwords
  u32 km[64];   // key | local replica mask << 24 (P <= 2^24, RF <= 8)
  u32 key[64];
  u32 imgoff[64];
  u32 len[64];
  u32 so[64];
  u32 mask[64];
};

struct AppendSmem {
  u32 crc[8][256];
  u32 pow8[kCrcPow8];
  WaveSmem wv[kWaves];
};

__device__ __forceinline__ u32 load_payload_dw(const uint8_t* payload, u64 byte, u32 nb) {
  const uint8_t* p = payload + byte;
  const u64 a = reinterpret_cast<u64>(p) & ~3ull;
  const u32 sh = (u32)(reinterpret_cast<u64>(p) & 3ull);
  u32 v = *reinterpret_cast<const u32*>(a);
  if (sh) {
    v >>= 8 * sh;
    if (sh + nb > 4) v |= *reinterpret_cast<const u32*>(a + 4) << (32 - 8 * sh);
  }
  if (nb < 4) v &= (1u << (8 * nb)) - 1u;
  return v;
}

// x^(8n) mod P applied to crc (append n zero bytes), via the power-of-two shift table.
__device__ __forceinline__ u32 crc_shift(const CrcConsts* cc, u32 crc, u32 n) {
  for (u32 j = 0; n; ++j, n >>= 1)
    if (n & 1u) crc = gf2_mulmod(cc->shift_pow2[j], crc);
  return crc;
}

// Whole-wave CRC32C of a payload. Lane l takes bytes [l*c, min((l+1)*c, L)), c = ceil(L/64)
// rounded to 4; partial CRCs are shifted by the bytes that follow them and XOR-reduced
// (crc(A||B) = crc(A) * x^(8|B|) ^ crc(B), linear in each part).
template <bool kFromLds>
__device__ u32 wave_crc32c(const u32 (*t)[256], const CrcConsts* cc, const u32* lds_dw,
                           const uint8_t* payload, u64 src, u32 L) {
  const u32 lane = lane_id();
  const u32 c = ((L + 63u) / 64u + 3u) & ~3u;
  const u32 b0 = lane * c < L ? lane * c : L;
  const u32 b1 = b0 + c < L ? b0 + c : L;
  u32 crc = 0xFFFFFFFFu;
  for (u32 b = b0; b < b1; b += 4) {
    const u32 nb = b1 - b < 4 ? b1 - b : 4;
    const u32 w = kFromLds ? lds_dw[b >> 2] : load_payload_dw(payload, src + b, nb);
    if (nb == 4) {
      crc = crc_step4(t, crc, w);
    } else {
      for (u32 k = 0; k < nb; ++k) crc = crc_step1(t, crc, (w >> (8 * k)) & 0xFF);
    }
  }
  crc = b1 > b0 ? ~crc : 0u;
  crc = crc_shift(cc, crc, L - b1);
  for (int d = 32; d >= 1; d >>= 1) crc ^= __shfl_xor(crc, d, 64);
  return crc;
}

// Phase stamps for the diagnostic run (RMQ_STAMPS): never read by the kernel itself.
#define RMQ_STAMP(i)                                                                  \
  do {                                                                                \
    if (a.stamps) {                                                                   \
      const u64 t_ = __builtin_amdgcn_s_memrealtime();                                \
      if (lane == 0) a.stamps[(u64)tile * 8 + (i)] = t_;                              \
    }                                                                                 \
  } while (0)

__global__ __launch_bounds__(kAppendThreads, 2) void append_kernel(AppendArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  AppendSmem& S = *reinterpret_cast<AppendSmem*>(smem_raw);
  const u32 lane = threadIdx.x & 63;
  const u32 wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  WaveSmem& W = S.wv[wv];
  const DevState& st = a.st;
  const u64 nospace_limit = ((u64)a.nospace_limit_hi << 32) | a.nospace_limit_lo;
  const bool nospace = a.batch_info[0] > nospace_limit;
  const u32 RF = st.RF;

  for (u32 k = threadIdx.x; k < 8 * 256; k += kAppendThreads) (&S.crc[0][0])[k] = a.crc->table[k >> 8][k & 255];
  for (u32 k = threadIdx.x; k < kCrcPow8; k += kAppendThreads) S.pow8[k] = a.crc->pow8[k];
  __syncthreads();

  // Static tile assignment: wave gw takes tiles gw, gw + nw, ...; every wave of the grid is
  // resident (<= 2 workgroups per CU), and a wave only ever waits on lower tiles, which their
  // owners reach first, so the look-back cannot deadlock.
  const u32 nw = gridDim.x * kWaves;
  for (u32 tile = blockIdx.x * kWaves + wv; tile < a.tiles; tile += nw) {
    const u32 s0 = tile * 64u, s = s0 + lane;
    const bool in = s < a.n;
    const u32 nin = a.n - s0 < 64u ? a.n - s0 : 64u;  // valid slots in this tile
    const u32 last = nin - 1;
    RMQ_STAMP(0);

    // ---- 1. slot records, then the partition state (clamped indices, unbranched)
    const uint4 sr = a.slots[in ? s : a.n - 1];
    const u32 e_prev = a.slots[s0 ? s0 - 1 : 0].x;
    const u32 e_next = a.slots[s0 + nin < a.n ? s0 + nin : a.n - 1].x;
    const u32 key = sr.x, rec = sr.y, L = sr.z & ~kBadPart, so = sr.w;
    const u32 lead = st.is_leader[key];
    const u32 lmask = st.local_mask[key];
    // batch-start state of the record's partition. Safe to read here: the partition's finalizer
    // (this or a later tile) writes it only after this tile's look-back granules are published,
    // and those are published only after these loads have returned (vmcnt below).
    const u64 base_off = st.leo[key], base_pos = st.used[key];
    const u64 f_start = st.start_pos[key], f_term = st.term_start[key], f_commit = st.commit[key];
    u64 row[kMaxRF];
#pragma unroll
    for (u32 r = 0; r < kMaxRF; ++r) row[r] = r < RF ? st.match[(u64)key * RF + r] : 0ull;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    if (nospace) {
      if (in) a.out_offsets[rec] = ~0ull;
      if (lane == 0) a.tile_stats[tile] = make_uint4(0, 0, 0, nin);
      continue;
    }

    // ---- 2. image layout of every record with a valid partition and payload range (leadership
    // is not known yet; rejected records occupy image space but are never stored)
    const bool okp = in && !(sr.z & kBadPart);
    const bool range_ok = (u64)so + L <= a.payload_bytes;
    const bool img_rec = okp && range_ok;
    const u32 rs_img = img_rec ? record_bytes(L) : 0u;
    const u32 ioff = wave_incl_scan(rs_img) - rs_img;
    const u32 tb = __builtin_amdgcn_readlane(ioff + rs_img, 63);
    const bool aligned = __all(!img_rec || (so & 3u) == 0u);
    const bool image = tb <= kAppendImageBytes && aligned;
    const u32 ndw = tb >> 2;
    if (image) {
      // map: image dword -> owning lane (store pass); the image slots themselves carry each
      // payload dword's source offset until the DMA overwrites them (header slots: dummy 0)
      const u32 d0 = ioff / 4, pend = 4u + ((L + 3u) >> 2);  // payload dwords [4, pend)
      for (u32 d = 0; d < rs_img / 4; ++d) {
        W.map[d0 + d] = (uint8_t)lane;
        W.img[d0 + d] = (d < 4 || d >= pend) ? 0u : so + 4u * (d - 4u);
      }
    }
    __builtin_amdgcn_wave_barrier();

    // ---- 3. LDS-DMA gather: always exactly kDmaChunks wave-instructions (dummy source when not
    // needed), so `vmcnt(kDmaChunks)` below waits for the state loads alone. All source offsets
    // are read in one batch before the first DMA; DMA c overwrites only the slots of chunk c.
    {
      u32 srcoff[kDmaChunks];
#pragma unroll
      for (u32 c = 0; c < kDmaChunks; ++c) srcoff[c] = W.img[c * 64 + lane];
      const u32 imgm = 0u - (u32)image;
#pragma unroll
      for (u32 c = 0; c < kDmaChunks; ++c) {
        const u32 use = imgm & (0u - (u32)(c * 64 + lane < ndw));
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a.payload + (srcoff[c] & use)),
                                         (__attribute__((address_space(3))) void*)&W.img[c * 64], 4, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDmaChunks) : "memory");
    RMQ_STAMP(1);

    // ---- 4. segmented wave scans: count / bytes relative to the run start (or the tile start)
    u32 prev_key = __shfl_up(key, 1, 64), next_key = __shfl_down(key, 1, 64);
    prev_key = lane == 0 ? (s0 ? e_prev : 0xFFFFFFFFu) : prev_key;
    next_key = lane == last ? (s0 + nin < a.n ? e_next : 0xFFFFFFFFu) : next_key;
    const bool ok = img_rec && lead;
    const u32 cnt = ok ? 1u : 0u;
    const u32 rs = ok ? rs_img : 0u;
    const u32 head = in && (s == 0 || prev_key != key) ? 1u : 0u;
    const bool run_end = in && next_key != key;
    u32 fc = head, fb = head, c_inc = cnt, b_inc = rs;
    wave_seg_incl_scan(fc, c_inc);
    wave_seg_incl_scan(fb, b_inc);
    const u32 run_id = wave_incl_scan(head);  // 0: run continued from the previous tile
    const u32 c_exc = c_inc - cnt, b_exc = b_inc - rs;
    const u32 tile_heads = __builtin_amdgcn_readlane(run_id, last);
    const bool cont = __builtin_amdgcn_readfirstlane(head) == 0u;

    // publish {count, bytes} of the tile's last run relative to its batch start: INCL when the
    // run starts here, AGG (the tile's whole contribution) when it continued from before.
    if (lane == last) {
      const u32 tag = (a.epoch << 2) | (tile_heads ? kStIncl : kStAgg);
      gran_store(&a.lb_cnt[tile], tag, c_inc);
      gran_store(&a.lb_bytes[tile], tag, b_inc);
    }
    W.key[lane] = key;
    W.len[lane] = L;
    W.so[lane] = so;
    W.imgoff[lane] = ioff;
    W.mask[lane] = ok ? lmask : 0u;

    // ---- 5. CRC32C from the LDS image (pad bytes zeroed first: they are log bytes too)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA landed
    RMQ_STAMP(2);
    u32 crc = 0;
    if (image) {
      __builtin_amdgcn_wave_barrier();
      if (ok) {  // pad bytes: the tail of the last payload dword, then whole pad dwords
        const u32 d0 = ioff / 4, pend = 4u + ((L + 3u) >> 2);
        if (L & 3u) W.img[d0 + 4 + L / 4] &= (1u << (8 * (L & 3u))) - 1u;
        for (u32 d = pend; d < rs / 4; ++d) W.img[d0 + d] = 0u;
      }
      __builtin_amdgcn_wave_barrier();
      if (ok && L <= kLongCrc) crc = crc32c_lds4(S.crc, S.pow8, &W.img[ioff / 4 + 4], L);
      u64 longs = __ballot(ok && L > kLongCrc);
      while (longs) {
        const u32 k = (u32)__ffsll((long long)longs) - 1u;
        longs &= longs - 1;
        const u32 cr = wave_crc32c<true>(S.crc, a.crc, &W.img[W.imgoff[k] / 4 + 4], nullptr, 0, W.len[k]);
        crc = lane == k ? cr : crc;
      }
    }
    RMQ_STAMP(3);

    // ---- 6. look-back: relative count/bytes of the run before this tile
    u32 carry_c = 0, carry_b = 0;
    if (cont) {
      u32 acc_c = 0, acc_b = 0;
      long look = (long)tile - 1;
      for (u32 spins = 0;;) {
        const long t = look - (long)lane;
        const u64 tc = t >= 0 ? (u64)t : 0ull;  // predicated, not branched
        const u64 xc = gran_load(&a.lb_cnt[tc]);
        const u64 xb = gran_load(&a.lb_bytes[tc]);
        const u32 tag = (u32)(xc >> 32);
        const bool ready = t >= 0 && (tag >> 2) == a.epoch && (u32)(xb >> 32) == tag;
        const u64 stop = __ballot(!ready || (tag & 3u) == kStIncl);
        const u32 fl = stop ? (u32)__ffsll((long long)stop) - 1u : 64u;
        u32 ac = lane < fl ? (u32)xc : 0u, ab = lane < fl ? (u32)xb : 0u;
        for (int d = 32; d >= 1; d >>= 1) {
          ac += __shfl_xor(ac, d, 64);
          ab += __shfl_xor(ab, d, 64);
        }
        acc_c += ac;
        acc_b += ab;
        if (fl == 64) {
          look -= 64;
          continue;
        }
        if (__builtin_amdgcn_readlane(ready ? 1u : 0u, fl)) {
          carry_c = acc_c + __builtin_amdgcn_readlane((u32)xc, fl);
          carry_b = acc_b + __builtin_amdgcn_readlane((u32)xb, fl);
          break;
        }
        look -= (long)fl;  // consumed fl aggregates; wait for the unpublished tile
        if (++spins >= a.spin_limit) {
          atomicOr(a.err, kErrSpinTimeout);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!tile_heads && lane == last) {
        const u32 tag = (a.epoch << 2) | kStIncl;
        gran_store(&a.lb_cnt[tile], tag, carry_c + c_inc);
        gran_store(&a.lb_bytes[tile], tag, carry_b + b_inc);
      }
    }
    RMQ_STAMP(4);

    // ---- 7. absolute offset / position of every record, offsets out, sparse index
    const u32 rel_c = (run_id ? 0u : carry_c) + c_exc;
    const u32 rel_b = (run_id ? 0u : carry_b) + b_exc;
    const u64 off_abs = base_off + rel_c;
    const u64 pos_abs = base_pos + rel_b;
    W.pos[lane] = pos_abs;
    if (in) a.out_offsets[rec] = ok ? off_abs : ~0ull;
    if (ok) {  // sparse offset index: multiples m*I in (pos, pos + rs] name the next record
      const u64 end = pos_abs + rs;
      for (u64 m = (pos_abs >> st.interval_log2) + 1; (m << st.interval_log2) <= end; ++m) {
        u64* e = st.index + ((u64)key * st.icap + m % st.icap) * 2;
        e[0] = off_abs + 1;
        e[1] = end;
      }
    }

    const u64 segmask = st.seg - 1;
    const u64 rstride = (u64)st.P * st.seg;
    if (image) {
      W.ra[lane] = pos_abs - ioff;  // ring position of image byte 0 for this record's dwords
      W.km[lane] = key | (ok ? lmask << 24 : 0u);
      if (ok) {
        const u32 d0 = ioff / 4;
        W.img[d0 + 0] = (u32)off_abs;
        W.img[d0 + 1] = (u32)(off_abs >> 32);
        W.img[d0 + 2] = L;
        W.img[d0 + 3] = crc;
      }
      __builtin_amdgcn_wave_barrier();
      RMQ_STAMP(5);
      // ---- 8. stream the image into every local replica ring in 16-B pieces (records are
      // 16-B aligned in the image and in the ring, so a piece never straddles records or the
      // ring end): one dwordx4 store per lane per replica per KiB; all LDS reads of a batch of 4
      // chunks are issued before any store.
      const u32 npc = ndw >> 2;
      for (u32 c0 = 0; c0 * 64 < npc; c0 += 4) {
        u32 k[4], km[4];
        u64 ra[4];
        uint4 v[4];
#pragma unroll
        for (u32 j = 0; j < 4; ++j) k[j] = W.map[(((c0 + j) * 64 + lane) * 4) & (kImgDw - 1)];
#pragma unroll
        for (u32 j = 0; j < 4; ++j) {
          v[j] = *reinterpret_cast<const uint4*>(&W.img[(((c0 + j) * 64 + lane) * 4) & (kImgDw - 1)]);
          ra[j] = W.ra[k[j] & 63u];
          km[j] = W.km[k[j] & 63u];
        }
#pragma unroll
        for (u32 j = 0; j < 4; ++j) {
          const u32 q = (c0 + j) * 64 + lane;
          u32 msk = q < npc ? km[j] >> 24 : 0u;
          if (a.debug & 12u) msk = (a.debug & 4u) ? 0u : (msk & 1u);  // diagnostics: no stores / one replica
          if (msk) {
            const u64 lp = (ra[j] + 16ull * q) & segmask;
            uint8_t* dst = st.logs + (u64)(km[j] & 0xFFFFFFu) * st.seg + lp;
            for (u32 r = 0; r < RF; ++r)
              if (msk >> r & 1u) *reinterpret_cast<uint4*>(dst + r * rstride) = v[j];
          }
        }
      }
    } else {
      __builtin_amdgcn_wave_barrier();
      RMQ_STAMP(5);
      // ---- wave-per-record path (large or unaligned payloads)
      for (u32 k = 0; k < nin; ++k) {
        const u32 msk = __builtin_amdgcn_readfirstlane(W.mask[k]);
        if (!msk) continue;
        const u32 Lk = __builtin_amdgcn_readfirstlane(W.len[k]);
        const u64 sk = W.so[k], P0 = W.pos[k];
        const u32 cr = wave_crc32c<false>(S.crc, a.crc, nullptr, a.payload, sk, Lk);
        uint8_t* rb = st.logs + (u64)W.key[k] * st.seg;
        const u32 pdw = (Lk + 3u) >> 2, rdw = record_bytes(Lk) >> 2;
        const u64 ko = ((u64)__builtin_amdgcn_readlane((u32)(off_abs >> 32), k) << 32) |
                       __builtin_amdgcn_readlane((u32)off_abs, k);
        for (u32 d = lane; d < rdw; d += 64) {
          u32 v;
          if (d >= 4 + pdw) {
            v = 0u;  // pad dwords
          } else if (d >= 4) {
            const u32 b = 4 * (d - 4);
            v = load_payload_dw(a.payload, sk + b, Lk - b < 4 ? Lk - b : 4);
          } else {
            v = d == 0 ? (u32)ko : d == 1 ? (u32)(ko >> 32) : d == 2 ? Lk : cr;
          }
          const u64 lp = P0 + 4ull * d;
          for (u32 r = 0; r < RF; ++r)
            if (msk >> r & 1u) *reinterpret_cast<u32*>(rb + r * rstride + (lp & segmask)) = v;
        }
      }
    }

    RMQ_STAMP(6);
    // ---- 9. the lane that ends a run finalizes its partition (state prefetched in step 1)
    const u32 end_c = rel_c + cnt;
    if (run_end && end_c) {
      const u64 end_off = base_off + end_c, end_pos = base_pos + rel_b + rs;
      st.leo[key] = end_off;
      st.used[key] = end_pos;
#pragma unroll
      for (u32 r = 0; r < kMaxRF; ++r)
        if (r < RF && (lmask >> r & 1u)) {
          row[r] = end_off;
          st.match[(u64)key * RF + r] = end_off;
        }
      const u64 c = quorum_commit(row, RF, f_commit, f_term);
      st.commit[key] = c;
      st.hw[key] = c;
      if (end_pos - f_start > st.seg) {  // size retention, FORMAT.md §4
        const u64 I = 1ull << st.interval_log2;
        const u64 m = (end_pos - st.seg + I - 1) >> st.interval_log2;
        const u64* e = st.index + ((u64)key * st.icap + m % st.icap) * 2;
        st.start_off[key] = e[0];
        st.start_pos[key] = e[1];
      }
    }

    // ---- per-tile stats (no atomics): appended, not leader, unknown partition, no space
    {
      const u32 n_app = (u32)__popcll(__ballot(ok));
      const u32 n_nl = (u32)__popcll(__ballot(okp && range_ok && !lead));
      const u32 n_np = (u32)__popcll(__ballot(in && !okp));
      if (lane == 0) a.tile_stats[tile] = make_uint4(n_app, n_nl, n_np, 0);
    }
    if (a.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    RMQ_STAMP(7);
  }
}

int append_blocks_per_cu() { return 2; }
int append_waves_per_block() { return (int)kWaves; }

void launch_append(const AppendArgs& a, uint32_t grid, hipStream_t s) {
  hipLaunchKernelGGL(append_kernel, dim3(grid), dim3(kAppendThreads), sizeof(AppendSmem), s, a);
}

}  // namespace rmq
