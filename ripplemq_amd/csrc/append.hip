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
// Input: the batch in the sort's partition-major order (slot s -> record svals[s] of partition
// skeys[s], stable). One workgroup = 256 slots ("tile"), tiles taken from a monotonic ticket so
// every predecessor a tile waits for has already started.
//
// Per tile:
//  1. segmented block scan of (record count, record bytes) over the slots -> rank and byte offset
//     of every record inside its partition run;
//  2. the head of each run reads the partition's log end (offset, byte position) from state; a
//     run continued from earlier tiles gets its absolute base from a decoupled look-back over
//     {epoch|status|count} granules (wave-wide 64-tile window);
//  3. payloads are gathered into an LDS image laid out exactly as the log records (FORMAT.md:
//     u64 offset | u32 len | u32 crc32c | payload | pad to 4), CRC32C computed from LDS with
//     slicing-by-8 tables (one lane per record; one wave per record above 512 B, GF(2) combine);
//  4. the image is streamed to every local replica ring with dword stores that are contiguous
//     across lanes inside a partition run;
//  5. the slot that ends a run finalizes the partition: log end, local matchIndex, quorum commit,
//     high watermark, size retention.
// Tiles whose record bytes exceed the LDS image go through a wave-per-record direct path.
#include "device_common.hpp"
#include "kernels.hpp"
#include "partition_ops.hpp"

namespace rmq {

constexpr u32 kT = kAppendThreads;
constexpr u32 kTW = kT / 64;
constexpr u32 kImgDw = kAppendImageBytes / 4;
constexpr u32 kLongCrc = 512;  // payloads above this are CRC'd by a whole wave
constexpr u32 kStAgg = 1u, kStIncl = 2u;

struct AppendSmem {
  u32 crc[8][256];
  u32 img[kImgDw];
  uint8_t map[kImgDw];
  u64 rb_off[kT + 1];  // absolute base per run id (0 = run continued from earlier tiles)
  u64 rb_pos[kT + 1];
  u64 so[kT];          // payload source offset per slot
  u64 pos[kT];         // absolute logical byte position of the record
  u32 len[kT];
  u32 key[kT];
  u32 mask[kT];
  u32 imgoff[kT];
  u32 crcv[kT];
  u32 wsum[3][kTW];
  u32 wflag[kTW];
  u32 scan[kTW];
  u32 misc[8];
  u32 longlist[kT];
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
// rounded to 4; partial CRCs are shifted by the bytes that follow them and XOR-reduced.
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

__device__ __forceinline__ void finalize_partition(const DevState& st, u32 p, u64 end_off, u64 end_pos) {
  if (end_off == st.leo[p]) return;  // no record of this run was appended
  st.leo[p] = end_off;
  st.used[p] = end_pos;
  const u32 lm = st.local_mask[p];
  for (u32 r = 0; r < st.RF; ++r)
    if (lm >> r & 1u) st.match[(u64)p * st.RF + r] = end_off;
  commit_rule(st, p);
  const u64 sp = st.start_pos[p];
  if (end_pos - sp > st.seg) {  // size retention, FORMAT.md §4
    const u64 I = 1ull << st.interval_log2;
    const u64 m = (end_pos - st.seg + I - 1) >> st.interval_log2;
    const u64* e = st.index + ((u64)p * st.icap + m % st.icap) * 2;
    st.start_off[p] = e[0];
    st.start_pos[p] = e[1];
  }
}

__global__ __launch_bounds__(kT, 2) void append_kernel(AppendArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  AppendSmem& S = *reinterpret_cast<AppendSmem*>(smem_raw);
  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const DevState& st = a.st;
  const u64 nospace_limit = ((u64)a.nospace_limit_hi << 32) | a.nospace_limit_lo;
  const bool nospace = a.batch_info[0] > nospace_limit;

  for (u32 k = tid; k < 8 * 256; k += kT) (&S.crc[0][0])[k] = a.crc->table[k >> 8][k & 255];

  for (;;) {
    __syncthreads();
    if (tid == 0) S.misc[0] = (u32)(atomicAdd((unsigned long long*)a.tile_counter, 1ull) - a.tile_base);
    __syncthreads();
    const u32 tile = S.misc[0];
    if (tile >= a.tiles) break;

    const u32 s0 = tile * kT;
    const u32 s = s0 + tid;
    const bool in = s < a.n;
    const u32 last_slot = (s0 + kT < a.n ? s0 + kT : a.n) - 1 - s0;  // tid of the tile's last slot

    // ---- 1. per-slot record metadata
    u32 key = 0, rec = 0, L = 0, praw = 0;
    u64 so = 0;
    bool range_ok = false;
    if (in) {
      key = a.skeys[s];
      rec = a.svals[s];
      if (rec < a.n && key < st.P) {
        praw = a.pidx[rec];
        L = a.len[rec];
        so = a.src_off64 ? a.src_off64[rec] : (u64)a.src_off32[rec];
        range_ok = so <= a.payload_bytes && L <= a.payload_bytes - so;
      } else {
        rec = 0;
        key = 0;
        praw = 0xFFFFFFFFu;
        atomicOr(a.err, 2u);
      }
    }
    const bool okp = in && praw < st.P;
    const bool ok = okp && range_ok && st.is_leader[key] && !nospace;
    const u32 cnt = ok ? 1u : 0u;
    const u32 rs = ok ? 16u + ((L + 3u) & ~3u) : 0u;
    S.key[tid] = key;
    __syncthreads();
    u32 prev_key = 0, next_key = 0xFFFFFFFFu;
    if (in) {
      prev_key = tid ? S.key[tid - 1] : (s ? a.skeys[s - 1] : 0xFFFFFFFFu);
      if (s + 1 < a.n) next_key = tid + 1 < kT ? S.key[tid + 1] : a.skeys[s + 1];
    }
    const u32 head = in && (s == 0 || prev_key != key) ? 1u : 0u;
    const bool run_end = in && (s + 1 == a.n || next_key != key);

    if (nospace) {
      if (in) a.out_offsets[rec] = ~0ull;
      const u64 bm = __ballot(in);
      if (lane == 0 && bm) atomicAdd(&a.stats[3], (u32)__popcll(bm));
      continue;
    }

    // ---- 2. segmented scan of (cnt, bytes) with run heads; inclusive count of heads = run id
    u32 f = head, c_inc = cnt, b_inc = rs;
    {
      u32 f2 = head;
      wave_seg_incl_scan(f, c_inc);
      wave_seg_incl_scan(f2, b_inc);
    }
    u32 h_inc = wave_incl_scan(head);
    if (lane == 63) {
      S.wsum[0][w] = c_inc;
      S.wsum[1][w] = b_inc;
      S.wsum[2][w] = h_inc;
      S.wflag[w] = f;
    }
    __syncthreads();
    {
      u32 cc = 0, cb = 0, ch = 0;
      for (u32 k = 0; k < w; ++k) {
        if (S.wflag[k]) {
          cc = S.wsum[0][k];
          cb = S.wsum[1][k];
        } else {
          cc += S.wsum[0][k];
          cb += S.wsum[1][k];
        }
        ch += S.wsum[2][k];
      }
      if (!f) {
        c_inc += cc;
        b_inc += cb;
      }
      h_inc += ch;
    }
    const u32 c_exc = c_inc - cnt, b_exc = b_inc - rs;
    const u32 run_id = h_inc;  // 0: the run continued from the previous tile
    u32 tile_heads;
    if (tid == last_slot) S.misc[1] = h_inc;
    if (tid == 0) S.misc[3] = head;

    // ---- 3. run heads read the partition log end
    if (head) {
      S.rb_off[run_id] = st.leo[key];
      S.rb_pos[run_id] = st.used[key];
    }
    S.len[tid] = L;
    S.so[tid] = so;
    S.mask[tid] = ok ? st.local_mask[key] : 0u;
    __syncthreads();
    tile_heads = S.misc[1];
    const bool cont = S.misc[3] == 0u;  // slot s0 continues a run of the previous tile

    // publish the tile's state for the look-back of later tiles
    if (tid == last_slot) {
      if (tile_heads) {
        store_sc1_u64(&a.lb_abs[(u64)tile * 4 + 0], S.rb_off[run_id] + c_inc);
        store_sc1_u64(&a.lb_abs[(u64)tile * 4 + 1], S.rb_pos[run_id] + b_inc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gran_store(&a.lb_status[tile], a.epoch, (kStIncl << 30) | c_inc);
      } else {
        store_sc1_u64(&a.lb_abs[(u64)tile * 4 + 2], b_inc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gran_store(&a.lb_status[tile], a.epoch, (kStAgg << 30) | c_inc);
      }
    }

    // ---- image layout (non-segmented prefix of record bytes)
    u32 tb;
    const u32 ioff = block_excl_scan<kTW>(rs, S.scan, &tb);
    S.imgoff[tid] = ioff;
    const bool image = tb <= kAppendImageBytes;

    if (image) {
      for (u32 d = 0; d < rs / 4; ++d) S.map[ioff / 4 + d] = (uint8_t)tid;
      __syncthreads();
      // ---- 4a. gather payloads into the image (lanes walk consecutive dwords of a record)
      const u32 ndw = tb / 4;
      for (u32 dw = tid; dw < ndw; dw += kT) {
        const u32 k = S.map[dw];
        const u32 rel = dw - S.imgoff[k] / 4;
        if (rel >= 4) {
          const u32 b = 4 * (rel - 4), Lk = S.len[k];
          S.img[dw] = b < Lk ? load_payload_dw(a.payload, S.so[k] + b, Lk - b < 4 ? Lk - b : 4) : 0u;
        }
      }
      __syncthreads();
      // ---- 4b. CRC32C from LDS: one lane per short record, one wave per long record
      u32 crc = 0;
      if (ok && L <= kLongCrc) crc = crc32c_lds(S.crc, &S.img[ioff / 4 + 4], L);
      S.crcv[tid] = crc;
      {
        if (tid == 0) S.misc[2] = 0;
        __syncthreads();
        if (ok && L > kLongCrc) S.longlist[atomicAdd(&S.misc[2], 1u)] = tid;
        __syncthreads();
        const u32 nlong = S.misc[2];
        for (u32 q = w; q < nlong; q += kTW) {
          const u32 k = S.longlist[q];
          const u32 cr = wave_crc32c<true>(S.crc, a.crc, &S.img[S.imgoff[k] / 4 + 4], nullptr, 0, S.len[k]);
          if (lane == 0) S.crcv[k] = cr;
        }
      }
    }

    // ---- 2b. look-back for a run continued from earlier tiles (wave 0)
    if (cont && w == 0) {
      u64 acc_c = 0, acc_b = 0;
      long look = (long)tile - 1;
      u32 spins = 0;
      for (;;) {
        const long t = look - (long)lane;
        u64 x = 0;
        if (t >= 0) x = gran_load(&a.lb_status[t]);
        const bool ready = t >= 0 && (u32)(x >> 32) == a.epoch;
        const u32 stt = ((u32)x) >> 30;
        const u64 stop = __ballot(!ready || stt == kStIncl);
        const u32 fl = stop ? (u32)__ffsll((long long)stop) - 1u : 64u;
        // lanes below the first stop lane are aggregates: add them
        u64 ab = 0, ac = 0;
        if (lane < fl) {
          ac = ((u32)x) & 0x3FFFFFFFu;
          ab = load_sc1_u64(&a.lb_abs[(u64)t * 4 + 2]);
        }
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
        const u32 fready = __shfl(ready ? 1u : 0u, fl, 64);
        if (fready) {
          const long tf = look - (long)fl;
          u64 bo = 0, bp = 0;
          if (lane == 0) {
            bo = load_sc1_u64(&a.lb_abs[(u64)tf * 4 + 0]);
            bp = load_sc1_u64(&a.lb_abs[(u64)tf * 4 + 1]);
          }
          bo = __shfl(bo, 0, 64);
          bp = __shfl(bp, 0, 64);
          if (lane == 0) {
            S.rb_off[0] = bo + acc_c;
            S.rb_pos[0] = bp + acc_b;
          }
          break;
        }
        look -= (long)fl;  // consumed fl aggregates; wait for the not-yet-published tile
        if (++spins >= kSpinLimit) {
          if (lane == 0) {
            atomicOr(a.err, kErrSpinTimeout);
            S.rb_off[0] = 0;
            S.rb_pos[0] = 0;
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (cont && !tile_heads && tid == last_slot) {
      store_sc1_u64(&a.lb_abs[(u64)tile * 4 + 0], S.rb_off[0] + c_inc);
      store_sc1_u64(&a.lb_abs[(u64)tile * 4 + 1], S.rb_pos[0] + b_inc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      gran_store(&a.lb_status[tile], a.epoch, (kStIncl << 30) | c_inc);
    }

    // ---- absolute offset / position of every record
    const u64 off_abs = S.rb_off[run_id] + c_exc;
    const u64 pos_abs = S.rb_pos[run_id] + b_exc;
    S.pos[tid] = pos_abs;
    if (in) a.out_offsets[rec] = ok ? off_abs : ~0ull;
    if (ok) {
      // sparse offset index: multiples m*I in (pos, pos + rs] name the next record
      const u64 end = pos_abs + rs;
      for (u64 m = (pos_abs >> st.interval_log2) + 1; (m << st.interval_log2) <= end; ++m) {
        u64* e = st.index + ((u64)key * st.icap + m % st.icap) * 2;
        e[0] = off_abs + 1;
        e[1] = end;
      }
    }
    __syncthreads();

    if (image) {
      if (ok) {
        const u32 d0 = ioff / 4;
        S.img[d0 + 0] = (u32)off_abs;
        S.img[d0 + 1] = (u32)(off_abs >> 32);
        S.img[d0 + 2] = L;
        S.img[d0 + 3] = S.crcv[tid];
      }
      __syncthreads();
      // ---- 4c. stream the image into every local replica ring
      const u32 ndw = tb / 4;
      const u64 segmask = st.seg - 1;
      const u64 rstride = (u64)st.P * st.seg;
      for (u32 dw = tid; dw < ndw; dw += kT) {
        const u32 k = S.map[dw];
        const u32 v = S.img[dw];
        const u64 lp = S.pos[k] + (u64)(dw * 4 - S.imgoff[k]);
        uint8_t* dst = st.logs + (u64)S.key[k] * st.seg + (lp & segmask);
        const u32 msk = S.mask[k];
        for (u32 r = 0; r < st.RF; ++r)
          if (msk >> r & 1u) *reinterpret_cast<u32*>(dst + r * rstride) = v;
      }
    } else {
      // ---- direct path: one wave per record (tiles holding more bytes than the LDS image)
      const u64 segmask = st.seg - 1;
      const u64 rstride = (u64)st.P * st.seg;
      for (u32 k = w; k < kT; k += kTW) {
        const u32 msk = S.mask[k];
        if (!msk) continue;
        const u32 Lk = S.len[k];
        const u64 sk = S.so[k], P0 = S.pos[k];
        const u32 cr = wave_crc32c<false>(S.crc, a.crc, nullptr, a.payload, sk, Lk);
        uint8_t* base = st.logs + (u64)S.key[k] * st.seg;
        const u32 pdw = (Lk + 3u) >> 2;
        for (u32 d = lane; d < pdw; d += 64) {
          const u32 b = 4 * d;
          const u32 v = load_payload_dw(a.payload, sk + b, Lk - b < 4 ? Lk - b : 4);
          const u64 lp = P0 + 16 + b;
          for (u32 r = 0; r < st.RF; ++r)
            if (msk >> r & 1u) *reinterpret_cast<u32*>(base + r * rstride + (lp & segmask)) = v;
        }
        if (lane == 0) S.crcv[k] = cr;
      }
      __syncthreads();
      if (ok) {  // headers: the owner thread writes its record's 4 header dwords
        uint8_t* base = st.logs + (u64)key * st.seg;
        const u32 h[4] = {(u32)off_abs, (u32)(off_abs >> 32), L, S.crcv[tid]};
        const u32 msk = S.mask[tid];
        for (u32 d = 0; d < 4; ++d) {
          const u64 lp = pos_abs + 4ull * d;
          for (u32 r = 0; r < st.RF; ++r)
            if (msk >> r & 1u) *reinterpret_cast<u32*>(base + r * rstride + (lp & segmask)) = h[d];
        }
      }
    }

    // ---- 5. finalize partitions whose run ends in this tile
    if (run_end) finalize_partition(st, key, off_abs + cnt, pos_abs + rs);

    // ---- stats
    {
      const u64 m_app = __ballot(ok), m_nl = __ballot(okp && range_ok && !st.is_leader[key]),
                m_np = __ballot(in && !okp);
      if (lane == 0) {
        if (m_app) atomicAdd(&a.stats[0], (u32)__popcll(m_app));
        if (m_nl) atomicAdd(&a.stats[1], (u32)__popcll(m_nl));
        if (m_np) atomicAdd(&a.stats[2], (u32)__popcll(m_np));
      }
    }
  }
}

int append_blocks_per_cu() { return 2; }

void launch_append(const AppendArgs& a, uint32_t grid, hipStream_t s) {
  hipLaunchKernelGGL(append_kernel, dim3(grid), dim3(kT), sizeof(AppendSmem), s, a);
}

}  // namespace rmq
