/*
 * ripple_oracle.c — sequential CPU restatement of the reference partition state machine plus the
 * FORMAT.md byte layout. TEST INFRASTRUCTURE ONLY (see ripple_oracle.h for what it restates and
 * how it is pinned). Plain C99, one record at a time in apply order; no attempt to mirror how the
 * GPU engine computes anything (no sort, no scans, no sparse-index walk for lookups).
 */
#define _GNU_SOURCE /* pthread_setaffinity_np, CPU_SET: the sharded baseline pins its threads */
#include "ripple_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__) && defined(__SSE4_2__)
#include <nmmintrin.h>
#define RO_HAVE_SSE42 1
#else
#define RO_HAVE_SSE42 0
#endif

#define RO_POLY 0x82F63B78u /* CRC32C (Castagnoli), reflected */
#define RO_LTERM_BOUND (1ull << 63) /* lterm flag: the last entry's term is unknown, at most the value */

/* ------------------------------------------------------------------------------------------ */
/* CRC32C                                                                                      */
/* ------------------------------------------------------------------------------------------ */

uint32_t ro_crc32c_bitwise(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (RO_POLY & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}

static uint32_t ro_tab[8][256];
static int ro_tab_ready = 0;

static void ro_tab_init(void) {
  if (ro_tab_ready) return;
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (RO_POLY & (0u - (c & 1u)));
    ro_tab[0][b] = c;
  }
  for (uint32_t b = 0; b < 256; ++b)
    for (int t = 1; t < 8; ++t) ro_tab[t][b] = (ro_tab[t - 1][b] >> 8) ^ ro_tab[0][ro_tab[t - 1][b] & 0xFF];
  ro_tab_ready = 1;
}

int ro_crc32c_hw_available(void) { return RO_HAVE_SSE42; }

uint32_t ro_crc32c(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
#if RO_HAVE_SSE42
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c64 = _mm_crc32_u64(c64, v);
    p += 8;
    n -= 8;
  }
  c = (uint32_t)c64;
  while (n--) c = _mm_crc32_u8(c, *p++);
  return c ^ 0xFFFFFFFFu;
#else
  ro_tab_init();
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = ro_tab[7][lo & 0xFF] ^ ro_tab[6][(lo >> 8) & 0xFF] ^ ro_tab[5][(lo >> 16) & 0xFF] ^
        ro_tab[4][lo >> 24] ^ ro_tab[3][hi & 0xFF] ^ ro_tab[2][(hi >> 8) & 0xFF] ^
        ro_tab[1][(hi >> 16) & 0xFF] ^ ro_tab[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ ro_tab[0][(c ^ *p++) & 0xFF];
  return c ^ 0xFFFFFFFFu;
#endif
}

/* ------------------------------------------------------------------------------------------ */
/* State                                                                                       */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
  uint64_t* v;
  uint64_t n, cap;
} u64vec;

static int vec_push(u64vec* a, uint64_t x) {
  if (a->n == a->cap) {
    uint64_t nc = a->cap ? a->cap * 2 : 1024;
    uint64_t* nv = (uint64_t*)realloc(a->v, nc * sizeof(uint64_t));
    if (!nv) return -1;
    a->v = nv;
    a->cap = nc;
  }
  a->v[a->n++] = x;
  return 0;
}

typedef struct {
  uint64_t leo, used, start_off, start_pos, commit, hw, term, term_start;
  uint64_t match[RMQ_MAX_RF];
  uint32_t ranks[RMQ_MAX_RF];
  uint32_t leader_slot, is_leader;
  u64vec idx_off, idx_pos; /* sparse index entries E[m], m = 0.. (unbounded, logical) */
  u64vec rec_pos;          /* dense logical position of every record (oracle-only lookup) */
  uint64_t* cons;          /* consumer offsets (reference: HashMap<String,Long>, default 0) */
  uint64_t key;            /* placement key (FORMAT.md §9 list order), default pidx */
  uint64_t seg;            /* ring bytes of this partition (rmq_set_segments) */
  uint8_t* round;          /* records appended in the current replication round, log layout */
  uint64_t round_bytes, round_cap, round_count, round_first;
  uint64_t prev_round_bytes; /* record bytes of the round before (C = B less them: FORMAT.md §9) */
  /* leader, per replica slot (FORMAT.md §9 catch-up): expected follower log end before the next
     round, pending catch-up request {offset, position, round + 1 (0: none)}, last catch-up round */
  uint64_t nx_off[RMQ_MAX_RF], nx_pos[RMQ_MAX_RF];
  uint64_t rq_off[RMQ_MAX_RF], rq_pos[RMQ_MAX_RF], rq_r1[RMQ_MAX_RF], cu[RMQ_MAX_RF];
  uint8_t dirty; /* consumer offsets changed since the last round (the row travels with it) */
  uint64_t lc;   /* follower: the newest leader commit learned (round entries, commit notices) */
  /* consumer-offset rows on a quorum (offset tickets, FORMAT.md §8): the leader's row version (one
     per commit call touching the partition), per replica slot the newest version its follower
     acknowledged, and the version the last round carried to it (0: no row) */
  uint64_t cver, eackv[RMQ_MAX_RF], rowv[RMQ_MAX_RF];
  /* leader election (jraft's RequestVote, election timer and raft_meta,
     PartitionRaftServer.java:85,89): lterm = Raft's lastLogTerm, the newest term whose leader-start
     entry this log holds (0 = unknown older); mterm = the term in which this log was last verified
     against its leader's (a round entry accepted, or its own leadership): a commit notice of another
     term cannot move the commit over a tail never matched in it; heard = the round stamp of the last
     round entry or commit notice of the current term from the leader; vterm / vfor / led = the last
     vote (term, candidate) and whether this replica led that term */
  uint64_t lterm, mterm, heard, vterm;
  uint32_t vfor, led;
  uint64_t rcur; /* replica cursor: where an RMQ_FETCH_REPLICA read starts (local, never replicated) */
} ro_part;

struct ro_engine {
  rmq_config cfg;
  ro_part* parts;
  uint8_t** rings; /* [replica][partition] -> that partition's ring bytes */
  uint8_t* touched;
  uint64_t* pbytes; /* [P] record bytes of the current batch per partition */
  uint8_t* full;    /* [P] 1: the partition takes no record of the current batch (FORMAT.md §3) */
  uint32_t world;   /* replication ranks (1: none; FORMAT.md §9 rounds when > 1) */
  uint64_t counters[6]; /* follower: records ingested, refused (CRC), refused (log), bytes;
                           leader: catch-up entries, detached entry plans */
  uint64_t round_no;    /* replication round being formed (FORMAT.md §9 round number) */
};

/* leader: a partition's catch-up state starts over (placement, leader start: Raft's nextIndex =
   the leader's last index + 1) */
static void reset_catchup(ro_part* s) {
  for (uint32_t r = 0; r < RMQ_MAX_RF; ++r) {
    s->nx_off[r] = s->leo;
    s->nx_pos[r] = s->used;
    s->rq_r1[r] = s->rq_off[r] = s->rq_pos[r] = 0;
    s->cu[r] = 0;
  }
}

static int cfg_ok(const rmq_config* c) {
  if (!c || c->num_partitions == 0 || c->replication_factor == 0 || c->replication_factor > RMQ_MAX_RF)
    return 0;
  if (c->index_interval < 64 || (c->index_interval & (c->index_interval - 1))) return 0;
  if (c->segment_bytes == 0 || c->segment_bytes % c->index_interval) return 0;
  if (c->segment_bytes <= 2ull * c->index_interval) return 0;
  if (c->max_consumers == 0) return 0;
  return 1;
}

ro_engine* ro_create(const rmq_config* cfg) {
  if (!cfg_ok(cfg)) return NULL;
  ro_tab_init();
  ro_engine* e = (ro_engine*)calloc(1, sizeof(ro_engine));
  if (!e) return NULL;
  e->cfg = *cfg;
  e->world = 1;
  uint32_t P = cfg->num_partitions, RF = cfg->replication_factor;
  e->parts = (ro_part*)calloc(P, sizeof(ro_part));
  e->touched = (uint8_t*)calloc(P, 1);
  e->pbytes = (uint64_t*)calloc(P, sizeof(uint64_t));
  e->full = (uint8_t*)calloc(P, 1);
  e->rings = (uint8_t**)calloc((size_t)P * RF, sizeof(uint8_t*));
  if (!e->parts || !e->touched || !e->pbytes || !e->full || !e->rings) {
    ro_destroy(e);
    return NULL;
  }
  for (uint32_t p = 0; p < P; ++p) {
    ro_part* s = &e->parts[p];
    for (uint32_t r = 0; r < RF; ++r) s->ranks[r] = cfg->rank; /* all replicas co-located */
    s->leader_slot = 0;
    s->is_leader = 1; /* this engine leads every partition it hosts, term 1 */
    s->term = 1;
    s->term_start = 0;
    s->lterm = s->mterm = s->vterm = 1; /* led term 1 from creation, its vote its own */
    s->vfor = cfg->rank;
    s->led = 1;
    s->key = p;
    s->seg = cfg->segment_bytes;
    s->cons = (uint64_t*)calloc(cfg->max_consumers, sizeof(uint64_t));
    if (!s->cons || vec_push(&s->idx_off, 0) || vec_push(&s->idx_pos, 0)) { /* E[0] = (0, 0) */
      ro_destroy(e);
      return NULL;
    }
  }
  for (size_t k = 0; k < (size_t)P * RF; ++k) {
    e->rings[k] = (uint8_t*)calloc(cfg->segment_bytes, 1);
    if (!e->rings[k]) {
      ro_destroy(e);
      return NULL;
    }
  }
  return e;
}

void ro_destroy(ro_engine* e) {
  if (!e) return;
  uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  if (e->parts)
    for (uint32_t p = 0; p < P; ++p) {
      free(e->parts[p].idx_off.v);
      free(e->parts[p].idx_pos.v);
      free(e->parts[p].rec_pos.v);
      free(e->parts[p].cons);
      free(e->parts[p].round);
    }
  if (e->rings)
    for (size_t k = 0; k < (size_t)P * RF; ++k) free(e->rings[k]);
  free(e->rings);
  free(e->parts);
  free(e->touched);
  free(e->pbytes);
  free(e->full);
  free(e);
}

static uint8_t* ring_of(ro_engine* e, uint32_t replica, uint32_t p) {
  return e->rings[(size_t)replica * e->cfg.num_partitions + p];
}

static void ring_write(uint64_t S, uint8_t* ring, uint64_t pos, const uint8_t* src, uint64_t n) {
  while (n) {
    uint64_t o = pos % S, k = S - o < n ? S - o : n;
    memcpy(ring + o, src, k);
    pos += k;
    src += k;
    n -= k;
  }
}

static void ring_read(uint64_t S, const uint8_t* ring, uint64_t pos, uint8_t* dst, uint64_t n) {
  while (n) {
    uint64_t o = pos % S, k = S - o < n ? S - o : n;
    memcpy(dst, ring + o, k);
    pos += k;
    dst += k;
    n -= k;
  }
}

/* Raft quorum commit: N = k-th largest match, k = RF/2 + 1; commit moves to N only
   if N > commit and N >= term_start. The leader's term starts with a virtual entry at term_start
   (jraft appends a configuration entry at leader start [jraft]); a replica holds it once its match
   in the new term reaches term_start (match is reset at leader start), and a quorum holding it
   commits every earlier-term record before it (Raft's current-term rule; FORMAT.md §6). */
static void commit_eval(ro_engine* e, ro_part* s) {
  uint32_t RF = e->cfg.replication_factor, k = RF / 2 + 1;
  uint64_t m[RMQ_MAX_RF];
  for (uint32_t r = 0; r < RF; ++r) m[r] = s->match[r];
  for (uint32_t i = 1; i < RF; ++i) /* insertion sort, descending */
    for (uint32_t j = i; j > 0 && m[j - 1] < m[j]; --j) {
      uint64_t t = m[j];
      m[j] = m[j - 1];
      m[j - 1] = t;
    }
  uint64_t N = m[k - 1];
  if (N > s->commit && N >= s->term_start) s->commit = N;
  s->hw = s->commit;
}

/* Size retention (FORMAT.md §4): evaluated once per append batch. */
static void retention_eval(ro_engine* e, ro_part* s) {
  uint64_t S = s->seg, I = e->cfg.index_interval;
  if (s->used - s->start_pos <= S) return;
  uint64_t m = (s->used - S + I - 1) / I;
  s->start_off = s->idx_off.v[m];
  s->start_pos = s->idx_pos.v[m];
}

/* ------------------------------------------------------------------------------------------ */
/* Control                                                                                     */
/* ------------------------------------------------------------------------------------------ */

int ro_set_replicas(ro_engine* e, uint32_t p, const uint32_t* ranks, uint32_t rf, uint32_t leader_slot) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  if (!ranks || rf != e->cfg.replication_factor || leader_slot >= rf) return RMQ_EINVAL;
  ro_part* s = &e->parts[p];
  const uint32_t lead = ranks[leader_slot] == e->cfg.rank;
  if (s->is_leader && !lead && s->commit > s->lc) s->lc = s->commit; /* a deposed leader knows its commit */
  for (uint32_t r = 0; r < rf; ++r) s->ranks[r] = ranks[r];
  s->leader_slot = leader_slot;
  /* a placement keeps or ends this replica's leadership; it never starts one: a replica the placement
     names leader leads once rmq_become_leader passes Raft's checks (a refused one stays a follower) */
  s->is_leader = lead && s->is_leader;
  s->heard = e->round_no; /* the election timer restarts */
  reset_catchup(s);
  /* the followers acknowledge the rows afresh under the new placement: a led partition with
     committed offsets sends its row with the next round */
  for (uint32_t r = 0; r < RMQ_MAX_RF; ++r) s->eackv[r] = s->rowv[r] = 0;
  if (lead && s->cver && e->world > 1) s->dirty = 1;
  return RMQ_OK;
}

static int become_leader_one(ro_engine* e, uint32_t p, uint64_t term) {
  ro_part* s = &e->parts[p];
  uint32_t RF = e->cfg.replication_factor, slot = RF;
  if (term < s->term) return RMQ_EINVAL;
  for (uint32_t r = 0; r < RF; ++r)
    if (s->ranks[r] == e->cfg.rank) {
      slot = r;
      break;
    }
  if (slot == RF) return RMQ_EINVAL; /* no replica of p lives here */
  /* one leader per term: not a term this replica led, nor one it gave its vote to another candidate */
  if (s->vterm == term && (s->led || s->vfor != e->cfg.rank)) return RMQ_ETERM;
  return RMQ_OK;
}

/* Raft's vote restriction as far as a replica can tell: not a leader of a partition whose leader
   committed records its log does not hold. */
static int become_leader_check(ro_engine* e, uint32_t p) {
  /* the records this replica's log verifiably shares with its leader: all of it when it was matched in
     the current term, else its commit (committed records never change) */
  const ro_part* s = &e->parts[p];
  const uint64_t verified = s->mterm == s->term ? s->leo : s->commit;
  return verified < s->lc ? RMQ_ESTALE : RMQ_OK;
}

static void become_leader_apply(ro_engine* e, uint32_t p, uint64_t term) {
  ro_part* s = &e->parts[p];
  uint32_t RF = e->cfg.replication_factor, slot = 0;
  while (s->ranks[slot] != e->cfg.rank) ++slot;
  s->leader_slot = slot;
  s->is_leader = 1;
  s->term = term;
  s->term_start = s->leo; /* jraft: pendingIndex = lastLogIndex + 1 at leader start */
  s->lterm = s->mterm = term; /* its leader-start entry */
  s->vterm = term;
  s->vfor = e->cfg.rank;
  s->led = 1;
  for (uint32_t r = 0; r < RF; ++r) s->match[r] = s->ranks[r] == e->cfg.rank ? s->leo : 0;
  for (uint32_t r = 0; r < RF; ++r) s->eackv[r] = 0; /* rows acknowledged afresh in the new term */
  commit_eval(e, s);  /* the virtual leader-start entry: a local quorum holds it at once */
  s->dirty = 1;       /* the new leader's consumer offsets go to every follower with the next round */
  reset_catchup(s);
}

int ro_become_leader(ro_engine* e, uint32_t p, uint64_t term) {
  if (p != RMQ_ALL_PARTITIONS && p >= e->cfg.num_partitions) return RMQ_ENOPART;
  const uint32_t lo = p == RMQ_ALL_PARTITIONS ? 0 : p, hi = p == RMQ_ALL_PARTITIONS ? e->cfg.num_partitions : p + 1;
  for (uint32_t q = lo; q < hi; ++q) { /* every check before any change (as the engine) */
    int rc = become_leader_one(e, q, term);
    if (rc) return rc;
  }
  for (uint32_t q = lo; q < hi; ++q) {
    int rc = become_leader_check(e, q);
    if (rc) return rc;
  }
  for (uint32_t q = lo; q < hi; ++q) become_leader_apply(e, q, term);
  return RMQ_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Append: PartitionStateMachine.onApply -> handleMessageAppendRequest (messages.addAll)       */
/* ------------------------------------------------------------------------------------------ */

static uint64_t rec_size(uint32_t L) {
  return RMQ_RECORD_HEADER_BYTES + ((L + RMQ_RECORD_ALIGN - 1u) & ~(uint64_t)(RMQ_RECORD_ALIGN - 1u));
}

/* The payload-range check (RMQ_EINVAL) over every record. */
static int range_check(uint32_t n, const uint32_t* len, const uint64_t* payload_off, const uint8_t* payload,
                       uint64_t payload_bytes) {
  uint64_t run = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t off = payload_off ? payload_off[i] : run;
    if (len[i] && (!payload || off > payload_bytes || len[i] > payload_bytes - off)) return RMQ_EINVAL;
    run += len[i];
  }
  return RMQ_OK;
}

/* The FORMAT.md §3 space rule for the partitions p with p % T == t: bytes[p] = record bytes the
   batch holds for p; full[p] = 1 if they exceed segment - interval (p then takes no record of the
   batch). */
static void space_scan(const ro_engine* e, uint32_t n, const uint32_t* pidx, const uint32_t* len, uint64_t* bytes,
                       uint8_t* full, uint32_t t, uint32_t T) {
  const uint32_t P = e->cfg.num_partitions;
  for (uint32_t i = 0; i < n; ++i)
    if (pidx[i] < P && pidx[i] % T == t) bytes[pidx[i]] = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (pidx[i] < P && pidx[i] % T == t) bytes[pidx[i]] += rec_size(len[i]);
  for (uint32_t i = 0; i < n; ++i)
    if (pidx[i] < P && pidx[i] % T == t) full[pidx[i]] = bytes[pidx[i]] > e->parts[pidx[i]].seg - e->cfg.index_interval;
}

typedef struct {
  uint8_t* v;
  uint64_t cap;
} ro_buf;

/* One record of a partition this rank leads: header + payload + zero pad into every local replica
   ring at the log end, sparse-index entries, new log end. */
static int append_record(ro_engine* e, ro_part* s, uint32_t p, const uint8_t* src, uint32_t L, ro_buf* rec,
                         uint64_t* out_offset) {
  const rmq_config* c = &e->cfg;
  const uint64_t I = c->index_interval;
  const uint64_t rs = rec_size(L);
  if (rs > rec->cap) {
    uint8_t* nr = (uint8_t*)realloc(rec->v, rs);
    if (!nr) return RMQ_ENOMEM;
    rec->v = nr;
    rec->cap = rs;
  }
  uint8_t* r8 = rec->v;
  const uint64_t o = s->leo, pos = s->used;
  const uint32_t crc = ro_crc32c(src, L);
  memcpy(r8, &o, 8); /* little-endian host */
  memcpy(r8 + 8, &L, 4);
  memcpy(r8 + 12, &crc, 4);
  if (L) memcpy(r8 + 16, src, L);
  memset(r8 + 16 + L, 0, rs - 16 - L);
  for (uint32_t r = 0; r < c->replication_factor; ++r)
    if (s->ranks[r] == c->rank) ring_write(s->seg, ring_of(e, r, p), pos, r8, rs);
  /* sparse index: every multiple m*I in (pos, pos + rs] now names the next record */
  for (uint64_t m = pos / I + 1; m * I <= pos + rs; ++m)
    if (vec_push(&s->idx_off, o + 1) || vec_push(&s->idx_pos, pos + rs)) return RMQ_ENOMEM;
  if (vec_push(&s->rec_pos, pos)) return RMQ_ENOMEM;
  if (e->world > 1) { /* kept for the replication round (the ring may wrap inside a round) */
    if (s->round_bytes + rs > s->round_cap) {
      uint64_t nc = s->round_cap ? s->round_cap * 2 : 4096;
      while (nc < s->round_bytes + rs) nc *= 2;
      uint8_t* nr = (uint8_t*)realloc(s->round, nc);
      if (!nr) return RMQ_ENOMEM;
      s->round = nr;
      s->round_cap = nc;
    }
    memcpy(s->round + s->round_bytes, r8, rs);
    if (!s->round_count) s->round_first = o;
    s->round_bytes += rs;
    s->round_count++;
  }
  s->leo = o + 1;
  s->used = pos + rs;
  *out_offset = o;
  return RMQ_OK;
}

/* End of a batch for a partition that took records: co-located matchIndex, commit, retention. */
static void finish_partition(ro_engine* e, ro_part* s) {
  for (uint32_t r = 0; r < e->cfg.replication_factor; ++r)
    if (s->ranks[r] == e->cfg.rank) s->match[r] = s->leo; /* co-located replicas persisted */
  commit_eval(e, s);
  retention_eval(e, s);
}

int ro_append(ro_engine* e, uint32_t n, const uint32_t* pidx, const uint32_t* len,
              const uint64_t* payload_off, const uint8_t* payload, uint64_t payload_bytes,
              uint64_t* out_offsets, rmq_append_stats* stats) {
  const uint32_t P = e->cfg.num_partitions;
  rmq_append_stats st;
  memset(&st, 0, sizeof st);
  st.records = n;
  if (n && (!pidx || !len || !out_offsets)) return RMQ_EINVAL;
  int rc = range_check(n, len, payload_off, payload, payload_bytes);
  if (rc) return rc;
  space_scan(e, n, pidx, len, e->pbytes, e->full, 0, 1);
  memset(e->touched, 0, P);
  ro_buf rec = {NULL, 0};
  uint64_t run = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t off = payload_off ? payload_off[i] : run;
    run += len[i];
    const uint32_t p = pidx[i];
    if (p >= P) {
      out_offsets[i] = RMQ_OFFSET_NONE;
      st.rejected_no_partition++;
      continue;
    }
    ro_part* s = &e->parts[p];
    if (!s->is_leader) {
      out_offsets[i] = RMQ_OFFSET_NONE;
      st.rejected_not_leader++;
      continue;
    }
    if (e->full[p]) {
      out_offsets[i] = RMQ_OFFSET_NONE;
      st.rejected_no_space++;
      continue;
    }
    rc = append_record(e, s, p, payload + off, len[i], &rec, &out_offsets[i]);
    if (rc) {
      free(rec.v);
      return rc;
    }
    st.appended++;
    e->touched[p] = 1;
  }
  free(rec.v);
  for (uint32_t p = 0; p < P; ++p)
    if (e->touched[p]) finish_partition(e, &e->parts[p]);
  if (stats) *stats = st;
  return RMQ_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Partition-sharded append: the multi-core CPU baseline                        */
/* ------------------------------------------------------------------------------------------ */

/* Thread t of T applies, batch after batch, the records of the partitions it owns (p % T == t;
   unknown partitions go to thread 0). Partitions are independent Raft groups
   (mq-broker/src/main/java/metadata/PartitionManager.java:111-176), so this is ro_append batch by
   batch; every thread evaluates the batch rules itself and so stops at the same invalid batch. */
typedef struct {
  ro_engine* e;
  const rmq_batch* b;
  uint64_t* const* out;
  rmq_append_stats* st; /* [nb]: this thread's share */
  uint32_t nb, t, T, done;
  int cpu, rc;
} ro_shard;

static void* shard_main(void* arg) {
  ro_shard* j = (ro_shard*)arg;
  ro_engine* e = j->e;
  const uint32_t P = e->cfg.num_partitions;
  if (j->cpu >= 0) {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    CPU_SET(j->cpu, &cs);
    pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
  }
  ro_buf rec = {NULL, 0};
  uint32_t* mine = (uint32_t*)malloc(((size_t)P / j->T + 1) * sizeof(uint32_t));
  if (!mine) {
    j->rc = RMQ_ENOMEM;
    return NULL;
  }
  for (uint32_t k = 0; k < j->nb; ++k) {
    const rmq_batch* b = &j->b[k];
    uint64_t* out = j->out[k];
    rmq_append_stats* st = &j->st[k];
    int rc = range_check(b->n, b->len, b->payload_off, b->payload, b->payload_bytes);
    if (!rc) space_scan(e, b->n, b->pidx, b->len, e->pbytes, e->full, j->t, j->T); /* own partitions only */
    uint32_t nm = 0;
    uint64_t run = 0;
    for (uint32_t i = 0; i < b->n && !rc; ++i) {
      const uint32_t p = b->pidx[i];
      const uint64_t off = b->payload_off ? b->payload_off[i] : run;
      run += b->len[i];
      if ((p < P ? p % j->T : 0u) != j->t) continue;
      st->records++;
      if (p >= P) {
        out[i] = RMQ_OFFSET_NONE;
        st->rejected_no_partition++;
      } else if (!e->parts[p].is_leader) {
        out[i] = RMQ_OFFSET_NONE;
        st->rejected_not_leader++;
      } else if (e->full[p]) {
        out[i] = RMQ_OFFSET_NONE;
        st->rejected_no_space++;
      } else {
        rc = append_record(e, &e->parts[p], p, b->payload + off, b->len[i], &rec, &out[i]);
        if (rc) break;
        st->appended++;
        if (!e->touched[p]) {
          e->touched[p] = 1;
          mine[nm++] = p;
        }
      }
    }
    if (rc) {
      j->rc = rc;
      break;
    }
    for (uint32_t q = 0; q < nm; ++q) {
      finish_partition(e, &e->parts[mine[q]]);
      e->touched[mine[q]] = 0;
    }
    j->done = k + 1;
  }
  free(rec.v);
  free(mine);
  return NULL;
}

int ro_append_sharded(ro_engine* e, uint32_t nb, const rmq_batch* batches, uint64_t* const* out_offsets,
                      rmq_append_stats* stats, uint32_t threads, int pin, uint32_t* batches_done) {
  if (!e || (nb && (!batches || !out_offsets || !stats))) return RMQ_EINVAL;
  for (uint32_t k = 0; k < nb; ++k)
    if (batches[k].n && (!batches[k].pidx || !batches[k].len || !out_offsets[k])) return RMQ_EINVAL;
  const uint32_t P = e->cfg.num_partitions;
  uint32_t T = threads ? threads : 1u;
  if (T > P) T = P;
  int cpus[CPU_SETSIZE];
  int ncpu = 0;
  if (pin) {
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0)
      for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &cs)) cpus[ncpu++] = c;
  }
  ro_shard* J = (ro_shard*)calloc(T, sizeof *J);
  rmq_append_stats* S = (rmq_append_stats*)calloc((size_t)T * (nb ? nb : 1u), sizeof *S);
  pthread_t* th = (pthread_t*)calloc(T, sizeof *th);
  uint8_t* started = (uint8_t*)calloc(T, 1);
  if (!J || !S || !th || !started) {
    free(J);
    free(S);
    free(th);
    free(started);
    return RMQ_ENOMEM;
  }
  memset(e->touched, 0, P);
  for (uint32_t t = 0; t < T; ++t) {
    J[t].e = e;
    J[t].b = batches;
    J[t].out = out_offsets;
    J[t].st = S + (size_t)t * nb;
    J[t].nb = nb;
    J[t].t = t;
    J[t].T = T;
    J[t].cpu = ncpu ? cpus[t % (uint32_t)ncpu] : -1;
  }
  for (uint32_t t = 0; t < T; ++t) started[t] = pthread_create(&th[t], NULL, shard_main, &J[t]) == 0;
  for (uint32_t t = 0; t < T; ++t) {
    if (started[t]) {
      pthread_join(th[t], NULL);
    } else {
      J[t].cpu = -1; /* runs on the calling thread: leave its affinity alone */
      shard_main(&J[t]);
    }
  }
  int rc = RMQ_OK;
  uint32_t done = nb;
  for (uint32_t t = 0; t < T; ++t) {
    if (J[t].rc && rc == RMQ_OK) rc = J[t].rc;
    if (J[t].done < done) done = J[t].done;
  }
  for (uint32_t k = 0; k < nb; ++k) {
    rmq_append_stats a;
    memset(&a, 0, sizeof a);
    for (uint32_t t = 0; t < T; ++t) {
      const rmq_append_stats* x = &S[(size_t)t * nb + k];
      a.records += x->records;
      a.appended += x->appended;
      a.rejected_not_leader += x->rejected_not_leader;
      a.rejected_no_partition += x->rejected_no_partition;
      a.rejected_no_space += x->rejected_no_space;
      a.rejected_invalid += x->rejected_invalid;
    }
    stats[k] = a;
  }
  if (batches_done) *batches_done = done;
  free(J);
  free(S);
  free(th);
  free(started);
  return rc;
}

int ro_reserve(ro_engine* e, const uint64_t* bytes) {
  if (!e || !bytes) return RMQ_EINVAL;
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  for (uint32_t p = 0; p < P; ++p) {
    const uint64_t S = e->parts[p].seg;
    const uint64_t n = bytes[p] < S ? bytes[p] : S;
    for (uint32_t r = 0; r < RF; ++r) {
      if (e->parts[p].ranks[r] != e->cfg.rank) continue;
      volatile uint8_t* ring = ring_of(e, r, p);
      for (uint64_t o = 0; o < n; o += 4096) ring[o] = ring[o]; /* first touch, content unchanged */
    }
  }
  return RMQ_OK;
}

/* rmq_set_segments: ring sizes of n partitions. A smaller ring first applies retention at its size
   (FORMAT.md §4 rule); the retained records keep their offsets and logical positions in every
   replica ring; the rest of a new ring is zero. No pool limit here (the engine's RMQ_ENOMEM is
   engine-only). */
int ro_set_segments(ro_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* seg) {
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  const uint64_t I = e->cfg.index_interval;
  for (uint32_t i = 0; i < n; ++i) {
    if (pidx[i] >= P) return RMQ_ENOPART;
    if (!seg[i] || (seg[i] & (seg[i] - 1)) || seg[i] < 4 * I) return RMQ_EINVAL;
    for (uint32_t k = 0; k < i; ++k)
      if (pidx[k] == pidx[i]) return RMQ_EINVAL;
  }
  for (uint32_t i = 0; i < n; ++i) {
    ro_part* s = &e->parts[pidx[i]];
    const uint64_t S0 = s->seg, S1 = seg[i];
    if (S1 == S0) continue;
    if (s->used - s->start_pos > S1) {
      const uint64_t m = (s->used - S1 + I - 1) / I;
      s->start_off = s->idx_off.v[m];
      s->start_pos = s->idx_pos.v[m];
    }
    const uint64_t keep = s->used - s->start_pos;
    uint8_t* tmp = (uint8_t*)malloc(keep ? keep : 1);
    if (!tmp) return RMQ_ENOMEM;
    for (uint32_t r = 0; r < RF; ++r) {
      uint8_t** slot = &e->rings[(size_t)r * P + pidx[i]];
      uint8_t* nr = (uint8_t*)calloc(S1, 1);
      if (!nr) {
        free(tmp);
        return RMQ_ENOMEM;
      }
      ring_read(S0, *slot, s->start_pos, tmp, keep);
      ring_write(S1, nr, s->start_pos, tmp, keep);
      free(*slot);
      *slot = nr;
    }
    free(tmp);
    s->seg = S1;
  }
  return RMQ_OK;
}

int ro_ack(ro_engine* e, const uint32_t* pidx, const uint32_t* slot, const uint64_t* match, uint32_t n) {
  uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  for (uint32_t i = 0; i < n; ++i) {
    if (pidx[i] >= P) return RMQ_ENOPART;
    if (slot[i] >= RF) return RMQ_EINVAL;
  }
  for (uint32_t i = 0; i < n; ++i) {
    ro_part* s = &e->parts[pidx[i]];
    uint64_t m = match[i] < s->leo ? match[i] : s->leo; /* matchIndex <= leader's last index */
    if (m > s->match[slot[i]]) s->match[slot[i]] = m;
  }
  for (uint32_t i = 0; i < n; ++i) commit_eval(e, &e->parts[pidx[i]]);
  return RMQ_OK;
}

/* PartitionStateMachine.handleConsumerOffsetUpdateRequest: put, last writer wins, unchecked. */
int ro_commit_consumer_offset(ro_engine* e, const uint32_t* pidx, const uint32_t* consumer,
                              const uint64_t* offset, uint32_t n, int32_t* status) {
  int rc = RMQ_OK;
  memset(e->touched, 0, e->cfg.num_partitions); /* the row version moves once per call */
  for (uint32_t i = 0; i < n; ++i) {
    int st = RMQ_OK;
    if (pidx[i] >= e->cfg.num_partitions)
      st = RMQ_ENOPART;
    else if (!e->parts[pidx[i]].is_leader)
      st = RMQ_ENOTLEADER;
    else if (consumer[i] >= e->cfg.max_consumers)
      st = RMQ_EINVAL;
    else {
      e->parts[pidx[i]].cons[consumer[i]] = offset[i];
      e->parts[pidx[i]].dirty = 1; /* the row travels with the next replication round (§9) */
      if (!e->touched[pidx[i]]) {
        e->touched[pidx[i]] = 1;
        e->parts[pidx[i]].cver++;
      }
    }
    if (status) status[i] = st;
    if (st && !rc) rc = st;
  }
  return rc;
}

/* PartitionStateMachine.handleBatchRead: off = consumerOffsets.getOrDefault(id, 0);
   returns messages[off, min(off + max, size)) with size = applied (committed) records. */
/* The lowest replica slot this engine stores (the engine reads a replica read from it; the bytes of
   every local slot are equal), else the leader's. */
static uint32_t local_slot(const ro_engine* e, const ro_part* s) {
  for (uint32_t r = 0; r < e->cfg.replication_factor; ++r)
    if (s->ranks[r] == e->cfg.rank) return r;
  return s->leader_slot;
}

int ro_set_replica_cursor(ro_engine* e, uint32_t n, const uint32_t* pidx, const uint64_t* offset) {
  for (uint32_t i = 0; i < n; ++i)
    if (pidx[i] >= e->cfg.num_partitions) return RMQ_ENOPART;
  for (uint32_t i = 0; i < n; ++i) e->parts[pidx[i]].rcur = offset[i];
  return RMQ_OK;
}

int ro_fetch(ro_engine* e, const rmq_fetch_req* reqs, uint32_t n, uint8_t* out, uint64_t out_cap,
             rmq_fetch_res* res, uint64_t* bytes_used) {
  uint64_t cursor = 0;
  int rc = RMQ_OK;
  /* RMQ_FETCH_COMMIT: at most one committing request per (partition, consumer); with
     RMQ_FETCH_REPLICA (the partition's replica cursor) one per partition */
  for (uint32_t r = 0; r < n; ++r) {
    if (reqs[r].flags & ~(RMQ_FETCH_COMMIT | RMQ_FETCH_REPLICA)) return RMQ_EINVAL;
    if (!(reqs[r].flags & RMQ_FETCH_COMMIT) || reqs[r].pidx >= e->cfg.num_partitions ||
        reqs[r].consumer >= e->cfg.max_consumers)
      continue;
    const uint32_t rep = reqs[r].flags & RMQ_FETCH_REPLICA;
    for (uint32_t q = 0; q < r; ++q)
      if ((reqs[q].flags & RMQ_FETCH_COMMIT) && (reqs[q].flags & RMQ_FETCH_REPLICA) == rep &&
          reqs[q].pidx == reqs[r].pidx && (rep || reqs[q].consumer == reqs[r].consumer))
        return RMQ_EINVAL;
  }
  for (uint32_t r = 0; r < n; ++r) {
    rmq_fetch_res* x = &res[r];
    memset(x, 0, sizeof *x);
    x->out_pos = cursor;
    uint32_t p = reqs[r].pidx;
    if (p >= e->cfg.num_partitions) {
      x->status = RMQ_ENOPART;
      continue;
    }
    ro_part* s = &e->parts[p];
    const int rep = (reqs[r].flags & RMQ_FETCH_REPLICA) != 0; /* this engine's own replica */
    if (!s->is_leader && !rep) {
      x->status = RMQ_ENOTLEADER;
      continue;
    }
    if (reqs[r].consumer >= e->cfg.max_consumers) {
      x->status = RMQ_EINVAL;
      continue;
    }
    uint64_t off = rep ? s->rcur : s->cons[reqs[r].consumer];
    x->start_offset = off;
    uint64_t lim = off + reqs[r].max_records;
    if (lim < off) lim = UINT64_MAX;
    uint64_t end = lim < s->hw ? lim : s->hw;
    if (off >= end) continue; /* empty list */
    if (off < s->start_off) {
      x->status = RMQ_EOFFSET;
      x->start_offset = s->start_off; /* where the consumer can resume (FORMAT.md §7) */
      continue;
    }
    uint64_t p0 = s->rec_pos.v[off];
    uint64_t p1 = end < s->leo ? s->rec_pos.v[end] : s->used;
    uint64_t nb = p1 - p0;
    if (cursor + nb > out_cap) {
      x->status = RMQ_ENOSPC;
      cursor += nb;
      rc = RMQ_ENOSPC;
      continue;
    }
    if (out) ring_read(s->seg, ring_of(e, rep ? local_slot(e, s) : s->leader_slot, p), p0, out + cursor, nb);
    x->count = (uint32_t)(end - off);
    x->bytes = (uint32_t)nb;
    cursor += nb;
  }
  /* the committing requests' next offsets, after every request read its own (read-then-commit) */
  for (uint32_t r = 0; r < n; ++r) {
    const rmq_fetch_res* x = &res[r];
    if (!(reqs[r].flags & RMQ_FETCH_COMMIT) || (x->status != RMQ_OK && x->status != RMQ_EOFFSET)) continue;
    ro_part* s = &e->parts[reqs[r].pidx];
    const uint64_t nx = x->start_offset + (x->status == RMQ_OK ? x->count : 0);
    if (reqs[r].flags & RMQ_FETCH_REPLICA) {
      s->rcur = nx; /* local: no round carries it */
    } else {
      s->cons[reqs[r].consumer] = nx;
      s->dirty = 1;
    }
  }
  if (bytes_used) *bytes_used = cursor;
  return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* Read-back                                                                                   */
/* ------------------------------------------------------------------------------------------ */

int ro_get_partition_state(ro_engine* e, uint32_t p, rmq_partition_state* o) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  ro_part* s = &e->parts[p];
  memset(o, 0, sizeof *o);
  o->log_end_offset = s->leo;
  o->log_end_pos = s->used;
  o->log_start_offset = s->start_off;
  o->log_start_pos = s->start_pos;
  o->commit = s->commit;
  o->high_watermark = s->hw;
  o->term = s->term;
  o->term_start = s->term_start;
  for (uint32_t r = 0; r < RMQ_MAX_RF; ++r) {
    o->match[r] = r < e->cfg.replication_factor ? s->match[r] : 0;
    o->replica_rank[r] = r < e->cfg.replication_factor ? s->ranks[r] : 0;
  }
  o->leader_slot = s->leader_slot;
  o->is_leader = s->is_leader;
  o->segment_bytes = s->seg;
  o->leader_commit = s->is_leader ? s->commit : s->lc;
  o->last_log_term = (s->lterm & RO_LTERM_BOUND) ? 0 : s->lterm;
  o->voted_term = s->vterm;
  o->voted_for = s->vfor;
  o->led = s->led;
  o->heard_round = s->heard;
  return RMQ_OK;
}

int ro_get_partition_states(ro_engine* e, uint32_t first, uint32_t n, rmq_partition_state* out) {
  if (first > e->cfg.num_partitions || n > e->cfg.num_partitions - first) return RMQ_ENOPART;
  for (uint32_t i = 0; i < n; ++i) ro_get_partition_state(e, first + i, &out[i]);
  return RMQ_OK;
}

int ro_read_segment(ro_engine* e, uint32_t replica, uint32_t p, uint64_t ring_off, uint64_t len, uint8_t* out) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  if (replica >= e->cfg.replication_factor || ring_off > e->parts[p].seg || len > e->parts[p].seg - ring_off)
    return RMQ_EINVAL;
  memcpy(out, ring_of(e, replica, p) + ring_off, len);
  return RMQ_OK;
}

int ro_read_index(ro_engine* e, uint32_t p, uint64_t m_first, uint64_t count, uint64_t* out) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  ro_part* s = &e->parts[p];
  if (m_first > s->idx_off.n || count > s->idx_off.n - m_first) return RMQ_EINVAL;
  for (uint64_t k = 0; k < count; ++k) {
    out[2 * k] = s->idx_off.v[m_first + k];
    out[2 * k + 1] = s->idx_pos.v[m_first + k];
  }
  return RMQ_OK;
}

int ro_read_consumer_offsets(ro_engine* e, uint32_t p, uint64_t* out) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  memcpy(out, e->parts[p].cons, e->cfg.max_consumers * sizeof(uint64_t));
  return RMQ_OK;
}

int ro_record_pos(ro_engine* e, uint32_t p, uint64_t offset, uint64_t* pos) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  ro_part* s = &e->parts[p];
  if (offset > s->leo) return RMQ_EINVAL;
  *pos = offset == s->leo ? s->used : s->rec_pos.v[offset];
  return RMQ_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Replication rounds (FORMAT.md §9): the leader's region per destination, the follower's      */
/* ingest, the leader's ack application. Restated from the format, record by record.          */
/* ------------------------------------------------------------------------------------------ */


#define RO_XMAGIC 0x34514D52u /* "RMQ4" */
#define RO_HDR 64u
#define RO_DIR 48u
#define RO_ACK_REFUSED (1ull << 62)
#define RO_ACK_LEO_MASK ((1ull << 62) - 1ull)
#define RO_REBASE (1ull << 63) /* directory term flag: the entry restarts the follower's log */

typedef struct {
  uint64_t key;
  uint32_t slot, p;
} ro_entry;

static int entry_cmp(const void* a, const void* b) {
  const ro_entry *x = (const ro_entry*)a, *y = (const ro_entry*)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->slot < y->slot ? -1 : x->slot > y->slot;
}

/* Entries exchanged between leader `src` and follower `dst`, ascending (key, slot): the
   (partition, slot) pairs whose leader is src and whose replica slot lives on dst. */
static uint32_t pair_entries(const ro_engine* e, uint32_t src, uint32_t dst, ro_entry** out) {
  const uint32_t P = e->cfg.num_partitions, RF = e->cfg.replication_factor;
  ro_entry* v = (ro_entry*)malloc(((size_t)P * RF + 1) * sizeof(ro_entry));
  uint32_t n = 0;
  for (uint32_t p = 0; p < P && v; ++p) {
    const ro_part* s = &e->parts[p];
    if (s->ranks[s->leader_slot] != src) continue;
    for (uint32_t r = 0; r < RF; ++r)
      if (s->ranks[r] == dst && dst != src) v[n++] = (ro_entry){s->key, r, p};
  }
  if (v) qsort(v, n, sizeof *v, entry_cmp);
  *out = v;
  return v ? n : 0;
}

int ro_set_world(ro_engine* e, uint32_t world) {
  if (!e || world == 0 || world <= e->cfg.rank) return RMQ_EINVAL;
  e->world = world;
  return RMQ_OK;
}

int ro_set_key(ro_engine* e, uint32_t p, uint64_t key) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  e->parts[p].key = key;
  return RMQ_OK;
}

uint64_t ro_round_no(ro_engine* e) { return e->round_no; }

uint64_t ro_catchup_reserve(const rmq_config* c) {
  const uint64_t G = c->pipeline_depth ? c->pipeline_depth : 2u;
  return G * (39ull * c->max_batch_records + c->max_batch_bytes);
}

/* The leader's plan of one entry for the current round (FORMAT.md §9 catch-up). */
typedef struct {
  uint64_t first, pos0;       /* where the entry starts in the leader's log (offset, position) */
  uint64_t count, bytes;      /* records / record bytes it carries */
  uint64_t gap_count, gap_bytes; /* of which the catch-up part [first, B) read from the ring */
  uint64_t nx_off, nx_pos;    /* next after the round */
  int set_cu, row, detached, catchup;
  int rebase;                 /* the catch-up part starts at the rebase point R, not at the follower */
} ro_plan;

/* Largest sparse-index entry E[m] (m I <= lim, E[m].pos <= lim, E[m].pos > pos0, m <= mmax):
   the end of a partial catch-up. Returns 0 if none. */
static int partial_end(const ro_engine* e, const ro_part* s, uint64_t pos0, uint64_t lim, uint64_t mmax,
                       uint64_t* off, uint64_t* pos) {
  const uint64_t I = e->cfg.index_interval;
  uint64_t m = lim / I;
  if (m > mmax) m = mmax;
  for (;; --m) {
    if (m < s->idx_pos.n && s->idx_pos.v[m] <= lim && s->idx_pos.v[m] > pos0) {
      *off = s->idx_off.v[m];
      *pos = s->idx_pos.v[m];
      return 1;
    }
    if (m == 0 || (m - 1) * I < pos0) return 0;
  }
}

/* Plans every entry of the pair (me -> dst) for the current round, without changing state. */
static void plan_pair(const ro_engine* e, const ro_entry* v, uint32_t n, ro_plan* pl) {
  const uint64_t I = e->cfg.index_interval;
  uint64_t left = ro_catchup_reserve(&e->cfg);
  int stop = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const ro_part* s = &e->parts[v[k].p];
    const uint32_t sl = v[k].slot;
    ro_plan* x = &pl[k];
    memset(x, 0, sizeof *x);
    const uint64_t Boff = s->leo - s->round_count, Bpos = s->used - s->round_bytes;
    /* index entries complete when the round is planned: up to C = B less the round before */
    const uint64_t Cpos = Bpos - s->prev_round_bytes;
    uint64_t Foff = s->nx_off[sl], Fpos = s->nx_pos[sl];
    int req = 0;
    if (s->rq_r1[sl] && s->rq_r1[sl] - 1 >= s->cu[sl]) {
      Foff = s->rq_off[sl];
      Fpos = s->rq_pos[sl];
      req = 1;
    }
    if (Foff >= Boff) {
      Foff = Boff;
      Fpos = Bpos;
    }
    x->row = s->dirty || req;
    /* default: the round's records from B (refused by a follower behind B) */
    x->first = Boff;
    x->pos0 = Bpos;
    x->count = s->round_count;
    x->bytes = s->round_bytes;
    x->nx_off = s->leo;
    x->nx_pos = s->used;
    if (Foff == Boff) {
      x->set_cu = req;
      continue;
    }
    int rebase = 0;
    if (Fpos + s->seg < s->used) {
      /* the ring no longer holds [F, E) after the round: the follower's log restarts at the rebase
         point R = E[m], m = ceil((E.pos - S) / I), the oldest index entry [R, E) fits the ring from
         (Raft's InstallSnapshot, the leader's retained log as the snapshot); without a complete
         E[m] (m I > C) the follower stays detached this round */
      const uint64_t m = (s->used - s->seg + I - 1) / I;
      if (m * I > Cpos) {
        x->detached = 1;
        continue;
      }
      Foff = s->idx_off.v[m];
      Fpos = s->idx_pos.v[m];
      rebase = 1;
    }
    const uint64_t g = Bpos - Fpos;
    if (!stop && g <= left) {
      x->first = Foff;
      x->pos0 = Fpos;
      x->gap_count = Boff - Foff;
      x->gap_bytes = g;
      x->count += x->gap_count;
      x->bytes += g;
      x->set_cu = x->row = x->catchup = 1;
      x->rebase = rebase;
      left -= g;
      continue;
    }
    uint64_t Xoff = 0, Xpos = 0;
    if (!stop && partial_end(e, s, Fpos, Fpos + left, Cpos / I, &Xoff, &Xpos)) {
      x->first = Foff;
      x->pos0 = Fpos;
      x->gap_count = x->count = Xoff - Foff;
      x->gap_bytes = x->bytes = Xpos - Fpos;
      x->nx_off = Xoff;
      x->nx_pos = Xpos;
      x->set_cu = x->row = x->catchup = 1;
      x->rebase = rebase;
    }
    stop = 1;
    left = 0;
  }
}

/* The region this engine (leader) sends to rank dst for the current round; *size = its bytes
   (0 when the two ranks share no partition). out may be NULL to ask for the size. */
int ro_round_region(ro_engine* e, uint32_t dst, uint8_t* out, uint64_t cap, uint64_t* size) {
  const uint32_t me = e->cfg.rank, C = e->cfg.max_consumers;
  ro_entry* v = NULL;
  const uint32_t n = pair_entries(e, me, dst, &v);
  if (!v) return RMQ_ENOMEM;
  ro_plan* pl = (ro_plan*)calloc(n ? n : 1, sizeof(ro_plan));
  if (!pl) {
    free(v);
    return RMQ_ENOMEM;
  }
  plan_pair(e, v, n, pl);
  uint64_t N = 0, B = 0, keysum = 0, M = 0;
  for (uint32_t k = 0; k < n; ++k) {
    N += pl[k].count;
    B += pl[k].bytes;
    M += pl[k].row ? 1 : 0;
    keysum += v[k].key * RMQ_MAX_RF + v[k].slot;
  }
  const uint64_t tab = RO_HDR + (uint64_t)RO_DIR * n, data = tab + ((8 * N + 15) & ~15ull), rows = data + B;
  const uint64_t rowb = 16 + 8ull * C;
  *size = n ? rows + M * rowb : 0;
  if (!out || !n) {
    free(pl);
    free(v);
    return RMQ_OK;
  }
  if (*size > cap) {
    free(pl);
    free(v);
    return RMQ_ENOSPC;
  }
  memset(out, 0, *size);
  const uint32_t h[4] = {RO_XMAGIC, n, (uint32_t)N, me};
  memcpy(out, h, 16);
  memcpy(out + 16, &keysum, 8);
  memcpy(out + 24, &data, 8);
  memcpy(out + 32, &rows, 8);
  const uint32_t mc[2] = {(uint32_t)M, C};
  memcpy(out + 40, mc, 8);
  memcpy(out + 48, &e->round_no, 8);
  uint64_t t = 0, b16 = 0, mrow = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const ro_part* s = &e->parts[v[k].p];
    const ro_plan* x = &pl[k];
    uint8_t* d = out + RO_HDR + (uint64_t)RO_DIR * k;
    const uint32_t cnt = (uint32_t)x->count, by16 = (uint32_t)(x->bytes / 16);
    const uint32_t ts = (uint32_t)t, ds = (uint32_t)b16;
    memcpy(d, &cnt, 4);
    memcpy(d + 4, &by16, 4);
    memcpy(d + 8, &x->first, 8);
    memcpy(d + 16, &ts, 4);
    memcpy(d + 20, &ds, 4);
    const uint64_t tf = s->term | (x->rebase ? RO_REBASE : 0ull);
    memcpy(d + 24, &tf, 8);
    /* the leader's commit (v4: Raft's leaderCommit), as it stood before the round's records */
    const uint64_t boff = s->leo - s->round_count, lcm = s->commit < boff ? s->commit : boff;
    memcpy(d + 32, &lcm, 8);
    /* (v5) the term of the entry's last entry as far as the follower may count it: the leader's term
       when the entry reaches its term start (the leader-start entry), else 0 (an older, unknown term) */
    const uint64_t ltm = x->first + x->count >= s->term_start ? s->term : 0;
    memcpy(d + 40, &ltm, 8);
    uint8_t* dd = out + data + 16 * b16;
    /* the catch-up part from the leader's ring, then the round's records (if carried) */
    if (x->gap_bytes) ring_read(s->seg, ring_of(e, s->leader_slot, v[k].p), x->pos0, dd, x->gap_bytes);
    if (x->bytes > x->gap_bytes) memcpy(dd + x->gap_bytes, s->round, s->round_bytes);
    uint64_t rel = 0;
    for (uint64_t r = 0; r < x->count; ++r) { /* record table: {entry, record position / 16} */
      uint32_t len;
      memcpy(&len, dd + rel + 8, 4);
      const uint64_t slot = (uint64_t)k | ((uint64_t)(ds + rel / 16) << 32);
      memcpy(out + tab + 8 * (t + r), &slot, 8);
      rel += rec_size(len);
    }
    if (x->row) {
      uint8_t* rw = out + rows + rowb * mrow++;
      memcpy(rw, &k, 4);
      if (x->rebase) memcpy(rw + 8, &x->pos0, 8); /* the rebase point's position */
      memcpy(rw + 16, s->cons, 8ull * C);
    }
    t += cnt;
    b16 += by16;
  }
  free(pl);
  free(v);
  return RMQ_OK;
}

/* Closes the round: the leader applies its plan's per-entry state to every destination, forgets
   the records it kept for the round and marks the consumer-offset rows sent. */
void ro_end_round(ro_engine* e) {
  const uint32_t me = e->cfg.rank;
  for (uint32_t d = 0; d < e->world; ++d) {
    if (d == me) continue;
    ro_entry* v = NULL;
    const uint32_t n = pair_entries(e, me, d, &v);
    ro_plan* pl = v ? (ro_plan*)calloc(n ? n : 1, sizeof(ro_plan)) : NULL;
    if (pl) {
      plan_pair(e, v, n, pl);
      for (uint32_t k = 0; k < n; ++k) {
        ro_part* s = &e->parts[v[k].p];
        const uint32_t sl = v[k].slot;
        s->nx_off[sl] = pl[k].nx_off;
        s->nx_pos[sl] = pl[k].nx_pos;
        s->rowv[sl] = pl[k].row ? s->cver : 0; /* the row version this round carries to the slot */
        if (pl[k].set_cu) s->cu[sl] = e->round_no;
        e->counters[4] += pl[k].catchup ? 1u : 0u;
        e->counters[5] += pl[k].detached ? 1u : 0u;
      }
    }
    free(pl);
    free(v);
  }
  for (uint32_t p = 0; p < e->cfg.num_partitions; ++p) {
    e->parts[p].prev_round_bytes = e->parts[p].round_bytes;
    e->parts[p].round_bytes = e->parts[p].round_count = 0;
    e->parts[p].dirty = 0;
  }
  e->round_no++;
}

/* Follower: truncate partition p's log to offset t (start_off <= t < leo): the records from t on
   are dropped (their ring bytes stay, outside the log), index entries past the new end too. */
static void truncate_log(ro_engine* e, ro_part* s, uint64_t t) {
  const uint64_t I = e->cfg.index_interval;
  s->used = s->rec_pos.v[t];
  s->leo = t;
  s->rec_pos.n = t;
  s->idx_off.n = s->idx_pos.n = s->used / I + 1;
}

/* Follower: partition p's log restarts at offset t, position pos (a rebase entry, FORMAT.md §9):
   the old records leave the log (their ring bytes and index slots stay, outside it); the dense
   lookups get placeholders below the new start, which no lookup reads. */
static int rebase_log(ro_engine* e, ro_part* s, uint64_t t, uint64_t pos) {
  const uint64_t I = e->cfg.index_interval;
  s->rec_pos.n = t < s->rec_pos.n ? t : s->rec_pos.n;
  while (s->rec_pos.n < t)
    if (vec_push(&s->rec_pos, 0)) return RMQ_ENOMEM;
  const uint64_t ni = pos / I + 1;
  s->idx_off.n = ni < s->idx_off.n ? ni : s->idx_off.n;
  s->idx_pos.n = s->idx_off.n;
  while (s->idx_off.n < ni)
    if (vec_push(&s->idx_off, 0) || vec_push(&s->idx_pos, 0)) return RMQ_ENOMEM;
  if (pos % I == 0) { /* E[m] of a start on an interval multiple is its first record (as the leader's) */
    s->idx_off.v[ni - 1] = t;
    s->idx_pos.v[ni - 1] = pos;
  }
  s->leo = s->start_off = t;
  s->used = s->start_pos = pos;
  return RMQ_OK;
}

/* The consumer-offset row of entry k in a region (rows ascend by entry), or NULL. */
static const uint8_t* row_of(const uint8_t* region, uint64_t rows, uint32_t M, uint32_t C, uint32_t k) {
  const uint64_t rowb = 16 + 8ull * C;
  for (uint32_t r = 0; r < M; ++r) {
    uint32_t rk;
    memcpy(&rk, region + rows + rowb * r, 4);
    if (rk == k) return region + rows + rowb * r;
    if (rk > k) break;
  }
  return NULL;
}

/* A follower learns its leader's commit (FORMAT.md §9 v4): leader_commit = the newest, its own
   commit = the part of its log below it (never past its log end). */
static void learn_commit(ro_part* s, uint64_t c) {
  if (c > s->lc) s->lc = c;
  const uint64_t k = s->lc < s->leo ? s->lc : s->leo;
  if (k > s->commit) s->commit = k;
  if (s->commit > s->leo) s->commit = s->leo;
  s->hw = s->commit;
}

static void ack_of(const ro_part* s, int refused, uint64_t* ack) {
  ack[0] = s->leo | (refused ? RO_ACK_REFUSED : 0ull);
  ack[1] = s->used;
}

/* Follower: ingest the region leader `src` sent (FORMAT.md §9); acks[2k..2k+1] = this engine's
   log end after the round for entry k with its status. size 0: the round from src is missed (every
   entry refused). */
int ro_ingest(ro_engine* e, uint32_t src, const uint8_t* region, uint64_t size, uint64_t* acks) {
  const uint32_t me = e->cfg.rank, C = e->cfg.max_consumers;
  const uint64_t I = e->cfg.index_interval;
  ro_entry* v = NULL;
  const uint32_t n = pair_entries(e, src, me, &v);
  if (!v) return RMQ_ENOMEM;
  if (!n || !size) {
    for (uint32_t k = 0; k < n; ++k) {
      ack_of(&e->parts[v[k].p], 1, acks + 2 * k);
      e->counters[2]++;
    }
    free(v);
    return n && size ? RMQ_EINVAL : RMQ_OK;
  }
  uint32_t h[4] = {0, 0, 0, 0}, mc[2] = {0, 0};
  uint64_t keysum = 0, data = 0, rows = 0, want = 0;
  if (size >= RO_HDR) {
    memcpy(h, region, 16);
    memcpy(&keysum, region + 16, 8);
    memcpy(&data, region + 24, 8);
    memcpy(&rows, region + 32, 8);
    memcpy(mc, region + 40, 8);
  }
  for (uint32_t k = 0; k < n; ++k) want += v[k].key * RMQ_MAX_RF + v[k].slot;
  const uint64_t tab = RO_HDR + (uint64_t)RO_DIR * n, rowb = 16 + 8ull * C;
  /* the header (FORMAT.md §9): a region that does not describe this pair's entry list, or whose
     sections do not fit it, is unreadable: every entry refused (counted as log, like a missed round) */
  if (size < RO_HDR || h[0] != RO_XMAGIC || h[1] != n || h[3] != src || keysum != want || mc[1] != C ||
      data != tab + ((8ull * h[2] + 15) & ~15ull) || rows < data || rows > size || (rows - data) % 16 ||
      mc[0] > n || (size - rows) / rowb < mc[0]) {
    for (uint32_t k = 0; k < n; ++k) {
      ack_of(&e->parts[v[k].p], 1, acks + 2 * k);
      e->counters[2]++;
    }
    free(v);
    return RMQ_OK;
  }
  /* structure (FORMAT.md §9): the directory entries tile the record table and the data section in
     list order, every table slot names the entry whose range holds it, and the consumer-offset rows
     name ascending entries. A region that breaks any of these was corrupted on the way: every entry
     is refused (the leader's catch-up sends it again) */
  int insane = 0;
  {
    uint64_t t = 0, d16 = 0;
    for (uint32_t k = 0; k < n && !insane; ++k) {
      const uint8_t* d = region + RO_HDR + (uint64_t)RO_DIR * k;
      uint32_t cnt, by16, ts, ds;
      memcpy(&cnt, d, 4);
      memcpy(&by16, d + 4, 4);
      memcpy(&ts, d + 16, 4);
      memcpy(&ds, d + 20, 4);
      insane = ts != t || ds != d16;
      t += cnt;
      d16 += by16;
    }
    if (t != h[2] || 16 * d16 != rows - data) insane = 1;
    t = 0;
    for (uint32_t k = 0; k < n && !insane; ++k) {
      uint32_t cnt;
      memcpy(&cnt, region + RO_HDR + (uint64_t)RO_DIR * k, 4);
      for (uint32_t r = 0; r < cnt && !insane; ++r) {
        uint32_t sk;
        memcpy(&sk, region + tab + 8 * (t + r), 4);
        insane = sk != k;
      }
      t += cnt;
    }
    for (uint32_t r = 0; r < mc[0] && !insane; ++r) {
      uint32_t rk, pk = 0;
      memcpy(&rk, region + rows + rowb * r, 4);
      if (r) memcpy(&pk, region + rows + rowb * (r - 1), 4);
      insane = rk >= n || (r && pk >= rk);
    }
  }
  /* pass 1: the verdict of every entry against the state every entry of a partition sees (the log
     end it continues, decided once by the owner: two local slots, the first keeps the state) */
  int* okv = (int*)malloc((size_t)n * sizeof(int));
  uint64_t* base = (uint64_t*)malloc((size_t)n * 2 * sizeof(uint64_t));
  if (!okv || !base) {
    free(okv);
    free(base);
    free(v);
    return RMQ_ENOMEM;
  }
  uint64_t leo = 0, used = 0;
  int stale = 0;
  for (uint32_t k = 0; k < n; ++k) {
    ro_part* s = &e->parts[v[k].p];
    const int owner = k == 0 || v[k - 1].p != v[k].p;
    const uint8_t* d = region + RO_HDR + (uint64_t)RO_DIR * k;
    uint32_t cnt, by16, ts, ds;
    uint64_t first, term;
    memcpy(&cnt, d, 4);
    memcpy(&by16, d + 4, 4);
    memcpy(&first, d + 8, 8);
    memcpy(&ts, d + 16, 4);
    memcpy(&ds, d + 20, 4);
    memcpy(&term, d + 24, 8);
    const int rebase = (term & RO_REBASE) != 0;
    term &= ~RO_REBASE;
    if (owner) {
      stale = term < s->term; /* a leader of an older term */
      if (!stale) s->heard = e->round_no; /* its current leader is alive (the election timer restarts) */
      leo = s->leo;
      used = s->used;
      if (!stale && rebase) { /* the log restarts at the entry's first record (its row holds the position) */
        const uint8_t* row = row_of(region, rows, mc[0], C, k);
        leo = first;
        used = 0;
        if (row) memcpy(&used, row + 8, 8);
        else stale = 1; /* malformed: a rebase entry always carries its row */
      } else if (!stale && first < leo && first >= s->start_off) { /* the leader's log wins: truncate */
        used = s->rec_pos.v[first];
        leo = first;
      }
    }
    base[2 * k] = leo;
    base[2 * k + 1] = used;
    int ok = !stale && first == leo && !insane;
    uint64_t rel = 0;
    for (uint32_t r = 0; r < cnt && ok; ++r) {
      uint64_t slot, off;
      uint32_t len, crc;
      memcpy(&slot, region + tab + 8ull * (ts + r), 8);
      const uint8_t* rec = region + data + 16ull * (ds + rel / 16);
      ok = (slot >> 32) == ds + rel / 16 && rel + 16 <= 16ull * by16;
      if (!ok) break;
      memcpy(&off, rec, 8);
      memcpy(&len, rec + 8, 4);
      memcpy(&crc, rec + 12, 4);
      ok = off == first + r && rel + rec_size(len) <= 16ull * by16 && ro_crc32c(rec + 16, len) == crc;
      for (uint64_t z = 16 + len; ok && z < rec_size(len); ++z) ok = rec[z] == 0; /* zero padding (§1) */
      rel += rec_size(len);
    }
    if (ok && rel != 16ull * by16) ok = 0; /* the records fill the entry's bytes exactly */
    okv[k] = ok;
    if (!ok) e->counters[!stale && first == leo ? 1 : 2]++;
  }
  /* a refusal of either slot of a partition is a refusal of both */
  for (uint32_t k = 0; k < n; ++k)
    for (uint32_t q = k + 1; q < n && v[q].p == v[k].p; ++q)
      if (!okv[k] || !okv[q]) okv[k] = okv[q] = 0;
  /* pass 2: apply the accepted entries */
  uint64_t mrow = 0;
  for (uint32_t k = 0; k < n; ++k) {
    ro_part* s = &e->parts[v[k].p];
    const int owner = k == 0 || v[k - 1].p != v[k].p;
    const uint8_t* d = region + RO_HDR + (uint64_t)RO_DIR * k;
    uint32_t cnt, by16, ds;
    uint64_t first, term, lcm;
    memcpy(&cnt, d, 4);
    memcpy(&by16, d + 4, 4);
    memcpy(&first, d + 8, 8);
    memcpy(&ds, d + 20, 4);
    memcpy(&term, d + 24, 8);
    memcpy(&lcm, d + 32, 8);
    leo = base[2 * k];
    used = base[2 * k + 1];
    const int rebase = (term & RO_REBASE) != 0;
    term &= ~RO_REBASE;
    /* this entry's consumer-offset row, if any (rows ascend by entry) */
    const uint8_t* row = NULL;
    while (mrow < mc[0]) {
      uint32_t rk;
      memcpy(&rk, region + rows + rowb * mrow, 4);
      if (rk > k) break;
      if (rk == k) row = region + rows + rowb * mrow + 16;
      ++mrow;
    }
    if (!okv[k]) {
      ack_of(s, 1, acks + 2 * k);
      continue;
    }
    if (owner) {
      if (term > s->term) s->term = term;
      uint64_t ltm;
      memcpy(&ltm, d + 40, 8);
      /* the entry's last entry term; 0: older than the leader's term start, so the log ends in a
         term below the leader's: kept as that upper bound (the vote compares against it), reported
         as 0 (a candidate claims no more than it knows) */
      s->lterm = ltm ? ltm : RO_LTERM_BOUND | (term ? term - 1 : 0);
      s->mterm = term;  /* the log now matches the term-`term` leader's through the entry's end */
      if (rebase) {
        if (rebase_log(e, s, leo, used)) {
          free(okv);
          free(base);
          free(v);
          return RMQ_ENOMEM;
        }
      } else if (leo < s->leo) {
        truncate_log(e, s, leo);
      }
      if (row) memcpy(s->cons, row, 8ull * C);
    }
    if (cnt) {
      const uint8_t* bytes = region + data + 16ull * ds;
      ring_write(s->seg, ring_of(e, v[k].slot, v[k].p), used, bytes, 16ull * by16);
      if (owner) {
        uint64_t rel = 0;
        for (uint32_t r = 0; r < cnt; ++r) {
          uint32_t len;
          memcpy(&len, bytes + rel + 8, 4);
          const uint64_t pos = used + rel, rs = rec_size(len);
          for (uint64_t m = pos / I + 1; m * I <= pos + rs; ++m)
            if (vec_push(&s->idx_off, first + r + 1) || vec_push(&s->idx_pos, pos + rs)) {
              free(okv);
              free(base);
              free(v);
              return RMQ_ENOMEM;
            }
          if (vec_push(&s->rec_pos, pos)) {
            free(okv);
            free(base);
            free(v);
            return RMQ_ENOMEM;
          }
          rel += rs;
        }
        s->leo = first + cnt;
        s->used = used + 16ull * by16;
        if (s->used - s->start_pos > s->seg) { /* retention once per round (FORMAT.md §4 rule) */
          const uint64_t m = (s->used - s->seg + I - 1) / I;
          s->start_off = s->idx_off.v[m];
          s->start_pos = s->idx_pos.v[m];
        }
        e->counters[3] += 16ull * by16;
      }
      e->counters[0] += cnt; /* records written into this replica slot */
    }
    if (owner) learn_commit(s, lcm); /* the leader's commit the entry carries (Raft leaderCommit) */
    /* the owner's state after the round: both slots ack it */
    acks[2 * k] = first + cnt;
    acks[2 * k + 1] = used + 16ull * by16;
  }
  free(okv);
  free(base);
  free(v);
  return RMQ_OK;
}

/* Leader: the acks follower `dst` returned for round `round` (FORMAT.md §9): an accepted entry
   moves match = max(match, min(ack, log end)), a refused one leaves a catch-up request; then the
   quorum commit rule of every partition they name. */
int ro_apply_acks(ro_engine* e, uint32_t dst, const uint64_t* acks, uint32_t n_acks, uint64_t round) {
  ro_entry* v = NULL;
  const uint32_t n = pair_entries(e, e->cfg.rank, dst, &v);
  if (!v) return RMQ_ENOMEM;
  if (n != n_acks) {
    free(v);
    return RMQ_EINVAL;
  }
  for (uint32_t k = 0; k < n; ++k) {
    ro_part* s = &e->parts[v[k].p];
    const uint32_t sl = v[k].slot;
    const uint64_t a = acks[2 * k] & RO_ACK_LEO_MASK;
    if (acks[2 * k] & RO_ACK_REFUSED) {
      s->rq_off[sl] = a;
      s->rq_pos[sl] = acks[2 * k + 1];
      s->rq_r1[sl] = round + 1;
      continue;
    }
    const uint64_t m = a < s->leo ? a : s->leo;
    if (m > s->match[sl]) s->match[sl] = m;
    if (s->rowv[sl] > s->eackv[sl]) s->eackv[sl] = s->rowv[sl];
  }
  for (uint32_t k = 0; k < n; ++k) commit_eval(e, &e->parts[v[k].p]);
  free(v);
  return RMQ_OK;
}

/* Commit notices (FORMAT.md §9 v4, a drain's heartbeat): the leader's {commit, term} for every
   entry of the pair (me -> dst), and the follower learning them (an older term is ignored, a newer
   one adopted). */
int ro_commit_notice(ro_engine* e, uint32_t dst, uint64_t* out) {
  ro_entry* v = NULL;
  const uint32_t n = pair_entries(e, e->cfg.rank, dst, &v);
  if (!v) return RMQ_ENOMEM;
  for (uint32_t k = 0; k < n; ++k) {
    out[2 * k] = e->parts[v[k].p].commit;
    out[2 * k + 1] = e->parts[v[k].p].term;
  }
  free(v);
  return RMQ_OK;
}

int ro_apply_notice(ro_engine* e, uint32_t src, const uint64_t* in, uint32_t n_in) {
  ro_entry* v = NULL;
  const uint32_t n = pair_entries(e, src, e->cfg.rank, &v);
  if (!v) return RMQ_ENOMEM;
  if (n != n_in) {
    free(v);
    return RMQ_EINVAL;
  }
  for (uint32_t k = 0; k < n; ++k) {
    ro_part* s = &e->parts[v[k].p];
    if (in[2 * k + 1] < s->term) continue; /* an older term's (or a lost notice, term 0) */
    s->term = in[2 * k + 1];
    s->heard = e->round_no;
    /* the commit moves over this log only if it was matched in the notice's term; the leader's commit
       is learned either way (rmq_become_leader's RMQ_ESTALE) */
    if (s->mterm == s->term) learn_commit(s, in[2 * k]);
    else if (in[2 * k] > s->lc) s->lc = in[2 * k];
  }
  free(v);
  return RMQ_OK;
}

/* The row version of partition p and the newest one a quorum of its replicas holds (co-located
   slots: the leader's own; a remote slot: what its follower acknowledged). */
int ro_offset_quorum(ro_engine* e, uint32_t p, uint64_t* cver, uint64_t* cq) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  const ro_part* s = &e->parts[p];
  const uint32_t RF = e->cfg.replication_factor, k = RF / 2 + 1;
  uint64_t m[RMQ_MAX_RF];
  for (uint32_t r = 0; r < RF; ++r) m[r] = s->ranks[r] == e->cfg.rank ? s->cver : s->eackv[r];
  for (uint32_t i = 1; i < RF; ++i)
    for (uint32_t j = i; j > 0 && m[j - 1] < m[j]; --j) {
      uint64_t t = m[j];
      m[j] = m[j - 1];
      m[j - 1] = t;
    }
  *cver = s->cver;
  *cq = m[k - 1];
  return RMQ_OK;
}

uint32_t ro_pair_entries(ro_engine* e, uint32_t src, uint32_t dst) {
  ro_entry* v = NULL;
  const uint32_t n = pair_entries(e, src, dst, &v);
  free(v);
  return n;
}

/* Raft RequestVote (rmq_vote): an older term is denied; a newer one adopted (a leader steps down and
   keeps its commit as the leader's); the vote goes to a candidate whose (lastLogTerm, log end) is at
   least this replica's, once per term. */
int ro_vote(ro_engine* e, uint32_t p, uint64_t term, uint32_t cand, uint64_t cand_lterm, uint64_t cand_leo,
            uint32_t* granted) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  ro_part* s = &e->parts[p];
  *granted = 0;
  if (term < s->term) return RMQ_OK;
  if (term > s->term) {
    s->term = term;
    if (s->is_leader) {
      s->is_leader = 0;
      if (s->commit > s->lc) s->lc = s->commit;
    }
  }
  const uint64_t lt = s->lterm & ~RO_LTERM_BOUND; /* unknown: its upper bound (a stricter vote) */
  const int up = cand_lterm > lt || (cand_lterm == lt && cand_leo >= s->leo);
  const int free_vote = s->vterm != term || (!s->led && s->vfor == cand);
  if (up && free_vote) {
    s->vterm = term;
    s->vfor = cand;
    s->led = 0;
    *granted = 1;
  }
  return RMQ_OK;
}

int ro_set_vote(ro_engine* e, uint32_t p, uint64_t term, uint32_t voted_for) {
  if (p >= e->cfg.num_partitions) return RMQ_ENOPART;
  ro_part* s = &e->parts[p];
  if (term > s->term) s->term = term;
  s->vterm = term;
  s->vfor = voted_for;
  s->led = 0;
  return RMQ_OK;
}

/* Followed partitions whose leader was not heard in the last `silent_rounds` rounds (rmq_leader_silent
   without the wall-clock part). */
int ro_leader_silent(ro_engine* e, uint32_t silent_rounds, uint32_t* out, uint32_t cap, uint32_t* n) {
  uint32_t k = 0;
  for (uint32_t p = 0; p < e->cfg.num_partitions; ++p) {
    const ro_part* s = &e->parts[p];
    if (s->is_leader || s->heard + silent_rounds > e->round_no) continue;
    if (k < cap && out) out[k] = p;
    ++k;
  }
  *n = k;
  return RMQ_OK;
}

void ro_counters(ro_engine* e, uint64_t* out) { memcpy(out, e->counters, sizeof e->counters); }
