// Connection lookup for gfx950: the ConnTracker::process table step (conntrack/mod.rs:80-169) for a
// whole batch of forwarded frames at once, on a table that stays resident in HBM across batches.
//
// Table: `cap` (a power of two) 64-byte slots, linear probing from the rtn_conn_t hash.
//   [0]  u64 tag      64-bit fingerprint of the canonical ConnId; 0 = empty, 1 = removed
//   [8]  u32 epoch    batch that inserted the slot
//   [12] u32 first    lowest frame index of this batch's opening frames (atomicMin; 0xffffffff when
//                     the slot was created, so it is only meaningful when epoch == this batch)
//   [16] u32 key[10]  max ip (4 words; IPv4 in word 0), min ip, max port << 16 | min port,
//                     proto | 0x100 for IPv6: ConnId (conntrack/conn_id.rs:115-117)
//
// Occupancy bitmap: one bit per slot, set when a slot is claimed and cleared only by a rebuild
// (2 MiB for 2^24 slots: it stays in each XCD's 4-MiB L2). A probe whose start slot has a clear
// bit is a miss without touching the table, which is what most frames of a busy link are.
//
// Two launches per batch, so every frame sees the same table state:
//   rtn_ct_insert  frames that open a connection on a miss (rtn_conn_t creates bit; a TCP opener
//                  whose first-packet filter drops is not inserted: remove_from_table after
//                  filter_first_packet, conntrack/mod.rs:139-141) find or claim their key's slot
//                  (CAS on the tag), then lower the slot's `first` to their frame index.
//   rtn_ct_lookup  every forwarded frame finds its key (tags, then the whole key, so a 64-bit
//                  fingerprint collision is reported instead of aliasing) and gets its status.
// A wave walks one 256-frame chunk record by record (lane = record, see below), records ranked by
// the fwd bitmap exactly as rtn_pc_run wrote them.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

typedef unsigned int rtn_u32;
typedef unsigned long long rtn_u64;

#define RTN_CT_CHUNK 256u   // RTN_CHUNK_FRAMES
#define RTN_CT_GROUPS (RTN_CT_CHUNK / 64u)
#define RTN_CT_MAXPROBE 256u
#define RTN_CT_NO_SLOT_K 0xffffffffu  // RTN_CT_NO_SLOT
#define RTN_CT_EMPTY 0ull
#define RTN_CT_REMOVED 1ull

// per-record status (rtn_ct_entry_t.status, include/retina_ct.h)
#define RTN_CT_HIT 1u         // the connection exists when this frame arrives
#define RTN_CT_NEW 2u         // this frame opens it (first opener of the batch, frame order)
#define RTN_CT_MISS 3u        // no connection and this frame cannot open one: dropped
#define RTN_CT_NEW_DROPPED 4u // would open, but its first-packet filter drops it (TCP): no entry
#define RTN_CT_FULL 5u        // would open, but the table has no room
#define RTN_CT_COLLISION 6u   // 64-bit fingerprint collision: the host resolves this frame
#define RTN_CT_PRIOR 0x100u   // flag: the connection existed before this batch

struct rtn_ct_args {
  const rtn_u64* fwd_bm;
  const rtn_u32* recs;        // rtn_l4ctx_t, 4 words each (w0, w1, ports, meta)
  const rtn_u32* addr6;       // 6 words per IPv6 record (source bytes 8..15, destination)
  const rtn_u64* conn;        // rtn_conn_t
  rtn_u64* out;               // rtn_ct_entry_t (slot | status << 32), indexed like recs
  rtn_u32* table;             // cap * 16 words
  rtn_u32* occ;               // cap bits: slot not empty (live or removed); small enough for L2
  rtn_u32* live;              // [64] live-slot counters (their sum); [0] alone in checked mode
  rtn_u32 n;                  // frames in the batch
  rtn_u32 cap_mask;
  rtn_u32 max_live;
  rtn_u32 epoch;
  rtn_u32 check;              // 1: admit against max_live (host folded the counters into [0])
};

struct rtn_ct_key {
  rtn_u32 w[10];
  rtn_u64 fp;
  rtn_u32 h;
  bool v6, tcp;
  rtn_u32 info;
};

__device__ __forceinline__ rtn_u32 rtn_ct_rotl(rtn_u32 x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ rtn_u32 rtn_ct_mix(rtn_u32 h, rtn_u32 k) {
  k *= 0xcc9e2d51u;
  k = rtn_ct_rotl(k, 15);
  k *= 0x1b873593u;
  h ^= k;
  h = rtn_ct_rotl(h, 13);
  return h * 5u + 0xe6546b64u;
}
__device__ __forceinline__ rtn_u32 rtn_ct_fmix(rtn_u32 h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  return h ^ (h >> 16);
}

// Canonical key of a record (its 4 words, its rtn_conn_t, its IPv6 addresses or null) + its
// 64-bit fingerprint. An IPv4 record's words 0 and 1 are its addresses.
__device__ __forceinline__ void rtn_ct_make_key(const rtn_ct_args& a, const rtn_u32 (&rec)[4], rtn_u64 c,
                                                const rtn_u32* a6, rtn_ct_key& k) {
  const rtn_u32 meta = rec[3];
  k.h = (rtn_u32)c;
  k.info = (rtn_u32)(c >> 32);
  k.v6 = (meta >> 7) & 1u;
  k.tcp = !((meta >> 6) & 1u);
  const bool gt = (k.info >> 27) & 1u;  // src is the max endpoint
  rtn_u32 s[4], d[4];
  if (k.v6) {  // source bytes 0..7 in the record, 8..15 and the destination in addr6 (24 B, 8-B aligned)
    const uint2 x = reinterpret_cast<const uint2*>(a6)[0], y = reinterpret_cast<const uint2*>(a6)[1],
                z = reinterpret_cast<const uint2*>(a6)[2];
    s[0] = __builtin_bswap32(rec[0]); s[1] = __builtin_bswap32(rec[1]); s[2] = __builtin_bswap32(x.x); s[3] = __builtin_bswap32(x.y);
    d[0] = __builtin_bswap32(y.x); d[1] = __builtin_bswap32(y.y); d[2] = __builtin_bswap32(z.x); d[3] = __builtin_bswap32(z.y);
  } else {
    s[0] = rec[0];
    d[0] = rec[1];
#pragma unroll
    for (int j = 1; j < 4; ++j) s[j] = d[j] = 0u;
  }
  const rtn_u32 sp = rec[2] & 0xffffu, dp = rec[2] >> 16;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    k.w[j] = gt ? s[j] : d[j];
    k.w[4 + j] = gt ? d[j] : s[j];
  }
  k.w[8] = gt ? (sp << 16 | dp) : (dp << 16 | sp);
  k.w[9] = (k.tcp ? 6u : 17u) | (k.v6 ? 0x100u : 0u);
  // two independent 32-bit chains; an IPv4 key's words 1-3 and 5-7 are zero and are skipped
  rtn_u32 f0 = 0x0C0FFEEu, f1 = 0x5EED5EEDu;
  if (k.v6) {
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      f0 = rtn_ct_mix(f0, k.w[j]);
      f1 = rtn_ct_mix(f1, k.w[j] ^ 0x9E3779B9u);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 10; j += (j == 0 || j == 4) ? 4 : 1) {
      f0 = rtn_ct_mix(f0, k.w[j]);
      f1 = rtn_ct_mix(f1, k.w[j] ^ 0x9E3779B9u);
    }
  }
  k.fp = ((rtn_u64)rtn_ct_fmix(f0 ^ 40u) << 32) | rtn_ct_fmix(f1 ^ 40u);
  if (k.fp < 2ull) k.fp += 2ull;
}

// LDS visibility between lanes of one wave
__device__ __forceinline__ void rtn_ct_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bool rtn_ct_occupied(const rtn_u32* occ, rtn_u32 slot) {
  return (occ[slot >> 5] >> (slot & 31u)) & 1u;
}
// the same at device scope, for the insert pass, which sets bits while it reads them
__device__ __forceinline__ bool rtn_ct_occupied_now(rtn_u32* occ, rtn_u32 slot) {
  return (__hip_atomic_load(&occ[slot >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (slot & 31u)) & 1u;
}

__device__ __forceinline__ rtn_u64* rtn_ct_tag(const rtn_ct_args& a, rtn_u32 slot) {
  return reinterpret_cast<rtn_u64*>(a.table + (rtn_u64)slot * 16u);
}

// Record-major walk. One wave per 256-frame chunk (RTN_CT_CPB chunks per block); lane l takes the
// chunk's records l, l + 64, ... (a pass per 64 records), so that a wave's loads do not wait for
// the forwarded bitmap: the first pass's rtn_conn_t loads go out with the bitmap words (record
// slot RTN_REC_INDEX(n, c, k) needs only k), and every lane of a pass holds a record. A record's
// frame index is recovered from the chunk's bitmap words (the k-th set bit). The records that
// need the table (openers in the insert pass, frames whose start slot is occupied in the lookup)
// are then compacted into a per-wave LDS list and handled 64 at a time, so the dependent table
// reads run on full waves.
#define RTN_CT_CPB 4u     // chunks (waves) per block
#define RTN_CT_PASSES 4u  // RTN_CT_CHUNK / 64

// position of the r-th set bit of x (r < popcount(x))
__device__ __forceinline__ rtn_u32 rtn_ct_select(rtn_u64 x, rtn_u32 r) {
  rtn_u32 pos = 0u;
#pragma unroll
  for (rtn_u32 w = 32u; w >= 1u; w >>= 1) {
    const rtn_u64 low = x & ((1ull << w) - 1ull);
    const rtn_u32 c = (rtn_u32)__popcll(low);
    const bool up = r >= c;
    r = up ? r - c : r;
    x = up ? x >> w : low;
    pos += up ? w : 0u;
  }
  return pos;
}

struct rtn_ct_chunk {
  rtn_u32 c;          // chunk index (wave-uniform)
  rtn_u64 nch;        // chunks in the batch
  rtn_u64 w[4];       // the chunk's forwarded-bitmap words (wave-uniform)
  rtn_u32 p0, p01, p012, total;  // prefix popcounts
};

// All-ones/zero lane mask hidden from the optimiser, so that a select chain stays v_cndmask /
// v_bfi instead of being folded into a dynamically indexed private array (scratch).
__device__ __forceinline__ rtn_u32 rtn_ct_mask(bool b) {
  rtn_u32 m = b ? 0xffffffffu : 0u;
  asm("" : "+v"(m));
  return m;
}
__device__ __forceinline__ rtn_u32 rtn_ct_sel(rtn_u32 m, rtn_u32 x, rtn_u32 y) { return (x & m) | (y & ~m); }

// frame index of the chunk's k-th forwarded frame
__device__ __forceinline__ rtn_u32 rtn_ct_frame(const rtn_ct_chunk& ch, rtn_u32 k) {
  const rtn_u32 ma = rtn_ct_mask(k < ch.p0), mb = rtn_ct_mask(k < ch.p01), md = rtn_ct_mask(k < ch.p012);
  const rtn_u32 lo = rtn_ct_sel(ma, (rtn_u32)ch.w[0], rtn_ct_sel(mb, (rtn_u32)ch.w[1], rtn_ct_sel(md, (rtn_u32)ch.w[2], (rtn_u32)ch.w[3])));
  const rtn_u32 hi = rtn_ct_sel(ma, (rtn_u32)(ch.w[0] >> 32),
                                rtn_ct_sel(mb, (rtn_u32)(ch.w[1] >> 32), rtn_ct_sel(md, (rtn_u32)(ch.w[2] >> 32), (rtn_u32)(ch.w[3] >> 32))));
  const rtn_u32 before = rtn_ct_sel(ma, 0u, rtn_ct_sel(mb, ch.p0, rtn_ct_sel(md, ch.p01, ch.p012)));
  const rtn_u32 base = rtn_ct_sel(ma, 0u, rtn_ct_sel(mb, 64u, rtn_ct_sel(md, 128u, 192u)));
  return ch.c * RTN_CT_CHUNK + base + rtn_ct_select((rtn_u64)lo | ((rtn_u64)hi << 32), k - before);
}

__device__ __forceinline__ rtn_u64 rtn_ct_rslot(const rtn_ct_chunk& ch, rtn_u32 k) {  // RTN_REC_INDEX
  return ((rtn_u64)(k >> 6) * ch.nch + ch.c) * 64u + (k & 63u);
}

// lane l's 64-bit value (readlane returns int: go through u32, or the low half sign-extends)
__device__ __forceinline__ rtn_u64 rtn_ct_rl64(rtn_u64 v, int l) {
  const rtn_u32 lo = (rtn_u32)__builtin_amdgcn_readlane((int)(rtn_u32)v, l);
  const rtn_u32 hi = (rtn_u32)__builtin_amdgcn_readlane((int)(rtn_u32)(v >> 32), l);
  return (rtn_u64)lo | ((rtn_u64)hi << 32);
}

// The chunk's bitmap words and the rtn_conn_t of its records: cv[j] / has[j] for record
// k = 64 j + lane; pass 0's load is issued with the bitmap words. v6r[j]: the record's rank
// among the chunk's IPv6 records (its addr6 row is c * 256 + v6r).
__device__ __forceinline__ void rtn_ct_begin(const rtn_ct_args& a, rtn_u32 c, rtn_u32 lane, rtn_ct_chunk& ch,
                                             rtn_u64 (&cv)[RTN_CT_PASSES], bool (&has)[RTN_CT_PASSES],
                                             rtn_u32 (&v6r)[RTN_CT_PASSES]) {
  const rtn_u32 nw = (a.n + 63u) / 64u;
  ch.c = c;
  ch.nch = ((rtn_u64)a.n + RTN_CT_CHUNK - 1u) / RTN_CT_CHUNK;
  const rtn_u32 gi = c * 4u + (lane & 3u);
  const rtn_u64 word = gi < nw ? a.fwd_bm[gi] : 0ull;
  // streamed once: non-temporal, so the occupancy bitmap keeps its place in L2
  cv[0] = __builtin_nontemporal_load(a.conn + (rtn_u64)c * 64u + lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) ch.w[j] = rtn_ct_rl64(word, j);
  const rtn_u32 p[4] = {(rtn_u32)__popcll(ch.w[0]), (rtn_u32)__popcll(ch.w[1]), (rtn_u32)__popcll(ch.w[2]),
                        (rtn_u32)__popcll(ch.w[3])};
  ch.p0 = p[0];
  ch.p01 = p[0] + p[1];
  ch.p012 = ch.p01 + p[2];
  ch.total = ch.p012 + p[3];
#pragma unroll
  for (rtn_u32 j = 1; j < RTN_CT_PASSES; ++j) {
    cv[j] = 0ull;
    if (64u * j + lane < ch.total) cv[j] = __builtin_nontemporal_load(a.conn + rtn_ct_rslot(ch, 64u * j + lane));
  }
  const rtn_u64 lane_lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  rtn_u32 v6before = 0u;
#pragma unroll
  for (rtn_u32 j = 0; j < RTN_CT_PASSES; ++j) {
    has[j] = 64u * j + lane < ch.total;
    if (!has[j]) cv[j] = 0ull;
    const rtn_u64 m6 = __ballot(has[j] && ((cv[j] >> 61) & 1ull));  // RTN_CONN_IPV6
    v6r[j] = v6before + (rtn_u32)__popcll(m6 & lane_lt);
    v6before += (rtn_u32)__popcll(m6);
  }
}

// A record the table step needs, staged in LDS: its rank k, IPv6 rank, rtn_conn_t.
struct rtn_ct_item {
  rtn_u64 cv;
  rtn_u32 k, v6r;
};

// Appends the lanes with `take` of every pass to the wave's list; returns the list length.
__device__ __forceinline__ rtn_u32 rtn_ct_compact(rtn_ct_item* list, rtn_u32 lane, const bool (&take)[RTN_CT_PASSES],
                                                  const rtn_u64 (&cv)[RTN_CT_PASSES],
                                                  const rtn_u32 (&v6r)[RTN_CT_PASSES]) {
  const rtn_u64 lane_lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  rtn_u32 cnt = 0u;
#pragma unroll
  for (rtn_u32 j = 0; j < RTN_CT_PASSES; ++j) {
    const rtn_u64 m = __ballot(take[j]);
    if (take[j]) {
      rtn_ct_item& it = list[cnt + (rtn_u32)__popcll(m & lane_lt)];
      it.cv = cv[j];
      it.k = 64u * j + lane;
      it.v6r = v6r[j];
    }
    cnt += (rtn_u32)__popcll(m);
  }
  return cnt;
}

// The record (4 words) of item `it` and its key.
__device__ __forceinline__ void rtn_ct_item_key(const rtn_ct_args& a, const rtn_ct_chunk& ch, const rtn_ct_item& it,
                                                rtn_ct_key& k) {
  const rtn_u64* rp = reinterpret_cast<const rtn_u64*>(a.recs + rtn_ct_rslot(ch, it.k) * 4u);
  rtn_u32 rec[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const rtn_u64 x = __builtin_nontemporal_load(rp + j);
    rec[2 * j] = (rtn_u32)x;
    rec[2 * j + 1] = (rtn_u32)(x >> 32);
  }
  const bool v6 = (it.cv >> 61) & 1ull;
  rtn_ct_make_key(a, rec, it.cv, v6 ? a.addr6 + ((rtn_u64)ch.c * RTN_CT_CHUNK + it.v6r) * 6u : nullptr, k);
}

extern "C" __global__ void __launch_bounds__(64u * RTN_CT_CPB) rtn_ct_insert(rtn_ct_args a) {
  __shared__ rtn_u32 blk[4];  // openers needing a new slot (then tickets drawn), reservation base, granted, rounds
  __shared__ rtn_ct_item lists[RTN_CT_CPB][RTN_CT_CHUNK];
  const rtn_u32 lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const rtn_u32 c = blockIdx.x * RTN_CT_CPB + wv;
  const rtn_u32 nch = (a.n + RTN_CT_CHUNK - 1u) / RTN_CT_CHUNK;
  if (threadIdx.x == 0) {
    blk[0] = 0u;
    blk[3] = 0u;
  }
  rtn_ct_item* list = lists[wv];
  rtn_ct_chunk ch;
  rtn_u64 cv[RTN_CT_PASSES];
  bool has[RTN_CT_PASSES], op[RTN_CT_PASSES];
  rtn_u32 v6r[RTN_CT_PASSES];
  rtn_u32 nop = 0u;
  if (c < nch) {  // wave-uniform
    rtn_ct_begin(a, c, lane, ch, cv, has, v6r);
#pragma unroll
    for (rtn_u32 j = 0; j < RTN_CT_PASSES; ++j) {
      // openers: creates, and not a TCP opener dropped by filter_first_packet
      const rtn_u32 info = (rtn_u32)(cv[j] >> 32);
      const bool tcp = !((info >> 30) & 1u);  // RTN_CONN_UDP
      op[j] = has[j] && ((info >> 26) & 1u) && !(tcp && (info & 0x3ffffffu) == 0u);
    }
    nop = rtn_ct_compact(list, lane, op, cv, v6r);
  }
  __syncthreads();
  // every wave runs the block's largest number of 64-opener rounds (the admission below takes
  // block-wide barriers)
  if (lane == 0u && nop) atomicMax(&blk[3], (nop + 63u) / 64u);
  __syncthreads();
  const rtn_u32 rounds = blk[3];
  for (rtn_u32 rd = 0; rd < rounds; ++rd) {
    const rtn_u32 e = rd * 64u + lane;
    bool active = e < nop;
    rtn_ct_item it = {0ull, 0u, 0u};
    rtn_ct_key k;
    rtn_u32 slot = 0u, frame = 0u;
    if (active) {
      it = list[e];
      rtn_ct_item_key(a, ch, it, k);
      slot = (rtn_u32)it.cv & a.cap_mask;
      frame = rtn_ct_frame(ch, it.k);
    }
    // Phase A: find the key or the first empty slot of its probe chain (no writes), remembering the
    // chain's first removed slot: a key known to be absent reuses it, so that removals do not
    // leave the chains to fill up with tombstones until a rebuild.
    bool at_empty = false;
    rtn_u32 tomb = 0xffffffffu;
    for (rtn_u32 p = 0; p < RTN_CT_MAXPROBE; ++p) {
      bool more = false;
      if (active && !at_empty) {
        // occupancy, tag and epoch are read at device scope (through to L2): slots are claimed
        // during this launch, by other blocks and by this wave's earlier rounds, and a copy of the
        // line in this CU's L1 would show a claimed slot as empty
        const rtn_u64 t = rtn_ct_occupied_now(a.occ, slot)
                              ? __hip_atomic_load(rtn_ct_tag(a, slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : RTN_CT_EMPTY;
        if (t == k.fp) {
          // `first` only matters for a slot opened in this batch (epoch == this batch, or 0 while
          // its claimer is still writing it); an older connection's frames are plain hits
          const rtn_u32 ep = __hip_atomic_load(&a.table[(rtn_u64)slot * 16u + 2u], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
          if (ep == 0u || ep == a.epoch) atomicMin(&a.table[(rtn_u64)slot * 16u + 3u], frame);
          active = false;
        } else if (t == RTN_CT_EMPTY) {
          at_empty = true;
        } else {
          if (t == RTN_CT_REMOVED && tomb == 0xffffffffu) tomb = slot;
          slot = (slot + 1u) & a.cap_mask;
          more = true;
        }
      }
      if (!__ballot(more)) break;
    }
    active = active && at_empty;  // probe limit reached without an empty slot: full
    if (active && tomb != 0xffffffffu) slot = tomb;  // claim from the first removed slot
    const rtn_u32 want = (rtn_u32)__popcll(__ballot(active));
    // Admission (ConnTracker's size < max_connections): the block reserves one ticket per opener
    // that still needs a slot with a single atomic (none once its connections exist) and returns
    // the unused tickets at the end.
    if (a.check) {
      __syncthreads();
      if (threadIdx.x == 0) blk[0] = 0u;
      __syncthreads();
      if (lane == 0u && want) atomicAdd(&blk[0], want);
      __syncthreads();
      if (threadIdx.x == 0) {
        const rtn_u32 all = blk[0];
        const rtn_u32 b = all ? atomicAdd(&a.live[0], all) : 0u;
        blk[1] = all;
        blk[2] = b >= a.max_live ? 0u : (a.max_live - b < all ? a.max_live - b : all);
        blk[0] = 0u;
      }
      __syncthreads();
      const rtn_u32 ticket = active ? atomicAdd(&blk[0], 1u) : 0u;
      if (active && ticket >= blk[2]) active = false;  // table full for this opener
    }
    // Phase B: claim from the first free (empty or removed) slot on (another lane may take it
    // first: keep probing). A removed slot was reset to epoch 0 / first 0xffffffff by its removal,
    // so until its claimer has written the epoch, lanes of the same key lower `first` (phase A).
    rtn_u32 claims = 0u;
    for (rtn_u32 p = 0; p < RTN_CT_MAXPROBE; ++p) {
      bool more = false;
      if (active) {
        rtn_u64* tag = rtn_ct_tag(a, slot);
        rtn_u64 t = __hip_atomic_load(tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const rtn_u64 seen = t;
        if (t <= RTN_CT_REMOVED) t = atomicCAS(tag, seen, k.fp);
        if (t == seen && seen <= RTN_CT_REMOVED) {
          atomicOr(&a.occ[slot >> 5], 1u << (slot & 31u));
          rtn_u32* s = a.table + (rtn_u64)slot * 16u;
          s[2] = a.epoch;
#pragma unroll
          for (int j = 0; j < 10; ++j) s[4 + j] = k.w[j];
          atomicMin(&s[3], frame);
          active = false;
          ++claims;
        } else if (t == k.fp) {
          atomicMin(&a.table[(rtn_u64)slot * 16u + 3u], frame);
          active = false;
        } else {
          slot = (slot + 1u) & a.cap_mask;
          more = true;
        }
      }
      if (!__ballot(more)) break;
    }
    rtn_u32 nclaim = claims;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) nclaim += __shfl_xor(nclaim, d);
    if (a.check) {
      // return the reserved tickets that did not become a connection
      __syncthreads();
      if (threadIdx.x == 0) blk[0] = 0u;
      __syncthreads();
      if (lane == 0u && nclaim) atomicAdd(&blk[0], nclaim);
      __syncthreads();
      if (threadIdx.x == 0 && blk[1] > blk[0]) atomicSub(&a.live[0], blk[1] - blk[0]);
    } else if (lane == 0u && nclaim) {
      // one atomic per wave, spread over 64 counters (live = their sum)
      atomicAdd(&a.live[(blockIdx.x * 8u + wv) & 63u], nclaim);
    }
  }
}

// status of a frame whose key sits at slot s (epoch / first decide the branch)
__device__ __forceinline__ rtn_u32 rtn_ct_status(const rtn_ct_args& a, rtn_u32 epoch, rtn_u32 first, rtn_u32 frame,
                                                 bool opens) {
  if (epoch != a.epoch) return RTN_CT_HIT | RTN_CT_PRIOR;
  return frame > first ? RTN_CT_HIT : frame == first ? RTN_CT_NEW : (opens ? RTN_CT_NEW_DROPPED : RTN_CT_MISS);
}

// outcome of a frame whose key is not in the table
__device__ __forceinline__ rtn_u32 rtn_ct_absent(rtn_u64 cv) {
  const rtn_u32 info = (rtn_u32)(cv >> 32);
  const bool opens = (info >> 26) & 1u;
  const bool dropped = !((info >> 30) & 1u) && (info & 0x3ffffffu) == 0u;  // TCP opener the filter drops
  return !opens ? RTN_CT_MISS : dropped ? RTN_CT_NEW_DROPPED : RTN_CT_FULL;
}

extern "C" __global__ void __launch_bounds__(64u * RTN_CT_CPB) rtn_ct_lookup(rtn_ct_args a) {
  __shared__ rtn_ct_item lists[RTN_CT_CPB][RTN_CT_CHUNK];
  const rtn_u32 lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const rtn_u32 c = blockIdx.x * RTN_CT_CPB + wv;
  const rtn_u32 nch = (a.n + RTN_CT_CHUNK - 1u) / RTN_CT_CHUNK;
  if (c >= nch) return;  // wave-uniform (no block barriers below)
  rtn_ct_item* list = lists[wv];
  rtn_ct_chunk ch;
  rtn_u64 cv[RTN_CT_PASSES];
  bool has[RTN_CT_PASSES], occ0[RTN_CT_PASSES];
  rtn_u32 v6r[RTN_CT_PASSES];
  rtn_ct_begin(a, c, lane, ch, cv, has, v6r);
  // the start slot's occupancy bit (in L2) settles most frames: a clear bit is a miss
#pragma unroll
  for (rtn_u32 j = 0; j < RTN_CT_PASSES; ++j) occ0[j] = has[j] && rtn_ct_occupied(a.occ, (rtn_u32)cv[j] & a.cap_mask);
#pragma unroll
  for (rtn_u32 j = 0; j < RTN_CT_PASSES; ++j)
    if (has[j] && !occ0[j])
      __builtin_nontemporal_store((rtn_u64)RTN_CT_NO_SLOT_K | ((rtn_u64)rtn_ct_absent(cv[j]) << 32),
                                  a.out + rtn_ct_rslot(ch, 64u * j + lane));
  const rtn_u32 nocc = rtn_ct_compact(list, lane, occ0, cv, v6r);
  rtn_ct_wave_sync();
  // The frames whose start slot is occupied, 64 at a time: the slot is read whole (tag, epoch,
  // first, key: one 64-B line) together with the record; only chains walk further.
  for (rtn_u32 e0 = 0; e0 < nocc; e0 += 64u) {
    const rtn_u32 e = e0 + lane;
    if (e >= nocc) break;
    const rtn_ct_item it = list[e];
    rtn_u32 slot = (rtn_u32)it.cv & a.cap_mask;
    const uint4* sp = reinterpret_cast<const uint4*>(a.table + (rtn_u64)slot * 16u);
    const uint4 s0 = sp[0], s1 = sp[1], s2 = sp[2];
    const uint2 s3 = reinterpret_cast<const uint2*>(sp + 3)[0];
    rtn_ct_key k;
    rtn_ct_item_key(a, ch, it, k);
    const rtn_u32 frame = rtn_ct_frame(ch, it.k);
    const bool opens = (it.cv >> 58) & 1ull;  // RTN_CONN_CREATES (info bit 26)
    const rtn_u64 t = (rtn_u64)s0.x | ((rtn_u64)s0.y << 32);
    rtn_u32 status = 0u, found = RTN_CT_NO_SLOT_K;
    if (t == k.fp) {
      const rtn_u32 w[10] = {s1.x, s1.y, s1.z, s1.w, s2.x, s2.y, s2.z, s2.w, s3.x, s3.y};
      bool same = true;
#pragma unroll
      for (int j = 0; j < 10; ++j) same = same && w[j] == k.w[j];
      if (same) {
        found = slot;
        status = rtn_ct_status(a, s0.z, s0.w, frame, opens);
      } else {
        status = RTN_CT_COLLISION;
      }
    } else if (t != RTN_CT_EMPTY) {
      // the start slot holds another key (or was removed): walk the chain
      for (rtn_u32 p = 1; p < RTN_CT_MAXPROBE; ++p) {
        slot = (slot + 1u) & a.cap_mask;
        if (!rtn_ct_occupied(a.occ, slot)) break;
        const rtn_u32* q = a.table + (rtn_u64)slot * 16u;
        const rtn_u64 tt = *reinterpret_cast<const rtn_u64*>(q);
        if (tt == RTN_CT_EMPTY) break;
        if (tt != k.fp) continue;
        bool same = true;
#pragma unroll
        for (int j = 0; j < 10; ++j) same = same && q[4 + j] == k.w[j];
        if (!same) {
          status = RTN_CT_COLLISION;
          break;
        }
        found = slot;
        status = rtn_ct_status(a, q[2], q[3], frame, opens);
        break;
      }
    }
    if (status == 0u) status = rtn_ct_absent(it.cv);
    if (status == RTN_CT_COLLISION) found = RTN_CT_NO_SLOT_K;
    __builtin_nontemporal_store((rtn_u64)found | ((rtn_u64)status << 32), a.out + rtn_ct_rslot(ch, it.k));
  }
}

extern "C" __global__ void __launch_bounds__(256) rtn_ct_remove_k(rtn_u32* table, rtn_u32* occ, rtn_u32* live,
                                                                 const rtn_u32* slots, rtn_u32 n, rtn_u32 cap_mask) {
  const rtn_u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const rtn_u32 slot = slots[i] & cap_mask;
  rtn_u64* tag = reinterpret_cast<rtn_u64*>(table + (rtn_u64)slot * 16u);
  const rtn_u64 t = __hip_atomic_load(tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t <= RTN_CT_REMOVED) return;
  // a tombstone: lookups walk past it, an insert reuses it (epoch 0 and first 0xffffffff: the
  // state of a slot whose claimer has not written it yet). The CAS makes a slot listed twice
  // count once.
  table[(rtn_u64)slot * 16u + 2u] = 0u;
  table[(rtn_u64)slot * 16u + 3u] = 0xffffffffu;
  if (atomicCAS(tag, t, RTN_CT_REMOVED) != t) return;
  atomicSub(&live[0], 1u);
  // A tombstone followed by an empty slot ends no probe chain (every chain through it would have
  // stopped at that empty slot), so it becomes empty again, and so does the run of tombstones
  // before it. Without this, keys whose home slot is empty keep consuming empty slots while
  // tombstones pile up elsewhere, until no chain reaches an empty slot (FULL) before a rebuild.
  // Two removals racing on neighbours: each publishes its own write, fences, then reads the
  // other's slot, so at least one of them sees both tombstones and clears the pair. No insert or
  // lookup runs during this launch, so an empty slot stays empty throughout.
  __threadfence();
  rtn_u32 s = slot;
  for (rtn_u32 p = 0; p < cap_mask; ++p) {
    const rtn_u32 nx = (s + 1u) & cap_mask;
    if ((__hip_atomic_load(&occ[nx >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (nx & 31u)) & 1u) break;
    rtn_u64* ts = reinterpret_cast<rtn_u64*>(table + (rtn_u64)s * 16u);
    if (atomicCAS(ts, RTN_CT_REMOVED, RTN_CT_EMPTY) != RTN_CT_REMOVED) break;
    atomicAnd(&occ[s >> 5], ~(1u << (s & 31u)));
    __threadfence();
    s = (s - 1u) & cap_mask;
  }
}

// Fresh table: every slot empty with first = 0xffffffff.
extern "C" __global__ void __launch_bounds__(256) rtn_ct_clear(rtn_u32* table, rtn_u32 cap) {
  const rtn_u64 i = (rtn_u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  uint4* s = reinterpret_cast<uint4*>(table + i * 16u);
  s[0] = make_uint4(0u, 0u, 0u, 0xffffffffu);
  s[1] = make_uint4(0u, 0u, 0u, 0u);
  s[2] = make_uint4(0u, 0u, 0u, 0u);
  s[3] = make_uint4(0u, 0u, 0u, 0u);
}

// Rebuild: move the live slots of `src` into the cleared table `dst` (same capacity), dropping
// tombstones. Keys and epochs move; `first` restarts at 0xffffffff. new_slot[i] = where slot i
// went (0xffffffff if it was not live) so the host can re-index its per-connection state.
extern "C" __global__ void __launch_bounds__(256) rtn_ct_rehash(const rtn_u32* src, rtn_u32* dst, rtn_u32* dst_occ,
                                                               rtn_u32* new_slot,
                                                               rtn_u32 cap_mask) {
  const rtn_u64 i = (rtn_u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > cap_mask) return;
  const rtn_u32* s = src + i * 16u;
  const rtn_u64 t = *reinterpret_cast<const rtn_u64*>(s);
  if (t <= RTN_CT_REMOVED) {
    new_slot[i] = 0xffffffffu;
    return;
  }
  // the probe start is the rtn_conn_t hash of the key (rtn_conn_hash)
  rtn_u32 h = 0x5EEDu;
  const bool v6 = (s[13] >> 8) & 1u;
  if (v6) {
#pragma unroll
    for (int j = 0; j < 8; ++j) h = rtn_ct_mix(h, s[4 + j]);
  } else {
    h = rtn_ct_mix(h, s[4]);
    h = rtn_ct_mix(h, s[8]);
  }
  h = rtn_ct_mix(h, s[12]);
  h = rtn_ct_mix(h, s[13]);
  h = rtn_ct_fmix(h ^ (v6 ? 40u : 16u));
  rtn_u32 slot = h & cap_mask;
  for (rtn_u32 p = 0; p <= cap_mask; ++p, slot = (slot + 1u) & cap_mask) {
    rtn_u64* tag = reinterpret_cast<rtn_u64*>(dst + (rtn_u64)slot * 16u);
    if (atomicCAS(tag, RTN_CT_EMPTY, t) == RTN_CT_EMPTY) {
      atomicOr(&dst_occ[slot >> 5], 1u << (slot & 31u));
      rtn_u32* d = dst + (rtn_u64)slot * 16u;
      d[2] = s[2];
#pragma unroll
      for (int j = 4; j < 14; ++j) d[j] = s[j];
      new_slot[i] = slot;
      return;
    }
  }
  new_slot[i] = 0xffffffffu;
}
