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
// A block walks one 256-frame chunk, a wave one group: lane = frame, records ranked by the fwd
// bitmap exactly as rtn_pc_run wrote them.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

typedef unsigned int rtn_u32;
typedef unsigned long long rtn_u64;

#define RTN_CT_CHUNK 256u   // RTN_CHUNK_FRAMES
#define RTN_CT_GROUPS (RTN_CT_CHUNK / 64u)
#define RTN_CT_MAXPROBE 256u
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
  const rtn_u32* recs;        // rtn_l4ctx_t, 6 words each
  const rtn_u32* addr6;       // 8 words per IPv6 record
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

// Canonical key of a record (its 6 words, its rtn_conn_t, its IPv6 addresses or null) + its
// 64-bit fingerprint.
__device__ __forceinline__ void rtn_ct_make_key(const rtn_ct_args& a, const rtn_u32 (&rec)[6], rtn_u64 c,
                                                const rtn_u32* a6, rtn_ct_key& k) {
  const rtn_u32 meta = rec[5];
  k.h = (rtn_u32)c;
  k.info = (rtn_u32)(c >> 32);
  k.v6 = (meta >> 7) & 1u;
  k.tcp = !((meta >> 6) & 1u);
  const bool gt = (k.info >> 27) & 1u;  // src is the max endpoint
  rtn_u32 s[4], d[4];
  if (k.v6) {
    const uint4 x = reinterpret_cast<const uint4*>(a6)[0], y = reinterpret_cast<const uint4*>(a6)[1];
    s[0] = __builtin_bswap32(x.x); s[1] = __builtin_bswap32(x.y); s[2] = __builtin_bswap32(x.z); s[3] = __builtin_bswap32(x.w);
    d[0] = __builtin_bswap32(y.x); d[1] = __builtin_bswap32(y.y); d[2] = __builtin_bswap32(y.z); d[3] = __builtin_bswap32(y.w);
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

__device__ __forceinline__ bool rtn_ct_occupied(const rtn_u32* occ, rtn_u32 slot) {
  return (occ[slot >> 5] >> (slot & 31u)) & 1u;
}

__device__ __forceinline__ rtn_u64* rtn_ct_tag(const rtn_ct_args& a, rtn_u32 slot) {
  return reinterpret_cast<rtn_u64*>(a.table + (rtn_u64)slot * 16u);
}

#ifndef RTN_CT_GPW
#define RTN_CT_GPW 2u  // 64-frame groups per wave (cfg2 steady pass: 1 -> 0.62, 2 -> 0.52, 4 -> 0.62, 8 -> 1.13 ms)
#endif
// Chunks per block. The insert pass's block takes 2 (4 waves), so its admission costs one
// reservation atomic per 512 frames (one per 256-frame chunk: cfg2 first pass 1.37 -> 1.98 ms);
// the lookup's takes 1 (2 waves: steady pass 0.512 ms with 2 chunks per block, 0.484 with 1).
#define RTN_CT_INSERT_CPB 2u
#define RTN_CT_LOOKUP_CPB 1u
#define RTN_CT_WPC (RTN_CT_GROUPS / RTN_CT_GPW)  // waves per chunk

// One block per chunk; each wave takes RTN_CT_GPW groups and issues all of their loads
// before using any (the walk is latency-bound: a wave per group left too few loads in flight).
// The record rank comes from the chunk's RTN_CT_GROUPS bitmap words; the IPv6 rank needs the IPv6 counts of
// the earlier groups, exchanged through LDS. fn(lane has a record, record index, frame index,
// record words, rtn_conn_t, IPv6 addresses or null) runs for every lane of every wave (lanes
// without a record pass has == false) so that waves can cooperate inside it; it builds the key
// only if it needs it.
struct rtn_ct_frames {  // this lane's frame in each of the wave's RTN_CT_GPW groups
  bool has[RTN_CT_GPW];
  rtn_u64 r[RTN_CT_GPW], cv[RTN_CT_GPW];
  rtn_u32 frame[RTN_CT_GPW];
  rtn_u32 rec[RTN_CT_GPW][6];
  const rtn_u32* a6[RTN_CT_GPW];
};

template <rtn_u32 CPB>
__device__ __forceinline__ void rtn_ct_load(const rtn_ct_args& a, rtn_ct_frames& f) {
  constexpr rtn_u32 G = RTN_CT_GPW;
  __shared__ rtn_u32 v6cnt_all[CPB][RTN_CT_GROUPS];
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 wb = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const rtn_u32 w = wb % RTN_CT_WPC;                   // wave within its chunk
  const rtn_u32 c = blockIdx.x * CPB + wb / RTN_CT_WPC;
  rtn_u32* v6cnt = v6cnt_all[wb / RTN_CT_WPC];
  const rtn_u64 lane_lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  const rtn_u32 nw = (a.n + 63u) / 64u;
  const rtn_u64 nch = ((rtn_u64)a.n + RTN_CT_CHUNK - 1u) / RTN_CT_CHUNK;
  // the chunk's bitmap words: lane j < RTN_CT_GROUPS holds word j; pre[j] = records before group j
  const rtn_u32 gj = c * RTN_CT_GROUPS + (lane & (RTN_CT_GROUPS - 1u));
  const rtn_u64 word = gj < nw ? a.fwd_bm[gj] : 0ull;
  const rtn_u32 pop = (rtn_u32)__popcll(word);
  // (q = w * G + u is not a compile-time index: accumulate per group instead of indexing an array)
  rtn_u32 pre[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) pre[u] = 0u;
#pragma unroll
  for (rtn_u32 j = 0; j < RTN_CT_GROUPS; ++j) {
    const rtn_u32 pj = __shfl(pop, (int)j);
#pragma unroll
    for (rtn_u32 u = 0; u < G; ++u) pre[u] += j < w * G + u ? pj : 0u;
  }
  rtn_u64 m6[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    const rtn_u32 q = w * G + u;  // group within the chunk
    const rtn_u64 m = __shfl(word, (int)q);
    f.has[u] = c * (RTN_CT_CHUNK / 64u) + q < nw && ((m >> lane) & 1ull);
    // record slot (RTN_REC_INDEX, retina_pc.h): block k / 64 of chunk c at block slot
    // (k / 64) * nchunks + c
    const rtn_u32 k = pre[u] + (rtn_u32)__popcll(m & lane_lt);
    f.r[u] = ((rtn_u64)(k >> 6) * nch + c) * 64u + (k & 63u);
    f.frame[u] = (c * (RTN_CT_CHUNK / 64u) + q) * 64u + lane;
#pragma unroll
    for (int j = 0; j < 6; ++j) f.rec[u][j] = 0u;
    // streamed once: non-temporal, so the occupancy bitmap keeps its place in L2. The record
    // itself is read only by frames that need their key (rtn_ct_load_rec): rtn_conn_t carries
    // the IPv6 and UDP bits the rest needs.
    f.cv[u] = f.has[u] ? __builtin_nontemporal_load(a.conn + f.r[u]) : 0ull;
  }
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    m6[u] = __ballot(f.has[u] && ((f.cv[u] >> 61) & 1ull));  // RTN_CONN_IPV6
    if (lane == 0u) v6cnt[w * G + u] = (rtn_u32)__popcll(m6[u]);
  }
  __syncthreads();
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    const rtn_u32 q = w * G + u;
    rtn_u32 v6base = 0u;
    for (rtn_u32 j = 0; j < q; ++j) v6base += v6cnt[j];
    const rtn_u64 v6r = (rtn_u64)c * RTN_CT_CHUNK + v6base + (rtn_u32)__popcll(m6[u] & lane_lt);
    f.a6[u] = (m6[u] >> lane) & 1ull ? a.addr6 + v6r * 8u : nullptr;
  }
}

// The record of group u's frame (for its key).
__device__ __forceinline__ void rtn_ct_load_rec(const rtn_ct_args& a, rtn_ct_frames& f, rtn_u32 u) {
  const rtn_u64* rp = reinterpret_cast<const rtn_u64*>(a.recs + f.r[u] * 6u);  // 8-byte aligned
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const rtn_u64 x = __builtin_nontemporal_load(rp + j);
    f.rec[u][2 * j] = (rtn_u32)x;
    f.rec[u][2 * j + 1] = (rtn_u32)(x >> 32);
  }
}

extern "C" __global__ void __launch_bounds__(64u * RTN_CT_WPC * RTN_CT_INSERT_CPB) rtn_ct_insert(rtn_ct_args a) {
  constexpr rtn_u32 G = RTN_CT_GPW;
  __shared__ rtn_u32 blk[3];  // openers needing a new slot (then tickets drawn), reservation base, granted
  if (threadIdx.x == 0) blk[0] = 0u;
  rtn_ct_frames f;
  rtn_ct_load<RTN_CT_INSERT_CPB>(a, f);
  const rtn_u32 lane = threadIdx.x & 63u;
  bool active[G];
  rtn_u32 slot[G];
  rtn_ct_key k[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    // openers: creates, and not a TCP opener dropped by filter_first_packet
    const rtn_u32 info = (rtn_u32)(f.cv[u] >> 32);
    const bool tcp = !((info >> 30) & 1u);  // RTN_CONN_UDP
    active[u] = f.has[u] && ((info >> 26) & 1u) && !(tcp && (info & 0x3ffffffu) == 0u);
    if (active[u]) rtn_ct_load_rec(a, f, u);
    slot[u] = (rtn_u32)f.cv[u] & a.cap_mask;
  }
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u)
    if (active[u]) rtn_ct_make_key(a, f.rec[u], f.cv[u], f.a6[u], k[u]);
  // Phase A: find the key or the first empty slot of its probe chain (no writes), remembering the
  // chain's first removed slot: a key known to be absent reuses it, so that removals do not
  // leave the chains to fill up with tombstones until a rebuild.
  bool at_empty[G];
  rtn_u32 tomb[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    at_empty[u] = false;
    tomb[u] = 0xffffffffu;
  }
  for (rtn_u32 p = 0; p < RTN_CT_MAXPROBE; ++p) {
    bool more = false;
#pragma unroll
    for (rtn_u32 u = 0; u < G; ++u) {
      if (active[u] && !at_empty[u]) {
        const rtn_u64 t = rtn_ct_occupied(a.occ, slot[u])
                              ? __hip_atomic_load(rtn_ct_tag(a, slot[u]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : RTN_CT_EMPTY;
        if (t == k[u].fp) {
          // `first` only matters for a slot opened in this batch (epoch == this batch, or 0 while
          // its claimer is still writing it); an older connection's frames are plain hits
          const rtn_u32 ep = a.table[(rtn_u64)slot[u] * 16u + 2u];
          if (ep == 0u || ep == a.epoch) atomicMin(&a.table[(rtn_u64)slot[u] * 16u + 3u], f.frame[u]);
          active[u] = false;
        } else if (t == RTN_CT_EMPTY) {
          at_empty[u] = true;
        } else {
          if (t == RTN_CT_REMOVED && tomb[u] == 0xffffffffu) tomb[u] = slot[u];
          slot[u] = (slot[u] + 1u) & a.cap_mask;
          more = true;
        }
      }
    }
    if (!__ballot(more)) break;
  }
  rtn_u32 want = 0u;
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    active[u] = active[u] && at_empty[u];  // probe limit reached without an empty slot: full
    if (active[u] && tomb[u] != 0xffffffffu) slot[u] = tomb[u];  // claim from the first removed slot
    want += (rtn_u32)__popcll(__ballot(active[u]));
  }
  // Admission (ConnTracker's size < max_connections): the block reserves one ticket per opener
  // that still needs a slot with a single atomic (none once its connections exist) and returns
  // the unused tickets at the end.
  if (a.check) {
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
#pragma unroll
    for (rtn_u32 u = 0; u < G; ++u) {
      const rtn_u32 ticket = active[u] ? atomicAdd(&blk[0], 1u) : 0u;
      if (active[u] && ticket >= blk[2]) active[u] = false;  // table full for this opener
    }
  }
  // Phase B: claim from the first free (empty or removed) slot on (another lane may take it
  // first: keep probing). A removed slot was reset to epoch 0 / first 0xffffffff by its removal,
  // so until its claimer has written the epoch, lanes of the same key lower `first` (phase A).
  rtn_u32 claims = 0u;
  for (rtn_u32 p = 0; p < RTN_CT_MAXPROBE; ++p) {
    bool more = false;
#pragma unroll
    for (rtn_u32 u = 0; u < G; ++u) {
      if (active[u]) {
        rtn_u64* tag = rtn_ct_tag(a, slot[u]);
        rtn_u64 t = __hip_atomic_load(tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const rtn_u64 seen = t;
        if (t <= RTN_CT_REMOVED) t = atomicCAS(tag, seen, k[u].fp);
        if (t == seen && seen <= RTN_CT_REMOVED) {
          atomicOr(&a.occ[slot[u] >> 5], 1u << (slot[u] & 31u));
          rtn_u32* s = a.table + (rtn_u64)slot[u] * 16u;
          s[2] = a.epoch;
#pragma unroll
          for (int j = 0; j < 10; ++j) s[4 + j] = k[u].w[j];
          atomicMin(&s[3], f.frame[u]);
          active[u] = false;
          ++claims;
        } else if (t == k[u].fp) {
          atomicMin(&a.table[(rtn_u64)slot[u] * 16u + 3u], f.frame[u]);
          active[u] = false;
        } else {
          slot[u] = (slot[u] + 1u) & a.cap_mask;
          more = true;
        }
      }
    }
    if (!__ballot(more)) break;
  }
  rtn_u32 n = claims;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) n += __shfl_xor(n, d);
  if (a.check) {
    // return the reserved tickets that did not become a connection
    __syncthreads();
    if (threadIdx.x == 0) blk[0] = 0u;
    __syncthreads();
    if (lane == 0u && n) atomicAdd(&blk[0], n);
    __syncthreads();
    if (threadIdx.x == 0 && blk[1] > blk[0]) atomicSub(&a.live[0], blk[1] - blk[0]);
  } else if (lane == 0u && n) {
    // one atomic per wave, spread over 64 counters (live = their sum)
    atomicAdd(&a.live[(blockIdx.x * 8u + (threadIdx.x >> 6)) & 63u], n);
  }
}

// status of a frame whose key sits at slot s (epoch / first decide the branch)
__device__ __forceinline__ rtn_u32 rtn_ct_status(const rtn_ct_args& a, rtn_u32 epoch, rtn_u32 first, rtn_u32 frame,
                                                 bool opens) {
  if (epoch != a.epoch) return RTN_CT_HIT | RTN_CT_PRIOR;
  return frame > first ? RTN_CT_HIT : frame == first ? RTN_CT_NEW : (opens ? RTN_CT_NEW_DROPPED : RTN_CT_MISS);
}

extern "C" __global__ void __launch_bounds__(64u * RTN_CT_WPC * RTN_CT_LOOKUP_CPB) rtn_ct_lookup(rtn_ct_args a) {
  constexpr rtn_u32 G = RTN_CT_GPW;
  rtn_ct_frames f;
  rtn_ct_load<RTN_CT_LOOKUP_CPB>(a, f);
  // Every group's first probe is issued before any is used: the start slot's occupancy bit (in
  // L2; most misses end here), then the tags of occupied start slots, then the slots whose tag
  // matches. Only chains (start slot held by another key or removed) probe further, one by one.
  bool occ0[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    occ0[u] = f.has[u] && rtn_ct_occupied(a.occ, (rtn_u32)f.cv[u] & a.cap_mask);
  }
  // an occupied start slot is read whole (tag, epoch, first, key: one 64-B line) in one go
  rtn_ct_key k[G];
  rtn_u64 t[G];
  uint4 s0[G], s1[G], s2[G];  // words 0-11 (tag, epoch, first, key 0-7); key 8-9 in s3
  uint2 s3[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    t[u] = RTN_CT_EMPTY;
    if (occ0[u]) {
      const uint4* sp = reinterpret_cast<const uint4*>(a.table + (rtn_u64)((rtn_u32)f.cv[u] & a.cap_mask) * 16u);
      s0[u] = sp[0];
      s1[u] = sp[1];
      s2[u] = sp[2];
      s3[u] = reinterpret_cast<const uint2*>(sp + 3)[0];
      rtn_ct_load_rec(a, f, u);
    }
  }
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    if (occ0[u]) {
      rtn_ct_make_key(a, f.rec[u], f.cv[u], f.a6[u], k[u]);
      t[u] = (rtn_u64)s0[u].x | ((rtn_u64)s0[u].y << 32);
    }
  }
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    if (!f.has[u]) continue;
    const rtn_u64 cv = f.cv[u];
    const rtn_u32 info = (rtn_u32)(cv >> 32), frame = f.frame[u];
    const bool opens = (info >> 26) & 1u;
    const bool dropped = !((info >> 30) & 1u) && (info & 0x3ffffffu) == 0u;  // TCP opener the filter drops
    rtn_u32 slot = (rtn_u32)cv & a.cap_mask, status = 0u, found = 0xffffffffu;
    if (occ0[u] && t[u] == k[u].fp) {
      const rtn_u32 w[10] = {s1[u].x, s1[u].y, s1[u].z, s1[u].w, s2[u].x, s2[u].y, s2[u].z, s2[u].w, s3[u].x, s3[u].y};
      bool same = true;
#pragma unroll
      for (int j = 0; j < 10; ++j) same = same && w[j] == k[u].w[j];
      if (same) {
        found = slot;
        status = rtn_ct_status(a, s0[u].z, s0[u].w, frame, opens);
      } else {
        status = RTN_CT_COLLISION;
      }
    } else if (occ0[u] && t[u] != RTN_CT_EMPTY) {
      // the start slot holds another key (or was removed): walk the chain
      for (rtn_u32 p = 1; p < RTN_CT_MAXPROBE; ++p) {
        slot = (slot + 1u) & a.cap_mask;
        if (!rtn_ct_occupied(a.occ, slot)) break;
        const rtn_u32* sp = a.table + (rtn_u64)slot * 16u;
        const rtn_u64 tt = *reinterpret_cast<const rtn_u64*>(sp);
        if (tt == RTN_CT_EMPTY) break;
        if (tt != k[u].fp) continue;
        bool same = true;
#pragma unroll
        for (int j = 0; j < 10; ++j) same = same && sp[4 + j] == k[u].w[j];
        if (!same) {
          status = RTN_CT_COLLISION;
          break;
        }
        found = slot;
        status = rtn_ct_status(a, sp[2], sp[3], frame, opens);
        break;
      }
    }
    if (status == 0u) status = !opens ? RTN_CT_MISS : dropped ? RTN_CT_NEW_DROPPED : RTN_CT_FULL;
    if (status == RTN_CT_COLLISION) found = 0xffffffffu;
    __builtin_nontemporal_store((rtn_u64)found | ((rtn_u64)status << 32), a.out + f.r[u]);
  }
}

extern "C" __global__ void __launch_bounds__(256) rtn_ct_remove_k(rtn_u32* table, rtn_u32* live, const rtn_u32* slots,
                                                                 rtn_u32 n, rtn_u32 cap_mask) {
  const rtn_u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const rtn_u32 slot = slots[i] & cap_mask;
  rtn_u64* tag = reinterpret_cast<rtn_u64*>(table + (rtn_u64)slot * 16u);
  const rtn_u64 t = *tag;
  if (t > RTN_CT_REMOVED) {
    // a tombstone: lookups walk past it, an insert reuses it (epoch 0 and first 0xffffffff: the
    // state of a slot whose claimer has not written it yet)
    table[(rtn_u64)slot * 16u + 2u] = 0u;
    table[(rtn_u64)slot * 16u + 3u] = 0xffffffffu;
    *tag = RTN_CT_REMOVED;
    atomicSub(&live[0], 1u);
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
