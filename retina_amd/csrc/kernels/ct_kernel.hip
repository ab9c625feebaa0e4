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
// Two launches per batch, so every frame sees the same table state:
//   rtn_ct_insert  frames that open a connection on a miss (rtn_conn_t creates bit; a TCP opener
//                  whose first-packet filter drops is not inserted: remove_from_table after
//                  filter_first_packet, conntrack/mod.rs:139-141) find or claim their key's slot
//                  (CAS on the tag), then lower the slot's `first` to their frame index.
//   rtn_ct_lookup  every forwarded frame finds its key (tags, then the whole key, so a 64-bit
//                  fingerprint collision is reported instead of aliasing) and gets its status.
// A wave walks one 512-frame chunk: lane = frame, records ranked by the fwd bitmap exactly as
// rtn_pc_run wrote them.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

typedef unsigned int rtn_u32;
typedef unsigned long long rtn_u64;

#define RTN_CT_CHUNK 512u   // RTN_CHUNK_FRAMES
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
  rtn_u32* live;              // [0] live slots, [1] batch epoch
  rtn_u32 n;                  // frames in the batch
  rtn_u32 cap_mask;
  rtn_u32 max_live;
  rtn_u32 epoch;
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

// Canonical key of record r (v6r: its rank among the chunk's IPv6 records) + its 64-bit fingerprint.
__device__ __forceinline__ void rtn_ct_make_key(const rtn_ct_args& a, rtn_u64 r, rtn_u64 v6r, rtn_ct_key& k) {
  const rtn_u32* rec = a.recs + r * 6u;
  const rtn_u32 meta = rec[5];
  const rtn_u64 c = a.conn[r];
  k.h = (rtn_u32)c;
  k.info = (rtn_u32)(c >> 32);
  k.v6 = (meta >> 7) & 1u;
  k.tcp = !((meta >> 6) & 1u);
  const bool gt = (k.info >> 27) & 1u;  // src is the max endpoint
  rtn_u32 s[4], d[4];
  if (k.v6) {
    const rtn_u32* a6 = a.addr6 + v6r * 8u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = __builtin_bswap32(a6[j]);      // raw bytes -> big-endian words, most significant first
      d[j] = __builtin_bswap32(a6[4 + j]);
    }
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
  rtn_u32 f0 = 0x0C0FFEEu, f1 = 0x5EED5EEDu;
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    f0 = rtn_ct_mix(f0, k.w[j]);
    f1 = rtn_ct_mix(f1, k.w[j] ^ 0x9E3779B9u);
  }
  k.fp = ((rtn_u64)rtn_ct_fmix(f0 ^ 40u) << 32) | rtn_ct_fmix(f1 ^ 40u);
  if (k.fp < 2ull) k.fp += 2ull;
}

__device__ __forceinline__ rtn_u64* rtn_ct_tag(const rtn_ct_args& a, rtn_u32 slot) {
  return reinterpret_cast<rtn_u64*>(a.table + (rtn_u64)slot * 16u);
}

// Walk one chunk; fn(record index, ipv6 rank, frame index) for every forwarded frame.
template <typename F>
__device__ __forceinline__ void rtn_ct_walk(const rtn_ct_args& a, F&& fn) {
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const rtn_u32 nchunks = (a.n + RTN_CT_CHUNK - 1u) / RTN_CT_CHUNK;
  if (wave >= nchunks) return;
  const rtn_u64 lane_lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  const rtn_u32 gb = wave * (RTN_CT_CHUNK / 64u);
  const rtn_u32 nw = (a.n + 63u) / 64u;
  const rtn_u32 ge = gb + RTN_CT_CHUNK / 64u < nw ? gb + RTN_CT_CHUNK / 64u : nw;
  rtn_u32 nrec = 0, nv6 = 0;
  for (rtn_u32 g = gb; g < ge; ++g) {
    const rtn_u64 m = a.fwd_bm[g];
    const bool mine = (m >> lane) & 1ull;
    const rtn_u64 r = (rtn_u64)wave * RTN_CT_CHUNK + nrec + (rtn_u32)__popcll(m & lane_lt);
    const bool v6 = mine && ((a.recs[r * 6u + 5u] >> 7) & 1u);
    const rtn_u64 m6 = __ballot(v6);
    const rtn_u64 v6r = (rtn_u64)wave * RTN_CT_CHUNK + nv6 + (rtn_u32)__popcll(m6 & lane_lt);
    if (mine) fn(r, v6r, g * 64u + lane);
    nrec += (rtn_u32)__popcll(m);
    nv6 += (rtn_u32)__popcll(m6);
  }
}

extern "C" __global__ void __launch_bounds__(256) rtn_ct_insert(rtn_ct_args a) {
  rtn_ct_walk(a, [&](rtn_u64 r, rtn_u64 v6r, rtn_u32 frame) {
    const rtn_u64 c = a.conn[r];
    const rtn_u32 info = (rtn_u32)(c >> 32);
    if (!((info >> 26) & 1u)) return;                 // cannot open a connection
    const bool tcp = !((a.recs[r * 6u + 5u] >> 6) & 1u);
    if (tcp && (info & 0x3ffffffu) == 0u) return;     // TCP opener dropped by filter_first_packet
    rtn_ct_key k;
    rtn_ct_make_key(a, r, v6r, k);
    rtn_u32 slot = k.h & a.cap_mask;
    for (rtn_u32 p = 0; p < RTN_CT_MAXPROBE; ++p, slot = (slot + 1u) & a.cap_mask) {
      rtn_u64* tag = rtn_ct_tag(a, slot);
      rtn_u64 t = __hip_atomic_load(tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == RTN_CT_EMPTY) {
        if (atomicAdd(&a.live[0], 1u) >= a.max_live) {  // ConnTracker's max_connections
          atomicSub(&a.live[0], 1u);
          return;
        }
        const rtn_u64 old = atomicCAS(tag, RTN_CT_EMPTY, k.fp);
        if (old == RTN_CT_EMPTY) {
          rtn_u32* s = a.table + (rtn_u64)slot * 16u;
          s[2] = a.epoch;
#pragma unroll
          for (int j = 0; j < 10; ++j) s[4 + j] = k.w[j];
          atomicMin(&s[3], frame);
          return;
        }
        atomicSub(&a.live[0], 1u);
        t = old;
      }
      if (t == k.fp) {
        atomicMin(&a.table[(rtn_u64)slot * 16u + 3u], frame);
        return;
      }
    }
  });
}

extern "C" __global__ void __launch_bounds__(256) rtn_ct_lookup(rtn_ct_args a) {
  rtn_ct_walk(a, [&](rtn_u64 r, rtn_u64 v6r, rtn_u32 frame) {
    rtn_ct_key k;
    rtn_ct_make_key(a, r, v6r, k);
    const bool opens = (k.info >> 26) & 1u;
    const bool dropped = k.tcp && (k.info & 0x3ffffffu) == 0u;
    rtn_u32 slot = k.h & a.cap_mask, status = 0u, found = 0xffffffffu;
    for (rtn_u32 p = 0; p < RTN_CT_MAXPROBE; ++p, slot = (slot + 1u) & a.cap_mask) {
      const rtn_u32* s = a.table + (rtn_u64)slot * 16u;
      const rtn_u64 t = *reinterpret_cast<const rtn_u64*>(s);
      if (t == RTN_CT_EMPTY) break;
      if (t != k.fp) continue;
      bool same = true;
#pragma unroll
      for (int j = 0; j < 10; ++j) same = same && s[4 + j] == k.w[j];
      if (!same) {
        status = RTN_CT_COLLISION;
        break;
      }
      found = slot;
      if (s[2] != a.epoch) {
        status = RTN_CT_HIT | RTN_CT_PRIOR;
      } else {
        const rtn_u32 first = s[3];
        status = frame > first ? RTN_CT_HIT : frame == first ? RTN_CT_NEW : (opens ? RTN_CT_NEW_DROPPED : RTN_CT_MISS);
      }
      break;
    }
    if (status == 0u) status = !opens ? RTN_CT_MISS : dropped ? RTN_CT_NEW_DROPPED : RTN_CT_FULL;
    if (status == RTN_CT_COLLISION) found = 0xffffffffu;
    a.out[r] = (rtn_u64)found | ((rtn_u64)status << 32);
  });
}

// Host-requested removals (terminated / expired / dropped connections): the slots become
// tombstones (probe chains stay intact); rtn_ct_rebuild compacts them away.
extern "C" __global__ void __launch_bounds__(256) rtn_ct_remove_k(rtn_u32* table, rtn_u32* live, const rtn_u32* slots,
                                                                 rtn_u32 n, rtn_u32 cap_mask) {
  const rtn_u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const rtn_u32 slot = slots[i] & cap_mask;
  rtn_u64* tag = reinterpret_cast<rtn_u64*>(table + (rtn_u64)slot * 16u);
  const rtn_u64 t = *tag;
  if (t > RTN_CT_REMOVED) {
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
extern "C" __global__ void __launch_bounds__(256) rtn_ct_rehash(const rtn_u32* src, rtn_u32* dst, rtn_u32* new_slot,
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
