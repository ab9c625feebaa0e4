// Capture walk on the GPU (rtn_pcap_next_batch_gpu, include/retina_ingest.h): a window of a
// libpcap / pcapng file, copied to HBM as it is, -> the compact split layout of retina_pc.h.
//
// The reference reads a capture record by record (Capture::next_packet of the pcap crate behind
// core/src/runtime/offline.rs:64-82): each record's offset is the previous one's plus its
// length, a chain of dependent reads that bounds a host walk at one cache miss per record. Here
// the window is cut into RTN_CAP_SEG-byte segments and the record chain is found in parallel:
//   1. rtn_cap_cand: per segment, the first RTN_CAP_C offsets whose bytes read as a plausible
//      record header (two chained headers); segment 0's only candidate is offset 0, the window's
//      first record. A segment's true first record is almost always among them: a misread that
//      stays in phase with the true records (fixed-size frames) is just another candidate;
//   2. rtn_cap_nodes: every candidate walks its chain to the first record at or past its
//      segment's end, counting records and frames kept under the mtu rule; where that exit is a
//      candidate of the segment it falls in, it links to it (a graph of candidate "nodes");
//   3. rtn_cap_jump: pointer jumping over the links (log2(segments) launches);
//   4. rtn_cap_lift: per segment, binary lifting from the window's first record finds the node
//      on the true chain in that segment (if a record starts there); the chain ends at a stop (a
//      record past the window, the end of the file) or, rarely, at an exit that no candidate
//      matched: the batch then ends at that true record and the next call starts there;
//   5. rtn_cap_scan / rtn_cap_emit: exclusive prefixes of the chain's counts, then each segment
//      writes the device address and data_len of its kept frames at their batch positions;
//   6. rtn_cap_pack: the frames' first 64 bytes into head slots and, where rtn_ext_needed holds,
//      bytes [64, 128) into ext rows compact within each 256-frame chunk (the layout of
//      rtn_stage_gather), reading 4-byte-aligned words (records are not aligned) and shifting.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

typedef unsigned int rtn_u32;
typedef unsigned long long rtn_u64;
typedef unsigned int rtn_v4u __attribute__((ext_vector_type(4)));

#define RTN_CAP_SEG 4096u
#define RTN_CAP_C 8u  // candidates per segment
// exit markers (the low 48 bits hold a window offset)
#define RTN_CAP_STOP (1ull << 63)   // the chain ends at the offset: the record is past the window
#define RTN_CAP_EOF (1ull << 61)    // ... and the file ends there (truncated or malformed record)
#define RTN_CAP_ERR (1ull << 60)    // ... a pcapng section in another byte order (host path only)
#define RTN_CAP_DEAD (1ull << 59)   // the chain reached a record no candidate matched: the batch
                                    // ends there, the next one starts there
#define RTN_CAP_OFF(x) ((x) & 0xFFFFFFFFFFFFull)
// link targets that are not nodes
#define RTN_CAP_INVALID 0xFFFFFFFFu
#define RTN_CAP_STOPN 0xFFFFFFFEu
#define RTN_CAP_ENDN 0xFFFFFFFDu
#define RTN_CAP_NOPATH 0xFFFFFFFFu

struct rtn_cap_args {
  const unsigned char* win;  // window bytes, readable up to win + bytes + 256
  rtn_u64 bytes;             // window length
  rtn_u32 nseg;              // ceil(bytes / RTN_CAP_SEG)
  rtn_u32 fmt;               // 0 libpcap, 1 pcapng
  rtn_u32 swap;              // fields in the other byte order
  rtn_u32 mtu;               // a frame whose original length exceeds it is skipped (offline.rs:68)
  rtn_u32 at_eof;            // the window ends at the end of the file
  rtn_u32 levels;            // pointer-jumping levels K (jump tables 0..K)
  rtn_u32 k;                 // rtn_cap_jump: the level it builds
  rtn_u32 pad0;
  rtn_u64* cand;             // [nseg][C] candidate offsets
  rtn_u32* ncand;            // [nseg]
  rtn_u64* nexit;            // [nseg * C] node exits (offset, or offset | stop bits)
  rtn_u32* ncnt;             // [nseg * C][3] records, kept frames, first bad kept frame (local)
  rtn_u32* jump;             // [levels + 1][nseg * C]
  rtn_u32* path;             // [nseg] the chain's node in the segment, or RTN_CAP_NOPATH
  rtn_u32* pre;              // [nseg][2] exclusive prefixes of records / kept frames
  rtn_u32* red;              // [4]: segments the chain covers, -, their records, their kept frames
  rtn_u32* tgt;              // [2]: frames in the batch (min(cap, first bad, kept)), first bad kept frame
  rtn_u32 cap;
  rtn_u32 pad1;
  rtn_u64* ptrs;             // [cap] device address of each kept frame's data
  unsigned short* dlen;      // [cap]
  rtn_u64* cut;              // [4]: window offset and record index of the first kept frame not in the
                             // batch; the chain's exit (offset | stop / dead bits); the captured
                             // bytes of the batch's frames (atomicAdd)
};

// 32 bits at any byte offset (records are not aligned): two aligned words and a shift.
__device__ __forceinline__ rtn_u32 rtn_cap_ld32(const unsigned char* w, rtn_u64 off, bool swap) {
  const rtn_u64 at = reinterpret_cast<rtn_u64>(w) + off;
  const rtn_u32* p = reinterpret_cast<const rtn_u32*>(at & ~3ull);
  const rtn_u32 v = __builtin_amdgcn_alignbyte(p[1], p[0], (rtn_u32)(at & 3u));
  return swap ? __builtin_bswap32(v) : v;
}

// One record at window offset off. kind: 0 = a record (len bytes, maybe a frame), 1 = the record
// does not fit in the window (not at the end of the file: the next window starts at it), 2 = end
// of the capture (truncated or malformed, as the host reader ends), 3 = pcapng byte-order change.
struct rtn_cap_rec {
  rtn_u32 kind;
  rtn_u64 len;
  bool frame;
  rtn_u32 caplen, origlen, data;
};

__device__ __forceinline__ rtn_cap_rec rtn_cap_read(const rtn_cap_args& a, rtn_u64 off) {
  rtn_cap_rec r = {0u, 0ull, false, 0u, 0u, 0u};
  const bool sw = a.swap != 0u;
  const rtn_u32 past = a.at_eof ? 2u : 1u;
  if (a.fmt == 0u) {  // libpcap: ts_sec, ts_usec, incl_len, orig_len, then incl_len bytes
    if (off + 16u > a.bytes) { r.kind = past; return r; }
    r.caplen = rtn_cap_ld32(a.win, off + 8u, sw);
    r.origlen = rtn_cap_ld32(a.win, off + 12u, sw);
    r.len = 16ull + r.caplen;
    if (off + r.len > a.bytes) { r.kind = past; return r; }
    r.frame = true;
    r.data = 16u;
    return r;
  }
  // pcapng: type, block total length, body, block total length
  if (off + 12u > a.bytes) { r.kind = past; return r; }
  const rtn_u32 type = rtn_cap_ld32(a.win, off, sw);
  // a section header in the other byte order (its length reads wrong in this one)
  if (type == 0x0A0D0D0Au && rtn_cap_ld32(a.win, off + 8u, false) != (sw ? 0x4D3C2B1Au : 0x1A2B3C4Du)) {
    r.kind = 3u;
    return r;
  }
  const rtn_u32 blen = rtn_cap_ld32(a.win, off + 4u, sw);
  if (blen < 12u) { r.kind = 2u; return r; }
  r.len = blen;
  if (off + blen > a.bytes) { r.kind = past; return r; }
  if (type == 6u && blen >= 32u) {  // enhanced packet block
    r.caplen = rtn_cap_ld32(a.win, off + 20u, sw);
    r.origlen = rtn_cap_ld32(a.win, off + 24u, sw);
    if (28ull + r.caplen > blen) { r.kind = 2u; return r; }
    r.frame = true;
    r.data = 28u;
  } else if (type == 3u && blen >= 16u) {  // simple packet block
    r.origlen = rtn_cap_ld32(a.win, off + 8u, sw);
    r.caplen = r.origlen < blen - 16u ? r.origlen : blen - 16u;
    r.frame = true;
    r.data = 12u;
  }
  return r;
}

// A plausible record header at off (the speculation of step 1; the walk confirms it). libpcap:
// a non-empty frame with incl_len <= orig_len <= 256 KiB and a sub-second field below 10^9, whose
// successor header is plausible too (zero runs and payload bytes rarely chain twice); pcapng: a
// block length that is a multiple of 4 and repeated at the block's end.
__device__ __forceinline__ bool rtn_cap_hdr_ok(const rtn_cap_args& a, rtn_u64 off, rtn_u32& len) {
  const bool sw = a.swap != 0u;
  if (a.fmt == 0u) {
    if (off + 16u > a.bytes) return false;
    const rtn_u32 usec = rtn_cap_ld32(a.win, off + 4u, sw), cl = rtn_cap_ld32(a.win, off + 8u, sw),
                  ol = rtn_cap_ld32(a.win, off + 12u, sw);
    len = 16u + cl;
    return usec < 1000000000u && cl >= 1u && cl <= ol && ol <= 0x40000u && off + len <= a.bytes;
  }
  if (off + 12u > a.bytes) return false;
  const rtn_u32 blen = rtn_cap_ld32(a.win, off + 4u, sw);
  len = blen;
  return blen >= 12u && (blen & 3u) == 0u && blen <= 0x40100u && off + blen <= a.bytes &&
         rtn_cap_ld32(a.win, off + blen - 4u, sw) == blen;
}
__device__ __forceinline__ bool rtn_cap_plausible(const rtn_cap_args& a, rtn_u64 off) {
  rtn_u32 len = 0u, len2 = 0u;
  if (!rtn_cap_hdr_ok(a, off, len)) return false;
  // the successor must read as a header too, unless the record ends the window
  return off + len >= a.bytes || rtn_cap_hdr_ok(a, off + len, len2);
}

// 1. One wave per segment: lanes test 64 consecutive offsets at a time, the first RTN_CAP_C
// plausible ones are the segment's candidates.
extern "C" __global__ void __launch_bounds__(256) rtn_cap_cand(rtn_cap_args a) {
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 s = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  if (s >= a.nseg) return;
  rtn_u64* c = a.cand + (rtn_u64)s * RTN_CAP_C;
  if (s == 0u) {  // the window starts at a record
    if (lane == 0u) {
      c[0] = 0ull;
      a.ncand[0] = 1u;
    }
    return;
  }
  const rtn_u64 b = (rtn_u64)s * RTN_CAP_SEG, e = b + RTN_CAP_SEG < a.bytes ? b + RTN_CAP_SEG : a.bytes;
  const rtn_u64 lane_lt = lane == 0u ? 0ull : (~0ull >> (64u - lane));
  rtn_u32 got = 0u;
  for (rtn_u64 o = b; o < e && got < RTN_CAP_C; o += 64u) {
    const bool ok = o + lane < e && rtn_cap_plausible(a, o + lane);
    const rtn_u64 m = __ballot(ok);
    const rtn_u32 r = got + (rtn_u32)__popcll(m & lane_lt);
    if (ok && r < RTN_CAP_C) c[r] = o + lane;
    got += (rtn_u32)__popcll(m);
  }
  if (lane == 0u) a.ncand[s] = got < RTN_CAP_C ? got : RTN_CAP_C;
}

// 2. One lane per node (segment s, candidate j): walk to the exit, count, link.
extern "C" __global__ void __launch_bounds__(256) rtn_cap_nodes(rtn_cap_args a) {
  const rtn_u32 v = blockIdx.x * blockDim.x + threadIdx.x;
  const rtn_u32 s = v / RTN_CAP_C, j = v % RTN_CAP_C;
  if (s >= a.nseg) return;
  if (j >= a.ncand[s]) {
    a.jump[v] = RTN_CAP_INVALID;
    return;
  }
  const rtn_u64 end = (rtn_u64)(s + 1u) * RTN_CAP_SEG;
  rtn_u64 x = a.cand[v];
  rtn_u32 recs = 0u, kept = 0u, bad = 0xFFFFFFFFu;
  while (x < end) {
    const rtn_cap_rec r = rtn_cap_read(a, x);
    if (r.kind != 0u) {
      x |= RTN_CAP_STOP | (r.kind >= 2u ? RTN_CAP_EOF : 0ull) | (r.kind == 3u ? RTN_CAP_ERR : 0ull);
      break;
    }
    if (r.frame) {
      ++recs;
      if (r.origlen <= a.mtu) {  // offline.rs:68-70
        if (r.caplen > 0xFFFFu && bad == 0xFFFFFFFFu) bad = kept;  // Mbuf::data_len is a u16
        ++kept;
      }
    }
    x += r.len;
  }
  a.nexit[v] = x;
  a.ncnt[3u * v] = recs;
  a.ncnt[3u * v + 1u] = kept;
  a.ncnt[3u * v + 2u] = bad;
  rtn_u32 nx = RTN_CAP_INVALID;
  if (x & RTN_CAP_STOP) {
    nx = RTN_CAP_STOPN;
  } else if (x / RTN_CAP_SEG >= a.nseg) {
    nx = RTN_CAP_ENDN;  // (the last record ends exactly at a segment-aligned window end)
  } else {
    const rtn_u32 t = (rtn_u32)(x / RTN_CAP_SEG), nt = a.ncand[t];
    const rtn_u64* ct = a.cand + (rtn_u64)t * RTN_CAP_C;
    for (rtn_u32 i = 0; i < nt; ++i)
      if (ct[i] == x) {
        nx = t * RTN_CAP_C + i;
        break;
      }
  }
  a.jump[v] = nx;
}

// 3. jump[k][v] = jump[k-1][jump[k-1][v]]; the link targets that are not nodes absorb.
extern "C" __global__ void __launch_bounds__(256) rtn_cap_jump(rtn_cap_args a) {
  const rtn_u32 v = blockIdx.x * blockDim.x + threadIdx.x;
  const rtn_u32 n = a.nseg * RTN_CAP_C;
  if (v >= n) return;
  const rtn_u32* p = a.jump + (rtn_u64)(a.k - 1u) * n;
  const rtn_u32 u = p[v];
  a.jump[(rtn_u64)a.k * n + v] = u >= RTN_CAP_ENDN ? u : p[u];
}

// 4. One lane per segment: the last node of the true chain at or before the segment (binary
// lifting from the window's first record, node 0); the lane of the last segment also records
// where the chain ends.
extern "C" __global__ void __launch_bounds__(256) rtn_cap_lift(rtn_cap_args a) {
  const rtn_u32 s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.nseg) return;
  const rtn_u32 n = a.nseg * RTN_CAP_C;
  rtn_u32 v = 0u;
  for (int k = (int)a.levels; k >= 0; --k) {
    const rtn_u32 u = a.jump[(rtn_u64)k * n + v];
    if (u < RTN_CAP_ENDN && u / RTN_CAP_C <= s) v = u;
  }
  a.path[s] = v / RTN_CAP_C == s ? v : RTN_CAP_NOPATH;
  if (s + 1u == a.nseg) {
    const rtn_u32 t = a.jump[v];
    a.red[0] = v / RTN_CAP_C + 1u;
    a.cut[2] = a.nexit[v] | (t == RTN_CAP_INVALID ? RTN_CAP_DEAD : 0ull);
  }
}

// 5a. One block: exclusive prefixes of records / kept frames over the segments the chain covers,
// totals, and the batch size.
extern "C" __global__ void __launch_bounds__(1024) rtn_cap_scan(rtn_cap_args a) {
  __shared__ rtn_u32 wsum[2][16];
  __shared__ rtn_u32 wbad[16];
  const rtn_u32 t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const rtn_u32 nseg = a.red[0];
  const rtn_u32 per = (nseg + 1023u) / 1024u;
  const rtn_u32 s0 = t * per;
  rtn_u32 r = 0u, k = 0u, bad = 0xFFFFFFFFu;
  for (rtn_u32 j = 0; j < per; ++j) {
    const rtn_u32 s = s0 + j;
    const rtn_u32 v = s < nseg ? a.path[s] : RTN_CAP_NOPATH;
    if (v != RTN_CAP_NOPATH) {
      const rtn_u32 b = a.ncnt[3u * v + 2u];
      if (b != 0xFFFFFFFFu && bad == 0xFFFFFFFFu) bad = k + b;  // local kept index, this thread's run
      r += a.ncnt[3u * v];
      k += a.ncnt[3u * v + 1u];
    }
  }
  // inclusive scan within the wave
  rtn_u32 ri = r, ki = k;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const rtn_u32 rr = __shfl_up(ri, d), kk = __shfl_up(ki, d);
    if (lane >= (rtn_u32)d) { ri += rr; ki += kk; }
  }
  if (lane == 63u) { wsum[0][wv] = ri; wsum[1][wv] = ki; }
  __syncthreads();
  rtn_u32 rb = 0u, kb = 0u;
  for (rtn_u32 w = 0; w < wv; ++w) { rb += wsum[0][w]; kb += wsum[1][w]; }
  rtn_u32 rx = rb + ri - r, kx = kb + ki - k;  // exclusive prefix of this thread's run
  const rtn_u32 gbad = bad == 0xFFFFFFFFu ? 0xFFFFFFFFu : kx + bad;
  rtn_u32 mb = gbad;  // first bad kept frame of the batch: min over threads
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mb = min(mb, (rtn_u32)__shfl_xor(mb, d));
  if (lane == 0u) wbad[wv] = mb;
  for (rtn_u32 j = 0; j < per; ++j) {
    const rtn_u32 s = s0 + j;
    if (s < nseg) {
      a.pre[2u * s] = rx;
      a.pre[2u * s + 1u] = kx;
      const rtn_u32 v = a.path[s];
      if (v != RTN_CAP_NOPATH) {
        rx += a.ncnt[3u * v];
        kx += a.ncnt[3u * v + 1u];
      }
    }
  }
  __syncthreads();
  if (t == 1023u) {
    rtn_u32 fb = 0xFFFFFFFFu;
    for (rtn_u32 w = 0; w < 16u; ++w) fb = min(fb, wbad[w]);
    a.red[2] = rx;  // records and kept frames of the chain
    a.red[3] = kx;
    const rtn_u32 n = kx < a.cap ? kx : a.cap;
    a.tgt[0] = fb < n ? fb : n;
    a.tgt[1] = fb;
  }
}

// 5b. One lane per segment on the chain: its kept frames of the batch, and where the batch ends.
extern "C" __global__ void __launch_bounds__(256) rtn_cap_emit(rtn_cap_args a) {
  const rtn_u32 s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.red[0]) return;
  const rtn_u32 v = a.path[s];
  if (v == RTN_CAP_NOPATH) return;
  const rtn_u32 tgt = a.tgt[0];
  rtn_u32 r = a.pre[2u * s], f = a.pre[2u * s + 1u];
  if (f > tgt || (f == tgt && a.ncnt[3u * v + 1u] == 0u)) return;
  const rtn_u64 end = (rtn_u64)(s + 1u) * RTN_CAP_SEG;
  rtn_u64 x = a.cand[v], bytes = 0ull;
  while (x < end) {
    const rtn_cap_rec rec = rtn_cap_read(a, x);
    if (rec.kind != 0u) break;
    if (rec.frame) {
      if (rec.origlen <= a.mtu) {
        if (f == tgt) {  // the first frame not in the batch
          a.cut[0] = x;
          a.cut[1] = r;
          break;
        }
        a.ptrs[f] = reinterpret_cast<rtn_u64>(a.win) + x + rec.data;
        a.dlen[f] = (unsigned short)rec.caplen;
        bytes += rec.caplen;
        ++f;
      }
      ++r;
    }
    x += rec.len;
  }
  if (bytes) atomicAdd(&a.cut[3], bytes);
}

struct rtn_cap_pack_args {
  const rtn_u64* ptrs;        // [n] device addresses of the frames' data
  const unsigned short* dl;   // [n]
  unsigned char* head;        // [ceil(n/256)*256][64]
  unsigned char* ext;         // [ceil(n/256)*256][64]: chunk c's rows at [c*256, ...)
  rtn_u32* ext_chunk;         // [ceil(n/256)] = c * 256
  unsigned short* dlen;       // [n]
  rtn_u32 n;
};

// rtn_ext_needed (retina_pc.h) on a frame's first 20 bytes (words 3 and 4).
__device__ __forceinline__ bool rtn_cap_need(rtn_u32 w3, rtn_u32 w4, rtn_u32 dl) {
  const rtn_u32 et = __builtin_amdgcn_perm(0u, w3, 0x0c0c0001u);
  const bool q = et == 0x8100u;
  const rtn_u32 inner = q ? __builtin_amdgcn_perm(0u, w4, 0x0c0c0001u) : et;
  const rtn_u32 vihl = q ? (w4 >> 16) & 0xffu : (w3 >> 16) & 0xffu;
  const rtn_u32 l4 = (q ? 18u : 14u) + (inner == 0x86DDu ? 40u : ((vihl & 0xfu) << 2));
  const bool ip = inner == 0x0800u || inner == 0x86DDu;
  return ip && dl > 64u && l4 + 20u > 64u;
}

// 64 bytes at byte address p (any alignment), as 16 words: 17 aligned loads and a shift.
__device__ __forceinline__ void rtn_cap_load64(rtn_u64 p, rtn_u32 (&w)[16]) {
  const rtn_u32* q = reinterpret_cast<const rtn_u32*>(p & ~3ull);
  const rtn_u32 sh = (rtn_u32)(p & 3u);
  rtn_u32 x[17];
#pragma unroll
  for (int j = 0; j < 17; ++j) x[j] = q[j];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
}

// 5. One wave per 256-frame chunk; lane l packs frames l, l + 64, l + 128, l + 192.
extern "C" __global__ void __launch_bounds__(256) rtn_cap_pack(rtn_cap_pack_args a) {
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  const rtn_u32 nch = (a.n + 255u) >> 8;
  if (c >= nch) return;
  const rtn_u32 base = c << 8;
  const rtn_u64 lane_lt = lane == 0u ? 0ull : (~0ull >> (64u - lane));
  rtn_u32 rows = 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const rtn_u32 i = base + lane + 64u * j;
    const bool ok = i < a.n;
    const rtn_u64 p = ok ? a.ptrs[i] : 0ull;
    const rtn_u32 dl = ok ? a.dl[i] : 0u;
    rtn_u32 w[16];
    bool need = false;
    if (ok) {
      rtn_cap_load64(p, w);
      rtn_v4u* h = reinterpret_cast<rtn_v4u*>(a.head + (rtn_u64)i * 64u);
#pragma unroll
      for (int k = 0; k < 4; ++k) h[k] = rtn_v4u{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
      a.dlen[i] = (unsigned short)dl;
      need = rtn_cap_need(w[3], w[4], dl);
    }
    const rtn_u64 m = __ballot(need);
    if (need) {
      rtn_cap_load64(p + 64u, w);
      rtn_v4u* e = reinterpret_cast<rtn_v4u*>(a.ext + (rtn_u64)(base + rows + (rtn_u32)__popcll(m & lane_lt)) * 64u);
#pragma unroll
      for (int k = 0; k < 4; ++k) e[k] = rtn_v4u{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
    }
    rows += (rtn_u32)__popcll(m);
  }
  if (lane == 0u) a.ext_chunk[c] = base;
}
