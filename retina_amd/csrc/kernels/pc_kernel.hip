// Packet-stage filter kernel for gfx950 (MI355X). One lane = one packet (mbuf), one wave = 64
// consecutive packets (a "group"). The filter compiler splices a tree-specialised `rtn_filter` at
// the RTN_FILTER marker below (the analogue of filtergen's generated `packet_continue`), and the
// whole translation unit is compiled once per subscription set (hiprtc at rtn_pc_create, or
// hipcc --genco ahead of time). It holds the packet-stage kernels -- rtn_pc_kernel_s64 for 64-byte
// slots, rtn_pc_kernel_split for 64-byte head slots + 64-byte ext slots (rtn_pc_kernel_splitc when
// the ext rows are compact), rtn_pc_kernel for any larger stride (a multiple of 64) -- and rtn_pd_kernel, the PacketDeliver filter (rtn_pd_run),
// whose generated tree (RTN_PD_FILTER marker) comes from the same program.
//
// Per packet it reproduces, bit for bit:
//   * Mbuf::get_data bounds (core/src/memory/mbuf.rs:125-135): offset < data_len && offset+size <= data_len
//   * Ethernet/Ipv4/Ipv6/Tcp/Udp::parse_from (core/src/protocols/packet/*.rs), including
//     802.1Q (header 18 B), 802.1ad -> no next header, IPv4 IHL without sanity checks,
//     no IPv6 extension headers
//   * the generated packet_continue (filtergen/src/packet_filter.rs) via rtn_filter
//   * L4Context::new (core/src/conntrack/pdu.rs:86-171) for forwarded packets
//   * Payload::from_mbuf guard (datatypes/src/packet.rs:18-29) for Payload deliveries
//
// Memory layout: slab = n slots of `stride` bytes (slot i holds the first
// min(data_len, stride) bytes of packet i), data_len = n x u16. Outputs are segmented per group
// (64 packets): record j of group g lives at [g*64 + j], counts are popcounts of the bitmaps.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

typedef unsigned int rtn_u32;
typedef unsigned long long rtn_u64;
typedef unsigned int rtn_v4u __attribute__((ext_vector_type(4)));

#ifndef RTN_DELIVER_WORDS
#define RTN_DELIVER_WORDS 0
#endif
#define RTN_DM_WORDS (RTN_DELIVER_WORDS > 0 ? RTN_DELIVER_WORDS : 1)
// groups per output chunk: 256 frames (RTN_CHUNK_FRAMES in retina_pc.h). A chunk is one wave's
// unit of work. In-process A/B with the interleaved record blocks and non-temporal stores (round
// 2, four boxes): 256-frame chunks cfg2 -3.1 to -3.6 % against 512 (128-frame chunks +4 %;
// 512-frame chunks in 128-thread blocks, +1 %). (Round 1, before those two: 512 beat 1024 by 6-9 %
// and 256 by 2-3 %.)
#define RTN_CHUNK_GROUPS 4u
// Record-block stores (records, rtn_conn_t, IPv6 addresses) are non-temporal: each line is
// written once and read by a later launch, so it streams past the caches (measured against plain
// stores, in-process on one box, with the interleaved record layout: cfg2 -1.1 %, cfg3 -14.5 %,
// cfg4 -10.4 %). The 8-B stores (bitmap words, delivery records) stay plain: the two half-line
// bitmap stores of a block merge in L2.
#define RTN_ST(p, v) __builtin_nontemporal_store((v), (p))
#define RTN_ST8(p, v) (*(p) = (v))
// 64-byte slots load coalesced + LDS transpose with non-temporal loads: every line is touched
// once, so streaming it past the caches costs nothing (per-lane loads of wider slots touch each
// line four times and stay plain).
#define RTN_LD_STREAM(p) __builtin_nontemporal_load(p)

struct rtn_l4rec {       // 16 B, the compacted L4Context of a forwarded packet (rtn_l4ctx_t)
  rtn_u32 w0;            // IPv4: u32::from(src Ipv4Addr); IPv6: source address bytes 0..3 (raw)
  rtn_u32 w1;            // IPv4: dst; IPv6: source address bytes 4..7 (raw)
  rtn_u32 ports;         // src_port | dst_port << 16
  rtn_u32 meta;          // offset >> 2 | udp << 6 | ipv6 << 7 | tcp flags << 8 | length << 16
};
// TCP records keep seq_no | ack_no << 32 in the seqack side stream (rtn_pc_out_t.seqack), ranked
// among the chunk's TCP records; IPv6 records the rest of their addresses (source bytes 8..15,
// destination) in addr6, 24 B each: no record carries a field that is always zero for its kind
// (UDP has no seq/ack; pdu.rs:66-84).

struct rtn_args {
  const unsigned char* slab;
  rtn_u64 stride;
  const unsigned short* dlen;
  rtn_u32 n;
  rtn_u32 flags;              // bit0: addr6, bit1: counters, bit2: conn, bit3: caller asserts data_len <= 64,
                              // bit4: compact ext rows (RTN_BATCH_EXT_COMPACT), bit5: seqack
  rtn_u64* pc_bm;             // [ceil(n/64)]  PacketContinue bit
  rtn_u64* fwd_bm;            // [ceil(n/64)]  PacketContinue && L4Context::new Ok
  rtn_l4rec* recs;            // [ceil(n/256)*256] at RTN_REC_INDEX
  unsigned char* addr6;       // [ceil(n/256)*256][24] (rtn_out_addr6_bytes) source bytes 8..15 and
                              // destination (raw) of the IPv6 records; rtn_flush6 pads a chunk's
                              // last store to whole 64-B requests, up to 2 entries past its last
                              // record (inside the chunk's 256)
  rtn_u64* dlv_bm;            // [ceil(n/64)]  any packet-level delivery
  rtn_u64* dlv_recs;          // [ceil(n/256)*256][RTN_DELIVER_WORDS] statement masks, ranked by dlv_bm per chunk
  rtn_u32* counters;          // [0] pc, [1] fwd, [2] dlv, [3] status, [4..5] bytes, [6..7] ignored bytes,
                              // [8] tcp, [9] udp (forwarded), [10..11] tcp bytes, [12..13] udp bytes
  const unsigned char* ext;   // split layout: bytes 64..127 of each frame (64-byte slots), or null
  rtn_u64* conn;              // optional [ceil(n/256)*256] rtn_conn_t, indexed like recs (flags bit2)
  rtn_u64* conn_dlv;          // [ceil(n/256)*256][RTN_CONN_WORDS] first-packet statement masks
  const rtn_u32* ext_chunk;   // flags bit4 (compact ext): row of each chunk's first needing frame
  rtn_u32 ext_rows;           // ... and the rows ext holds
  rtn_u32 cpw;                // compact split kernel: consecutive chunks per wave (1 or 2)
  rtn_u64* seqack;            // optional [ceil(n/256)*256] seq | ack << 32 of the TCP records, at
                              // RTN_REC_INDEX of their rank among the chunk's TCP records (bit5)
};

struct rtn_view {
  rtn_u32 dl;
  bool eth_ok, v4, v6, tcp, udp, l4ok, payload_ok;
  rtn_u32 l3off, l4off;
  rtn_u32 l3w[10];  // 40 bytes starting at the L3 offset (memory order, little-endian words)
  rtn_u32 l4w[5];   // 20 bytes starting at the L4 offset
};

#define RTN_B(w, off) (((w)[(off) >> 2] >> (((off) & 3u) * 8u)) & 0xffu)
#define rtn_l3_b(v, off) RTN_B((v).l3w, (off))
#define rtn_l4_b(v, off) RTN_B((v).l4w, (off))
#define rtn_l3_be16(v, off) ((rtn_l3_b(v, off) << 8) | rtn_l3_b(v, (off) + 1))
#define rtn_l4_be16(v, off) ((rtn_l4_b(v, off) << 8) | rtn_l4_b(v, (off) + 1))
#define rtn_l3_be32(v, off) ((rtn_l3_be16(v, off) << 16) | rtn_l3_be16(v, (off) + 2))
#define rtn_l4_be32(v, off) ((rtn_l4_be16(v, off) << 16) | rtn_l4_be16(v, (off) + 2))

// Statement-mask bit b of word w, set under a node's reach flag r (the generated filters' only
// form for delivery bits).
#define RTN_DM_SET(m, w, b, r) ((m)[w] |= (r) ? (1ull << (b)) : 0ull)
// ... and at a bit the lane computes (a range run's offset, codegen.cpp RangeRun).
#define RTN_DM_SETV(m, w, b, r) ((m)[w] |= (r) ? (1ull << (b)) : 0ull)
// Predicate constants of the generated filters are RTN_K(literal), and each filter body opens
// with RTN_KZ_DECL(view): the identity and nothing here (tools/variants.py redefines them to time
// constants that are not hoisted out of the group loop).
#ifndef RTN_K
#define RTN_K(c) (c)
#endif
#ifndef RTN_KZ_DECL
#define RTN_KZ_DECL(x)
#endif

//@@RTN_FILTER@@

#ifndef RTN_CONN_WORDS
#define RTN_CONN_WORDS 0
#endif
#define RTN_CM_WORDS (RTN_CONN_WORDS > 0 ? RTN_CONN_WORDS : 1)

// A forwarded frame as the first-packet filter sees it (FilterLayer::Packet may only test the
// connection-invariant fields: ast.rs:118-133). Addresses and ports are host-order values.
struct rtn_cview {
  bool v4, v6, tcp, udp;
  rtn_u32 src4, dst4;
  rtn_u32 s6[4], d6[4];  // big-endian words of the IPv6 addresses, most significant first
  rtn_u32 sport, dport;
};

//@@RTN_CONN_FILTER@@

// ConnId::new (conntrack/conn_id.rs:115-117) orders the endpoints by Rust's SocketAddr order: ip
// (as its big-endian integer), then port. Its hash (rtn_conn_hash in retina_pc.h) is MurmurHash3's
// 32-bit block and finaliser steps over the canonical words (max endpoint first).
__device__ __forceinline__ rtn_u32 rtn_rotl(rtn_u32 x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ rtn_u32 rtn_mix(rtn_u32 h, rtn_u32 k) {
  k *= 0xcc9e2d51u;
  k = rtn_rotl(k, 15);
  k *= 0x1b873593u;
  h ^= k;
  h = rtn_rotl(h, 13);
  return h * 5u + 0xe6546b64u;
}
__device__ __forceinline__ rtn_u32 rtn_fmix(rtn_u32 h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  return h ^ (h >> 16);
}

__device__ __forceinline__ rtn_u32 rtn_alignbyte2(rtn_u32 hi, rtn_u32 lo) {
  return __builtin_amdgcn_alignbyte(hi, lo, 2u);
}

// All-ones/zero lane mask hidden from the optimiser: without it LLVM folds the select trees
// below into a private array indexed dynamically (scratch + LDS round trips). With it every
// select is one v_bfi_b32.
__device__ __forceinline__ rtn_u32 rtn_mask(bool b) {
  rtn_u32 m = b ? 0xffffffffu : 0u;
  asm("" : "+v"(m));
  return m;
}
__device__ __forceinline__ rtn_u32 rtn_sel(rtn_u32 m, rtn_u32 a, rtn_u32 b) { return (a & m) | (b & ~m); }

// LDS visibility between lanes of one wave (LDS executes a wave's instructions in order; this
// keeps the compiler from reordering across the hand-off).
__device__ __forceinline__ void rtn_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NW>
__device__ __forceinline__ rtn_u32 rtn_w(const rtn_u32 (&w)[NW], int k) { return k < NW ? w[k] : 0u; }

// Every header offset the parse can produce is 2 mod 4: L3 starts at 14, 18 or 22
// (ethernet.rs:195-203) and the L4 offset adds 4*IHL or 40. So a view at offset o is
// alignbyte(w[o/4 + j + 1], w[o/4 + j], 2) for its words j.

// Wave-uniform offsets known at compile time: pure register selection (15 v_alignbyte).
template <int NW, int L3, int L4>
__device__ __forceinline__ void rtn_extract_c(const rtn_u32 (&w)[NW], rtn_view& v) {
  static_assert(L3 % 4 == 2 && L4 % 4 == 2, "offsets are 2 mod 4");
#pragma unroll
  for (int j = 0; j < 10; ++j) v.l3w[j] = rtn_alignbyte2(rtn_w(w, L3 / 4 + j + 1), rtn_w(w, L3 / 4 + j));
#pragma unroll
  for (int j = 0; j < 5; ++j) v.l4w[j] = rtn_alignbyte2(rtn_w(w, L4 / 4 + j + 1), rtn_w(w, L4 / 4 + j));
}

// Per-lane offsets: L3 at word 3 or 4, L4 window at word k = l4off/4 in [3, 19] through a
// barrel shifter (shifts 8, 4, 2, 1, then the lone k-3 == 16 case).
template <int NW>
__device__ __forceinline__ void rtn_extract_v(const rtn_u32 (&w)[NW], bool q, rtn_u32 l4off, rtn_view& v) {
  const rtn_u32 mq = rtn_mask(q);
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const rtn_u32 lo = rtn_sel(mq, rtn_w(w, 4 + j), rtn_w(w, 3 + j));
    const rtn_u32 hi = rtn_sel(mq, rtn_w(w, 5 + j), rtn_w(w, 4 + j));
    v.l3w[j] = rtn_alignbyte2(hi, lo);
  }
  const rtn_u32 m = (l4off >> 2) - 3u;  // 0..16
  const rtn_u32 m8 = rtn_mask(m & 8u), m4 = rtn_mask(m & 4u), m2 = rtn_mask(m & 2u), m1 = rtn_mask(m & 1u),
                m16 = rtn_mask(m & 16u);
  rtn_u32 s3[13], s2[9], s1[7], s0[6];
#pragma unroll
  for (int i = 0; i < 13; ++i) s3[i] = rtn_sel(m8, rtn_w(w, 11 + i), rtn_w(w, 3 + i));
#pragma unroll
  for (int i = 0; i < 9; ++i) s2[i] = rtn_sel(m4, s3[i + 4], s3[i]);
#pragma unroll
  for (int i = 0; i < 7; ++i) s1[i] = rtn_sel(m2, s2[i + 2], s2[i]);
#pragma unroll
  for (int i = 0; i < 6; ++i) s0[i] = rtn_sel(m1, s1[i + 1], s1[i]);
#pragma unroll
  for (int i = 0; i < 6; ++i) s0[i] = rtn_sel(m16, rtn_w(w, 19 + i), s0[i]);
#pragma unroll
  for (int j = 0; j < 5; ++j) v.l4w[j] = rtn_alignbyte2(s0[j + 1], s0[j]);
}

// Per-lane offsets from the four common stacks only: L3 at 14 or 18 (802.1Q) and L4 right after
// an IPv4 header without options or the IPv6 fixed header, so the L4 window starts at word
// 8 + q + 5 * v6. Every candidate view word is one alignbyte of two neighbours, then two selects
// (q, then v6) pick a lane's: 41 VALU against the barrel shifter's 81 (cfg3 / cfg4 mix all four
// in every wave).
template <int NW>
__device__ __forceinline__ void rtn_extract_q6(const rtn_u32 (&w)[NW], bool q, bool six, rtn_view& v) {
  const rtn_u32 mq = rtn_mask(q), m6 = rtn_mask(six);
  rtn_u32 x[16];  // x[i] = the view word at byte 4 * (i + 3) + 2
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = rtn_alignbyte2(rtn_w(w, i + 4), rtn_w(w, i + 3));
#pragma unroll
  for (int j = 0; j < 10; ++j) v.l3w[j] = rtn_sel(mq, x[j + 1], x[j]);
  rtn_u32 y[10];  // the L4 window of a lane without IPv6 (word 8 + q), then 5 words further
#pragma unroll
  for (int i = 0; i < 10; ++i) y[i] = rtn_sel(mq, x[i + 6], x[i + 5]);
#pragma unroll
  for (int j = 0; j < 5; ++j) v.l4w[j] = rtn_sel(m6, y[j + 5], y[j]);
}

// Parse one slot held in registers (w = its first 64 * NW/16 bytes).
template <int NW>
__device__ __forceinline__ void rtn_parse(const rtn_u32 (&w)[NW], rtn_u32 dl, rtn_view& v) {
  v.dl = dl;
  // Ethernet::parse_from: get_data::<EthernetHeader>(0) -> 0 < dl && 14 <= dl (ethernet.rs:170-183)
  v.eth_ok = dl >= 14u;
  const rtn_u32 et = __builtin_amdgcn_perm(0u, w[3], 0x0c0c0001u);  // bytes 12..13 big-endian
  const bool q = et == 0x8100u, ad = et == 0x88a8u;
  // EthernetHeader::length (ethernet.rs:195-203)
  v.l3off = q ? 18u : (ad ? 22u : 14u);
  // Ethernet::next_header (ethernet.rs:151-168): 0x8100 -> Dot1q at 14 (needs 18 <= dl)
  const rtn_u32 inner = __builtin_amdgcn_perm(0u, w[4], 0x0c0c0001u);  // bytes 16..17
  const bool has_next = q ? (dl >= 18u) : !ad;
  const rtn_u32 next = q ? inner : et;
  // Ipv4 / Ipv6::parse_from (ipv4.rs:174-191, ipv6.rs:116-133)
  v.v4 = v.eth_ok && has_next && next == 0x0800u && v.l3off + 20u <= dl;
  v.v6 = v.eth_ok && has_next && next == 0x86DDu && v.l3off + 40u <= dl;
  // IHL (byte l3off), IPv4 protocol (l3off + 9), IPv6 next header (l3off + 6)
  const rtn_u32 vihl = q ? (w[4] >> 16) & 0xffu : (w[3] >> 16) & 0xffu;
  const rtn_u32 ihl4 = (vihl & 0xfu) << 2;                     // Ipv4Header::length
  v.l4off = v.l3off + (v.v4 ? ihl4 : 40u);                    // next_header_offset
  const rtn_u32 proto = v.v4 ? (q ? w[6] >> 24 : w[5] >> 24) : (q ? w[6] & 0xffu : w[5] & 0xffu);
  const bool ip = v.v4 || v.v6;
  // Tcp / Udp::parse_from (tcp.rs:182-199, udp.rs:67-84)
  v.tcp = ip && proto == 6u && v.l4off < dl && v.l4off + 20u <= dl;
  v.udp = ip && proto == 17u && v.l4off < dl && v.l4off + 8u <= dl;
  // Header views. Only IP lanes read them, so when every IP lane of the wave has the same
  // (l3off, l4off) one constant-offset extraction serves the whole wave.
  const rtn_u32 key = v.l3off | (v.l4off << 8);
  const rtn_u64 ipm = __ballot(ip);
  const rtn_u32 src = ipm ? (rtn_u32)__builtin_ctzll(ipm) : 0u;
  const rtn_u32 ukey = __builtin_amdgcn_readlane(key, src);
  const bool uni = __ballot(ip && key != ukey) == 0ull;
  if (uni && ukey == (14u | (34u << 8))) {
    rtn_extract_c<NW, 14, 34>(w, v);         // Eth / IPv4 (IHL 5)
  } else if (uni && ukey == (18u | (38u << 8))) {
    rtn_extract_c<NW, 18, 38>(w, v);         // Eth / 802.1Q / IPv4 (IHL 5)
  } else if (uni && ukey == (14u | (54u << 8))) {
    rtn_extract_c<NW, 14, 54>(w, v);         // Eth / IPv6
  } else if (uni && ukey == (18u | (58u << 8))) {
    rtn_extract_c<NW, 18, 58>(w, v);         // Eth / 802.1Q / IPv6
  } else if (__ballot(ip && v.l4off != v.l3off + (v.v6 ? 40u : 20u)) == 0ull) {  // (802.1ad is never IP here)
    rtn_extract_q6<NW>(w, q, v.v6, v);     // {Eth, 802.1Q} x {IPv4 (IHL 5), IPv6}, per lane
  } else {
    rtn_extract_v<NW>(w, q, v.l4off, v);
  }
  // L4Context::new (pdu.rs:86-171): payload = ip length - headers, checked_sub
  const rtn_u32 thl = v.tcp ? ((rtn_l4_b(v, 12) & 0xf0u) >> 2) : 8u;  // TcpHeader::length / UDP 8
  const rtn_u32 iplen = v.v4 ? rtn_l3_be16(v, 2) : rtn_l3_be16(v, 4);  // total_length / payload_length
  const rtn_u32 sub = v.v4 ? ihl4 + thl : thl;
  v.l4ok = (v.tcp || v.udp) && iplen >= sub;
  const rtn_u32 off = v.l4off + thl, len = iplen - sub;
  // Payload::from_mbuf -> get_data_slice(offset, length) (mbuf.rs:109-120)
  v.payload_ok = v.l4ok && off < dl && off + len <= dl;
}

struct rtn_acc {
  rtn_u32 pc, fwd, dlv, status, tcp;
  rtn_u64 bytes, ignored;  // this lane's data_len sums: all frames / frames not accepted (rx_core.rs:129-141)
  rtn_u64 tcpb, udpb;      // ... forwarded TCP / UDP frames (process_packet, subscription/mod.rs:102-111)
};

// First 64 B of slot i. Lanes past n re-read the last slot (no branch, no zero fill); their
// data_len is forced to 0 so nothing parses.
__device__ __forceinline__ void rtn_load_lo(const rtn_args& a, rtn_u32 i, rtn_u32 (&w)[16], rtn_u32& dl) {
  const bool valid = i < a.n;
  const rtn_u32 ic = valid ? i : a.n - 1u;
  const rtn_v4u* slot = reinterpret_cast<const rtn_v4u*>(a.slab + (rtn_u64)ic * a.stride);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const rtn_v4u x = slot[k];
    w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
  }
  const rtn_u32 d = a.dlen[ic];
  dl = valid ? d : 0u;
}

// 64-byte slots, coalesced: the group's 4 KB arrive as four full-width 16-B-per-lane loads
// (lane l of load k holds quarter l%4 of slot 16k + l/4) and an LDS tile (one 64-B row per slot,
// 16-B quarters XOR-swizzled by (row >> 2) & 3: conflict-free ds_write_b128 / ds_read_b128)
// turns them back into one slot per lane.
#define RTN_XPITCH 16u  // one 64-B slot per row, 16-B chunks XOR-swizzled by (row >> 2) & 3
__device__ __forceinline__ void rtn_load_group(const rtn_args& a, rtn_u32 g, rtn_u32 lane, rtn_v4u (&q)[4], rtn_u32& dl) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const rtn_u32 slot = g * 64u + 16u * k + (lane >> 2);
    const rtn_u32 sc = slot < a.n ? slot : a.n - 1u;
    q[k] = RTN_LD_STREAM(reinterpret_cast<const rtn_v4u*>(a.slab + (rtn_u64)sc * 64u) + (lane & 3u));
  }
  const rtn_u32 i = g * 64u + lane;
  const rtn_u32 d = a.dlen[i < a.n ? i : a.n - 1u];
  dl = i < a.n ? d : 0u;
}
__device__ __forceinline__ void rtn_xpose(rtn_u32* tile, rtn_u32 lane, const rtn_v4u (&q)[4], rtn_u32 (&w)[16]) {
  rtn_wave_sync();
#pragma unroll
  for (int k = 0; k < 4; ++k)
    *reinterpret_cast<rtn_v4u*>(tile + (16u * k + (lane >> 2)) * RTN_XPITCH +
                                ((lane & 3u) ^ ((lane >> 4) & 3u)) * 4u) = q[k];
  rtn_wave_sync();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const rtn_v4u x = *reinterpret_cast<const rtn_v4u*>(tile + lane * RTN_XPITCH + ((j ^ (lane >> 2)) & 3u) * 4u);
    w[4 * j + 0] = x.x; w[4 * j + 1] = x.y; w[4 * j + 2] = x.z; w[4 * j + 3] = x.w;
  }
}

// Second 64 B of a slot, only for lanes whose headers can reach past byte 64 (IPv6, IPv4
// options, VLAN + options) and only when the slot holds them.
__device__ __forceinline__ bool rtn_need_hi(const rtn_u32 (&w)[16], rtn_u32 dl) {
  const rtn_u32 et = __builtin_amdgcn_perm(0u, w[3], 0x0c0c0001u);
  const bool q = et == 0x8100u;
  const rtn_u32 vihl = q ? (w[4] >> 16) & 0xffu : (w[3] >> 16) & 0xffu;
  const rtn_u32 inner = q ? __builtin_amdgcn_perm(0u, w[4], 0x0c0c0001u) : et;
  const rtn_u32 l4 = (q ? 18u : 14u) + (inner == 0x86DDu ? 40u : ((vihl & 0xfu) << 2));
  const bool is_ip = inner == 0x0800u || inner == 0x86DDu;
  return is_ip && dl > 64u && l4 + 20u > 64u;
}

// Wave-uniform state of the chunk a wave is working on. Outputs are dense per chunk of
// RTN_CHUNK_GROUPS groups (RTN_CHUNK_FRAMES = 64 * RTN_CHUNK_GROUPS frames): the chunk's k-th
// forwarded frame has record index chunk * RTN_CHUNK_FRAMES + k (likewise for deliveries).
struct rtn_chunk {
  rtn_u64 rec_base;         // chunk * RTN_CHUNK_FRAMES
  rtn_u32 nrec, nflushed;   // records produced / already stored in this chunk
  rtn_u32 ndlv;             // delivery records produced in this chunk
  rtn_u32 nv6, nv6flushed;  // IPv6 address records (addr6) produced / stored in this chunk
  rtn_u32 next;             // compact ext: needing frames of this chunk so far
  rtn_u32 ntcp, ntflushed;  // TCP records (seqack side stream) produced / stored in this chunk
  rtn_u64 my_pc, my_fwd, my_dlv;  // lane k holds group k's bitmap words until the chunk ends
};

// Record slot of the k-th forwarded frame of chunk c (RTN_REC_INDEX in retina_pc.h): a chunk's
// records leave in blocks of RTN_REC_BLOCK = 64, and block j of chunk c sits at block slot
// j * nchunks + c. The chunks' first blocks are then one dense stream, their second blocks the
// next, and so on: at cfg2's 25 % forwarded the record stores fill two dense streams instead of
// a quarter of every chunk-sized region (-4 % kernel time, in-process A/B on one box).
__device__ __forceinline__ rtn_u64 rtn_nchunks(rtn_u32 n) {
  return ((rtn_u64)n + 64u * RTN_CHUNK_GROUPS - 1u) / (64u * RTN_CHUNK_GROUPS);
}
#define RTN_RB 64u  // RTN_REC_BLOCK (retina_pc.h); the table and PacketDeliver kernels read 64-record blocks
__device__ __forceinline__ rtn_u64 rtn_rec_slot(rtn_u64 nch, rtn_u64 c, rtn_u32 k) {
  return ((rtn_u64)(k / RTN_RB) * nch + c) * RTN_RB + (k % RTN_RB);
}


// Records leave through a per-wave LDS ring of 128 records (2 KB) as whole 64-record blocks:
// full-width 16-B-per-lane stores (one record per lane), every line written whole; the IPv4 TCP
// records' seq/ack through a second ring of 128 8-B entries (1 KB), 64-entry blocks of 512 B.
#define RTN_RING 128u
#define RTN_FLUSH 64u

template <bool CONN>
__device__ __forceinline__ void rtn_flush(const rtn_args& a, const rtn_u64* ring, const rtn_u64* cring,
                                          const rtn_chunk& ch, rtn_u32 lane, rtn_u32 nrecs) {
  const rtn_u64 nch = rtn_nchunks(a.n);
  const rtn_u64 c = ch.rec_base / (64u * RTN_CHUNK_GROUPS);
  if (CONN) {
    // connection-stage entries (8 B) share the records' indices: same block, 128-B lines
    const rtn_u32 nc = ((nrecs + 1u) / 2u + 7u) & ~7u;
    // (a block of RTN_RB entries is RTN_RB / 2 lanes; a flush may span several blocks)
    const rtn_v4u* csrc = reinterpret_cast<const rtn_v4u*>(cring + (ch.nflushed & (RTN_RING - 1u)));
    rtn_v4u* cdst = reinterpret_cast<rtn_v4u*>(a.conn + rtn_rec_slot(nch, c, ch.nflushed));
    if (lane < nc) RTN_ST(cdst + (lane / (RTN_RB / 2u)) * nch * (RTN_RB / 2u) + lane % (RTN_RB / 2u), csrc[lane]);
  }
  // whole 64-B write requests only (4 records; TCC_EA0_WRREQ_64B is the memory-side write size): the
  // block starts line-aligned and the tail is padded with stale ring bytes into the chunk's unused
  // record space (a partial request costs a read-modify-write; padding to 128-B lines instead
  // writes 32 B more per stream and chunk on average: cfg4 +1 %, tools/variants.py pad64)
  const rtn_u32 nl = (nrecs + 3u) & ~3u;
  const rtn_v4u* src = reinterpret_cast<const rtn_v4u*>(ring) + (ch.nflushed & (RTN_RING - 1u));
  rtn_v4u* dst = reinterpret_cast<rtn_v4u*>(a.recs + rtn_rec_slot(nch, c, ch.nflushed));
  // (a block of RTN_RB records is RTN_RB lanes; a flush may span several blocks)
  if (lane < nl) RTN_ST(dst + (lane / RTN_RB) * nch * RTN_RB + lane % RTN_RB, src[lane]);
}

// seq/ack entries of TCP records [ntflushed, ntflushed + nent): 8 B each, two per lane, whole
// 64-B requests, 64-entry blocks at RTN_REC_INDEX of the chunk's TCP rank.
__device__ __forceinline__ void rtn_flush_t4(const rtn_args& a, const rtn_u64* ring4, const rtn_chunk& ch,
                                             rtn_u32 lane, rtn_u32 nent) {
  const rtn_u64 nch = rtn_nchunks(a.n);
  const rtn_u32 nl = ((nent + 1u) / 2u + 3u) & ~3u;
  const rtn_v4u* src = reinterpret_cast<const rtn_v4u*>(ring4 + (ch.ntflushed & (RTN_RING - 1u)));
  rtn_v4u* dst = reinterpret_cast<rtn_v4u*>(a.seqack + rtn_rec_slot(nch, ch.rec_base / (64u * RTN_CHUNK_GROUPS), ch.ntflushed));
  if (lane < nl) RTN_ST(dst + (lane / (RTN_RB / 2u)) * nch * (RTN_RB / 2u) + lane % (RTN_RB / 2u), src[lane]);
}

// IPv6 address records (24 B: source bytes 8..15, destination; the record holds source bytes
// 0..7) are dense per chunk over the chunk's forwarded IPv6 frames. Where IPv6 is common (the
// split / wide-slot kernels) they leave through their own per-wave LDS ring (96 entries, 2.25 KB)
// in whole 768-B blocks: scattered stores with holes between them cost about 4x their bytes in HBM
// time. A group adds up to 64 entries, so the ring holds them on top of the < 32 a group starts
// with. (A 128-entry ring of the 32-B entries held the block to 3 per CU by LDS: cfg4 0.2028 ->
// 0.1942 ms with 64, in-process A/B; a 64-entry ring needs a second store pass in IPv6-dense
// groups: cfg3 +2 %.)
#define RTN_RING6 96u
#define RTN_FLUSH6 32u

// Ring slot of position x < 2 * RTN_RING6 (a wave-uniform base below RTN_RING6 plus a lane's rank
// below 64): one subtract and a min instead of the modulo's quarter-rate multiplies.
__device__ __forceinline__ rtn_u32 rtn_ring6_at(rtn_u32 x) { return min(x, x - RTN_RING6); }

// Stores ring entries [nv6flushed, nv6flushed + nent) (nent <= 64; nv6flushed is a multiple
// of RTN_FLUSH6, so the run starts on a 16-B unit of the ring and of addr6), rounded up to whole
// 64-B write requests: a partial request costs a read-modify-write. Only a chunk's last store is
// partial, and its padding (stale ring bytes) lands in the chunk's unused addr6 space, as for the
// record blocks. The ring is 96 x 24 B = 144 16-B units, so a unit never straddles its wrap.
__device__ __forceinline__ void rtn_flush6(const rtn_args& a, const rtn_v4u* ring6, const rtn_chunk& ch, rtn_u32 lane,
                                           rtn_u32 nent) {
  const rtn_u32 nu = ((nent * 24u + 63u) & ~63u) / 16u;  // 16-B units, whole 64-B requests
  const rtn_u32 u0 = (ch.nv6flushed % RTN_RING6) * 24u / 16u;
  rtn_v4u* dst = reinterpret_cast<rtn_v4u*>(a.addr6 + (ch.rec_base + ch.nv6flushed) * 24u);
#pragma unroll
  for (rtn_u32 j = 0; j < 2u; ++j) {
    const rtn_u32 k = lane + 64u * j;
    if (k < nu) {
      const rtn_u32 u = u0 + k;
      RTN_ST(dst + k, ring6[min(u, u - RTN_RING6 * 24u / 16u)]);
    }
  }
}

// Everything after the slot's bytes arrived: parse, generated filter, L4Context, wave-level
// compaction of the outputs of group g (the k-th group of the current chunk).
template <int NW, bool STAGE6, bool CONN>
__device__ __forceinline__ void rtn_group(const rtn_args& a, rtn_u32 g, rtn_u32 k, rtn_u32 lane, rtn_u64 lane_lt,
                                          const rtn_u32 (&w)[NW], rtn_u32 dl, rtn_u64* ring, rtn_u64* cring,
                                          rtn_u64* ring4, rtn_v4u* ring6, rtn_chunk& ch, rtn_acc& acc) {
  const rtn_u32 i = g * 64u + lane;
  const bool valid = i < a.n;
  rtn_view v;
  rtn_parse<NW>(w, dl, v);
  // 64-byte slots: a packet whose headers run past byte 64 cannot be parsed from its slot
  // (RTN_STATUS_HDR_PAST_SLOT); with RTN_BATCH_DL_LE64 asserted no frame may be longer than its
  // slot (RTN_STATUS_DL_PAST_SLOT).
  if (NW == 16 && (v.v4 || v.v6) && dl > 64u && v.l4off + 20u > 64u) acc.status |= 1u;
  if (NW == 16 && (a.flags & 8u) && dl > 64u) acc.status |= 2u;
  rtn_u32 act = 0;
  rtn_u64 dm[RTN_DM_WORDS];
#pragma unroll
  for (int j = 0; j < RTN_DM_WORDS; ++j) dm[j] = 0ull;
  rtn_filter(v, act, dm);
  const bool pc = valid && (act & 1u) != 0u;
  const bool fwd = pc && v.l4ok;
  const rtn_u64 pcm = __ballot(pc);
  const rtn_u64 fwdm = __ballot(fwd);
  const rtn_u32 nfwd = (rtn_u32)__popcll(fwdm);
  acc.pc += (rtn_u32)__popcll(pcm);
  acc.fwd += nfwd;
  acc.bytes += dl;               // lanes past n have dl == 0
  acc.ignored += pc ? 0u : dl;
  acc.tcp += (rtn_u32)__popcll(__ballot(fwd && v.tcp));
  acc.tcpb += (fwd && v.tcp) ? dl : 0u;
  acc.udpb += (fwd && !v.tcp) ? dl : 0u;
  ch.my_pc = lane == k ? pcm : ch.my_pc;
  ch.my_fwd = lane == k ? fwdm : ch.my_fwd;
  // TCP records: their seq/ack go to the seqack side stream (when requested)
  const bool t4 = fwd && v.tcp && (a.flags & 32u);
  const rtn_u64 t4m = __ballot(t4);
  if (fwd) {
    const rtn_u32 r = ch.nrec + (rtn_u32)__popcll(fwdm & lane_lt);
    const bool tcp = v.tcp;
    const rtn_u32 thl = tcp ? ((rtn_l4_b(v, 12) & 0xf0u) >> 2) : 8u;
    const rtn_u32 ihl4 = (rtn_l3_b(v, 0) & 0xfu) << 2;
    const rtn_u32 iplen = v.v4 ? rtn_l3_be16(v, 2) : rtn_l3_be16(v, 4);
    const rtn_u32 len = iplen - (v.v4 ? ihl4 + thl : thl);
    const rtn_u32 off = v.l4off + thl;  // 2 mod 4: l4off is, thl is a multiple of 4
    const rtn_u32 meta = (off >> 2) | (tcp ? 0u : 64u) | (v.v6 ? 128u : 0u) |
                         ((tcp ? rtn_l4_b(v, 13) : 0u) << 8) | (len << 16);
    const rtn_u32 src4 = v.v4 ? rtn_l3_be32(v, 12) : 0u, dst4 = v.v4 ? rtn_l3_be32(v, 16) : 0u;
    const rtn_u32 ports = rtn_l4_be16(v, 0) | (rtn_l4_be16(v, 2) << 16);
    const rtn_u32 seq = tcp ? rtn_l4_be32(v, 4) : 0u, ack = tcp ? rtn_l4_be32(v, 8) : 0u;
    rtn_u64* rp = ring + (r & (RTN_RING - 1u)) * 2u;
    rp[0] = v.v4 ? ((rtn_u64)src4 | ((rtn_u64)dst4 << 32)) : ((rtn_u64)v.l3w[2] | ((rtn_u64)v.l3w[3] << 32));
    rp[1] = (rtn_u64)ports | ((rtn_u64)meta << 32);
    if (t4) ring4[(ch.ntcp + (rtn_u32)__popcll(t4m & lane_lt)) & (RTN_RING - 1u)] = (rtn_u64)seq | ((rtn_u64)ack << 32);
    if (CONN) {
      // Connection stage of the first packet (conntrack/mod.rs:80-169): ConnId, whether the frame
      // may open a connection (Conn::new_tcp / new_udp, conn/mod.rs:53-96) and the generated
      // packet_filter (ConnInfo::filter_first_packet, conn_info.rs:42-50) on this frame.
      rtn_cview c;
      c.v4 = v.v4;
      c.v6 = v.v6;
      c.tcp = tcp;
      c.udp = !tcp;
      c.src4 = src4;
      c.dst4 = dst4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c.s6[j] = v.v6 ? rtn_l3_be32(v, 8 + 4 * j) : 0u;
        c.d6[j] = v.v6 ? rtn_l3_be32(v, 24 + 4 * j) : 0u;
      }
      c.sport = ports & 0xffffu;
      c.dport = ports >> 16;
      rtn_u32 pdata = 0u, pterm = 0u;
      rtn_u64 cm[RTN_CM_WORDS];
#pragma unroll
      for (int j = 0; j < RTN_CM_WORDS; ++j) cm[j] = 0ull;
      rtn_conn_filter(c, pdata, pterm, cm);
      // src > dst in SocketAddr order (V4 vs V4 or V6 vs V6 here): ip first, then port
      bool gt = c.sport > c.dport;
      if (v.v6) {
#pragma unroll
        for (int j = 3; j >= 0; --j) {
          gt = c.s6[j] != c.d6[j] ? c.s6[j] > c.d6[j] : gt;
        }
      } else {
        gt = src4 != dst4 ? src4 > dst4 : gt;
      }
      rtn_u32 h = 0x5EEDu;
      if (v.v6) {
#pragma unroll
        for (int j = 0; j < 4; ++j) h = rtn_mix(h, gt ? c.s6[j] : c.d6[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) h = rtn_mix(h, gt ? c.d6[j] : c.s6[j]);
      } else {
        h = rtn_mix(h, gt ? src4 : dst4);
        h = rtn_mix(h, gt ? dst4 : src4);
      }
      const rtn_u32 pmax = gt ? c.sport : c.dport, pmin = gt ? c.dport : c.sport;
      h = rtn_mix(h, (pmax << 16) | pmin);
      h = rtn_mix(h, (tcp ? 6u : 17u) | (v.v6 ? 0x100u : 0u));
      h = rtn_fmix(h ^ (v.v6 ? 40u : 16u));
      const rtn_u32 fl = tcp ? rtn_l4_b(v, 13) : 0u;
      const bool creates = !tcp || ((fl & 0x02u) && !(fl & 0x10u) && !(fl & 0x04u));  // SYN, not ACK/RST
      rtn_u64 anyc = 0ull;
#pragma unroll
      for (int j = 0; j < RTN_CM_WORDS; ++j) anyc |= cm[j];
      const rtn_u32 info = (pdata & 0x1fffu) | ((pterm & 0x1fffu) << 13) | (creates ? 1u << 26 : 0u) |
                           (gt ? 1u << 27 : 0u) | (anyc ? 1u << 28 : 0u) | (v.v6 ? 1u << 29 : 0u) |
                           (tcp ? 0u : 1u << 30);
      cring[r & (RTN_RING - 1u)] = (rtn_u64)h | ((rtn_u64)info << 32);
#if RTN_CONN_WORDS > 0
#pragma unroll
      for (int j = 0; j < RTN_CONN_WORDS; ++j) RTN_ST8(a.conn_dlv + rtn_rec_slot(rtn_nchunks(a.n), ch.rec_base / (64u * RTN_CHUNK_GROUPS), r) * RTN_CONN_WORDS + j, cm[j]);
#endif
    }
  }
  ch.nrec += nfwd;
  ch.ntcp += (rtn_u32)__popcll(t4m);
  // IPv6 source/destination addresses, ranked among the chunk's forwarded IPv6 frames
  const bool six = fwd && v.v6 && (a.flags & 1u);
  const rtn_u64 m6 = __ballot(six);
  const rtn_u32 rank6 = (rtn_u32)__popcll(m6 & lane_lt), cnt6 = (rtn_u32)__popcll(m6);
  const rtn_u32 r6 = ch.nv6 + rank6;
  const rtn_u64 s0 = (rtn_u64)v.l3w[4] | ((rtn_u64)v.l3w[5] << 32), s1 = (rtn_u64)v.l3w[6] | ((rtn_u64)v.l3w[7] << 32),
                s2 = (rtn_u64)v.l3w[8] | ((rtn_u64)v.l3w[9] << 32);
  if (STAGE6) {
    // Fewer than RTN_FLUSH6 entries are pending when a group starts (every whole block is stored
    // below), so the group's at most 64 entries always find free slots in the 96-entry ring.
    if (six) {
      rtn_u64* e = reinterpret_cast<rtn_u64*>(ring6) + rtn_ring6_at(ch.nv6 % RTN_RING6 + rank6) * 3u;
      e[0] = s0;
      e[1] = s1;
      e[2] = s2;
    }
    ch.nv6 += cnt6;
    if (ch.nv6 - ch.nv6flushed >= RTN_FLUSH6) {  // every whole block pending (at most 64 entries)
      const rtn_u32 nb = (ch.nv6 - ch.nv6flushed) & ~(RTN_FLUSH6 - 1u);
      rtn_wave_sync();
      rtn_flush6(a, ring6, ch, lane, nb);
      ch.nv6flushed += nb;
      rtn_wave_sync();
    }
  } else {
    if (six) {
      rtn_u64* ap = reinterpret_cast<rtn_u64*>(a.addr6 + (ch.rec_base + r6) * 24u);
      ap[0] = s0;
      ap[1] = s1;
      ap[2] = s2;
    }
    ch.nv6 += cnt6;
  }
  // pending < RTN_FLUSH + 64 <= RTN_RING: at most one block per group and ring
  const bool fr = ch.nrec - ch.nflushed >= RTN_FLUSH, ft = ch.ntcp - ch.ntflushed >= RTN_FLUSH;
  if (fr || ft) {
    rtn_wave_sync();
    if (fr) {
      rtn_flush<CONN>(a, ring, cring, ch, lane, RTN_FLUSH);
      ch.nflushed += RTN_FLUSH;
    }
    if (ft) {
      rtn_flush_t4(a, ring4, ch, lane, RTN_FLUSH);
      ch.ntflushed += RTN_FLUSH;
    }
    rtn_wave_sync();
  }
#if RTN_DELIVER_WORDS > 0
  {
    rtn_u64 any = 0;
#pragma unroll
    for (int j = 0; j < RTN_DELIVER_WORDS; ++j) any |= dm[j];
    const bool d = valid && any != 0ull;
    const rtn_u64 dlvm = __ballot(d);
    ch.my_dlv = lane == k ? dlvm : ch.my_dlv;
    acc.dlv += (rtn_u32)__popcll(dlvm);
    if (d) {
      const rtn_u64 slot_i = ch.rec_base + ch.ndlv + (rtn_u32)__popcll(dlvm & lane_lt);
      // the frame index is implied by the record's rank in dlv_bm (like the L4Context records)
      rtn_u64* dp = a.dlv_recs + slot_i * RTN_DELIVER_WORDS;
#pragma unroll
      for (int j = 0; j < RTN_DELIVER_WORDS; ++j) RTN_ST8(dp + j, dm[j]);
    }
    ch.ndlv += (rtn_u32)__popcll(dlvm);
  }
#endif
}

// Chunk loop. Each wave takes chunks wave_g, wave_g + nwaves, ... and walks a chunk's groups in
// order. MODE: RTN_S64 (64-byte slots), RTN_SPLIT (64-byte slots + ext slab holding bytes
// 64..127 of every frame), RTN_SPLITC (the same with compact ext rows, RTN_BATCH_EXT_COMPACT),
// RTN_MONO (monolithic slots of any stride >= 64).
#define RTN_S64 0
#define RTN_SPLIT 1
#define RTN_MONO 2
#define RTN_SPLITC 3
template <int MODE, bool CONN>
__device__ __forceinline__ void rtn_run(const rtn_args& a) {
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 wave_g = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const rtn_u32 nwaves = (gridDim.x * blockDim.x) >> 6;
  const rtn_u32 nw = (a.n + 63u) >> 6;
  const rtn_u32 nchunks = (nw + RTN_CHUNK_GROUPS - 1u) / RTN_CHUNK_GROUPS;
  const rtn_u64 lane_lt = (lane == 0u) ? 0ull : (~0ull >> (64u - lane));
  constexpr bool slots64 = MODE != RTN_MONO;
  rtn_acc acc = {0u, 0u, 0u, 0u, 0u, 0ull, 0ull, 0ull, 0ull};
  __shared__ __attribute__((aligned(16))) rtn_u64 rtn_ring[4][RTN_RING * 2u];
  rtn_u64* ring = rtn_ring[threadIdx.x >> 6];
  __shared__ __attribute__((aligned(16))) rtn_u64 rtn_ring4[4][RTN_RING];  // TCP seq/ack
  rtn_u64* ring4 = rtn_ring4[threadIdx.x >> 6];
  __shared__ __attribute__((aligned(16))) rtn_u64 rtn_cring[4][CONN ? RTN_RING : 2u];  // connection-stage entries
  rtn_u64* cring = rtn_cring[threadIdx.x >> 6];
  constexpr bool stage6 = MODE != RTN_S64;  // 64-byte slots rarely forward IPv6 (only short UDP)
  __shared__ __attribute__((aligned(16))) rtn_v4u rtn_ring6[4][stage6 ? RTN_RING6 * 24u / 16u : 1u];
  rtn_v4u* ring6 = rtn_ring6[threadIdx.x >> 6];
  __shared__ __attribute__((aligned(16))) rtn_u32 rtn_tile[4][slots64 ? 64 * RTN_XPITCH : 1];
  rtn_u32* tile = rtn_tile[threadIdx.x >> 6];
  // The compact split kernel may walk cpw consecutive chunks per wave (the runtime picks 2 when
  // the kernel's registers allow fewer than 4 waves per SIMD: in-process A/B, cfg4 (3 waves)
  // 0.1772 -> 0.1722 ms with 2, cfg3 (4 waves) 0.2656 -> 0.2754 ms, so 1 there).
  const rtn_u32 cpw = MODE == RTN_SPLITC ? a.cpw : 1u;
  for (rtn_u32 cw = wave_g * cpw; cw < nchunks; cw += nwaves * cpw)
  for (rtn_u32 c = cw; c < cw + cpw && c < nchunks; ++c) {
    const rtn_u32 gb = c * RTN_CHUNK_GROUPS;
    const rtn_u32 ge = gb + RTN_CHUNK_GROUPS < nw ? gb + RTN_CHUNK_GROUPS : nw;
    rtn_chunk ch = {(rtn_u64)c * (64u * RTN_CHUNK_GROUPS), 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0ull, 0ull, 0ull};
    // compact ext: the chunk's first row, read once per chunk (its latency overlaps the first
    // group's loads; read per group it was a dependent round trip in every group)
    const rtn_u32 xrow0 = MODE == RTN_SPLITC ? a.ext_chunk[c] : 0u;
    // 64-byte slots without ext: the loads of the next two groups are issued before this group is
    // parsed, so two groups of loads are in flight per wave (one group ahead: cfg2 -2.2 %, two:
    // -0.4 % more, in-process A/B; with the split layout's dependent ext loads one group ahead
    // measured 5 % slower on cfg4 and is not used there)
    constexpr bool prefetch = MODE == RTN_S64;
    // (the connection-stage instance keeps one group ahead: two would take it to 134 VGPRs, 3
    // waves per SIMD)
    constexpr bool ahead2 = prefetch && !CONN;
    rtn_v4u qn[4], qn2[4];
    rtn_u32 dln = 0u, dln2 = 0u;
    if (prefetch) {
      rtn_load_group(a, gb, lane, qn, dln);
      if (ahead2 && gb + 1u < ge) rtn_load_group(a, gb + 1u, lane, qn2, dln2);
    }
    for (rtn_u32 g = gb; g < ge; ++g) {
      rtn_u32 lo[16], dl;
      if (prefetch) {
        rtn_v4u q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = qn[k];
        dl = dln;
        if (ahead2) {
#pragma unroll
          for (int k = 0; k < 4; ++k) qn[k] = qn2[k];
          dln = dln2;
          if (g + 2u < ge) rtn_load_group(a, g + 2u, lane, qn2, dln2);
        } else if (g + 1u < ge) {
          rtn_load_group(a, g + 1u, lane, qn, dln);
        }
        rtn_xpose(tile, lane, q, lo);
      } else if (slots64) {
        rtn_v4u q[4];
        rtn_load_group(a, g, lane, q, dl);
        rtn_xpose(tile, lane, q, lo);
      } else {
        rtn_load_lo(a, g * 64u + lane, lo, dl);
      }
      if (MODE == RTN_S64) {
        rtn_group<16, stage6, CONN>(a, g, g - gb, lane, lane_lt, lo, dl, ring, cring, ring4, ring6, ch, acc);
      } else {
        rtn_u32 w[32];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = lo[j];
#pragma unroll
        for (int j = 16; j < 32; ++j) w[j] = 0u;
        const bool need = rtn_need_hi(lo, dl);
        // compact ext (rtn_ext_needed in retina_pc.h): the row is the chunk's first row plus the
        // number of needing frames of the chunk before this one
        rtn_u64 row = (rtn_u64)g * 64u + lane;
        bool load = need;
        if (MODE == RTN_SPLITC) {
          const rtn_u64 nm = __ballot(need);
          row = (rtn_u64)xrow0 + ch.next + (rtn_u32)__popcll(nm & lane_lt);
          ch.next += (rtn_u32)__popcll(nm);
          load = need && row < a.ext_rows;
          if (need && !load) acc.status |= 4u;  // RTN_STATUS_EXT_ROWS
        }
        if (load) {
          // bytes 64..127: the ext slot (split layout) or the slot's second half (monolithic)
          const rtn_v4u* hi = MODE != RTN_MONO
                                  ? reinterpret_cast<const rtn_v4u*>(a.ext + row * 64u)
                                  : reinterpret_cast<const rtn_v4u*>(a.slab + (rtn_u64)(g * 64u + lane) * a.stride) + 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const rtn_v4u x = hi[j];
            w[16 + 4 * j + 0] = x.x; w[16 + 4 * j + 1] = x.y; w[16 + 4 * j + 2] = x.z; w[16 + 4 * j + 3] = x.w;
          }
        }
        rtn_group<32, stage6, CONN>(a, g, g - gb, lane, lane_lt, w, dl, ring, cring, ring4, ring6, ch, acc);
      }
    }
    // chunk epilogue: the partial last record block, then one store per bitmap for the chunk
    rtn_wave_sync();
    rtn_flush<CONN>(a, ring, cring, ch, lane, ch.nrec - ch.nflushed);
    if (ch.ntcp != ch.ntflushed) rtn_flush_t4(a, ring4, ch, lane, ch.ntcp - ch.ntflushed);
    if (stage6) rtn_flush6(a, ring6, ch, lane, ch.nv6 - ch.nv6flushed);
    rtn_wave_sync();
    if (lane < ge - gb) {
      RTN_ST8(a.pc_bm + gb + lane, ch.my_pc);
      RTN_ST8(a.fwd_bm + gb + lane, ch.my_fwd);
#if RTN_DELIVER_WORDS > 0
      RTN_ST8(a.dlv_bm + gb + lane, ch.my_dlv);
#endif
    }
  }
  // one set of atomics per wave: status bits always (RTN_STATUS_*), totals when requested
  const rtn_u32 st = (__ballot((acc.status & 1u) != 0u) ? 1u : 0u) | (__ballot((acc.status & 2u) != 0u) ? 2u : 0u) |
                     (__ballot((acc.status & 4u) != 0u) ? 4u : 0u);
  if (lane == 0u && st) atomicOr(&a.counters[3], st);
  if (!(a.flags & 2u)) return;
  rtn_u64 bytes = acc.bytes, ignored = acc.ignored, tcpb = acc.tcpb, udpb = acc.udpb;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    bytes += __shfl_xor(bytes, off);
    ignored += __shfl_xor(ignored, off);
    tcpb += __shfl_xor(tcpb, off);
    udpb += __shfl_xor(udpb, off);
  }
  if (lane == 0u) {
    if (acc.pc) atomicAdd(&a.counters[0], acc.pc);
    if (acc.fwd) atomicAdd(&a.counters[1], acc.fwd);
    if (acc.dlv) atomicAdd(&a.counters[2], acc.dlv);
    if (bytes) atomicAdd(reinterpret_cast<unsigned long long*>(a.counters + 4), bytes);
    if (ignored) atomicAdd(reinterpret_cast<unsigned long long*>(a.counters + 6), ignored);
    if (acc.tcp) atomicAdd(&a.counters[8], acc.tcp);
    if (acc.fwd - acc.tcp) atomicAdd(&a.counters[9], acc.fwd - acc.tcp);
    if (tcpb) atomicAdd(reinterpret_cast<unsigned long long*>(a.counters + 10), tcpb);
    if (udpb) atomicAdd(reinterpret_cast<unsigned long long*>(a.counters + 12), udpb);
  }
}

// One instance per slot layout, each with and without the connection stage (rtn_pc_out_t.conn):
// compiled out, the stage's code and its LDS ring no longer hold registers and LDS the plain
// packet stage needs (cfg4's compact split kernel: 134 -> 121 VGPRs, 3 -> 4 waves per SIMD, SGPR
// spills 68 -> 40).
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel(rtn_args a) { rtn_run<RTN_MONO, false>(a); }
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel_s64(rtn_args a) { rtn_run<RTN_S64, false>(a); }
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel_split(rtn_args a) { rtn_run<RTN_SPLIT, false>(a); }
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel_splitc(rtn_args a) { rtn_run<RTN_SPLITC, false>(a); }
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel_conn(rtn_args a) { rtn_run<RTN_MONO, true>(a); }
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel_s64_conn(rtn_args a) { rtn_run<RTN_S64, true>(a); }
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel_split_conn(rtn_args a) { rtn_run<RTN_SPLIT, true>(a); }
extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel_splitc_conn(rtn_args a) { rtn_run<RTN_SPLITC, true>(a); }

// ---------------------------------------------------------------------------------------------
// PacketDeliver filter (rtn_pd_run): the generated `packet_deliver` (filtergen/src/lib.rs:357-362,
// deliver_filter.rs) for the forwarded frames of connections that hold the PacketDeliver action
// (ConnInfo::update_sdata, conntrack/conn/conn_info.rs:70-75). Runs after the connection lookup:
// a frame takes part if its connection predates the batch (RTN_CT_HIT | RTN_CT_PRIOR) and the
// host's per-slot state says PacketDeliver is on. Packet predicates test the frame's own L4Context
// (the deliver tree holds only connection-invariant packet fields: ptree.rs:406-415); service and
// session predicates read the connection's facts, which the host keeps per slot.
#ifndef RTN_PD_STMTS
#define RTN_PD_STMTS 0
#endif
#ifndef RTN_PD_FACTS
#define RTN_PD_FACTS 0
#endif
#define RTN_PD_S (RTN_PD_STMTS > 0 ? RTN_PD_STMTS : 1)
#define RTN_PD_F (RTN_PD_FACTS > 0 ? RTN_PD_FACTS : 1)

//@@RTN_PD_FILTER@@

struct rtn_pd_args {
  const rtn_u64* fwd_bm;
  const rtn_l4rec* recs;
  const unsigned char* addr6;
  const rtn_u64* conn;         // rtn_conn_t, indexed like recs (its IPv6 bit gives the addr6 rank)
  const rtn_u32* ct;           // rtn_ct_entry_t {slot, status}, indexed like recs
  const unsigned short* dlen;
  const rtn_u32* state;        // [state_slots][1 + RTN_PD_FACTS]: flags (bit 0: PacketDeliver), facts
  rtn_u32 state_slots;
  rtn_u32 n;
  rtn_u32* counts;             // [record][RTN_PD_S]: written for delivered frames only
  rtn_u64* pd_bm;              // [ceil(n/64)]: the frame has at least one delivery
};

// groups (64 frames) per wave (1, 2, 4 and 8 measured within 3 % on cfg2: 0.40-0.41 ms; 1 is
// the fastest)
#define RTN_PD_GPW 1u
#define RTN_PD_THREADS (64u * RTN_CHUNK_GROUPS / RTN_PD_GPW)

// One block per chunk, RTN_PD_GPW 64-frame groups per wave, one lane per frame of each.
extern "C" __global__ void __launch_bounds__(RTN_PD_THREADS) rtn_pd_kernel(rtn_pd_args a) {
  constexpr rtn_u32 G = RTN_PD_GPW;
  __shared__ rtn_u32 v6n[RTN_CHUNK_GROUPS];
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const rtn_u32 ch = blockIdx.x;
  const rtn_u32 nw = (a.n + 63u) >> 6;
  const rtn_u64 lane_lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  // the chunk's bitmap words: lane j < RTN_CHUNK_GROUPS holds word j; pre[j] = records before group j
  const rtn_u32 gj = ch * RTN_CHUNK_GROUPS + (lane & (RTN_CHUNK_GROUPS - 1u));
  const rtn_u64 wj = gj < nw ? a.fwd_bm[gj] : 0ull;
  const rtn_u32 pop = (rtn_u32)__popcll(wj);
  // (q = w * G + u is not a compile-time index: accumulate per group instead of indexing an array)
  rtn_u32 pre[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) pre[u] = 0u;
#pragma unroll
  for (rtn_u32 j = 0; j < RTN_CHUNK_GROUPS; ++j) {
    const rtn_u32 pj = __shfl(pop, (int)j);
#pragma unroll
    for (rtn_u32 u = 0; u < G; ++u) pre[u] += j < w * G + u ? pj : 0u;
  }
  bool has[G];
  rtn_u64 r[G], cv[G];
  rtn_u32 rec[G][4], slot[G], st[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    const rtn_u32 q = w * G + u;
    const rtn_u64 word = __shfl(wj, (int)q);
    has[u] = ch * RTN_CHUNK_GROUPS + q < nw && ((word >> lane) & 1ull);
    r[u] = rtn_rec_slot(rtn_nchunks(a.n), ch, pre[u] + (rtn_u32)__popcll(word & lane_lt));
#pragma unroll
    for (int j = 0; j < 4; ++j) rec[u][j] = 0u;
    slot[u] = 0xFFFFFFFFu;
    st[u] = 0u;
    cv[u] = 0ull;
    if (has[u]) {
      // 16 B per forwarded frame; the 16-B record only for frames that take part (below)
      const rtn_u64 e = __builtin_nontemporal_load(reinterpret_cast<const rtn_u64*>(a.ct) + r[u]);
      slot[u] = (rtn_u32)e;
      st[u] = (rtn_u32)(e >> 32);
      cv[u] = __builtin_nontemporal_load(a.conn + r[u]);
    }
  }
  // the connection's state row: flags and facts in one go (RTN_CT_HIT | RTN_CT_PRIOR only)
  bool on[G];
  rtn_u32 sv[G][1 + RTN_PD_F];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    on[u] = has[u] && st[u] == (1u | 0x100u) && slot[u] < a.state_slots;
#pragma unroll
    for (int j = 0; j <= RTN_PD_F; ++j) sv[u][j] = 0u;
    if (on[u]) {
      const rtn_u32* sp = a.state + (rtn_u64)slot[u] * (1u + RTN_PD_FACTS);
#pragma unroll
      for (int j = 0; j <= RTN_PD_FACTS; ++j) sv[u][j] = sp[j];
      const rtn_u64* rp = reinterpret_cast<const rtn_u64*>(a.recs + r[u]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const rtn_u64 x = __builtin_nontemporal_load(rp + j);
        rec[u][2 * j] = (rtn_u32)x;
        rec[u][2 * j + 1] = (rtn_u32)(x >> 32);
      }
    }
  }
  // IPv6 records are dense per chunk in addr6: rank among the chunk's IPv6 records
  rtn_u64 m6[G];
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    m6[u] = __ballot(has[u] && ((cv[u] >> 61) & 1ull));  // RTN_CONN_IPV6
    if (lane == 0u) v6n[w * G + u] = (rtn_u32)__popcll(m6[u]);
  }
  __syncthreads();
#pragma unroll
  for (rtn_u32 u = 0; u < G; ++u) {
    const rtn_u32 q = w * G + u;
    const bool v6 = (m6[u] >> lane) & 1ull;
    rtn_u32 cnt[RTN_PD_S];
#pragma unroll
    for (int j = 0; j < RTN_PD_S; ++j) cnt[j] = 0u;
    bool dl = false;
    if (on[u] && (sv[u][0] & 1u)) {
      rtn_u32 p6 = 0u;
#pragma unroll
      for (rtn_u32 j = 0; j < RTN_CHUNK_GROUPS; ++j) p6 += j < q ? v6n[j] : 0u;
      const rtn_u64 r6 = (rtn_u64)ch * (64u * RTN_CHUNK_GROUPS) + p6 + (rtn_u32)__popcll(m6[u] & lane_lt);
      rtn_cview c;
      c.v6 = v6;
      c.v4 = !v6;
      c.udp = (rec[u][3] >> 6) & 1u;
      c.tcp = !c.udp;
      c.src4 = v6 ? 0u : rec[u][0];  // (an IPv6 record holds its source's first 8 bytes there)
      c.dst4 = v6 ? 0u : rec[u][1];
      c.sport = rec[u][2] & 0xffffu;
      c.dport = rec[u][2] >> 16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c.s6[j] = 0u;
        c.d6[j] = 0u;
      }
      if (v6) {  // source bytes 0..7 in the record, 8..15 and the destination in addr6 (24 B)
        const rtn_u32* ap = reinterpret_cast<const rtn_u32*>(a.addr6 + r6 * 24u);
        c.s6[0] = __builtin_bswap32(rec[u][0]);
        c.s6[1] = __builtin_bswap32(rec[u][1]);
        c.s6[2] = __builtin_bswap32(ap[0]);
        c.s6[3] = __builtin_bswap32(ap[1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) c.d6[j] = __builtin_bswap32(ap[2 + j]);
      }
      // Payload::from_mbuf (datatypes/src/packet.rs:18-29): get_data_slice(offset, length)
      const rtn_u32 dlen = a.dlen[(ch * RTN_CHUNK_GROUPS + q) * 64u + lane];
      const rtn_u32 off = ((rec[u][3] & 0x3fu) << 2) | 2u, len = rec[u][3] >> 16;
      const bool pok = off < dlen && off + len <= dlen;
      rtn_pd_filter(c, pok, &sv[u][1], cnt);
#pragma unroll
      for (int j = 0; j < RTN_PD_S; ++j) dl = dl || cnt[j] != 0u;
    }
    const rtn_u64 mb = __ballot(dl);
    if (lane == 0u && ch * RTN_CHUNK_GROUPS + q < nw) a.pd_bm[ch * RTN_CHUNK_GROUPS + q] = mb;
    if (dl) {
#pragma unroll
      for (int j = 0; j < RTN_PD_S; ++j) {
// written once, read by the host or a later launch: non-temporal (cfg2 PacketDeliver
        // 0.4387 -> 0.4177 ms, in-process A/B on one box)
        __builtin_nontemporal_store(cnt[j], a.counts + r[u] * RTN_PD_S + j);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// accepted_idx / n_accepted (rtn_pc_index): the frame indices of a bitmap's set bits
// in frame order, their count, and each chunk's first position in that order. Three launches: a
// per-block popcount over RTN_IDX_WORDS bitmap words, an exclusive scan of the block sums in one
// block, then per block a wave-level scan that writes the indices (lane = frame bit, one coalesced
// store per word) and the chunk bases.
#define RTN_IDX_WORDS 4096u  // bitmap words per block (4 waves x 1024)

struct rtn_idx_args {
  const rtn_u64* bm;
  rtn_u32 n;          // frames
  rtn_u32 nblocks;    // ceil(words / RTN_IDX_WORDS)
  rtn_u32* block_sum; // [nblocks]: set bits per block, then their exclusive prefix
  rtn_u32* idx;       // [set bits]
  rtn_u32* n_set;     // [1]
  rtn_u32* chunk_base;  // optional [nchunks + 1]
};

__device__ __forceinline__ rtn_u64 rtn_idx_word(const rtn_idx_args& a, rtn_u32 w) {
  const rtn_u32 nw = (a.n + 63u) >> 6;
  if (w >= nw) return 0ull;
  const rtn_u64 x = a.bm[w];
  const rtn_u32 tail = a.n & 63u;  // bits past n are not frames
  return (w == nw - 1u && tail) ? x & ((1ull << tail) - 1ull) : x;
}

extern "C" __global__ void __launch_bounds__(256) rtn_idx_count(rtn_idx_args a) {
  __shared__ rtn_u32 part[4];
  const rtn_u32 w0 = blockIdx.x * RTN_IDX_WORDS;
  rtn_u32 s = 0;
  for (rtn_u32 j = threadIdx.x; j < RTN_IDX_WORDS; j += 256u) s += (rtn_u32)__popcll(rtn_idx_word(a, w0 + j));
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63u) == 0u) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0u) a.block_sum[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// one block of 1024 threads: exclusive prefix of the block sums in place, total to n_set
extern "C" __global__ void __launch_bounds__(1024) rtn_idx_scan(rtn_idx_args a) {
  __shared__ rtn_u32 wsum[16];
  const rtn_u32 t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const rtn_u32 per = (a.nblocks + 1023u) / 1024u;  // consecutive block sums per thread
  rtn_u32 local = 0;
  for (rtn_u32 j = 0; j < per; ++j) {
    const rtn_u32 b = t * per + j;
    local += b < a.nblocks ? a.block_sum[b] : 0u;
  }
  rtn_u32 incl = local;  // inclusive scan within the wave
  for (rtn_u32 off = 1; off < 64u; off <<= 1) {
    const rtn_u32 y = __shfl_up(incl, off);
    incl += lane >= off ? y : 0u;
  }
  if (lane == 63u) wsum[wv] = incl;
  __syncthreads();
  rtn_u32 before = 0;
  for (rtn_u32 k = 0; k < wv; ++k) before += wsum[k];
  rtn_u32 run = before + incl - local;  // exclusive prefix of this thread's first block
  for (rtn_u32 j = 0; j < per; ++j) {
    const rtn_u32 b = t * per + j;
    if (b < a.nblocks) {
      const rtn_u32 v = a.block_sum[b];
      a.block_sum[b] = run;
      run += v;
    }
  }
  if (t == 1023u) {
    a.n_set[0] = run;
    if (a.chunk_base) a.chunk_base[(a.n + RTN_CHUNK_GROUPS * 64u - 1u) / (RTN_CHUNK_GROUPS * 64u)] = run;
  }
}

extern "C" __global__ void __launch_bounds__(256) rtn_idx_write(rtn_idx_args a) {
  __shared__ rtn_u32 wtot[4];
  const rtn_u32 lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const rtn_u64 lane_lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  const rtn_u32 wbeg = blockIdx.x * RTN_IDX_WORDS + wv * (RTN_IDX_WORDS / 4u);  // this wave's 1024 words
  // this wave's total, then the waves before it
  rtn_u32 s = 0;
  for (rtn_u32 j = lane; j < RTN_IDX_WORDS / 4u; j += 64u) s += (rtn_u32)__popcll(rtn_idx_word(a, wbeg + j));
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0u) wtot[wv] = s;
  __syncthreads();
  rtn_u32 base = a.block_sum[blockIdx.x];
  for (rtn_u32 k = 0; k < wv; ++k) base += wtot[k];
  const rtn_u32 nw = (a.n + 63u) >> 6;
  for (rtn_u32 j0 = 0; j0 < RTN_IDX_WORDS / 4u && wbeg + j0 < nw; j0 += 64u) {
    const rtn_u64 mine = rtn_idx_word(a, wbeg + j0 + lane);  // lane l holds word j0 + l
    const rtn_u32 c = (rtn_u32)__popcll(mine);
    rtn_u32 incl = c;
    for (rtn_u32 off = 1; off < 64u; off <<= 1) {
      const rtn_u32 y = __shfl_up(incl, off);
      incl += lane >= off ? y : 0u;
    }
    const rtn_u32 wd = wbeg + j0 + lane;
    if (a.chunk_base && wd < nw && (wd % RTN_CHUNK_GROUPS) == 0u) a.chunk_base[wd / RTN_CHUNK_GROUPS] = base + incl - c;
    for (rtn_u32 l = 0; l < 64u && wbeg + j0 + l < nw; ++l) {
      const rtn_u64 word = __shfl(mine, (int)l);
      const rtn_u32 wb = base + __shfl(incl - c, (int)l);
      if ((word >> lane) & 1ull) a.idx[wb + (rtn_u32)__popcll(word & lane_lt)] = (wbeg + j0 + l) * 64u + lane;
    }
    base += __shfl(incl, 63);
  }
}
