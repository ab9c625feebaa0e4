// Packet-stage filter kernel for gfx950 (MI355X). One lane = one packet (mbuf), one wave = 64
// consecutive packets. The filter compiler splices a tree-specialised `rtn_filter` at the
// RTN_FILTER marker below (the analogue of filtergen's generated `packet_continue`), and the
// whole translation unit is compiled once per subscription set (hiprtc at rtn_pc_create, or
// hipcc --genco ahead of time).
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
// min(data_len, stride) bytes of packet i), data_len = n x u16. Outputs are segmented per wave
// (64 packets): record j of wave w lives at [w*64 + j], counts are popcounts of the bitmaps.
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

struct rtn_l4rec {       // 32 B, the compacted L4Context of a forwarded packet
  rtn_u32 pkt_idx;       // index of the packet in the batch
  rtn_u32 src_ip4;       // u32::from(Ipv4Addr) (0 for IPv6; addresses in addr6 side array)
  rtn_u32 dst_ip4;
  rtn_u32 ports;         // src_port | dst_port << 16
  rtn_u32 seq_no;
  rtn_u32 ack_no;
  rtn_u32 off_len;       // offset | length << 16
  rtn_u32 proto_flags;   // proto | flags << 8 | ip_version << 16
};

struct rtn_args {
  const unsigned char* slab;
  rtn_u64 stride;
  const unsigned short* dlen;
  rtn_u32 n;
  rtn_u32 flags;              // bit0: write addr6 side array, bit1: accumulate counters
  rtn_u64* pc_bm;             // [ceil(n/64)]  PacketContinue bit
  rtn_u64* fwd_bm;            // [ceil(n/64)]  PacketContinue && L4Context::new Ok
  rtn_l4rec* recs;            // [ceil(n/64)*64]
  unsigned char* addr6;       // [ceil(n/64)*64][32] (src, dst) raw bytes, IPv6 records only
  rtn_u64* dlv_bm;            // [ceil(n/64)]  any packet-level delivery
  rtn_u64* dlv_recs;          // [ceil(n/64)*64][1 + RTN_DELIVER_WORDS]  (pkt_idx, statement mask words)
  rtn_u32* counters;          // [0] pc, [1] fwd, [2] dlv, [3] status bits
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

//@@RTN_FILTER@@

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

// Parse one slot held in registers (w[0..31] = first 128 bytes; upper half zero unless loaded).
__device__ __forceinline__ void rtn_parse(const rtn_u32 (&w)[32], rtn_u32 dl, rtn_view& v) {
  v.dl = dl;
  // Ethernet::parse_from: get_data::<EthernetHeader>(0) -> 0 < dl && 14 <= dl (ethernet.rs:170-183)
  v.eth_ok = dl >= 14u;
  const rtn_u32 et = ((w[3] & 0xffu) << 8) | ((w[3] >> 8) & 0xffu);
  const bool q = et == 0x8100u, ad = et == 0x88a8u;
  // EthernetHeader::length (ethernet.rs:195-203)
  v.l3off = q ? 18u : (ad ? 22u : 14u);
  // Ethernet::next_header (ethernet.rs:151-168): 0x8100 -> Dot1q at 14 (needs 18 <= dl)
  const rtn_u32 inner = ((w[4] & 0xffu) << 8) | ((w[4] >> 8) & 0xffu);
  const bool has_next = q ? (dl >= 18u) : !ad;
  const rtn_u32 next = q ? inner : et;
  // Ipv4 / Ipv6::parse_from (ipv4.rs:174-191, ipv6.rs:116-133)
  v.v4 = v.eth_ok && has_next && next == 0x0800u && v.l3off + 20u <= dl;
  v.v6 = v.eth_ok && has_next && next == 0x86DDu && v.l3off + 40u <= dl;
  const rtn_u32 mq = rtn_mask(q);
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const rtn_u32 lo = rtn_sel(mq, w[4 + j], w[3 + j]);
    const rtn_u32 hi = rtn_sel(mq, w[5 + j], w[4 + j]);
    v.l3w[j] = rtn_alignbyte2(hi, lo);
  }
  const rtn_u32 ihl4 = (rtn_l3_b(v, 0) & 0xfu) << 2;           // Ipv4Header::length
  v.l4off = v.l3off + (v.v4 ? ihl4 : 40u);                    // next_header_offset
  const rtn_u32 proto = v.v4 ? rtn_l3_b(v, 9) : rtn_l3_b(v, 6);
  const bool ip = v.v4 || v.v6;
  // Tcp / Udp::parse_from (tcp.rs:182-199, udp.rs:67-84)
  v.tcp = ip && proto == 6u && v.l4off < dl && v.l4off + 20u <= dl;
  v.udp = ip && proto == 17u && v.l4off < dl && v.l4off + 8u <= dl;
  // 20 bytes at l4off (even, 14..78): barrel-shift the word window, then realign by 2 bytes.
  const rtn_u32 m = ((v.l4off >> 2) - 3u) & 31u;
  rtn_u32 s4[21], s3[13], s2[9], s1[7], s0[6];
  const rtn_u32 m4 = rtn_mask(m & 16u), m3 = rtn_mask(m & 8u), m2 = rtn_mask(m & 4u), m1 = rtn_mask(m & 2u),
                m0 = rtn_mask(m & 1u), mph = rtn_mask((v.l4off & 2u) != 0u);
#pragma unroll
  for (int i = 0; i < 21; ++i) {
    const rtn_u32 a0 = (3 + i < 32) ? w[3 + i] : 0u;
    const rtn_u32 a1 = (19 + i < 32) ? w[19 + i] : 0u;
    s4[i] = rtn_sel(m4, a1, a0);
  }
#pragma unroll
  for (int i = 0; i < 13; ++i) s3[i] = rtn_sel(m3, s4[i + 8], s4[i]);
#pragma unroll
  for (int i = 0; i < 9; ++i) s2[i] = rtn_sel(m2, s3[i + 4], s3[i]);
#pragma unroll
  for (int i = 0; i < 7; ++i) s1[i] = rtn_sel(m1, s2[i + 2], s2[i]);
#pragma unroll
  for (int i = 0; i < 6; ++i) s0[i] = rtn_sel(m0, s1[i + 1], s1[i]);
#pragma unroll
  for (int j = 0; j < 5; ++j) v.l4w[j] = rtn_sel(mph, rtn_alignbyte2(s0[j + 1], s0[j]), s0[j]);
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
  rtn_u32 pc, fwd, dlv, status;
};

// Load the first 64 B of frame i's slot (the only part a 64-B-stride batch has).
__device__ __forceinline__ void rtn_load_lo(const rtn_args& a, rtn_u32 i, bool valid, rtn_u32 (&lo)[16], rtn_u32& dl) {
  dl = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) lo[k] = 0u;
  if (valid) {
    const uint4* slot = reinterpret_cast<const uint4*>(a.slab + (rtn_u64)i * a.stride);
    dl = a.dlen[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 x = slot[k];
      lo[4 * k + 0] = x.x; lo[4 * k + 1] = x.y; lo[4 * k + 2] = x.z; lo[4 * k + 3] = x.w;
    }
  }
}

// Coalesced variant: 4 lanes per slot read the slot's first 64 B (each wave instruction covers
// 16 slots), then a wave-private LDS tile (80-B pitch: conflict-free ds_read_b128) turns it back
// into one frame per lane.
#define RTN_XPITCH 20u  // dwords per frame in the LDS tile
__device__ __forceinline__ void rtn_load_raw(const rtn_args& a, rtn_u32 wv, rtn_u32 lane, uint4 (&q)[4], rtn_u32& dl) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const rtn_u32 p = wv * 64u + 16u * k + (lane >> 2);
    q[k] = make_uint4(0u, 0u, 0u, 0u);
    if (p < a.n) q[k] = *reinterpret_cast<const uint4*>(a.slab + (rtn_u64)p * a.stride + (lane & 3u) * 16u);
  }
  const rtn_u32 i = wv * 64u + lane;
  dl = i < a.n ? (rtn_u32)a.dlen[i] : 0u;
}
__device__ __forceinline__ void rtn_xpose(rtn_u32* tile, rtn_u32 lane, const uint4 (&q)[4], rtn_u32 (&lo)[16]) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
    *reinterpret_cast<uint4*>(tile + (16u * k + (lane >> 2)) * RTN_XPITCH + (lane & 3u) * 4u) = q[k];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint4 x = *reinterpret_cast<const uint4*>(tile + lane * RTN_XPITCH + 4u * j);
    lo[4 * j + 0] = x.x; lo[4 * j + 1] = x.y; lo[4 * j + 2] = x.z; lo[4 * j + 3] = x.w;
  }
}

// Everything after the first 64 B arrived: optional second 64 B, parse, generated filter,
// L4Context, wave-level compaction of the outputs of group wv.
__device__ __forceinline__ void rtn_group(const rtn_args& a, rtn_u32 wv, rtn_u32 lane, rtn_u64 lane_lt,
                                          const rtn_u32 (&lo)[16], rtn_u32 dl, rtn_acc& acc) {
  const rtn_u32 i = wv * 64u + lane;
  const bool valid = i < a.n;
  rtn_u32 w[32];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = lo[k];
#pragma unroll
  for (int k = 16; k < 32; ++k) w[k] = 0u;
  // Second 64 B only where a header can reach past byte 64 (IPv6, IPv4 options, VLAN+options).
  {
    const rtn_u32 et = ((w[3] & 0xffu) << 8) | ((w[3] >> 8) & 0xffu);
    const rtn_u32 l3 = et == 0x8100u ? 18u : 14u;
    const rtn_u32 vihl = l3 == 18u ? (w[4] >> 16) & 0xffu : (w[3] >> 16) & 0xffu;
    const rtn_u32 inner = et == 0x8100u ? (((w[4] & 0xffu) << 8) | ((w[4] >> 8) & 0xffu)) : et;
    const rtn_u32 l4 = l3 + (inner == 0x86DDu ? 40u : ((vihl & 0xfu) << 2));
    const bool is_ip = inner == 0x0800u || inner == 0x86DDu;
    const bool need_hi = valid && is_ip && dl > 64u && l4 + 20u > 64u;
    if (need_hi) {
      if (a.stride >= 128u) {
        const uint4* slot = reinterpret_cast<const uint4*>(a.slab + (rtn_u64)i * a.stride);
#pragma unroll
        for (int k = 4; k < 8; ++k) {
          const uint4 x = slot[k];
          w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
        }
      } else {
        acc.status |= 1u;  // slot narrower than the headers this packet needs
      }
    }
  }
  rtn_view v;
  rtn_parse(w, dl, v);
  rtn_u32 act = 0;
  rtn_u64 dm[RTN_DM_WORDS];
#pragma unroll
  for (int k = 0; k < RTN_DM_WORDS; ++k) dm[k] = 0ull;
  rtn_filter(v, act, dm);
  const bool pc = valid && (act & 1u) != 0u;
  const bool fwd = pc && v.l4ok;
  const rtn_u64 pcm = __ballot(pc);
  const rtn_u64 fwdm = __ballot(fwd);
  acc.pc += (rtn_u32)__popcll(pcm);
  acc.fwd += (rtn_u32)__popcll(fwdm);
#if !defined(RTN_NO_PREFETCH) && !defined(RTN_NO_DRAIN) && !defined(RTN_UNROLL2) && !defined(RTN_LDS_XPOSE)
  // Drain point: the next group's loads (issued before this group was processed) have had the
  // whole parse to land. Waiting here, before this group's stores, means no later wait ever has
  // to cover a store (vmcnt counts stores on CDNA and drains in issue order).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  if (lane == 0u) {
    a.pc_bm[wv] = pcm;
    a.fwd_bm[wv] = fwdm;
  }
#ifndef RTN_EXP_NO_STORES
  if (fwd) {
    const rtn_u32 slot_i = wv * 64u + (rtn_u32)__popcll(fwdm & lane_lt);
    const bool tcp = v.tcp;
    const rtn_u32 thl = tcp ? ((rtn_l4_b(v, 12) & 0xf0u) >> 2) : 8u;
    const rtn_u32 ihl4 = (rtn_l3_b(v, 0) & 0xfu) << 2;
    const rtn_u32 iplen = v.v4 ? rtn_l3_be16(v, 2) : rtn_l3_be16(v, 4);
    const rtn_u32 len = iplen - (v.v4 ? ihl4 + thl : thl);
    uint4 r0, r1;
    r0.x = i;
    r0.y = v.v4 ? rtn_l3_be32(v, 12) : 0u;
    r0.z = v.v4 ? rtn_l3_be32(v, 16) : 0u;
    r0.w = rtn_l4_be16(v, 0) | (rtn_l4_be16(v, 2) << 16);
    r1.x = tcp ? rtn_l4_be32(v, 4) : 0u;
    r1.y = tcp ? rtn_l4_be32(v, 8) : 0u;
    r1.z = (v.l4off + thl) | (len << 16);
    r1.w = (tcp ? 6u : 17u) | ((tcp ? rtn_l4_b(v, 13) : 0u) << 8) | ((v.v4 ? 4u : 6u) << 16);
#ifdef RTN_EXP_STORE_WINDOW
    uint4* rp = reinterpret_cast<uint4*>(a.recs + (slot_i & 0xFFFFu));
#else
    uint4* rp = reinterpret_cast<uint4*>(a.recs + slot_i);
#endif
#ifdef RTN_NT_STORES
    rtn_v4u* vp = reinterpret_cast<rtn_v4u*>(rp);
    __builtin_nontemporal_store(rtn_v4u{r0.x, r0.y, r0.z, r0.w}, vp);
    __builtin_nontemporal_store(rtn_v4u{r1.x, r1.y, r1.z, r1.w}, vp + 1);
#else
    rp[0] = r0;
    rp[1] = r1;
#endif
    if (v.v6 && (a.flags & 1u)) {
      uint4* ap = reinterpret_cast<uint4*>(a.addr6 + (rtn_u64)slot_i * 32u);
      ap[0] = make_uint4(v.l3w[2], v.l3w[3], v.l3w[4], v.l3w[5]);
      ap[1] = make_uint4(v.l3w[6], v.l3w[7], v.l3w[8], v.l3w[9]);
    }
  }
#endif
#if RTN_DELIVER_WORDS > 0
  {
    rtn_u64 any = 0;
#pragma unroll
    for (int k = 0; k < RTN_DELIVER_WORDS; ++k) any |= dm[k];
    const bool d = valid && any != 0ull;
    const rtn_u64 dlvm = __ballot(d);
    if (lane == 0u) a.dlv_bm[wv] = dlvm;
    acc.dlv += (rtn_u32)__popcll(dlvm);
    if (d) {
      const rtn_u64 slot_i = (rtn_u64)wv * 64u + (rtn_u64)__popcll(dlvm & lane_lt);
      rtn_u64* dp = a.dlv_recs + slot_i * (1u + RTN_DELIVER_WORDS);
      dp[0] = (rtn_u64)i;
#pragma unroll
      for (int k = 0; k < RTN_DELIVER_WORDS; ++k) dp[1 + k] = dm[k];
    }
  }
#endif
}

extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel(rtn_args a) {
#ifdef RTN_EXP_CEILING
  {  // experiment only: fully coalesced read of the slab (16 B per lane), the HBM-read ceiling
    const rtn_u64 n16 = (rtn_u64)a.n * a.stride / 16u;
    const uint4* p = reinterpret_cast<const uint4*>(a.slab);
    rtn_u32 x = 0;
    for (rtn_u64 k = blockIdx.x * (rtn_u64)blockDim.x + threadIdx.x; k < n16; k += (rtn_u64)gridDim.x * blockDim.x) {
      const uint4 v = p[k];
      x ^= v.x + v.y + v.z + v.w;
    }
    if (x == 0x9E3779B9u) a.counters[3] = x;
    return;
  }
#endif
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 wave_g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const rtn_u32 nwaves = (gridDim.x * blockDim.x) >> 6;
  const rtn_u32 nw = (a.n + 63u) >> 6;
  const rtn_u64 lane_lt = (lane == 0u) ? 0ull : (~0ull >> (64u - lane));
  rtn_acc acc = {0u, 0u, 0u, 0u};
#if defined(RTN_LDS_XPOSE)
  __shared__ __attribute__((aligned(16))) rtn_u32 xtile[4][64 * RTN_XPITCH];
  rtn_u32* tile = xtile[threadIdx.x >> 6];
#if defined(RTN_UNROLL2)
  for (rtn_u32 wv = wave_g; wv < nw; wv += 2u * nwaves) {
    uint4 q0[4], q1[4];
    rtn_u32 dl0, dl1 = 0, lo[16];
    const rtn_u32 w1 = wv + nwaves;
    rtn_load_raw(a, wv, lane, q0, dl0);
    if (w1 < nw) rtn_load_raw(a, w1, lane, q1, dl1);
    rtn_xpose(tile, lane, q0, lo);
    rtn_group(a, wv, lane, lane_lt, lo, dl0, acc);
    if (w1 < nw) {
      rtn_xpose(tile, lane, q1, lo);
      rtn_group(a, w1, lane, lane_lt, lo, dl1, acc);
    }
  }
#else
  uint4 q[4];
  rtn_u32 dl = 0;
  if (wave_g < nw) rtn_load_raw(a, wave_g, lane, q, dl);
  for (rtn_u32 wv = wave_g; wv < nw; wv += nwaves) {
    rtn_u32 lo[16];
    rtn_xpose(tile, lane, q, lo);
    const rtn_u32 cdl = dl;
    const rtn_u32 nx = wv + nwaves;
    if (nx < nw) rtn_load_raw(a, nx, lane, q, dl);
    rtn_group(a, wv, lane, lane_lt, lo, cdl, acc);
  }
#endif
#elif defined(RTN_UNROLL2)
  // Two groups per iteration: both groups' loads are in flight before either is processed.
  for (rtn_u32 wv = wave_g; wv < nw; wv += 2u * nwaves) {
    rtn_u32 lo0[16], lo1[16], dl0, dl1 = 0;
    const rtn_u32 w1 = wv + nwaves;
    rtn_load_lo(a, wv * 64u + lane, wv * 64u + lane < a.n, lo0, dl0);
    if (w1 < nw) rtn_load_lo(a, w1 * 64u + lane, w1 * 64u + lane < a.n, lo1, dl1);
    rtn_group(a, wv, lane, lane_lt, lo0, dl0, acc);
    if (w1 < nw) rtn_group(a, w1, lane, lane_lt, lo1, dl1, acc);
  }
#elif !defined(RTN_NO_PREFETCH)
  // Software pipeline: the next group's first 64 B are in flight while this group is processed.
  rtn_u32 lo[16], dl;
  if (wave_g < nw) rtn_load_lo(a, wave_g * 64u + lane, wave_g * 64u + lane < a.n, lo, dl);
  for (rtn_u32 wv = wave_g; wv < nw; wv += nwaves) {
    rtn_u32 nlo[16], ndl = 0;
    const rtn_u32 nx = wv + nwaves;
    if (nx < nw) rtn_load_lo(a, nx * 64u + lane, nx * 64u + lane < a.n, nlo, ndl);
    rtn_group(a, wv, lane, lane_lt, lo, dl, acc);
#pragma unroll
    for (int k = 0; k < 16; ++k) lo[k] = nlo[k];
    dl = ndl;
  }
#else
  for (rtn_u32 wv = wave_g; wv < nw; wv += nwaves) {
    rtn_u32 lo[16], dl;
    rtn_load_lo(a, wv * 64u + lane, wv * 64u + lane < a.n, lo, dl);
    rtn_group(a, wv, lane, lane_lt, lo, dl, acc);
  }
#endif
  // one set of atomics per wave
  const rtn_u64 st = __ballot(acc.status != 0u);
  if (lane == 0u && st) atomicOr(&a.counters[3], 1u);
  if (!(a.flags & 2u)) return;
  if (lane == 0u) {
    if (acc.pc) atomicAdd(&a.counters[0], acc.pc);
    if (acc.fwd) atomicAdd(&a.counters[1], acc.fwd);
    if (acc.dlv) atomicAdd(&a.counters[2], acc.dlv);
  }
}
