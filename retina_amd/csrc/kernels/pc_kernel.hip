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

extern "C" __global__ void __launch_bounds__(256) rtn_pc_kernel(rtn_args a) {
  const rtn_u32 lane = threadIdx.x & 63u;
  const rtn_u32 wave_g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const rtn_u32 nwaves = (gridDim.x * blockDim.x) >> 6;
  const rtn_u32 nw = (a.n + 63u) >> 6;
  const rtn_u64 lane_lt = (lane == 0u) ? 0ull : (~0ull >> (64u - lane));
  rtn_u32 c_pc = 0, c_fwd = 0, c_dlv = 0, status = 0;
  for (rtn_u32 wv = wave_g; wv < nw; wv += nwaves) {
    const rtn_u32 i = wv * 64u + lane;
    const bool valid = i < a.n;
    rtn_u32 w[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) w[k] = 0u;
    rtn_u32 dl = 0;
    const uint4* slot = reinterpret_cast<const uint4*>(a.slab + (rtn_u64)i * a.stride);
    if (valid) {
      dl = a.dlen[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 x = slot[k];
        w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
      }
    }
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
#pragma unroll
          for (int k = 4; k < 8; ++k) {
            const uint4 x = slot[k];
            w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
          }
        } else {
          status |= 1u;  // slot narrower than the headers this packet needs
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
    if (lane == 0u) {
      a.pc_bm[wv] = pcm;
      a.fwd_bm[wv] = fwdm;
    }
    c_pc += (rtn_u32)__popcll(pcm);
    c_fwd += (rtn_u32)__popcll(fwdm);
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
      uint4* rp = reinterpret_cast<uint4*>(a.recs + slot_i);
      rp[0] = r0;
      rp[1] = r1;
      if (v.v6 && (a.flags & 1u)) {
        uint4* ap = reinterpret_cast<uint4*>(a.addr6 + (rtn_u64)slot_i * 32u);
        ap[0] = make_uint4(v.l3w[2], v.l3w[3], v.l3w[4], v.l3w[5]);
        ap[1] = make_uint4(v.l3w[6], v.l3w[7], v.l3w[8], v.l3w[9]);
      }
    }
#if RTN_DELIVER_WORDS > 0
    {
      rtn_u64 any = 0;
#pragma unroll
      for (int k = 0; k < RTN_DELIVER_WORDS; ++k) any |= dm[k];
      const bool d = valid && any != 0ull;
      const rtn_u64 dlvm = __ballot(d);
      if (lane == 0u) a.dlv_bm[wv] = dlvm;
      c_dlv += (rtn_u32)__popcll(dlvm);
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
  // one set of atomics per wave
  if (!(a.flags & 2u)) return;
  if (lane == 0u) {
    if (c_pc) atomicAdd(&a.counters[0], c_pc);
    if (c_fwd) atomicAdd(&a.counters[1], c_fwd);
    if (c_dlv) atomicAdd(&a.counters[2], c_dlv);
  }
  const rtn_u64 st = __ballot(status != 0u);
  if (lane == 0u && st) atomicOr(&a.counters[3], 1u);
}
