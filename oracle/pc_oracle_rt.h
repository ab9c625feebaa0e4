/* ORACLE — TEST INFRASTRUCTURE ONLY.
 * Plain-C restatement of Retina's packet parsers and L4Context, shaped like the code the
 * reference runs per mbuf. Included by the C that oracle/cgen.py generates for a subscription
 * set (the analogue of filtergen's packet_continue). Reference lines:
 *   core/src/memory/mbuf.rs:109-135 (get_data bounds), core/src/protocols/packet/*.rs (parse_from,
 *   header_len, next_header, accessors), core/src/conntrack/pdu.rs:86-171 (L4Context::new),
 *   datatypes/src/packet.rs:18-29 (Payload::from_mbuf).
 */
#ifndef PC_ORACLE_RT_H
#define PC_ORACLE_RT_H
#include <stdint.h>
#include <string.h>

typedef struct { const uint8_t* d; uint32_t dl; } mbuf_t;
typedef struct { uint32_t off, hlen; int32_t next; } hdr_t; /* next = -1: None */

static inline int get_data(const mbuf_t* m, uint32_t off, uint32_t size) {
  return off < m->dl && off + size <= m->dl;
}
static inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static inline uint32_t be32(const uint8_t* p) { return (be16(p) << 16) | be16(p + 2); }

/* Ethernet::parse_from (ethernet.rs:170-183), header length (195-203), next_header (151-168) */
static inline int parse_ethernet(const mbuf_t* m, hdr_t* h) {
  if (!get_data(m, 0, 14)) return 0;
  uint32_t et = be16(m->d + 12);
  h->off = 0;
  if (et == 0x8100) {
    h->hlen = 18;
    h->next = get_data(m, 14, 4) ? (int32_t)be16(m->d + 16) : -1;
  } else if (et == 0x88a8) {
    h->hlen = 22;
    h->next = -1;
  } else {
    h->hlen = 14;
    h->next = (int32_t)et;
  }
  return 1;
}
/* Ipv4::parse_from (ipv4.rs:174-191) */
static inline int parse_ipv4(const mbuf_t* m, const hdr_t* o, hdr_t* h) {
  uint32_t off = o->off + o->hlen;
  if (!get_data(m, off, 20) || o->next != 0x0800) return 0;
  h->off = off;
  h->hlen = (uint32_t)(m->d[off] & 0xf) << 2;
  h->next = m->d[off + 9];
  return 1;
}
/* Ipv6::parse_from (ipv6.rs:116-133) */
static inline int parse_ipv6(const mbuf_t* m, const hdr_t* o, hdr_t* h) {
  uint32_t off = o->off + o->hlen;
  if (!get_data(m, off, 40) || o->next != 0x86DD) return 0;
  h->off = off;
  h->hlen = 40;
  h->next = m->d[off + 6];
  return 1;
}
/* Tcp::parse_from (tcp.rs:182-199) */
static inline int parse_tcp(const mbuf_t* m, const hdr_t* o, hdr_t* h) {
  uint32_t off = o->off + o->hlen;
  if (!get_data(m, off, 20) || o->next != 6) return 0;
  h->off = off;
  h->hlen = (uint32_t)(m->d[off + 12] & 0xf0) >> 2;
  h->next = -1;
  return 1;
}
/* Udp::parse_from (udp.rs:67-84) */
static inline int parse_udp(const mbuf_t* m, const hdr_t* o, hdr_t* h) {
  uint32_t off = o->off + o->hlen;
  if (!get_data(m, off, 8) || o->next != 17) return 0;
  h->off = off;
  h->hlen = 8;
  h->next = -1;
  return 1;
}

#define F8(m, h, k) ((uint32_t)(m)->d[(h)->off + (k)])
#define F16(m, h, k) be16((m)->d + (h)->off + (k))
#define F32(m, h, k) be32((m)->d + (h)->off + (k))

typedef struct {
  uint32_t ver, proto, sport, dport, offset, length, seq, ack, flags;
  uint8_t src[16], dst[16]; /* IPv4: first 4 bytes */
} l4ctx_t;

/* L4Context::new (pdu.rs:86-171) */
static inline int l4context(const mbuf_t* m, l4ctx_t* c) {
  hdr_t eth, ip, l4;
  if (!parse_ethernet(m, &eth)) return 0;
  uint32_t iplen, pre;
  memset(c, 0, sizeof *c);
  if (parse_ipv4(m, &eth, &ip)) {
    iplen = F16(m, &ip, 2);
    pre = ip.hlen;
    c->ver = 4;
    memcpy(c->src, m->d + ip.off + 12, 4);
    memcpy(c->dst, m->d + ip.off + 16, 4);
  } else if (parse_ipv6(m, &eth, &ip)) {
    iplen = F16(m, &ip, 4);
    pre = 0;
    c->ver = 6;
    memcpy(c->src, m->d + ip.off + 8, 16);
    memcpy(c->dst, m->d + ip.off + 24, 16);
  } else {
    return 0;
  }
  if (parse_tcp(m, &ip, &l4)) {
    if (iplen < pre + l4.hlen) return 0;
    c->proto = 6;
    c->length = iplen - (pre + l4.hlen);
    c->seq = F32(m, &l4, 4);
    c->ack = F32(m, &l4, 8);
    c->flags = F8(m, &l4, 13);
  } else if (parse_udp(m, &ip, &l4)) {
    if (iplen < pre + 8) return 0;
    c->proto = 17;
    c->length = iplen - (pre + 8);
  } else {
    return 0;
  }
  c->sport = F16(m, &l4, 0);
  c->dport = F16(m, &l4, 2);
  c->offset = l4.off + l4.hlen;
  return 1;
}

/* Payload::from_mbuf (datatypes/src/packet.rs:18-29) via get_data_slice (mbuf.rs:109-120) */
static inline int payload_from_mbuf(const mbuf_t* m) {
  l4ctx_t c;
  if (!l4context(m, &c)) return 0;
  return c.offset < m->dl && c.offset + c.length <= m->dl;
}

#endif
