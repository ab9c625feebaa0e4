"""Deterministic adversarial frame corpus for parity tests:
truncation at every header boundary, IHL 0-15, TCP doff 0-15, 802.1Q / 802.1ad / QinQ,
IPv6 next-header values (extension headers are not parsed by the reference), length fields
smaller than the headers (L4Context checked_sub underflow), Payload slice edge cases.
"""
from __future__ import annotations

import random
import struct

ETH_DST = bytes.fromhex("001122334455")
ETH_SRC = bytes.fromhex("66778899aabb")


def eth(ethertype: int, vlan: int | None = None, outer: int | None = None) -> bytes:
    h = ETH_DST + ETH_SRC
    if outer is not None:
        h += struct.pack(">HH", outer, 0x0064)
    if vlan is not None:
        h += struct.pack(">HH", 0x8100, vlan)
    return h + struct.pack(">H", ethertype)


def ipv4(proto: int, payload_len: int, ihl: int = 5, total: int | None = None, src=0x0A000001, dst=0x0A000002,
         ttl=64, flags=0x4000) -> bytes:
    opts = bytes(max(0, ihl - 5) * 4)
    tot = total if total is not None else ihl * 4 + payload_len
    tot &= 0xFFFF
    return struct.pack(">BBHHHBBHII", 0x40 | (ihl & 15), 0, tot, 0x1234, flags, ttl, proto, 0, src, dst) + opts


def ipv6(nh: int, payload_len: int, plen: int | None = None, src=(0x20010DB8 << 96) | 1, dst=(0x20010DB8 << 96) | 2) -> bytes:
    pl = plen if plen is not None else payload_len
    return struct.pack(">IHBB", 0x60012345, pl & 0xFFFF, nh, 64) + src.to_bytes(16, "big") + dst.to_bytes(16, "big")


def tcp(sport=1234, dport=80, seq=1, ack=2, doff=5, flags=0x18, payload=b"") -> bytes:
    opts = bytes(max(0, doff - 5) * 4)
    return struct.pack(">HHIIBBHHH", sport, dport, seq, ack, (doff & 15) << 4, flags, 8192, 0, 0) + opts + payload


def udp(sport=5353, dport=53, payload=b"", length=None) -> bytes:
    ln = length if length is not None else 8 + len(payload)
    return struct.pack(">HHHH", sport, dport, ln & 0xFFFF, 0) + payload


def base_frames() -> list[bytes]:
    out = []
    pl = b"PAYLOADPAYLOAD"
    for ports in ((1234, 80), (80, 1234), (53, 53), (443, 50000), (5714, 31789), (31790, 31789), (10101, 135)):
        t = tcp(*ports, payload=pl)
        u = udp(*ports, payload=pl)
        out.append(eth(0x0800) + ipv4(6, len(t)) + t)
        out.append(eth(0x0800) + ipv4(17, len(u)) + u)
        out.append(eth(0x86DD) + ipv6(6, len(t)) + t)
        out.append(eth(0x86DD) + ipv6(17, len(u)) + u)
        out.append(eth(0x0800, vlan=7) + ipv4(6, len(t)) + t)
        out.append(eth(0x86DD, vlan=7) + ipv6(17, len(u)) + u)
    return out


def adversarial() -> list[bytes]:
    out: list[bytes] = []
    pl = b"0123456789abcdef"
    t = tcp(payload=pl)
    u = udp(payload=pl)
    goods = [eth(0x0800) + ipv4(6, len(t)) + t, eth(0x86DD) + ipv6(17, len(u)) + u,
             eth(0x0800, vlan=3) + ipv4(17, len(u)) + u, eth(0x86DD, vlan=3) + ipv6(6, len(t)) + t]
    # truncation at every byte up to the end of the headers (+ a few)
    for g in goods:
        for k in range(0, min(len(g), 100) + 1):
            out.append(g[:k])
    # IHL 0..15 with matching/non-matching total_length
    for ihl in range(16):
        for proto, l4 in ((6, t), (17, u)):
            out.append(eth(0x0800) + ipv4(proto, len(l4), ihl=ihl) + l4)
            out.append(eth(0x0800) + ipv4(proto, len(l4), ihl=ihl, total=ihl * 4 + 3) + l4)
            out.append(eth(0x0800, vlan=9) + ipv4(proto, len(l4), ihl=ihl) + l4)
    # TCP doff 0..15, payload lengths around the frame end
    for doff in range(16):
        tt = tcp(doff=doff, payload=pl)
        for extra in (-4, 0, 3):
            out.append(eth(0x0800) + ipv4(6, len(tt) + extra) + tt)
            out.append(eth(0x86DD) + ipv6(6, len(tt) + extra) + tt)
    # total_length / payload_length smaller than the headers (checked_sub underflow)
    for tot in (0, 19, 20, 39, 40, 41, 47, 48):
        out.append(eth(0x0800) + ipv4(6, 0, total=tot) + t)
        out.append(eth(0x0800) + ipv4(17, 0, total=tot) + u)
    for plen in (0, 7, 8, 19, 20, 21):
        out.append(eth(0x86DD) + ipv6(6, 0, plen=plen) + t)
        out.append(eth(0x86DD) + ipv6(17, 0, plen=plen) + u)
    # Payload slice edge cases: payload ends exactly at / past data_len, zero-length payload
    tt = tcp(payload=b"")
    out.append(eth(0x0800) + ipv4(6, len(tt)) + tt)                        # offset == data_len
    out.append(eth(0x0800) + ipv4(6, len(tt) + 10) + tt)                   # length past the end
    out.append(eth(0x0800) + ipv4(6, len(tt)) + tt + b"\x00")              # 1 byte of trailer
    uu = udp(payload=b"")
    out.append(eth(0x86DD) + ipv6(17, len(uu)) + uu)
    # VLAN variants: 802.1ad (no next header), QinQ, double 0x8100, VLAN truncated tag
    for g in (eth(0x0800, outer=0x88A8) + ipv4(6, len(t)) + t, eth(0x0800, vlan=5, outer=0x8100) + ipv4(6, len(t)) + t,
              eth(0x8100) + struct.pack(">H", 5), eth(0x88A8) + bytes(30), eth(0x0806) + bytes(28)):
        out.append(g)
    # IPv6 next-header values that are extension headers (parsed as-is: not TCP/UDP)
    for nh in (0, 43, 44, 50, 51, 58, 59, 60, 135, 6, 17):
        out.append(eth(0x86DD) + ipv6(nh, len(t)) + t)
    # IPv4 fragments (no fragment handling in the reference) and odd protocols
    out.append(eth(0x0800) + ipv4(6, len(t), flags=0x2000) + t)
    out.append(eth(0x0800) + ipv4(6, len(t), flags=0x00B9) + t)
    for proto in (0, 1, 2, 41, 47, 132, 255):
        out.append(eth(0x0800) + ipv4(proto, len(t)) + t)
    # version nibble ignored by the reference
    b = bytearray(eth(0x0800) + ipv4(6, len(t)) + t)
    b[14] = 0x65
    out.append(bytes(b))
    # filter-relevant field values: TTLs, flags, addresses, ports around the filter_stats predicates
    for ttl in (0, 1, 64, 220, 221, 255):
        out.append(eth(0x0800) + ipv4(17, len(u), ttl=ttl) + u)
        out.append(eth(0x0800) + ipv4(6, len(t), ttl=ttl) + tcp(sport=10101, flags=0x02, payload=pl))
    for fl in (0x00, 0x01, 0x02, 0x03, 0x07, 0x10, 0x12, 0x18, 0x20, 0xFF):
        for dport in (25, 80, 135, 137, 139, 140):
            tt = tcp(sport=5714, dport=dport, flags=fl, seq=1958810375 if fl & 2 else 5, payload=pl)
            out.append(eth(0x0800) + ipv4(6, len(tt)) + tt)
    for dst in (0xFFFFFFFF, 0x0A000000, 0x0A12FFFF, 0x0A130000, 0x03030303):
        out.append(eth(0x0800) + ipv4(17, len(u), dst=dst, src=dst) + udp(dport=161, payload=pl))
        out.append(eth(0x0800) + ipv4(1, 8, src=0x03030303) + bytes(8))
    for ln in (20, 100, 101):
        out.append(eth(0x0800) + ipv4(17, 28) + udp(dport=1434, length=ln, payload=bytes(20)))
        out.append(eth(0x0800) + ipv4(17, 28) + udp(dport=53, length=ln, payload=bytes(20)))
    out.append(eth(0x0800) + ipv4(17, 0, total=0) + udp(dport=161))
    return out


def random_frames(n: int, seed: int = 1) -> list[bytes]:
    """Random byte mutations of well-formed frames (hypothesis-style, but seeded)."""
    rng = random.Random(seed)
    base = base_frames() + adversarial()[:200]
    out = []
    for _ in range(n):
        f = bytearray(rng.choice(base))
        for _ in range(rng.randint(0, 4)):
            if not f:
                break
            k = rng.randrange(len(f))
            f[k] = rng.randrange(256)
        if rng.random() < 0.2 and len(f) > 1:
            f = f[:rng.randrange(len(f))]
        out.append(bytes(f))
    return out


def all_frames() -> list[bytes]:
    return base_frames() + adversarial() + random_frames(3000)
