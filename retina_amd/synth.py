"""Seeded synthetic traffic for the benchmark configurations (BASELINE.json `configs`).

Every byte is a function of (seed, frame index) through splitmix64, vectorised with numpy, so
the GPU run, the CPU baseline and the parity tests see identical frames at any size or shard.
Configs:
  cfg2: 64 B Eth/IPv4/TCP, dport 80 with p=1/4 (filter `tcp.dst_port = 80`)
  cfg3: IMIX 64/594/1518 (7:4:1), 20% 802.1Q, 70% IPv4 / 30% IPv6, 60% TCP / 35% UDP / 5% ICMP,
        1% malformed (truncated, IHL<5, 802.1ad); ports 50% from a hot set
  cfg4: 1500 B IPv4/IPv6 x TCP/UDP, 20% VLAN, dst 50% inside 10.0-18/16
"""
from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
HOT_PORTS = np.array([7, 19, 25, 53, 80, 161, 443, 1434, 8080], np.uint64)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _rand(seed: int, idx: np.ndarray, k: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        return splitmix64(np.uint64(seed) + idx * np.uint64(16) + np.uint64(k))


def _put(buf: np.ndarray, off: int, val: np.ndarray, nbytes: int) -> None:
    """Big-endian store of val (uint64 array) into buf[:, off:off+nbytes]."""
    for b in range(nbytes):
        buf[:, off + b] = ((val >> np.uint64(8 * (nbytes - 1 - b))) & np.uint64(0xFF)).astype(np.uint8)


def cfg2(n: int, start: int = 0, seed: int = 0x5EED0002) -> tuple[np.ndarray, np.ndarray]:
    """Frames [start, start+n) of config 2: returns (slab uint8[n*64], data_len uint16[n])."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    r = [_rand(seed, idx, k) for k in range(7)]
    b = np.zeros((n, 64), np.uint8)
    _put(b, 0, r[0], 6)                       # dst MAC
    _put(b, 6, r[1], 6)                       # src MAC
    b[:, 12] = 0x08                           # EtherType IPv4
    b[:, 14] = 0x45
    b[:, 17] = 50                             # total_length = 20 + 20 + 10
    _put(b, 18, r[2] & np.uint64(0xFFFF), 2)  # identification
    b[:, 22] = 64                             # TTL
    b[:, 23] = 6                              # TCP
    _put(b, 26, r[3] & np.uint64(0xFFFFFFFF), 4)
    _put(b, 30, r[3] >> np.uint64(32), 4)
    _put(b, 34, r[4] & np.uint64(0xFFFF), 2)  # sport
    hit = ((r[4] >> np.uint64(16)) & np.uint64(3)) == 0
    other = (r[4] >> np.uint64(24)) & np.uint64(0xFFFF)
    other = np.where(other == 80, np.uint64(81), other)
    _put(b, 36, np.where(hit, np.uint64(80), other), 2)
    _put(b, 38, r[5] & np.uint64(0xFFFFFFFF), 4)   # seq
    _put(b, 42, r[5] >> np.uint64(32), 4)           # ack
    b[:, 46] = 0x50                                 # doff 5
    b[:, 47] = (r[6] & np.uint64(0xFF)).astype(np.uint8)  # flags
    _put(b, 48, (r[6] >> np.uint64(8)) & np.uint64(0xFFFF), 2)  # window
    return b.reshape(-1), np.full(n, 64, np.uint16)


CFG2_SPEC = """[[subscriptions]]
filter = "tcp.dst_port = 80"
datatypes = ["ConnRecord"]
callback = "cb"
"""


# ----------------------------------------------------------------------------------------------
# variable-layout frames (configs 3 and 4)

def _put_rows(b: np.ndarray, rows: np.ndarray, off: np.ndarray, val: np.ndarray, nbytes: int) -> None:
    """Big-endian store of val[k] at b[rows[k], off[k]:off[k]+nbytes] (per-row offsets)."""
    for j in range(nbytes):
        col = off + j
        ok = col < b.shape[1]
        b[rows[ok], col[ok]] = ((val[ok] >> np.uint64(8 * (nbytes - 1 - j))) & np.uint64(0xFF)).astype(np.uint8)


def _frames(n: int, start: int, seed: int, sizes: np.ndarray, p_vlan: float, p_v6: float,
            p_tcp: float, p_udp: float, p_bad: float, dst_mode: str, stride: int):
    """Shared generator: Eth [802.1Q] / IPv4|IPv6 / TCP|UDP|ICMP frames with the given size per
    frame; writes only the first `stride` bytes (the header slab) and returns data_len = size."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    r = [_rand(seed, idx, k) for k in range(12)]
    u = lambda k: (r[k] >> np.uint64(11)).astype(np.float64) / float(1 << 53)  # noqa: E731
    b = np.zeros((n, stride), np.uint8)
    rows = np.arange(n)
    dl = sizes.astype(np.int64).copy()
    _put(b, 0, r[0], 6)
    _put(b, 6, r[1], 6)
    vlan = u(2) < p_vlan
    v6 = u(3) < p_v6
    l4r = u(4)
    tcp = l4r < p_tcp
    udp = (l4r >= p_tcp) & (l4r < p_tcp + p_udp)
    l3 = np.where(vlan, 18, 14)
    et = np.where(v6, np.uint64(0x86DD), np.uint64(0x0800))
    b[vlan, 12] = 0x81
    b[vlan, 13] = 0x00
    _put_rows(b, rows[vlan], np.full(vlan.sum(), 14), (r[5][vlan] & np.uint64(0x0FFF)), 2)  # TCI
    _put_rows(b, rows, l3 - 2, et, 2)
    proto = np.where(tcp, np.uint64(6), np.where(udp, np.uint64(17), np.where(v6, np.uint64(58), np.uint64(1))))
    l4h = np.where(tcp, 20, 8)
    iphl = np.where(v6, 40, 20)
    l4 = l3 + iphl
    # addresses
    src4 = r[6] & np.uint64(0xFFFFFFFF)
    dst4 = r[6] >> np.uint64(32)
    if dst_mode == "ten16":  # 50% inside 10.0-18/16
        inside = u(7) < 0.5
        k = (r[7] >> np.uint64(8)) % np.uint64(19)
        dst4 = np.where(inside, (np.uint64(10) << np.uint64(24)) | (k << np.uint64(16)) | (r[7] >> np.uint64(40)) & np.uint64(0xFFFF), dst4)
    dst4 = np.where(u(8) < 0.002, np.uint64(0xFFFFFFFF), dst4)         # some broadcasts
    src4 = np.where(u(8) > 0.998, np.uint64(0x03030303), src4)          # 3.3.3.3
    v4r, v6r = rows[~v6], rows[v6]
    # IPv4
    o = l3[~v6]
    b[v4r, o] = 0x45
    _put_rows(b, v4r, o + 2, (dl[~v6] - l3[~v6]).astype(np.uint64), 2)      # total_length
    _put_rows(b, v4r, o + 4, r[9][~v6] & np.uint64(0xFFFF), 2)
    b[v4r, o + 8] = ((r[9][~v6] >> np.uint64(16)) & np.uint64(0xFF)).astype(np.uint8)  # TTL
    b[v4r, o + 9] = proto[~v6].astype(np.uint8)
    _put_rows(b, v4r, o + 12, src4[~v6], 4)
    _put_rows(b, v4r, o + 16, dst4[~v6], 4)
    # IPv6
    o = l3[v6]
    _put_rows(b, v6r, o, np.uint64(0x60000000) | (r[9][v6] & np.uint64(0xFFFFF)), 4)
    _put_rows(b, v6r, o + 4, (dl[v6] - l3[v6] - 40).astype(np.uint64), 2)   # payload_length
    b[v6r, o + 6] = proto[v6].astype(np.uint8)
    b[v6r, o + 7] = 64
    _put_rows(b, v6r, o + 8, np.uint64(0x20010DB8) << np.uint64(32) | (r[6][v6] >> np.uint64(32)), 8)
    _put_rows(b, v6r, o + 16, r[10][v6], 8)
    _put_rows(b, v6r, o + 24, np.uint64(0x20010DB8) << np.uint64(32) | (r[6][v6] & np.uint64(0xFFFFFFFF)), 8)
    _put_rows(b, v6r, o + 32, r[11][v6], 8)
    # ports: 50% hot
    hot_s = (u(9) < 0.5)
    hot_d = (u(10) < 0.5)
    sp = np.where(hot_s, HOT_PORTS[(r[11] % np.uint64(len(HOT_PORTS))).astype(np.int64)], r[5] >> np.uint64(16) & np.uint64(0xFFFF))
    dp = np.where(hot_d, HOT_PORTS[((r[11] >> np.uint64(8)) % np.uint64(len(HOT_PORTS))).astype(np.int64)], r[5] >> np.uint64(32) & np.uint64(0xFFFF))
    tr, ur = rows[tcp], rows[udp]
    o = l4[tcp]
    _put_rows(b, tr, o, sp[tcp], 2)
    _put_rows(b, tr, o + 2, dp[tcp], 2)
    _put_rows(b, tr, o + 4, r[8][tcp] & np.uint64(0xFFFFFFFF), 4)
    _put_rows(b, tr, o + 8, r[8][tcp] >> np.uint64(32), 4)
    b[tr, o + 12] = 0x50
    b[tr, o + 13] = (r[10][tcp] & np.uint64(0xFF)).astype(np.uint8)
    o = l4[udp]
    _put_rows(b, ur, o, sp[udp], 2)
    _put_rows(b, ur, o + 2, dp[udp], 2)
    _put_rows(b, ur, o + 4, (dl[udp] - l4[udp]).astype(np.uint64), 2)
    # malformed 1%: truncation, IHL < 5, 802.1ad
    bad = u(11) < p_bad
    kind = (r[11] >> np.uint64(20)) % np.uint64(3)
    trunc = bad & (kind == 0)
    dl = np.where(trunc, (r[11] >> np.uint64(24)) % np.uint64(70), dl)
    ihl = bad & (kind == 1) & ~v6
    b[rows[ihl], l3[ihl]] = (0x40 | ((r[11][ihl] >> np.uint64(32)) % np.uint64(5))).astype(np.uint8)
    qq = bad & (kind == 2)
    b[qq, 12] = 0x88
    b[qq, 13] = 0xA8
    # slab content beyond data_len is zero (as a NIC/mbuf copy would leave it)
    cols = np.arange(stride)
    b[cols[None, :] >= dl[:, None]] = 0
    return b.reshape(-1), dl.astype(np.uint16)


def cfg3(n: int, start: int = 0, seed: int = 0x5EED0003, stride: int = 128):
    """IMIX 64/594/1518 at 7:4:1 with VLAN/IPv6 variants and 1% malformed frames."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    c = (_rand(seed, idx, 15) % np.uint64(12)).astype(np.int64)
    sizes = np.where(c < 7, 64, np.where(c < 11, 594, 1518))
    return _frames(n, start, seed, sizes, 0.2, 0.3, 0.6, 0.35, 0.01, "uniform", stride)


def cfg4(n: int, start: int = 0, seed: int = 0x5EED0004, stride: int = 128):
    """1500 B IPv4/IPv6 x TCP/UDP, 20% VLAN, destinations 50% inside 10.0-18/16."""
    sizes = np.full(n, 1500)
    return _frames(n, start, seed, sizes, 0.2, 0.3, 0.6, 0.4, 0.0, "ten16", stride)


def _toml(subs) -> str:
    """[[subscriptions]] entries from (filter, datatypes, callback[, streaming]) tuples."""
    out = []
    for f, dts, cb, *rest in subs:
        d = ", ".join(f'"{x}"' for x in dts)
        st = f'streaming = "{rest[0]}"\n' if rest else ""
        out.append(f'[[subscriptions]]\nfilter = "{f}"\ndatatypes = [{d}]\ncallback = "{cb}"\n{st}')
    return "\n".join(out)


# examples/protocols/src/main.rs:92, 106, 120, 133 (filters of the four subscriptions)
PROTOCOLS_SUBS = [
    ("dns and ((tcp and tcp.port != 53) or (udp and udp.port != 53))", ["DnsTransaction", "FiveTuple", "CoreId"], "dns_cb"),
    ("http and tcp and tcp.port != 80 and tcp.port != 8080", ["HttpTransaction", "FiveTuple", "CoreId"], "http_cb"),
    ("tls and tcp and tcp.port != 443", ["TlsHandshake", "FiveTuple", "CoreId"], "tls_cb"),
    ("quic and udp.port != 443", ["QuicStream", "FiveTuple", "CoreId"], "quic_cb"),
]
# examples/filter_stats/spec.toml: the 19 subscriptions whose filters are packet/connection level
FILTER_STATS_PKT = [
    ("udp and ipv4.time_to_live = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.src_port = 5714 and tcp.ack = 1 and tcp.syn = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.dst_port = 25 and tcp.ack = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.src_port = 10101 and tcp.syn = 1 and tcp.ack = 0 and ipv4.time_to_live > 220", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.src_port = 31790 and tcp.dst_port = 31789 and tcp.ack = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.dst_port = 80 and tcp.syn = 1 and tcp.fin = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.syn = 1 and tcp.seq_no = 1958810375", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.ack = 1 and tcp.psh = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.dst_port in 135..139 and tcp.urg = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("tcp.fin = 1 and tcp.rst = 1 and tcp.syn = 1", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("udp and ipv4.total_length = 0 and udp.dst_port = 161", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("udp and udp.dst_port = 1434 and udp.length > 100", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("udp and udp.dst_port = 53 and udp.length = 20", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("ipv4.protocol = 2", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("ipv4.protocol = 1 and ipv4.src_addr = 3.3.3.3/32", ["ZcFrame", "CoreId", "FilterStr"], "packet_cb"),
    ("udp.port = 19 and udp.port = 7", ["CoreId", "FilterStr"], "conn_cb"),
    ("udp.dst_port = 161", ["CoreId", "FilterStr"], "conn_cb"),
    ("tcp.src_port = 1010", ["CoreId", "FilterStr"], "conn_cb"),
    ("ipv4.dst_addr = 255.255.255.255 and (udp.dst_port = 161 or udp.dst_port = 162)", ["CoreId", "FilterStr"], "conn_cb"),
]

CFG3_SUBS = PROTOCOLS_SUBS + [FILTER_STATS_PKT[14], FILTER_STATS_PKT[7]]
CFG4_SUBS = FILTER_STATS_PKT + PROTOCOLS_SUBS + [
    (f"ipv4.dst_addr = 10.{k}.0.0/16", ["ZcFrame", "FilterStr"], "subnet_cb") for k in range(19)]
CFG3_SPEC = _toml(CFG3_SUBS)
CFG4_SPEC = _toml(CFG4_SUBS)
# examples/basic/src/main.rs:5-17
BASIC_SPEC = _toml([("tls", ["TlsHandshake", "ConnRecord"], "tls_cb"), ("dns", ["DnsTransaction", "ConnRecord"], "dns_cb")])


def alg_read_bytes(slab: np.ndarray, dlen: np.ndarray, stride: int) -> int:
    """sum over frames of min(data_len, 64*ceil(hdr_end/64)) + 2, hdr_end = end of the
    last fixed header the parse touches (L2 + L3 + L4 fixed headers, as far as they parse)."""
    b = slab.reshape(-1, stride)
    n = len(dlen)
    dl = dlen.astype(np.int64)
    et = (b[:, 12].astype(np.int64) << 8) | b[:, 13]
    vl = et == 0x8100
    l3 = np.where(vl, 18, np.where(et == 0x88A8, 22, 14))
    inner = np.where(vl, (b[:, 16].astype(np.int64) << 8) | b[:, 17], et)
    rows = np.arange(n)
    vihl = b[rows, np.minimum(l3, stride - 1)].astype(np.int64)
    v4 = inner == 0x0800
    v6 = inner == 0x86DD
    l4 = l3 + np.where(v6, 40, (vihl & 15) * 4)
    hdr_end = np.where(v4 | v6, l4 + 20, l3)
    hdr_end = np.minimum(hdr_end, np.maximum(dl, 14))
    need = 64 * ((hdr_end + 63) // 64)
    return int(np.minimum(dl, need).sum() + 2 * n)
