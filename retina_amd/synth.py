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
