"""ORACLE (test infrastructure only): minimal libpcap / pcapng readers for traces/.

Mirrors what the reference's offline runtime feeds to the filter (core/src/runtime/offline.rs:67-82):
every captured frame becomes an mbuf whose data is the captured bytes; frames whose *original*
length exceeds the configured MTU are skipped before the filter runs.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass


@dataclass
class Frame:
    data: bytes      # captured bytes (-> Mbuf data, data_len = len(data))
    orig_len: int    # length on the wire (pcap `len`)
    linktype: int


def _read_pcap(b: bytes) -> list[Frame]:
    magic = struct.unpack_from("<I", b, 0)[0]
    if magic in (0xA1B2C3D4, 0xA1B23C4D):
        e = "<"
    elif magic in (0xD4C3B2A1, 0x4D3CB2A1):
        e = ">"
    else:
        raise ValueError("not a libpcap file")
    linktype = struct.unpack_from(e + "I", b, 20)[0]
    off = 24
    out = []
    while off + 16 <= len(b):
        _, _, incl, orig = struct.unpack_from(e + "IIII", b, off)
        off += 16
        out.append(Frame(b[off:off + incl], orig, linktype))
        off += incl
    return out


def _read_pcapng(b: bytes) -> list[Frame]:
    out = []
    off = 0
    e = "<"
    links: list[int] = []
    while off + 12 <= len(b):
        btype = struct.unpack_from(e + "I", b, off)[0]
        if btype == 0x0A0D0D0A:  # section header: byte order magic decides endianness
            bom = struct.unpack_from("<I", b, off + 8)[0]
            e = "<" if bom == 0x1A2B3C4D else ">"
            links = []
        blen = struct.unpack_from(e + "I", b, off + 4)[0]
        if btype == 1:  # interface description
            links.append(struct.unpack_from(e + "H", b, off + 8)[0])
        elif btype == 6:  # enhanced packet
            iface, _, _, cap, orig = struct.unpack_from(e + "IIIII", b, off + 8)
            out.append(Frame(b[off + 28:off + 28 + cap], orig, links[iface] if iface < len(links) else 1))
        elif btype == 3:  # simple packet
            orig = struct.unpack_from(e + "I", b, off + 8)[0]
            cap = min(orig, blen - 16)
            out.append(Frame(b[off + 12:off + 12 + cap], orig, links[0] if links else 1))
        if blen < 12:
            break
        off += blen
    return out


def read(path) -> list[Frame]:
    b = open(path, "rb").read()
    if struct.unpack_from("<I", b, 0)[0] == 0x0A0D0D0A:
        return _read_pcapng(b)
    return _read_pcap(b)


def offline_frames(path, mtu: int = 9702) -> list[bytes]:
    """The frames OfflineRuntime hands to continue_packet (offline.rs:67-75): orig len <= mtu."""
    return [f.data for f in read(path) if f.orig_len <= mtu]
