"""ORACLE (test infrastructure only): per-packet semantics in pure Python.

  core/src/memory/mbuf.rs:109-135          get_data / get_data_slice bounds (strict `<` on offset)
  core/src/protocols/packet/ethernet.rs    EthernetHeader length (14/18/22), next_header (802.1Q via
                                           Dot1q at 14; 802.1ad -> None)
  core/src/protocols/packet/ipv4.rs        20-byte fixed header, IHL*4 with no sanity check
  core/src/protocols/packet/ipv6.rs        40-byte header, no extension headers
  core/src/protocols/packet/tcp.rs         20-byte header, doff*4
  core/src/protocols/packet/udp.rs         8-byte header
  core/src/conntrack/pdu.rs:86-171         L4Context::new
  datatypes/src/packet.rs:7-29             ZcFrame / Payload from_mbuf
  filtergen (packet_filter.rs, utils.rs)   control flow of the generated packet_continue
"""
from __future__ import annotations

from dataclasses import dataclass

from .filterlang import Node, PacketTree, Pred


def get_data(dl: int, off: int, size: int) -> bool:
    return off < dl and off + size <= dl


def be(d: bytes, off: int, n: int) -> int:
    return int.from_bytes(d[off:off + n], "big")


@dataclass
class Hdr:
    proto: str
    off: int          # header offset in the frame
    hlen: int         # header_len()
    nxt: int | None   # next_header()


def parse(d: bytes, dl: int, proto: str, outer: Hdr | None) -> Hdr | None:
    """Packet::parse_to::<proto>(outer)."""
    if proto == "ethernet":
        if not get_data(dl, 0, 14):
            return None
        et = be(d, 12, 2)
        hlen = 18 if et == 0x8100 else 22 if et == 0x88A8 else 14
        if et == 0x8100:
            nxt = be(d, 16, 2) if get_data(dl, 14, 4) else None
        elif et == 0x88A8:
            nxt = None
        else:
            nxt = et
        return Hdr("ethernet", 0, hlen, nxt)
    off = outer.off + outer.hlen
    if proto == "ipv4":
        if not get_data(dl, off, 20) or outer.nxt != 0x0800:
            return None
        return Hdr("ipv4", off, (d[off] & 0xF) << 2, d[off + 9])
    if proto == "ipv6":
        if not get_data(dl, off, 40) or outer.nxt != 0x86DD:
            return None
        return Hdr("ipv6", off, 40, d[off + 6])
    if proto == "tcp":
        if not get_data(dl, off, 20) or outer.nxt != 6:
            return None
        return Hdr("tcp", off, (d[off + 12] & 0xF0) >> 2, None)
    if proto == "udp":
        if not get_data(dl, off, 8) or outer.nxt != 17:
            return None
        return Hdr("udp", off, 8, None)
    raise ValueError(proto)


def field_value(d: bytes, h: Hdr, name: str):
    """Accessor methods of the header structs; returns (type, value)."""
    o = h.off
    if h.proto == "ipv4":
        b0, b1, ff = d[o], d[o + 1], be(d, o + 6, 2)
        table = {
            "version": ("u8", (b0 & 0xF0) >> 4), "ihl": ("u8", b0 & 0x0F), "version_ihl": ("u8", b0),
            "dscp": ("u8", b1 >> 2), "ecn": ("u8", b1 & 3), "dscp_ecn": ("u8", b1), "type_of_service": ("u8", b1),
            "total_length": ("u16", be(d, o + 2, 2)), "identification": ("u16", be(d, o + 4, 2)),
            "flags_to_fragment_offset": ("u16", ff), "flags": ("u8", ff >> 13),
            "rf": ("bool", int(ff & 0x8000 != 0)), "df": ("bool", int(ff & 0x4000 != 0)),
            "mf": ("bool", int(ff & 0x2000 != 0)), "fragment_offset": ("u16", ff & 0x1FFF),
            "time_to_live": ("u8", d[o + 8]), "protocol": ("u8", d[o + 9]),
            "header_checksum": ("u16", be(d, o + 10, 2)), "src_addr": ("v4", be(d, o + 12, 4)),
            "dst_addr": ("v4", be(d, o + 16, 4)),
        }
    elif h.proto == "ipv6":
        v = be(d, o, 4)
        table = {
            "version": ("u8", (v & 0xF0000000) >> 28), "dscp": ("u8", (v & 0x0FC00000) >> 22),
            "ecn": ("u8", (v & 0x00300000) >> 20), "traffic_class": ("u8", (v & 0x0FF00000) >> 20),
            "flow_label": ("u32", v & 0xFFFFF), "version_to_flow_label": ("u32", v),
            "payload_length": ("u16", be(d, o + 4, 2)), "next_header": ("u8", d[o + 6]),
            "hop_limit": ("u8", d[o + 7]), "src_addr": ("v6", be(d, o + 8, 16)), "dst_addr": ("v6", be(d, o + 24, 16)),
        }
    elif h.proto == "tcp":
        fl, dn = d[o + 13], d[o + 12]
        table = {
            "src_port": ("u16", be(d, o, 2)), "dst_port": ("u16", be(d, o + 2, 2)), "seq_no": ("u32", be(d, o + 4, 4)),
            "ack_no": ("u32", be(d, o + 8, 4)), "data_offset": ("u8", (dn & 0xF0) >> 4), "reserved": ("u8", dn & 0x0F),
            "data_offset_to_ns": ("u8", dn), "flags": ("u8", fl), "window": ("u16", be(d, o + 14, 2)),
            "checksum": ("u16", be(d, o + 16, 2)), "urgent_pointer": ("u16", be(d, o + 18, 2)),
            "ns": ("u8", dn & 1), "cwr": ("u8", fl >> 7 & 1), "ece": ("u8", fl >> 6 & 1), "urg": ("u8", fl >> 5 & 1),
            "ack": ("u8", fl >> 4 & 1), "psh": ("u8", fl >> 3 & 1), "rst": ("u8", fl >> 2 & 1),
            "syn": ("u8", fl >> 1 & 1), "fin": ("u8", fl & 1), "synack": ("u8", int(fl & 0x12 != 0)),
        }
    else:
        table = {"src_port": ("u16", be(d, o, 2)), "dst_port": ("u16", be(d, o + 2, 2)),
                 "length": ("u16", be(d, o + 4, 2)), "checksum": ("u16", be(d, o + 6, 2))}
    return table[name]


def eval_binary(d: bytes, h: Hdr, p: Pred) -> bool:
    """binary_to_tokens semantics (filtergen/src/utils.rs:18-121) on a parsed header."""
    _, x = field_value(d, h, p.field)
    k, op = p.value.kind, p.op
    if k == "Int":
        c = p.value.data[0]
        return {"Eq": x == c, "Ne": x != c, "Ge": x >= c, "Le": x <= c, "Gt": x > c, "Lt": x < c}[op]
    if k == "IntRange":
        a, b = p.value.data
        return a <= x <= b
    addr, plen = p.value.data
    bits = 32 if k == "Ipv4" else 128
    if plen == bits:
        eq = x == addr
    else:
        mask = ((1 << bits) - 1) ^ ((1 << (bits - plen)) - 1) if plen else 0
        eq = (x & mask) == (addr & mask)
    return (not eq) if op == "Ne" else eq


@dataclass
class L4Ctx:
    ver: int
    src: int
    dst: int
    sport: int
    dport: int
    proto: int
    offset: int
    length: int
    seq: int
    ack: int
    flags: int


def l4context(d: bytes, dl: int) -> L4Ctx | None:
    """L4Context::new (pdu.rs:86-171)."""
    eth = parse(d, dl, "ethernet", None)
    if eth is None:
        return None
    for ipn in ("ipv4", "ipv6"):
        ip = parse(d, dl, ipn, eth)
        if ip is None:
            continue
        if ipn == "ipv4":
            iplen, pre = be(d, ip.off + 2, 2), ip.hlen
            src, dst, ver = be(d, ip.off + 12, 4), be(d, ip.off + 16, 4), 4
        else:
            iplen, pre = be(d, ip.off + 4, 2), 0
            src, dst, ver = be(d, ip.off + 8, 16), be(d, ip.off + 24, 16), 6
        tcp = parse(d, dl, "tcp", ip)
        if tcp is not None:
            n = iplen - (pre + tcp.hlen)
            if n < 0:
                return None
            o = tcp.off
            return L4Ctx(ver, src, dst, be(d, o, 2), be(d, o + 2, 2), 6, o + tcp.hlen, n, be(d, o + 4, 4),
                         be(d, o + 8, 4), d[o + 13])
        udp = parse(d, dl, "udp", ip)
        if udp is not None:
            n = iplen - (pre + 8)
            if n < 0:
                return None
            o = udp.off
            return L4Ctx(ver, src, dst, be(d, o, 2), be(d, o + 2, 2), 17, o + 8, n, 0, 0, 0)
        return None
    return None


def payload_ok(d: bytes, dl: int) -> bool:
    c = l4context(d, dl)
    return c is not None and c.offset < dl and c.offset + c.length <= dl


def evaluate(tree: PacketTree, frame: bytes, dl: int | None = None, chains: bool = True,
             trace: dict | None = None):
    """Run the generated packet_continue for `tree` on one frame.
    Returns (actions_data, [deliver statement index, ...] in call order).

    chains=False runs every sibling whose condition holds, as if no `else if` had been emitted
    (test instrument: the tree's content without filtergen's chaining). `trace`, if given, counts
    in trace["skipped"] the siblings an `else if` chain skipped although their condition held."""
    d = bytes(frame)
    dl = len(d) if dl is None else dl
    d = d + bytes(max(0, 256 - len(d)))
    subs = tree.subs
    act = 0
    fired: list[int] = []
    stmt = [0]
    stmts = statement_table(tree)

    def update_body(node: Node, run: bool):
        nonlocal act
        if run and node.act:
            act |= node.act
        for sid in sorted(node.deliver):
            k = stmt[0]
            stmt[0] += 1
            if run:
                if stmts[k][1] == "Payload":
                    if payload_ok(d, dl):
                        fired.append(k)
                else:
                    fired.append(k)

    def children(node: Node, env: dict, run: bool):
        chain_taken = False
        first_unary = True
        for c in node.kids:
            if c.pred.unary:
                cont = not first_unary
                first_unary = False
            else:
                cont = c.if_else
            if not cont:
                chain_taken = False
            go = run and (not chain_taken or not chains)
            matched = False
            env2 = env
            if trace is not None and run and chain_taken and chains:
                hit = (parse(d, dl, c.pred.proto, env[node.pred.proto]) is not None) if c.pred.unary \
                    else eval_binary(d, env[c.pred.proto], c.pred)
                trace["skipped"] = trace.get("skipped", 0) + int(hit)
            if go:
                if c.pred.unary:
                    h = parse(d, dl, c.pred.proto, env[node.pred.proto])
                    if h is not None:
                        matched = True
                        env2 = dict(env)
                        env2[c.pred.proto] = h
                else:
                    matched = eval_binary(d, env[c.pred.proto], c.pred)
            if matched:
                chain_taken = True
            # statement indices are assigned in code order whether or not the branch runs
            children(c, env2, matched)
            update_body(c, matched)

    root = tree.root
    wraps = any(True for _ in root.kids) and (bool(root.act) or bool(root.deliver) or bool(root.kids))
    eth = parse(d, dl, "ethernet", None)
    run = (eth is not None) if wraps else True
    if root.act or root.deliver:
        update_body(root, run)
    children(root, {"ethernet": eth}, run)
    _ = subs
    return act, fired


def statement_table(tree: PacketTree) -> list[tuple[int, str]]:
    """(subscription id, packet datatype) of every callback site, in generated-code order."""
    out = []

    def body(n: Node):
        for sid in sorted(n.deliver):
            dts = tree.subs[sid].datatypes
            out.append((sid, "Payload" if "Payload" in dts else "ZcFrame"))

    def kids(n: Node):
        for c in n.kids:
            kids(c)
            body(c)

    body(tree.root)
    kids(tree.root)
    return out
