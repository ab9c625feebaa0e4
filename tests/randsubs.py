"""Seeded random subscription sets for the pattern-semantics cross-checks: packet predicates of
every kind the generated code compiles (int ops, ranges, combined addr/port fields, IPv4/IPv6
prefixes, TCP flag accessors), L7 terms that cut patterns at PacketContinue, packet-level and
connection-level datatypes, and shared callback names so that prune_branches' `as_str`
deduplication is exercised. Values are drawn from those the corpora actually hold (tests/corpus.py,
retina_amd/synth.py)."""
from __future__ import annotations

import random

from oracle import filterlang

PORTS = [7, 19, 25, 53, 80, 135, 137, 139, 161, 443, 1234, 1434, 5353, 5714, 8080, 10101, 31789, 31790, 50000]
V4 = ["10.0.0.1", "10.0.0.2", "10.0.0.0/8", "10.1.0.0/16", "3.3.3.3", "3.3.3.3/32", "255.255.255.255",
      "10.18.0.0/16", "0.0.0.0/0", "192.168.0.0/16"]
V6 = ["2001:db8::1", "2001:db8::2", "2001:db8::/32", "::1", "fe80::/10", "::/0"]
L7 = ["tls", "dns", "http", "quic", "ssh", "tls.sni ~ 'x'", "http.user_agent = 'curl'", "dns.query_domain ~ 'a'"]


# every spelling grammar.pest accepts for an operator (core/src/filter/grammar.pest:57-75)
_OPS = {"=": ["="], "!=": ["!=", "ne"], ">=": [">=", "ge"], "<=": ["<=", "le"], ">": [">", "gt"], "<": ["<", "lt"],
        "in": ["in"]}


def _spell(rng: random.Random, pred: str) -> str:
    """Re-spell the operator of `proto.field OP value` with one of its grammar synonyms."""
    parts = pred.split(" ")
    if len(parts) >= 3 and parts[1] in _OPS:
        parts[1] = rng.choice(_OPS[parts[1]])
    return " ".join(parts)


def _pred(rng: random.Random) -> str:
    return _spell(rng, _pred0(rng))


def _pred0(rng: random.Random) -> str:
    k = rng.randrange(14)
    p = rng.choice(PORTS)
    if k == 0:
        return rng.choice(["ipv4", "ipv6", "tcp", "udp"])
    if k == 1:
        return f"{rng.choice(['tcp', 'udp'])}.{rng.choice(['port', 'src_port', 'dst_port'])} {rng.choice(['=', '!=', '>=', '<=', '>', '<'])} {p}"
    if k == 2:
        a = rng.choice(PORTS)
        b = rng.choice([x for x in PORTS if x > a] or [65535])
        return f"{rng.choice(['tcp', 'udp'])}.{rng.choice(['port', 'dst_port'])} in {a}..{b}"
    if k == 3:
        return f"ipv4.{rng.choice(['addr', 'src_addr', 'dst_addr'])} {rng.choice(['=', '!=', 'in'])} {rng.choice(V4)}"
    if k == 4:
        return f"ipv6.{rng.choice(['addr', 'src_addr', 'dst_addr'])} {rng.choice(['=', '!=', 'in'])} {rng.choice(V6)}"
    if k == 5:
        return f"ipv4.time_to_live {rng.choice(['=', '>', '<', '>='])} {rng.choice([1, 64, 220, 255])}"
    if k == 6:
        return f"ipv4.protocol = {rng.choice([1, 2, 6, 17])}"
    if k == 7:
        return f"tcp.{rng.choice(['syn', 'ack', 'fin', 'rst', 'psh', 'urg', 'synack'])} = {rng.choice([0, 1])}"
    if k == 8:
        return f"tcp.flags = {rng.choice([2, 16, 18, 24])}"
    if k == 9:
        return f"udp.length {rng.choice(['>', '=', '<'])} {rng.choice([20, 30, 100])}"
    if k == 10:
        return f"ipv6.{rng.choice(['next_header', 'hop_limit'])} = {rng.choice([6, 17, 64])}"
    if k == 11:
        return f"ipv4.total_length {rng.choice(['=', '<', '>'])} {rng.choice([0, 40, 50, 100])}"
    if k == 12:
        if rng.random() < 0.5:  # an IP literal on a port field compiles (u32::from(u16), utils.rs:52-84)
            return f"{rng.choice(['tcp', 'udp'])}.{rng.choice(['port', 'dst_port'])} {rng.choice(['=', '!='])} {rng.choice(['0.0.0.80', '0.0.0.53', '::50', '1.2.3.4'])}"
        return f"tcp.data_offset {rng.choice(['>', '='])} {rng.choice([5, 6])}"
    return rng.choice(L7)


def _filter(rng: random.Random) -> str:
    if rng.random() < 0.06:
        return ""
    terms = []
    for _ in range(rng.randint(1, 3)):
        conj = f" {rng.choice(['and', 'and', '&&', 'AND'])} ".join(_pred(rng) for _ in range(rng.randint(1, 3)))
        terms.append(f"({conj})" if rng.random() < 0.3 else conj)
    return f" {rng.choice(['or', 'or', '||', 'OR'])} ".join(terms)


DTS = [["ConnRecord"], ["ZcFrame"], ["Payload"], ["ZcFrame", "FilterStr"], ["Payload", "CoreId"],
       ["ZcFrame", "CoreId", "FilterStr"], ["FiveTuple"], ["CoreId", "FilterStr"], ["PktCount"]]


def random_subs(seed: int, max_subs: int = 8) -> list[filterlang.Sub]:
    """A valid subscription set (both compilers must accept it: filters the oracle refuses are
    redrawn)."""
    rng = random.Random(seed)
    out: list[filterlang.Sub] = []
    want = rng.randint(1, max_subs)
    tries = 0
    while len(out) < want and tries < 200:
        tries += 1
        s = filterlang.Sub(_filter(rng), list(rng.choice(DTS)), rng.choice(["cb_a", "cb_b", "cb_c"]))
        try:
            filterlang.PacketTree(out + [s])
        except filterlang.FilterError:
            continue
        out.append(s)
    return out


def to_toml(subs: list[filterlang.Sub]) -> str:
    from retina_amd import synth

    return synth._toml([(s.filter.replace('"', '\\"'), s.datatypes, s.callback) for s in subs])
