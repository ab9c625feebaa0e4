"""ORACLE (test infrastructure only): Retina's filter language and its packet-side predicate trees
(PacketContinue, Packet, PacketDeliver).

Restates, in plain Python:
  core/src/filter/grammar.pest:5-75       the PEG (pest 2.5: ordered choice, greedy repetition,
                                           implicit WHITESPACE = " " | NEWLINE in non-atomic rules)
  core/src/filter/parser.rs:94-357        AST -> disjunctive normal form (flatten_*)
  core/src/filter/ast.rs:19-46, 78-832    LAYERS graph, predicate classes, is_excl / is_child
  core/src/filter/pattern.rs:64-130       to_fully_qualified
  core/src/filter/ptree_flat.rs:91-267    FlatPTree + prune_branches (inside Filter::new)
  core/src/filter/mod.rs:113-139          Filter::new
  core/src/filter/ptree.rs:321-461        PTree::add_filter/build_tree/add_pattern
  core/src/filter/ptree.rs:482-634,752-776 collapse for FilterLayer::PacketContinue
                                           (prune_branches, sort, mark_mutual_exclusion, update_size)
  core/src/filter/datatypes.rs:560-638    should_deliver / packet_continue actions
  datatypes/src/typedefs.rs:15-86         DATATYPES levels
  filtergen/src/lib.rs:241-261            filter_subtree
  filtergen/src/packet_filter.rs, utils.rs:18-379, data.rs:262-331   generated packet_continue
  core/src/filter/ptree.rs:641-748         prune_packet_conditions / prune_redundant_branches
                                           (FilterLayer::Packet and PacketDeliver, ConnTree /
                                           DeliverTree below)
  core/src/filter/datatypes.rs:108-345, 563-637  DataType flags, packet_filter actions,
                                           should_deliver / should_stream at the Packet layer
The Protocol, Session and ConnectionDeliver layers run on the host and are not restated.
"""
from __future__ import annotations

import functools
import ipaddress
import re
from dataclasses import dataclass, field

OPS = ["Eq", "Ne", "Ge", "Le", "Gt", "Lt", "In", "Re", "En", "ByteRe", "Contains", "NotContains"]
OP_TEXT = {"Eq": "=", "Ne": "!=", "Ge": ">=", "Le": "<=", "Gt": ">", "Lt": "<", "In": "in", "Re": "matches",
           "En": "eq", "ByteRe": "~b", "Contains": "contains", "NotContains": "not contains"}
VKINDS = ["Int", "IntRange", "Ipv4", "Ipv6", "Text", "Byte"]


class FilterError(Exception):
    pass


# ----------------------------------------------------------------------------------------------
# values / predicates

@dataclass(frozen=True)
class Value:
    kind: str
    data: tuple

    def key(self):
        if self.kind == "Text":
            return (VKINDS.index(self.kind), (self.data[0].encode(),))
        return (VKINDS.index(self.kind), self.data)

    def __str__(self):
        k, d = self.kind, self.data
        if k == "Int":
            return str(d[0])
        if k == "IntRange":
            return f"{d[0]}..{d[1]}"
        if k == "Ipv4":
            return f"{ipaddress.IPv4Address(d[0])}/{d[1]}"
        if k == "Ipv6":
            return f"{rust_ipv6_str(d[0])}/{d[1]}"
        if k == "Text":
            return d[0]
        return "|" + " ".join(f"{b:02X}" for b in d[0]) + "|"


def rust_ipv6_str(a: int) -> str:
    """std::net::Ipv6Addr Display."""
    segs = [(a >> (112 - 16 * i)) & 0xFFFF for i in range(8)]
    if a == 0:
        return "::"
    if a == 1:
        return "::1"
    if segs[:5] == [0] * 5 and segs[5] == 0xFFFF:
        return "::ffff:" + str(ipaddress.IPv4Address(a & 0xFFFFFFFF))
    best = (0, -1)
    i = 0
    while i < 8:
        if segs[i] == 0:
            j = i
            while j < 8 and segs[j] == 0:
                j += 1
            if j - i > best[0]:
                best = (j - i, i)
            i = j
        else:
            i += 1
    if best[0] > 1:
        s, ln = best[1], best[0]
        return ":".join(f"{x:x}" for x in segs[:s]) + "::" + ":".join(f"{x:x}" for x in segs[s + ln:])
    return ":".join(f"{x:x}" for x in segs)


@functools.total_ordering
@dataclass(frozen=True)
class Pred:
    proto: str
    field: str | None = None   # None for unary
    op: str | None = None
    value: Value | None = None

    @property
    def unary(self) -> bool:
        return self.field is None

    def key(self):
        if self.unary:
            return (0, self.proto)
        return (1, self.proto, self.field, OPS.index(self.op), self.value.key())

    def __lt__(self, other):
        return self.key() < other.key()

    def __str__(self):
        if self.unary:
            return self.proto
        return f"{self.proto}.{self.field} {OP_TEXT[self.op]} {self.value}"


# LAYERS (ast.rs:19-46): inner -> outer
EDGES = {("ipv4", "ethernet"), ("ipv6", "ethernet"), ("tcp", "ipv4"), ("tcp", "ipv6"), ("udp", "ipv4"),
         ("udp", "ipv6"), ("tls", "tcp"), ("http", "tcp"), ("dns", "udp"), ("dns", "tcp"), ("quic", "udp"),
         ("ssh", "tcp")}
NODES = {"ethernet", "ipv4", "ipv6", "tcp", "udp", "tls", "http", "dns", "quic", "ssh"}


def simple_paths(src: str, dst: str) -> list[list[str]]:
    out = []

    def walk(path):
        for (a, b) in EDGES:
            if a != path[-1]:
                continue
            if b == dst:
                out.append(path + [b])
            elif b not in path:
                walk(path + [b])

    walk([src])
    return out


def has_path(a: str, b: str) -> bool:
    return a in NODES and b in NODES and bool(simple_paths(a, b))


def on_packet(p: Pred) -> bool:
    return not (has_path(p.proto, "tcp") or has_path(p.proto, "udp"))


CONN_PROTOCOLS = ("ipv4", "ipv6", "tcp", "udp")                      # protocols/stream/mod.rs:165-167
CONN_FIELDS = ("src_addr", "dst_addr", "src_port", "dst_port")        # stream/conn/layer{3,4}.rs


def req_packet(p: Pred) -> bool:
    """Predicate::req_packet (ast.rs:118-133): needs the raw packet, not connection data."""
    if not on_packet(p):
        return False
    if not p.unary:
        return p.field not in ("port", "addr") and p.field not in CONN_FIELDS
    return p.proto not in CONN_PROTOCOLS


# ----------------------------------------------------------------------------------------------
# is_excl / is_child (ast.rs:215-452 and helpers 455-832)

def _excl_int(f, t, op, pf, pt, pop):
    M = 1 << 64
    if op == "Eq":
        return {"Eq": f != pf, "Ne": f == pf, "In": f < pf or f > pt, "Ge": pf > f, "Le": pf < f,
                "Gt": pf >= f, "Lt": pf <= f}.get(pop, False)
    if op == "Ne":
        return f == pf if pop == "Eq" else False
    if op == "Ge":
        return f > pt if pop in ("Le", "In", "Eq") else (f >= pf if pop == "Lt" else False)
    if op == "Le":
        return f < pf if pop in ("Ge", "In", "Eq") else (f <= pf if pop == "Gt" else False)
    if op == "Gt":
        return f >= pt if pop in ("Le", "In", "Eq") else (f > pf if pop == "Lt" else False)
    if op == "Lt":
        return f <= pf if pop in ("Ge", "In", "Eq") else (f <= (pf + 1) % M if pop == "Gt" else False)
    if op == "In":
        return {"Eq": pf < f or pf > t, "Ge": pf > t, "Gt": pf >= t, "Le": pf < f, "Lt": pf <= f,
                "In": pt < f or pf > t}.get(pop, False)
    return False


def _net(v: Value):
    addr, plen = v.data
    bits = 32 if v.kind == "Ipv4" else 128
    mask = ((1 << bits) - 1) ^ ((1 << (bits - plen)) - 1) if plen else 0
    return addr & mask, addr | (((1 << bits) - 1) ^ mask)


def _contains(a: Value, b: Value) -> bool:   # ipnet Contains<&Net>
    an, ab = _net(a)
    bn, bb = _net(b)
    return an <= bn and bb <= ab


def _excl_ip(a, op, b, pop):
    if op in ("Eq", "In"):
        if pop in ("Eq", "In"):
            return not _contains(b, a) and not _contains(a, b)
        if pop == "Ne":
            return a == b
        return False
    if op == "Ne" and pop in ("Eq", "In"):
        return a == b
    return False


def _re_search(pat: str, txt: str) -> bool:
    try:
        return re.search(pat, txt) is not None
    except re.error as e:
        raise FilterError(f"Invalid Regex string {pat}: {e}")


def _excl_text(t, op, pt, pop):
    if op == "Eq" and pop == "Eq":
        return pt != t
    if (op, pop) in (("Ne", "Eq"), ("Eq", "Ne")):
        return pt == t
    if "Ne" in (op, pop):
        return False
    if op == "Re" and pop == "Re":
        return False
    if op == "Contains" and pop == "Eq":
        return t not in pt
    if op == "Eq" and pop == "Contains":
        return pt not in t
    if op == "Contains" and pop == "Contains":
        return False
    if (op, pop) in (("Re", "Contains"), ("Contains", "Re")):
        return False
    rx, tx = (t, pt) if op == "Re" else (pt, t)
    return not _re_search(rx, tx)


def _find(needle: bytes, hay: bytes) -> bool:
    return needle in hay


def _excl_byte(b, op, pb, pop):
    if op == "Eq" and pop == "Eq":
        return pb != b
    if (op, pop) in (("Ne", "Eq"), ("Eq", "Ne")):
        return pb == b
    if "Ne" in (op, pop):
        return False
    if op == "Contains" and pop == "Eq":
        return not _find(b, pb)
    if op == "Eq" and pop == "Contains":
        return not _find(pb, b)
    return False


def is_excl(a: Pred, b: Pred) -> bool:
    if a.unary and b.unary:
        return True
    if a.unary != b.unary or a.proto != b.proto or a.field != b.field:
        return False
    va, vb = a.value, b.value
    ints = ("Int", "IntRange")
    if va.kind in ints:
        if vb.kind not in ints:
            return False
        f, t = (va.data[0], va.data[0]) if va.kind == "Int" else va.data
        pf, pt = (vb.data[0], vb.data[0]) if vb.kind == "Int" else vb.data
        return _excl_int(f, t, a.op, pf, pt, b.op)
    if va.kind in ("Ipv4", "Ipv6"):
        return vb.kind == va.kind and _excl_ip(va, a.op, vb, b.op)
    if va.kind == "Text":
        return vb.kind == "Text" and _excl_text(va.data[0], a.op, vb.data[0], b.op)
    if va.kind == "Byte":
        return vb.kind == "Byte" and _excl_byte(bytes(va.data[0]), a.op, bytes(vb.data[0]), b.op)
    return False


def _parent_int(cf, ct, cop, pf, pt, pop):
    if cop in ("Eq", "In"):
        return {"Ge": pf <= cf, "Gt": pf < cf, "Le": pf >= ct, "Lt": pf > ct,
                "In": pf <= cf and pt >= ct}.get(pop, False)
    if cop == "Ge":
        return pf < cf if pop in ("Ge", "Gt") else False
    if cop == "Le":
        return pf > cf if pop in ("Le", "Lt") else False
    if cop == "Gt":
        return pf <= cf if pop in ("Gt", "Ge") else False
    if cop == "Lt":
        return pf >= cf if pop in ("Le", "Lt") else False
    return False


def is_child(c: Pred, p: Pred) -> bool:
    """`c` is a strict subset of `p` (ast.rs:312-452)."""
    if c.proto != p.proto or c == p:
        return False
    if not c.unary and not p.unary:
        if c.field != p.field:
            return False
        cop, pop = c.op, p.op
        if pop == "Ne":
            return False
        if pop == "Eq" and p.value.kind not in ("Ipv4", "Ipv6"):
            return False
        if "Ne" in (cop, pop) or "En" in (cop, pop):
            return False
        if cop == "Re" and pop == "Re":
            return False
        if cop in ("Ge", "Gt") and pop in ("Le", "Lt"):
            return False
        if pop in ("Ge", "Gt") and cop in ("Le", "Lt"):
            return False
        vc, vp = c.value, p.value
        ints = ("Int", "IntRange")
        if vc.kind in ints:
            if vp.kind not in ints:
                return False
            cf, ct = (vc.data[0], vc.data[0]) if vc.kind == "Int" else vc.data
            pf, pt = (vp.data[0], vp.data[0]) if vp.kind == "Int" else vp.data
            return _parent_int(cf, ct, cop, pf, pt, pop)
        if vc.kind in ("Ipv4", "Ipv6"):
            if vp.kind != vc.kind:
                return False
            if cop in ("Eq", "In"):
                return _contains(vp, vc) if pop in ("Eq", "In") else False
            if cop == "Ne":
                return _contains(vp, vc) if pop == "Ne" else False
            return False
        if vc.kind == "Text":
            if vp.kind != "Text":
                return False
            if pop == "Contains" and cop in ("Eq", "Contains"):
                return vp.data[0] in vc.data[0]
            if pop != "Re" or cop != "Eq":
                return False
            return _re_search(vp.data[0], vc.data[0])
        if vc.kind == "Byte":
            if vp.kind != "Byte":
                return False
            if pop == "Contains" and cop in ("Eq", "Contains"):
                return _find(bytes(vp.data[0]), bytes(vc.data[0]))
            return False
        return False
    return (not c.unary) and p.unary


# ----------------------------------------------------------------------------------------------
# parser: grammar.pest as a PEG over the raw string

_WS = " \n\r"


class _P:
    def __init__(self, s: str):
        self.s = s

    def ws(self, i):
        while i < len(self.s) and self.s[i] in _WS:
            i += 1
        return i

    def lit(self, i, t):
        return i + len(t) if self.s.startswith(t, i) else None

    def ident(self, i):
        m = re.compile(r"[A-Za-z][A-Za-z0-9_]*").match(self.s, i)
        return m.end() if m else None

    # filter = _{ SOI ~ expr? ~ EOI }
    def top(self):
        i = self.ws(0)
        r = self.expr(i)
        node = ("or", [])
        if r is not None:
            node, j = r
            i = self.ws(j)
        if i != len(self.s):
            raise FilterError("Invalid filter format")
        return node

    def expr(self, i):
        r = self.sub(i)
        if r is None:
            return None
        terms = [r[0]]
        i = r[1]
        while True:
            j = self.ws(i)
            k = None
            for t in ("||", "or", "OR"):
                k = self.lit(j, t)
                if k is not None:
                    break
            if k is None:
                break
            r = self.sub(self.ws(k))
            if r is None:
                break
            terms.append(r[0])
            i = r[1]
        return ("or", terms), i

    def sub(self, i):
        items = []
        r = self.term(i)
        if r is None:
            return None
        items += r[0]
        i = r[1]
        while True:
            j = self.ws(i)
            k = None
            for t in ("&&", "and", "AND"):
                k = self.lit(j, t)
                if k is not None:
                    break
            if k is None:
                break
            r = self.term(self.ws(k))
            if r is None:
                break
            items += r[0]
            i = r[1]
        return ("and", items), i

    def term(self, i):
        r = self.predicate(i)
        if r is not None:
            return r
        if self.lit(i, "(") is not None:
            r = self.expr(self.ws(i + 1))
            if r is not None:
                j = self.ws(r[1])
                if self.lit(j, ")") is not None:
                    return [r[0]], j + 1
        return None

    def predicate(self, i):
        j = self.ident(i)
        if j is None:
            return None
        proto = self.s[i:j]
        got = self.binary_tail(j)
        if got is None:
            return [Pred(proto)], j
        (field_name, combined, op, val), end = got
        if not combined:
            return [Pred(proto, field_name, op, val)], end
        src = Pred(proto, "src_" + field_name, op, val)
        dst = Pred(proto, "dst_" + field_name, op, val)
        if op == "Ne":
            return [src, dst], end
        return [("or", [("and", [src]), ("and", [dst])])], end

    def binary_tail(self, j):
        g = self.ws(j)
        if self.lit(g, ".") is None:
            return None
        f0 = self.ws(g + 1)
        combined = False
        if self.s.startswith("addr", f0) or self.s.startswith("port", f0):
            f1, combined = f0 + 4, True
        else:
            f1 = self.ident(f0)
            if f1 is None:
                return None
        r = self.binop(self.ws(f1))
        if r is None:
            return None
        op, o1 = r
        r = self.value(self.ws(o1))
        if r is None:
            return None
        val, end = r
        return (self.s[f0:f1], combined, op, val), end

    BINOPS = [("=", "Eq"), ("!=", "Ne"), ("ne", "Ne"), (">=", "Ge"), ("ge", "Ge"), ("<=", "Le"), ("le", "Le"),
              (">", "Gt"), ("gt", "Gt"), ("<", "Lt"), ("lt", "Lt"), ("in", "In"), ("~b", "ByteRe"), ("~", "Re"),
              ("matches", "Re"), ("eq", "En"), ("contains", "Contains"), ("!contains", "NotContains"),
              ("not contains", "NotContains")]

    def binop(self, i):
        for t, op in self.BINOPS:
            if self.s.startswith(t, i):
                return op, i + len(t)
        return None

    _IPV4 = re.compile(r"[0-9]{1,3}(\.[0-9]{1,3}){3}")

    def ipv6_span(self, i):
        s = self.s
        if i < len(s) and s[i] == ":":
            i += 1
        else:
            m = re.compile(r"[A-Za-z0-9]{1,4}").match(s, i)
            if not m:
                return None
            i = m.end()
        if i >= len(s) or s[i] != ":":
            return None
        i += 1
        while True:
            m = self._IPV4.match(s, i)
            if m:
                i = m.end()
                continue
            m = re.compile(r"[A-Za-z0-9]{1,4}").match(s, i)
            if m:
                i = m.end()
                continue
            if i < len(s) and s[i] == ":":
                i += 1
                continue
            return i

    def value(self, i):
        s = self.s
        m = self._IPV4.match(s, i)
        if m:
            addr = m.group(0)
            end = m.end()
            prefix = 32
            m2 = re.compile(r"/([0-9]{1,2})").match(s, end)
            if m2:
                prefix, end = int(m2.group(1)), m2.end()
            a = rust_parse_ipv4(addr)
            if a is None:
                raise FilterError("Invalid Address")
            if prefix > 32:
                raise FilterError("Invalid Prefix Len")
            return Value("Ipv4", (a, prefix)), end
        j = self.ipv6_span(i)
        if j is not None:
            end = j
            prefix = 128
            m2 = re.compile(r"/([0-9]{1,3})").match(s, end)
            if m2:
                prefix, end = int(m2.group(1)), m2.end()
                if prefix > 255:
                    raise FilterError("Invalid Integer")
            a = rust_parse_ipv6(s[i:j])
            if a is None:
                raise FilterError("Invalid Address")
            if prefix > 128:
                raise FilterError("Invalid Prefix Len")
            return Value("Ipv6", (a, prefix)), end
        m = re.compile(r"[0-9]+").match(s, i)
        if m:
            m2 = re.compile(r"\.\.([0-9]+)").match(s, m.end())
            if m2:
                a, b = int(m.group(0)), int(m2.group(1))
                if a >= 1 << 64 or b >= 1 << 64:
                    raise FilterError("Invalid Integer")
                if a >= b:
                    raise FilterError(f"Invalid Range: {a}..{b}")
                return Value("IntRange", (a, b)), m2.end()
            v = int(m.group(0))
            if v >= 1 << 64:
                raise FilterError("Invalid Integer")
            return Value("Int", (v,)), m.end()
        if i < len(s) and s[i] == "|":
            r = self.byte_lit(i)
            if r is not None:
                return r
        if i < len(s) and s[i] == "'":
            r = self.text(i)
            if r is not None:
                return r
        return None

    def byte_lit(self, i):
        s = self.s
        hexd = "0123456789abcdefABCDEF"
        r = i + 1
        n = 0
        while True:
            t = self.ws(r)
            if t < len(s) and s[t] == "|":
                break
            if t >= len(s) or s[t] not in hexd:
                break
            t3 = self.ws(t + 1)
            if t3 >= len(s) or s[t3] not in hexd:
                break
            t4 = self.ws(t3 + 1)
            if t4 < len(s) and s[t4] == " ":
                t4 += 1
            r = t4
            n += 1
        if n == 0:
            return None
        t = self.ws(r)
        if t >= len(s) or s[t] != "|":
            return None
        raw = s[i:t + 1]
        out = []
        for tok in raw.replace("|", "").split():
            v = int(tok, 16)
            if v > 255:
                raise FilterError(f"Failed to parse {tok} in {raw}")
            out.append(v)
        return Value("Byte", (tuple(out),)), t + 1

    def text(self, i):
        s = self.s
        t0 = self.ws(i + 1)
        cur = t0
        it = 0
        while True:
            save = cur
            a = self.ws(cur) if it else cur
            if a < len(s) and s[a] == "'":
                cur = save
                break
            a = self.ws(a)
            if a >= len(s):
                cur = save
                break
            cur = a + 1
            it += 1
        if it == 0:
            return None
        e = self.ws(cur)
        if e < len(s) and s[e] == "'":
            return Value("Text", (s[t0:cur],)), e + 1
        return None


def rust_parse_ipv4(t: str):
    parts = t.split(".")
    if len(parts) != 4:
        return None
    v = 0
    for p in parts:
        if not p or len(p) > 3 or not p.isdigit() or (len(p) > 1 and p[0] == "0") or int(p) > 255:
            return None
        v = (v << 8) | int(p)
    return v


def rust_parse_ipv6(t: str):
    """core::net::parser::read_ipv6_addr semantics (strict; embedded IPv4 allowed at the end)."""
    pos = [0]

    def num(radix, maxd, zero_prefix, maxv):
        i = pos[0]
        j = i
        v = 0
        digits = "0123456789abcdef"
        while j < len(t) and j - i < maxd and t[j].lower() in digits[:radix]:
            v = v * radix + digits.index(t[j].lower())
            if v > maxv:
                return None
            j += 1
        if j == i or (not zero_prefix and t[i] == "0" and j - i > 1):
            return None
        pos[0] = j
        return v

    def v4():
        save = pos[0]
        a = 0
        for k in range(4):
            if k:
                if pos[0] >= len(t) or t[pos[0]] != ".":
                    pos[0] = save
                    return None
                pos[0] += 1
            o = num(10, 3, False, 255)
            if o is None:
                pos[0] = save
                return None
            a = (a << 8) | o
        return a

    def groups(limit):
        g = []
        for i in range(limit):
            if i < limit - 1:
                save = pos[0]
                ok = True
                if i > 0:
                    if pos[0] < len(t) and t[pos[0]] == ":":
                        pos[0] += 1
                    else:
                        ok = False
                a = v4() if ok else None
                if a is not None:
                    return g + [a >> 16, a & 0xFFFF], True
                pos[0] = save
            save = pos[0]
            if i > 0:
                if pos[0] < len(t) and t[pos[0]] == ":":
                    pos[0] += 1
                else:
                    return g, False
            x = num(16, 4, True, 0xFFFF)
            if x is None:
                pos[0] = save
                return g, False
            g.append(x)
        return g, False

    head, h4 = groups(8)
    if len(head) < 8:
        if h4 or not t.startswith("::", pos[0]):
            return None
        pos[0] += 2
        tail, _ = groups(8 - (len(head) + 1))
        head = head + [0] * (8 - len(head) - len(tail)) + tail
    if pos[0] != len(t):
        return None
    v = 0
    for x in head:
        v = (v << 16) | x
    return v


def _flatten_or(node) -> list[list[Pred]]:
    out = []
    for conj in node[1]:
        out += _flatten_and(conj)
    return out


def _flatten_and(node) -> list[list[Pred]]:
    flat = [[]]
    for t in node[1]:
        if isinstance(t, Pred):
            for f in flat:
                f.append(t)
        else:
            dis = _flatten_or(t)
            cur = [list(f) for f in flat]
            flat = [c + d for d in dis for c in cur]
    return flat


def parse_filter(s: str) -> list[list[Pred]]:
    """FilterParser::parse_filter (parser.rs:94-97)."""
    return _flatten_or(_P(s).top())


# ----------------------------------------------------------------------------------------------
# Filter::new

def fully_qualified(preds: list[Pred]) -> list[list[Pred]]:
    """pattern.rs:64-130; returns flat fully-qualified patterns, sorted."""
    if not preds:
        return []
    headers = {p.proto for p in preds}
    paths = set()
    for h in headers:
        if h not in NODES:
            raise FilterError(f"Predicate header invalid: {h}")
        for p in simple_paths(h, "ethernet"):
            paths.add(tuple(reversed(p[:-1])))
    out = []
    for path in paths:
        if not headers <= set(path):
            continue
        flat = []
        for proto in path:
            flat.append(Pred(proto))
            flat += sorted({p for p in preds if p.proto == proto and not p.unary})
        out.append(flat)
    if not out:
        raise FilterError("Invalid pattern. Contains unsupported layer encapsulation: [" +
                          ", ".join(map(str, preds)) + "]")
    return sorted(out, key=lambda f: [p.key() for p in f])


def filter_patterns(s: str) -> list[list[Pred]]:
    """Filter::new(s).get_patterns_flat() (mod.rs:113-152)."""
    fq = []
    for raw in parse_filter(s):
        fq += fully_qualified(raw)
    uniq = []
    for f in sorted(fq, key=lambda f: [p.key() for p in f]):
        if not uniq or uniq[-1] != f:
            uniq.append(f)
    # FlatPTree: exact-match trie, terminal nodes drop their children
    root = {"kids": [], "term": False}
    for f in uniq:
        n = root
        for p in f:
            nxt = next((k for k in n["kids"] if k["pred"] == p), None)
            if nxt is None:
                nxt = {"pred": p, "kids": [], "term": False}
                n["kids"].append(nxt)
            n = nxt
        n["term"] = True
    if not root["kids"]:
        root["term"] = True
    out = []

    def walk(n, acc):
        if n["term"]:
            out.append(list(acc))
            return
        for k in n["kids"]:
            walk(k, acc + [k["pred"]])

    walk(root, [])
    res = []
    for f in out:
        res += fully_qualified(f)
    return res


# ----------------------------------------------------------------------------------------------
# subscriptions

CONNECTION_DT = {"ConnRecord", "ConnDuration", "PktCount", "ByteCount", "InterArrivals", "ConnHistory",
                 "SessionList", "BidirZcPktStream", "OrigZcPktStream", "RespZcPktStream",
                 "OrigZcPktsReassembled", "RespZcPktsReassembled", "BidirPktStream", "OrigPktStream",
                 "RespPktStream", "OrigPktsReassembled", "RespPktsReassembled"}
SESSION_DT = {"HttpTransaction", "DnsTransaction", "TlsHandshake", "QuicStream", "SshHandshake"}
PACKET_DT = {"ZcFrame", "Payload"}
STATIC_DT = {"CoreId", "FiveTuple", "EtherTCI", "EthAddr", "FilterStr"}


@dataclass
class Sub:
    filter: str
    datatypes: list[str]
    callback: str = "cb"
    streaming: bool = False

    @property
    def level(self) -> str:
        """SubscriptionSpec.level after add_datatype (datatypes.rs:433-443, 507-512)."""
        if self.streaming:
            return "Streaming"
        lvl = "Static"
        for d in self.datatypes:
            if lvl == "Connection":
                break
            dl = dt_level(d)
            if lvl == "Connection" or dl == "Connection":
                lvl = "Connection"
            elif lvl == "Session" or dl == "Session":
                lvl = "Session"
            elif lvl == "Packet" or dl == "Packet":
                lvl = "Packet"
        return lvl

    @property
    def as_str(self) -> str:
        return f"{self.callback}({', '.join(self.datatypes)})"


def dt_level(d: str) -> str:
    if d in CONNECTION_DT:
        return "Connection"
    if d in SESSION_DT:
        return "Session"
    if d in PACKET_DT:
        return "Packet"
    if d in STATIC_DT:
        return "Static"
    raise FilterError(f"Invalid datatype: {d}")


def validate(sub: Sub) -> None:
    """validate_spec (datatypes.rs:449-504) + build_packet_params restrictions (data.rs:262-297)."""
    lv = [dt_level(d) for d in sub.datatypes]
    if not sub.datatypes:
        raise FilterError("subscription without datatypes")
    if sub.level == "Packet":
        if len(lv) > 1 and (lv.count("Packet") != 1 or lv.count("Static") < len(lv) - 1):
            raise FilterError("bad packet-level subscription")
        for d in sub.datatypes:
            if dt_level(d) != "Packet" and d not in ("FilterStr", "CoreId"):
                raise FilterError(f"Invalid datatype in packet callback: {d}")
    elif "Packet" in lv:
        raise FilterError("Packet-level datatype in non-packet subscription")
    if sub.streaming and sum(x in ("Connection", "Packet") for x in lv) != 1:
        raise FilterError("Must have one streamable datatype in streaming subscription")
    if lv.count("Session") > 1:
        raise FilterError("Multiple session-level datatypes in subscription")
    check_after_packet_layer(sub)


def check_after_packet_layer(sub: Sub) -> None:
    """filtergen builds the FilterLayer::Packet tree for every subscription (lib.rs:284); its
    add_pattern panics on a per-packet field (ptree.rs:406-415) in any pattern that is not
    already resolved at PacketContinue (FlatPattern::is_prev_layer, pattern.rs:53-61: all of a
    packet-level subscription's predicates on_packet), up to the first predicate of a later layer."""
    for pat in filter_patterns(sub.filter):
        if sub.level == "Packet" and all(on_packet(p) for p in pat):
            continue
        for p in pat:
            if not on_packet(p):
                break
            if req_packet(p):
                raise FilterError("Cannot access per-packet fields (e.g., TCP flags, length) after packet filter.")


def load_spec(text: str) -> list[Sub]:
    """The #[subscription("spec.toml")] format (filtergen/src/parse.rs:7-66)."""
    try:
        import tomllib  # py>=3.11
    except ImportError:  # pragma: no cover
        import tomli as tomllib
    d = tomllib.loads(text)
    subs = []
    for s in d.get("subscriptions", []):
        dts = s["datatypes"]
        if isinstance(dts, str):
            dts = [dts]
        sub = Sub(s["filter"], list(dts), s["callback"], "streaming" in s)
        validate(sub)
        subs.append(sub)
    return subs


# ----------------------------------------------------------------------------------------------
# PacketContinue tree

PC = 1  # ActionData::PacketContinue


@dataclass
class Node:
    pred: Pred
    id: int = 0
    act: int = 0
    deliver: dict = field(default_factory=dict)   # id -> (as_str, must_deliver)
    kids: list = field(default_factory=list)
    if_else: bool = False

    def label(self) -> str:
        """PNode Display (ptree.rs:246-274), delivers in ascending id."""
        s = str(self.pred)
        if self.act:
            s += " -- A: Actions { data: [PacketContinue], terminal_actions: [] }"
        if self.deliver:
            s += " D: ( " + "".join(self.deliver[k][0] + ", " for k in sorted(self.deliver)) + ")"
        if self.if_else:
            s += " x"
        return s


def _paths(n: Node) -> list[str]:
    out = []

    def rec(node, acc):
        if not node.kids and acc:
            out.append(",".join(acc))
            return
        for k in node.kids:
            rec(k, acc + [k.label()])

    rec(n, [])
    return out


def _outcome_eq(a: Node, b: Node) -> bool:
    if a.act != b.act or a.deliver != b.deliver:
        return False
    if not a.kids and not b.kids:
        return True
    return _paths(a) == _paths(b)


def _sort_key_cmp(a: Node, b: Node) -> int:
    if not a.pred.unary and not b.pred.unary and a.pred.proto == b.pred.proto:
        return (a.pred.field > b.pred.field) - (a.pred.field < b.pred.field)
    return (a.pred.proto > b.pred.proto) - (a.pred.proto < b.pred.proto)


def _stable_sort(nodes: list) -> list:
    out = list(nodes)
    if len(out) <= 20:
        for i in range(1, len(out)):      # insertion sort (Rust slice::sort, len <= 20)
            x = out[i]
            j = i
            while j > 0 and _sort_key_cmp(x, out[j - 1]) < 0:
                j -= 1
            out[i:i + 1] = []
            out.insert(j, x)
        return out
    return sorted(out, key=functools.cmp_to_key(_sort_key_cmp))


class PacketTree:
    """PTree for FilterLayer::PacketContinue built by filter_subtree + collapse."""

    def __init__(self, subs: list[Sub]):
        self.subs = subs
        self.root = Node(Pred("ethernet"))
        self.size = 1
        for sid, sub in enumerate(subs):
            validate(sub)
            self._add_filter(sid, sub, filter_patterns(sub.filter))
        self._collapse()

    # ptree.rs:344-385 / 389-461 specialised to PacketContinue
    def _add_filter(self, sid, sub, patterns):
        is_pkt = sub.level == "Packet"
        deliver = (sub.as_str, "FilterStr" in sub.datatypes)
        added = False
        for pat in patterns:
            added = added or bool(pat)
            self._add_pattern(sid, is_pkt, deliver, pat)
        if not added:
            if is_pkt:                       # should_deliver(ethernet): on_packet
                self.root.deliver[sid] = deliver
            else:
                self.root.act |= PC

    def _add_pattern(self, sid, is_pkt, deliver, pat):
        node = self.root
        for p in pat:
            if not on_packet(p):
                node.act |= PC               # with_nonterm_filter(PacketContinue)
                return
            d = self._descendant(node, p)
            if d is not None:
                node = d
                continue
            par = self._narrowest_parent(node, p)
            if par is not None:
                node = par
            moved = [k for k in node.kids if is_child(k.pred, p)]
            node.kids = [k for k in node.kids if not is_child(k.pred, p)]
            nxt = next((k for k in node.kids if k.pred == p), None)
            if nxt is None:
                nxt = Node(p, id=self.size)
                self.size += 1
                node.kids.append(nxt)
            nxt.kids += moved
            node = nxt
        if is_pkt:
            node.deliver[sid] = deliver      # should_deliver at PacketContinue = on_packet
        else:
            node.act |= PC                   # with_term_filter(PacketContinue)

    @staticmethod
    def _descendant(node, p):
        for k in node.kids:
            if k.pred == p:
                return k
            if is_child(p, k.pred):
                r = PacketTree._descendant(k, p)
                if r is not None:
                    return r
        return None

    @staticmethod
    def _narrowest_parent(node, p):
        cur = None
        n = node
        while True:
            cand = next((k for k in n.kids if is_child(p, k.pred)), None)
            if cand is None:
                return cur
            cur = cand
            n = cand

    def _collapse(self):
        # prune_branches (ptree.rs:570-634)
        def prune(n, on_act, on_d):
            my_d = set(on_d)
            keep = {}
            for k in sorted(n.deliver):
                s, must = n.deliver[k]
                if s not in my_d:
                    my_d.add(s)
                    keep[k] = n.deliver[k]
                elif must:
                    keep[k] = n.deliver[k]
            n.deliver = keep
            my_act = on_act
            if n.act:
                n.act &= ~on_act
                my_act |= n.act
            for k in n.kids:
                prune(k, my_act, my_d)
            n.kids = [k for k in n.kids if k.act or k.kids or k.deliver]

        prune(self.root, 0, set())

        def srt(n):
            for k in n.kids:
                srt(k)
            n.kids = _stable_sort(n.kids)

        srt(self.root)

        def mark(n):
            for i, k in enumerate(n.kids):
                mark(k)
                if i == 0:
                    continue
                if is_excl(k.pred, n.kids[i - 1].pred):
                    k.if_else = True
                if _outcome_eq(k, n.kids[i - 1]):
                    k.if_else = True

        mark(self.root)
        counter = [0]

        def number(n):
            n.id = counter[0]
            counter[0] += 1
            for k in n.kids:
                number(k)

        number(self.root)
        self.size = counter[0]

    def to_filter_string(self) -> str:
        """PTree::to_filter_string (ptree.rs:841-870): root-to-leaf paths, "and"-joined
        predicates in parentheses, paths "or"-joined; "" for a childless root."""
        if not self.root.kids:
            return ""
        out = []

        def rec(n, curr):
            curr = "(" if not curr else curr + f"({n.pred})"
            if not n.kids:
                out.append(curr + ")")
                return
            if curr != "(":
                curr += " and "
            for k in n.kids:
                rec(k, curr)

        rec(self.root, "")
        return " or ".join(out)

    def pprint(self) -> str:
        lines = []

        def rec(n, prefix, last):
            lines.append(prefix + ("`- " if last else "|- ") + f"{n.id}: {n.label()}")
            for i, k in enumerate(n.kids):
                rec(k, prefix + ("   " if last else "|  "), i == len(n.kids) - 1)

        rec(self.root, "", True)
        return "Tree Pkt (pass)\n," + "\n".join(lines) + "\n"


# ----------------------------------------------------------------------------------------------
# PacketDeliver tree (FilterLayer::PacketDeliver): filter_subtree + collapse for the packet
# deliver filter. Only packet-level subscriptions take part (ptree.rs:330-333); no layer stops
# a pattern and no actions are attached (with_term_filter / with_nonterm_filter are empty there,
# datatypes.rs:704-721), so a node carries its predicate and its deliveries only.

def _node_label(n: Node) -> str:
    s = str(n.pred)
    if n.deliver:
        s += " D: ( " + "".join(n.deliver[k][0] + ", " for k in sorted(n.deliver)) + ")"
    if n.if_else:
        s += " x"
    return s


def _paths_lbl(n: Node) -> list[str]:
    out = []

    def rec(node, acc):
        if not node.kids and acc:
            out.append(",".join(acc))
            return
        for k in node.kids:
            rec(k, acc + [_node_label(k)])

    rec(n, [])
    return out


def _all_paths_eq(a: Node, b: Node) -> bool:
    if not a.kids and not b.kids:
        return True
    return _paths_lbl(a) == _paths_lbl(b)


def _windows_all_excl(kids: list) -> bool:
    return all(is_excl(kids[k - 1].pred, kids[k].pred) for k in range(1, len(kids)))


class DeliverTree:
    """PTree for FilterLayer::PacketDeliver built by filter_subtree + collapse (ptree.rs)."""

    def __init__(self, subs: list[Sub]):
        self.subs = subs
        self.root = Node(Pred("ethernet"))
        self.size = 1
        for sid, sub in enumerate(subs):
            validate(sub)
            if sub.level != "Packet":       # add_filter (ptree.rs:330-333)
                continue
            self._build(sid, sub, filter_patterns(sub.filter))
        self._collapse()

    # build_tree (ptree.rs:344-385): a pattern whose predicates all resolve at an earlier layer
    # (for a packet-level subscription: all on_packet, ast.rs pred_is_prev_layer) is skipped --
    # it was delivered at PacketContinue; nothing is attached to the root for PacketDeliver
    def _build(self, sid, sub, patterns):
        deliver = (sub.as_str, "FilterStr" in sub.datatypes)
        for pat in patterns:
            if all(on_packet(p) for p in pat):
                continue
            self._add_pattern(sid, deliver, pat)

    # add_pattern (ptree.rs:389-461)
    def _add_pattern(self, sid, deliver, pat):
        node = self.root
        for p in pat:
            if req_packet(p):
                raise FilterError("Cannot access per-packet fields (e.g., TCP flags, length) after packet filter.")
            d = PacketTree._descendant(node, p)
            if d is not None:
                node = d
                continue
            par = PacketTree._narrowest_parent(node, p)
            if par is not None:
                node = par
            moved = [k for k in node.kids if is_child(k.pred, p)]
            node.kids = [k for k in node.kids if not is_child(k.pred, p)]
            nxt = next((k for k in node.kids if k.pred == p), None)
            if nxt is None:
                nxt = Node(p, id=self.size)
                self.size += 1
                node.kids.append(nxt)
            nxt.kids += moved
            node = nxt
        node.deliver[sid] = deliver          # should_deliver(PacketDeliver) for packet-level data

    @staticmethod
    def _extracts_protocol(n: Node) -> bool:
        """ptree.rs:206-222 at PacketDeliver."""
        if n.pred.unary and any(k.pred.unary for k in n.kids):
            return True
        if not n.pred.unary:
            return False
        return any(k.pred.proto == n.pred.proto and not k.pred.unary for k in n.kids)

    def _collapse(self):
        # ptree.rs:752-767: one possible callback needs no condition
        seen: dict = {}

        def single(n):
            for k, v in n.deliver.items():
                seen[k] = v
            if len(seen) > 1:
                return
            for c in n.kids:
                single(c)

        single(self.root)
        if len(seen) == 1:
            self.root = Node(Pred("ethernet"), deliver=dict(seen))
            self.size = 1
            return

        # prune_redundant_branches (ptree.rs:693-748); every predicate is a previous layer's here
        def redundant(n, can_prune):
            nxt = _windows_all_excl(n.kids)
            for c in n.kids:
                redundant(c, nxt)
            if not can_prune:
                return
            must, could = [], []
            for c in n.kids:
                (must if c.deliver or self._extracts_protocol(c) else could).append(c)
            nc = []
            for c in could:
                if all(_all_paths_eq(c, o) for o in n.kids):
                    nc += c.kids
                else:
                    nc.append(c)
            nc += must
            nc = _stable_sort(nc)
            dd = []
            for c in nc:
                if not dd or not (dd[-1].pred == c.pred and dd[-1].deliver == c.deliver):
                    dd.append(c)
            n.kids = dd

        redundant(self.root, _windows_all_excl(self.root.kids))

        # prune_packet_conditions (ptree.rs:641-687)
        def packet_conds(n, can_prune):
            if not on_packet(n.pred):
                return
            nxt = _windows_all_excl(n.kids)
            for c in n.kids:
                packet_conds(c, nxt)
            if not can_prune:
                return
            while len(n.kids) == 1 and on_packet(n.kids[0].pred):
                c = n.kids[0]
                if self._extracts_protocol(c):
                    break
                n.deliver.update(c.deliver)
                n.kids = c.kids

        packet_conds(self.root, _windows_all_excl(self.root.kids))

        # prune_branches (ptree.rs:570-634), deliveries only
        def prune(n, on_d):
            my_d = set(on_d)
            keep = {}
            for k in sorted(n.deliver):
                s, must = n.deliver[k]
                if s not in my_d:
                    my_d.add(s)
                    keep[k] = n.deliver[k]
                elif must:
                    keep[k] = n.deliver[k]
            n.deliver = keep
            for c in n.kids:
                prune(c, my_d)
            n.kids = [c for c in n.kids if c.kids or c.deliver]

        prune(self.root, set())

        def srt(n):
            for c in n.kids:
                srt(c)
            n.kids = _stable_sort(n.kids)

        srt(self.root)

        def mark(n):
            for i, c in enumerate(n.kids):
                mark(c)
                if i == 0:
                    continue
                prev = n.kids[i - 1]
                if is_excl(c.pred, prev.pred):
                    c.if_else = True
                if c.deliver == prev.deliver and _all_paths_eq(c, prev):
                    c.if_else = True

        mark(self.root)
        counter = [0]

        def number(n):
            n.id = counter[0]
            counter[0] += 1
            for c in n.kids:
                number(c)

        number(self.root)
        self.size = counter[0]

    def structure(self, n: Node | None = None):
        """(predicate text, delivered subscription ids, if_else, children) for comparisons."""
        n = self.root if n is None else n
        return (str(n.pred), sorted(n.deliver), n.if_else, [self.structure(c) for c in n.kids])

    def to_json(self, n: Node | None = None) -> dict:
        """The tree in the shape of the compiler's JSON export (Program.tree_json)."""
        n = self.root if n is None else n
        return {"id": n.id, "pred": str(n.pred), "unary": n.pred.unary, "protocol": n.pred.proto, "data": 0,
                "terminal": 0, "if_else": n.if_else, "deliver": sorted(n.deliver), "stream": [],
                "children": [self.to_json(c) for c in n.kids]}


# ----------------------------------------------------------------------------------------------
# Packet-layer tree (FilterLayer::Packet): the first-packet `packet_filter` tree. Subscriptions
# attach the actions of SubscriptionSpec::packet_filter (datatypes.rs:306-345, 626-637) and
# deliver static-only data on the first packet (datatypes.rs:226-236).

ACT = {"PacketContinue": 1 << 0, "PacketDeliver": 1 << 1, "PacketCache": 1 << 2, "PacketTrack": 1 << 3,
       "ProtoProbe": 1 << 4, "ProtoFilter": 1 << 5, "SessionFilter": 1 << 6, "SessionDeliver": 1 << 7,
       "SessionTrack": 1 << 8, "UpdatePDU": 1 << 9, "Reassemble": 1 << 10, "ConnDeliver": 1 << 11,
       "Stream": 1 << 12}   # actions.rs:17-49 (bit order pinned by test_actions, actions.rs:390-421)

# typedefs.rs:15-86 with the DataType constructors of datatypes.rs:108-198:
# name -> (level, needs_parse, needs_update, needs_reassembly, needs_packet_track)
_DT = {}
for _n in ("ConnRecord", "ConnDuration", "PktCount", "ByteCount", "InterArrivals", "ConnHistory"):
    _DT[_n] = ("Connection", False, True, False, False)
for _n in ("HttpTransaction", "DnsTransaction", "TlsHandshake", "QuicStream", "SshHandshake"):
    _DT[_n] = ("Session", True, False, False, False)
for _n in ("ZcFrame", "Payload"):
    _DT[_n] = ("Packet", False, False, False, False)
_DT["SessionList"] = ("Connection", True, False, False, False)
for _n in ("BidirZcPktStream", "OrigZcPktStream", "RespZcPktStream", "BidirPktStream", "OrigPktStream", "RespPktStream"):
    _DT[_n] = ("Connection", False, False, False, True)
for _n in ("OrigZcPktsReassembled", "RespZcPktsReassembled", "OrigPktsReassembled", "RespPktsReassembled"):
    _DT[_n] = ("Connection", False, False, True, True)
for _n in ("CoreId", "FiveTuple", "EtherTCI", "EthAddr", "FilterStr"):
    _DT[_n] = ("Static", False, False, False, False)


def _dt_packet_filter(name: str, sub_level: str) -> tuple[list[int], list[int]]:
    """DataType::packet_filter (datatypes.rs:306-345): ([data, terminal] if matched, if matching)."""
    lvl, parse, upd, reas, track = _DT[name]
    m, g = [0, 0], [0, 0]
    if lvl == "Packet" and sub_level == "Packet":
        g[0] |= ACT["PacketCache"]
    for flag, bit in ((upd, "UpdatePDU"), (reas, "Reassemble"), (track, "PacketTrack")):   # needs_update
        if flag:
            m[0] |= ACT[bit]
            m[1] |= ACT[bit]
            g[0] |= ACT[bit]
    if sub_level == "Connection":                                                          # conn_deliver
        m[0] |= ACT["ConnDeliver"]
        m[1] |= ACT["ConnDeliver"]
    if parse:
        m[0] |= ACT["ProtoProbe"]
        m[1] |= ACT["ProtoProbe"]
        if sub_level == "Connection":
            m[0] |= ACT["SessionTrack"]
            m[1] |= ACT["SessionTrack"]
    if lvl == "Session" and sub_level in ("Session", "Streaming"):
        m[0] |= ACT["SessionDeliver"]
        m[1] |= ACT["SessionDeliver"]
    return m, g


def _sub_packet_filter(sub: Sub) -> tuple[tuple[int, int], tuple[int, int]]:
    """SubscriptionSpec::packet_filter (datatypes.rs:626-637)."""
    m, g = [0, 0], [0, 0]
    for d in sub.datatypes:
        a, b = _dt_packet_filter(d, sub.level)
        m = [m[0] | a[0], m[1] | a[1]]
        g = [g[0] | b[0], g[1] | b[1]]
    g[0] |= ACT["ProtoFilter"]
    if sub.level == "Streaming":
        m[0] |= ACT["Stream"]
        m[1] |= ACT["Stream"]
    return (m[0], m[1]), (g[0], g[1])


def _can_stream(level: str) -> bool:
    return level in ("Connection", "Packet")


def _pkt_should_deliver(sub: Sub, p: Pred) -> bool:
    """SubscriptionSpec::should_deliver at FilterLayer::Packet (datatypes.rs:563-573, 203-265):
    only static data of a static-only subscription is delivered there, on a packet predicate."""
    if sub.level == "Streaming":
        return False
    lv = [_DT[d][0] for d in sub.datatypes]
    anyd = any(l == "Static" and sub.level == "Static" and on_packet(p) for l in lv)
    alld = all(l in ("Packet", "Static") for l in lv)                        # can_deliver
    return anyd and alld


def _pkt_should_stream(sub: Sub, p: Pred) -> bool:
    """SubscriptionSpec::should_stream at FilterLayer::Packet (datatypes.rs:584-615)."""
    if sub.level != "Streaming":
        return False
    lv = [_DT[d][0] for d in sub.datatypes]
    if any(l not in ("Packet", "Static") and not _can_stream(l) for l in lv):
        return False
    if all(_can_stream(l) or l == "Static" for l in lv):
        return on_packet(p)
    return False   # no datatype's should_deliver holds at the Packet layer for a streaming sub


@dataclass
class CNode:
    pred: Pred
    id: int = 0
    data: int = 0
    term: int = 0
    deliver: dict = field(default_factory=dict)   # sid -> (as_str, must_deliver)
    stream: dict = field(default_factory=dict)
    kids: list = field(default_factory=list)
    if_else: bool = False

    def label(self) -> str:
        s = str(self.pred)
        if self.data or self.term:
            s += f" -- A: {self.data}/{self.term}"
        if self.deliver:
            s += " D: ( " + "".join(self.deliver[k][0] + ", " for k in sorted(self.deliver)) + ")"
        if self.stream:
            s += " S: ( " + "".join(self.stream[k][0] + ", " for k in sorted(self.stream)) + ")"
        if self.if_else:
            s += " x"
        return s

    def same(self, o: "CNode") -> bool:          # PartialEq for PNode (ptree.rs:871-876)
        return self.pred == o.pred and (self.data, self.term) == (o.data, o.term) and self.deliver == o.deliver


def _cpaths(n: CNode) -> list[str]:
    out = []

    def rec(node, acc):
        if not node.kids and acc:
            out.append(",".join(acc))
            return
        for k in node.kids:
            rec(k, acc + [k.label()])

    rec(n, [])
    return out


def _c_all_paths_eq(a: CNode, b: CNode) -> bool:
    return (not a.kids and not b.kids) or _cpaths(a) == _cpaths(b)


class ConnTree:
    """PTree for FilterLayer::Packet built by filter_subtree + collapse (ptree.rs)."""

    def __init__(self, subs: list[Sub]):
        self.subs = subs
        self.root = CNode(Pred("ethernet"))
        self.size = 1
        for sid, sub in enumerate(subs):
            validate(sub)
            self._build(sid, sub, filter_patterns(sub.filter))
        self._collapse()

    # build_tree (ptree.rs:344-385)
    def _build(self, sid, sub, patterns):
        deliver = (sub.as_str, "FilterStr" in sub.datatypes)
        prev = lambda p: on_packet(p) and sub.level == "Packet"  # noqa: E731  is_prev_layer (ast.rs:173-176)
        added = False
        for pat in patterns:
            if all(prev(p) for p in pat):
                continue
            added = added or bool(pat)
            self._add_pattern(sid, sub, deliver, pat)
        eth = Pred("ethernet")
        if not added and prev(eth) and not _pkt_should_stream(sub, eth):
            return
        if not added:
            if _pkt_should_deliver(sub, eth):
                self.root.deliver[sid] = deliver
            elif _pkt_should_stream(sub, eth):
                self.root.stream[sid] = deliver
            else:
                (m, _) = _sub_packet_filter(sub)
                self.root.data |= m[0]
                self.root.term |= m[1]

    # add_pattern (ptree.rs:389-461)
    def _add_pattern(self, sid, sub, deliver, pat):
        node = self.root
        matched, matching = _sub_packet_filter(sub)
        for p in pat:
            if not on_packet(p):                 # is_next_layer: non-terminal leaf
                node.data |= matching[0]
                node.term |= matching[1]
                return
            if req_packet(p):
                raise FilterError("Cannot access per-packet fields (e.g., TCP flags, length) after packet filter.")
            d = PacketTree._descendant(node, p)
            if d is not None:
                node = d
                continue
            par = PacketTree._narrowest_parent(node, p)
            if par is not None:
                node = par
            moved = [k for k in node.kids if is_child(k.pred, p)]
            node.kids = [k for k in node.kids if not is_child(k.pred, p)]
            nxt = next((k for k in node.kids if k.pred == p), None)
            if nxt is None:
                nxt = CNode(p, id=self.size)
                self.size += 1
                node.kids.append(nxt)
            nxt.kids += moved
            node = nxt
        if _pkt_should_deliver(sub, node.pred):
            node.deliver[sid] = deliver
        elif _pkt_should_stream(sub, node.pred):
            node.stream[sid] = deliver
        node.data |= matched[0]
        node.term |= matched[1]

    @staticmethod
    def _extracts_protocol(n: CNode) -> bool:
        if n.pred.unary and any(k.pred.unary for k in n.kids):
            return True
        if not n.pred.unary:
            return False
        return any(k.pred.proto == n.pred.proto and not k.pred.unary for k in n.kids)

    def _collapse(self):
        ex = _windows_all_excl

        def redundant(n, can_prune):                 # ptree.rs:693-748
            if not on_packet(n.pred):
                return
            nxt = ex(n.kids)
            for c in n.kids:
                redundant(c, nxt)
            if not can_prune:
                return
            must, could = [], []
            for c in n.kids:
                keep = c.data or c.term or c.stream or c.deliver or not on_packet(c.pred) or self._extracts_protocol(c)
                (must if keep else could).append(c)
            nc = []
            for c in could:
                if all(_c_all_paths_eq(c, o) for o in n.kids):
                    nc += c.kids
                else:
                    nc.append(c)
            nc = _stable_sort(nc + must)
            dd = []
            for c in nc:
                if not dd or not dd[-1].same(c):
                    dd.append(c)
            n.kids = dd

        redundant(self.root, ex(self.root.kids))

        def packet_conds(n, can_prune):              # ptree.rs:641-687
            if not on_packet(n.pred):
                return
            nxt = ex(n.kids)
            for c in n.kids:
                packet_conds(c, nxt)
            if not can_prune:
                return
            while len(n.kids) == 1 and on_packet(n.kids[0].pred):
                c = n.kids[0]
                if self._extracts_protocol(c):
                    break
                n.data |= c.data
                n.term |= c.term
                n.deliver.update(c.deliver)
                n.stream.update(c.stream)
                n.kids = c.kids

        packet_conds(self.root, ex(self.root.kids))

        def prune(n, on_a, on_d, on_s):              # ptree.rs:570-634
            my_d = set(on_d)
            keep = {}
            for k in sorted(n.deliver):
                s, must = n.deliver[k]
                if s not in my_d:
                    my_d.add(s)
                    keep[k] = n.deliver[k]
                elif must:
                    keep[k] = n.deliver[k]
            n.deliver = keep
            my_s = set(on_s)
            keep = {}
            for k in sorted(n.stream):
                s, must = n.stream[k]
                if s not in my_s:
                    my_s.add(s)
                    keep[k] = n.stream[k]
                elif must:
                    keep[k] = n.stream[k]
            n.stream = keep
            my_a = on_a
            if n.data or n.term:
                n.data &= ~on_a                      # Actions::clear_intersection (actions.rs)
                n.term &= ~on_a
                my_a = on_a | n.data
                # push: data and terminal both accumulate; clear_intersection only reads `data`
            for c in n.kids:
                prune(c, my_a, my_d, my_s)
            n.kids = [c for c in n.kids if c.data or c.term or c.kids or c.deliver]

        prune(self.root, 0, set(), set())

        def srt(n):
            for c in n.kids:
                srt(c)
            n.kids = _stable_sort(n.kids)

        srt(self.root)

        def mark(n):                                 # ptree.rs:527-552
            for i, c in enumerate(n.kids):
                mark(c)
                if i == 0:
                    continue
                prev = n.kids[i - 1]
                if is_excl(c.pred, prev.pred):
                    c.if_else = True
                if (c.data, c.term) == (prev.data, prev.term) and c.deliver == prev.deliver and \
                        _c_all_paths_eq(c, prev):
                    c.if_else = True

        mark(self.root)
        counter = [0]

        def number(n):
            n.id = counter[0]
            counter[0] += 1
            for c in n.kids:
                number(c)

        number(self.root)
        self.size = counter[0]

    def to_json(self, n: CNode | None = None) -> dict:
        n = self.root if n is None else n
        return {"id": n.id, "pred": str(n.pred), "unary": n.pred.unary, "protocol": n.pred.proto, "data": n.data,
                "terminal": n.term, "if_else": n.if_else, "deliver": sorted(n.deliver), "stream": sorted(n.stream),
                "children": [self.to_json(c) for c in n.kids]}
