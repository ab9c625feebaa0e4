"""ORACLE (test infrastructure only): the connection stage of a forwarded frame.

  core/src/conntrack/conn_id.rs:111-117    ConnId::new = (max(src, dst), min(src, dst), proto) in
                                           Rust's SocketAddr order (ip as its integer, then port)
  core/src/conntrack/conn/mod.rs:53-96     Conn::new_tcp opens a connection only on SYN without
                                           ACK or RST; Conn::new_udp on any UDP frame
  core/src/conntrack/conn/conn_info.rs:42-50  filter_first_packet -> the generated packet_filter
  filtergen/src/packet_filter.rs:7-73      gen_packet_filter (FilterLayer::Packet): root body
                                           first, first unary child `if`, later ones `else if`,
                                           binary children by if_else, children before a node's
                                           own body, Ethernet wrap iff the root has packet children
  filtergen/src/utils.rs:251-285           update_body: actions, then delivers, then streams
  include/retina_pc.h (rtn_conn_t)         the hash this repo defines over the canonical ConnId

The FilterLayer::Packet tree is the oracle's own (filterlang.ConnTree: filter_subtree + collapse
with SubscriptionSpec::packet_filter's actions, restated from ptree.rs / datatypes.rs); the
compiler's tree is checked against it on every filter set and on random subscription sets
(tests/test_conn.py), and the compiler's tree build is also pinned by the reference's own
ptree.rs KATs (tests/cpp/test_kats.cpp). This module evaluates that tree on the frame's bytes --
re-parsing the headers as packet_filter's parse_to chain does -- where the kernel evaluates it
on the L4Context view it already holds.
"""
from __future__ import annotations

from . import filterlang
from .packet import Hdr, be, eval_binary, l4context, parse

SYN, RST, ACK = 0x02, 0x04, 0x10  # core/src/protocols/packet/tcp.rs:13-20

STMT_TRACKED_PACKETS, STMT_CALLBACK, STMT_STREAM = 1, 2, 3


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF


def _mix(h: int, k: int) -> int:
    k = (k * 0xCC9E2D51) & 0xFFFFFFFF
    k = _rotl(k, 15)
    k = (k * 0x1B873593) & 0xFFFFFFFF
    h ^= k
    h = _rotl(h, 13)
    return (h * 5 + 0xE6546B64) & 0xFFFFFFFF


def _fmix(h: int) -> int:
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    return h ^ (h >> 16)


def conn_hash(v6: bool, ip_max: int, ip_min: int, port_max: int, port_min: int, proto: int) -> int:
    """rtn_conn_hash (include/retina_pc.h): MurmurHash3-x86-32 steps over the canonical words."""
    nw = 4 if v6 else 1
    h = 0x5EED
    for ip in (ip_max, ip_min):
        for j in range(nw - 1, -1, -1):
            h = _mix(h, (ip >> (32 * j)) & 0xFFFFFFFF)
    h = _mix(h, (port_max << 16) | port_min)
    h = _mix(h, proto | (0x100 if v6 else 0))
    return _fmix(h ^ (40 if v6 else 16))


def conn_id(ctx) -> tuple[bool, tuple, tuple]:
    """ConnId::new(src, dst, proto): (src_is_max, max endpoint, min endpoint). cmp::max returns
    its second argument on equality, so src is the max endpoint only when strictly greater."""
    src, dst = (ctx.src, ctx.sport), (ctx.dst, ctx.dport)
    gt = src > dst
    return gt, (src if gt else dst), (dst if gt else src)


def creates(ctx) -> bool:
    if ctx.proto == 17:
        return True
    return bool(ctx.flags & SYN) and not ctx.flags & ACK and not ctx.flags & RST


class PacketFilter:
    """The generated packet_filter for a FilterLayer::Packet tree (JSON nodes as exported by the
    compiler); evaluate() runs it on one frame."""

    def __init__(self, tree: dict, subs: list):
        self.root = tree
        self.subs = subs
        self.stmts: list[tuple[int, int]] = []   # (sub id, STMT_*) in generated-code order
        self._preds: dict[int, filterlang.Pred] = {}
        self._number(tree, is_root=True)

    def _pred(self, node: dict) -> filterlang.Pred:
        if node["id"] not in self._preds:
            dnf = filterlang.parse_filter(node["pred"])
            assert len(dnf) == 1 and len(dnf[0]) == 1, node["pred"]
            self._preds[node["id"]] = dnf[0][0]
        return self._preds[node["id"]]

    def _body_stmts(self, node: dict) -> list[int]:
        ks = []
        for sid in sorted(node["deliver"]):
            kind = STMT_TRACKED_PACKETS if self.subs[sid].level == "Packet" else STMT_CALLBACK
            ks.append(len(self.stmts))
            self.stmts.append((sid, kind))
        for sid in sorted(node["stream"]):
            ks.append(len(self.stmts))
            self.stmts.append((sid, STMT_STREAM))
        return ks

    def _root_has_body(self) -> bool:
        r = self.root
        return bool(r["data"] or r["terminal"] or r["deliver"])  # packet_filter.rs:15

    def _number(self, node: dict, is_root: bool = False) -> None:
        """Statement indices in code order: the root's body, then every child subtree (a child's
        children before its own body)."""
        if is_root:
            node["_stmts"] = self._body_stmts(node) if self._root_has_body() else []
            for c in node["children"]:
                if filterlang.on_packet(self._pred(c)):
                    self._number(c)
            return
        for c in node["children"]:
            if filterlang.on_packet(self._pred(c)):
                self._number(c)
        node["_stmts"] = self._body_stmts(node)

    def evaluate(self, frame: bytes, dl: int) -> tuple[int, int, list[int]]:
        """(Actions.data, Actions.terminal, [fired statement index, ...])."""
        d = bytes(frame) + bytes(max(0, 256 - len(frame)))
        out = {"data": 0, "term": 0, "fired": []}

        def body(node: dict):
            out["data"] |= node["data"]
            out["term"] |= node["terminal"]
            out["fired"].extend(node["_stmts"])

        def children(node: dict, env: dict):
            chain_taken = False
            first_unary = True
            for c in node["children"]:
                if not filterlang.on_packet(self._pred(c)):
                    continue
                if c["unary"]:
                    cont = not first_unary
                    first_unary = False
                else:
                    cont = c["if_else"]
                if not cont:
                    chain_taken = False
                if chain_taken:
                    continue
                p = self._pred(c)
                env2 = env
                if c["unary"]:
                    h = parse(d, dl, p.proto, env[node["protocol"]])
                    ok = h is not None
                    if ok:
                        env2 = dict(env)
                        env2[p.proto] = h
                else:
                    ok = eval_binary(d, env[p.proto], p)
                if ok:
                    chain_taken = True
                    children(c, env2)
                    body(c)

        root = self.root
        any_pkt = any(filterlang.on_packet(self._pred(c)) for c in root["children"])
        has_body = self._root_has_body()
        eth = parse(d, dl, "ethernet", None)
        if (has_body or any_pkt) and any_pkt and eth is None:   # add_root_pred's Ethernet wrap
            return 0, 0, []
        if has_body:
            body(root)
        children(root, {"ethernet": eth})
        return out["data"], out["term"], out["fired"]


def stage(pf: PacketFilter, frame: bytes, dl: int) -> tuple[int, int, list[int]] | None:
    """Connection stage of one frame: (hash, info, fired statements), or None if the frame is
    not forwarded to conntrack (the caller checks the PacketContinue gate)."""
    ctx = l4context(bytes(frame) + bytes(max(0, 256 - len(frame))), dl)
    if ctx is None:
        return None
    gt, mx, mn = conn_id(ctx)
    h = conn_hash(ctx.ver == 6, mx[0], mn[0], mx[1], mn[1], ctx.proto)
    data, term, fired = pf.evaluate(frame, dl)
    info = (data & 0x1FFF) | ((term & 0x1FFF) << 13) | (int(creates(ctx)) << 26) | (int(gt) << 27) | \
        (int(bool(fired)) << 28) | (int(ctx.ver == 6) << 29) | (int(ctx.proto == 17) << 30)
    return h, info, fired


__all__ = ["PacketFilter", "DeliverFilter", "stage", "conn_hash", "conn_id", "creates", "Hdr", "be"]


# ----------------------------------------------------------------------------------------------
# The table step of ConnTracker::process (conntrack/mod.rs:80-169), batch by batch.

CT_HIT, CT_NEW, CT_MISS, CT_NEW_DROPPED, CT_FULL, CT_COLLISION, CT_PRIOR = 1, 2, 3, 4, 5, 6, 0x100


def conn_key(ctx) -> tuple:
    """The canonical ConnId of a forwarded frame's L4Context (direction-free)."""
    _, mx, mn = conn_id(ctx)
    return (ctx.ver, mx, mn, ctx.proto)


class TableModel:
    """Sequential restatement of the table outcome of every forwarded frame, in frame order.

    Within a batch an existing connection is assumed to stay (the host sees its own removals and
    reports them with remove() between batches). A frame finds its key Occupied (HIT), or, on a
    Vacant key, opens the connection if it may (Conn::new_tcp: SYN without ACK/RST; Conn::new_udp:
    any UDP frame) unless it is a TCP frame whose first-packet filter drops (remove_from_table
    right after filter_first_packet: no entry, mod.rs:139-141), else it is dropped (MISS).
    Slots are opaque here: the model hands out ids; tests compare the GPU's slot *partition*."""

    def __init__(self, max_connections: int = 1 << 62):
        self.present: dict = {}   # key -> (model id, epoch inserted)
        self.max = max_connections
        self.epoch = 0
        self._ids = 0

    def process(self, frames: list[tuple]) -> list[tuple]:
        """frames: (key, opens, pf_drops) per forwarded frame in frame order.
        Returns (model id or None, status) per frame."""
        self.epoch += 1
        first: dict = {}
        for i, (key, opens, drops) in enumerate(frames):
            inserting = opens and not (key[3] == 6 and drops)
            if inserting and key not in self.present and key not in first:
                first[key] = i
        for key, i in sorted(first.items(), key=lambda kv: kv[1]):
            if len(self.present) < self.max:
                self.present[key] = (self._ids, self.epoch)
                self._ids += 1
        out = []
        for i, (key, opens, drops) in enumerate(frames):
            dropped_opener = opens and key[3] == 6 and drops
            if key in self.present:
                mid, ep = self.present[key]
                if ep != self.epoch:
                    out.append((mid, CT_HIT | CT_PRIOR))
                elif i > first[key]:
                    out.append((mid, CT_HIT))
                elif i == first[key]:
                    out.append((mid, CT_NEW))
                else:
                    out.append((mid, CT_NEW_DROPPED if opens else CT_MISS))
            else:
                out.append((None, CT_MISS if not opens else CT_NEW_DROPPED if dropped_opener else CT_FULL))
        return out

    def remove(self, keys) -> None:
        for k in keys:
            self.present.pop(k, None)


# ----------------------------------------------------------------------------------------------
# The generated packet_deliver (FilterLayer::PacketDeliver), run on one packet of a connection
# that holds the PacketDeliver action (conntrack/conn/conn_info.rs:70-75).
#
#   filtergen/src/deliver_filter.rs:9-29     the root's deliveries first, then its children;
#                                            add_root_pred's Ethernet wrap iff packet children
#   filtergen/src/deliver_filter.rs:31-121   packet unary -> `if let`/`else if let` chain (first
#                                            unary child opens it), packet binary -> if/else if by
#                                            if_else, service -> `if matches!(conn.service(), X)`
#                                            (else if by if_else), session binary -> a loop over
#                                            tracked.sessions() (never part of an else chain)
#   filtergen/src/utils.rs:251-285           update_body: children first, then the node's delivers
#   filtergen/src/data.rs:299-317            build_packet_callback: `if let Some(p) =
#                                            T::from_mbuf(mbuf)`; datatypes/src/packet.rs:18-29
#                                            Payload needs offset < data_len, offset+len <= data_len
#
# The tree is the oracle's own (filterlang.DeliverTree, restating filter_subtree + collapse for
# FilterLayer::PacketDeliver); tests/test_pd.py also checks it against the compiler's export.
# The connection-dependent conditions are given per connection as `facts` (fact index by the
# predicate's text, as exported in Program.pd_program()["facts"]): a service fact is 1 when the
# connection's service is that protocol; a session fact is the number of tracked sessions that
# satisfy the predicate, i.e. how many times the loop body runs.

class DeliverFilter:
    def __init__(self, tree: dict, subs: list, fact_preds: list[str]):
        self.root = tree
        self.subs = subs
        self.fact = {p: k for k, p in enumerate(fact_preds)}
        self.stmts: list[int] = []   # statement -> subscription id, in code order
        self._preds: dict[int, filterlang.Pred] = {}
        self._number(tree, True)

    def _pkt(self, node: dict) -> bool:
        return node["protocol"] in ("ethernet", "ipv4", "ipv6", "tcp", "udp")

    def _pred(self, node: dict) -> filterlang.Pred:
        if node["id"] not in self._preds:
            dnf = filterlang.parse_filter(node["pred"])
            assert len(dnf) == 1 and len(dnf[0]) == 1, node["pred"]
            self._preds[node["id"]] = dnf[0][0]
        return self._preds[node["id"]]

    def _number(self, node: dict, is_root: bool = False) -> None:
        own = []
        if is_root:
            for sid in sorted(node["deliver"]):
                own.append(len(self.stmts))
                self.stmts.append(sid)
        for c in node["children"]:
            self._number(c)
        if not is_root:
            for sid in sorted(node["deliver"]):
                own.append(len(self.stmts))
                self.stmts.append(sid)
        node["_stmts"] = own

    def evaluate(self, frame: bytes, dl: int, facts) -> list[int]:
        """Statement indices in the order the callbacks run."""
        d = bytes(frame) + bytes(max(0, 256 - len(frame)))
        ctx = l4context(d, dl)
        payload_ok = ctx is not None and ctx.offset < dl and ctx.offset + ctx.length <= dl
        fired: list[int] = []

        def body(node: dict):
            for k in node["_stmts"]:
                dts = self.subs[self.stmts[k]].datatypes
                if "Payload" in dts and not payload_ok:
                    continue
                fired.append(k)

        def children(node: dict, env: dict):
            chain_taken = False
            first_unary = True
            for c in node["children"]:
                pkt = self._pkt(c)
                if not pkt and not c["unary"]:
                    # for session in tracked.sessions() { if let X(x) = &session.data { if pred {..} } }
                    for _ in range(int(facts[self.fact[c["pred"]]])):
                        children(c, env)
                        body(c)
                    chain_taken = False
                    continue
                if pkt and c["unary"]:
                    cont = not first_unary
                    first_unary = False
                else:
                    cont = c["if_else"]
                if not cont:
                    chain_taken = False
                if chain_taken:
                    continue
                env2 = env
                if not pkt:
                    ok = int(facts[self.fact[c["pred"]]]) != 0
                elif c["unary"]:
                    p = self._pred(c)
                    h = parse(d, dl, p.proto, env[node["protocol"]])
                    ok = h is not None
                    if ok:
                        env2 = dict(env)
                        env2[p.proto] = h
                else:
                    p = self._pred(c)
                    ok = eval_binary(d, env[p.proto], p)
                if ok:
                    chain_taken = True
                    children(c, env2)
                    body(c)

        root = self.root
        eth = parse(d, dl, "ethernet", None)
        any_pkt = any(self._pkt(c) for c in root["children"])
        if any_pkt and eth is None:
            return []
        body(root)
        children(root, {"ethernet": eth})
        return fired
