"""ORACLE (test infrastructure only): the rte_flow rules of Retina's hardware-assist filter.

Restates, in plain Python over oracle/filterlang.py's parser and patterns:
  core/src/runtime/online.rs:39, 184-191    Filter::new(filter_str), set_hardware_filter per port
  core/src/filter/hardware/mod.rs:38-73     HardwareFilter::new
  core/src/filter/hardware/mod.rs:76-93     install: pattern rules (group 0, priority 0, RSS) then
                                            add_redirect (:332-392, group 0 -> 1, priority 3)
  core/src/filter/hardware/mod.rs:124-203   device_supported / predicate_supported / pattern_supported
  core/src/filter/hardware/flow_item.rs:49-501  FlowPattern::from_layered_pattern (spec/mask in
                                            the rte_ipv4_hdr / rte_ipv6_hdr / rte_tcp_hdr /
                                            rte_udp_hdr byte layout, i.e. wire order)
  core/src/filter/pattern.rs:28-49, 133-142 is_fully_qualified / retain_hardware_predicates
  core/src/filter/ptree_flat.rs:91-267      FlatPTree build / prune_branches / to_flat_patterns
Parity: no reference test covers this module (it needs a NIC); the rules follow the code above
line by line, and the device's rte_flow_validate is a caller-supplied model.
"""
from __future__ import annotations

from .filterlang import EDGES, Pred, filter_patterns, fully_qualified

ITEM_END, ITEM_ETH, ITEM_IPV4, ITEM_IPV6, ITEM_TCP, ITEM_UDP = range(6)
ACTION_RSS, ACTION_JUMP = 1, 2
REDIRECT = 0xFFFFFFFF

# field -> (offset, bytes) in the DPDK header struct (flow_item.rs); addresses handled apart
_FIELDS = {
    "ipv4": (ITEM_IPV4, 20, {"version_ihl": (0, 1), "type_of_service": (1, 1), "total_length": (2, 2),
                             "identification": (4, 2), "flags_to_fragment_offset": (6, 2),
                             "time_to_live": (8, 1), "protocol": (9, 1), "header_checksum": (10, 2)}),
    "ipv6": (ITEM_IPV6, 40, {"version_to_flow_label": (0, 4), "payload_length": (4, 2),
                             "next_header": (6, 1), "hop_limit": (7, 1)}),
    # flow_item.rs:362 matches "data_offset_to_nw", which no filter field is called
    "tcp": (ITEM_TCP, 20, {"src_port": (0, 2), "dst_port": (2, 2), "seq_no": (4, 4), "ack_no": (8, 4),
                           "data_offset_to_nw": (12, 1), "flags": (13, 1), "window": (14, 2),
                           "checksum": (16, 2), "urgent_pointer": (18, 2)}),
    "udp": (ITEM_UDP, 8, {"src_port": (0, 2), "dst_port": (2, 2), "length": (4, 2), "checksum": (6, 2)}),
}
_ADDR = {("ipv4", "src_addr"): (12, 4), ("ipv4", "dst_addr"): (16, 4),
         ("ipv6", "src_addr"): (8, 16), ("ipv6", "dst_addr"): (24, 16)}


class InvalidRule(Exception):
    pass


def _item(kind: int, size: int = 0, spec: bytes = bytes(40), mask: bytes = bytes(40)) -> tuple:
    return (kind, size, bytes(spec), bytes(mask))


def _layer_item(proto: str, preds: list[Pred]) -> tuple:
    """append_ipv4 / append_ipv6 / append_tcp / append_udp (flow_item.rs:81-500)."""
    if proto not in _FIELDS:
        raise InvalidRule(f"Invalid header: {proto}")
    kind, size, fields = _FIELDS[proto]
    spec, mask = bytearray(40), bytearray(40)
    for p in preds:
        if p.unary:
            raise InvalidRule("Invalid predicate type: unary")
        v = p.value
        if (proto, p.field) in _ADDR:
            off, n = _ADDR[(proto, p.field)]
            want = "Ipv4" if proto == "ipv4" else "Ipv6"
            if v.kind != want:
                raise InvalidRule(f"Invalid RHS type: {v}")
            addr, plen = v.data
            bits = 8 * n
            netmask = ((1 << bits) - 1) ^ ((1 << (bits - plen)) - 1) if plen else 0
            spec[off:off + n] = addr.to_bytes(n, "big")       # the address as written (ipnet addr())
            mask[off:off + n] = netmask.to_bytes(n, "big")
            continue
        if p.field not in fields:
            raise InvalidRule(f"Invalid field: {p.field}")
        if v.kind != "Int":
            raise InvalidRule(f"Invalid RHS type: {v}")
        off, n = fields[p.field]
        if v.data[0] >= 1 << (8 * n):                          # uN::try_from
            raise InvalidRule(f"Invalid RHS value: {v}")
        spec[off:off + n] = v.data[0].to_bytes(n, "big")
        mask[off:off + n] = b"\xff" * n
    return _item(kind, size, spec, mask)


def layers_of(flat: list[Pred]) -> list[tuple[str, list[Pred]]]:
    """A fully-qualified flat pattern as its LayeredPattern (one entry per unary predicate)."""
    out = []
    for p in flat:
        if p.unary:
            out.append((p.proto, []))
        else:
            out[-1][1].append(p)
    return out


def flow_items(flat: list[Pred]) -> list[tuple]:
    """ETH, FlowPattern::from_layered_pattern's items, END (hardware/mod.rs:273-282)."""
    return [_item(ITEM_ETH)] + [_layer_item(proto, preds) for proto, preds in layers_of(flat)] + [_item(ITEM_END)]


def _rule(items, group=0, priority=0, action=ACTION_RSS, jump_group=0, pattern=0) -> dict:
    return {"group": group, "priority": priority, "action": action, "jump_group": jump_group,
            "pattern": pattern, "items": items}


def device_supported(p: Pred, validate) -> bool:
    """hardware/mod.rs:124-203."""
    if p.proto not in ("ipv4", "ipv6", "tcp", "udp"):
        return False
    if not p.unary and not (p.op == "Eq" or (p.proto in ("ipv4", "ipv6") and p.op == "In")):
        return False
    for fq in fully_qualified([p]):
        try:
            rule = _rule(flow_items(fq))
        except InvalidRule:
            return False
        if validate is not None and not validate(rule):
            return False
    return True


def is_fully_qualified(flat: list[Pred]) -> bool:
    """pattern.rs:28-49."""
    prev, ok = "ethernet", True
    for p in flat:
        if p.unary:
            ok = ok and (p.proto, prev) in EDGES
            prev = p.proto
        else:
            ok = ok and p.proto == prev
    return ok


def _flat_ptree_pruned(patterns: list[list[Pred]]) -> list[list[Pred]]:
    """FlatPTree::new + prune_branches + to_flat_patterns (ptree_flat.rs)."""
    root = {"kids": [], "term": False}
    for f in patterns:
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
    return out


def hardware_patterns(filter_str: str, validate=None) -> list[list[Pred]]:
    """HardwareFilter::new(&Filter::new(filter_str)).patterns, as flat patterns."""
    hw = [[p for p in f if device_supported(p, validate)] for f in filter_patterns(filter_str)]
    layered = []
    for f in _flat_ptree_pruned(hw):
        f = list(f)
        while not is_fully_qualified(f):
            f.pop()
        layered += fully_qualified(f)
    layered.sort(key=lambda f: [p.key() for p in f])
    uniq = []
    for f in layered:
        if not uniq or uniq[-1] != f:
            uniq.append(f)
    return uniq


def hardware_rules(filter_str: str, validate=None) -> list[dict]:
    """The rules HardwareFilter::install creates, in order."""
    pats = hardware_patterns(filter_str, validate)
    if not pats:                                # "Empty filter, skipping."
        return []
    rules = [_rule(flow_items(f), pattern=k) for k, f in enumerate(pats)]
    rules.append(_rule([_item(ITEM_ETH), _item(ITEM_END)], priority=3, action=ACTION_JUMP, jump_group=1,
                       pattern=REDIRECT))
    return rules


def patterns_text(filter_str: str, validate=None) -> str:
    return "".join("[" + ", ".join(map(str, f)) + "]\n" for f in hardware_patterns(filter_str, validate))
