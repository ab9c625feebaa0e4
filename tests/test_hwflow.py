"""Hardware-assist filter (include/retina_hw.h): the rte_flow rules the product
library emits for a filter equal the oracle's restatement of HardwareFilter::new + install
(core/src/filter/hardware/mod.rs:38-93, flow_item.rs:49-501), rule for rule and byte for byte,
under several device models standing in for rte_flow_validate. No reference test covers this
module (it needs a NIC): parity here is against the restatement (oracle/hwflow.py)."""
from __future__ import annotations

import random

import pytest

from golden.filter_sets import SETS
from oracle import hwflow
from randsubs import random_subs, to_toml
from retina_amd import pc

IPV4, IPV6, TCP, UDP = hwflow.ITEM_IPV4, hwflow.ITEM_IPV6, hwflow.ITEM_TCP, hwflow.ITEM_UDP


def _item(rule, kind):
    return next(it for it in rule["items"] if it[0] == kind)


# device models: rule dict -> accepted (rte_flow_validate == 0)
MODELS = {
    "all": None,
    "no_ipv6_match": lambda r: not any(it[0] == IPV6 and any(it[3]) for it in r["items"]),
    "no_udp": lambda r: not any(it[0] == UDP for it in r["items"]),
    "no_seq_ack": lambda r: not any(it[0] == TCP and any(it[3][4:12]) for it in r["items"]),
    "exact_addrs_only": lambda r: all(
        it[3][12:20] in (bytes(8), b"\xff" * 8) for it in r["items"] if it[0] == IPV4),
    "none": lambda r: False,
}


def _check(filter_str: str, model: str):
    v = MODELS[model]
    got = pc.hw_rules(filter_str, v)
    want = hwflow.hardware_rules(filter_str, v)
    assert got == want, (filter_str, model)
    assert pc.hw_patterns(filter_str, v) == hwflow.patterns_text(filter_str, v)
    return got


def test_known_rules():
    assert pc.hw_rules("") == []                      # empty filter: nothing installed
    r = _check("tcp.dst_port = 80", "all")
    assert [x["pattern"] for x in r] == [0, 1, hwflow.REDIRECT]
    assert pc.hw_patterns("tcp.dst_port = 80") == "[ipv4, tcp, tcp.dst_port = 80]\n[ipv6, tcp, tcp.dst_port = 80]\n"
    tcp = _item(r[0], TCP)
    assert tcp[1] == 20 and tcp[2][2:4] == b"\x00\x50" and tcp[3][2:4] == b"\xff\xff" and not any(tcp[3][4:])
    assert [it[0] for it in r[0]["items"]] == [hwflow.ITEM_ETH, IPV4, TCP, hwflow.ITEM_END]
    assert not any(_item(r[0], IPV4)[3])              # ipv4 layer present, matches any header
    jump = r[-1]
    assert (jump["action"], jump["jump_group"], jump["priority"], jump["group"]) == (hwflow.ACTION_JUMP, 1, 3, 0)
    assert [it[0] for it in jump["items"]] == [hwflow.ITEM_ETH, hwflow.ITEM_END]
    # an IPv4 prefix: spec = the address as written, mask = the netmask
    r = _check("ipv4.src_addr in 10.1.2.3/16 and tcp.dst_port != 443", "all")
    assert pc.hw_patterns("ipv4.src_addr in 10.1.2.3/16 and tcp.dst_port != 443") == \
        "[ipv4, ipv4.src_addr in 10.1.2.3/16, tcp]\n"     # `!=` stays in software
    v4 = _item(r[0], IPV4)
    assert v4[2][12:16] == bytes([10, 1, 2, 3]) and v4[3][12:16] == b"\xff\xff\x00\x00"
    # IPv6 address and scalar fields
    r = _check("ipv6.dst_addr = 2001:db8::1 and ipv6.hop_limit = 64 and udp.length = 300", "all")
    v6 = _item(r[0], IPV6)
    assert v6[1] == 40 and v6[2][24:40] == bytes.fromhex("20010db8000000000000000000000001")
    assert v6[3][24:40] == b"\xff" * 16 and v6[2][7] == 64 and v6[3][7] == 0xFF
    assert _item(r[0], UDP)[2][4:6] == (300).to_bytes(2, "big")


def test_unsupported_predicates_broaden_the_pattern():
    # flow_item.rs matches "data_offset_to_nw", not the filter field data_offset_to_ns
    assert pc.hw_patterns("tcp.data_offset_to_ns = 80") == "[ipv4, tcp]\n[ipv6, tcp]\n"
    # out of range for the header field (u16::try_from fails), L7 protocols, other operators
    assert pc.hw_patterns("tcp.window = 70000") == "[ipv4, tcp]\n[ipv6, tcp]\n"
    assert pc.hw_patterns("tls") == "[ipv4, tcp]\n[ipv6, tcp]\n"
    assert pc.hw_patterns("ipv4.time_to_live > 3") == "[ipv4]\n"
    assert pc.hw_patterns("tcp.port in 80..90") == "[ipv4, tcp]\n[ipv6, tcp]\n"
    # pruning after the unsupported predicates are gone: [ipv4, tcp] covers the narrower pattern
    f = "ipv4 and tcp.dst_port != 80 or ipv4 and tcp.dst_port = 80"
    assert pc.hw_patterns(f) == "[ipv4, tcp]\n"
    _check(f, "all")
    # a device that refuses every rule: nothing is installed
    assert pc.hw_rules("tcp.dst_port = 80", MODELS["none"]) == []
    # a device without UDP matching: the udp layer goes, the pattern broadens to ipv4 / ipv6
    assert pc.hw_patterns("udp.dst_port = 53", MODELS["no_udp"]) == "[ipv4]\n[ipv6]\n"


def test_errors():
    with pytest.raises(pc.FilterError):
        pc.hw_rules("tcp.dst_port = = 80")
    L = pc.lib()
    assert L.rtn_hw_rules(b"tcp", pc._FLOW_VALIDATE(), None, None, 0, None) == -22
    import ctypes as C
    n = C.c_uint32(0)
    assert L.rtn_hw_rules(b"tcp", pc._FLOW_VALIDATE(), None, None, 0, C.byref(n)) == -34 and n.value == 3


@pytest.mark.parametrize("model", list(MODELS))
@pytest.mark.parametrize("fset", list(SETS))
def test_filter_sets(fset, model):
    prog = pc.Program.from_spec(SETS[fset])
    v = MODELS[model]
    got = pc.hw_rules(validate=v, program=prog)
    assert got == hwflow.hardware_rules(prog.hw_filter, v)
    assert got == pc.hw_rules(prog.hw_filter, v)


def _rand_pred(rng: random.Random) -> str:
    k = rng.randrange(12)
    if k == 0:
        return rng.choice(["ipv4", "ipv6", "tcp", "udp", "tls", "dns", "http", "quic"])
    if k == 1:
        net = rng.choice(["10.0.0.1", "10.1.2.3/16", "3.3.3.3/32", "0.0.0.0/0", "192.168.7.0/24"])
        return f"ipv4.{rng.choice(['src_addr', 'dst_addr', 'addr'])} {rng.choice(['=', 'in', '!='])} {net}"
    if k == 2:
        net = rng.choice(["2001:db8::1", "2001:db8::/32", "::/0", "fe80::1/64"])
        return f"ipv6.{rng.choice(['src_addr', 'dst_addr', 'addr'])} {rng.choice(['=', 'in', '!='])} {net}"
    fields = {
        "ipv4": ["version_ihl", "type_of_service", "total_length", "identification", "flags_to_fragment_offset",
                 "time_to_live", "protocol", "header_checksum", "dscp", "flags"],
        "ipv6": ["version_to_flow_label", "payload_length", "next_header", "hop_limit", "flow_label"],
        "tcp": ["src_port", "dst_port", "seq_no", "ack_no", "data_offset_to_ns", "flags", "window", "checksum",
                "urgent_pointer", "syn", "port"],
        "udp": ["src_port", "dst_port", "length", "checksum", "port"],
    }
    proto = rng.choice(list(fields))
    field = rng.choice(fields[proto])
    op = rng.choice(["=", "=", "=", "!=", ">=", "<", "in"])
    if op == "in":
        a = rng.randrange(0, 300)
        return f"{proto}.{field} in {a}..{a + rng.randrange(1, 100)}"
    val = rng.choice([0, 1, 6, 17, 64, 80, 255, 256, 443, 65535, 65536, 2 ** 32 - 1, 2 ** 32])
    return f"{proto}.{field} {op} {val}"


def _rand_filter(rng: random.Random) -> str:
    return " or ".join(" and ".join(_rand_pred(rng) for _ in range(rng.randrange(1, 4)))
                       for _ in range(rng.randrange(1, 4)))


@pytest.mark.parametrize("seed", range(8))
def test_random_filters(seed):
    rng = random.Random(0x4857 + seed)
    for _ in range(40):
        f = _rand_filter(rng)
        for model in MODELS:
            try:
                want = hwflow.hardware_rules(f, MODELS[model])
            except Exception:                       # not a valid filter for Filter::new
                with pytest.raises(pc.FilterError):
                    pc.hw_rules(f, MODELS[model])
                break
            assert pc.hw_rules(f, MODELS[model]) == want, (f, model)


@pytest.mark.parametrize("seed", range(4))
def test_random_subscription_sets(seed):
    for k in range(10):
        subs = random_subs(1000 * seed + k)
        try:
            prog = pc.Program.from_spec(to_toml(subs))
        except pc.FilterError:
            continue
        for model in ("all", "no_ipv6_match", "no_udp"):
            v = MODELS[model]
            assert pc.hw_rules(validate=v, program=prog) == hwflow.hardware_rules(prog.hw_filter, v)
