"""CPU tests of the oracle: it reproduces the committed golden fixtures, its two restatements
(pure Python vs generated C) agree, and its independent compiler agrees with the product's C++
compiler (tree shape, else-if marking, callback statement order) on the reference's filters."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from oracle import filterlang, packet, pcap
from retina_amd import pc, synth

GOLD = Path(__file__).resolve().parent / "golden"


def _corpus(name):
    if name == "traces":
        t = np.load(GOLD / "traces.npz")
        return t["slab"], t["dlen"]
    t = np.load(GOLD / "corpus_adversarial.npz")
    return t["slab"], t["dlen"]


@pytest.mark.parametrize("corpus", ["traces", "adversarial"])
@pytest.mark.parametrize("fset", list(SETS))
def test_c_oracle_reproduces_golden(fset, corpus):
    g = np.load(GOLD / f"golden_{fset}.npz")
    slab, dlen = _corpus(corpus)
    r = helpers.oracle_run(SETS[fset], slab, 128, dlen)
    n = len(dlen)
    assert np.array_equal(r["pc"], np.unpackbits(g[f"{corpus}_pc"])[:n].astype(bool))
    assert np.array_equal(r["fwd"], np.unpackbits(g[f"{corpus}_fwd"])[:n].astype(bool))
    assert np.array_equal(r["rec"], g[f"{corpus}_rec"])
    assert np.array_equal(r["dm"], g[f"{corpus}_dm"])


@pytest.mark.parametrize("fset", ["cfg3", "quirks", "payload", "match_all"])
def test_python_oracle_matches_golden(fset):
    """Independent restatement (oracle/packet.py) against the fixture, frame by frame."""
    g = np.load(GOLD / f"golden_{fset}.npz")
    slab, dlen = _corpus("adversarial")
    tree = filterlang.PacketTree(filterlang.load_spec(SETS[fset]))
    pcb = np.unpackbits(g["adversarial_pc"])
    dm = g["adversarial_dm"]
    b = slab.reshape(-1, 128)
    for i in range(0, len(dlen), 3):
        act, fired = packet.evaluate(tree, b[i].tobytes(), int(dlen[i]))
        assert bool(act & 1) == bool(pcb[i])
        m = 0
        for k in fired:
            m |= 1 << k
        assert m == (int(dm[i, 0]) if dm.shape[1] else 0)


def test_traces_fixture_matches_pcaps(reference_dir):
    """traces.npz is exactly what offline.rs would hand to continue_packet."""
    t = np.load(GOLD / "traces.npz")
    frames = []
    for name in t["names"]:
        frames += pcap.offline_frames(reference_dir / "traces" / str(name), mtu=9702)
    slab, dlen = pc.pack_frames(frames, 128)
    assert np.array_equal(slab, t["slab"]) and np.array_equal(dlen, t["dlen"])


def test_l4context_examples():
    """Hand-checked L4Context values (pdu.rs:86-171) including the checked_sub underflow."""
    import corpus as C

    t = C.tcp(sport=1111, dport=2222, seq=7, ack=9, flags=0x12, payload=b"abcd")
    f = C.eth(0x0800) + C.ipv4(6, len(t)) + t
    c = packet.l4context(f, len(f))
    assert (c.sport, c.dport, c.proto, c.offset, c.length, c.seq, c.ack, c.flags) == (1111, 2222, 6, 54, 4, 7, 9, 0x12)
    f = C.eth(0x0800) + C.ipv4(6, 0, total=39) + t
    assert packet.l4context(f, len(f)) is None
    u = C.udp(payload=b"xyz")
    f = C.eth(0x86DD, vlan=4) + C.ipv6(17, len(u)) + u
    c = packet.l4context(f, len(f))
    assert (c.ver, c.proto, c.offset, c.length) == (6, 17, 18 + 40 + 8, 3)
    f = C.eth(0x0800) + C.ipv4(6, len(t), ihl=2) + t   # IHL 2: L4 inside the IPv4 header
    c = packet.l4context(f, len(f))
    assert c is not None and c.offset == 22 + ((f[34] & 0xF0) >> 2)


FILTERS = [
    "tcp.dst_port = 80", "tls", "dns", "ipv4", "ipv6 and udp", "tcp.port != 80", "ipv4.addr = 1.1.1.1",
    "tcp.port in 80..90 or udp.dst_port >= 53", "ipv4.src_addr in 10.0.0.0/8 and tcp.syn = 1",
    "ipv6.dst_addr = ::1 or ipv6.src_addr = fe80::/10", "(tcp or udp) and ipv4.time_to_live < 3",
    "http.uri = '/x' and tcp.dst_port = 8080", "quic and udp.port != 443", "tcp.flags = 2 or tcp.flags = 18",
    "ipv4.protocol = 1", "udp.length > 100 and udp.dst_port = 1434", "",
]


@pytest.mark.parametrize("dts", [["ConnRecord"], ["ZcFrame", "FilterStr"], ["Payload"], ["TlsHandshake"]])
@pytest.mark.parametrize("flt", FILTERS)
def test_compilers_agree_single(flt, dts):
    if "TlsHandshake" in dts and "tls" not in flt:
        dts = ["ConnRecord"]
    try:
        ora = filterlang.PacketTree([filterlang.Sub(flt, dts)])
    except filterlang.FilterError:
        # both compilers refuse it (e.g. per-packet fields in a connection-level filter)
        with pytest.raises(pc.FilterError):
            pc.Program.from_filter(flt, dts)
        return
    prod = pc.Program.from_filter(flt, dts)
    assert prod.tree == ora.pprint()
    subs, pay = prod.deliver_table()
    st = packet.statement_table(ora)
    assert [s for s, _ in st] == list(subs)
    assert [k == "Payload" for _, k in st] == [bool(x) for x in pay]


@pytest.mark.parametrize("fset", list(SETS))
def test_compilers_agree_sets(fset):
    prod = pc.Program.from_spec(SETS[fset])
    ora = filterlang.PacketTree(filterlang.load_spec(SETS[fset]))
    assert prod.tree == ora.pprint()


def test_compilers_agree_filter_stats(reference_dir):
    """The reference's largest subscription file (1575 subscriptions, mostly L7) compiles to the
    same PacketContinue tree in both compilers."""
    text = (reference_dir / "examples/filter_stats/spec.toml").read_text()
    prod = pc.Program.from_spec(text)
    ora = filterlang.PacketTree(filterlang.load_spec(text))
    assert prod.tree == ora.pprint()
    assert prod.info["n_subscriptions"] == 1575


BAD = ["tcp.dst_port = 70000", "ipv4 and ipv6", "ipv4.rf = 1", "tcp.port in 90..80", "ipv4.src_addr = 1.2.3.256",
       "ipv4.src_addr = 1.2.3.4/33", "tcp.foo = 1", "tcp and", "(tcp", "tcp.dst_port = 'x'", "ethernet",
       "ipv4.src_addr = 01.2.3.4", "tcp.dst_port in 5", "ipv6.src_addr = 1.2.3.4", "ipv4.src_addr = ::1", "bogus"]


@pytest.mark.parametrize("flt", BAD)
def test_both_compilers_reject(flt):
    with pytest.raises(pc.FilterError):
        pc.Program.from_filter(flt, ["ConnRecord"])
    with pytest.raises(Exception):
        t = filterlang.PacketTree([filterlang.Sub(flt, ["ConnRecord"])])
        from oracle import cgen
        cgen.generate_c(t)


def test_synth_alg_bytes():
    s, d = synth.cfg2(1000)
    assert synth.alg_read_bytes(s, d, 64) == 66 * 1000


@pytest.mark.parametrize("fset", list(SETS))
def test_hw_filter_string_matches_oracle(fset):
    """get_hw_filter (filtergen/src/lib.rs:233-238) = PTree::to_filter_string (ptree.rs:841-870)
    of the PacketContinue tree: the product's string equals the oracle's restatement, and it
    re-parses (filtergen panics on an invalid HW filter). Note the reference's string lists leaf
    paths only, so a frame that ends at an inner node with a delivery is not kept by it."""
    hw = pc.Program.from_spec(SETS[fset]).hw_filter
    assert hw == filterlang.PacketTree(filterlang.load_spec(SETS[fset])).to_filter_string()
    if hw:
        filterlang.parse_filter(hw)


def _l4_corpora():
    import corpus as C

    t = np.load(GOLD / "traces.npz")
    a = np.load(GOLD / "corpus_adversarial.npz")
    r, rd = pc.pack_frames(C.random_frames(4000, seed=77), 128)
    s3, d3 = synth.cfg3(3000, start=4242)
    s4, d4 = synth.cfg4(3000, start=4343)
    s2, d2 = synth.cfg2(1000, start=99)
    s2 = np.pad(s2.reshape(-1, 64), ((0, 0), (0, 64))).reshape(-1)
    return {"traces": (t["slab"], t["dlen"]), "adversarial": (a["slab"], a["dlen"]), "random": (r, rd),
            "synth": (np.concatenate([s2, s3, s4]), np.concatenate([d2, d3, d4]))}


@pytest.mark.parametrize("name", ["traces", "adversarial", "random", "synth"])
def test_python_l4context_every_field_vs_c_oracle(name):
    """The two restatements of L4Context::new (pdu.rs:86-171) -- oracle/packet.py (pure Python)
    and the generated C (oracle/cgen.py) -- agree on every field of every frame: existence,
    IP version, both addresses (all 16 bytes for IPv6), ports, protocol, offset, length, seq, ack
    and flags. Under the match-all set every frame is accepted, so the C oracle builds the
    L4Context of every frame that has one."""
    slab, dlen = _l4_corpora()[name]
    r = helpers.oracle_run(SETS["match_all"], slab, 128, dlen)
    assert r["pc"].all()
    recs = {int(x["idx"]): x for x in r["rec"]}
    b = slab.reshape(-1, 128)
    n_v6 = 0
    for i in range(len(dlen)):
        c = packet.l4context(b[i].tobytes() + bytes(128), int(dlen[i]))
        assert (c is not None) == bool(r["fwd"][i]) == (i in recs), (name, i)
        if c is None:
            continue
        x = recs[i]
        w = 4 if c.ver == 4 else 16
        src = c.src.to_bytes(w, "big") + bytes(16 - w)
        dst = c.dst.to_bytes(w, "big") + bytes(16 - w)
        got = (int(x["ver"]), int(x["proto"]), int(x["sport"]), int(x["dport"]), int(x["offset"]), int(x["length"]),
               int(x["seq"]), int(x["ack"]), int(x["flags"]), bytes(x["src"]), bytes(x["dst"]))
        assert got == (c.ver, c.proto, c.sport, c.dport, c.offset, c.length, c.seq, c.ack, c.flags, src, dst), (name, i)
        n_v6 += c.ver == 6
    assert len(recs) > 0
    if name in ("adversarial", "random", "synth"):
        assert n_v6 > 0


@pytest.mark.parametrize("flt,port,want", [("tcp.dst_port = 0.0.0.80", 80, True), ("tcp.dst_port = 0.0.0.80", 81, False),
                                           ("tcp.port = 1.2.3.4", 80, False), ("tcp.dst_port = ::50", 80, True),
                                           ("udp.port != 0.0.0.53", 53, False)])
def test_ip_literal_on_port_field_compiles(flt, port, want):
    """binary_to_tokens (filtergen/src/utils.rs:52-121) emits `u32::from(tcp.dst_port()) == <addr>`
    for an IPv4 literal on an integer field (u128::from for IPv6), which compiles in Rust
    (From<u16> for u32/u128). Both compilers accept it and the comparison is on the port's value."""
    import corpus as C

    prod = pc.Program.from_filter(flt, ["ConnRecord"])
    tree = filterlang.PacketTree([filterlang.Sub(flt, ["ConnRecord"])])
    assert prod.tree == tree.pprint()
    if flt.startswith("udp"):
        u = C.udp(sport=port, dport=port)
        f = C.eth(0x0800) + C.ipv4(17, len(u)) + u
    else:
        t = C.tcp(sport=1234, dport=port)
        f = C.eth(0x0800) + C.ipv4(6, len(t)) + t
    assert bool(packet.evaluate(tree, f)[0] & 1) is want
    slab, dlen = pc.pack_frames([f], 128)
    assert bool(helpers.oracle_run(prod_spec := synth._toml([(flt, ["ConnRecord"], "cb")]), slab, 128, dlen)["pc"][0]) is want
    assert prod_spec
