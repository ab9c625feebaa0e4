"""Connection stage of forwarded frames (rtn_conn_t): ConnId hash + orientation, the creates bit
(Conn::new_tcp / new_udp) and the first-packet packet_filter (FilterLayer::Packet).

CPU tests pin the oracle (oracle/conn.py) on hand-built frames and the committed fixtures, and
check that the product compiler rejects what filtergen rejects at the Packet layer. GPU tests
compare the kernel's conn outputs with the fixtures and with the oracle, bit for bit."""
from __future__ import annotations

import struct
from pathlib import Path

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from oracle import conn as oconn
from oracle import filterlang
from oracle import packet
from retina_amd import pc, synth

GOLD = Path(__file__).resolve().parent / "golden"


def _frame(v6=False, src=0x0A000001, dst=0x0A000002, sport=1234, dport=80, proto=6, flags=0x02) -> bytes:
    l4 = struct.pack(">HHIIBBHHH", sport, dport, 1, 2, 0x50, flags, 1024, 0, 0) if proto == 6 else \
        struct.pack(">HHHH", sport, dport, 8, 0)
    if v6:
        ip = struct.pack(">IHBB", 0x60000000, len(l4), proto, 64) + src.to_bytes(16, "big") + dst.to_bytes(16, "big")
        et = 0x86DD
    else:
        ip = struct.pack(">BBHHHBBHII", 0x45, 0, 20 + len(l4), 0, 0, 64, proto, 0, src, dst)
        et = 0x0800
    return bytes(6) + bytes(5) + b"\x01" + struct.pack(">H", et) + ip + l4


def _ctx(fr: bytes):
    return packet.l4context(fr + bytes(64), len(fr))


# ---------------------------------------------------------------------------------------------
# CPU: oracle semantics

def test_connid_orientation_follows_socketaddr_order():
    # ip decides first (as its integer), then the port; equal endpoints: src is not the max
    c = _ctx(_frame(src=0x0A000002, dst=0x0A000001, sport=1, dport=2))
    assert oconn.conn_id(c)[0] is True
    c = _ctx(_frame(src=0x0A000001, dst=0x0A000001, sport=9, dport=8))
    assert oconn.conn_id(c)[0] is True
    c = _ctx(_frame(src=0x0A000001, dst=0x0A000001, sport=8, dport=8))
    assert oconn.conn_id(c)[0] is False
    hi, lo = 0x20010DB8 << 96, (0x20010DB8 << 96) | 5
    c = _ctx(_frame(v6=True, src=lo, dst=hi, sport=1, dport=65535))
    assert oconn.conn_id(c)[0] is True


def test_conn_hash_is_direction_free():
    a = _ctx(_frame(src=0xC0A80001, dst=0x08080808, sport=5555, dport=53, proto=17))
    b = _ctx(_frame(src=0x08080808, dst=0xC0A80001, sport=53, dport=5555, proto=17))
    ha = oconn.conn_hash(False, *[x for pair in zip(oconn.conn_id(a)[1], oconn.conn_id(a)[2]) for x in pair], 17)
    hb = oconn.conn_hash(False, *[x for pair in zip(oconn.conn_id(b)[1], oconn.conn_id(b)[2]) for x in pair], 17)
    assert ha == hb
    # and tells protocol and address family apart
    assert oconn.conn_hash(False, 1, 2, 3, 4, 6) != oconn.conn_hash(False, 1, 2, 3, 4, 17)
    assert oconn.conn_hash(False, 1, 2, 3, 4, 6) != oconn.conn_hash(True, 1, 2, 3, 4, 6)


@pytest.mark.parametrize("flags,exp", [(0x02, True), (0x12, False), (0x06, False), (0x10, False), (0x00, False),
                                       (0x03, True), (0x0A, True)])
def test_creates_is_syn_without_ack_or_rst(flags, exp):
    assert oconn.creates(_ctx(_frame(flags=flags))) is exp


def test_creates_on_any_udp():
    assert oconn.creates(_ctx(_frame(proto=17, flags=0)))


@pytest.mark.parametrize("filt,dts", [("ipv4.protocol = 17 and udp.length < 30", "SessionList"),
                                      ("tcp.flags = 2", "ConnRecord"),
                                      ("ipv4.time_to_live > 3 and tls", "TlsHandshake")])
def test_per_packet_fields_after_packet_filter_are_rejected(filt, dts):
    """ptree.rs:406-415: a connection/session-level filter may not test per-packet fields; the
    reference panics while building the FilterLayer::Packet tree (filtergen rejects it)."""
    with pytest.raises(pc.FilterError):
        pc.Program.from_filter(filt, (dts,))
    # the same predicates are fine in a packet-level subscription
    pc.Program.from_filter(filt.replace(" and tls", ""), ("ZcFrame",))


@pytest.mark.parametrize("fset", list(SETS))
def test_statement_table_matches_oracle(fset):
    prog = pc.Program.from_spec(SETS[fset])
    subs = helpers.subs_from_spec(SETS[fset])
    pf = oconn.PacketFilter(filterlang.ConnTree(subs).to_json(), subs)
    subs, kinds = prog.conn_table()
    assert [(int(s), int(k)) for s, k in zip(subs, kinds)] == pf.stmts
    assert prog.info["n_conn_stmts"] == len(pf.stmts)


def _cshape(j: dict):
    return (j["pred"], j["data"], j["terminal"], sorted(j["deliver"]), sorted(j["stream"]), j["if_else"],
            [_cshape(c) for c in j["children"]])


CONN_FILTERS = ["tcp.port = 80", "ipv4.addr = 10.0.0.0/8 and tcp", "tls", "http and tcp.port != 80", "udp.port = 53",
                "ipv6.dst_addr = 2001:db8::/32 and udp", "tcp.src_port >= 1024 and ipv4.dst_addr != 10.0.0.0/8",
                "dns and ((tcp and tcp.port != 53) or (udp and udp.port != 53))", "tls.sni ~ 'a'", "ipv4 or ipv6",
                "quic", "ssh and tcp.dst_port = 22", "tcp.dst_port in 1000..2000", "", "udp"]
CONN_DTS = [["ConnRecord"], ["FiveTuple"], ["FiveTuple", "FilterStr"], ["TlsHandshake"], ["ZcFrame"],
            ["Payload", "CoreId"], ["PktCount", "FiveTuple"], ["SessionList"], ["OrigZcPktStream"],
            ["HttpTransaction", "FiveTuple"], ["ConnRecord", "CoreId"]]


def test_conn_tree_matches_oracle_restatement():
    """The compiler's FilterLayer::Packet tree equals the oracle's (filterlang.ConnTree, a
    restatement of filter_subtree + collapse with SubscriptionSpec::packet_filter's actions) on
    every filter set and on random subscription sets."""
    for fset, spec in SETS.items():
        prog = pc.Program.from_spec(spec)
        assert _cshape(prog.tree_json(1)) == _cshape(filterlang.ConnTree(helpers.subs_from_spec(spec)).to_json()), fset
    rng = np.random.default_rng(8)
    checked = 0
    for _ in range(150):
        subs = []
        for k in range(int(rng.integers(1, 6))):
            f = CONN_FILTERS[int(rng.integers(0, len(CONN_FILTERS)))]
            d = CONN_DTS[int(rng.integers(0, len(CONN_DTS)))]
            stream = ("packets=1",) if rng.random() < 0.1 and d in (["PktCount", "FiveTuple"], ["ConnRecord"]) else ()
            subs.append((f, d, f"cb{k}", *stream))
        spec = synth._toml(subs)
        try:
            prog = pc.Program.from_spec(spec)
        except pc.FilterError:
            with pytest.raises(filterlang.FilterError):
                filterlang.ConnTree(helpers.subs_from_spec(spec))
            continue
        want = filterlang.ConnTree(helpers.subs_from_spec(spec))
        assert _cshape(prog.tree_json(1)) == _cshape(want.to_json()), spec
        assert prog.info["conn_tree_size"] == want.size
        checked += 1
    assert checked > 100


def test_conn_tree_json_matches_display():
    prog = pc.Program.from_spec(SETS["conn"])
    t = prog.tree_json(1)
    n = [0]

    def walk(x):
        n[0] += 1
        for c in x["children"]:
            walk(c)

    walk(t)
    assert n[0] == prog.info["conn_tree_size"]
    assert t["pred"] == "ethernet" and "0: ethernet" in prog.conn_tree


@pytest.mark.parametrize("fset", ["conn", "cfg4", "quirks", "cfg3"])
def test_oracle_reproduces_conn_golden(fset):
    g = np.load(GOLD / f"golden_{fset}.npz")
    t = np.load(GOLD / "corpus_adversarial.npz")
    slab, dlen = t["slab"], t["dlen"]
    fwd = np.unpackbits(g["adversarial_fwd"])[:len(dlen)].astype(bool)
    hi, cdm = helpers.oracle_conn(SETS[fset], slab, 128, dlen, fwd)
    assert np.array_equal(hi, g["adversarial_conn"])
    assert np.array_equal(cdm, g["adversarial_cdm"])


def test_conn_golden_covers_every_outcome():
    g = np.load(GOLD / "golden_conn.npz")
    info = np.concatenate([g[f"{c}_conn"][:, 1] for c in ("traces", "adversarial", "synth")])
    assert (info >> 26 & 1).any() and not (info >> 26 & 1).all()       # creates both ways
    assert (info >> 27 & 1).any() and not (info >> 27 & 1).all()       # both orientations
    assert (info >> 28 & 1).any()                                         # statements fired
    terms = set((info >> 13 & 0x1FFF).tolist())
    assert len(terms) >= 3
    cdm = np.concatenate([g[f"{c}_cdm"] for c in ("traces", "adversarial", "synth")])
    stmts = pc.Program.from_spec(SETS["conn"]).conn_table()[1]
    fired_kinds = {int(stmts[k]) for k in range(len(stmts)) if (cdm[:, 0] >> np.uint64(k) & np.uint64(1)).any()}
    assert fired_kinds == {oconn.STMT_CALLBACK, oconn.STMT_STREAM}


# ---------------------------------------------------------------------------------------------
# GPU: the kernel's connection stage

def _corpus(name: str):
    if name == "traces":
        t = np.load(GOLD / "traces.npz")
        return t["slab"], t["dlen"]
    if name == "adversarial":
        t = np.load(GOLD / "corpus_adversarial.npz")
        return t["slab"], t["dlen"]
    s2, d2 = synth.cfg2(2048, start=12345)
    s2 = np.pad(s2.reshape(-1, 64), ((0, 0), (0, 64))).reshape(-1)
    s3, d3 = synth.cfg3(2048, start=777)
    s4, d4 = synth.cfg4(2048, start=999)
    return np.concatenate([s2, s3, s4]), np.concatenate([d2, d3, d4])


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["mono", "split"])
@pytest.mark.parametrize("corpus", ["traces", "adversarial", "synth"])
@pytest.mark.parametrize("fset", list(SETS))
def test_conn_stage_golden(fset, corpus, layout, gpu):
    g = np.load(GOLD / f"golden_{fset}.npz")
    slab, dlen = _corpus(corpus)
    got = helpers.gpu_run(SETS[fset], slab, 128, dlen, split=layout == "split", conn=True)
    n = len(dlen)
    assert np.array_equal(got["fwd"], np.unpackbits(g[f"{corpus}_fwd"])[:n].astype(bool))
    exp = g[f"{corpus}_conn"]
    assert got["conn"].shape == exp.shape
    bad = np.nonzero((got["conn"] != exp).any(1))[0]
    assert bad.size == 0, f"{fset}/{corpus}: conn differs at records {bad[:8]}: {got['conn'][bad[:4]]} vs {exp[bad[:4]]}"
    if got["program"].info["conn_words"]:
        assert np.array_equal(got["cdm"], g[f"{corpus}_cdm"])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,fset,stride", [("cfg3", "conn", 128), ("cfg4", "cfg4", 128), ("cfg2", "conn", 64)])
def test_conn_stage_vs_oracle(cfg, fset, stride, gpu):
    n = (1 << 14) + 29
    gen = {"cfg2": synth.cfg2, "cfg3": synth.cfg3, "cfg4": synth.cfg4}[cfg]
    slab, dlen = gen(n, start=31337)
    got = helpers.gpu_run(SETS[fset], slab, stride, dlen, conn=True)
    hi, cdm = helpers.oracle_conn(SETS[fset], slab, stride, dlen, got["fwd"])
    assert np.array_equal(got["conn"], hi)
    if got["program"].info["conn_words"]:
        assert np.array_equal(got["cdm"], cdm)


@pytest.mark.gpu
def test_conn_stage_leaves_other_outputs_alone(gpu):
    slab, dlen = synth.cfg3((1 << 15) + 3, start=99)
    a = helpers.gpu_run(SETS["conn"], slab, 128, dlen, conn=True)
    b = helpers.gpu_run(SETS["conn"], slab, 128, dlen, conn=False)
    helpers.assert_same(a, b, "conn on/off")


def _random_conn_spec(seed: int) -> str | None:
    """A random subscription set over CONN_FILTERS x CONN_DTS (as the tree test above draws them),
    or None when filtergen would reject it."""
    rng = np.random.default_rng(100 + seed)
    subs = []
    for k in range(int(rng.integers(2, 7))):
        f = CONN_FILTERS[int(rng.integers(0, len(CONN_FILTERS)))]
        d = CONN_DTS[int(rng.integers(0, len(CONN_DTS)))]
        stream = ("packets=1",) if rng.random() < 0.1 and d in (["PktCount", "FiveTuple"], ["ConnRecord"]) else ()
        subs.append((f, d, f"cb{k}", *stream))
    spec = synth._toml(subs)
    try:
        pc.Program.from_spec(spec)
    except pc.FilterError:
        return None
    return spec


def test_random_conn_specs_compile():
    """Most of the GPU test's random sets are valid (the test below is not vacuous)."""
    assert sum(_random_conn_spec(s) is not None for s in range(12)) >= 8


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_conn_stage_random_sets(seed, gpu):
    """The first-packet filter (FilterLayer::Packet), ConnId and creates bits of random
    subscription sets, bit-exact against the oracle on the adversarial + synthetic corpora, in
    the monolithic, split and compact split layouts."""
    spec = _random_conn_spec(seed)
    if spec is None:
        pytest.skip("filtergen rejects this random set")
    s1, d1 = _corpus("adversarial")
    s2, d2 = _corpus("synth")
    slab, dlen = np.concatenate([s1, s2]), np.concatenate([d1, d2])
    layout = ("mono", "split", "compact")[seed % 3]
    got = helpers.gpu_run(spec, slab, 128, dlen, split=False if layout == "mono" else
                          ("compact" if layout == "compact" else True), conn=True)
    hi, cdm = helpers.oracle_conn(spec, slab, 128, dlen, got["fwd"])
    assert np.array_equal(got["conn"], hi), f"seed {seed} ({layout})"
    if got["program"].info["conn_words"]:
        assert np.array_equal(got["cdm"], cdm), f"seed {seed} ({layout})"
