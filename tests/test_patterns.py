"""The accept bit and the delivered-callback set against pattern semantics (oracle/patterns.py),
which needs no PTree: every golden fixture (their expected outputs come from the tree-based
oracle), and seeded random subscription sets through the tree-based C oracle. A bug the
product compiler and the oracle's tree share would show up here."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import helpers
import randsubs
from golden.filter_sets import SETS
from oracle import cgen, filterlang, packet, patterns
from retina_amd import synth

GOLD = Path(__file__).resolve().parent / "golden"


def _fixture_corpora() -> dict:
    t = np.load(GOLD / "traces.npz")
    a = np.load(GOLD / "corpus_adversarial.npz")
    # the synthetic corpus of make_golden.py:corpora (cfg2 padded to 128-B slots, cfg3, cfg4)
    s2, d2 = synth.cfg2(2048, start=12345)
    s2 = np.pad(s2.reshape(-1, 64), ((0, 0), (0, 64))).reshape(-1)
    s3, d3 = synth.cfg3(2048, start=777)
    s4, d4 = synth.cfg4(2048, start=999)
    return {"traces": (t["slab"], t["dlen"]), "adversarial": (a["slab"], a["dlen"]),
            "synth": (np.concatenate([s2, s3, s4]), np.concatenate([d2, d3, d4]))}


CORPORA = _fixture_corpora()


def _stmt_as_str(subs, tree) -> list[str]:
    return [subs[sid].as_str for sid, _ in packet.statement_table(tree)]


def _dm_sets(dm: np.ndarray, names: list[str]) -> list[set[str]]:
    out = []
    for row in dm:
        s = set()
        for k, nm in enumerate(names):
            if (int(row[k // 64]) >> (k % 64)) & 1:
                s.add(nm)
        out.append(s)
    return out


def _check(ps: patterns.PatternSet, slab, dlen, pc, dm, names, what):
    epc, edl = patterns.evaluate_batch(ps, slab, 128, dlen)
    bad = [i for i in range(len(dlen)) if bool(pc[i]) != epc[i]]
    assert not bad, f"{what}: accept bit differs from pattern semantics at frames {bad[:10]} ({len(bad)})"
    got = _dm_sets(dm, names) if names else [set()] * len(dlen)
    bad = [i for i in range(len(dlen)) if got[i] != edl[i]]
    assert not bad, f"{what}: delivered callbacks differ at {bad[:5]}: {[got[i] for i in bad[:3]]} vs {[edl[i] for i in bad[:3]]}"


@pytest.mark.parametrize("corpus", list(CORPORA))
@pytest.mark.parametrize("fset", list(SETS))
def test_golden_fixtures_follow_pattern_semantics(fset, corpus):
    subs = filterlang.load_spec(SETS[fset])
    g = np.load(GOLD / f"golden_{fset}.npz")
    slab, dlen = CORPORA[corpus]
    n = len(dlen)
    pc = np.unpackbits(g[f"{corpus}_pc"])[:n]
    tree = filterlang.PacketTree(subs)
    _check(patterns.PatternSet(subs), slab, dlen, pc, g[f"{corpus}_dm"], _stmt_as_str(subs, tree),
           f"{fset}/{corpus}")


def _random_corpus():
    slab, dlen = CORPORA["adversarial"]
    s, d = CORPORA["synth"]
    return np.concatenate([slab, s[: 1000 * 128]]), np.concatenate([dlen, d[:1000]])


QUIRK_FRAMES: dict[int, int] = {}


@pytest.mark.parametrize("seed", range(32))
def test_random_sets_tree_oracle_vs_pattern_semantics(seed):
    """Per frame: (1) the generated C oracle equals the Python tree walk (accept bit and statement
    mask); (2) the tree walked without `else if` chaining equals pattern semantics (accept bit and
    delivered callback set), which pins the tree's content -- nodes, nesting, actions, deliveries,
    pruning -- independently of the tree compiler; (3) where the real, chained walk differs from
    pattern semantics, a chain skipped a sibling whose condition held. That is the reference's
    own behaviour: mark_mutual_exclusion (ptree.rs:527-552) compares adjacent siblings only, and
    filtergen chains every marked sibling into one `if / else if` run (utils.rs:348-360), so a
    later sibling is skipped when any earlier one of the run matched even if the two are neither
    exclusive nor outcome-equal."""
    subs = randsubs.random_subs(1000 + seed)
    slab, dlen = _random_corpus()
    tree = filterlang.PacketTree(subs)
    r = cgen.OracleLib(tree).eval(slab, 128, dlen)
    names = _stmt_as_str(subs, tree)
    ps = patterns.PatternSet(subs)
    b = slab.reshape(-1, 128)
    quirks = 0
    for i in range(len(dlen)):
        fr, dl = b[i].tobytes(), int(dlen[i])
        tr: dict = {}
        act, fired = packet.evaluate(tree, fr, dl, trace=tr)
        mask = 0
        for k in fired:
            mask |= 1 << k
        got = sum(int(r["dm"][i, w]) << (64 * w) for w in range(r["dm"].shape[1]))
        assert bool(act & 1) == bool(r["pc"][i]) and mask == got, (seed, i)
        act0, fired0 = packet.evaluate(tree, fr, dl, chains=False)
        want = ps.evaluate(fr, dl)
        assert (bool(act0 & 1), {names[k] for k in fired0}) == want, \
            f"seed {seed} frame {i}: unchained tree {act0 & 1} {fired0} vs pattern semantics {want}"
        if (bool(act & 1), {names[k] for k in fired}) != want:
            assert tr.get("skipped", 0) > 0, f"seed {seed} frame {i}: differs from pattern semantics without a chain skip"
            quirks += 1
    QUIRK_FRAMES[seed] = quirks


def test_chain_quirk_minimal():
    """A hand-sized instance of the chaining quirk above (found by the random sets, seed 4). The
    collapsed tree has the binary siblings [src in 10.18.0.0/16 -> tcp -> ..., src = 10.0.0.2 (PC),
    src != 255.255.255.255 (PC)]: each is exclusive or outcome-equal with its left neighbour, so
    all three form one `if / else if` run. A UDP frame from 10.18.1.1 takes the first branch
    (which delivers only for TCP) and never reaches `src != 255.255.255.255`, so the reference's
    packet_continue drops it although the third subscription's filter matches it."""
    subs = [filterlang.Sub("tcp.rst = 0 and ipv4.src_addr = 10.18.0.0/16", ["ZcFrame"], "a"),
            filterlang.Sub("ipv4.src_addr = 10.0.0.2", ["ConnRecord"], "b"),
            filterlang.Sub("ipv4.src_addr != 255.255.255.255", ["ConnRecord"], "c")]
    tree = filterlang.PacketTree(subs)
    frame = helpers.build_frame(src=0x0A120101, dst=0x0A000002, proto=17)
    assert patterns.PatternSet(subs).evaluate(frame)[0] is True          # what the filters say
    tr: dict = {}
    assert packet.evaluate(tree, frame, trace=tr)[0] == 0 and tr["skipped"] == 1   # what the code does
    assert packet.evaluate(tree, frame, chains=False)[0] == 1
    slab = np.zeros(128, np.uint8)
    slab[:len(frame)] = np.frombuffer(frame, np.uint8)
    assert not cgen.OracleLib(tree).eval(slab, 128, np.array([len(frame)], np.uint16))["pc"][0]
    from retina_amd import pc

    prod = pc.Program.from_spec(randsubs.to_toml(subs))
    assert prod.tree == tree.pprint() and " x" in prod.tree


def test_random_sets_product_compiler_accepts_them():
    """Every random set the oracle accepts, the product compiler accepts with the same tree."""
    from retina_amd import pc

    for seed in range(40):
        subs = randsubs.random_subs(1000 + seed)
        prod = pc.Program.from_spec(randsubs.to_toml(subs))
        assert prod.tree == filterlang.PacketTree(subs).pprint(), seed


def test_ethernet_wrap_quirk():
    """The root outcome of a pattern-less subscription runs outside `if let Ok(ethernet)` only
    while the collapsed root has no children (utils.rs:371-378): a 10-byte frame is accepted by
    {"" ConnRecord} alone, and dropped once a ZcFrame subscription on `tcp` adds a child."""
    short = bytes(10)
    alone = [filterlang.Sub("", ["ConnRecord"], "c")]
    both = alone + [filterlang.Sub("tcp", ["ZcFrame"], "z")]
    same_cb = [filterlang.Sub("", ["ZcFrame"], "z"), filterlang.Sub("tcp", ["ZcFrame"], "z"),
               filterlang.Sub("", ["ConnRecord"], "c")]
    for subs, want in ((alone, True), (both, False), (same_cb, True)):
        ps = patterns.PatternSet(subs)
        assert ps.evaluate(short)[0] is want, [s.filter for s in subs]
        tree = filterlang.PacketTree(subs)
        act, _ = packet.evaluate(tree, short)
        assert bool(act & 1) is want
        slab = np.zeros(128, np.uint8)
        assert bool(cgen.OracleLib(tree).eval(slab, 128, np.array([10], np.uint16))["pc"][0]) is want


def test_cfg_sets_match_on_golden_with_helpers():
    """helpers.oracle_run (the GPU tests' reference) agrees with pattern semantics on cfg4's
    42 subscriptions over the synthetic corpus."""
    subs = filterlang.load_spec(SETS["cfg4"])
    slab, dlen = CORPORA["synth"]
    r = helpers.oracle_run(SETS["cfg4"], slab, 128, dlen)
    epc, _ = patterns.evaluate_batch(patterns.PatternSet(subs), slab, 128, dlen)
    assert np.array_equal(r["pc"], np.array(epc))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_random_sets(gpu, seed):
    """The product (compiler + gfx950 kernel) on random subscription sets: bit-exact against the
    tree-based C oracle on the adversarial + synthetic corpus (the CPU test above ties that
    oracle to pattern semantics), in 128-B monolithic slots and in the split layout."""
    spec = randsubs.to_toml(randsubs.random_subs(1000 + seed))
    slab, dlen = _random_corpus()
    exp = helpers.oracle_run(spec, slab, 128, dlen)
    helpers.assert_same(helpers.gpu_run(spec, slab, 128, dlen, split=bool(seed & 1)), exp, f"random set {seed}")
