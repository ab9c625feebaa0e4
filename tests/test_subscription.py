"""retina_amd.subscription: the host mirror of Retina's Subscription for the packet stage. Its
per-core stats (core/src/stats/mod.rs names) must equal what rx_core.rs:127-139 and
Subscription::process_packet (subscription/mod.rs:102-111) count for the same frames, computed
here from the oracle; its forwarded frames / L4Contexts and packet-level callbacks must equal the
oracle's."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from oracle import filterlang, packet

GOLD = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


def _expected_stats(spec, slab, dlen):
    r = helpers.oracle_run(spec, slab, 128, dlen)
    dl = dlen.astype(np.int64)
    idx = r["rec"]["idx"].astype(np.int64)
    tcp = r["rec"]["proto"] == 6
    return r, {"TOTAL_PKT": len(dlen), "TOTAL_BYTE": int(dl.sum()),
               "IGNORED_BY_PACKET_FILTER_PKT": int((~r["pc"]).sum()), "IGNORED_BY_PACKET_FILTER_BYTE": int(dl[~r["pc"]].sum()),
               "TCP_PKT": int(tcp.sum()), "TCP_BYTE": int(dl[idx[tcp]].sum()),
               "UDP_PKT": int((~tcp).sum()), "UDP_BYTE": int(dl[idx[~tcp]].sum())}


@pytest.mark.parametrize("fset", ["payload", "cfg3", "quirks"])
def test_subscription_mirror(fset, gpu):
    import torch

    from retina_amd.subscription import PACKET_CONTINUE, Subscription

    t = np.load(GOLD / "traces.npz")
    a = np.load(GOLD / "corpus_adversarial.npz")
    spec = SETS[fset]
    sub = Subscription(spec)
    totals = {}
    for slab, dlen in ((t["slab"], t["dlen"]), (a["slab"], a["dlen"])):
        r, want = _expected_stats(spec, slab, dlen)
        b = sub.run(torch.from_numpy(slab).cuda(), 128, torch.from_numpy(dlen.view(np.int16)).cuda())
        assert b.stats == want
        for k, v in want.items():
            totals[k] = totals.get(k, 0) + v
        assert [b.continue_packet(i) for i in range(len(dlen))] == [PACKET_CONTINUE if x else 0 for x in r["pc"]]
        got = list(b.process_packets())
        assert [i for i, _ in got] == list(r["rec"]["idx"])
        for (i, c), x in zip(got, r["rec"]):
            w = 4 if c.src[0].version == 4 else 16
            assert (c.src[0].packed + bytes(16 - w), c.dst[0].packed + bytes(16 - w)) == (bytes(x["src"]), bytes(x["dst"]))
            assert (c.src[1], c.dst[1], c.proto, c.offset, c.length, c.seq_no, c.ack_no, c.flags) == \
                (x["sport"], x["dport"], x["proto"], x["offset"], x["length"], x["seq"], x["ack"], x["flags"])
        # packet-level callbacks in call order, from the Python restatement of packet_continue
        tree = filterlang.PacketTree(filterlang.load_spec(spec))
        st = packet.statement_table(tree)
        subs = filterlang.load_spec(spec)
        cb = dict(b.packet_callbacks())
        rows = slab.reshape(-1, 128)
        for i in range(len(dlen)):
            _, fired = packet.evaluate(tree, rows[i].tobytes(), int(dlen[i]))
            want_calls = [(st[k][0], subs[st[k][0]].callback, st[k][1]) for k in fired]
            assert cb.get(i, []) == want_calls, i
    assert sub.stats == totals


CHECK = Path(__file__).resolve().parent.parent / "retina_amd" / "_lib" / "subscription_check"


def _run_cpp(spec: str, slab: np.ndarray, dlen: np.ndarray, tmp_path) -> dict:
    """tests/cpp/subscription_check.cpp (include/retina_subscription.hpp) on one burst."""
    import subprocess

    (tmp_path / "spec.toml").write_text(spec)
    (tmp_path / "slab.bin").write_bytes(np.ascontiguousarray(slab, np.uint8).tobytes())
    (tmp_path / "dlen.bin").write_bytes(np.ascontiguousarray(dlen, np.uint16).tobytes())
    r = subprocess.run([str(CHECK), str(tmp_path / "spec.toml"), str(tmp_path / "slab.bin"), str(tmp_path / "dlen.bin")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = {"pc": [], "l4": [], "cb": [], "stat": {}}
    for line in r.stdout.splitlines():
        f = line.split()
        if f[0] == "pc":
            out["pc"].append(int(f[1]))
        elif f[0] == "l4":
            out["l4"].append(f[1:])
        elif f[0] == "cb":
            out["cb"].append((int(f[1]), int(f[2]), f[3], f[4]))
        else:
            out["stat"][f[1]] = int(f[2])
    return out


@pytest.mark.parametrize("fset", ["payload", "cfg4", "quirks"])
def test_cpp_subscription_mirror(fset, gpu, tmp_path):
    """The C++ mirror (include/retina_subscription.hpp) over the C ABI: continue_packet,
    process_packet's L4Contexts, the packet-level callbacks in call order and the stats, each
    equal to the oracle on the traces + adversarial corpus."""
    t = np.load(GOLD / "traces.npz")
    a = np.load(GOLD / "corpus_adversarial.npz")
    slab, dlen = np.concatenate([t["slab"], a["slab"]]), np.concatenate([t["dlen"], a["dlen"]])
    spec = SETS[fset]
    got = _run_cpp(spec, slab, dlen, tmp_path)
    r, want_stats = _expected_stats(spec, slab, dlen)
    assert got["stat"] == want_stats
    assert got["pc"] == list(np.nonzero(r["pc"])[0])
    assert [int(x[0]) for x in got["l4"]] == list(r["rec"]["idx"])
    for g, x in zip(got["l4"], r["rec"]):
        v6 = "." not in g[1]
        src = bytes.fromhex(g[1]) if v6 else bytes(int(b) for b in g[1].split("."))
        dst = bytes.fromhex(g[3]) if v6 else bytes(int(b) for b in g[3].split("."))
        w = len(src)
        assert (src + bytes(16 - w), dst + bytes(16 - w)) == (bytes(x["src"]), bytes(x["dst"]))
        assert [int(v) for v in (g[2], g[4], g[5], g[6], g[7], g[8], g[9], g[10])] == \
            [x["sport"], x["dport"], x["proto"], x["offset"], x["length"], x["seq"], x["ack"], x["flags"]]
    tree = filterlang.PacketTree(filterlang.load_spec(spec))
    st = packet.statement_table(tree)
    subs = filterlang.load_spec(spec)
    rows = slab.reshape(-1, 128)
    want_cb = []
    for i in range(len(dlen)):
        _, fired = packet.evaluate(tree, rows[i].tobytes(), int(dlen[i]))
        want_cb += [(i, st[k][0], subs[st[k][0]].callback, st[k][1]) for k in fired]
    assert got["cb"] == want_cb
