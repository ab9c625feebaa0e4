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
