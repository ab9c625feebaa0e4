"""Per-packet parse and ConnId pinned by what the reference says about its own traces.

traces/README.md describes `tls_ciphers.pcap` as "OpenSSL client/server GET requests over TLS 1.2
with 73 different cipher suites" (one TCP connection per cipher suite) and `quic_xargs.pcap` as
the capture behind "The Illustrated QUIC Connection" (one QUIC connection). Counting connections
needs every layer of this path: the Ethernet / IPv4 / TCP / UDP parse, L4Context (the 5-tuple),
ConnId's canonical endpoint order (conn_id.rs:111-117) and the open rule (a TCP SYN, any UDP
frame; conn/mod.rs:53-96). The frames are the reference's own pcaps (tests/golden/traces.npz).
"""
from __future__ import annotations

import collections

import numpy as np
import pytest

from golden.filter_sets import SETS
from oracle import conn as oconn
from oracle import packet

TRACES = np.load(__import__("pathlib").Path(__file__).resolve().parent / "golden" / "traces.npz", allow_pickle=False)
STRIDE = 128
# trace -> (connections the README implies, protocol)
FACTS = {"tls_ciphers.pcap": (73, 6), "quic_xargs.pcap": (1, 17)}


def _frames(name: str):
    names = list(TRACES["names"])
    idx = np.flatnonzero(TRACES["trace"] == names.index(name))
    slab = TRACES["slab"].reshape(-1, STRIDE)[idx]
    return np.ascontiguousarray(slab).reshape(-1), np.ascontiguousarray(TRACES["dlen"][idx])


def test_readme_states_the_facts(reference_dir):
    text = (reference_dir / "traces" / "README.md").read_text()
    assert "73 different cipher suites" in text and "`tls_ciphers.pcap`" in text
    assert "The Illustrated QUIC Connection" in text and "`quic_xargs.pcap`" in text


@pytest.mark.parametrize("name", list(FACTS))
def test_oracle_connections(name):
    want, proto = FACTS[name]
    slab, dlen = _frames(name)
    model = oconn.TableModel()
    keys, items = collections.Counter(), []
    for i in range(len(dlen)):
        fr = bytes(slab[i * STRIDE:i * STRIDE + min(int(dlen[i]), STRIDE)])
        c = packet.l4context(fr, int(dlen[i]))
        assert c is not None and c.proto == proto
        keys[oconn.conn_key(c)] += 1
        items.append((oconn.conn_key(c), oconn.creates(c), False))
    st = [s for _, s in model.process(items)]
    assert len(keys) == want
    assert st.count(oconn.CT_NEW) == want


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(FACTS))
def test_gpu_connections(gpu, name):
    """The product's packet stage + connection stage + table open exactly the connections the
    README describes, one NEW per connection, every other frame a HIT on one of them."""
    import torch

    from retina_amd import pc

    want, proto = FACTS[name]
    slab, dlen = _frames(name)
    n = len(dlen)
    ctx = pc.PacketContinue(pc.Program.from_spec(SETS["basic"]), gpu)
    ct = pc.ConnTable(gpu, 12)
    out = ctx.alloc_outputs(n, conn=True)
    dev = torch.device("cuda", gpu)
    ctx.run(torch.from_numpy(slab).to(dev), STRIDE, torch.from_numpy(dlen.view(np.int16)).to(dev), n, out)
    ent = ct.process(out)
    torch.cuda.synchronize()
    d = out.decode()
    assert d["fwd"][:n].all() and (d["l4"]["proto"] == proto).all()
    cte = pc.decode_ct(ent, out)
    status = cte[:, 1] & 0xFF
    assert int((status == pc.CT_NEW).sum()) == want == ct.stats()["live"]
    assert ((status == pc.CT_NEW) | (status == pc.CT_HIT)).all()
    assert len(np.unique(cte[:, 0])) == want
    # one ConnId hash per connection: frames of a slot share it, different slots differ
    slot_hash = {}
    for s, h in zip(cte[:, 0], d["conn_hash"]):
        assert slot_hash.setdefault(int(s), int(h)) == int(h)
    assert len(set(slot_hash.values())) == want
