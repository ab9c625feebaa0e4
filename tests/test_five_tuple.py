"""FiveTuple orientation and format against the reference's own end-to-end golden output.

tests/golden/basic_five_tuples.json holds the 60 `five_tuple`s that the reference's basic_test
printed (tests/functionality/basic_test/expected_output_basic.txt; make_basic_tuples.py). Its
pcap is absent, so for every tuple the connection is re-created as frames: the originator's SYN,
the responder's SYN|ACK and a client data segment. Retina keys the connection by ConnId (the
SocketAddr max/min pair, conn_id.rs:111-117), opens it on the SYN (Conn::new_tcp,
conn/mod.rs:53-96) and keeps the first packet's L4Context as the FiveTuple
(FiveTuple::from_ctxt, conn_id.rs:32-38; ConnInfo::new, conn_info.rs:33-39), whose serde form
is {"orig": "<ip>:<port>", "resp": ..., "proto": 6}. The tests rebuild that object from the
product's outputs (the opener's L4Context, its rtn_conn_t orientation bit, the connection
table's NEW/HIT outcome) and compare it with the reference's text.
"""
from __future__ import annotations

import ipaddress
import json
from pathlib import Path

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from oracle import conn as oconn
from oracle import filterlang, packet

TUPLES = json.loads((Path(__file__).resolve().parent / "golden" / "basic_five_tuples.json").read_text())
SPEC = SETS["basic"]  # examples/basic: tls and dns subscriptions (PacketContinue at the L4 nodes)
SYN, SYNACK, PSHACK = 0x02, 0x12, 0x18


def _ep(s: str) -> tuple[int, int]:
    ip, port = s.rsplit(":", 1)
    return int(ipaddress.IPv4Address(ip)), int(port)


def _fmt(ip: int, port: int) -> str:
    return f"{ipaddress.IPv4Address(ip)}:{port}"  # SocketAddrV4 Display


def _frames() -> tuple[list[bytes], list[tuple[int, int]]]:
    """Per tuple: SYN orig->resp, SYN|ACK resp->orig, PSH|ACK orig->resp; (tuple index, kind)."""
    frames, tags = [], []
    for k, t in enumerate(TUPLES):
        (oa, op), (ra, rp) = _ep(t["orig"]), _ep(t["resp"])
        frames.append(helpers.build_frame(False, oa, ra, op, rp, 6, SYN))
        frames.append(helpers.build_frame(False, ra, oa, rp, op, 6, SYNACK))
        frames.append(helpers.build_frame(False, oa, ra, op, rp, 6, PSHACK, payload=b"\x16\x03\x01\x00\x05hello"))
        tags += [(k, 0), (k, 1), (k, 2)]
    return frames, tags


def test_fixture_is_the_reference_output(reference_dir):
    text = (reference_dir / "tests/functionality/basic_test/expected_output_basic.txt").read_text()
    recs, _ = json.JSONDecoder().raw_decode(text)
    assert [r["five_tuple"] for r in recs] == TUPLES and len(TUPLES) == 60


def test_oracle_five_tuples():
    """The oracle's L4Context / ConnId / TableModel give the reference's 60 FiveTuples."""
    frames, tags = _frames()
    subs = filterlang.load_spec(SPEC)
    tree = filterlang.PacketTree(subs)
    pf = oconn.PacketFilter(filterlang.ConnTree(subs).to_json(), subs)
    model = oconn.TableModel()
    ctxs = []
    for f in frames:
        act, _ = packet.evaluate(tree, f)
        assert act & 1
        ctxs.append(packet.l4context(f + bytes(64), len(f)))
    st = model.process([(oconn.conn_key(c), oconn.creates(c), pf.evaluate(f, len(f))[:2] == (0, 0))
                        for c, f in zip(ctxs, frames)])
    got = {}
    for (k, kind), c, (key, status) in zip(tags, ctxs, st):
        if kind == 0:
            assert status == oconn.CT_NEW
            got[k] = {"orig": _fmt(c.src, c.sport), "resp": _fmt(c.dst, c.dport), "proto": c.proto}
        else:
            assert status == oconn.CT_HIT
    assert [got[k] for k in range(len(TUPLES))] == TUPLES
    # the reply is the same connection seen the other way round
    for j in range(0, len(frames), 3):
        a, b = oconn.conn_id(ctxs[j]), oconn.conn_id(ctxs[j + 1])
        assert a[1:] == b[1:] and a[0] != b[0]


@pytest.mark.gpu
@pytest.mark.parametrize("batches", [1, 3])
def test_gpu_five_tuples(gpu, batches):
    """The product's packet stage + connection stage + connection table rebuild the reference's
    60 FiveTuples: the SYN opens the connection (NEW) and its record gives orig/resp; the SYN|ACK
    and the data segment find the same slot (HIT) with the same ConnId hash, and their
    RTN_CONN_SRC_IS_MAX bit says which endpoint sent them. batches=3 hands SYNs, replies and data
    over in three separate batches, so the later ones meet a connection that predates them."""
    import torch

    from retina_amd import pc

    frames, tags = _frames()
    prog = pc.Program.from_spec(SPEC)
    ctx = pc.PacketContinue(prog, 0)
    ct = pc.ConnTable(0, 12)
    dev = torch.device("cuda", 0)
    order = [list(range(len(frames)))] if batches == 1 else [list(range(kind, len(frames), 3)) for kind in range(3)]
    res: dict[int, dict] = {}
    for idx in order:
        slab, dlen = pc.pack_frames([frames[i] for i in idx], 128)
        out = ctx.alloc_outputs(len(idx), conn=True)
        ctx.run(torch.from_numpy(slab).to(dev), 128, torch.from_numpy(dlen.view(np.int16)).to(dev), len(idx), out)
        ent = ct.process(out)
        torch.cuda.synchronize()
        d = out.decode()
        assert d["fwd"].all()
        cte = pc.decode_ct(ent, out)
        for j, i in enumerate(idx):
            r = d["l4"][j]
            res[i] = {"src": (int(r["src_ip4"]), int(r["sport"])), "dst": (int(r["dst_ip4"]), int(r["dport"])),
                      "proto": int(r["proto"]), "hash": int(d["conn_hash"][j]),
                      "src_is_max": bool((int(d["conn_info"][j]) >> 27) & 1), "slot": int(cte[j, 0]),
                      "status": int(cte[j, 1])}
    got = []
    for k in range(len(TUPLES)):
        syn, rep, dat = res[3 * k], res[3 * k + 1], res[3 * k + 2]
        assert syn["status"] & 0xFF == pc.CT_NEW
        assert rep["status"] & 0xFF == pc.CT_HIT and dat["status"] & 0xFF == pc.CT_HIT
        assert bool(rep["status"] & pc.CT_PRIOR) == (batches == 3)
        assert syn["slot"] == rep["slot"] == dat["slot"] != pc.CT_NO_SLOT
        assert syn["hash"] == rep["hash"] == dat["hash"]
        # orientation: the opener's bit names the originator; a frame from the originator repeats it
        assert rep["src_is_max"] != syn["src_is_max"] and dat["src_is_max"] == syn["src_is_max"]
        got.append({"orig": _fmt(*syn["src"]), "resp": _fmt(*syn["dst"]), "proto": syn["proto"]})
        # FiveTuple of the later frames, oriented by the opener's bit
        for f in (rep, dat):
            o, r = (f["src"], f["dst"]) if f["src_is_max"] == syn["src_is_max"] else (f["dst"], f["src"])
            assert {"orig": _fmt(*o), "resp": _fmt(*r), "proto": f["proto"]} == got[-1]
    assert got == TUPLES
