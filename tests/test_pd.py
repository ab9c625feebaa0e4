"""PacketDeliver filter (include/retina_pd.h): the generated `packet_deliver` for the frames of
connections that hold the PacketDeliver action.

CPU tests pin the compiler's collapsed PacketDeliver tree against the oracle's own restatement
(oracle/filterlang.py DeliverTree) on fixed and random subscription sets, the statement table and
fact list against the oracle's numbering (oracle/conn.py DeliverFilter), the single-callback
collapse (ptree.rs:752-767), the session-loop replay, and hand-checked outcomes. The GPU test runs
batches through rtn_pc_run -> rtn_ct_process -> rtn_pd_run with random per-connection state and
compares every frame's callback sequence with the oracle's (on the oracle's own tree), exactly."""
from __future__ import annotations

import numpy as np
import pytest

import helpers
from oracle import conn as oconn
from oracle import filterlang
from retina_amd import pc

SPEC = """
[[subscriptions]]
filter = "tls"
datatypes = ["ZcFrame"]
callback = "tls_cb"

[[subscriptions]]
filter = "udp.dst_port = 53"
datatypes = ["ZcFrame"]
callback = "dns_cb"

[[subscriptions]]
filter = "tcp.port = 80 and http.user_agent ~ 'curl'"
datatypes = ["Payload"]
callback = "http_cb"

[[subscriptions]]
filter = "ipv4.addr = 10.0.0.0/8 and tls.sni ~ 'x'"
datatypes = ["ZcFrame", "FilterStr"]
callback = "t2_cb"

[[subscriptions]]
filter = "ipv6.src_addr = 2001:db8::/32 and dns"
datatypes = ["Payload", "CoreId"]
callback = "v6_cb"

[[subscriptions]]
filter = "http.user_agent ~ 'a' and http.method = 'GET'"
datatypes = ["ZcFrame"]
callback = "nested_cb"

[[subscriptions]]
filter = "tcp.port = 443"
datatypes = ["ConnRecord"]
callback = "conn_cb"
"""


def _setup(spec: str = SPEC):
    """Product program, its packet_deliver description, and the oracle's evaluator on the oracle's
    own tree (the facts are named by predicate text, which is the host interface)."""
    prog = pc.Program.from_spec(spec)
    pd = prog.pd_program()
    subs = helpers.subs_from_spec(spec)
    tree = filterlang.DeliverTree(subs).to_json()
    df = oconn.DeliverFilter(tree, subs, [f["pred"] for f in pd["facts"]])
    return prog, pd, df


def _shape(j: dict):
    return (j["pred"], sorted(j["deliver"]), j["if_else"], [_shape(c) for c in j["children"]])


PD_FILTERS = ["tls", "http", "dns", "quic", "ssh", "tcp.port = 80 and http", "ipv4.addr = 10.0.0.0/8 and tls",
              "tls.sni ~ 'a'", "http.user_agent ~ 'curl' and tcp.dst_port = 8080", "ipv6 and dns",
              "udp.port = 53 and dns", "tcp.port >= 1000 and ssh", "tls.sni = 'x.com'",
              "http.method = 'GET' and http.user_agent ~ 'a'", "ipv4.src_addr = 1.2.3.0/24 and quic",
              "tcp.port = 443", "udp", "ipv6.dst_addr = 2001:db8::/32 and tls.sni ~ 'b'", "tls or http",
              "tcp.dst_port = 443 and tls"]


def _random_spec(rng) -> str:
    out = []
    for k in range(int(rng.integers(2, 7))):
        f = PD_FILTERS[int(rng.integers(0, len(PD_FILTERS)))]
        r = rng.random()
        dts = ['"ZcFrame"'] if r < 0.4 else ['"Payload"'] if r < 0.6 else ['"ZcFrame"', '"FilterStr"'] if r < 0.8 \
            else ['"ConnRecord"']
        out.append(f'[[subscriptions]]\nfilter = "{f}"\ndatatypes = [{", ".join(dts)}]\ncallback = "cb{k}"\n')
    return "\n".join(out)


def test_pd_tree_matches_oracle_restatement():
    for spec in [SPEC]:
        prog = pc.Program.from_spec(spec)
        assert _shape(prog.tree_json(2)) == _shape(filterlang.DeliverTree(helpers.subs_from_spec(spec)).to_json())
    rng = np.random.default_rng(4)
    nontrivial = 0
    for _ in range(80):
        spec = _random_spec(rng)
        prog = pc.Program.from_spec(spec)
        want = filterlang.DeliverTree(helpers.subs_from_spec(spec))
        assert _shape(prog.tree_json(2)) == _shape(want.to_json()), spec
        assert prog.info["pd_tree_size"] == want.size
        nontrivial += want.size > 1
    assert nontrivial > 25


def test_pd_statement_table_matches_oracle_numbering():
    prog, pd, df = _setup()
    assert [s["sub"] for s in pd["stmts"]] == df.stmts
    assert prog.info["n_pd_stmts"] == len(pd["stmts"]) and prog.info["n_pd_facts"] == len(pd["facts"])
    kinds = {f["pred"]: f["kind"] for f in pd["facts"]}
    assert kinds["tls"] == "service" and kinds["dns"] == "service" and kinds["http"] == "service"
    assert kinds["tls.sni matches x"] == "session"
    assert len(kinds) == len(pd["facts"])  # one fact per distinct predicate
    # connection-level subscriptions never reach the packet-deliver tree (ptree.rs:330-333);
    # packet-only filters are delivered at PacketContinue (sub 1)
    subs = {s["sub"] for s in pd["stmts"]}
    assert 6 not in subs and 1 not in subs
    # nested session predicates give nested loops
    nested = [s for s in pd["stmts"] if s["sub"] == 5]
    assert nested and all(len(s["loops"]) == 2 for s in nested)
    assert "for session in tracked.sessions()" in prog.pd_rust


def test_pd_single_callback_collapses_to_root():
    # one packet-level callback: no disambiguation needed, the root delivers (ptree.rs:752-767)
    spec = '[[subscriptions]]\nfilter = "tls.sni ~ \'x\'"\ndatatypes = ["ZcFrame"]\ncallback = "cb"\n'
    prog, pd, df = _setup(spec)
    assert prog.info["pd_tree_size"] == 1 and pd["facts"] == []
    assert pd["stmts"] == [{"sub": 0, "payload": False, "callback": "cb", "loops": []}]
    f = helpers.build_frame(False, 1, 2, 3, 4, 17, 0)
    assert df.evaluate(f, len(f), []) == [0]


def test_pd_oracle_hand_checked():
    _, pd, df = _setup()
    st = [s["sub"] for s in pd["stmts"]]
    facts = {f["pred"]: k for k, f in enumerate(pd["facts"])}

    def F(**kv):
        v = [0] * len(pd["facts"])
        for p, x in kv.items():
            v[facts[p.replace("_", " ").replace("SNI", "tls.sni matches x").replace("UA", "http.user_agent matches a")
                     .replace("GET", "http.method = GET").replace("CURL", "http.user_agent matches curl")]] = x
        return v

    f = helpers.build_frame(False, 0x0A000001, 0x0B000002, 1234, 80, 6, 0x18, payload=b"abc")
    # src in 10/8 (dst is not): t2_cb once per matching TLS session
    seq = df.evaluate(f, len(f), F(tls=1, SNI=2))
    assert [st[k] for k in seq] == [3, 3, 0]
    # http service: nested loops 2 x 3, then the curl session once; Payload readable
    seq = df.evaluate(f, len(f), F(http=1, GET=2, UA=3, CURL=1))
    assert [st[k] for k in seq] == [5] * 6 + [2]
    # the same frame cut inside its payload: Payload::from_mbuf fails, ZcFrame still fires
    g = f[:-1]
    seq = df.evaluate(g, len(g), F(http=1, GET=1, UA=1, CURL=1))
    assert [st[k] for k in seq] == [5]
    # zero-length payload at the frame end: no Payload callback (offset < data_len fails)
    h = helpers.build_frame(False, 0x0A000001, 0x0B000002, 1234, 80, 6, 0x18)
    assert df.evaluate(h, len(h), F(http=1, CURL=1)) == []


def test_pd_replay_reproduces_loop_interleaving():
    prog, pd, df = _setup()
    rng = np.random.default_rng(2)
    for _ in range(300):
        facts = rng.integers(0, 4, len(pd["facts"]))
        for k, f in enumerate(pd["facts"]):
            if f["kind"] == "service":
                facts[k] = rng.integers(0, 2)
        v6 = bool(rng.random() < 0.4)
        src = (0x20010DB8 << 96 | int(rng.integers(0, 1 << 32))) if v6 and rng.random() < 0.5 else \
            int(rng.integers(0, 1 << 32)) << (96 if v6 else 0)
        f = helpers.build_frame(v6, src, int(rng.integers(0, 1 << 32)), int(rng.choice([80, 443, 53, 9])),
                                int(rng.choice([80, 53, 7])), int(rng.choice([6, 17])), 0x18,
                                payload=bytes(int(rng.integers(0, 3))))
        seq = df.evaluate(f, len(f), facts)
        counts = np.bincount(np.array(seq, np.int64), minlength=len(pd["stmts"]))
        assert pc.pd_replay(pd, counts, facts) == seq
        assert prog.pd_replay(counts, facts) == seq  # the C ABI's replay (rtn_program_pd_replay)


def _pd_pool(rng, n):
    pool, seen = [], set()
    while len(pool) < n:
        v6 = bool(rng.random() < 0.35)
        if v6:
            a = ((0x20010DB8 << 96) if rng.random() < 0.5 else (int(rng.integers(1, 1 << 31)) << 97)) | \
                int(rng.integers(0, 1 << 62))
            b = int(rng.integers(1, 1 << 62)) << 64
        else:
            a = (10 << 24 | int(rng.integers(0, 1 << 24))) if rng.random() < 0.4 else int(rng.integers(0, 1 << 32))
            b = int(rng.integers(0, 1 << 32))
        pa = int(rng.choice([80, 443, 53, 8080])) if rng.random() < 0.6 else int(rng.integers(1, 65536))
        pb = int(rng.integers(1024, 65536))
        proto = 6 if rng.random() < 0.7 else 17
        k = (v6, a, b, pa, pb, proto)
        if k not in seen:
            seen.add(k)
            pool.append(k)
    return pool


def _pd_frames(rng, pool, n, p_syn):
    frames = []
    for _ in range(n):
        v6, a, b, pa, pb, proto = pool[int(rng.integers(0, len(pool)))]
        if rng.random() < 0.5:
            a, b, pa, pb = b, a, pb, pa
        fl = 0x02 if rng.random() < p_syn else 0x18
        f = helpers.build_frame(v6, a, b, pa, pb, proto, fl, payload=bytes(int(rng.integers(0, 24))))
        if rng.random() < 0.1 and len(f) > 60:
            f = f[:-3]  # capture ends inside the payload: Payload::from_mbuf fails
        frames.append(f)
    return frames


@pytest.mark.gpu
def test_pd_gpu_vs_oracle(gpu):
    import torch

    prog, pd, df = _setup()
    ctx = pc.PacketContinue(prog, 0)
    ct = pc.ConnTable(0, 14)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    pool = _pd_pool(rng, 600)
    nf = len(pd["facts"])
    state = torch.zeros(ct.capacity * (1 + nf), dtype=torch.int32, device=dev)
    checked = delivered = 0
    for b, p_syn in enumerate((1.0, 0.1, 0.1)):
        frames = _pd_frames(rng, pool, 5000 + 77 * b, p_syn)
        slab, dlen = pc.pack_frames(frames, 128)
        d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
        out = ctx.alloc_outputs(len(frames), conn=True)
        ctx.run(torch.from_numpy(slab).to(dev), 128, d_dlen, len(frames), out)
        ent = ct.process(out)
        counts, bm = pc.pd_run(ctx, out, ent, d_dlen, state)
        torch.cuda.synchronize()
        fwd = np.nonzero(out.decode()["fwd"])[0]
        e = pc.decode_ct(ent, out)
        st_host = state.cpu().numpy().view(np.uint32).reshape(-1, 1 + nf)
        got_idx, got_cnt = pc.decode_pd(counts, bm, out, len(pd["stmts"]))
        got = dict(zip(got_idx.tolist(), got_cnt))
        for j, i in enumerate(fwd):
            slot, status = int(e[j, 0]), int(e[j, 1])
            exp = []
            if status == pc.CT_HIT | pc.CT_PRIOR and st_host[slot, 0] & pc.PD_ACTIVE:
                exp = df.evaluate(frames[i], len(frames[i]), st_host[slot, 1:])
                checked += 1
            if exp:
                assert i in got, f"frame {i}: expected {exp}, nothing delivered"
                assert pc.pd_replay(pd, got[i], st_host[slot, 1:]) == exp, f"frame {i}"
                delivered += 1
            else:
                assert i not in got, f"frame {i}: unexpected delivery {got[i]}"
        # the host's new per-connection state for the next batch: PacketDeliver on for ~60 %,
        # services 0/1, session counts 0..3
        live = np.unique(e[(e[:, 0] != pc.CT_NO_SLOT), 0])
        new = np.zeros((len(live), 1 + nf), np.uint32)
        new[:, 0] = rng.random(len(live)) < 0.6
        for k, f in enumerate(pd["facts"]):
            new[:, 1 + k] = rng.integers(0, 2 if f["kind"] == "service" else 4, len(live))
        st_all = state.view(-1, 1 + nf)
        st_all[torch.from_numpy(live.astype(np.int64)).to(dev)] = torch.from_numpy(new.view(np.int32)).to(dev)
    assert checked > 1000 and delivered > 200


@pytest.mark.gpu
def test_pd_gpu_ragged_batches_and_no_packet_subscriptions(gpu):
    import torch

    from golden.filter_sets import SETS

    prog, pd, df = _setup()
    ctx = pc.PacketContinue(prog, 0)
    ct = pc.ConnTable(0, 12)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(12)
    pool = _pd_pool(rng, 200)
    nf = len(pd["facts"])
    # open every flow, then give every connection PacketDeliver and facts of 1..2
    opener = _pd_frames(rng, pool, 3000, 1.0)
    slab, dlen = pc.pack_frames(opener, 128)
    out = ctx.alloc_outputs(len(opener), conn=True)
    ctx.run(torch.from_numpy(slab).to(dev), 128, torch.from_numpy(dlen.view(np.int16)).to(dev), len(opener), out)
    ct.process(out)
    st = np.zeros((ct.capacity, 1 + nf), np.uint32)
    st[:, 0] = pc.PD_ACTIVE
    st[:, 1:] = rng.integers(1, 3, (ct.capacity, nf))
    state = torch.from_numpy(st.view(np.int32)).to(dev).reshape(-1)
    for n in (1, 63, 65, 511, 513, 1025):
        frames = _pd_frames(rng, pool, n, 0.0)
        slab, dlen = pc.pack_frames(frames, 128)
        d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
        out = ctx.alloc_outputs(n, conn=True)
        ctx.run(torch.from_numpy(slab).to(dev), 128, d_dlen, n, out)
        ent = ct.process(out)
        counts, bm = pc.pd_run(ctx, out, ent, d_dlen, state)
        torch.cuda.synchronize()
        bits = np.unpackbits(bm.cpu().numpy()[:((n + 63) // 64) * 8], bitorder="little")
        assert not bits[n:].any(), n   # no bits past the batch
        got_idx, got_cnt = pc.decode_pd(counts, bm, out, len(pd["stmts"]))
        got = dict(zip(got_idx.tolist(), got_cnt))
        fwd = np.nonzero(out.decode()["fwd"])[0]
        e = pc.decode_ct(ent, out)
        for j, i in enumerate(fwd):
            slot, status = int(e[j, 0]), int(e[j, 1])
            exp = []
            if status == pc.CT_HIT | pc.CT_PRIOR:
                exp = df.evaluate(frames[i], len(frames[i]), st[slot, 1:])
            assert (i in got) == bool(exp), (n, i)
            if exp:
                assert pc.pd_replay(pd, got[i], st[slot, 1:]) == exp, (n, i)
    # a program without packet-level subscriptions delivers nothing (the bitmap is cleared)
    p2 = pc.PacketContinue(pc.Program.from_spec(SETS["cfg2"]), 0)
    assert p2.program.info["n_pd_stmts"] == 0
    out2 = p2.alloc_outputs(700, conn=True)
    frames = _pd_frames(rng, pool, 700, 0.0)
    slab, dlen = pc.pack_frames(frames, 128)
    d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
    p2.run(torch.from_numpy(slab).to(dev), 128, d_dlen, 700, out2)
    ent2 = pc.ConnTable(0, 10).process(out2)
    bm0 = torch.full((pc.lib().rtn_out_bitmap_bytes(700),), 0xFF, dtype=torch.uint8, device=dev)
    _, bm2 = pc.pd_run(p2, out2, ent2, d_dlen, torch.zeros(1024, dtype=torch.int32, device=dev), bitmap=bm0)
    torch.cuda.synchronize()
    assert not bm2.cpu().numpy().any()
