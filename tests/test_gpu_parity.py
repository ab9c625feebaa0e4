"""Parity of the HIP path (through the C ABI) against the oracle: bit-exact accept set,
forwarded set, L4Context records and packet-level callback statement masks."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from retina_amd import pc, synth

GOLD = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


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


@pytest.mark.parametrize("layout", ["mono", "split", "compact"])
@pytest.mark.parametrize("corpus", ["traces", "adversarial", "synth"])
@pytest.mark.parametrize("fset", list(SETS))
def test_golden_fixture(fset, corpus, layout, gpu):
    g = np.load(GOLD / f"golden_{fset}.npz")
    slab, dlen = _corpus(corpus)
    n = len(dlen)
    exp = {"pc": np.unpackbits(g[f"{corpus}_pc"])[:n].astype(bool),
           "fwd": np.unpackbits(g[f"{corpus}_fwd"])[:n].astype(bool),
           "rec": g[f"{corpus}_rec"], "dm": g[f"{corpus}_dm"]}
    got = helpers.gpu_run(SETS[fset], slab, 128, dlen, split={"mono": False, "split": True, "compact": "compact"}[layout])
    helpers.assert_same(got, exp, f"{fset}/{corpus}/{layout}")


@pytest.mark.parametrize("cfg,stride,split", [("cfg2", 64, False), ("cfg3", 128, False), ("cfg4", 128, False),
                                              ("cfg3", 128, True), ("cfg4", 128, True),
                                              ("cfg3", 128, "compact"), ("cfg4", 128, "compact")])
def test_synthetic_vs_oracle(cfg, stride, split, gpu):
    n = (1 << 18) + 37  # ragged tail: not a multiple of 64
    gen = {"cfg2": synth.cfg2, "cfg3": synth.cfg3, "cfg4": synth.cfg4}[cfg]
    slab, dlen = gen(n, start=1 << 20)
    spec = SETS[cfg]
    helpers.assert_same(helpers.gpu_run(spec, slab, stride, dlen, split=split),
                        helpers.oracle_run(spec, slab, stride, dlen), f"{cfg}/split={split}")


@pytest.mark.parametrize("fset", ["quirks", "payload", "port_count", "match_all", "basic"])
def test_sets_on_imix(fset, gpu):
    slab, dlen = synth.cfg3((1 << 16) + 5, start=4242)
    spec = SETS[fset]
    helpers.assert_same(helpers.gpu_run(spec, slab, 128, dlen), helpers.oracle_run(spec, slab, 128, dlen), fset)


def test_wide_stride_and_empty(gpu):
    """stride 256 (larger slots than needed) gives the same answer; n = 0 is a no-op."""
    slab, dlen = synth.cfg3(4099, start=31)
    wide = np.zeros((len(dlen), 256), np.uint8)
    wide[:, :128] = slab.reshape(-1, 128)
    spec = SETS["cfg3"]
    a = helpers.gpu_run(spec, wide.reshape(-1), 256, dlen)
    helpers.assert_same(a, helpers.oracle_run(spec, slab, 128, dlen), "stride256")
    import torch

    from retina_amd import pc

    ctx = pc.PacketContinue(pc.Program.from_spec(spec), 0)
    t = torch.zeros(64, dtype=torch.uint8, device="cuda")
    out = ctx.run(t, 128, torch.zeros(1, dtype=torch.int16, device="cuda"), 0)
    assert out.n == 0


def test_narrow_stride_flags_status(gpu):
    """stride 64 with frames whose headers reach past byte 64 raises status bit 0."""
    slab, dlen = synth.cfg3(4096, start=99)
    narrow = slab.reshape(-1, 128)[:, :64].copy().reshape(-1)
    got = helpers.gpu_run(SETS["cfg3"], narrow, 64, dlen)
    assert got["counters"][3] & 1


def test_slot_contract_is_never_silent(gpu):
    """64-byte slots without ext (include/retina_pc.h): refused unless the caller asserts
    RTN_BATCH_DL_LE64 or passes counters; an IPv6 frame with data_len > 64 is reported through
    counters (RTN_STATUS_HDR_PAST_SLOT) or, without counters, through the context's sticky status
    word (RTN_STATUS_DL_PAST_SLOT when the assertion was false); batches past RTN_MAX_FRAMES are
    refused."""
    import torch

    ctx = pc.PacketContinue(pc.Program.from_spec(SETS["cfg2"]), 0)
    frames = [helpers.build_frame(dport=80)] * 63 + [helpers.build_frame(True, 1, 2, payload=bytes(40))]
    slab, dlen = pc.pack_frames(frames, 64)
    assert dlen[-1] > 64 and dlen[:-1].max() <= 64
    d_slab, d_dlen = torch.from_numpy(slab).cuda(), torch.from_numpy(dlen.view(np.int16)).cuda()
    bare = ctx.alloc_outputs(64, counters=False)
    with pytest.raises(pc.RetinaError) as e:
        ctx.run(d_slab, 64, d_dlen, 64, bare)
    assert e.value.code == -22 and "RTN_BATCH_DL_LE64" in str(e.value)
    assert ctx.take_status() == 0
    ctx.run(d_slab, 64, d_dlen, 64, bare, dl_le64=True)          # a false assertion is reported (and
    assert ctx.take_status() == pc.STATUS_DL_PAST_SLOT | pc.STATUS_HDR_PAST_SLOT  # the IPv6 headers pass 64)
    assert ctx.take_status() == 0
    ctx.run(d_slab, 64, d_dlen, 63, bare, dl_le64=True)          # a true one raises nothing
    assert ctx.take_status() == 0
    out = ctx.run(d_slab, 64, d_dlen, 64, ctx.alloc_outputs(64))  # counters: the caller sees it
    torch.cuda.synchronize()
    assert out.counters_host()[3] == pc.STATUS_HDR_PAST_SLOT
    import dataclasses

    huge = dataclasses.replace(bare, n=pc.MAX_FRAMES + 1)  # (refused before anything is touched)
    with pytest.raises(pc.RetinaError) as e:
        ctx.run(d_slab, 64, d_dlen, pc.MAX_FRAMES + 1, huge, dl_le64=True)
    assert e.value.code == -22
    assert ctx.take_status() == 0


def test_full_size_cfg2_properties(gpu):
    """BASELINE config 2 at full size (2^25 frames): size-independent properties — the accept set
    is exactly dport == 80, every accepted frame is forwarded with offset 54 / length 10, records
    are in frame order, and totals match; a sampled window is checked against the oracle."""
    import torch

    from retina_amd import pc

    n = 1 << 25
    slab, dlen = synth.cfg2(n)
    b = slab.reshape(n, 64)
    exp = ((b[:, 36].astype(np.uint32) << 8) | b[:, 37]) == 80
    prog = pc.Program.from_spec(SETS["cfg2"])
    ctx = pc.PacketContinue(prog, 0)
    dev = torch.device("cuda", 0)
    out = ctx.run(torch.from_numpy(slab).to(dev), 64, torch.from_numpy(dlen.view(np.int16)).to(dev), n)
    torch.cuda.synchronize()
    d = out.decode()
    assert np.array_equal(d["pc"], exp)
    assert np.array_equal(d["fwd"], exp)
    l4 = d["l4"]
    assert np.array_equal(l4["pkt_idx"], np.nonzero(exp)[0])
    assert np.all(l4["offset"] == 54) and np.all(l4["length"] == 10)
    assert np.all(l4["dport"] == 80) and np.all(l4["proto"] == 6) and np.all(l4["ver"] == 4)
    c = out.counters_host()
    assert c[0] == exp.sum() and c[1] == exp.sum() and c[3] == 0
    total, ignored = out.byte_counters_host()
    assert total == int(dlen.astype(np.uint64).sum()) and ignored == int(dlen[~exp].astype(np.uint64).sum())
    lo = 3 << 22
    win = slice(lo, lo + (1 << 16))
    ora = helpers.oracle_run(SETS["cfg2"], slab[lo * 64:(lo + (1 << 16)) * 64], 64, dlen[win])
    sel = (l4["pkt_idx"] >= lo) & (l4["pkt_idx"] < lo + (1 << 16))
    assert np.array_equal(l4["pkt_idx"][sel] - lo, ora["rec"]["idx"])
    assert np.array_equal(l4["seq_no"][sel], ora["rec"]["seq"])


@pytest.mark.parametrize("layout", ["compact", "split"])
@pytest.mark.parametrize("cfg,n", [("cfg3", 1 << 24), ("cfg4", 1 << 23)])
def test_full_size_split_properties(cfg, n, layout, gpu):
    """BASELINE configs 3 and 4 at full size in the compact split layout bench.py times (and in
    the plain split layout): the counters
    equal the bitmaps' popcounts, the forwarded set is inside the accepted set, every record is a
    well-formed L4Context (protocol, version, offset, UDP fields), the TCP/UDP byte counters equal
    the data_len sums of the decoded records, and two 64K-frame windows (the start of the second
    quarter and the last frames) equal the oracle exactly."""
    import torch

    import bench

    slab, dlen = bench.gen_frames(cfg, n, 0)
    spec = SETS[cfg]
    ctx = pc.PacketContinue(pc.Program.from_spec(spec), 0)
    dev = torch.device("cuda", 0)
    chunk_t = None
    if layout == "compact":  # bench.py's layout (RTN_BATCH_EXT_COMPACT)
        head, ext, chunk = pc.split_slab(slab, 128, dlen, compact=True)
        chunk_t = torch.from_numpy(chunk.view(np.int32)).to(dev)
    else:
        head, ext = pc.split_slab(slab, 128)
    out = ctx.run(torch.from_numpy(head).to(dev), 64, torch.from_numpy(dlen.view(np.int16)).to(dev), n,
                  ext=torch.from_numpy(ext).to(dev), ext_chunk=chunk_t)
    del head, ext
    torch.cuda.synchronize()
    d = out.decode()
    c = out.counters_host()
    assert c[3] == 0
    assert c[0] == d["pc"].sum() and c[1] == d["fwd"].sum() and not (d["fwd"] & ~d["pc"]).any()
    dlv_frames = np.zeros(n, bool)
    dlv_frames[d["dlv"][:, 0].astype(np.int64)] = True
    assert c[2] == dlv_frames.sum() and (d["dlv"][:, 1:] != 0).any(1).all()
    l4 = d["l4"]
    v6 = l4["ver"] == 6
    tcp = l4["proto"] == 6
    assert set(np.unique(l4["proto"])) <= {6, 17} and set(np.unique(l4["ver"])) <= {4, 6}
    # IHL and doff are not sanity-checked (ipv4.rs:215-217, tcp.rs:222-224): 14 + 0 + 0 .. 22 + 60 + 60
    assert (l4["offset"] % 4 == 2).all() and (l4["offset"] >= 14).all() and (l4["offset"] <= 22 + 60 + 60).all()
    assert (l4["seq_no"][~tcp] == 0).all() and (l4["ack_no"][~tcp] == 0).all() and (l4["flags"][~tcp] == 0).all()
    assert (d["addr6"][v6] != 0).any(1).all() and (l4["src_ip4"][v6] == 0).all()
    st = out.stats_host()
    dl = dlen.astype(np.int64)
    fi = l4["pkt_idx"].astype(np.int64)
    assert st["TCP_PKT"] == tcp.sum() and st["TCP_BYTE"] == dl[fi[tcp]].sum() and st["UDP_BYTE"] == dl[fi[~tcp]].sum()
    assert st["TOTAL_BYTE"] == dl.sum() and st["IGNORED_BY_PACKET_FILTER_BYTE"] == dl[~d["pc"]].sum()
    for lo in (n // 4, n - (1 << 16)):
        w = slice(lo, lo + (1 << 16))
        ora = helpers.oracle_run(spec, slab[lo * 128:(lo + (1 << 16)) * 128], 128, dlen[w])
        assert np.array_equal(d["pc"][w], ora["pc"]) and np.array_equal(d["fwd"][w], ora["fwd"])
        sel = (fi >= lo) & (fi < lo + (1 << 16))
        got = l4[sel]
        rec = ora["rec"]
        assert np.array_equal(got["pkt_idx"] - lo, rec["idx"])
        for gf, of in (("sport", "sport"), ("dport", "dport"), ("offset", "offset"), ("length", "length"),
                       ("seq_no", "seq"), ("ack_no", "ack"), ("flags", "flags"), ("proto", "proto"), ("ver", "ver")):
            assert np.array_equal(got[gf], rec[of]), (cfg, lo, gf)
        gv4 = got["ver"] == 4
        assert np.array_equal(got["src_ip4"][gv4].astype(">u4").view(np.uint8).reshape(-1, 4), rec["src"][gv4, :4])
        assert np.array_equal(d["addr6"][sel][~gv4, :16], rec["src"][~gv4])
        assert np.array_equal(d["addr6"][sel][~gv4, 16:], rec["dst"][~gv4])
        dm = np.zeros((n, max(1, d["dlv"].shape[1] - 1)), np.uint64)
        dm[d["dlv"][:, 0].astype(np.int64)] = d["dlv"][:, 1:]
        assert np.array_equal(dm[w][:, :ora["dm"].shape[1]], ora["dm"])


def test_large_tree_uses_nested_form_and_matches(gpu):
    """Trees past the straight-line threshold are emitted as nested if/else (codegen.cpp
    kFlatMaxNodes): 300 packet-level port subscriptions (a 600-node tree) plus packet-level
    callbacks, on IMIX frames whose ports hit them."""
    subs = [(f"tcp.dst_port = {1000 + k} or udp.src_port = {2000 + k}", ["ConnRecord"], f"c{k}") for k in range(300)]
    subs += [("tcp.port = 1007", ["ZcFrame"], "z"), ("udp.port >= 2290", ["Payload"], "p")]
    spec = synth._toml(subs)
    prog = pc.Program.from_spec(spec)
    assert prog.info["tree_size"] > 256
    body = prog.source.split("void rtn_filter(")[1][:300]
    assert "if (" in body and "const bool k" not in body
    rng = np.random.default_rng(21)
    frames = []
    for j in range(6000):
        proto = 6 if rng.random() < 0.6 else 17
        port = int(rng.choice([1000 + int(rng.integers(0, 320)), 2000 + int(rng.integers(0, 320)), int(rng.integers(1, 65536))]))
        sp, dp = (int(rng.integers(1, 65536)), port) if rng.random() < 0.5 else (port, int(rng.integers(1, 65536)))
        frames.append(helpers.build_frame(bool(rng.random() < 0.3), int(rng.integers(0, 1 << 32)),
                                          int(rng.integers(0, 1 << 32)), sp, dp, proto, 0x18,
                                          payload=bytes(int(rng.integers(0, 5)))))
    slab, dlen = pc.pack_frames(frames, 128)
    helpers.assert_same(helpers.gpu_run(spec, slab, 128, dlen), helpers.oracle_run(spec, slab, 128, dlen), "large tree")


def test_misaligned_record_array_is_einval(gpu):
    """l4 / addr6 / conn / seqack take 16-B-per-lane stores: a misaligned array is refused
    (RTN_EINVAL) before anything is launched, and the same context still runs on aligned outputs."""
    import dataclasses

    import torch

    slab, dlen = synth.cfg2(1024, start=5)
    ctx = pc.PacketContinue(pc.Program.from_spec(SETS["cfg2"]), 0)
    d_slab = torch.from_numpy(slab).cuda()
    d_dlen = torch.from_numpy(dlen.view(np.int16)).cuda()
    out = ctx.alloc_outputs(len(dlen), conn=True)
    for field in ("l4", "addr6", "conn", "seqack"):
        t = getattr(out, field)
        bad = dataclasses.replace(out, **{field: torch.empty(t.numel() + 16, dtype=torch.uint8, device="cuda")[8:]})
        with pytest.raises(pc.RetinaError) as e:
            ctx.run(d_slab, 64, d_dlen, len(dlen), bad)
        assert e.value.code == -22 and "16-byte aligned" in str(e.value)
    ctx.run(d_slab, 64, d_dlen, len(dlen), out)
    torch.cuda.synchronize()
    assert int(out.counters.view(torch.int32)[1]) > 0


@pytest.mark.gpu
def test_outputs_in_mapped_host_memory(gpu):
    """rtn_pc_run takes plain pointers: records and IPv6 addresses written straight into pinned
    host memory (pc.MappedHost, the end-to-end path's zero-copy outputs) equal a run into HBM."""
    import dataclasses

    import torch

    n = (1 << 16) + 77
    slab, dlen = synth.cfg3(n, start=4242)
    dev = torch.device("cuda", 0)
    ctx = pc.PacketContinue(pc.Program.from_spec(SETS["cfg3"]), 0)
    d_slab = torch.from_numpy(slab).to(dev)
    d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
    ref = ctx.run(d_slab, 128, d_dlen, n, ctx.alloc_outputs(n, addr6=True))
    dev_out = ctx.alloc_outputs(n, addr6=True)
    mapped = dataclasses.replace(
        dev_out, l4=pc.MappedHost(torch.zeros(dev_out.l4.numel(), dtype=torch.uint8).pin_memory()),
        addr6=pc.MappedHost(torch.zeros(dev_out.addr6.numel(), dtype=torch.uint8).pin_memory()))
    ctx.run(d_slab, 128, d_dlen, n, mapped)
    torch.cuda.synchronize()
    a, b = ref.decode(), mapped.decode()
    assert np.array_equal(a["fwd"], b["fwd"]) and np.array_equal(a["l4"], b["l4"])
    assert np.array_equal(a["addr6"], b["addr6"])
    assert int(b["fwd"].sum()) > n // 2


@pytest.mark.parametrize("layout", [False, True, "compact"])
def test_ipv6_dense_batches(layout, gpu):
    """Runs of groups where (almost) every frame is a forwarded IPv6 frame: the IPv6 address
    records of a chunk pass through the per-wave LDS ring faster than one block per group, so the
    ring must be drained before it wraps onto records not yet stored (pc_kernel.hip rtn_group)."""
    rng = np.random.default_rng(66)
    frames = []
    for j in range(9 * 256 + 77):
        v6 = (j // 256) % 3 != 2 or rng.random() < 0.5   # two all-IPv6 chunks, then a mixed one
        proto = 6 if rng.random() < 0.8 else 17
        src = int(rng.integers(0, 1 << 62)) << 66 | j if v6 else int(rng.integers(0, 1 << 32))
        dst = int(rng.integers(0, 1 << 62)) << 66 | (j * 7) if v6 else int(rng.integers(0, 1 << 32))
        frames.append(helpers.build_frame(v6, src, dst, int(rng.integers(1, 65536)), int(rng.integers(1, 65536)),
                                          proto, 0x18, payload=bytes(int(rng.integers(0, 9)))))
    slab, dlen = pc.pack_frames(frames, 128)
    spec = synth._toml([("tcp or udp", ["ConnRecord"], "all"), ("ipv6.src_addr = ::/0 and tcp", ["ZcFrame"], "z6")])
    helpers.assert_same(helpers.gpu_run(spec, slab, 128, dlen, split=layout),
                        helpers.oracle_run(spec, slab, 128, dlen), f"ipv6 dense/{layout}")
