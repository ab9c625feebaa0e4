"""Shared test helpers: run the product (GPU, through the C ABI) and the oracle (CPU) on the same
frames and bring both to one canonical per-frame form."""
from __future__ import annotations

import numpy as np

from oracle import cgen, filterlang

# canonical per-forwarded-frame record
REC = np.dtype([("idx", "<u8"), ("ver", "<u4"), ("proto", "<u4"), ("sport", "<u4"), ("dport", "<u4"),
                ("offset", "<u4"), ("length", "<u4"), ("seq", "<u4"), ("ack", "<u4"), ("flags", "<u4"),
                ("src", "u1", 16), ("dst", "u1", 16)])


def subs_from_spec(spec: str) -> list[filterlang.Sub]:
    return filterlang.load_spec(spec)


_ORACLES: dict[str, cgen.OracleLib] = {}


def oracle_lib(spec: str) -> cgen.OracleLib:
    if spec not in _ORACLES:
        _ORACLES[spec] = cgen.OracleLib(filterlang.PacketTree(subs_from_spec(spec)))
    return _ORACLES[spec]


def oracle_run(spec: str, slab: np.ndarray, stride: int, dlen: np.ndarray) -> dict:
    lib = oracle_lib(spec)
    r = lib.eval(slab, stride, dlen)
    idx = np.nonzero(r["fwd"])[0]
    src = r["l4"][idx]
    rec = np.zeros(len(idx), REC)
    rec["idx"] = idx
    for f in ("ver", "proto", "sport", "dport", "offset", "length", "seq", "ack", "flags"):
        rec[f] = src[f]
    rec["src"] = src["src"]
    rec["dst"] = src["dst"]
    return {"pc": r["pc"], "fwd": r["fwd"], "rec": rec, "dm": r["dm"]}


def gpu_run(spec: str, slab: np.ndarray, stride: int, dlen: np.ndarray, device: int = 0, split: bool = False,
            conn: bool = False) -> dict:
    """Run the product on the GPU. split=True hands the frames over in the split layout
    (64-B head slots + 64-B ext slots, include/retina_pc.h) instead of `stride`-byte slots,
    split="compact" in the compact split layout (ext rows only where rtn_ext_needed);
    conn=True also computes the connection stage (rtn_conn_t per forwarded frame)."""
    import torch

    from retina_amd import pc

    prog = pc.Program.from_spec(spec)
    ctx = pc.PacketContinue(prog, device)
    dev = torch.device("cuda", device)
    n = len(dlen)
    ext_t = chunk_t = None
    if split == "compact":
        head, ext, chunk = pc.split_slab(np.ascontiguousarray(slab, np.uint8), stride, np.asarray(dlen), compact=True)
        slab, stride = head, 64
        ext_t, chunk_t = torch.from_numpy(ext).to(dev), torch.from_numpy(chunk.view(np.int32)).to(dev)
    elif split:
        head, ext = pc.split_slab(np.ascontiguousarray(slab, np.uint8), stride)
        slab, stride = head, 64
        ext_t = torch.from_numpy(ext).to(dev)
    slab_t = torch.from_numpy(np.ascontiguousarray(slab, np.uint8)).to(dev)
    dl_t = torch.from_numpy(np.ascontiguousarray(dlen, np.uint16).view(np.int16)).to(dev)
    out = ctx.run(slab_t, stride, dl_t, n, out=ctx.alloc_outputs(max(n, 1), conn=conn), ext=ext_t, ext_chunk=chunk_t)
    torch.cuda.synchronize()
    res = canonical(prog, out, dlen, conn=conn)
    assert res["counters"][3] == 0 or stride == 64, res["counters"]
    return res


def canonical(prog, out, dlen: np.ndarray, conn: bool = False) -> dict:
    """A finished run's outputs (pc.PCOutputs with counters) in the canonical per-frame form of
    oracle_run, after checking the byte / protocol counters of the same launch."""
    n = len(dlen)
    d = out.decode()
    cnt = out.counters_host()
    # TOTAL_BYTE / IGNORED_BY_PACKET_FILTER_BYTE (rx_core.rs:129-141) from the same launch
    total, ignored = out.byte_counters_host()
    dl64 = np.asarray(dlen, np.uint16).astype(np.uint64)
    assert total == int(dl64.sum()), (total, int(dl64.sum()))
    assert ignored == int(dl64[~d["pc"][:n]].sum()) if n else ignored == 0
    l4 = d["l4"]
    # TCP_PKT/BYTE, UDP_PKT/BYTE of process_packet (subscription/mod.rs:102-111), same launch
    st = out.stats_host()
    fidx = l4["pkt_idx"].astype(np.int64)
    tcp = l4["proto"] == 6
    assert (st["TCP_PKT"], st["UDP_PKT"]) == (int(tcp.sum()), int((~tcp).sum())), st
    assert (st["TCP_BYTE"], st["UDP_BYTE"]) == (int(dl64[fidx[tcp]].sum()), int(dl64[fidx[~tcp]].sum())), st
    rec = np.zeros(len(l4), REC)
    for f in ("ver", "proto", "flags", "sport", "dport", "offset", "length"):
        rec[f] = l4[f]
    rec["idx"] = l4["pkt_idx"]
    rec["seq"] = l4["seq_no"]
    rec["ack"] = l4["ack_no"]
    v4 = rec["ver"] == 4
    rec["src"][v4, :4] = l4["src_ip4"][v4].astype(">u4").view(np.uint8).reshape(-1, 4)
    rec["dst"][v4, :4] = l4["dst_ip4"][v4].astype(">u4").view(np.uint8).reshape(-1, 4)
    a6 = d["addr6"]
    rec["src"][~v4] = a6[~v4, :16]
    rec["dst"][~v4] = a6[~v4, 16:]
    nd = prog.info["deliver_words"]
    dm = np.zeros((n, nd), np.uint64)
    if nd:
        dl = d["dlv"]
        dm[dl[:, 0].astype(np.int64)] = dl[:, 1:]
    res = {"pc": d["pc"], "fwd": d["fwd"], "rec": rec, "dm": dm, "counters": cnt, "program": prog}
    if conn:
        res["conn"] = np.stack([d["conn_hash"], d["conn_info"]], 1) if len(l4) else np.zeros((0, 2), np.uint32)
        cw = prog.info["conn_words"]
        res["cdm"] = d["conn_dlv"] if cw else np.zeros((len(l4), 1), np.uint64)
    return res


def oracle_conn(spec: str, slab: np.ndarray, stride: int, dlen: np.ndarray, fwd: np.ndarray):
    """Connection stage of the forwarded frames from oracle/conn.py, in frame order."""
    from oracle import conn as oconn
    from retina_amd import pc

    subs = subs_from_spec(spec)
    pf = oconn.PacketFilter(filterlang.ConnTree(subs).to_json(), subs)
    words = max(1, (len(pf.stmts) + 63) // 64)
    b = np.ascontiguousarray(slab, np.uint8).reshape(-1, stride)
    idx = np.nonzero(fwd)[0]
    hi = np.zeros((len(idx), 2), np.uint32)
    cdm = np.zeros((len(idx), words), np.uint64)
    for j, i in enumerate(idx):
        h, info, fired = oconn.stage(pf, b[i].tobytes(), int(dlen[i]))
        hi[j] = h, info
        for k in fired:
            cdm[j, k // 64] |= np.uint64(1 << (k % 64))
    return hi, cdm


def assert_same(gpu: dict, ora: dict, what: str = "") -> None:
    n = len(ora["pc"])
    bad = np.nonzero(gpu["pc"] != ora["pc"])[0]
    assert bad.size == 0, f"{what}: PacketContinue differs at {bad[:10]} ({bad.size} of {n})"
    bad = np.nonzero(gpu["fwd"] != ora["fwd"])[0]
    assert bad.size == 0, f"{what}: forwarded set differs at {bad[:10]} ({bad.size} of {n})"
    g, o = gpu["rec"], ora["rec"]
    assert len(g) == len(o), f"{what}: {len(g)} vs {len(o)} L4Context records"
    for f in REC.names:
        if not np.array_equal(g[f], o[f]):
            k = np.nonzero((g[f] != o[f]).reshape(len(g), -1).any(1))[0][:5]
            raise AssertionError(f"{what}: L4Context field {f} differs at records {k}: {g[k]} vs {o[k]}")
    assert np.array_equal(gpu["dm"], ora["dm"]), f"{what}: packet-level deliveries differ"
    if "counters" in gpu:
        c = gpu["counters"]
        assert c[0] == ora["pc"].sum() and c[1] == ora["fwd"].sum(), f"{what}: counters {c}"
        assert c[2] == int((ora["dm"] != 0).any(1).sum()) if ora["dm"].size else c[2] == 0


def build_frame(v6=False, src=0x0A000001, dst=0x0A000002, sport=1234, dport=80, proto=6, flags=0x02,
                payload=b"") -> bytes:
    """One Eth/IPv4|IPv6/TCP|UDP frame with the given 5-tuple and TCP flags."""
    import struct

    if proto == 6:
        l4 = struct.pack(">HHIIBBHHH", sport, dport, 1, 2, 0x50, flags, 1024, 0, 0) + payload
    else:
        l4 = struct.pack(">HHHH", sport, dport, 8 + len(payload), 0) + payload
    if v6:
        ip = struct.pack(">IHBB", 0x60000000, len(l4), proto, 64) + src.to_bytes(16, "big") + dst.to_bytes(16, "big")
        et = 0x86DD
    else:
        ip = struct.pack(">BBHHHBBHII", 0x45, 0, 20 + len(l4), 0, 0, 64, proto, 0, src, dst)
        et = 0x0800
    return bytes(6) + bytes(5) + b"\x01" + struct.pack(">H", et) + ip + l4


def flow_pool(rng: np.random.Generator, nflows: int) -> list[tuple]:
    """Distinct connections: (v6, ip_a, ip_b, port_a, port_b, proto)."""
    pool, seen = [], set()
    while len(pool) < nflows:
        v6 = bool(rng.random() < 0.3)
        bits = 128 if v6 else 32
        a = int(rng.integers(0, 1 << 62)) << (bits - 62) if v6 else int(rng.integers(0, 1 << 32))
        b = int(rng.integers(0, 1 << 62)) << (bits - 62) if v6 else int(rng.integers(0, 1 << 32))
        pa, pb = int(rng.integers(1, 65536)), int(rng.integers(1, 65536))
        if rng.random() < 0.05:        # equal addresses: the port decides the orientation
            b = a
        proto = 6 if rng.random() < 0.7 else 17
        k = (v6, a, b, pa, pb, proto)
        if k not in seen:
            seen.add(k)
            pool.append(k)
    return pool


def flow_frames(rng: np.random.Generator, pool: list[tuple], n: int, p_syn: float = 0.3) -> list[bytes]:
    """n frames drawn from the flows of `pool`, random direction, TCP flags SYN-only with p_syn,
    otherwise a random mix (ACK, SYN|ACK, RST, FIN|ACK, PSH|ACK)."""
    frames = []
    other = [0x10, 0x12, 0x04, 0x11, 0x18, 0x06]
    for _ in range(n):
        v6, a, b, pa, pb, proto = pool[int(rng.integers(0, len(pool)))]
        if rng.random() < 0.5:
            a, b, pa, pb = b, a, pb, pa
        fl = 0x02 if rng.random() < p_syn else other[int(rng.integers(0, len(other)))]
        frames.append(build_frame(v6, a, b, pa, pb, proto, fl))
    return frames
