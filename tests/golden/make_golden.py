"""Regenerate the committed golden fixtures (run here, where /root/reference is mounted):

    python tests/golden/make_golden.py

  traces.npz          frames of the reference's traces/*.pcap[ng] (data files the reference
                      ships), as offline.rs:67-75 hands them to the filter (orig len <= mtu 9702):
                      128-byte header slab per frame + data_len + trace id.
  golden_<set>.npz    expected outputs for every named subscription set (filter_sets.py) over
                      three corpora (traces, adversarial, synthetic cfg2/3/4 samples): the
                      PacketContinue bit, the forwarded bit, the L4Context of forwarded frames and
                      the packet-level callback statement masks; and the connection stage of every
                      forwarded frame (oracle/conn.py: ConnId hash and orientation, the creates
                      bit, the first-packet packet_filter actions and statement masks).
Expected outputs come from the C oracle and are cross-checked frame by frame against the
independent pure-Python oracle (oracle/packet.py) before being written.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(HERE))

from oracle import conn, filterlang, packet, pcap  # noqa: E402
from retina_amd import pc as rpc, synth  # noqa: E402

import corpus  # noqa: E402
import helpers  # noqa: E402
from filter_sets import SETS  # noqa: E402

STRIDE = 128
TRACES = ["tls_ciphers.pcap", "quic.pcap", "quic_retry.pcapng", "quic_xargs.pcap", "quic_kyber.pcapng"]


def make_traces(ref: Path) -> None:
    frames, ids = [], []
    for k, t in enumerate(TRACES):
        fr = pcap.offline_frames(ref / "traces" / t, mtu=9702)
        frames += fr
        ids += [k] * len(fr)
    slab, dlen = rpc.pack_frames(frames, STRIDE)
    np.savez_compressed(HERE / "traces.npz", slab=slab, dlen=dlen, trace=np.array(ids, np.uint8),
                        names=np.array(TRACES))


def corpora() -> dict:
    t = np.load(HERE / "traces.npz")
    adv = corpus.all_frames()
    s_adv, d_adv = rpc.pack_frames(adv, STRIDE)
    s2, d2 = synth.cfg2(2048, start=12345)
    s2 = np.pad(s2.reshape(-1, 64), ((0, 0), (0, 64))).reshape(-1)
    s3, d3 = synth.cfg3(2048, start=777)
    s4, d4 = synth.cfg4(2048, start=999)
    return {
        "traces": (t["slab"], t["dlen"]),
        "adversarial": (s_adv, d_adv),
        "synth": (np.concatenate([s2, s3, s4]), np.concatenate([d2, d3, d4])),
    }


def python_crosscheck(spec: str, slab: np.ndarray, dlen: np.ndarray, res: dict, limit: int) -> None:
    tree = filterlang.PacketTree(filterlang.load_spec(spec))
    b = slab.reshape(-1, STRIDE)
    n = min(len(dlen), limit)
    for i in range(n):
        dl = int(dlen[i])
        fr = b[i].tobytes()
        act, fired = packet.evaluate(tree, fr, dl)
        assert bool(act & 1) == bool(res["pc"][i]), (spec, i)
        dm = 0
        for k in fired:
            dm |= 1 << k
        got = 0
        for w in range(res["dm"].shape[1]):
            got |= int(res["dm"][i, w]) << (64 * w)
        assert dm == got, (spec, i, fired)
        ctx = packet.l4context(fr, dl) if act & 1 else None
        assert (ctx is not None) == bool(res["fwd"][i]), (spec, i)
        if ctx is not None:
            # every L4Context field, addresses included (pdu.rs:66-84)
            x = res["l4"][i]
            w = 4 if ctx.ver == 4 else 16
            assert (int(x["ver"]), int(x["proto"]), int(x["sport"]), int(x["dport"]), int(x["offset"]),
                    int(x["length"]), int(x["seq"]), int(x["ack"]), int(x["flags"]), bytes(x["src"]),
                    bytes(x["dst"])) == (ctx.ver, ctx.proto, ctx.sport, ctx.dport, ctx.offset, ctx.length, ctx.seq,
                                         ctx.ack, ctx.flags, ctx.src.to_bytes(w, "big") + bytes(16 - w),
                                         ctx.dst.to_bytes(w, "big") + bytes(16 - w)), (spec, i)


def conn_expected(spec: str, slab: np.ndarray, dlen: np.ndarray, fwd: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Connection stage of the forwarded frames, in frame order: (hash, info) and statement masks."""
    subs = filterlang.load_spec(spec)
    pf = conn.PacketFilter(filterlang.ConnTree(subs).to_json(), subs)
    words = max(1, (len(pf.stmts) + 63) // 64)
    b = slab.reshape(-1, STRIDE)
    idx = np.nonzero(fwd)[0]
    hi = np.zeros((len(idx), 2), np.uint32)
    cdm = np.zeros((len(idx), words), np.uint64)
    for j, i in enumerate(idx):
        r = conn.stage(pf, b[i].tobytes(), int(dlen[i]))
        assert r is not None, (spec, i)
        hi[j] = r[0], r[1]
        for k in r[2]:
            cdm[j, k // 64] |= np.uint64(1 << (k % 64))
    return hi, cdm


def main() -> None:
    ref = Path("/root/reference")
    if ref.exists():
        make_traces(ref)
    cs = corpora()
    for name, spec in SETS.items():
        out = {}
        for cname, (slab, dlen) in cs.items():
            r = helpers.oracle_run(spec, slab, STRIDE, dlen)
            raw = helpers.oracle_lib(spec).eval(slab, STRIDE, dlen)
            python_crosscheck(spec, slab, dlen, raw, 100000 if cname != "synth" else 1500)
            out[f"{cname}_pc"] = np.packbits(r["pc"])
            out[f"{cname}_fwd"] = np.packbits(r["fwd"])
            out[f"{cname}_rec"] = r["rec"]
            out[f"{cname}_dm"] = r["dm"]
            out[f"{cname}_conn"], out[f"{cname}_cdm"] = conn_expected(spec, slab, dlen, r["fwd"])
        np.savez_compressed(HERE / f"golden_{name}.npz", **out)
        print(name, {k: int(np.unpackbits(v).sum()) for k, v in out.items() if k.endswith("_pc")})
    np.savez_compressed(HERE / "corpus_adversarial.npz", slab=cs["adversarial"][0], dlen=cs["adversarial"][1])


if __name__ == "__main__":
    main()
