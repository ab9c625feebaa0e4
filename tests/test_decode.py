"""Host decoder of rtn_pc_run's outputs (retina_amd/pc.py PCOutputs.decode) against the record
layout include/retina_pc.h documents, on CPU: the outputs of a batch are written here by a
straightforward per-frame encoder that follows the header's comments (RTN_REC_INDEX blocks for
l4 and seqack, chunk-dense addr6), then decoded. No GPU, no kernel: this pins the layout the
kernels (checked against the oracle in the GPU suite) and the host consumers agree on."""
import numpy as np
import torch

from retina_amd import pc

CF, RB = 256, 64  # RTN_CHUNK_FRAMES, RTN_REC_BLOCK


def rec_index(n: int, c: int, k: int) -> int:
    """RTN_REC_INDEX(n, chunk, k), as the macro in retina_pc.h writes it."""
    nch = (n + CF - 1) // CF
    return ((k // RB) * nch + c) * RB + k % RB


def encode(n: int, frames: list[dict]) -> pc.PCOutputs:
    """Outputs of a batch of n frames whose forwarded frames are `frames` (ascending 'i')."""
    nch = (n + CF - 1) // CF
    l4 = np.zeros((nch * CF, 4), np.uint32)
    seqack = np.zeros(nch * CF, np.uint64)
    addr6 = np.zeros((nch * CF, 24), np.uint8)
    fwd = np.zeros((n + 63) // 64, np.uint64)
    pcb = np.zeros_like(fwd)
    k = {}   # per chunk: records, TCP records, IPv6 records so far
    for f in frames:
        i, c = f["i"], f["i"] // CF
        kr, kt, k6 = k.get(c, (0, 0, 0))
        fwd[i // 64] |= np.uint64(1 << (i % 64))
        pcb[i // 64] |= np.uint64(1 << (i % 64))
        meta = ((f["offset"] >> 2) | (64 if f["udp"] else 0) | (128 if f["v6"] else 0) | (f["flags"] << 8)
                | (f["length"] << 16))
        if f["v6"]:
            w = np.frombuffer(f["src"][:8], "<u4")
            w0, w1 = int(w[0]), int(w[1])
            addr6[c * CF + k6] = np.frombuffer(f["src"][8:] + f["dst"], np.uint8)
            k6 += 1
        else:
            w0, w1 = f["src4"], f["dst4"]
        l4[rec_index(n, c, kr)] = [w0, w1, f["sport"] | f["dport"] << 16, meta]
        kr += 1
        if not f["udp"]:
            seqack[rec_index(n, c, kt)] = f["seq"] | f["ack"] << 32
            kt += 1
        k[c] = (kr, kt, k6)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1))  # noqa: E731
    return pc.PCOutputs(n=n, pc_bitmap=t(pcb), fwd_bitmap=t(fwd), l4=t(l4), addr6=t(addr6), dlv_bitmap=None,
                        dlv_records=None, counters=None, deliver_words=0, seqack=t(seqack))


def test_decode_matches_documented_layout():
    rng = np.random.default_rng(7)
    n = 1000  # four chunks, the last one partial
    # chunk 1 forwards more than one 64-record block, so RTN_REC_INDEX's interleave is exercised
    idx = sorted(set(rng.choice(n, 420, replace=False).tolist()) | set(range(256, 256 + 150)))
    frames = []
    for i in idx:
        v6, udp = bool(rng.random() < 0.4), bool(rng.random() < 0.4)
        frames.append({"i": i, "v6": v6, "udp": udp, "offset": 4 * int(rng.integers(3, 20)) + 2,
                       "flags": 0 if udp else int(rng.integers(0, 256)), "length": int(rng.integers(0, 65536)),
                       "sport": int(rng.integers(0, 65536)), "dport": int(rng.integers(0, 65536)),
                       "seq": 0 if udp else int(rng.integers(0, 1 << 32)), "ack": 0 if udp else int(rng.integers(0, 1 << 32)),
                       "src4": int(rng.integers(0, 1 << 32)), "dst4": int(rng.integers(0, 1 << 32)),
                       "src": rng.bytes(16), "dst": rng.bytes(16)})
    d = encode(n, frames).decode()
    assert np.flatnonzero(d["fwd"]).tolist() == idx
    l4, a6 = d["l4"], d["addr6"]
    for j, f in enumerate(frames):
        r = l4[j]
        assert int(r["pkt_idx"]) == f["i"]
        assert int(r["ver"]) == (6 if f["v6"] else 4) and int(r["proto"]) == (17 if f["udp"] else 6)
        assert (int(r["sport"]), int(r["dport"])) == (f["sport"], f["dport"])
        assert (int(r["offset"]), int(r["length"]), int(r["flags"])) == (f["offset"], f["length"], f["flags"])
        assert (int(r["seq_no"]), int(r["ack_no"])) == (f["seq"], f["ack"])
        if f["v6"]:
            assert bytes(a6[j, :16]) == f["src"] and bytes(a6[j, 16:]) == f["dst"]
            assert int(r["src_ip4"]) == 0 and int(r["dst_ip4"]) == 0
        else:
            assert (int(r["src_ip4"]), int(r["dst_ip4"])) == (f["src4"], f["dst4"])
