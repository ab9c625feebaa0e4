"""Offline ingest (include/retina_ingest.h) against the oracle's pcap reader: the same frames, in
the same order, with the reference's offline-runtime rules (core/src/runtime/offline.rs:64-82:
skip frames whose original length exceeds the mtu; mbuf data = the captured bytes). Captures are
written here in every on-disk variant (libpcap LE/BE, us/ns, pcapng LE/BE sections with EPB,
SPB and unknown blocks); the reference's own traces/ are checked when the tree is mounted."""
from __future__ import annotations

import struct

import numpy as np
import pytest

from oracle import pcap as opcap
from retina_amd import pc

RNG = np.random.default_rng(7)


def _frames(k=200):
    out = []
    for j in range(k):
        orig = int(RNG.choice([14, 60, 64, 65, 127, 128, 129, 600, 1514, 9000, 9702, 9703, 12000]))
        cap = min(orig, int(RNG.choice([orig, 96, 64, 200])))
        out.append((RNG.integers(0, 256, cap, dtype=np.uint8).tobytes(), orig))
    return out


def _write_pcap(path, frames, big=False, ns=False):
    e = ">" if big else "<"
    magic = 0xA1B23C4D if ns else 0xA1B2C3D4
    b = bytearray(struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, 65535, 1))
    for t, (data, orig) in enumerate(frames):
        b += struct.pack(e + "IIII", t, 0, len(data), orig) + data
    path.write_bytes(bytes(b))


def _pad4(b):
    return b + b"\0" * (-len(b) % 4)


def _write_pcapng(path, frames, big=False):
    e = ">" if big else "<"

    def block(t, body):
        body = _pad4(body)
        n = 12 + len(body)
        return struct.pack(e + "II", t, n) + body + struct.pack(e + "I", n)

    b = block(0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    b += block(1, struct.pack(e + "HHI", 1, 0, 65535))
    b += block(0xBAD, b"\x01\x02\x03\x04")  # unknown block: skipped
    for t, (data, orig) in enumerate(frames):
        if t % 5 == 4 and len(data) == orig:  # simple packet block (no caplen field)
            b += block(3, struct.pack(e + "I", orig) + data)
        else:
            b += block(6, struct.pack(e + "IIIII", 0, 0, t, len(data), orig) + data)
    path.write_bytes(b)


def _check_against_oracle(path, mtu, stride):
    want = opcap.offline_frames(path, mtu=mtu)
    r = pc.PcapReader(path, mtu=mtu)
    slab, dlen = r.read_all(stride=stride, batch=37)  # ragged batches
    assert len(dlen) == len(want)
    for i, f in enumerate(want):
        assert dlen[i] == len(f)
        k = min(len(f), stride)
        assert slab[i * stride:i * stride + k].tobytes() == f[:k], i
    st = r.stats()
    assert st["packed"] == len(want) and st["bytes"] == sum(map(len, want))
    assert st["frames"] == len(opcap.read(path)) and st["skipped_mtu"] == st["frames"] - st["packed"]
    r.rewind()
    s2, d2 = r.read_all(stride=stride)
    assert np.array_equal(d2, dlen) and np.array_equal(s2, slab)


@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("ns", [False, True])
def test_pcap_variants(tmp_path, big, ns):
    p = tmp_path / "a.pcap"
    _write_pcap(p, _frames(), big=big, ns=ns)
    for mtu, stride in ((9702, 128), (1500, 64), (100000, 256)):
        _check_against_oracle(p, mtu, stride)


@pytest.mark.parametrize("big", [False, True])
def test_pcapng_variants(tmp_path, big):
    p = tmp_path / "a.pcapng"
    _write_pcapng(p, _frames(), big=big)
    _check_against_oracle(p, 9702, 128)


def test_errors(tmp_path):
    with pytest.raises(pc.RetinaError) as e:
        pc.PcapReader(tmp_path / "missing.pcap")
    assert e.value.code == -22
    bad = tmp_path / "bad.pcap"
    bad.write_bytes(b"\x00" * 64)
    with pytest.raises(pc.RetinaError):
        pc.PcapReader(bad)
    big = tmp_path / "big.pcap"
    _write_pcap(big, [(b"\x01" * 70000, 70000)])
    r = pc.PcapReader(big, mtu=100000)
    with pytest.raises(pc.RetinaError) as e:
        r.read_all()
    assert e.value.code == -34


def test_empty_capture(tmp_path):
    p = tmp_path / "empty.pcap"
    _write_pcap(p, [])
    slab, dlen = pc.PcapReader(p).read_all()
    assert len(dlen) == 0


def test_reference_traces(reference_dir):
    traces = sorted((reference_dir / "traces").glob("*.pcap*"))
    assert traces
    for t in traces:
        if t.stat().st_size < 64:
            continue
        _check_against_oracle(t, 9702, 128)


@pytest.mark.parametrize("ext_cap", [None, 7])
def test_split_batches_match_the_slot_layout(tmp_path, ext_cap):
    """rtn_pcap_next_batch_split packs the compact split layout (retina_pc.h
    RTN_BATCH_EXT_COMPACT): the same frames as rtn_pcap_next_batch, their head slots, ext rows
    exactly for the frames rtn_ext_needed names, in order, and per-chunk first rows; with few
    rows (ext_cap) a batch ends early at a frame and the next one resumes there."""
    import corpus as C

    frames = [(f, len(f)) for f in C.base_frames() * 30 + C.adversarial()[:400]]
    frames += [(f + bytes(600), len(f) + 600) for f in C.base_frames()]  # long frames: ext rows
    p = tmp_path / "c.pcap"
    _write_pcap(p, frames)
    slab, dlen = pc.PcapReader(p).read_all(stride=128)
    need = pc.ext_needed(slab.reshape(-1, 128), dlen)
    assert need.any()
    r = pc.PcapReader(p)
    cap = 600
    got_head, got_dl, got_ext, got_need = [], [], [], []
    while True:
        head = np.zeros(cap * 64, np.uint8)
        ext = np.zeros((ext_cap or cap) * 64, np.uint8)
        ch = np.zeros((cap + pc.CHUNK_FRAMES - 1) // pc.CHUNK_FRAMES, np.uint32)
        d = np.zeros(cap, np.uint16)
        k, rows = r.next_batch_split(head, ext, ch, d)
        if k == 0:
            break
        hb = head[:k * 64].reshape(k, 64)
        nd = pc.ext_needed(np.pad(hb, ((0, 0), (0, 64))), d[:k])
        assert rows == nd.sum() and (ext_cap is None or rows <= ext_cap)
        for c in range(len(ch)):
            if c * pc.CHUNK_FRAMES < k:
                assert ch[c] == nd[:c * pc.CHUNK_FRAMES].sum()
        got_head.append(hb)
        got_dl.append(d[:k])
        got_ext.append(ext[:rows * 64].reshape(rows, 64))
        got_need.append(nd)
    assert np.array_equal(np.concatenate(got_dl), dlen)
    assert np.array_equal(np.concatenate(got_need), need)
    full = slab.reshape(-1, 128)
    heads = np.concatenate(got_head)
    for i in range(len(dlen)):
        k = min(int(dlen[i]), 64)
        assert heads[i, :k].tobytes() == full[i, :k].tobytes()
    exts = np.concatenate(got_ext)
    for j, i in enumerate(np.nonzero(need)[0]):
        k = min(int(dlen[i]), 128) - 64
        assert exts[j, :k].tobytes() == full[i, 64:64 + k].tobytes()


def test_split_batch_without_rows_is_not_eof(tmp_path):
    """A compact split batch that cannot take its first frame (no ext row free) fails with
    RTN_ERANGE instead of returning an empty batch, which callers read as end of file."""
    import corpus as C

    long = [(f + bytes(600), len(f) + 600) for f in C.base_frames()]
    s0, d0 = pc.pack_frames([f for f, _ in long], 128)
    nd = pc.ext_needed(s0.reshape(-1, 128), d0)
    long = [fr for fr, k in zip(long, nd) if k]  # frames that need an ext row
    assert len(long) > 2
    p = tmp_path / "d.pcap"
    _write_pcap(p, long)
    slab, dlen = pc.PcapReader(p).read_all(stride=128)
    r = pc.PcapReader(p)
    cap = 16
    head, ext = np.zeros(cap * 64, np.uint8), np.zeros(64, np.uint8)
    ch, d = np.zeros(1, np.uint32), np.zeros(cap, np.uint16)
    with pytest.raises(pc.RetinaError) as e:
        r.next_batch_split(head, ext[:0], ch, d)  # ext_cap 0
    assert e.value.code == -34
    k, rows = r.next_batch_split(head, ext, ch, d)  # one row: the same first frame, then stop
    assert k >= 1 and rows == 1 and d[0] == dlen[0]
