"""The capture walk on the GPU (rtn_pcap_next_batch_gpu, include/retina_ingest.h) against the
oracle's pcap reader: the same frames in the same order under the offline runtime's rules
(core/src/runtime/offline.rs:64-82: frames whose original length exceeds the mtu are skipped,
mbuf data = the captured bytes), packed in the gather layout, with the host reader's stats and
error behaviour. Small windows (64 KiB) and small batches force many windows, segment seams and
batch cuts; captures of IMIX frames with zero-filled payloads and of the reference traces' frames
exercise the speculation of record boundaries. One batch also runs through rtn_pc_run against the
oracle."""
from __future__ import annotations

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from oracle import pcap as opcap
from retina_amd import pc
from test_ingest import _frames, _write_pcap, _write_pcapng
from test_stage import corpus


def _slab_frames(slab: np.ndarray, dlen: np.ndarray, stride: int) -> list[tuple[bytes, int]]:
    """Frames of a slot slab as (captured bytes, original length): the slot's bytes, zero-filled
    up to data_len (a slot holds the first `stride` bytes)."""
    out = []
    for i, d in enumerate(dlen.tolist()):
        b = slab[i * stride:i * stride + min(d, stride)].tobytes()
        out.append((b + bytes(d - len(b)), d))
    return out


class _Batches:
    """Device buffers of one batch size, in the gather layout."""

    def __init__(self, cap: int):
        import torch

        dev = torch.device("cuda", 0)
        self.cap = cap
        self.head = torch.zeros(cap * 64, dtype=torch.uint8, device=dev)
        self.ext = torch.zeros(pc.gather_ext_rows(cap) * 64, dtype=torch.uint8, device=dev)
        self.chunk = torch.zeros((cap + 255) // 256, dtype=torch.int32, device=dev)
        self.dl = torch.zeros(cap, dtype=torch.int16, device=dev)

    def frames(self, n: int) -> list[tuple[bytes, int, bool]]:
        """(first bytes the layout holds, data_len, has an ext row) of the batch's n frames."""
        h = self.head[:n * 64].cpu().numpy().reshape(n, 64)
        d = self.dl[:n].cpu().numpy().view(np.uint16)
        e = self.ext.cpu().numpy().reshape(-1, 64)
        ch = self.chunk[:(n + 255) // 256].cpu().numpy().view(np.uint32)
        assert np.array_equal(ch, np.arange(len(ch), dtype=np.uint32) * 256)
        need = pc.ext_needed(h, d)
        out, rank = [], 0
        for i in range(n):
            if i % 256 == 0:
                rank = 0
            k = min(int(d[i]), 64)
            b = h[i, :k].tobytes()
            if need[i]:
                b += e[(i // 256) * 256 + rank, :min(int(d[i]), 128) - 64].tobytes()
                rank += 1
            out.append((b, int(d[i]), bool(need[i])))
        return out


def _walk(path, mtu=9702, cap=1000, window=1 << 16, bufs=None):
    import torch

    r = pc.PcapReader(path, mtu=mtu)
    if window:
        r.gpu_window(window)
    b = bufs or _Batches(cap)
    got, sizes = [], []
    while True:
        n = r.next_batch_gpu(b.head, b.ext, b.chunk, b.dl)
        torch.cuda.synchronize()
        if n == 0:
            break
        assert n <= b.cap
        sizes.append(n)
        got += b.frames(n)
    return got, r.stats(), sizes


def _check(path, mtu=9702, cap=1000, window=1 << 16):
    want = opcap.offline_frames(path, mtu=mtu)
    got, st, sizes = _walk(path, mtu, cap, window)
    assert len(got) == len(want)
    for i, ((b, d, need), f) in enumerate(zip(got, want)):
        assert d == len(f), i
        assert b == f[:min(len(f), 128 if need else 64)], i
    host = pc.PcapReader(path, mtu=mtu)
    host.read_all(stride=64, batch=4096)
    assert st == host.stats()
    return sizes


@pytest.mark.gpu
@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("ns", [False, True])
def test_pcap_variants(tmp_path, gpu, big, ns):
    p = tmp_path / "a.pcap"
    _write_pcap(p, _frames(600), big=big, ns=ns)
    for mtu, cap, window in ((9702, 37, 1 << 16), (1500, 1000, 1 << 16), (100000, 4096, 0)):
        _check(p, mtu, cap, window)


@pytest.mark.gpu
@pytest.mark.parametrize("big", [False, True])
def test_pcapng_variants(tmp_path, gpu, big):
    p = tmp_path / "a.pcapng"
    _write_pcapng(p, _frames(600), big=big)
    for cap, window in ((37, 1 << 16), (1000, 0)):
        _check(p, 9702, cap, window)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", [("cfg3", 40000), ("cfg4", 12000), ("cfg2", 50000), ("traces", 0),
                                    ("adversarial", 0)])
def test_synthetic_and_trace_captures(tmp_path, gpu, name, n):
    """IMIX / 1500-B frames whose payloads are zero-filled (every zero run reads as a chain of
    empty records), 64-B frames, and the reference traces' frames: many windows and batch cuts."""
    slab, dlen, stride, _ = corpus(name, n)
    p = tmp_path / "c.pcap"
    _write_pcap(p, _slab_frames(slab, dlen, stride))
    sizes = _check(p, 9702, 4096, 1 << 20)
    assert sum(sizes) == len(opcap.offline_frames(p))


@pytest.mark.gpu
def test_batch_runs_the_packet_stage(tmp_path, gpu):
    """A GPU-walked batch in the gather layout through rtn_pc_run equals the oracle on the same
    frames."""
    import torch

    slab, dlen, stride, fset = corpus("cfg3", 20000)
    p = tmp_path / "c.pcap"
    _write_pcap(p, _slab_frames(slab, dlen, stride))
    r = pc.PcapReader(p)
    b = _Batches(1 << 15)
    n = r.next_batch_gpu(b.head, b.ext, b.chunk, b.dl)
    assert n == len(dlen)
    prog = pc.Program.from_spec(SETS[fset])
    ctx = pc.PacketContinue(prog, 0)
    out = ctx.run(b.head, 64, b.dl, n, out=ctx.alloc_outputs(n), ext=b.ext, ext_chunk=b.chunk)
    torch.cuda.synchronize()
    got = helpers.canonical(prog, out, dlen)
    ora = helpers.oracle_run(SETS[fset], slab, stride, dlen)
    helpers.assert_same(got, ora, "GPU capture walk -> rtn_pc_run")


@pytest.mark.gpu
def test_long_frame_ends_the_batch(tmp_path, gpu):
    """A kept frame longer than 65535 bytes: the frames before it, then RTN_ERANGE at it, again on
    every later call (the host reader's behaviour); skipped by the mtu it is no error."""
    fr = _frames(50)
    fr.insert(30, (b"\x01" * 70000, 70000))
    p = tmp_path / "big.pcap"
    _write_pcap(p, fr)
    want = opcap.offline_frames(p, mtu=100000)
    r = pc.PcapReader(p, mtu=100000)
    r.gpu_window(1 << 18)
    b = _Batches(1000)
    with pytest.raises(pc.RetinaError) as e:
        r.next_batch_gpu(b.head, b.ext, b.chunk, b.dl)
    assert e.value.code == -34
    k = next(i for i, f in enumerate(want) if len(f) > 65535)
    assert r.stats()["packed"] == k
    with pytest.raises(pc.RetinaError):
        r.next_batch_gpu(b.head, b.ext, b.chunk, b.dl)
    _check(p, 9702, 1000, 1 << 18)  # skipped by the mtu


@pytest.mark.gpu
def test_record_larger_than_window(tmp_path, gpu):
    p = tmp_path / "big.pcap"
    _write_pcap(p, [(b"\x02" * 70000, 70000), (b"\x03" * 60, 60)])
    r = pc.PcapReader(p, mtu=9702)
    r.gpu_window(1 << 16)
    b = _Batches(16)
    with pytest.raises(pc.RetinaError) as e:
        r.next_batch_gpu(b.head, b.ext, b.chunk, b.dl)
    assert e.value.code == -34 and "window" in str(e.value)


@pytest.mark.gpu
def test_truncated_tail_and_empty(tmp_path, gpu):
    """A truncated last record ends the capture (libpcap's reader reports it as an error and the
    offline runtime's loop ends, offline.rs:67): the host reader's frames exactly."""
    p = tmp_path / "t.pcap"
    _write_pcap(p, _frames(300))
    raw = p.read_bytes()
    for cut in (1, 10, 17):
        q = tmp_path / f"t{cut}.pcap"
        q.write_bytes(raw[:-cut])
        host = pc.PcapReader(q)
        slab, dlen = host.read_all(stride=128, batch=1000)
        got, st, _ = _walk(q, 9702, 100, 1 << 16)
        assert st == host.stats() and len(got) == len(dlen)
        for i, (b, d, need) in enumerate(got):
            assert d == dlen[i] and b == slab[i * 128:i * 128 + min(d, 128 if need else 64)].tobytes(), i
    e = tmp_path / "e.pcap"
    _write_pcap(e, [])
    got, st, _ = _walk(e)
    assert got == [] and st["frames"] == 0


@pytest.mark.gpu
def test_host_and_gpu_batches_share_the_position(tmp_path, gpu):
    """Host and GPU batches read one capture in turn: together they are its frames, in order."""
    p = tmp_path / "m.pcap"
    _write_pcap(p, _frames(800))
    want = opcap.offline_frames(p)
    r = pc.PcapReader(p)
    r.gpu_window(1 << 16)
    b = _Batches(100)
    got = []
    for turn in range(100):
        if turn % 2:
            s = np.zeros(100 * 128, np.uint8)
            d = np.zeros(100, np.uint16)
            k = r.next_batch(s, 128, d)
            got += [(s[i * 128:i * 128 + min(int(d[i]), 64)].tobytes(), int(d[i])) for i in range(k)]
        else:
            k = r.next_batch_gpu(b.head, b.ext, b.chunk, b.dl)
            got += [(x[0][:min(x[1], 64)], x[1]) for x in b.frames(k)]
        if k == 0:
            break
    assert [(f[:min(len(f), 64)], len(f)) for f in want] == got


@pytest.mark.gpu
def test_pcapng_sections_in_other_byte_order(tmp_path, gpu):
    """The GPU walk takes one byte order per capture: the frames before a section header of the
    other order, then RTN_EINVAL there (the host reader, which switches, takes the rest)."""
    a, b = tmp_path / "a.pcapng", tmp_path / "b.pcapng"
    _write_pcapng(a, _frames(60), big=False)
    _write_pcapng(b, _frames(40), big=True)
    p = tmp_path / "ab.pcapng"
    p.write_bytes(a.read_bytes() + b.read_bytes())
    first = opcap.offline_frames(a)
    r = pc.PcapReader(p)
    bufs = _Batches(1000)
    got = []
    with pytest.raises(pc.RetinaError) as e:
        while True:
            n = r.next_batch_gpu(bufs.head, bufs.ext, bufs.chunk, bufs.dl)
            assert n > 0
            got += bufs.frames(n)
    assert e.value.code == -22
    assert [(x[0], x[1]) for x in got] == [(f[:min(len(f), 128 if g[2] else 64)], len(f)) for f, g in zip(first, got)]
    assert len(got) == len(first)


@pytest.mark.gpu
def test_staged_window_copy(tmp_path, gpu, monkeypatch):
    """The fallback window copy (worker threads into pinned memory, taken when the file's pages
    cannot be registered; forced here by RTN_GPU_WALK_STAGED): the same frames."""
    monkeypatch.setenv("RTN_GPU_WALK_STAGED", "1")
    slab, dlen, stride, _ = corpus("cfg3", 30000)
    p = tmp_path / "c.pcap"
    _write_pcap(p, _slab_frames(slab, dlen, stride))
    _check(p, 9702, 4096, 1 << 20)
    p2 = tmp_path / "a.pcapng"
    _write_pcapng(p2, _frames(600), big=True)
    _check(p2, 9702, 37, 1 << 16)


@pytest.mark.gpu
def test_frame_size_change_and_window_resize(tmp_path, gpu):
    """Small frames then large ones (the walk bounded by the last batch's bytes per frame falls
    short and the whole window is walked), and the window resized between batches while the next
    one is being prefetched (smaller, then larger: the device buffers are reallocated)."""
    import torch

    small = [(bytes([i % 251]) * 60, 60) for i in range(3000)]
    large = [(bytes([i % 241]) * 1400, 1400) for i in range(3000)]
    p = tmp_path / "mix.pcap"
    _write_pcap(p, small + large + small)
    want = opcap.offline_frames(p)
    r = pc.PcapReader(p)
    r.gpu_window(1 << 20)
    b = _Batches(500)
    got = []
    for turn in range(1000):
        if turn == 3:
            r.gpu_window(1 << 17)
        elif turn == 9:
            r.gpu_window(1 << 22)
        n = r.next_batch_gpu(b.head, b.ext, b.chunk, b.dl)
        torch.cuda.synchronize()
        if n == 0:
            break
        got += b.frames(n)
    assert len(got) == len(want)
    for i, ((x, d, need), f) in enumerate(zip(got, want)):
        assert d == len(f) and x == f[:min(len(f), 128 if need else 64)], i
    host = pc.PcapReader(p)
    host.read_all(stride=64, batch=4096)
    assert r.stats() == host.stats()
